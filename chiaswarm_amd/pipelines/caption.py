"""``workflow: img2txt`` (reference: swarm/captioning/caption_image.py:6-40).

Same contract: returns a text artifact ``{"caption": ...}`` and
``pipeline_config.caption``; errors are swallowed into the artifact (the
reference catches everything inside the callback and returns
``pipeline_config.error``).  ``parameters.processor_type/model_type`` name the
transformers classes in the reference; here they select the BLIP size.
"""
from __future__ import annotations

import torch

from ..models.blip import BLIP_BASE, BLIP_LARGE, TINY_BLIP, BlipCaptioner
from ..models.layers import init_random_fast_, prepare_model
from ..models.wordpiece import WordPiece
from ..output.processor import make_text_result
from ..runtime.model_cache import cache, find_weights


def load_captioner(model_name: str, device: str):
    def make():
        n = model_name.lower()
        cfg = TINY_BLIP if n.startswith("tiny") else (BLIP_LARGE if "large" in n else BLIP_BASE)
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        with torch.device(device):
            m = BlipCaptioner(cfg).to(dt).eval().requires_grad_(False)
        init_random_fast_(m, seed=11)
        w = find_weights(model_name)
        m.weights_source = "random-init"
        if w:
            from ..models.blip import convert_hf_blip
            from ..models.weights import _read_dir, load_into

            sd = _read_dir(w)
            if sd:
                m.load_report = load_into(m, convert_hf_blip(sd), name=model_name)
                m.weights_source = w
        prepare_model(m)
        return m, WordPiece(w, cfg.vocab)

    return cache().get(("blip", model_name, device), make)


def caption_callback(device_identifier, model_name, **kwargs):
    config, results = {}, {}
    try:
        print("Image captioning...")
        kwargs.pop("parameters", None)
        model, tok = load_captioner(model_name, device_identifier)
        image = kwargs["image"]
        prompt = kwargs.get("prompt") or ""
        prefix = tok.encode(prompt) if prompt else []
        mnt = kwargs.get("max_new_tokens")
        ids = model.generate(image, prefix, max_new_tokens=None if mnt is None else int(mnt),
                             max_length=int(kwargs.get("max_length", 20)))
        caption = tok.decode(ids)
        results["primary"] = make_text_result(caption)
        config["caption"] = caption
        return results, config
    except Exception as e:
        print(e)
        config["error"] = str(e)
        results["primary"] = make_text_result(str(e))
        return results, config
