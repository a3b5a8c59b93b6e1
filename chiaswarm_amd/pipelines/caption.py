"""``workflow: img2txt`` (reference: swarm/captioning/caption_image.py:6-40).

Same contract: returns a text artifact ``{"caption": ...}`` and
``pipeline_config.caption``; runtime errors are swallowed into the artifact
(the reference catches everything inside the callback and returns
``pipeline_config.error``).

``parameters.processor_type`` / ``parameters.model_type`` name transformers
classes in the reference (resolved by reflection, :11-13).  Here they select
the implementation:

* ``BlipForConditionalGeneration`` (+ ``BlipProcessor`` / ``AutoProcessor``):
  image captioning, conditional on the prompt when one is given;
* ``BlipForQuestionAnswering``: visual question answering — the prompt is the
  question (the reference's "conditional image captioning and VQA" branch,
  :21-23);
* ``GitForCausalLM`` (+ ``GitProcessor`` / ``AutoProcessor``): GIT captioning
  (``models/git.py``), conditional on the prompt when one is given ([CLS] +
  prompt tokens, the GIT conditional-captioning / VQA form);
* ``VisionEncoderDecoderModel`` (+ ``ViTImageProcessor`` / ``AutoProcessor``):
  ViT -> GPT-2 captioning (``models/vit_gpt2.py``, e.g.
  nlpconnect/vit-gpt2-image-captioning);
* ``Blip2ForConditionalGeneration`` / ``InstructBlipForConditionalGeneration``
  (+ ``Blip2Processor`` / ``InstructBlipProcessor`` / ``AutoProcessor``):
  BLIP-2 / InstructBLIP with an OPT, Flan-T5 or Vicuna language model
  (``models/blip2.py``); the
  prompt, when given, is the text the LM continues / answers ("Question: ...
  Answer:" for VQA);

any other class is refused with a ``ValueError`` that names it (a fatal job
error: retrying cannot help).  Model geometry comes from the checkpoint's
``config.json`` (a transformers ``BlipConfig`` / ``GitConfig`` / ``Blip2Config``), name heuristics
only without one.
"""
from __future__ import annotations

import os

import torch

from ..models.blip import BLIP_BASE, BLIP_LARGE, TINY_BLIP, BlipCaptioner, BlipConfig, BlipVQA
from ..models.layers import init_random_fast_, prepare_model
from ..models.wordpiece import WordPiece
from ..output.processor import make_text_result
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights

MODEL_TYPES = {"BlipForConditionalGeneration": "caption", "BlipForQuestionAnswering": "vqa", "GitForCausalLM": "git",
               "Blip2ForConditionalGeneration": "blip2", "InstructBlipForConditionalGeneration": "blip2",
               "VisionEncoderDecoderModel": "vitgpt2"}
PROCESSOR_TYPES = {"BlipProcessor", "AutoProcessor", "BlipImageProcessor", "GitProcessor", "CLIPImageProcessor",
                   "Blip2Processor", "InstructBlipProcessor", "ViTImageProcessor", "ViTFeatureExtractor", None}


def resolve_task(params: dict | None, model_name: str) -> str:
    """'caption' | 'vqa' | 'git' | 'blip2' | 'vitgpt2' from the hive's class names; ValueError for anything else."""
    params = params or {}
    mt, pt = params.get("model_type"), params.get("processor_type")
    if pt not in PROCESSOR_TYPES:
        raise ValueError(f"img2txt: processor_type {pt!r} is not supported "
                         "(supported: BlipProcessor, GitProcessor, Blip2Processor, ViTImageProcessor, AutoProcessor)")
    if mt is None:
        n = model_name.lower()
        if "blip2" in n or "instructblip" in n:
            return "blip2"
        if "vit-gpt2" in n:
            return "vitgpt2"
        return "vqa" if "vqa" in n else ("git" if "/git-" in n or n.startswith("git-") else "caption")
    if mt not in MODEL_TYPES:
        raise ValueError(f"img2txt: model_type {mt!r} is not supported "
                         f"(supported: {', '.join(sorted(MODEL_TYPES))})")
    return MODEL_TYPES[mt]


def _config(model_name: str, w: str | None) -> BlipConfig:
    from ..models.hf_config import component_config

    raw = component_config(w, "") if w else None
    if raw is not None and ("text_config" in raw or "vision_config" in raw):
        return BlipConfig.from_hf(raw)
    n = model_name.lower()
    return TINY_BLIP if n.startswith("tiny") else (BLIP_LARGE if "large" in n else BLIP_BASE)


def _git_config(model_name: str, w: str | None):
    from ..models.git import GIT_BASE, GIT_LARGE, TINY_GIT, GitConfig
    from ..models.hf_config import component_config

    raw = component_config(w, "") if w else None
    if raw is not None and "vision_config" in raw:
        return GitConfig.from_hf(raw)
    n = model_name.lower()
    return TINY_GIT if n.startswith("tiny") else (GIT_LARGE if "large" in n else GIT_BASE)


def load_git(model_name: str, device: str):
    def make():
        from ..models.git import GitCaptioner, convert_hf_git

        w = ensure_weights(model_name)
        cfg = _git_config(model_name, w)
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        with torch.device(device):
            m = GitCaptioner(cfg).to(dt).eval().requires_grad_(False)
        init_random_fast_(m, seed=11)
        m.weights_source = "random-init"
        if w:
            from ..models.weights import _read_dir, load_into

            sd = _read_dir(w)
            if sd:
                m.load_report = load_into(m, convert_hf_git(sd), name=model_name)
                m.weights_source = w
        prepare_model(m)
        return m, WordPiece(w, cfg.vocab)

    return cache().get(("git", model_name, device), make)


def load_blip2(model_name: str, device: str):
    def make():
        from ..models.blip2 import BLIP2_FLAN_T5_XL, BLIP2_OPT_2_7B, BLIP2_OPT_6_7B, TINY_BLIP2, Blip2Captioner, \
            Blip2Config, convert_hf_blip2
        from ..models.hf_config import component_config
        from ..models.tokenizer import ByteBPETokenizer

        w = ensure_weights(model_name)
        raw = component_config(w, "") if w else None
        if raw is not None and "qformer_config" in raw:
            cfg = Blip2Config.from_hf(raw)
        else:
            n = model_name.lower()
            if "instructblip" in n and not n.startswith("tiny"):
                raise ValueError(f"img2txt: {model_name}: InstructBLIP needs its config.json")
            if "t5" in n and "xxl" in n:
                raise ValueError(f"img2txt: no built-in geometry for {model_name}; its config.json is required")
            cfg = TINY_BLIP2 if n.startswith("tiny") else (
                BLIP2_FLAN_T5_XL if "flan-t5" in n else (BLIP2_OPT_6_7B if "6.7b" in n else BLIP2_OPT_2_7B))
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        with torch.device(device):
            m = Blip2Captioner(cfg).to(dt).eval().requires_grad_(False)
        init_random_fast_(m, seed=11)
        m.weights_source = "random-init"
        if w:
            from ..models.weights import _read_dir, load_into

            sd = _read_dir(w)
            if sd:
                m.load_report = load_into(m, convert_hf_blip2(sd), name=model_name)
                m.weights_source = w
        prepare_model(m)
        if cfg.instruct:  # the Q-Former's own BERT tokenizer, [CLS] instruction [SEP]
            m.qformer_tokenizer = WordPiece(os.path.join(w, "qformer_tokenizer") if w else None, cfg.q_vocab)
        if cfg.lm_type == "t5":
            from ..models.t5 import T5Tokenizer

            return m, T5Tokenizer(w, max_length=512, vocab=cfg.vocab, lower=False)
        if cfg.lm_type == "llama":
            return m, _SentencePiece(w, "tokenizer.model", cfg.vocab, skip=(cfg.bos_id, cfg.eos_id, cfg.pad_id))
        return m, ByteBPETokenizer(w, max_length=512, vocab_size=cfg.vocab, bos=cfg.bos_id, eos=cfg.eos_id,
                                   pad=cfg.pad_id)

    return cache().get(("blip2", model_name, device), make)


class _SentencePiece:
    """SentencePiece model file of a checkpoint (LLaMA ``tokenizer.model``), no
    special tokens added; hash fallback without one (random-init runs)."""

    def __init__(self, w: str | None, name: str, vocab: int, skip=()):
        self.sp, self.vocab, self.skip = None, vocab, set(skip)
        path = os.path.join(w, name) if w else None
        if path and os.path.exists(path):
            import sentencepiece

            self.sp = sentencepiece.SentencePieceProcessor(model_file=path)

    def encode(self, text: str) -> list[int]:
        if self.sp is not None:
            return list(self.sp.encode(text))
        import hashlib

        return [int.from_bytes(hashlib.blake2b(t.encode(), digest_size=8).digest(), "little") % (self.vocab - 10) + 3
                for t in text.split()]

    def decode(self, ids: list[int]) -> str:
        ids = [int(i) for i in ids if int(i) not in self.skip]
        return self.sp.decode(ids) if self.sp is not None else " ".join(f"w{i}" for i in ids)


def load_vitgpt2(model_name: str, device: str):
    def make():
        from ..models.hf_config import component_config
        from ..models.tokenizer import ByteBPETokenizer
        from ..models.vit_gpt2 import TINY_VIT_GPT2, VIT_GPT2, VitGpt2Captioner, VitGpt2Config, convert_hf_vit_gpt2

        w = ensure_weights(model_name)
        raw = component_config(w, "") if w else None
        if raw is not None and "encoder" in raw and "decoder" in raw:
            cfg = VitGpt2Config.from_hf(raw, component_config(w, "", "preprocessor_config.json"))
        else:
            cfg = TINY_VIT_GPT2 if model_name.lower().startswith("tiny") else VIT_GPT2
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        with torch.device(device):
            m = VitGpt2Captioner(cfg).to(dt).eval().requires_grad_(False)
        init_random_fast_(m, seed=11)
        m.weights_source = "random-init"
        if w:
            from ..models.weights import _read_dir, load_into

            sd = _read_dir(w)
            if sd:
                m.load_report = load_into(m, convert_hf_vit_gpt2(sd), name=model_name)
                m.weights_source = w
        prepare_model(m)
        return m, ByteBPETokenizer(w, max_length=1024, vocab_size=cfg.vocab, bos=cfg.start_id, eos=cfg.eos_id,
                                   pad=cfg.pad_id)

    return cache().get(("vitgpt2", model_name, device), make)


def load_captioner(model_name: str, device: str, task: str = "caption"):
    if task == "git":
        return load_git(model_name, device)
    if task == "blip2":
        return load_blip2(model_name, device)
    if task == "vitgpt2":
        return load_vitgpt2(model_name, device)

    def make():
        w = ensure_weights(model_name)
        cfg = _config(model_name, w)
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        cls = BlipVQA if task == "vqa" else BlipCaptioner
        with torch.device(device):
            m = cls(cfg).to(dt).eval().requires_grad_(False)
        init_random_fast_(m, seed=11)
        m.weights_source = "random-init"
        if w:
            from ..models.blip import convert_hf_blip, convert_hf_blip_vqa
            from ..models.weights import _read_dir, load_into

            sd = _read_dir(w)
            if sd:
                conv = convert_hf_blip_vqa if task == "vqa" else convert_hf_blip
                m.load_report = load_into(m, conv(sd), name=model_name)
                m.weights_source = w
        prepare_model(m)
        return m, WordPiece(w, cfg.vocab)

    return cache().get(("blip", task, model_name, device), make)


def caption_callback(device_identifier, model_name, **kwargs):
    config, results = {}, {}
    task = resolve_task(kwargs.pop("parameters", None), model_name)  # unsupported classes: fatal ValueError
    try:
        print("Visual question answering..." if task == "vqa" else "Image captioning...")
        model, tok = load_captioner(model_name, device_identifier, task)
        image = kwargs["image"]
        prompt = kwargs.get("prompt") or ""
        if task == "vqa":
            if not prompt:
                raise ValueError("img2txt VQA: a question (prompt) is required")
            qids = [model.cfg.cls_id] + tok.encode(prompt) + [model.cfg.sep_id]  # BertTokenizer [CLS] q [SEP]
            caption = tok.decode(model.answer(image, qids, max_length=int(kwargs.get("max_length", 20))))
        else:
            prefix = tok.encode(prompt) if prompt else []
            mnt = kwargs.get("max_new_tokens")
            extra = {}
            qt = getattr(model, "qformer_tokenizer", None)
            if qt is not None:  # InstructBLIP: the instruction also enters the Q-Former
                c = model.cfg  # [CLS] / [SEP] from the Q-Former vocab.txt (bert-base-uncased: 101 / 102)
                cls_id = qt.vocab.get("[CLS]", min(c.q_cls_id, c.q_vocab - 2))
                sep_id = qt.vocab.get("[SEP]", min(c.q_sep_id, c.q_vocab - 1))
                extra["qtext_ids"] = [cls_id] + (qt.encode(prompt) if prompt else []) + [sep_id]
            ids = model.generate(image, prefix, max_new_tokens=None if mnt is None else int(mnt),
                                 max_length=int(kwargs.get("max_length", 20)), **extra)
            caption = tok.decode(ids).strip()
        results["primary"] = make_text_result(caption)
        config["caption"] = caption
        return results, config
    except Exception as e:
        print(e)
        config["error"] = str(e)
        results["primary"] = make_text_result(str(e))
        return results, config
