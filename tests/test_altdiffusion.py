"""AltDiffusion (``AltDiffusionPipeline`` / ``AltDiffusionImg2ImgPipeline``,
diffusers 0.16.1 — reachable by class name in the reference,
swarm/job_arguments.py:143-145): the SD1.x UNet conditioned on
``RobertaSeriesModelWithTransformation`` (XLM-RoBERTa + a linear
transformation, models/xlmr.py).

Pinned against transformers: the encoder (``XLMRobertaModel`` + the
transformation, padded + attention-masked batch, and the pre-transformation
variant) and the tokenizer (``XLMRobertaTokenizer`` on a sentencepiece unigram
model trained here).  The diffusers wrapper class itself is not importable, so
its composition (transformation of the last hidden state; pre_LN +
transformation_pre of the second-to-last) is the part left unpinned."""
import json
import os

import pytest
import torch

from chiaswarm_amd.models.layers import prepare_model
from chiaswarm_amd.models.weights import load_into
from chiaswarm_amd.models.xlmr import XLMRConfig, XLMRobertaSeries, XLMRTokenizer
from chiaswarm_amd.pipelines import diffusion


def _hf_pair(d=32, proj=24, pre=False, seed=0):
    from transformers import XLMRobertaConfig, XLMRobertaModel

    torch.manual_seed(seed)
    hc = XLMRobertaConfig(vocab_size=1000, hidden_size=d, num_hidden_layers=3, num_attention_heads=2,
                          intermediate_size=2 * d, max_position_embeddings=80, type_vocab_size=1, layer_norm_eps=1e-5,
                          pad_token_id=1)
    hm = XLMRobertaModel(hc).eval()
    tr = torch.nn.Linear(d, proj)
    sd = {"roberta." + k: v for k, v in hm.state_dict().items()}
    sd.update({"transformation." + k: v.clone() for k, v in tr.state_dict().items()})
    extra = {}
    if pre:
        extra["transformation_pre"] = torch.nn.Linear(d, proj)
        extra["pre_LN"] = torch.nn.LayerNorm(d, eps=1e-5)
        with torch.no_grad():
            extra["pre_LN"].weight.uniform_(0.5, 1.5)
            extra["pre_LN"].bias.normal_(0, 0.1)
        for n, m in extra.items():
            sd.update({f"{n}.{k}": v.clone() for k, v in m.state_dict().items()})
    cfg = dict(hc.to_dict(), architectures=["RobertaSeriesModelWithTransformation"], project_dim=proj,
               has_pre_transformation=pre)
    return hm, tr, extra, sd, cfg


@pytest.mark.parametrize("pre", [False, True])
def test_xlmr_encoder_matches_transformers(pre):
    from chiaswarm_amd.models.xlmr import xlmr_text_config

    hm, tr, extra, sd, cfg = _hf_pair(pre=pre)
    ours = XLMRobertaSeries(xlmr_text_config(cfg))
    rep = load_into(ours, sd, ours.hf_renames, name="text_encoder")
    assert not rep.missing and not rep.unexpected
    prepare_model(ours)
    ids = torch.tensor([[0, 5, 17, 33, 2] + [1] * 10, [0, 9, 2] + [1] * 12, [0] + list(range(10, 23)) + [2]])
    with torch.no_grad():
        o = hm(input_ids=ids, attention_mask=(ids != 1).long(), output_hidden_states=True)
        want = extra["transformation_pre"](extra["pre_LN"](o.hidden_states[-2])) if pre else tr(o.last_hidden_state)
        got = ours(ids)[0]
    assert torch.allclose(got, want, atol=2e-5, rtol=1e-4), (got - want).abs().max()


def _spm_dir(tmp_path):
    import sentencepiece as spm

    d = tmp_path / "tok"
    d.mkdir(exist_ok=True)
    corpus = d / "c.txt"
    corpus.write_text("\n".join(["a photograph of an astronaut riding a horse", "un chat noir sur un toit",
                                 "ein Hund im Park", "一只猫在屋顶上", "the quick brown fox"] * 40))
    spm.SentencePieceTrainer.train(input=str(corpus), model_prefix=str(d / "sentencepiece.bpe"), vocab_size=40,
                                   hard_vocab_limit=False, model_type="unigram", character_coverage=1.0,
                                   minloglevel=2)
    return d


def test_xlmr_tokenizer_matches_transformers(tmp_path):
    from transformers import XLMRobertaTokenizer

    d = _spm_dir(tmp_path)
    ht = XLMRobertaTokenizer.from_pretrained(str(d), model_max_length=77)
    ot = XLMRTokenizer(str(d), 77, vocab_size=len(ht))
    assert ot.loaded
    for s in ["a photograph of an astronaut", "un chat noir xyz!", "一只猫", "", "Ein  Hund   im Park",
              " ".join(["horse"] * 100)]:
        want = ht(s, padding="max_length", max_length=77, truncation=True)["input_ids"]
        assert ot(s)[0].tolist() == want, s


def test_altdiffusion_checkpoint_end_to_end(tmp_path):
    from safetensors.torch import save_file

    from chiaswarm_amd.models import hf_config as hc
    from chiaswarm_amd.models import unet as unet_mod
    from chiaswarm_amd.models import vae as vae_mod
    from chiaswarm_amd.models.hf_config import pipeline_spec
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.pipelines.sd import StableDiffusion, resolve_family
    from tests.test_hf_config import _j, _save_st, _tiny_unet, _tiny_vae, _write_json

    root = tmp_path / "alt"
    sd15 = "runwayml--stable-diffusion-v1-5"
    uc = _tiny_unet(_j(sd15, "unet", "config.json"), 24)
    _write_json(str(root / "unet" / "config.json"), uc)
    u = unet_mod.UNet2DConditionModel(hc.unet_config(uc))
    init_random_(u, seed=7)
    _save_st(u, str(root / "unet"))
    vc = _tiny_vae(_j(sd15, "vae", "config.json"))
    _write_json(str(root / "vae" / "config.json"), vc)
    v = vae_mod.AutoencoderKL(hc.vae_config(vc))
    init_random_(v, seed=8)
    _save_st(v, str(root / "vae"))
    (root / "scheduler").mkdir()
    _write_json(str(root / "scheduler" / "scheduler_config.json"), _j(sd15, "scheduler", "scheduler_config.json"))
    hm, tr, _, sd, cfg = _hf_pair(d=32, proj=24)
    (root / "text_encoder").mkdir()
    save_file({k: t.contiguous() for k, t in sd.items()}, str(root / "text_encoder" / "model.safetensors"))
    with open(root / "text_encoder" / "config.json", "w") as f:
        json.dump(cfg, f)
    tok = _spm_dir(tmp_path)
    (root / "tokenizer").mkdir()
    os.replace(tok / "sentencepiece.bpe.model", root / "tokenizer" / "sentencepiece.bpe.model")
    with open(root / "model_index.json", "w") as f:
        json.dump({"_class_name": "AltDiffusionPipeline", "unet": ["diffusers", "UNet2DConditionModel"],
                   "vae": ["diffusers", "AutoencoderKL"],
                   "text_encoder": ["diffusers", "RobertaSeriesModelWithTransformation"],
                   "tokenizer": ["transformers", "XLMRobertaTokenizer"],
                   "scheduler": ["diffusers", "PNDMScheduler"]}, f)
    spec = pipeline_spec(str(root))
    assert spec.class_name == "AltDiffusionPipeline" and isinstance(spec.text[0], XLMRConfig)
    fam = resolve_family("BAAI/AltDiffusion", str(root))
    pipe = StableDiffusion(fam, device="cpu", weights_dir=str(root))
    assert pipe.weights_source == str(root) and pipe.tokenizers[0].loaded
    ids = pipe.tokenizers[0](["ein Hund im Park"])
    with torch.no_grad():
        want = tr(hm(input_ids=ids, attention_mask=(ids != 1).long()).last_hidden_state)
        got = pipe.text_encoders[0](ids)[0]
    assert torch.allclose(got, want, atol=2e-5, rtol=1e-4)
    out = pipe(prompt="ein Hund im Park", num_inference_steps=2, output_type="latent",
               generator=torch.Generator().manual_seed(0))
    assert torch.isfinite(out.latents).all()


def test_altdiffusion_jobs_cpu():
    import base64
    import io

    import numpy as np
    from PIL import Image

    for cls in ("AltDiffusionPipeline", "AltDiffusionImg2ImgPipeline"):
        kw = dict(prompt="un chat noir", num_inference_steps=2, scheduler_type="DDIMScheduler", upscale=False,
                  supports_xformers=True, generator=torch.Generator().manual_seed(0))
        if "Img2Img" in cls:
            kw["image"] = Image.fromarray((np.random.default_rng(0).random((64, 64, 3)) * 255).astype(np.uint8))
            kw["strength"] = 0.6
        res, cfg = diffusion.diffusion_callback("cpu", "tiny/altdiffusion", pipeline_type=cls, **kw)
        assert cfg["_pipeline_type"] == cls
        assert Image.open(io.BytesIO(base64.b64decode(res["primary"]["blob"]))).size == (64, 64)


@pytest.mark.gpu
def test_altdiffusion_on_gpu(gpu):
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    pipe = StableDiffusion("tiny-alt", device=gpu, seed=2)
    out = pipe(prompt="ein Hund im Park", num_inference_steps=3, output_type="latent",
               generator=torch.Generator(device=gpu).manual_seed(0))
    assert torch.isfinite(out.latents).all()
    # the encoder on the GPU (MFMA GEMMs + flash attention) against its fp32 CPU twin (same weights)
    import copy

    cpu = StableDiffusion("tiny-alt", device="cpu", seed=2)
    enc = copy.deepcopy(cpu.text_encoders[0]).to(gpu).to(torch.bfloat16)
    prepare_model(enc)
    ids = pipe.tokenizers[0](["ein Hund im Park", "un chat noir sur un toit"])
    with torch.no_grad():
        g = enc(ids.to(gpu))[0].float().cpu()
        c = cpu.text_encoders[0](ids)[0]
    assert ((g - c).norm() / c.norm()).item() < 2e-2
