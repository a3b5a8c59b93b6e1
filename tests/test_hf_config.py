"""Config-driven model construction (models/hf_config.py; the reference builds
every pipeline with ``from_pretrained`` from the checkpoint's own
``model_index.json`` / ``config.json`` / ``scheduler_config.json``:
swarm/diffusion/diffusion_func.py:41-46,72-74, swarm/audio/audioldm.py:19-20,
swarm/video/tx2vid.py:24-30).

Fixtures (tests/fixtures/hf_configs/<org>--<name>/) are builder-written
copies of the public configs of each model family.  Two layers of tests:

* the full-size configs parse to exactly the architectures the presets
  encode (SD1.5 / SD2.1 / SDXL ...), with the scheduler fields carried over;
* the same configs shrunk to tiny widths (same block structure, input
  channels, attention layout, conditioning) are written out as complete
  diffusers directories with safetensors weights + tokenizer files, loaded
  STRICTLY through the production loaders and run for one denoising step on
  the CPU.  The weights are produced by this package's own modules, so key
  parity with diffusers itself stays pinned only where transformers is
  available (tests/test_checkpoints.py); these tests pin config -> module.
"""
import copy
import dataclasses
import json
import os
import shutil

import pytest
import torch

from chiaswarm_amd.models import clip as clip_mod
from chiaswarm_amd.models import hf_config as hc
from chiaswarm_amd.models import unet as unet_mod
from chiaswarm_amd.models import vae as vae_mod
from chiaswarm_amd.models.weights import CheckpointMismatch

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "hf_configs")
SD_MODELS = ["runwayml--stable-diffusion-v1-5", "runwayml--stable-diffusion-inpainting",
             "stabilityai--stable-diffusion-2-1-base", "stabilityai--stable-diffusion-2-1",
             "stabilityai--stable-diffusion-2-inpainting", "stabilityai--stable-diffusion-xl-base-1.0",
             "stabilityai--stable-diffusion-xl-refiner-1.0", "timbrooks--instruct-pix2pix"]


def _j(*p):
    with open(os.path.join(FIX, *p)) as f:
        return json.load(f)


# --------------------------------------------------------------------------- full-size parsing
def test_full_size_configs_match_presets():
    spec = hc.pipeline_spec(os.path.join(FIX, "runwayml--stable-diffusion-v1-5"))
    assert spec.unet == unet_mod.SD15 and spec.vae == vae_mod.SD_VAE and spec.text == [clip_mod.CLIP_L]
    spec = hc.pipeline_spec(os.path.join(FIX, "stabilityai--stable-diffusion-2-1-base"))
    assert spec.unet == unet_mod.SD21 and spec.text == [clip_mod.OPENCLIP_H]
    spec = hc.pipeline_spec(os.path.join(FIX, "stabilityai--stable-diffusion-xl-base-1.0"))
    assert spec.unet == unet_mod.SDXL
    assert spec.vae.scaling_factor == pytest.approx(0.13025)
    assert spec.text == [clip_mod.CLIP_L, clip_mod.OPENCLIP_BIGG]
    assert hc.unet_config(_j("runwayml--stable-diffusion-inpainting", "unet", "config.json")) == \
        unet_mod.INPAINT_SD15
    assert hc.unet_config(_j("stabilityai--stable-diffusion-2-inpainting", "unet", "config.json")) == \
        unet_mod.INPAINT_SD2
    assert hc.unet_config(_j("timbrooks--instruct-pix2pix", "unet", "config.json")) == unet_mod.PIX2PIX
    a = hc.unet_config(_j("cvssp--audioldm-s-full-v2", "unet", "config.json"))
    assert a == unet_mod.AUDIOLDM
    m = hc.unet_config(_j("cvssp--audioldm-m-full", "unet", "config.json"))
    assert m.block_out_channels == (192, 384, 576, 960) and m.cross_attention_dim == (192, 384, 576, 960)
    from chiaswarm_amd.models import unet3d

    assert hc.unet3d_config(_j("damo-vilab--text-to-video-ms-1.7b", "unet", "config.json")) == \
        dataclasses.replace(unet3d.T2V, sample_size=32)
    from chiaswarm_amd.models.clap import CLAP_TEXT
    from chiaswarm_amd.models.vocoder import AUDIOLDM_HIFIGAN

    assert hc.clap_text_config(_j("cvssp--audioldm-s-full-v2", "text_encoder", "config.json")) == CLAP_TEXT
    assert hc.hifigan_config(_j("cvssp--audioldm-s-full-v2", "vocoder", "config.json")) == AUDIOLDM_HIFIGAN


def test_family_resolution_from_configs():
    from chiaswarm_amd.pipelines.sd import resolve_family

    f = resolve_family("x/any-name-at-all", os.path.join(FIX, "stabilityai--stable-diffusion-2-1"))
    assert f.prediction_type == "v_prediction" and f.default_size == 768 and f.from_config
    assert f.unet.in_channels == 4 and not f.is_xl and not f.is_pix2pix
    f = resolve_family("my/sd2-finetune", os.path.join(FIX, "stabilityai--stable-diffusion-2-inpainting"))
    assert f.unet.in_channels == 9 and f.pipeline_class == "StableDiffusionInpaintPipeline"
    assert f.unet.cross_attention_dim == 1024  # no "stable-diffusion-2" in the name: still an SD2 UNet
    f = resolve_family("runwayml/stable-diffusion-inpainting", os.path.join(FIX, "runwayml--stable-diffusion-inpainting"))
    assert f.unet.in_channels == 9 and f.unet.cross_attention_dim == 768
    f = resolve_family("timbrooks/instruct-pix2pix", os.path.join(FIX, "timbrooks--instruct-pix2pix"))
    assert f.is_pix2pix
    f = resolve_family("sdxl", os.path.join(FIX, "stabilityai--stable-diffusion-xl-base-1.0"))
    assert f.is_xl and f.default_size == 1024 and f.sched_config["timestep_spacing"] == "leading"
    # no config files: the name presets still apply
    assert resolve_family("runwayml/stable-diffusion-inpainting", None).unet.in_channels == 9


def test_scheduler_config_applied():
    from chiaswarm_amd.schedulers import get_scheduler

    kw = hc.scheduler_kwargs(_j("stabilityai--stable-diffusion-2-1", "scheduler", "scheduler_config.json"))
    s = get_scheduler("EulerDiscreteScheduler", **kw)
    assert s.prediction_type == "v_prediction" and s.steps_offset == 1
    kw = hc.scheduler_kwargs(_j("stabilityai--stable-diffusion-xl-base-1.0", "scheduler", "scheduler_config.json"))
    lead = get_scheduler("EulerDiscreteScheduler", **dict(kw, use_karras_sigmas=False))
    lin = get_scheduler("EulerDiscreteScheduler", use_karras_sigmas=False)
    lead.set_timesteps(10)
    lin.set_timesteps(10)
    assert lead.timesteps[0] == 901.0 and lin.timesteps[0] == 999.0  # "leading" + steps_offset vs linspace
    trail = get_scheduler("DDIMScheduler", timestep_spacing="trailing")
    trail.set_timesteps(10)
    assert trail.timesteps[0] == 999.0
    aud = hc.scheduler_kwargs(_j("cvssp--audioldm-s-full-v2", "scheduler", "scheduler_config.json"))
    assert aud["beta_start"] == 0.0015 and aud["beta_end"] == 0.0195


@pytest.mark.parametrize("patch,msg", [({"resnet_time_scale_shift": "scale_shift"}, "resnet_time_scale_shift"),
                                       ({"down_block_types": ["SimpleCrossAttnDownBlock2D"] * 4}, "block types"),
                                       ({"only_cross_attention": True}, "only_cross_attention"),
                                       ({"time_embedding_type": "fourier"}, "time_embedding_type")])
def test_unsupported_options_are_named(patch, msg):
    cfg = dict(_j("runwayml--stable-diffusion-v1-5", "unet", "config.json"), **patch)
    with pytest.raises(hc.UnsupportedConfig, match=msg):
        hc.unet_config(cfg)


# --------------------------------------------------------------------------- tiny directories, strict loads
def _tiny_unet(cfg, xdim, n_text_pool=0):
    cfg = copy.deepcopy(cfg)
    n = len(cfg["block_out_channels"])
    ch = [32, 64, 64, 64][:n]
    cfg["block_out_channels"] = ch
    hd = cfg.get("attention_head_dim")
    if isinstance(hd, list):
        cfg["attention_head_dim"] = [2, 4, 4, 4][:n]
    if isinstance(cfg.get("cross_attention_dim"), list):
        cfg["cross_attention_dim"] = ch
    else:
        cfg["cross_attention_dim"] = xdim
    if isinstance(cfg.get("transformer_layers_per_block"), list):
        cfg["transformer_layers_per_block"] = [min(t, 2) for t in cfg["transformer_layers_per_block"]]
    cfg["layers_per_block"] = 1
    if cfg.get("addition_embed_type") == "text_time":
        # 6 size / crop ids (base) or 5 with the aesthetic score (refiner) next to the pooled 1280
        n_ids = (cfg["projection_class_embeddings_input_dim"] - 1280) // cfg["addition_time_embed_dim"]
        cfg["addition_time_embed_dim"] = 8
        cfg["projection_class_embeddings_input_dim"] = n_text_pool + n_ids * 8
    if cfg.get("class_embed_type") == "simple_projection":
        cfg["projection_class_embeddings_input_dim"] = 32
    return cfg


def _tiny_vae(cfg):
    cfg = copy.deepcopy(cfg)
    cfg["block_out_channels"] = [32] * len(cfg["block_out_channels"])
    cfg["layers_per_block"] = 1
    return cfg


def _tiny_text(cfg, eos):
    cfg = copy.deepcopy(cfg)
    cfg.update(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2, vocab_size=1000,
               eos_token_id=eos)
    if cfg.get("projection_dim"):
        cfg["projection_dim"] = 32
    return cfg


def _save_st(module, d, name="diffusion_pytorch_model.safetensors"):
    from safetensors.torch import save_file

    os.makedirs(d, exist_ok=True)
    save_file({k: v.contiguous() for k, v in module.state_dict().items()}, os.path.join(d, name))


def _write_json(path, obj):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(obj, f)


def _tokenizer(dst, special):
    from test_checkpoints import _train_bpe

    vocab, _ = _train_bpe(dst)
    _write_json(os.path.join(dst, "special_tokens_map.json"), special)
    return vocab


def _tiny_sd_dir(name, root):
    """A complete tiny diffusers directory for fixture ``name`` under ``root``."""
    from chiaswarm_amd.models.layers import init_random_

    src = os.path.join(FIX, name)
    dst = os.path.join(root, name.replace("--", "/"))
    idx = _j(name, "model_index.json")
    _write_json(os.path.join(dst, "model_index.json"), idx)
    shutil.copytree(os.path.join(src, "scheduler"), os.path.join(dst, "scheduler"))
    texts = [s for s in ("text_encoder", "text_encoder_2") if s in idx and idx[s][0]]
    eos = None
    pool = 0
    for i, sub in enumerate(texts):
        tok = sub.replace("text_encoder", "tokenizer")
        vocab = _tokenizer(os.path.join(dst, tok), _j(name, tok, "special_tokens_map.json"))
        eos = vocab["<|endoftext|>"]
        tc = _tiny_text(_j(name, sub, "config.json"), eos)
        _write_json(os.path.join(dst, sub, "config.json"), tc)
        m = clip_mod.CLIPTextModel(hc.clip_text_config(tc if sub == "text_encoder" else dict(
            tc, architectures=[idx[sub][1]])))
        init_random_(m, seed=i)
        _save_st(m, os.path.join(dst, sub), "model.safetensors")
        pool = tc.get("projection_dim") or 0
    xdim = 32 * len(texts)
    uc = _tiny_unet(_j(name, "unet", "config.json"), xdim, pool)
    _write_json(os.path.join(dst, "unet", "config.json"), uc)
    u = unet_mod.UNet2DConditionModel(hc.unet_config(uc))
    init_random_(u, seed=7)
    _save_st(u, os.path.join(dst, "unet"))
    vc = _tiny_vae(_j(name, "vae", "config.json"))
    _write_json(os.path.join(dst, "vae", "config.json"), vc)
    v = vae_mod.AutoencoderKL(hc.vae_config(vc))
    init_random_(v, seed=8)
    _save_st(v, os.path.join(dst, "vae"))
    return dst


@pytest.mark.parametrize("name", SD_MODELS)
def test_sd_family_loads_strictly_and_steps(tmp_path, name, monkeypatch):
    from PIL import Image

    from chiaswarm_amd.pipelines.sd import StableDiffusion, resolve_family

    monkeypatch.setenv("SDAAS_PACKED_CACHE", "0")
    d = _tiny_sd_dir(name, str(tmp_path))
    fam = resolve_family(name.replace("--", "/"), d)
    pipe = StableDiffusion(fam, device="cpu", weights_dir=d)
    assert pipe.weights_source == d
    assert all(getattr(r, "complete", True) for r in pipe.load_reports.values()), pipe.load_reports
    assert pipe.config["_class_name"] == fam.pipeline_class
    kw = {}
    if fam.unet.in_channels != 4 or fam.aesthetics:  # inpaint (9) / pix2pix (8) / refiner: image-conditioned
        kw["image"] = Image.new("RGB", (64, 64), (120, 30, 200))
        if fam.unet.in_channels == 9:
            kw["mask_image"] = Image.new("L", (64, 64), 255)
    out = pipe(prompt="a red fox", num_inference_steps=1, height=64, width=64, guidance_scale=5.0,
               output_type="latent", generator=torch.Generator().manual_seed(0), **kw)
    assert torch.isfinite(out.latents).all()


def test_partial_checkpoint_is_an_error(tmp_path, monkeypatch):
    from chiaswarm_amd.pipelines.sd import StableDiffusion, resolve_family

    monkeypatch.setenv("SDAAS_PACKED_CACHE", "0")
    name = "stabilityai--stable-diffusion-2-1-base"
    d = _tiny_sd_dir(name, str(tmp_path / "a"))
    shutil.rmtree(os.path.join(d, "vae"))
    os.makedirs(os.path.join(d, "vae"))
    shutil.copy(os.path.join(FIX, name, "vae", "config.json"), os.path.join(d, "vae", "config.json"))
    with pytest.raises(CheckpointMismatch, match="vae"):
        StableDiffusion(resolve_family(name, d), device="cpu", weights_dir=d)
    d = _tiny_sd_dir(name, str(tmp_path / "b"))
    shutil.rmtree(os.path.join(d, "tokenizer"))
    with pytest.raises(CheckpointMismatch, match="tokenizer"):
        StableDiffusion(resolve_family(name, d), device="cpu", weights_dir=d)


@pytest.mark.parametrize("name", ["cvssp--audioldm-s-full-v2", "cvssp--audioldm-m-full", "cvssp--audioldm-l-full"])
def test_audioldm_sizes_load_strictly_and_step(tmp_path, name):
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.models.vocoder import HifiGan
    from chiaswarm_amd.pipelines.audio import AudioLDM

    dst = str(tmp_path / name)
    _write_json(os.path.join(dst, "model_index.json"), _j(name, "model_index.json"))
    shutil.copytree(os.path.join(FIX, name, "scheduler"), os.path.join(dst, "scheduler"))
    full = hc.unet_config(_j(name, "unet", "config.json"))
    uc = _tiny_unet(_j(name, "unet", "config.json"), None)
    tc = dict(_j(name, "text_encoder", "config.json"), hidden_size=32, intermediate_size=64, num_hidden_layers=2,
              num_attention_heads=2, vocab_size=1000, max_position_embeddings=80, projection_dim=32)
    vc = _tiny_vae(_j(name, "vae", "config.json"))
    hcfg = dict(_j(name, "vocoder", "config.json"), model_in_dim=16, upsample_initial_channel=32,
                upsample_rates=[4, 2], upsample_kernel_sizes=[8, 4], resblock_kernel_sizes=[3],
                resblock_dilation_sizes=[[1, 3]])
    from transformers import ClapTextConfig, ClapTextModelWithProjection

    torch.manual_seed(0)  # the text tower in the genuine transformers key layout
    hf = ClapTextModelWithProjection(ClapTextConfig(**{k: v for k, v in tc.items() if k not in (
        "architectures", "model_type")}))
    _write_json(os.path.join(dst, "text_encoder", "config.json"), tc)
    _save_st_dict(hf.state_dict(), os.path.join(dst, "text_encoder"), "model.safetensors")
    for sub, cfg, mod in (("unet", uc, unet_mod.UNet2DConditionModel(hc.unet_config(uc))),
                          ("vae", vc, vae_mod.AutoencoderKL(hc.vae_config(vc), with_encoder=False)),
                          ("vocoder", hcfg, HifiGan(hc.hifigan_config(hcfg)))):
        _write_json(os.path.join(dst, sub, "config.json"), cfg)
        init_random_(mod, seed=3)
        _save_st(mod, os.path.join(dst, sub))
    _tokenizer(os.path.join(dst, "tokenizer"), {"pad_token": "<pad>"})
    p = AudioLDM("cpu", weights_dir=dst)
    assert p.weights_source == dst
    assert p.unet.cfg.block_out_channels == (32, 64, 64, 64) and len(full.block_out_channels) == 4
    assert p.sched_config["beta_start"] == 0.0015 and p.sched_config["use_karras_sigmas"] is False
    audio = p(prompt="rain on a tin roof", num_inference_steps=1, audio_length_in_s=0.2)
    assert audio.shape[0] == 1 and torch.isfinite(torch.as_tensor(audio)).all()


def _save_st_dict(sd, d, name="diffusion_pytorch_model.safetensors"):
    from safetensors.torch import save_file

    os.makedirs(d, exist_ok=True)
    save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(d, name))


def test_text_to_video_unet3d_loads_strictly_and_steps(tmp_path, monkeypatch):
    from chiaswarm_amd.models import unet3d
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.pipelines.video import TextToVideo

    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    monkeypatch.setenv("SDAAS_PACKED_CACHE", "0")
    name = "damo-vilab--text-to-video-ms-1.7b"
    dst = str(tmp_path / "models" / "damo-vilab" / "text-to-video-ms-1.7b")
    _write_json(os.path.join(dst, "model_index.json"), _j(name, "model_index.json"))
    shutil.copytree(os.path.join(FIX, name, "scheduler"), os.path.join(dst, "scheduler"))
    vocab = _tokenizer(os.path.join(dst, "tokenizer"), _j(name, "tokenizer", "special_tokens_map.json"))
    uc = copy.deepcopy(_j(name, "unet", "config.json"))
    uc.update(block_out_channels=[32, 64, 64, 64], attention_head_dim=16, cross_attention_dim=32, layers_per_block=1)
    tc = _tiny_text(_j(name, "text_encoder", "config.json"), vocab["<|endoftext|>"])
    vc = _tiny_vae(_j(name, "vae", "config.json"))
    for sub, cfg, mod in (("unet", uc, unet3d.UNet3DConditionModel(hc.unet3d_config(uc))),
                          ("text_encoder", tc, clip_mod.CLIPTextModel(hc.clip_text_config(tc))),
                          ("vae", vc, vae_mod.AutoencoderKL(hc.vae_config(vc), with_encoder=False))):
        _write_json(os.path.join(dst, sub, "config.json"), cfg)
        init_random_(mod, seed=4)
        _save_st(mod, os.path.join(dst, sub))
    t2v = TextToVideo("damo-vilab/text-to-video-ms-1.7b", "cpu")
    assert t2v.config["weights"] == dst
    assert t2v.unet.cfg.num_heads == (2, 4, 4, 4)
    frames = t2v(prompt="a dog running", num_frames=2, num_inference_steps=1, height=64, width=64)
    assert frames.shape == (2, 64, 64, 3)


@pytest.mark.parametrize("cn", ["thibaud--controlnet-sd21-canny-diffusers", "lllyasviel--control_v11e_sd15_shuffle"])
def test_controlnet_from_config(tmp_path, cn, monkeypatch):
    """A ControlNet built from its own config.json (SD2.1: cross-attention 1024
    and linear projections; shuffle: global pooling) on a matching SD pipeline."""
    from PIL import Image

    from chiaswarm_amd.models.controlnet import ControlNetModel
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.pipelines.controlnet import load_controlnet
    from chiaswarm_amd.pipelines.sd import StableDiffusion, resolve_family

    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    monkeypatch.setenv("SDAAS_PACKED_CACHE", "0")
    base = "stabilityai--stable-diffusion-2-1-base" if "sd21" in cn else "runwayml--stable-diffusion-v1-5"
    d = _tiny_sd_dir(base, str(tmp_path / "models"))
    pipe = StableDiffusion(resolve_family(base, d), device="cpu", weights_dir=d)
    cc = _tiny_unet(_j(cn, "config.json"), 32)
    cc.pop("up_block_types", None)
    dst = str(tmp_path / "models" / cn.replace("--", "/"))
    _write_json(os.path.join(dst, "config.json"), cc)
    u, kw = hc.controlnet_config(cc)
    m = ControlNetModel(u, **kw)
    init_random_(m, seed=5)
    _save_st(m, dst)
    runner = load_controlnet(cn.replace("--", "/"), pipe, "cpu")
    assert runner.model.global_pool == ("shuffle" in cn)
    assert runner.model.cfg.use_linear_projection == ("sd21" in cn)
    pipe.controlnet = runner
    out = pipe(prompt="edges", image=Image.new("RGB", (64, 64), (255, 255, 255)), num_inference_steps=1,
               height=64, width=64, output_type="latent", generator=torch.Generator().manual_seed(0))
    assert torch.isfinite(out.latents).all()
    pipe.controlnet = None
    # a ControlNet built for another UNet is refused with both geometries named
    bad = dict(cc, cross_attention_dim=48)
    _write_json(os.path.join(dst, "config.json"), bad)
    with pytest.raises(ValueError, match="does not fit"):  # a new cache key (revision) re-reads the config
        load_controlnet(cn.replace("--", "/"), pipe, "cpu", revision="other")
