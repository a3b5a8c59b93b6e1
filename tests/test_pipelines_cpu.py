"""SD-family pipeline plumbing on CPU fp32 (tiny configs + BASELINE config #1)."""
import base64
import io

import numpy as np
import pytest
import torch
from PIL import Image

from chiaswarm_amd.pipelines.sd import StableDiffusion, family_for_model
from chiaswarm_amd.runtime.device import Device
from chiaswarm_amd.runtime.generator import synchronous_do_work_function
from chiaswarm_amd.schedulers import get_scheduler


@pytest.fixture(scope="module")
def tiny():
    return StableDiffusion("tiny", "cpu", seed=1)


def gen(s=0):
    return torch.Generator().manual_seed(s)


def test_family_mapping():
    assert family_for_model("stabilityai/stable-diffusion-2-1-base") == "sd21"
    assert family_for_model("stabilityai/stable-diffusion-2-1") == "sd21-v"
    assert family_for_model("runwayml/stable-diffusion-v1-5") == "sd15"
    assert family_for_model("stabilityai/stable-diffusion-xl-base-1.0") == "sdxl"
    assert family_for_model("timbrooks/instruct-pix2pix") == "pix2pix"


@pytest.mark.parametrize("sched", ["DPMSolverMultistepScheduler", "EulerAncestralDiscreteScheduler",
                                   "DDIMScheduler", "HeunDiscreteScheduler", "LMSDiscreteScheduler"])
def test_txt2img_schedulers(tiny, sched):
    out = tiny(prompt="x", num_inference_steps=3, height=64, width=64, generator=gen(),
               scheduler=get_scheduler(sched))
    assert out.images[0].size == (64, 64) and torch.isfinite(out.latents).all()


def test_seed_reproducible_and_negative_prompt(tiny):
    a = tiny(prompt="x", num_inference_steps=3, height=64, width=64, generator=gen(5)).latents
    b = tiny(prompt="x", num_inference_steps=3, height=64, width=64, generator=gen(5)).latents
    c = tiny(prompt="x", negative_prompt="blurry", num_inference_steps=3, height=64, width=64,
             generator=gen(5)).latents
    assert torch.equal(a, b) and not torch.equal(a, c)


def test_img2img_strength(tiny):
    img = Image.fromarray((np.random.default_rng(0).random((64, 64, 3)) * 255).astype(np.uint8))
    out = tiny(prompt="x", image=img, strength=0.5, num_inference_steps=4, generator=gen())
    assert out.images[0].size == (64, 64)


def test_inpaint_legacy(tiny):
    img = Image.new("RGB", (64, 64), (120, 30, 30))
    mask = Image.new("L", (64, 64), 0)
    mask.paste(255, (16, 16, 48, 48))
    out = tiny(prompt="x", image=img, mask_image=mask, strength=1.0, num_inference_steps=3, generator=gen())
    assert out.images[0].size == (64, 64)


def test_controlnet_tiny(tiny):
    from chiaswarm_amd.pipelines.controlnet import load_controlnet

    tiny.controlnet = load_controlnet("tiny/controlnet", tiny, "cpu")
    try:
        cond = Image.new("RGB", (64, 64), (255, 255, 255))
        out = tiny(prompt="x", image=cond, num_inference_steps=2, generator=gen(),
                   controlnet_conditioning_scale=0.7)
        assert out.images[0].size == (64, 64)
    finally:
        tiny.controlnet = None


def test_canny_matches_known_edges():
    from chiaswarm_amd.controlnet.preprocess import canny_np, image_to_canny

    a = np.zeros((32, 32), np.uint8)
    a[:, 16:] = 255
    e = canny_np(a, 100, 200)
    cols = np.nonzero(e.any(axis=0))[0]
    assert set(cols.tolist()) <= {15, 16} and e[5:27].any()
    im = image_to_canny(Image.fromarray(np.stack([a] * 3, -1)))
    assert im.mode == "RGB" and im.size == (32, 32)
    # colour input: an edge visible in ONE channel only (invisible in luma-equal mixes) is found
    rgb = np.zeros((32, 32, 3), np.uint8)
    rgb[:, 16:, 2] = 255
    e3 = canny_np(rgb, 100, 200)
    assert set(np.nonzero(e3.any(axis=0))[0].tolist()) <= {15, 16} and e3[5:27].any()
    # replicate border: a constant image has no edges at its border
    assert not canny_np(np.full((16, 16, 3), 200, np.uint8), 100, 200).any()


def test_baseline_config1_sd21_cpu():
    """BASELINE config #1: SD2.1 txt2img 64x64, 4 steps, batch 1, CPU fp32 via the generator."""
    r = synchronous_do_work_function({"id": "c1", "model_name": "stabilityai/stable-diffusion-2-1-base",
                                      "prompt": "spoons", "num_inference_steps": 4, "height": 64, "width": 64,
                                      "seed": 1}, Device("cpu"))
    assert "error" not in r["pipeline_config"], r["pipeline_config"]
    assert r["pipeline_config"]["family"] == "sd21" and r["pipeline_config"]["seed"] == 1
    im = Image.open(io.BytesIO(base64.b64decode(r["artifacts"]["primary"]["blob"])))
    assert im.size == (64, 64)


def test_controlnet_fused_merge_equals_residual_add(tiny):
    """skip + scale * zero_conv(feature) in the zero conv's epilogue == the
    diffusers-style residual tensors added to the skips (reference:
    StableDiffusionControlNetPipeline, swarm/diffusion/diffusion_func.py:29-39)."""
    import torch

    from chiaswarm_amd.pipelines.controlnet import ControlFeatures, load_controlnet

    runner = load_controlnet("tiny/controlnet-merge", tiny, "cpu")
    cn, unet = runner.model, tiny.unet
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 8, 8, 4, generator=g)
    ctx = torch.randn(2, 77, unet.cfg.cross_attention_dim, generator=g)
    cond = cn.embed_cond(torch.rand(2, 64, 64, 3, generator=g))
    t = torch.tensor([500.0])
    kv, ckv = unet.encode_context(ctx), cn.encode_context(ctx)
    with torch.no_grad():
        downs, mid = cn(x, t, cond, cross_kv=ckv, scale=0.7)
        ref = unet(x, t, cross_kv=kv, down_residuals=downs, mid_residual=mid)
        feats, m = cn.features(x, t, cond, cross_kv=ckv)
        got = unet(x, t, cross_kv=kv, control=ControlFeatures(cn, feats, m, 0.7))
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4)
    assert not torch.allclose(got, unet(x, t, cross_kv=kv), atol=1e-3)  # the control does something


def test_txt2vid_tiny_cpu_seeded():
    """txt2vid (reference swarm/video/tx2vid.py:17-76) on the tiny UNet3D: the
    eager CPU path gives uint8 frames and honours the seed."""
    from chiaswarm_amd.pipelines.video import TextToVideo

    p = TextToVideo("tiny-t2v", "cpu", tiny=True)
    kw = dict(prompt="a boat", num_frames=3, num_inference_steps=2, height=32, width=32)
    a = p(generator=gen(4), **kw)
    b = p(generator=gen(4), **kw)
    assert a.shape == (3, 32, 32, 3) and a.dtype == np.uint8
    assert np.array_equal(a, b)
    assert not p._graphs.graphs  # CPU: no graph capture


def test_img2txt_vqa_and_unsupported_class_envelopes(monkeypatch):
    """img2txt through the real router / generator: BLIP VQA answers the prompt
    (text artifact + pipeline_config.caption); an unsupported transformers class
    comes back fatal, naming the class."""
    import base64
    import io
    import json

    from PIL import Image

    import chiaswarm_amd.jobs.inputs as inputs

    img = Image.new("RGB", (64, 64), (10, 200, 30))
    monkeypatch.setattr(inputs, "get_image", lambda *a, **k: img)
    monkeypatch.setattr("chiaswarm_amd.jobs.router.get_image", lambda *a, **k: img, raising=False)
    buf = io.BytesIO()
    img.save(buf, "PNG")
    job = {"id": "v1", "model_name": "tiny/blip-vqa", "workflow": "img2txt", "prompt": "what color is it?",
           "start_image_uri": "http://x/img.png",
           "parameters": {"processor_type": "BlipProcessor", "model_type": "BlipForQuestionAnswering"}}
    r = synchronous_do_work_function(dict(job), Device("cpu"))
    assert "fatal_error" not in r and "error" not in r["pipeline_config"], r["pipeline_config"]
    blob = json.loads(base64.b64decode(r["artifacts"]["primary"]["blob"]))
    assert blob["caption"] == r["pipeline_config"]["caption"]
    git = dict(job, id="v2", model_name="tiny/git", prompt="",
               parameters={"processor_type": "AutoProcessor", "model_type": "GitForCausalLM"})
    r2 = synchronous_do_work_function(git, Device("cpu"))
    assert "fatal_error" not in r2 and "error" not in r2["pipeline_config"], r2["pipeline_config"]
    bad = dict(job, id="v3", parameters={"processor_type": "AutoProcessor",
                                         "model_type": "Kosmos2ForConditionalGeneration"})
    r3 = synchronous_do_work_function(bad, Device("cpu"))
    assert r3.get("fatal_error") is True and "Kosmos2ForConditionalGeneration" in r3["pipeline_config"]["error"]


def test_unet_cfg_shared_prefix_and_temb_table_cpu():
    """UNet forward with the CFG-shared prefix (cfg_dup) and with precomputed
    time projections (temb_table rows) equals the plain forward on identical
    CFG halves (fp32 reference ops)."""
    from chiaswarm_amd.models import unet as unet_mod
    from chiaswarm_amd.models.layers import init_random_fast_, prepare_model

    torch.manual_seed(0)
    m = unet_mod.UNet2DConditionModel(unet_mod.TINY).eval().requires_grad_(False)
    init_random_fast_(m, seed=1)
    prepare_model(m)
    xh = torch.randn(2, 8, 8, 4)
    x = torch.cat([xh, xh])
    ctx = torch.randn(4, 77, 32)
    t = torch.tensor([321.0])
    with torch.no_grad():
        ref = m(x, t, encoder_hidden_states=ctx)
        y = m(x, t, encoder_hidden_states=ctx, cfg_dup=True)
        tab = m.temb_table(torch.tensor([999.0, 321.0, 5.0]))
        y2 = m(x, t, encoder_hidden_states=ctx, temb_proj=tab[1:2].expand(4, -1).contiguous())
    assert torch.allclose(y, ref, rtol=1e-4, atol=1e-5)
    assert torch.allclose(y2, ref, rtol=1e-4, atol=1e-5)
