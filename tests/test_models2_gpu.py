"""fp32-twin parity of the non-headline model paths on the GPU (same method as
tests/test_models_gpu.py: the HIP bf16 forward against an fp32 copy of the SAME
bf16-rounded weights run through the plain-PyTorch reference ops):

* SDXL UNet (``text_time`` add-embedding, 10-layer transformer blocks) and its
  two text encoders (CLIP-L + OpenCLIP-bigG, penultimate hidden states and the
  pooled projection) — BASELINE config #3's model;
* SD1.5 inpaint (9-channel UNet), instruct-pix2pix (8-channel UNet) and the
  pix2pix 3-way classifier-free-guidance loop graph against the host loop;
* the ControlNet UNet branch (its residuals) and the Real-ESRGAN RRDBNet.

Reference call sites: swarm/diffusion/diffusion_func.py:29-46 (pipeline and
ControlNet loads), :96 (the forward pass)."""
import copy

import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.models import clip, unet
from chiaswarm_amd.models.layers import init_random_fast_, prepare_model

pytestmark = pytest.mark.gpu


def rel_err(y, ref, name=""):
    y, ref = y.float(), ref.float()
    e = ((y - ref).norm() / (ref.norm() + 1e-12)).item()
    if name:
        print(f"[parity] {name}: rel_err {e:.3e} (HIP bf16 vs fp32 twin)")
    return e


def _build(cls, cfg, dev, **kw):
    with torch.device(dev):
        m = cls(cfg, **kw).to(torch.bfloat16).eval().requires_grad_(False)
    init_random_fast_(m, seed=3)
    return prepare_model(m)


def _twin(m):
    return copy.deepcopy(m).float()


@torch.no_grad()
def test_sdxl_unet_text_time_parity_vs_fp32(gpu):
    m = _build(unet.UNet2DConditionModel, unet.SDXL, gpu)
    x = torch.randn(2, 32, 32, 4, device=gpu).bfloat16()
    ctx = torch.randn(2, 77, 2048, device=gpu).bfloat16()
    added = {"text_embeds": torch.randn(2, 1280, device=gpu).bfloat16(),
             "time_ids": torch.tensor([[1024, 1024, 0, 0, 1024, 1024]] * 2, device=gpu, dtype=torch.float32)}
    t = torch.tensor([700.0], device=gpu)
    m32 = _twin(m)
    with ops.ops_mode("reference"):
        ref = m32(x.float(), t, encoder_hidden_states=ctx.float(),
                  added_cond={"text_embeds": added["text_embeds"].float(), "time_ids": added["time_ids"]})
    del m32
    y = m(x, t, cross_kv=m.encode_context(ctx), added_cond=added)
    assert torch.isfinite(y).all()
    assert rel_err(y, ref, "unet_sdxl") <= 2e-2


@torch.no_grad()
def test_sdxl_graph_add_emb_cache_matches_eager(gpu):
    """The step graph reads SDXL's text_time addition embedding from a static
    buffer filled once per request (pipelines.sd._UNetGraph): same output as the
    eager UNet computing it inline, and a new request's conditioning is picked
    up."""
    from chiaswarm_amd.pipelines.sd import _UNetGraph

    m = _build(unet.UNet2DConditionModel, unet.SDXL, gpu)
    x = torch.randn(2, 32, 32, 4, device=gpu).bfloat16()
    kv = m.encode_context(torch.randn(2, 77, 2048, device=gpu).bfloat16())

    def cond(seed):
        g = torch.Generator(device=gpu).manual_seed(seed)
        return {"text_embeds": torch.randn(2, 1280, device=gpu, generator=g).bfloat16(),
                "time_ids": torch.tensor([[1024, 1024, 0, 0, 1024, 1024]] * 2, device=gpu, dtype=torch.float32)}

    a1, a2 = cond(1), cond(2)
    gph = _UNetGraph(m, x, kv, a1)
    assert "add_emb" in gph.added
    for req, added in ((1, a1), (2, a2)):
        y = gph.run(x, 700.0, kv, added, req=req).clone()
        ref = m(x, torch.tensor([700.0], device=gpu), cross_kv=kv, added_cond=added)
        assert rel_err(y, ref) <= 1e-2, req


@torch.no_grad()
@pytest.mark.parametrize("cfg_name", ["CLIP_L", "OPENCLIP_BIGG"])
def test_sdxl_text_encoders_parity_vs_fp32(gpu, cfg_name):
    cfg = getattr(clip, cfg_name)
    m = _build(clip.CLIPTextModel, cfg, gpu)
    ids = torch.randint(0, 49000, (2, 77), device=gpu)
    m32 = _twin(m)
    with ops.ops_mode("reference"):
        last_r, pen_r, pooled_r, proj_r = m32(ids)
    last, pen, pooled, proj = m(ids)
    assert rel_err(pen, pen_r, f"{cfg_name} penultimate") <= 2e-2  # SDXL conditions on the penultimate layer
    assert rel_err(last, last_r, f"{cfg_name} last") <= 2e-2
    if proj is not None:
        assert rel_err(proj, proj_r, f"{cfg_name} projection") <= 2e-2


@torch.no_grad()
@pytest.mark.parametrize("cfg_name,cin", [("INPAINT_SD15", 9), ("PIX2PIX", 8)])
def test_sd15_variant_unets_parity_vs_fp32(gpu, cfg_name, cin):
    """SD1.5-geometry UNets (head dims 40 / 80 / 160, 1x1-conv proj_in) with
    the image-latent channels concatenated to the input."""
    m = _build(unet.UNet2DConditionModel, getattr(unet, cfg_name), gpu)
    x = torch.randn(3, 32, 32, cin, device=gpu).bfloat16()
    ctx = torch.randn(3, 77, 768, device=gpu).bfloat16()
    t = torch.tensor([400.0], device=gpu)
    m32 = _twin(m)
    with ops.ops_mode("reference"):
        ref = m32(x.float(), t, encoder_hidden_states=ctx.float())
    del m32
    y = m(x, t, cross_kv=m.encode_context(ctx))
    assert rel_err(y, ref, cfg_name.lower()) <= 2e-2


@torch.no_grad()
def test_pix2pix_three_way_loop_graph_matches_host_loop(gpu):
    """instruct-pix2pix: [cond, image-only, uncond] CFG batch of 3 with the
    8-channel UNet input, device-resident loop graph vs the per-step host loop."""
    from PIL import Image

    from chiaswarm_amd.pipelines import sd as sd_mod
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.schedulers import get_scheduler

    pipe = StableDiffusion("pix2pix", device=gpu, seed=2)
    img = Image.new("RGB", (128, 128), (30, 160, 90))

    def run(loop):
        sd_mod.LOOP_GRAPHS = loop
        try:
            g = torch.Generator(device=gpu).manual_seed(4)
            return pipe(prompt="make it snow", image=img, image_guidance_scale=1.5, guidance_scale=7.0,
                        num_inference_steps=5, generator=g, scheduler=get_scheduler("EulerAncestralDiscreteScheduler"),
                        output_type="latent").latents.float()
        finally:
            sd_mod.LOOP_GRAPHS = True

    host = run(False)
    graph = run(True)
    assert torch.isfinite(graph).all()
    assert rel_err(graph, host, "pix2pix loop graph vs host loop") < 2e-3


@torch.no_grad()
def test_controlnet_branch_parity_vs_fp32(gpu):
    from chiaswarm_amd.models.controlnet import ControlNetModel

    m = _build(ControlNetModel, unet.SD15, gpu)
    x = torch.randn(2, 32, 32, 4, device=gpu).bfloat16()
    ctx = torch.randn(2, 77, 768, device=gpu).bfloat16()
    cond_img = torch.rand(2, 256, 256, 3, device=gpu).bfloat16()
    t = torch.tensor([300.0], device=gpu)
    m32 = _twin(m)
    with ops.ops_mode("reference"):
        emb_r = m32.controlnet_cond_embedding(cond_img.float())
        downs_r, mid_r = m32(x.float(), t, emb_r, ctx=ctx.float())
    emb = m.controlnet_cond_embedding(cond_img)
    downs, mid = m(x, t, emb, cross_kv=[mm.context_kv(ctx) for mm in m.cross_attention_modules()])
    assert len(downs) == len(downs_r) == 12
    for i, (d, dr) in enumerate(zip(downs, downs_r)):
        assert rel_err(d, dr, f"controlnet down {i}" if i in (0, 11) else "") <= 2e-2, i
    assert rel_err(mid, mid_r, "controlnet mid") <= 2e-2


@torch.no_grad()
def test_esrgan_rrdbnet_parity_vs_fp32(gpu):
    from chiaswarm_amd.models.rrdbnet import RRDBNet

    with torch.device(gpu):
        m = RRDBNet().to(torch.bfloat16).eval().requires_grad_(False)
    init_random_fast_(m, seed=5, std_scale=0.5)
    prepare_model(m)
    x = torch.rand(1, 64, 64, 3, device=gpu)
    m32 = _twin(m)
    with ops.ops_mode("reference"):
        ref = m32(x)
    y = m(x)
    assert y.shape == (1, 256, 256, 3)
    assert rel_err(y, ref, "rrdbnet x4") <= 2e-2
