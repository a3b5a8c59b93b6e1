"""Sampling-loop variant classes (pipelines/guided.py):
StableDiffusionPanoramaPipeline (MultiDiffusion), StableDiffusionSAGPipeline
(self-attention guidance), StableDiffusionPipelineSafe (safe latent diffusion),
SemanticStableDiffusionPipeline (SEGA) and StableDiffusionAttendAndExcitePipeline, reachable by class name like every diffusers class
the reference builds by reflection (swarm/job_arguments.py:143-145,
swarm/type_helpers.py:1-3).

diffusers is not importable here, so pipeline-level parity is unpinned; these
tests pin the pieces against their formulas and the degenerate cases against
the plain pipeline: one window == the plain txt2img loop, sag_scale = 0 == the
plain loop, the window geometry, per-window sampler state, the SAG mask / blur,
routing, and the never-batched / never-split rule.  The SEGA guidance is
checked against a transcription of diffusers 0.16.1's edit-guidance block
(the reference's pinned version) made for this test — parity with diffusers
itself is unpinned."""
import base64
import io

import pytest
import torch
from PIL import Image

from chiaswarm_amd.jobs import router
from chiaswarm_amd.pipelines import diffusion, guided
from chiaswarm_amd.pipelines.sd import StableDiffusion
from chiaswarm_amd.runtime import worker
from chiaswarm_amd.schedulers import get_scheduler


def _size(res):
    return Image.open(io.BytesIO(base64.b64decode(res["primary"]["blob"]))).size


def test_panorama_views_geometry():
    v = guided.panorama_views(64, 256)  # 512 x 2048 px, diffusers' default canvas
    assert len(v) == 25 and v[0] == (0, 64, 0, 64) and v[-1] == (0, 64, 192, 256)
    assert guided.panorama_views(64, 64) == [(0, 64, 0, 64)]
    assert len(guided.panorama_views(80, 128)) == 3 * 9
    c = guided.panorama_views(64, 128, circular=True)
    assert len(c) == 16 and c[-1] == (0, 64, 120, 184)  # wraps 56 columns round the seam
    # every latent pixel is covered, by the circular views too
    for views, lw in ((guided.panorama_views(64, 136), 136), (c, 128)):
        cnt = torch.zeros(64, lw)
        x = torch.zeros(1, 64, lw, 1)
        for w in views:
            guided._accumulate(x, cnt.view(1, 64, lw, 1), torch.ones(1, 64, 64, 1), w, lw)
        assert (cnt > 0).all()


def test_panorama_one_window_is_plain_txt2img():
    pipe = StableDiffusion("tiny", device="cpu", seed=3)
    kw = dict(prompt="a castle", num_inference_steps=4, guidance_scale=5.0, height=64, width=64,
              output_type="latent")
    ref = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
    got = guided.run_panorama(pipe, generator=torch.Generator().manual_seed(0), **kw).latents
    assert torch.allclose(got, ref, atol=1e-5, rtol=1e-5), (got - ref).abs().max()
    assert pipe.__dict__.get("_denoise_override") is None and "decode" not in pipe.__dict__


def test_panorama_wide_and_circular():
    pipe = StableDiffusion("tiny", device="cpu", seed=3)
    a = guided.run_panorama(pipe, prompt="a", num_inference_steps=3, height=64, width=128,
                            generator=torch.Generator().manual_seed(1))
    assert a.images[0].size == (128, 64) and torch.isfinite(a.latents).all()
    b = guided.run_panorama(pipe, prompt="a", num_inference_steps=3, height=64, width=128, circular_padding=True,
                            generator=torch.Generator().manual_seed(1))
    assert b.images[0].size == (128, 64)
    assert not torch.equal(a.latents, b.latents)  # the seam windows change the canvas
    with pytest.raises(TypeError, match="unexpected"):
        guided.run_panorama(pipe, prompt="a", num_inference_steps=2, image=Image.new("RGB", (64, 64)))


def test_panorama_windows_keep_their_own_sampler_history():
    """DPM-Solver++(2M) is multistep: each window keeps its own previous x0
    (diffusers copies the scheduler state per view)."""
    pipe = StableDiffusion("tiny", device="cpu", seed=3)
    seen = []
    orig = guided.copy.deepcopy

    def spy(o):
        c = orig(o)
        seen.append(c)
        return c

    guided.copy.deepcopy = spy
    try:
        guided.run_panorama(pipe, prompt="a", num_inference_steps=3, height=64, width=80, output_type="latent",
                            scheduler=get_scheduler("DPMSolverMultistepScheduler"),
                            generator=torch.Generator().manual_seed(0))
    finally:
        guided.copy.deepcopy = orig
    assert len(seen) == 3  # three 8-wide windows over 10 latent columns
    assert all(s.step_index == 3 for s in seen)
    assert not torch.equal(seen[0].prev_x0, seen[2].prev_x0)


def test_gaussian_blur_and_sag_mask():
    x = torch.full((1, 9, 9, 4), 3.0)
    assert torch.allclose(guided.gaussian_blur_nhwc(x), x, atol=1e-6)
    y = torch.zeros(1, 17, 17, 1)
    y[0, 8, 8, 0] = 1.0  # an impulse far enough from the reflected border: the blur is the kernel
    b = guided.gaussian_blur_nhwc(y)
    k = torch.exp(-0.5 * torch.arange(-4.0, 5.0) ** 2)
    k = k / k.sum()
    assert torch.allclose(b[0, 4:13, 4:13, 0], k[:, None] * k[None, :], atol=1e-7)
    y2 = torch.zeros(1, 9, 9, 1)
    y2[0, 1, 4, 0] = 1.0  # next to the border: reflect padding (row -1 reads row 1) counts it twice in row 0
    b2 = guided.gaussian_blur_nhwc(y2)
    assert torch.allclose(b2[0, 0, 4, 0], k[3] * k[4] + k[5] * k[4], atol=1e-7)
    s = 16
    uniform = torch.full((2, 3, s, s), 1.0 / s)
    assert guided.sag_mask(uniform, 8, 8).sum() == 0
    peaked = torch.zeros(2, 3, s, s)
    peaked[..., 5] = 1.0  # every query attends to key 5 (row 1, col 1 of the 4 x 4 grid)
    m = guided.sag_mask(peaked, 8, 8)
    assert m.shape == (2, 8, 8, 1) and m.sum() == 2 * 4
    assert m[0, 2:4, 2:4].eq(1).all()


def test_sag_scale_zero_is_plain_and_guidance_changes_result():
    pipe = StableDiffusion("tiny", device="cpu", seed=4)
    kw = dict(prompt="a dog", num_inference_steps=4, guidance_scale=6.0, output_type="latent")
    ref = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
    z = guided.run_sag(pipe, sag_scale=0.0, generator=torch.Generator().manual_seed(0), **kw).latents
    assert torch.allclose(z, ref, atol=1e-5, rtol=1e-5), (z - ref).abs().max()
    g = guided.run_sag(pipe, sag_scale=0.75, generator=torch.Generator().manual_seed(0), **kw).latents
    assert torch.isfinite(g).all() and not torch.allclose(g, ref)
    # no CFG: the conditional pass is the reference; k-space sampler; two-stage sampler
    for sched in ("EulerDiscreteScheduler", "HeunDiscreteScheduler", "DDIMScheduler"):
        o = guided.run_sag(pipe, prompt="a", num_inference_steps=3, guidance_scale=1.0, output_type="latent",
                           scheduler=get_scheduler(sched), generator=torch.Generator().manual_seed(0))
        assert torch.isfinite(o.latents).all(), sched
    assert pipe.unet.mid_block.attentions[0].transformer_blocks[0].attn1.__dict__.get("_store_probs") is None


def test_safe_latent_diffusion():
    pipe = StableDiffusion("tiny", device="cpu", seed=6)
    kw = dict(prompt="a street", num_inference_steps=4, guidance_scale=6.0, output_type="latent")
    ref = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
    # safety guidance off (sld_guidance_scale <= 1): the plain pipeline
    off = guided.run_safe(pipe, sld_guidance_scale=1.0, generator=torch.Generator().manual_seed(0), **kw)
    assert torch.equal(off.latents, ref)
    # on, but still warming up for every step: the CFG-3 batch gives the plain CFG result
    warm = guided.run_safe(pipe, sld_warmup_steps=100, generator=torch.Generator().manual_seed(0), **kw)
    assert torch.allclose(warm.latents, ref, atol=1e-5, rtol=1e-5), (warm.latents - ref).abs().max()
    assert warm.applied_safety_concept == guided.SAFETY_CONCEPT
    on = guided.run_safe(pipe, sld_warmup_steps=0, sld_threshold=1.0, generator=torch.Generator().manual_seed(0), **kw)
    assert torch.isfinite(on.latents).all() and not torch.allclose(on.latents, ref)
    # a different concept changes the safety direction
    other = guided.run_safe(pipe, sld_warmup_steps=0, sld_threshold=1.0, safety_concept="a cat",
                            generator=torch.Generator().manual_seed(0), **kw)
    assert not torch.equal(other.latents, on.latents)


def test_routing_and_jobs_end_to_end():
    for cls in guided.CLASSES:
        _, kw = router.format_args({"model_name": "m", "parameters": {"pipeline_type": cls}})
        assert kw["pipeline_type"] == cls
        job = {"model_name": "m", "prompt": "x", "num_images_per_prompt": 3, "parameters": {"pipeline_type": cls}}
        assert worker._raw_key(job) is None and worker.splittable(job) == 0 and not worker.cfg_splittable(job)
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type=guided.PANORAMA, prompt="a beach",
                                            height=64, width=128, num_inference_steps=2, generator=g,
                                            scheduler_type="DDIMScheduler", upscale=False, supports_xformers=True)
    assert cfg["_pipeline_type"] == guided.PANORAMA and _size(res) == (128, 64)
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type=guided.SAG, prompt="a beach",
                                            num_inference_steps=2, sag_scale=0.5, generator=g,
                                            scheduler_type="DPMSolverMultistepScheduler", upscale=False,
                                            supports_xformers=True)
    assert cfg["_pipeline_type"] == guided.SAG and _size(res) == (64, 64)
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type=guided.SAFE, prompt="a beach",
                                            num_inference_steps=2, sld_warmup_steps=0, generator=g,
                                            scheduler_type="DPMSolverMultistepScheduler", upscale=False,
                                            supports_xformers=True)
    assert cfg["_pipeline_type"] == guided.SAFE and _size(res) == (64, 64)
    with pytest.raises(TypeError, match="sag_scale"):  # a Panorama-only / SAG-only kwarg elsewhere
        diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type="StableDiffusionPipeline", prompt="a",
                                     num_inference_steps=2, sag_scale=0.5, generator=torch.Generator().manual_seed(0),
                                     upscale=False)
    with pytest.raises(ValueError, match="batch"):
        diffusion.diffusion_batch("cpu", [dict(model_name="tiny/sd", pipeline_type=guided.SAG, prompt="a",
                                               generator=torch.Generator().manual_seed(0))])


@pytest.mark.gpu
def test_panorama_and_sag_on_gpu(gpu):
    pipe = StableDiffusion("tiny", device=gpu, seed=5)
    out = guided.run_panorama(pipe, prompt="a", num_inference_steps=3, height=64, width=128,
                              generator=torch.Generator(device=gpu).manual_seed(0))
    assert out.images[0].size == (128, 64) and torch.isfinite(out.latents).all()
    out = guided.run_sag(pipe, prompt="a", num_inference_steps=3, generator=torch.Generator(device=gpu).manual_seed(0))
    assert len(out.images) == 1 and torch.isfinite(out.latents).all()
    out = guided.run_safe(pipe, prompt="a", num_inference_steps=3, sld_warmup_steps=0,
                          generator=torch.Generator(device=gpu).manual_seed(0))
    assert len(out.images) == 1 and torch.isfinite(out.latents).all()
    out = guided.run_sega(pipe, prompt="a", num_inference_steps=3, editing_prompt=["b", "c"], edit_warmup_steps=0,
                          generator=torch.Generator(device=gpu).manual_seed(0))
    assert len(out.images) == 1 and torch.isfinite(out.latents).all()
    # Attend-and-Excite: the gradient passes run the torch implementation of the ops on the HIP-prepared
    # model (mode switched for those passes only), the denoising steps the HIP graph
    from chiaswarm_amd import ops

    kw = dict(prompt="a cat and a frog", num_inference_steps=3, height=128, width=128, output_type="latent")
    ref = pipe(generator=torch.Generator(device=gpu).manual_seed(0), **kw).latents
    out = guided.run_attend_and_excite(pipe, token_indices=[2, 5], max_iter_to_alter=2, thresholds={0: 0.99},
                                       generator=torch.Generator(device=gpu).manual_seed(0), **kw)
    assert ops.get_mode() == "hip" and torch.isfinite(out.latents).all() and not torch.allclose(out.latents, ref)


def _sega_reference(i, e_u, e_t, edits, gs, opt, mom, n_steps):
    """diffusers 0.16.1 SemanticStableDiffusionPipeline's edit-guidance block,
    transcribed on [b, C, H, W] tensors (the layout diffusers uses)."""
    k = len(edits)
    lst = lambda v: list(v) if isinstance(v, (list, tuple)) else [v] * k  # noqa: E731
    scale, warmup, thr, rev = lst(opt["edit_guidance_scale"]), lst(opt["edit_warmup_steps"]), \
        lst(opt["edit_threshold"]), lst(opt["reverse_editing_direction"])
    cool = [n_steps + 1 if v is None else v for v in lst(opt["edit_cooldown_steps"])]
    wts = lst(opt["edit_weights"]) if opt["edit_weights"] is not None else [1.0] * k
    ng = gs * (e_t - e_u)
    cw = torch.zeros(k, ng.shape[0])
    nge = torch.zeros((k,) + tuple(ng.shape))
    warm = []
    for c, ec in enumerate(edits):
        if i >= warmup[c]:
            warm.append(c)
        if i >= cool[c]:
            nge[c] = torch.zeros_like(ec)
            continue
        t = ec - e_u
        if rev[c]:
            t = t * -1
        cw[c, :] = wts[c]
        t = t * scale[c]
        q = torch.quantile(torch.abs(t).flatten(start_dim=2), thr[c], dim=2, keepdim=False)
        nge[c] = torch.where(torch.abs(t) >= q[:, :, None, None], t, torch.zeros_like(t))
    wi = torch.tensor(warm, dtype=torch.long)
    if k > wi.shape[0] > 0:
        cwt = torch.index_select(cw, 0, wi)
        cwt = torch.where(cwt < 0, torch.zeros_like(cwt), cwt)
        cwt = cwt / cwt.sum(dim=0)
        ng = ng + torch.einsum("cb,cbijk->bijk", cwt, torch.index_select(nge, 0, wi))
    cw = torch.nan_to_num(torch.where(cw < 0, torch.zeros_like(cw), cw))
    edit = torch.einsum("cb,cbijk->bijk", cw, nge) + opt["edit_momentum_scale"] * mom
    mom = opt["edit_mom_beta"] * mom + (1 - opt["edit_mom_beta"]) * edit
    if wi.shape[0] == k:
        ng = ng + edit
    return ng, mom


@pytest.mark.parametrize("opt", [
    dict(edit_guidance_scale=5.0, edit_warmup_steps=1, edit_cooldown_steps=None, edit_threshold=0.9,
         reverse_editing_direction=False, edit_weights=None, edit_momentum_scale=0.1, edit_mom_beta=0.4),
    dict(edit_guidance_scale=[3.0, 7.0], edit_warmup_steps=[0, 2], edit_cooldown_steps=[None, 3],
         edit_threshold=[0.8, 0.95], reverse_editing_direction=[True, False], edit_weights=[0.7, 1.6],
         edit_momentum_scale=0.3, edit_mom_beta=0.6),
])
def test_sega_guidance_matches_the_diffusers_block(opt):
    torch.manual_seed(0)
    b, C, H, W, steps = 2, 4, 8, 8, 5
    k = 2 if isinstance(opt["edit_guidance_scale"], list) else 1
    st = guided.SegaState(k, steps, **opt)
    mom = torch.zeros(b, C, H, W)
    for i in range(steps):
        e_u, e_t = torch.randn(b, C, H, W), torch.randn(b, C, H, W)
        edits = [torch.randn(b, C, H, W) for _ in range(k)]
        want, mom = _sega_reference(i, e_u, e_t, edits, 7.5, opt, mom, steps)
        nhwc = lambda t: t.permute(0, 2, 3, 1)  # noqa: E731  (this repo's latent layout)
        got = st.guidance(i, nhwc(e_u), nhwc(e_t), [nhwc(e) for e in edits], 7.5)
        assert torch.allclose(got, nhwc(want), atol=1e-5, rtol=1e-5), (i, (got - nhwc(want)).abs().max())


def test_sega_pipeline():
    pipe = StableDiffusion("tiny", device="cpu", seed=7)
    kw = dict(prompt="a house", num_inference_steps=4, guidance_scale=6.0, output_type="latent")
    ref = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
    plain = guided.run_sega(pipe, generator=torch.Generator().manual_seed(0), **kw)  # no editing prompt
    assert torch.equal(plain.latents, ref)
    # edits still warming up for every step: the CFG-(2 + k) batch gives the plain CFG result
    warm = guided.run_sega(pipe, editing_prompt=["snow", "night"], edit_warmup_steps=100,
                           generator=torch.Generator().manual_seed(0), **kw)
    assert torch.allclose(warm.latents, ref, atol=1e-5, rtol=1e-5), (warm.latents - ref).abs().max()
    on = guided.run_sega(pipe, editing_prompt="snow", edit_warmup_steps=0,
                         generator=torch.Generator().manual_seed(0), **kw)
    assert torch.isfinite(on.latents).all() and not torch.allclose(on.latents, ref)
    rev = guided.run_sega(pipe, editing_prompt="snow", edit_warmup_steps=0, reverse_editing_direction=True,
                          generator=torch.Generator().manual_seed(0), **kw)
    assert not torch.allclose(rev.latents, on.latents)
    with pytest.raises(ValueError, match="edit_weights"):
        guided.run_sega(pipe, editing_prompt=["a", "b"], edit_weights=[1.0], **kw)
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type=guided.SEGA, prompt="a beach",
                                            num_inference_steps=2, editing_prompt=["sunset"], edit_warmup_steps=0,
                                            generator=g, scheduler_type="DDIMScheduler", upscale=False,
                                            supports_xformers=True)
    assert cfg["_pipeline_type"] == guided.SEGA and _size(res) == (64, 64)


def test_attend_and_excite_pieces():
    k = guided.ae_gauss_kernel()
    g = torch.exp(-((torch.tensor([-1.0, 0.0, 1.0]) / 1.0) ** 2))  # (x / (2 * 0.5))^2
    want = g[:, None] * g[None, :]
    assert torch.allclose(k, want / want.sum(), atol=1e-7)
    # one map, all queries attend to token 3 (index 3 = the 3rd prompt token): its max is ~1, the others ~0
    res, skv = 4, 8
    p = torch.full((1, 2, res * res, skv), 1e-4)
    p[..., 3] = 1.0
    m = guided.ae_max_attention([p], [3, 5], res)
    assert m[0].item() > 0.99 and m[1].item() < 0.01
    assert abs(guided.ae_loss(m).item() - (1 - m[1].item())) < 1e-6


def test_attend_and_excite_pipeline():
    pipe = StableDiffusion("tiny", device="cpu", seed=8)
    kw = dict(prompt="a cat and a frog", num_inference_steps=4, guidance_scale=6.0, height=128, width=128,
              output_type="latent")
    ref = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
    off = guided.run_attend_and_excite(pipe, token_indices=[2, 5], max_iter_to_alter=0,
                                       generator=torch.Generator().manual_seed(0), **kw)
    assert torch.allclose(off.latents, ref, atol=1e-5, rtol=1e-5), (off.latents - ref).abs().max()
    on = guided.run_attend_and_excite(pipe, token_indices=[2, 5], max_iter_to_alter=3, thresholds={"0": 0.99},
                                      generator=torch.Generator().manual_seed(0), **kw)
    assert torch.isfinite(on.latents).all() and not torch.allclose(on.latents, ref)
    for m in pipe.unet.modules():
        assert "_store_probs" not in m.__dict__
    with pytest.raises(TypeError, match="token_indices"):
        guided.run_attend_and_excite(pipe, **kw)
    with pytest.raises(ValueError, match="one prompt"):
        guided.run_attend_and_excite(pipe, token_indices=[2], num_images_per_prompt=2, **kw)
    with pytest.raises(ValueError, match="attn_res"):  # 64 px: no 16 x 16 maps
        guided.run_attend_and_excite(pipe, token_indices=[2], prompt="a", num_inference_steps=2, height=64, width=64)
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type=guided.AE, prompt="a red cube",
                                            token_indices=[2], max_iter_to_alter=1, height=128, width=128,
                                            num_inference_steps=2, generator=g, scheduler_type="DDIMScheduler",
                                            upscale=False, supports_xformers=True)
    assert cfg["_pipeline_type"] == guided.AE and _size(res) == (128, 128)
