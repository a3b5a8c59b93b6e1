"""Device-resident sampler loop (pipelines/sd.py::_denoise_loop: one hipGraph
replay per step, sched_loop_kernel writing the next UNet input) against the
per-step host loop (fused sched_step + torch glue) on the same pipeline and
seeds, plus the sched_loop kernel itself against an fp32 PyTorch reference."""
import pytest
import torch

from chiaswarm_amd.pipelines import sd as sd_mod
from chiaswarm_amd.pipelines.sd import StableDiffusion
from chiaswarm_amd.schedulers import get_scheduler

pytestmark = pytest.mark.gpu


def _run(pipe, dev, loop, sched_name, guidance=7.5, steps=6, **kw):
    sd_mod.LOOP_GRAPHS = loop
    try:
        g = torch.Generator(device=dev).manual_seed(11)
        out = pipe(prompt="a red fox", negative_prompt="blur", num_inference_steps=steps, guidance_scale=guidance,
                   num_images_per_prompt=2, height=64, width=64, generator=g,
                   scheduler=get_scheduler(sched_name), output_type="latent", **kw)
        torch.cuda.synchronize()
        return out.latents.float()
    finally:
        sd_mod.LOOP_GRAPHS = True


@pytest.mark.parametrize("sched_name,guidance", [("DPMSolverMultistepScheduler", 7.5),
                                                 ("EulerAncestralDiscreteScheduler", 5.0),
                                                 ("DDIMScheduler", 1.0)])
def test_loop_matches_host_loop(gpu, sched_name, guidance):
    pipe = StableDiffusion("tiny", device=gpu, seed=0)
    a = _run(pipe, gpu, False, sched_name, guidance)
    b = _run(pipe, gpu, True, sched_name, guidance)
    assert torch.isfinite(b).all()
    err = ((a - b).norm() / a.norm()).item()
    assert err < 1e-3, err
    # a second request through the cached loop graph (new guidance / step count) stays consistent
    a2 = _run(pipe, gpu, False, sched_name, guidance + 1.0, steps=9)
    b2 = _run(pipe, gpu, True, sched_name, guidance + 1.0, steps=9)
    assert ((a2 - b2).norm() / a2.norm()).item() < 1e-3


def test_sched_loop_kernel_vs_torch(gpu):
    from chiaswarm_amd.ops import hip_ops

    B, H, W = 2, 8, 8
    n = 5
    for mode in (0, 1, 2):
        nrep = mode + 1
        cin = 9 if mode == 1 else (8 if mode == 2 else 4)
        x = torch.randn(B, H, W, 4, device=gpu)
        prev = torch.randn(B, H, W, 4, device=gpu)
        e = torch.randn(nrep * B, H, W, 4, device=gpu).bfloat16()
        coef = torch.randn(n, hip_ops.LOOP_COEF_STRIDE, device=gpu)
        noise = torch.randn(n, B, H, W, 4, device=gpu)
        cur = torch.tensor([3], dtype=torch.int32, device=gpu)
        x_in = torch.randn(nrep * B, H, W, cin, device=gpu).bfloat16()
        extra = x_in[..., 4:].clone()
        xr, pr = x.clone(), prev.clone()
        hip_ops.sched_loop(e, x, prev, noise, cur, coef, x_in, mode)
        c = coef[3].tolist()
        ef = e.float()
        if mode == 0:
            eg = ef
        elif mode == 1:
            u, cc = ef.chunk(2)
            eg = u + c[7] * (cc - u)
        else:
            cc, i, u = ef.chunk(3)
            eg = u + c[7] * (cc - i) + c[8] * (i - u)
        x0 = c[0] * xr + c[1] * eg
        xn = c[2] * xr + c[3] * x0 + c[4] * pr + c[5] * noise[3]
        torch.testing.assert_close(x, xn, rtol=1e-4, atol=1e-4)
        torch.testing.assert_close(prev, x0, rtol=1e-4, atol=1e-4)
        want = (xn * c[6]).bfloat16()
        for r in range(nrep):
            torch.testing.assert_close(x_in[r * B:(r + 1) * B, ..., :4].float(), want.float(), rtol=1e-2, atol=1e-2)
        assert torch.equal(x_in[..., 4:], extra)  # image-latent channels untouched


def test_sdxl_loop_matches_host_loop(gpu):
    """SDXL in the device loop (the text_time addition embedding from the
    graph's per-request buffer) — same latents as the per-step host loop,
    across two requests with different prompts."""
    pipe = StableDiffusion("sdxl", device=gpu, seed=0)
    for prompt in ("a red fox", "a blue car"):
        outs = []
        for loop in (False, True):
            sd_mod.LOOP_GRAPHS = loop
            try:
                g = torch.Generator(device=gpu).manual_seed(5)
                out = pipe(prompt=prompt, negative_prompt="blur", num_inference_steps=4, guidance_scale=5.0,
                           num_images_per_prompt=1, height=128, width=128, generator=g,
                           scheduler=get_scheduler("EulerDiscreteScheduler"), output_type="latent")
                torch.cuda.synchronize()
                outs.append(out.latents.float())
            finally:
                sd_mod.LOOP_GRAPHS = True
        a, b = outs
        assert torch.isfinite(b).all()
        assert ((a - b).norm() / a.norm()).item() < 1e-3, prompt
