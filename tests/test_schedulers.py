"""Closed-form sampler checks (no diffusers available: SURVEY §7.4 hard part 3).

With an oracle denoiser that returns the exact noise / velocity of the current
sample for a known clean x0, every deterministic sampler must land on x0 at
sigma = 0; Karras ladders and timestep mapping are checked against their
defining formulas."""
import math

import numpy as np
import pytest
import torch

from chiaswarm_amd.schedulers import get_scheduler, karras_sigmas, scheduler_names

DET = ["DPMSolverMultistepScheduler", "EulerDiscreteScheduler", "DDIMScheduler", "LMSDiscreteScheduler",
       "HeunDiscreteScheduler", "PNDMScheduler"]


def oracle(s, x, x0, pred):
    """Exact model output for sample x at the scheduler's current evaluation."""
    if s.space == "vp":
        sig = s.sigmas[s.step_index]
        if hasattr(s, "eval_sigma"):
            sig = s.eval_sigma()
        a = 1 / math.sqrt(sig * sig + 1)
        sv = sig * a
        eps = (x - a * x0) / sv
        return eps if pred == "epsilon" else a * eps - sv * x0
    sig = s.eval_sigma() if hasattr(s, "eval_sigma") else s.sigmas[s.step_index]
    eps = (x - x0) / sig
    if pred == "epsilon":
        return eps
    a = 1 / math.sqrt(sig * sig + 1)
    return a * eps - sig * a * x0  # v = alpha*eps - sigma_vp*x0 on the VP-scaled sample


@pytest.mark.parametrize("name", DET)
@pytest.mark.parametrize("n", [4, 10, 30])
def test_oracle_recovers_x0(name, n):
    torch.manual_seed(0)
    x0 = torch.randn(2, 8, 8, 4)
    s = get_scheduler(name, prediction_type="epsilon")
    s.set_timesteps(n)
    x = torch.randn_like(x0) * s.init_noise_sigma
    if s.space == "vp":
        x = s.add_noise(x0, torch.randn_like(x0), 0)
    while s.step_index < s.n:
        x = s.step(oracle(s, x, x0, "epsilon"), x)
    if name in ("DDIMScheduler", "PNDMScheduler"):
        # DDIM ends at alphas_cumprod[0] (set_alpha_to_one=False), not at sigma 0
        assert (s.prev_x0 - x0).abs().max().item() < 1e-4
        a0 = 1 / math.sqrt(s.sigmas[-1] ** 2 + 1)
        assert (x - a0 * x0).abs().max().item() < 6 * s.sigmas[-1] * a0
    else:
        assert (x - x0).abs().max().item() < 1e-4


@pytest.mark.parametrize("name", ["DPMSolverMultistepScheduler", "DDIMScheduler"])
def test_oracle_v_prediction(name):
    x0 = torch.randn(1, 8, 8, 4)
    s = get_scheduler(name, prediction_type="v_prediction")
    s.set_timesteps(12)
    x = s.add_noise(x0, torch.randn_like(x0), 0)
    while s.step_index < s.n:
        x = s.step(oracle(s, x, x0, "v_prediction"), x)
    assert (s.prev_x0 - x0).abs().max().item() < 1e-4


def test_karras_ladder():
    s = get_scheduler("DPMSolverMultistepScheduler")
    s.set_timesteps(50)
    sig = s.sigmas[:-1]
    assert s.sigmas[-1] == 0.0
    assert np.all(np.diff(sig) < 0)
    ref = karras_sigmas(s.train_sigmas[0], s.train_sigmas[-1], 50)
    np.testing.assert_allclose(sig, ref, rtol=1e-6)
    # rho=7 spacing: sigma^(1/7) is linear in the step index
    r = sig ** (1 / 7)
    np.testing.assert_allclose(np.diff(r), np.full(49, np.diff(r).mean()), rtol=1e-6)
    assert s.timesteps[0] == 999.0 and s.timesteps[-1] < 5


def test_sigma_to_t_roundtrip():
    s = get_scheduler("EulerDiscreteScheduler")
    for t in [0, 10, 250, 500, 999]:
        assert abs(s.sigma_to_t(float(s.train_sigmas[t])) - t) < 1e-6


def test_ancestral_adds_noise_and_is_seeded():
    s = get_scheduler("EulerAncestralDiscreteScheduler")
    s.set_timesteps(10)
    x = torch.randn(1, 4, 4, 4) * s.init_noise_sigma
    e = torch.zeros_like(x)
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    a = s.step(e, x.clone(), g1)
    s.reset()
    b = s.step(e, x.clone(), g2)
    assert torch.equal(a, b)
    c = s.coeffs(0)
    assert c.D > 0


def test_registry_and_unknown():
    assert "DPMSolverMultistepScheduler" in scheduler_names()
    assert "UniPCMultistepScheduler" in scheduler_names()
    with pytest.raises(ValueError):
        get_scheduler("NoSuchScheduler")


def test_fused_coeffs_match_step():
    """The linear-form coefficients (fed to the HIP step kernel) reproduce step()."""
    from chiaswarm_amd import ops

    for name in ["DPMSolverMultistepScheduler", "EulerDiscreteScheduler", "DDIMScheduler"]:
        s1, s2 = get_scheduler(name), get_scheduler(name)
        s1.set_timesteps(8)
        s2.set_timesteps(8)
        x = torch.randn(1, 4, 4, 4)
        x1, x2 = x.clone(), x.clone()
        for _ in range(8):
            e = torch.randn_like(x)
            x1 = s1.step(e, x1)
            c = s2.fused_coeffs()
            out, x0 = ops._ref_sched_step(e, x2, s2.prev_x0, c, None, None)
            s2.prev_x0, s2.step_index, x2 = x0, s2.step_index + 1, out
        assert torch.allclose(x1, x2, atol=1e-5)


# --------------------------------------------------------------------------
# Gaussian data: the probability-flow ODE has a closed form, so each sampler's
# integration error is measurable (no diffusers needed).  x0 ~ N(mu, s^2):
#   D(x, sigma) = (s^2 x + sigma^2 mu) / (s^2 + sigma^2)   (exact denoiser)
#   x(sigma)    = mu + (x(sigma_0) - mu) * sqrt(s^2 + sigma^2) / sqrt(s^2 + sigma_0^2)
# --------------------------------------------------------------------------
MU, SD = 0.5, 0.8
ALL_DET = ["DPMSolverMultistepScheduler", "DPMSolverSinglestepScheduler", "UniPCMultistepScheduler",
           "DEISMultistepScheduler", "EulerDiscreteScheduler", "HeunDiscreteScheduler", "KDPM2DiscreteScheduler",
           "LMSDiscreteScheduler", "DDIMScheduler", "PNDMScheduler"]
STOCH = ["EulerAncestralDiscreteScheduler", "KDPM2AncestralDiscreteScheduler", "DPMSolverSDEScheduler",
         "DDPMScheduler"]


def _gauss_eps(s, x):
    sig = s.eval_sigma()
    xk = x * math.sqrt(sig * sig + 1) if s.space == "vp" else x
    d = (SD * SD * xk + sig * sig * MU) / (SD * SD + sig * sig)
    return (xk - d) / sig


def _run_gauss(name, n, z, generator=None):
    s = get_scheduler(name)
    s.set_timesteps(n)
    s0 = float(s.sigmas[0]) if not hasattr(s, "plms") else float(s.train_sigmas[int(s.plms[0])])
    xk0 = MU + z * math.sqrt(SD * SD + s0 * s0)
    x = xk0 / math.sqrt(s0 * s0 + 1) if s.space == "vp" else xk0
    while s.step_index < s.n:
        x = s.step(_gauss_eps(s, x), x, generator)
    s_end = float(s.sigmas[-1])
    exact = MU + (xk0 - MU) * math.sqrt(SD * SD + s_end * s_end) / math.sqrt(SD * SD + s0 * s0)
    if s.space == "vp":
        exact = exact / math.sqrt(s_end * s_end + 1)
    return x, exact


@pytest.mark.parametrize("n", [10, 25])
def test_every_deterministic_sampler_integrates_the_gaussian_ode(n):
    z = torch.randn(4096, generator=torch.Generator().manual_seed(0), dtype=torch.float64).float()
    err = {}
    for name in ALL_DET:
        x, exact = _run_gauss(name, n, z)
        err[name] = (x - exact).abs().max().item()
    # (the common floor: every sampler's last step returns the denoised sample
    # at sigma_min, an O(sigma_min^2) error of the ODE solution itself)
    assert all(e < (0.6 if n == 10 else 0.3) for e in err.values()), err
    # second-order methods beat first-order Euler on the same ladder family
    for name in ("DPMSolverMultistepScheduler", "DPMSolverSinglestepScheduler", "UniPCMultistepScheduler",
                 "DEISMultistepScheduler", "LMSDiscreteScheduler", "HeunDiscreteScheduler", "KDPM2DiscreteScheduler"):
        assert err[name] < err["EulerDiscreteScheduler"], (name, err)


def test_solver_errors_shrink_with_steps():
    z = torch.randn(1024, generator=torch.Generator().manual_seed(1))
    for name in ("UniPCMultistepScheduler", "DEISMultistepScheduler", "DPMSolverSinglestepScheduler",
                 "LMSDiscreteScheduler", "KDPM2DiscreteScheduler", "PNDMScheduler"):
        e = []
        for n in (8, 16, 32):
            x, exact = _run_gauss(name, n, z)
            e.append((x - exact).abs().max().item())
        assert e[2] < e[0], (name, e)


@pytest.mark.parametrize("name", STOCH)
def test_stochastic_samplers_sample_the_data_distribution(name):
    g = torch.Generator().manual_seed(2)
    z = torch.randn(20000, generator=g)
    x, _ = _run_gauss(name, 100, z, generator=g)
    s = get_scheduler(name)
    s.set_timesteps(100)
    s_end = float(s.sigmas[-1])
    xk = x * math.sqrt(s_end * s_end + 1) if s.space == "vp" else x
    # ancestral samplers under-disperse by O(1/n) (Euler-a's per-step variance
    # deficit s^2 (sigma - sigma_down)^2 / (s^2 + sigma^2)); at 100 steps < 5 %
    assert abs(xk.mean().item() - MU) < 0.02
    assert abs(xk.std().item() - math.sqrt(SD * SD + s_end * s_end)) < 0.04


def test_lms_coefficients_integrate_lagrange_basis():
    s = get_scheduler("LMSDiscreteScheduler")
    s.set_timesteps(12)
    for i in range(3, 11):
        c = [s.lms_coeff(4, i, k) for k in range(4)]
        assert abs(sum(c) - (s.sigmas[i + 1] - s.sigmas[i])) < 1e-9  # basis sums to 1
    assert abs(s.lms_coeff(1, 0, 0) - (s.sigmas[1] - s.sigmas[0])) < 1e-12  # order 1 == Euler


def test_pndm_plms_schedule_repeats_second_timestep():
    s = get_scheduler("PNDMScheduler")
    s.set_timesteps(10)
    assert s.n == 11 and s.plms[1] == s.plms[2] and s.plms[0] == 901 and s.plms[-1] == 1


def test_no_scheduler_is_an_alias():
    from chiaswarm_amd.schedulers import _ALIASES, _REGISTRY

    assert not _ALIASES
    for n in scheduler_names():
        assert type(get_scheduler(n)).__name__ == n


def test_dynamic_thresholding_matches_imagen_rule():
    """IF's samplers threshold x0 per sample (diffusers DDPMScheduler
    _threshold_sample semantics): s = clamp(quantile(|x0|, r), 1, max)."""
    import torch

    from chiaswarm_amd.schedulers import get_scheduler

    sch = get_scheduler("DDPMScheduler", thresholding=True, dynamic_thresholding_ratio=0.95,
                        sample_max_value=1.5, use_karras_sigmas=False)
    assert sch.fused_coeffs() is None  # non-linear: never the fused kernel
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(3, 8, 8, 3, generator=g) * torch.tensor([0.3, 1.2, 9.0]).reshape(3, 1, 1, 1)
    y = sch.threshold_x0(x0)
    for b in range(3):
        s = min(max(torch.quantile(x0[b].abs().flatten(), 0.95).item(), 1.0), 1.5)
        ref = x0[b].clamp(-s, s) / s
        assert torch.allclose(y[b], ref, atol=1e-6)
    assert y[0].equal(x0[0].clamp(-1, 1))  # quantile < 1 -> s = 1: a plain [-1, 1] clip
    assert y.abs().max() <= 1.0 + 1e-6
    off = get_scheduler("DDPMScheduler", use_karras_sigmas=False)
    assert off.threshold_x0(x0) is x0


def _diffusers_ddim_step(acp, t, t_prev, x, eps, eta, noise):
    """diffusers DDIMScheduler.step (epsilon prediction, no clipping) written
    from its formulas: x0, std = eta sqrt(var(t, t_prev)), eps direction."""
    a_t = acp[t]
    a_p = acp[t_prev] if t_prev >= 0 else acp[0]
    x0 = (x - math.sqrt(1 - a_t) * eps) / math.sqrt(a_t)
    var = (1 - a_p) / (1 - a_t) * (1 - a_t / a_p)
    std = eta * math.sqrt(var)
    return math.sqrt(a_p) * x0 + math.sqrt(1 - a_p - std * std) * eps + std * noise


@pytest.mark.parametrize("eta", [0.0, 0.3, 1.0])
def test_ddim_eta_matches_diffusers_formula(eta):
    s = get_scheduler("DDIMScheduler", use_karras_sigmas=False)
    s.eta = eta
    n = 10
    s.set_timesteps(n)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(64, generator=g, dtype=torch.float64)
    ts = [int(t) for t in s.timesteps]
    for i in range(n):
        eps = torch.randn(64, generator=g, dtype=torch.float64)
        c = s.coeffs(i)
        noise = torch.randn(64, generator=g, dtype=torch.float64)
        ours = c.A * x + c.B * (c.p * x + c.q * eps) + c.D * noise
        ref = _diffusers_ddim_step(s.alphas_cumprod, ts[i], ts[i] - 1000 // n, x, eps, eta, noise)
        assert torch.allclose(ours, ref, atol=1e-9), (i, (ours - ref).abs().max())
        assert (c.D == 0.0) == (eta == 0.0)
        x = ref


def test_eta_is_ddim_only_and_reaches_the_sampler():
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    assert get_scheduler("DDIMScheduler").accepts_eta
    for n in ("DDPMScheduler", "PNDMScheduler", "DPMSolverMultistepScheduler", "EulerDiscreteScheduler"):
        assert not get_scheduler(n).accepts_eta, n
    pipe = StableDiffusion("tiny", "cpu", seed=1)
    kw = dict(prompt="x", num_inference_steps=3, height=64, width=64)
    a = pipe(generator=torch.Generator().manual_seed(0), scheduler=get_scheduler("DDIMScheduler"), **kw).latents
    b = pipe(generator=torch.Generator().manual_seed(0), scheduler=get_scheduler("DDIMScheduler"), eta=0.0,
             **kw).latents
    c = pipe(generator=torch.Generator().manual_seed(0), scheduler=get_scheduler("DDIMScheduler"), eta=1.0,
             **kw).latents
    assert torch.equal(a, b) and not torch.allclose(a, c)
    # samplers whose step takes no eta ignore it (diffusers prepare_extra_step_kwargs)
    d = pipe(generator=torch.Generator().manual_seed(0), scheduler=get_scheduler("EulerDiscreteScheduler"), **kw)
    e = pipe(generator=torch.Generator().manual_seed(0), scheduler=get_scheduler("EulerDiscreteScheduler"), eta=1.0,
             **kw)
    assert torch.equal(d.latents, e.latents)


def test_unknown_pipeline_kwarg_raises():
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    pipe = StableDiffusion("tiny", "cpu", seed=1)
    with pytest.raises(TypeError, match="not_a_diffusers_arg"):
        pipe(prompt="x", num_inference_steps=1, height=64, width=64, not_a_diffusers_arg=3)


def test_dpmpp_2m_sde_via_algorithm_type():
    """diffusers' 2M SDE is DPMSolverMultistepScheduler(algorithm_type="sde-dpmsolver++"):
    fresh noise every step but the last, the deterministic limit of its
    first-order update is the data-prediction exponential integrator."""
    s = get_scheduler("DPMSolverMultistepScheduler", algorithm_type="sde-dpmsolver++")
    s.set_timesteps(20)
    rows = s.loop_table()[1]
    assert all(r[5] > 0 for r in rows[:-1]) and rows[-1][5] == 0.0
    c = s.coeffs(0)
    s_s, s_t = float(s.sigmas[0]), float(s.sigmas[1])
    h = math.log(s_s / s_t)
    a_t = 1 / math.sqrt(s_t ** 2 + 1)
    assert abs(c.B - a_t * (1 - math.exp(-2 * h))) < 1e-12
    assert abs(c.D - s_t * a_t * math.sqrt(1 - math.exp(-2 * h))) < 1e-12
    with pytest.raises(ValueError):
        get_scheduler("DPMSolverMultistepScheduler", algorithm_type="dpmsolver")
    # the k-diffusion DPM++ SDE keeps its own name
    assert type(get_scheduler("DPMSolverSDEScheduler")).__mro__[1].__name__ == "_TwoStageK"


def test_clip_sample_only_where_diffusers_takes_it():
    for n in ("DDIMScheduler", "DDPMScheduler"):
        assert get_scheduler(n, clip_sample=True).clip_sample, n
    for n in ("DPMSolverMultistepScheduler", "EulerDiscreteScheduler", "PNDMScheduler", "HeunDiscreteScheduler"):
        s = get_scheduler(n, clip_sample=True)
        assert not s.clip_sample, n
        s.set_timesteps(5)
        assert s.fused_coeffs() is not None or s.coeffs(0) is None  # never demoted by the key
    assert not get_scheduler("EulerDiscreteScheduler", thresholding=True).thresholding
    assert get_scheduler("DPMSolverMultistepScheduler", thresholding=True).thresholding
