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
