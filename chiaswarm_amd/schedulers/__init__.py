"""Diffusion samplers, selected by diffusers class *name* (the hive sends
``parameters.scheduler_type`` as a string, resolved by reflection in the
reference: swarm/job_arguments.py:146-148, swarm/type_helpers.py:1-3; always
built with ``use_karras_sigmas=True``, swarm/diffusion/diffusion_func.py:71-74).

All samplers are written in one linear form so that a single fused HIP kernel
(``ops.hip_ops.sched_step``: CFG combine + x0 conversion + update + bf16 cast of
the next UNet input) executes every step of every sampler:

    e      = e_u + g (e_c - e_u)                 (CFG; 3-way for pix2pix)
    x0     = p x + q e                            (epsilon / v / sample prediction)
    x_next = A x + B x0 + C x0_prev + D noise
    unet_in(next) = s_next * x_next

The per-step scalars (p, q, A, B, C, D, s) are computed here on the host in
float64.  Samplers whose update is not of this form (Heun: two evaluations per
step) implement ``step`` directly.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np
import torch


@dataclasses.dataclass
class StepCoeffs:
    p: float
    q: float
    A: float
    B: float
    C: float = 0.0
    D: float = 0.0
    s_next: float = 1.0


def _betas(n=1000, start=0.00085, end=0.012, schedule="scaled_linear"):
    if schedule == "scaled_linear":
        return np.linspace(start ** 0.5, end ** 0.5, n, dtype=np.float64) ** 2
    if schedule == "squaredcos_cap_v2":  # DeepFloyd IF / improved-DDPM cosine schedule
        f = lambda t: math.cos((t + 0.008) / 1.008 * math.pi / 2) ** 2  # noqa: E731
        return np.array([min(1 - f((i + 1) / n) / f(i / n), 0.999) for i in range(n)], dtype=np.float64)
    return np.linspace(start, end, n, dtype=np.float64)


def batch_randn(shape, generator=None, device=None) -> torch.Tensor:
    """fp32 N(0, 1) of ``shape``.  ``generator`` may be a list of
    ``(generator, rows)`` pairs: a coalesced batch (runtime.batcher) draws each
    job's rows from that job's own generator, so a stochastic sampler gives
    every job exactly the images it would get alone."""
    if isinstance(generator, (list, tuple)):
        parts = [torch.randn((n,) + tuple(shape[1:]), generator=g, device=device, dtype=torch.float32)
                 for g, n in generator]
        out = torch.cat(parts, 0)
        assert out.shape == tuple(shape), (out.shape, shape)
        return out
    return torch.randn(shape, generator=generator, device=device, dtype=torch.float32)


def karras_sigmas(sigma_min, sigma_max, n, rho=7.0):
    ramp = np.linspace(0, 1, n)
    lo, hi = sigma_min ** (1 / rho), sigma_max ** (1 / rho)
    return (hi + ramp * (lo - hi)) ** rho


class Scheduler:
    """Common state: training noise schedule and the inference sigma ladder
    (k-diffusion convention: sigma = sqrt((1 - abar) / abar))."""

    name = "base"
    order = 1
    space = "vp"
    karras_full_range = False  # DPM-Solver: Karras over the whole training sigma range  # "vp": sample lives in x_t = a x0 + s eps; "k": x = x0 + sigma eps

    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                 beta_schedule="scaled_linear", prediction_type="epsilon", use_karras_sigmas=True,
                 steps_offset=1, **_):
        self.T = num_train_timesteps
        self.betas = _betas(num_train_timesteps, beta_start, beta_end, beta_schedule)
        self.alphas_cumprod = np.cumprod(1.0 - self.betas)
        self.train_sigmas = np.sqrt((1 - self.alphas_cumprod) / self.alphas_cumprod)
        self.log_sigmas = np.log(self.train_sigmas)
        self.prediction_type = prediction_type
        self.use_karras = use_karras_sigmas
        self.steps_offset = steps_offset
        self.timesteps: list[float] = []
        self.sigmas = np.zeros(1)

    # -- sigma <-> t ------------------------------------------------------
    def sigma_to_t(self, sigma):
        log_sigma = np.log(max(sigma, 1e-10))
        dists = log_sigma - self.log_sigmas
        low = int(np.clip(np.cumsum(dists >= 0).argmax(), 0, len(self.log_sigmas) - 2))
        high = low + 1
        lo, hi = self.log_sigmas[low], self.log_sigmas[high]
        w = np.clip((lo - log_sigma) / (lo - hi), 0, 1)
        return float((1 - w) * low + w * high)

    def _ladder(self, n):
        """Decreasing sigma ladder of length n (+ final sigma appended by caller)."""
        ts = np.linspace(0, self.T - 1, n + 1).round()[::-1][:-1].copy()
        sig = np.interp(ts, np.arange(self.T), self.train_sigmas)
        if self.use_karras:
            if self.karras_full_range:
                sig = karras_sigmas(self.train_sigmas[0], self.train_sigmas[-1], n)
            else:
                sig = karras_sigmas(sig[-1], sig[0], n)
            ts = np.array([round(self.sigma_to_t(s)) for s in sig], dtype=np.float64)
        return ts, sig

    def set_timesteps(self, n: int):
        ts, sig = self._ladder(n)
        self.timesteps = [float(t) for t in ts]
        self.sigmas = np.concatenate([sig, [0.0]])
        self.n = n
        self.reset()

    def reset(self):
        self.prev_x0 = None
        self.step_index = 0

    @property
    def init_noise_sigma(self) -> float:
        return 1.0 if self.space == "vp" else float(math.sqrt(self.sigmas[0] ** 2 + 1))

    def scale_in(self, i: int) -> float:
        if self.space == "vp" or i >= self.n:
            return 1.0
        return float(1.0 / math.sqrt(self.sigmas[i] ** 2 + 1))

    def x0_coeffs(self, i: int):
        """x0 = p x + q e for the sample convention of this sampler."""
        s = float(self.sigmas[i])
        a = 1.0 / math.sqrt(s * s + 1.0)
        sv = s * a
        pt = self.prediction_type
        if self.space == "vp":
            if pt == "epsilon":
                return 1.0 / a, -sv / a
            if pt == "v_prediction":
                return a, -sv
            return 0.0, 1.0
        if pt == "epsilon":
            return 1.0, -s
        if pt == "v_prediction":
            return 1.0 / (s * s + 1.0), -s / math.sqrt(s * s + 1.0)
        return 0.0, 1.0

    def coeffs(self, i: int) -> StepCoeffs | None:  # pragma: no cover - overridden
        raise NotImplementedError

    # -- evaluation schedule (Heun-type samplers evaluate twice per interval) --
    @property
    def num_evals(self) -> int:
        return self.n

    def current_t(self) -> float:
        return self.timesteps[self.step_index]

    def current_scale(self) -> float:
        return self.scale_in(self.step_index)

    def fused_coeffs(self) -> StepCoeffs | None:
        """Coefficients for the fused HIP step kernel, or None if this step must
        run through ``step`` (non-linear-form samplers)."""
        return self.coeffs(self.step_index)

    # -- generic torch step (CPU path and reference mode) ---------------------
    def step(self, e: torch.Tensor, x: torch.Tensor, generator=None) -> torch.Tensor:
        """One update on fp32 tensors given the (guided) model output ``e``."""
        i = self.step_index
        c = self.coeffs(i)
        x0 = c.p * x + c.q * e.float()
        out = c.A * x + c.B * x0
        if c.C != 0.0 and self.prev_x0 is not None:
            out = out + c.C * self.prev_x0
        if c.D != 0.0:
            out = out + c.D * batch_randn(x.shape, generator, x.device)
        self.prev_x0 = x0
        self.step_index += 1
        return out

    def add_noise(self, x0, noise, i: int):
        """Noise clean latents to the level of step i (img2img / inpaint)."""
        s = float(self.sigmas[i])
        if self.space == "vp":
            a = 1.0 / math.sqrt(s * s + 1)
            return a * x0 + s * a * noise
        return x0 + s * noise


class DPMSolverMultistepScheduler(Scheduler):
    """DPM-Solver++(2M), midpoint, lower-order first and final steps."""

    name = "DPMSolverMultistepScheduler"
    order = 2
    karras_full_range = True

    def __init__(self, solver_order=2, lower_order_final=True, **kw):
        super().__init__(**kw)
        self.solver_order = solver_order
        self.lower_order_final = lower_order_final

    def coeffs(self, i):
        s_s, s_t = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        a_t = 1.0 / math.sqrt(s_t * s_t + 1)
        sv_t, sv_s = s_t * a_t, s_s / math.sqrt(s_s * s_s + 1)
        if s_t == 0.0:  # final step to sigma 0: x = x0
            return StepCoeffs(p, q, 0.0, 1.0, 0.0, 0.0, 1.0)
        h = math.log(s_s / s_t)
        em1 = math.expm1(-h)  # e^{-h} - 1
        A = sv_t / sv_s
        first = (i == 0 or self.solver_order == 1 or
                 (self.lower_order_final and i == self.n - 1 and self.n < 15))
        if first:
            return StepCoeffs(p, q, A, -a_t * em1, 0.0, 0.0, 1.0)
        s_prev = float(self.sigmas[i - 1])
        h0 = math.log(s_prev / s_s)
        r0 = h0 / h
        B = -a_t * em1 * (1.0 + 0.5 / r0)
        C = a_t * em1 * (0.5 / r0)
        return StepCoeffs(p, q, A, B, C, 0.0, 1.0)


class DPMSolverSDEScheduler(DPMSolverMultistepScheduler):
    """DPM-Solver++(2M) SDE variant (stochastic), same linear form + noise."""

    name = "DPMSolverSDEScheduler"

    def coeffs(self, i):
        s_s, s_t = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        if s_t == 0.0:
            return StepCoeffs(p, q, 0.0, 1.0)
        a_t = 1.0 / math.sqrt(s_t * s_t + 1)
        sv_t, sv_s = s_t * a_t, s_s / math.sqrt(s_s * s_s + 1)
        h = math.log(s_s / s_t)
        A = sv_t / sv_s * math.exp(-h)
        em = -math.expm1(-2.0 * h)  # 1 - e^{-2h}
        D = sv_t * math.sqrt(max(em, 0.0))
        if i == 0 or (i == self.n - 1 and self.n < 15):
            return StepCoeffs(p, q, A, a_t * em, 0.0, D)
        h0 = math.log(float(self.sigmas[i - 1]) / s_s)
        r0 = h0 / h
        B = a_t * em * (1.0 + 0.5 / r0)
        C = -a_t * em * (0.5 / r0)
        return StepCoeffs(p, q, A, B, C, D)


class EulerDiscreteScheduler(Scheduler):
    name = "EulerDiscreteScheduler"
    space = "k"

    def coeffs(self, i):
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        r = sn / s
        return StepCoeffs(p, q, r, 1.0 - r, 0.0, 0.0, self.scale_in(i + 1))


class EulerAncestralDiscreteScheduler(Scheduler):
    name = "EulerAncestralDiscreteScheduler"
    space = "k"

    def coeffs(self, i):
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        up = math.sqrt(max(sn ** 2 * (s ** 2 - sn ** 2) / s ** 2, 0.0))
        down = math.sqrt(max(sn ** 2 - up ** 2, 0.0))
        r = down / s
        return StepCoeffs(p, q, r, 1.0 - r, 0.0, up, self.scale_in(i + 1))


class DDIMScheduler(Scheduler):
    """DDIM (eta = 0), "leading" timestep spacing with steps_offset."""

    name = "DDIMScheduler"

    def _ladder(self, n):
        ratio = self.T // n
        ts = (np.arange(0, n) * ratio).round()[::-1].astype(np.float64) + self.steps_offset
        ts = np.clip(ts, 0, self.T - 1)
        sig = self.train_sigmas[ts.astype(int)]
        return ts, sig

    def set_timesteps(self, n):
        super().set_timesteps(n)
        # DDIM's final "previous" level is alphas_cumprod[0] (set_alpha_to_one=False)
        self.sigmas[-1] = self.train_sigmas[0]

    def coeffs(self, i):
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        a, an = 1 / math.sqrt(s * s + 1), 1 / math.sqrt(sn * sn + 1)
        sv, svn = s * a, sn * an
        A = svn / sv
        B = an - svn * a / sv
        return StepCoeffs(p, q, A, B)


class PNDMScheduler(DDIMScheduler):
    """Served with the DDIM update (PLMS warm-up not reproduced; documented)."""

    name = "PNDMScheduler"


class DDPMScheduler(DDIMScheduler):
    """Ancestral DDPM posterior sampling on the leading-spacing ladder."""

    name = "DDPMScheduler"

    def coeffs(self, i):
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        abar, abar_p = 1 / (s * s + 1), 1 / (sn * sn + 1)
        beta_t = 1 - abar / abar_p
        A = math.sqrt(1 - beta_t) * (1 - abar_p) / (1 - abar)
        B = math.sqrt(abar_p) * beta_t / (1 - abar)
        var = (1 - abar_p) / (1 - abar) * beta_t
        D = math.sqrt(max(var, 0.0)) if i < self.n - 1 else 0.0
        return StepCoeffs(p, q, A, B, 0.0, D)


class LMSDiscreteScheduler(EulerDiscreteScheduler):
    """Linear multistep (order 2 Adams-Bashforth in sigma), k-space."""

    name = "LMSDiscreteScheduler"

    def reset(self):
        super().reset()
        self._d_prev = None

    def coeffs(self, i):  # not of the single-history linear form -> torch step
        return None

    def step(self, e, x, generator=None):
        i = self.step_index
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        x0 = p * x + q * e.float()
        d = (x - x0) / s
        dt = sn - s
        if self._d_prev is None:
            out = x + dt * d
        else:  # 2nd-order Adams-Bashforth in sigma
            out = x + dt * (1.5 * d - 0.5 * self._d_prev)
        self._d_prev = d
        self.prev_x0 = x0
        self.step_index += 1
        return out


class HeunDiscreteScheduler(EulerDiscreteScheduler):
    """Heun (2nd order, two UNet evaluations per sigma interval)."""

    name = "HeunDiscreteScheduler"
    order = 2

    @property
    def num_evals(self):
        return 2 * self.n - 1

    def current_t(self):
        return self.sigma_to_t(self.eval_sigma())

    def current_scale(self):
        s = self.eval_sigma()
        return 1.0 / math.sqrt(s * s + 1)

    def coeffs(self, i):
        return None

    def reset(self):
        super().reset()
        self._d1 = None
        self._x_orig = None
        self._phase = 0
        self._i = 0

    def eval_sigma(self):
        if self._phase == 0:
            return float(self.sigmas[self._i])
        return float(self.sigmas[self._i + 1])

    def step(self, e, x, generator=None):
        i = self._i
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        if self._phase == 0:
            p, q = self.x0_coeffs(i)
            x0 = p * x + q * e.float()
            d = (x - x0) / s
            if sn == 0.0:
                self._i += 1
                self.step_index += 1
                return x + (sn - s) * d
            self._d1, self._x_orig = d, x
            self._phase = 1
            return x + (sn - s) * d
        # second evaluation at sn
        s2 = sn
        pt = self.prediction_type
        x0 = x - s2 * e.float() if pt == "epsilon" else e.float()
        d2 = (x - x0) / s2
        out = self._x_orig + (sn - s) * 0.5 * (self._d1 + d2)
        self._phase = 0
        self._i += 1
        self.step_index += 1
        return out


_REGISTRY = {c.name: c for c in [
    DPMSolverMultistepScheduler, DPMSolverSDEScheduler, EulerDiscreteScheduler,
    EulerAncestralDiscreteScheduler, DDIMScheduler, PNDMScheduler, DDPMScheduler,
    LMSDiscreteScheduler, HeunDiscreteScheduler]}
# names the hive may send whose update we serve with the closest sampler
_ALIASES = {
    "DPMSolverSinglestepScheduler": "DPMSolverMultistepScheduler",
    "UniPCMultistepScheduler": "DPMSolverMultistepScheduler",
    "DEISMultistepScheduler": "DPMSolverMultistepScheduler",
    "KDPM2DiscreteScheduler": "HeunDiscreteScheduler",
    "KDPM2AncestralDiscreteScheduler": "EulerAncestralDiscreteScheduler",
}


def scheduler_names():
    return sorted(list(_REGISTRY) + list(_ALIASES))


def get_scheduler(name: str | type | None, **config) -> Scheduler:
    """Build a sampler by diffusers class name (unknown names raise ValueError,
    which the worker reports as a fatal, non-retryable job error)."""
    if name is None:
        name = "DPMSolverMultistepScheduler"
    if isinstance(name, type):
        name = name.__name__
    name = _ALIASES.get(name, name)
    if name not in _REGISTRY:
        raise ValueError(f"Unknown scheduler_type {name}")
    config.setdefault("use_karras_sigmas", True)
    return _REGISTRY[name](**config)
