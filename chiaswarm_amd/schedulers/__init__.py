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
    default_spacing = "linspace"
    karras_full_range = False  # DPM-Solver: Karras over the whole training sigma range
    # config keys only some diffusers classes take (from_config drops them for the others):
    accepts_eta = False  # DDIMScheduler.step(eta=...)
    accepts_clip_sample = False  # DDIM / DDPM
    accepts_thresholding = False  # DDIM / DDPM / DPM-Solver family / DEIS / UniPC

    def __init__(self, num_train_timesteps=1000, beta_start=0.00085, beta_end=0.012,
                 beta_schedule="scaled_linear", prediction_type="epsilon", use_karras_sigmas=True,
                 steps_offset=1, thresholding=False, dynamic_thresholding_ratio=0.995, sample_max_value=1.0,
                 timestep_spacing=None, clip_sample=False, clip_sample_range=1.0, **_):
        self.T = num_train_timesteps
        # the checkpoint's scheduler_config.json fields (models/hf_config.scheduler_kwargs)
        timestep_spacing = timestep_spacing or self.default_spacing  # diffusers: each class's own default
        if timestep_spacing not in ("linspace", "leading", "trailing"):
            raise ValueError(f"timestep_spacing={timestep_spacing!r} is not supported")
        self.timestep_spacing = timestep_spacing
        self.clip_sample = bool(clip_sample) and self.accepts_clip_sample
        self.clip_sample_range = float(clip_sample_range)
        # Imagen dynamic thresholding of the x0 prediction (DeepFloyd IF:
        # ratio 0.95, max 1.5) -- non-linear in x0, so those steps skip the fused kernel
        self.thresholding = bool(thresholding) and self.accepts_thresholding
        self.dyn_ratio = dynamic_thresholding_ratio
        self.sample_max = sample_max_value
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

    def _spaced_timesteps(self, n):
        """Decreasing inference timesteps per ``timestep_spacing`` (diffusers
        semantics): "linspace" n points over [0, T-1] (the DPM-Solver form:
        n + 1 rounded points, last dropped), "leading" multiples of T // n
        plus ``steps_offset``, "trailing" from T - 1 down in steps of T / n."""
        if self.timestep_spacing == "leading":
            ts = (np.arange(0, n) * (self.T // n)).round()[::-1].astype(np.float64) + self.steps_offset
        elif self.timestep_spacing == "trailing":
            ts = np.round(np.arange(self.T, 0, -self.T / n)).astype(np.float64) - 1
        else:
            ts = np.linspace(0, self.T - 1, n + 1).round()[::-1][:-1]
        return np.clip(ts, 0, self.T - 1).copy()

    def _ladder(self, n):
        """Decreasing sigma ladder of length n (+ final sigma appended by caller)."""
        ts = self._spaced_timesteps(n)
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
            if pt == "k_denoiser":
                raise ValueError(f"{self.name}: k_denoiser outputs need a k-space sampler (Euler / Heun / DPM2 ...)")
            if pt == "epsilon":
                return 1.0 / a, -sv / a
            if pt == "v_prediction":
                return a, -sv
            return 0.0, 1.0
        if pt == "epsilon":
            return 1.0, -s
        if pt == "v_prediction":
            return 1.0 / (s * s + 1.0), -s / math.sqrt(s * s + 1.0)
        if pt == "k_denoiser":  # Karras preconditioning, sigma_data = 1: x0 = c_skip x + c_out F
            return 1.0 / (s * s + 1.0), s / math.sqrt(s * s + 1.0)
        return 0.0, 1.0

    def coeffs(self, i: int) -> StepCoeffs | None:  # pragma: no cover - overridden
        raise NotImplementedError

    # -- evaluation schedule (Heun-type samplers evaluate twice per interval) --
    @property
    def num_evals(self) -> int:
        return self.n

    def current_t(self) -> float:
        return self.timesteps[self.step_index]

    def eval_sigma(self) -> float:
        """k-diffusion sigma of the sample the next model evaluation sees."""
        return float(self.sigmas[self.step_index])

    def current_scale(self) -> float:
        return self.scale_in(self.step_index)

    def fused_coeffs(self) -> StepCoeffs | None:
        """Coefficients for the fused HIP step kernel, or None if this step must
        run through ``step`` (non-linear-form samplers)."""
        if self.thresholding or self.clip_sample:
            return None
        return self.coeffs(self.step_index)

    def loop_table(self):
        """The remaining steps as a device-loop table, or None when a step is
        not the plain linear form (thresholding, two evaluations per step, a
        sampler-specific ``step``): ``(timesteps, rows, s_first)`` with one
        ``[p, q, A, B, C, D, s_next]`` row per step from ``step_index`` on and
        the input scale of the first evaluation.  Every row is a pure function
        of its step index, so the table is exactly what ``fused_coeffs`` would
        return step by step."""
        cls = type(self)
        if (self.thresholding or self.clip_sample or cls.step is not Scheduler.step or cls.current_t is not Scheduler.current_t
                or cls.current_scale is not Scheduler.current_scale
                or cls.fused_coeffs is not Scheduler.fused_coeffs or self.num_evals != self.n):
            return None
        rows = []
        for i in range(self.step_index, self.n):
            c = self.coeffs(i)
            if c is None:
                return None
            rows.append([c.p, c.q, c.A, c.B, c.C, c.D, c.s_next])
        ts = [float(t) for t in self.timesteps[self.step_index:self.n]]
        return ts, rows, self.current_scale()

    def threshold_x0(self, x0: torch.Tensor) -> torch.Tensor:
        """Per-sample dynamic thresholding: s = quantile(|x0|, ratio) clamped to
        [1, sample_max]; x0 -> clamp(x0, -s, s) / s (identity when disabled)."""
        if self.clip_sample and not self.thresholding:
            return x0.clamp(-self.clip_sample_range, self.clip_sample_range)
        if not self.thresholding:
            return x0
        b = x0.shape[0]
        flat = x0.reshape(b, -1).float()
        s = torch.quantile(flat.abs(), self.dyn_ratio, dim=1).clamp(1.0, self.sample_max)
        s = s.reshape((b,) + (1,) * (x0.dim() - 1))
        return (torch.maximum(torch.minimum(x0, s), -s) / s).to(x0.dtype)

    # -- generic torch step (CPU path and reference mode) ---------------------
    def step(self, e: torch.Tensor, x: torch.Tensor, generator=None) -> torch.Tensor:
        """One update on fp32 tensors given the (guided) model output ``e``."""
        i = self.step_index
        c = self.coeffs(i)
        x0 = self.threshold_x0(c.p * x + c.q * e.float())
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

    accepts_thresholding = True

    def __init__(self, solver_order=2, lower_order_final=True, algorithm_type="dpmsolver++", **kw):
        super().__init__(**kw)
        if algorithm_type not in ("dpmsolver++", "sde-dpmsolver++"):
            raise ValueError(f"{self.name}: algorithm_type={algorithm_type!r} is not supported")
        self.solver_order = solver_order
        self.lower_order_final = lower_order_final
        self.algorithm_type = algorithm_type

    def coeffs(self, i):
        if self.algorithm_type == "sde-dpmsolver++":
            return self._sde_coeffs(i)
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

    def _sde_coeffs(self, i):
        """DPM-Solver++(2M) SDE (diffusers ``algorithm_type="sde-dpmsolver++"``):
        the same midpoint form with e^{-h}-damped x and fresh noise of
        std sigma_t sqrt(1 - e^{-2h}) every step but the last."""
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
        if i == 0 or self.solver_order == 1 or (self.lower_order_final and i == self.n - 1 and self.n < 15):
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
    """DDIM, "leading" timestep spacing with steps_offset.  ``eta`` (the
    pipeline call's kwarg, forwarded to ``DDIMScheduler.step`` by diffusers)
    interpolates between deterministic DDIM (0) and DDPM-like ancestral
    sampling (1): std_t = eta sqrt((1 - a_prev)/(1 - a_t) (1 - a_t/a_prev)) of fresh
    noise, the eps direction shrunk to sqrt(1 - a_prev - std_t^2)."""

    name = "DDIMScheduler"
    accepts_eta = True
    accepts_clip_sample = True
    accepts_thresholding = True

    default_spacing = "leading"
    eta = 0.0

    def _ladder(self, n):
        ts = self._spaced_timesteps(n)
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
        std = 0.0
        if self.eta:
            abar, abar_p = a * a, an * an
            std = float(self.eta) * math.sqrt(max((1 - abar_p) / (1 - abar) * (1 - abar / abar_p), 0.0))
        c = math.sqrt(max(svn * svn - std * std, 0.0))  # eps-direction weight
        A = c / sv
        B = an - c * a / sv
        return StepCoeffs(p, q, A, B, 0.0, std)


class DDPMScheduler(DDIMScheduler):
    """Ancestral DDPM posterior sampling on the leading-spacing ladder."""

    name = "DDPMScheduler"
    accepts_eta = False

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


# ---------------------------------------------------------------------------
# Samplers whose update keeps more history than (x, x0, x0_prev): torch step
# path (a handful of elementwise ops per step; the UNet dominates).  Reference
# semantics: the diffusers classes of the same names that the reference
# instantiates by name (swarm/job_arguments.py:146-148) from the pipeline's
# scheduler config with ``use_karras_sigmas=True``
# (swarm/diffusion/diffusion_func.py:71-74).
# ---------------------------------------------------------------------------
def _vp(sig):
    """(alpha, sigma_vp, lambda) of a k-diffusion sigma."""
    a = 1.0 / math.sqrt(sig * sig + 1.0)
    return a, sig * a, (-math.log(sig) if sig > 0 else float("inf"))


class PNDMScheduler(DDIMScheduler):
    """Pseudo linear multistep (PLMS, ``skip_prk_steps=True`` as in every SD
    scheduler config): n+1 model evaluations on the "leading" ladder with the
    second-highest timestep evaluated twice, 1st..4th-order Adams-Bashforth
    combinations of the noise predictions, and PNDM's transfer formula
    x_prev = sqrt(a_prev/a_t) x - (a_prev - a_t) e / (a_t sqrt(1-a_prev) + sqrt(a_t (1-a_t) a_prev))."""

    name = "PNDMScheduler"
    accepts_eta = False
    accepts_clip_sample = False
    accepts_thresholding = False

    def set_timesteps(self, n):
        super().set_timesteps(n)  # DDIM ladder: leading spacing + steps_offset, final level acp[0]
        ts = [int(t) for t in self.timesteps]  # descending e_{n-1} .. e_0
        asc = ts[::-1]
        plms = asc[:-1] + asc[-2:-1] + asc[-1:] if n > 1 else asc
        self.plms = plms[::-1]
        self.ratio = self.T // n
        self.n = len(self.plms)

    def reset(self):
        super().reset()
        self._ets: list = []
        self._cur = None
        self._counter = 0

    def current_t(self):
        return float(self.plms[self.step_index])

    def eval_sigma(self):
        return float(self.train_sigmas[int(self.plms[self.step_index])])

    def coeffs(self, i):
        return None

    def _acp(self, t):
        return float(self.alphas_cumprod[t]) if t >= 0 else float(self.alphas_cumprod[0])

    def step(self, e, x, generator=None):
        t = int(self.plms[self.step_index])
        e = e.float()
        if self.prediction_type == "v_prediction":
            a_t = self._acp(t)
            e = math.sqrt(a_t) * e + math.sqrt(1 - a_t) * x
        prev_t = t - self.ratio
        if self._counter != 1:
            self._ets = (self._ets + [e])[-4:]
        else:
            prev_t, t = t, t + self.ratio
        ets = self._ets
        if len(ets) == 1 and self._counter == 0:
            eps, self._cur = e, x
        elif len(ets) == 1 and self._counter == 1:
            eps, x = (e + ets[-1]) / 2, self._cur
            self._cur = None
        elif len(ets) == 2:
            eps = (3 * ets[-1] - ets[-2]) / 2
        elif len(ets) == 3:
            eps = (23 * ets[-1] - 16 * ets[-2] + 5 * ets[-3]) / 12
        else:
            eps = (55 * ets[-1] - 59 * ets[-2] + 37 * ets[-3] - 9 * ets[-4]) / 24
        a_t, a_p = self._acp(t), self._acp(prev_t)
        den = a_t * math.sqrt(1 - a_p) + math.sqrt(a_t * (1 - a_t) * a_p)
        out = math.sqrt(a_p / a_t) * x - (a_p - a_t) * eps / den
        self.prev_x0 = (x - math.sqrt(1 - a_t) * eps) / math.sqrt(a_t)
        self._counter += 1
        self.step_index += 1
        return out


class LMSDiscreteScheduler(EulerDiscreteScheduler):
    """Linear multistep, order 4 (diffusers default): the derivative history
    d_k = (x_k - x0_k) / sigma_k combined with the integrals over
    [sigma_i, sigma_{i+1}] of the Lagrange basis polynomials through the last
    (up to) four sigmas — integrated exactly (polynomials) where diffusers
    uses scipy quad."""

    name = "LMSDiscreteScheduler"
    order = 4

    def reset(self):
        super().reset()
        self._ds: list = []

    def coeffs(self, i):
        return None

    def lms_coeff(self, order, t, k):
        sig = self.sigmas
        num = np.poly1d([1.0])
        den = 1.0
        for j in range(order):
            if j == k:
                continue
            num = num * np.poly1d([1.0, -sig[t - j]])
            den *= sig[t - k] - sig[t - j]
        P = np.polyint(num)
        return float((P(sig[t + 1]) - P(sig[t])) / den)

    def step(self, e, x, generator=None):
        i = self.step_index
        p, q = self.x0_coeffs(i)
        x0 = p * x + q * e.float()
        d = (x - x0) / float(self.sigmas[i])
        self._ds = (self._ds + [d])[-self.order:]
        order = min(i + 1, self.order)
        out = x
        for k in range(order):
            out = out + self.lms_coeff(order, i, k) * self._ds[-1 - k]
        self.prev_x0 = x0
        self.step_index += 1
        return out


class _TwoStageK(EulerDiscreteScheduler):
    """k-diffusion two-evaluation samplers (sample_dpm_2 / _ancestral /
    sample_dpmpp_sde): each sigma interval evaluates the model at sigma_i and
    at an intermediate sigma; a final interval to sigma = 0 is one Euler step."""

    order = 2

    def reset(self):
        super().reset()
        self._phase = 0
        self._x = self._d = None
        self._mid = None

    def coeffs(self, i):
        return None

    def eval_sigma(self):
        return float(self.sigmas[self.step_index]) if self._phase == 0 else float(self._mid)

    def current_t(self):
        return self.sigma_to_t(self.eval_sigma())

    def current_scale(self):
        s = self.eval_sigma()
        return 1.0 / math.sqrt(s * s + 1)

    def _x0(self, e, x, sig):
        pt = self.prediction_type
        e = e.float()
        if pt == "epsilon":
            return x - sig * e
        if pt == "v_prediction":
            return x / (sig * sig + 1) - sig / math.sqrt(sig * sig + 1) * e
        return e


def ancestral_step(s_from: float, s_to: float, eta: float = 1.0):
    up = min(s_to, eta * math.sqrt(max(s_to ** 2 * (s_from ** 2 - s_to ** 2) / s_from ** 2, 0.0)))
    return math.sqrt(max(s_to ** 2 - up ** 2, 0.0)), up


class KDPM2DiscreteScheduler(_TwoStageK):
    """DPM-Solver-2 (k-diffusion sample_dpm_2): Euler to the log-midpoint
    sigma, re-evaluate, full step with the midpoint derivative."""

    name = "KDPM2DiscreteScheduler"

    def _target(self, i):
        return float(self.sigmas[i + 1]), 0.0

    def step(self, e, x, generator=None):
        i = self.step_index
        s = float(self.sigmas[i])
        s_to, up = self._target(i)
        if self._phase == 0:
            d = (x - self._x0(e, x, s)) / s
            if s_to == 0.0:
                self.step_index += 1
                return x + d * (s_to - s)
            self._mid = math.exp(0.5 * (math.log(s) + math.log(s_to)))
            self._x, self._d, self._phase = x, d, 1
            return x + d * (self._mid - s)
        d2 = (x - self._x0(e, x, self._mid)) / self._mid
        out = self._x + d2 * (s_to - s)
        if up > 0.0:
            out = out + up * batch_randn(out.shape, generator, out.device)
        self._phase = 0
        self.step_index += 1
        return out


class KDPM2AncestralDiscreteScheduler(KDPM2DiscreteScheduler):
    """sample_dpm_2_ancestral: the DPM-2 step aimed at sigma_down, then
    sigma_up of fresh noise (eta = 1)."""

    name = "KDPM2AncestralDiscreteScheduler"

    def _target(self, i):
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        if sn == 0.0:
            return 0.0, 0.0
        return ancestral_step(s, sn)


class DPMSolverSDEScheduler(_TwoStageK):
    """DPM-Solver++ SDE (k-diffusion sample_dpmpp_sde, r = 1/2, eta = 1): two
    evaluations per interval with ancestral noise after each half.  The
    reference draws that noise from torchsde's Brownian tree in sigma
    (normalised increments (W(s1) - W(s0)) / sqrt|s1 - s0|); torchsde is not
    available, so the two increments of an interval are built from two seeded
    N(0, 1) draws with the Brownian-path correlation: n1 = z1 over
    [sigma, sigma_mid], n2 = (sqrt(d1) z1 + sqrt(d2) z2) / sqrt(d1 + d2) over
    [sigma, sigma_next] — the same joint law as the tree (parity with
    diffusers' exact noise stream unpinned)."""

    name = "DPMSolverSDEScheduler"

    def step(self, e, x, generator=None):
        i = self.step_index
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        if self._phase == 0:
            x0 = self._x0(e, x, s)
            if sn == 0.0:
                self.step_index += 1
                return x0  # Euler to sigma 0 lands on the denoised sample
            t, t_next = -math.log(s), -math.log(sn)
            self._mid = math.exp(-(t + 0.5 * (t_next - t)))
            sd, su = ancestral_step(s, self._mid)
            self._z1 = batch_randn(x.shape, generator, x.device)
            x2 = (sd / s) * x - math.expm1(t + math.log(sd)) * x0 + su * self._z1
            self._x, self._phase = x, 1
            return x2
        x0_2 = self._x0(e, x, self._mid)
        sd, su = ancestral_step(s, sn)
        out = (sd / s) * self._x - math.expm1(-math.log(s) + math.log(sd)) * x0_2
        d1, d2 = s - self._mid, self._mid - sn
        z2 = batch_randn(out.shape, generator, out.device)
        out = out + su * (math.sqrt(d1) * self._z1 + math.sqrt(d2) * z2) / math.sqrt(d1 + d2)
        self._z1 = None
        self._phase = 0
        self.step_index += 1
        return out


class UniPCMultistepScheduler(DPMSolverMultistepScheduler):
    """UniPC (bh2, predict-x0, order 2, lower-order final steps): the UniP
    multistep predictor plus the UniC corrector applied to the previous step's
    result with the new model output.  Coefficients from the phi-function
    recursion (B(h) = e^{-h} - 1), as in diffusers' multistep_uni_p/c_bh_update."""

    name = "UniPCMultistepScheduler"

    def reset(self):
        super().reset()
        self._hist: list = []  # (lambda, x0) of the last solver_order steps
        self._last_x = None
        self._this_order = 1
        self._lower = 0

    def coeffs(self, i):
        return None

    def _lam(self, i):
        return _vp(float(self.sigmas[i]))

    @staticmethod
    def _rb(rks, h, order):
        hh = -h
        h_phi_1 = math.expm1(hh)
        h_phi_k = h_phi_1 / hh - 1.0
        fact = 1.0
        B_h = math.expm1(hh)
        R, b = [], []
        for i in range(1, order + 1):
            R.append([r ** (i - 1) for r in rks])
            b.append(h_phi_k * fact / B_h)
            fact *= i + 1
            h_phi_k = h_phi_k / hh - 1.0 / fact
        return np.array(R, dtype=np.float64), np.array(b, dtype=np.float64), h_phi_1, B_h

    def _update(self, x, lam_t, a_t, sv_t, sv_s0, order, model_t=None):
        """UniP (model_t None) or UniC update from the history's last point."""
        lam_s0, m0 = self._hist[-1]
        h = lam_t - lam_s0
        rks, D1s = [], []
        for k in range(1, order):
            lam_si, mi = self._hist[-(k + 1)]
            rk = (lam_si - lam_s0) / h
            rks.append(rk)
            D1s.append((mi - m0) / rk)
        rks.append(1.0)
        R, b, h_phi_1, B_h = self._rb(rks, h, order)
        x_t_ = (sv_t / sv_s0) * x - a_t * h_phi_1 * m0
        if model_t is None:
            if not D1s:
                return x_t_
            rhos = [0.5] if order == 2 else list(np.linalg.solve(R[:-1, :-1], b[:-1]))
            res = sum(r * d for r, d in zip(rhos, D1s))
            return x_t_ - a_t * B_h * res
        rhos_c = [0.5] if order == 1 else list(np.linalg.solve(R, b))
        res = sum(r * d for r, d in zip(rhos_c[:-1], D1s)) if D1s else 0.0
        return x_t_ - a_t * B_h * (res + rhos_c[-1] * (model_t - m0))

    def step(self, e, x, generator=None):
        i = self.step_index
        s = float(self.sigmas[i])
        p, q = self.x0_coeffs(i)
        x0 = p * x + q * e.float()
        a_s, sv_s, lam_s = _vp(s)
        if i > 0 and self._last_x is not None:  # UniC corrector of the previous step's output
            a_p, sv_p, _ = self._lam(i - 1)
            x = self._update(self._last_x, lam_s, a_s, sv_s, sv_p, self._this_order, model_t=x0)
        self._hist = (self._hist + [(lam_s, x0)])[-self.solver_order:]
        order = min(self.solver_order, self.n - i) if self.lower_order_final else self.solver_order
        self._this_order = min(order, self._lower + 1)
        self._last_x = x
        sn = float(self.sigmas[i + 1])
        if sn == 0.0:
            out = x0
        else:
            a_t, sv_t, lam_t = _vp(sn)
            out = self._update(x, lam_t, a_t, sv_t, sv_s, self._this_order)
        self._lower = min(self._lower + 1, self.solver_order)
        self.prev_x0 = x0
        self.step_index += 1
        return out


class DEISMultistepScheduler(DPMSolverMultistepScheduler):
    """DEIS (order 2, log-rho): exponential-integrator steps on the noise
    prediction, the 2nd-order weights integrating the Lagrange interpolant of
    the last two noise predictions in log(sigma) (diffusers
    multistep_deis_second_order_update)."""

    name = "DEISMultistepScheduler"

    def reset(self):
        super().reset()
        self._eps: list = []

    def coeffs(self, i):
        return None

    def step(self, e, x, generator=None):
        i = self.step_index
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        x0 = p * x + q * e.float()
        a_s, sv_s, _ = _vp(s)
        eps = (x - a_s * x0) / sv_s
        self._eps = (self._eps + [(s, eps)])[-2:]
        first = (i == 0 or self.solver_order == 1 or
                 (self.lower_order_final and i == self.n - 1 and self.n < 15) or len(self._eps) < 2)
        self.prev_x0 = x0
        self.step_index += 1
        if sn == 0.0:
            return x0
        a_t, sv_t, _ = _vp(sn)
        if first:
            h = math.log(s / sn)  # lambda_t - lambda_s
            return (a_t / a_s) * x - sv_t * math.expm1(h) * eps
        (s1, m1), (_, m0) = self._eps[-2], self._eps[-1]
        rho_t, rho_s0, rho_s1 = sn, s, s1  # sigma_vp / alpha = k-sigma

        def ind(t, b, c):
            return t * (-math.log(c) + math.log(t) - 1.0) / (math.log(b) - math.log(c))

        c1 = ind(rho_t, rho_s0, rho_s1) - ind(rho_s0, rho_s0, rho_s1)
        c2 = ind(rho_t, rho_s1, rho_s0) - ind(rho_s0, rho_s1, rho_s0)
        return a_t * (x / a_s + c1 * m0 + c2 * m1)


class DPMSolverSinglestepScheduler(DPMSolverMultistepScheduler):
    """DPM-Solver++ singlestep, order 2 (orders [1, 2, 1, 2, ...], a trailing
    1 for odd step counts): the second step of each pair restarts from the
    pair's first sample with both x0 predictions (midpoint form)."""

    name = "DPMSolverSinglestepScheduler"

    def reset(self):
        super().reset()
        self._block = None  # (sigma, x, x0) at the start of the current 2-step block

    def coeffs(self, i):
        return None

    def orders(self):
        n = self.n
        if self.solver_order == 1:
            return [1] * n
        out = [1, 2] * (n // 2)
        return out + [1] if n % 2 else out

    def step(self, e, x, generator=None):
        i = self.step_index
        s, sn = float(self.sigmas[i]), float(self.sigmas[i + 1])
        p, q = self.x0_coeffs(i)
        x0 = p * x + q * e.float()
        order = self.orders()[i]
        self.prev_x0 = x0
        self.step_index += 1
        if sn == 0.0:
            return x0
        a_t, sv_t, lam_t = _vp(sn)
        if order == 1:
            self._block = (s, x, x0)
            _, sv_s, lam_s = _vp(s)
            h = lam_t - lam_s
            return (sv_t / sv_s) * x - a_t * math.expm1(-h) * x0
        s1, x_s1, m1 = self._block
        _, sv_s1, lam_s1 = _vp(s1)
        lam_s0 = _vp(s)[2]
        h, h0 = lam_t - lam_s1, lam_s0 - lam_s1
        r0 = h0 / h
        D0, D1 = m1, (x0 - m1) / r0
        em = math.expm1(-h)
        return (sv_t / sv_s1) * x_s1 - a_t * em * D0 - 0.5 * a_t * em * D1


_REGISTRY = {c.name: c for c in [
    DPMSolverMultistepScheduler, DPMSolverSinglestepScheduler, DPMSolverSDEScheduler, EulerDiscreteScheduler,
    EulerAncestralDiscreteScheduler, DDIMScheduler, PNDMScheduler, DDPMScheduler, LMSDiscreteScheduler,
    HeunDiscreteScheduler, KDPM2DiscreteScheduler, KDPM2AncestralDiscreteScheduler, UniPCMultistepScheduler,
    DEISMultistepScheduler]}
# exact equivalents only
_ALIASES: dict = {}


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
