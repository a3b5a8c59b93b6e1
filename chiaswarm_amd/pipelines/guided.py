"""Sampling-loop variants of Stable Diffusion that the hive can name as a
diffusers class (``parameters.pipeline_type``; the reference builds any such
name by reflection, swarm/job_arguments.py:143-145, swarm/type_helpers.py:1-3,
swarm/diffusion/diffusion_func.py:41-46).  All three run a plain SD
checkpoint on the resident bundle; only the denoising loop differs.

* ``StableDiffusionPanoramaPipeline`` (MultiDiffusion, Bar-Tal et al. 2023):
  the latent canvas (default 512 x 2048 px) is covered by 64 x 64 latent
  windows at stride 8; every step each window is denoised on its own (the
  UNet graph of a 512 x 512 image, CFG batch) with its OWN sampler state —
  multistep samplers keep per-window history, as diffusers does since it
  copies the scheduler state per view — and the canvas is the per-pixel mean
  of the windows' updates.  ``circular_padding`` wraps windows around the
  horizontal seam (360-degree panoramas) and decodes with 8 latent columns of
  wrap-around padding on each side.  ``view_batch_size`` is accepted; windows
  are evaluated one at a time (the same math as a batched evaluation).
* ``StableDiffusionSAGPipeline`` (Self-Attention Guidance, Hong et al. 2023):
  the mid-block self-attention map of the unconditional pass marks the
  regions the model attends to (mean over heads, summed over queries > 1);
  the predicted x0 is Gaussian-blurred there (9 taps, sigma 1, reflect
  padding), re-noised to the current level with the predicted noise, and the
  UNet's unconditional prediction on that degraded sample pulls the guided
  prediction away: ``e += sag_scale * (e_uncond - e_degraded)``.  x0 / noise
  use this sampler's own sigma (diffusers reads ``alphas_cumprod[t]``, equal
  up to the rounding of Karras timesteps; exact for DDIM / PNDM ladders).
* ``StableDiffusionPipelineSafe`` (Safe Latent Diffusion, Schramowski et al.
  2023; AIML-TUDA/stable-diffusion-safe): a third CFG row conditioned on a
  safety concept text; where the text prediction comes within
  ``sld_threshold`` of the concept's, the concept direction (scaled by
  ``sld_guidance_scale``, clamped to 1, with momentum) is removed from the
  guidance after ``sld_warmup_steps``.  The UNet runs as one CFG-3 graph.
* ``SemanticStableDiffusionPipeline`` (SEGA, Brack et al. 2023; diffusers
  0.16.1, the reference's pin): one extra CFG row per ``editing_prompt``; each
  concept's direction (edit - uncond, sign-flipped for reverse edits, times
  ``edit_guidance_scale``) keeps only its values at or above the
  ``edit_threshold`` quantile of |direction| per (image, channel), the
  concepts are combined with ``edit_weights`` (re-normalised over the concepts
  that are past warm-up while others still warm up), with momentum, and added
  to the CFG direction between ``edit_warmup_steps`` and
  ``edit_cooldown_steps``.  The UNet runs as one CFG-(2 + k) evaluation.
* ``StableDiffusionAttendAndExcitePipeline`` (Chefer et al. 2023; diffusers
  0.16.1): for the first ``max_iter_to_alter`` steps the text-conditioned UNet
  runs once more with autograd (the torch implementation of every op: the HIP
  kernels have no backward), the cross-attention maps at 16 x 16 queries are
  averaged over heads and layers, softmaxed over the prompt tokens (x100,
  start / end token dropped), Gaussian-smoothed, and the latents take a
  gradient step against max over ``token_indices`` of (1 - max attention),
  step ``scale_factor * sqrt(linspace(1, 0.5))``, with up to 20 refinement
  iterations at the ``thresholds`` steps; the denoising step itself is the
  plain CFG graph.

Parity against diffusers is unpinned (diffusers is not importable here); the
CPU tests pin the window geometry, the per-window sampler independence, the
SAG mask / blur against their formulas, and that sag_scale = 0 and a single
window reproduce the plain pipeline exactly.
"""
from __future__ import annotations

import contextlib
import copy
import math

import torch
import torch.nn.functional as F

PANORAMA = "StableDiffusionPanoramaPipeline"
SAG = "StableDiffusionSAGPipeline"
SAFE = "StableDiffusionPipelineSafe"
SEGA = "SemanticStableDiffusionPipeline"
AE = "StableDiffusionAttendAndExcitePipeline"
CLASSES = (PANORAMA, SAG, SAFE, SEGA, AE)

# StableDiffusionPipelineSafe's default safety concept (Schramowski et al. 2023, I2P categories)
SAFETY_CONCEPT = ("an image showing hate, harassment, violence, suffering, humiliation, harm, suicide, sexual, nudity,"
                  " bodily fluids, blood, obscene gestures, illegal activity, drug use, theft, vandalism, weapons,"
                  " child abuse, brutality, cruelty")

# diffusers StableDiffusionPanoramaPipeline.get_views / decode_latents_with_padding
WINDOW, STRIDE, CIRC_PAD = 64, 8, 8


def panorama_views(lh: int, lw: int, window: int = WINDOW, stride: int = STRIDE, circular: bool = False):
    """(h0, h1, w0, w1) latent windows covering an lh x lw canvas; with
    ``circular`` the windows start every ``stride`` columns all the way round
    (w1 may exceed lw: those wrap)."""
    nh = (lh - window) // stride + 1 if lh > window else 1
    if circular:
        nw = lw // stride if lw > window else 1
    else:
        nw = (lw - window) // stride + 1 if lw > window else 1
    out = []
    for i in range(nh * nw):
        h0 = (i // nw) * stride
        w0 = (i % nw) * stride
        out.append((h0, h0 + window, w0, w0 + window))
    return out


def _take(x, v, lw):
    h0, h1, w0, w1 = v
    if w1 <= lw:
        return x[:, h0:h1, w0:w1]
    return torch.cat([x[:, h0:h1, w0:], x[:, h0:h1, :w1 - lw]], dim=2)


def _accumulate(value, count, xv, v, lw):
    h0, h1, w0, w1 = v
    if w1 <= lw:
        value[:, h0:h1, w0:w1] += xv
        count[:, h0:h1, w0:w1] += 1
        return
    k = lw - w0
    value[:, h0:h1, w0:] += xv[:, :, :k]
    count[:, h0:h1, w0:] += 1
    value[:, h0:h1, :w1 - lw] += xv[:, :, k:]
    count[:, h0:h1, :w1 - lw] += 1


def _guide(e, guidance, cfg):
    if not cfg:
        return e
    e_u, e_c = e.chunk(2)
    return e_u + guidance * (e_c - e_u)


def window_for(pipe) -> tuple[int, int]:
    """(window, stride) in latent pixels: diffusers' 64 / 8 for real checkpoints;
    the family's own latent size / 8 for the test-size families."""
    d = int(pipe.family.default_size) // 8
    if d >= WINDOW:
        return WINDOW, STRIDE
    return d, max(1, d // 8)


@torch.no_grad()
def panorama_denoise(pipe, x, sched, cross_kv, guidance, added, generator, circular=False):
    """MultiDiffusion loop on NHWC fp32 latents [B, lh, lw, 4]."""
    b, lh, lw, _ = x.shape
    window, stride = window_for(pipe)
    views = panorama_views(lh, lw, window, stride, circular=circular)
    cfg = guidance > 1.0
    states = [copy.deepcopy(sched) for _ in views]  # per-window multistep history
    while states[0].step_index < states[0].n:
        value = torch.zeros_like(x)
        count = torch.zeros_like(x[..., :1])
        for v, s in zip(views, states):
            xv = _take(x, v, lw)
            xi = (xv * s.current_scale()).to(pipe.dtype)
            e = pipe._unet_eval(torch.cat([xi, xi], 0) if cfg else xi, s.current_t(), cross_kv, added)
            _accumulate(value, count, s.step(_guide(e.float(), guidance, cfg), xv, generator), v, lw)
        x = torch.where(count > 0, value / count.clamp_min(1), value)
    sched.step_index = sched.n
    return x


def gaussian_blur_nhwc(x: torch.Tensor, kernel_size: int = 9, sigma: float = 1.0) -> torch.Tensor:
    """Depthwise Gaussian blur with reflect padding (diffusers SAG gaussian_blur_2d) on NHWC."""
    half = (kernel_size - 1) * 0.5
    t = torch.linspace(-half, half, kernel_size, device=x.device, dtype=torch.float32)
    pdf = torch.exp(-0.5 * (t / sigma) ** 2)
    k1 = pdf / pdf.sum()
    k2 = (k1[:, None] @ k1[None, :]).to(x.dtype)
    c = x.shape[-1]
    w = k2.expand(c, 1, kernel_size, kernel_size)
    xn = x.permute(0, 3, 1, 2)
    p = kernel_size // 2
    xn = F.pad(xn, (p, p, p, p), mode="reflect")
    return F.conv2d(xn, w, groups=c).permute(0, 2, 3, 1)


def sag_mask(probs: torch.Tensor, lh: int, lw: int) -> torch.Tensor:
    """[B, heads, S, S] attention probabilities of the mid block -> [B, lh, lw, 1]
    {0, 1} mask: keys whose attention (mean over heads, summed over queries)
    exceeds 1, nearest-resized from the mid-block grid to the latent grid."""
    b, _, s, _ = probs.shape
    f = int(round(math.sqrt(lh * lw / s)))
    mh, mw = lh // f, lw // f
    m = (probs.mean(1).sum(1) > 1.0).to(torch.float32).reshape(b, 1, mh, mw)
    return F.interpolate(m, (lh, lw)).permute(0, 2, 3, 1)


def _at_sigma(sched):
    """A view of the sampler at the sigma its NEXT evaluation sees (the second
    stage of Heun / DPM2 evaluates between ladder points), for the x0 / noise
    formulas of ``Scheduler.x0_coeffs`` / ``Scheduler.add_noise``."""
    from types import SimpleNamespace

    return SimpleNamespace(sigmas=[float(sched.eval_sigma())], space=sched.space, n=1,
                           prediction_type=sched.prediction_type, name=sched.name)


def _eps_from(view, x, x0):
    """Noise of sample x given its x0, at the view's sigma."""
    s = float(view.sigmas[0])
    if view.space == "vp":
        a = 1.0 / math.sqrt(s * s + 1.0)
        return (x - a * x0) / (s * a)
    return (x - x0) / s


def _mid_attn(unet):
    return unet.mid_block.attentions[0].transformer_blocks[0].attn1


@torch.no_grad()
def sag_denoise(pipe, x, sched, cross_kv, guidance, added, generator, sag_scale=0.75):
    """Self-attention-guided loop on NHWC fp32 latents.  The UNet runs eagerly
    (its mid-block attention map is read back every step)."""
    b, lh, lw, _ = x.shape
    cfg = guidance > 1.0
    attn = _mid_attn(pipe.unet)
    kv_ref = [t[:b] for t in cross_kv] if cfg else list(cross_kv)
    while sched.step_index < sched.n:
        t = sched.current_t()
        s_in = sched.current_scale()
        tt = torch.tensor([t], device=x.device, dtype=torch.float32)
        xi = (x * s_in).to(pipe.dtype)
        store: list = []
        attn._store_probs = store
        try:
            e = pipe.unet(torch.cat([xi, xi], 0) if cfg else xi, tt, cross_kv=cross_kv, added_cond=added).float()
        finally:
            attn._store_probs = None
        e_ref = e[:b]  # unconditional half (or the only one)
        eg = _guide(e, guidance, cfg)
        if sag_scale != 0.0:
            from ..schedulers import Scheduler

            view = _at_sigma(sched)
            p, q = Scheduler.x0_coeffs(view, 0)
            x0 = p * x + q * e_ref
            eps = _eps_from(view, x, x0)
            m = sag_mask(store[0][:b], lh, lw)
            deg = gaussian_blur_nhwc(x0) * m + x0 * (1 - m)
            deg = Scheduler.add_noise(view, deg, eps, 0)
            ed = pipe.unet((deg * s_in).to(pipe.dtype), tt, cross_kv=kv_ref, added_cond=None).float()
            eg = eg + sag_scale * (e_ref - ed)
        x = sched.step(eg, x, generator)
    return x


@torch.no_grad()
def sld_denoise(pipe, x, sched, cross_kv, guidance, added, generator, safety_kv, sld_guidance_scale=1000.0,
                sld_warmup_steps=10, sld_threshold=0.01, sld_momentum_scale=0.3, sld_mom_beta=0.4):
    """Safe Latent Diffusion loop: CFG batch [uncond, cond, safety concept];
    the guidance direction loses the part of the text direction that points at
    the concept, element-wise where the text prediction is within
    ``sld_threshold`` of the concept's (SLD eqs. 3-8), with momentum, after
    ``sld_warmup_steps`` evaluations."""
    b = x.shape[0]
    kv3 = [torch.cat([kv, s], 0) for kv, s in zip(cross_kv, safety_kv)]
    pipe._kv_static = False  # the UNet graph copies this 3-way K/V, it is not the text graph's output
    mom = None
    i = 0
    while sched.step_index < sched.n:
        xi = (x * sched.current_scale()).to(pipe.dtype)
        e = pipe._unet_eval(torch.cat([xi, xi, xi], 0), sched.current_t(), kv3, added).float()
        e_u, e_t, e_s = e[:b], e[b:2 * b], e[2 * b:]
        g = e_t - e_u
        d = e_t - e_s
        scale = torch.clamp(d.abs() * sld_guidance_scale, max=1.0)
        scale = torch.where(d >= sld_threshold, torch.zeros_like(scale), scale)
        gs = (e_s - e_u) * scale
        if mom is None:
            mom = torch.zeros_like(g)
        gs = gs + sld_momentum_scale * mom
        mom = sld_mom_beta * mom + (1 - sld_mom_beta) * gs
        if i >= sld_warmup_steps:
            g = g - gs
        x = sched.step(e_u + guidance * g, x, generator)
        i += 1
    return x


def _per_concept(v, k, name):
    """a SEGA per-concept option: a scalar for every concept or a list of k"""
    if isinstance(v, (list, tuple)):
        if len(v) != k:
            raise ValueError(f"{name} has {len(v)} entries for {k} editing prompts")
        return list(v)
    return [v] * k


class SegaState:
    """Per-job SEGA guidance (diffusers 0.16.1 SemanticStableDiffusionPipeline
    __call__, the ``enable_edit_guidance`` block), one call per step on fp32
    [b, C, H, W]-shaped predictions (the layout here is NHWC; the quantile is
    over the spatial positions of each (image, channel) either way)."""

    def __init__(self, k, n_steps, edit_guidance_scale=5.0, edit_warmup_steps=10, edit_cooldown_steps=None,
                 edit_threshold=0.9, reverse_editing_direction=False, edit_weights=None, edit_momentum_scale=0.1,
                 edit_mom_beta=0.4):
        self.k = k
        self.scale = [float(v) for v in _per_concept(edit_guidance_scale, k, "edit_guidance_scale")]
        self.warm = [int(v) for v in _per_concept(edit_warmup_steps, k, "edit_warmup_steps")]
        self.cool = [n_steps + 1 if v is None else int(v)
                     for v in _per_concept(edit_cooldown_steps, k, "edit_cooldown_steps")]
        self.thr = [float(v) for v in _per_concept(edit_threshold, k, "edit_threshold")]
        self.rev = [bool(v) for v in _per_concept(reverse_editing_direction, k, "reverse_editing_direction")]
        self.weight = [1.0] * k if edit_weights is None else [float(v) for v in
                                                               _per_concept(edit_weights, k, "edit_weights")]
        self.mom_scale, self.mom_beta = float(edit_momentum_scale), float(edit_mom_beta)
        self.mom = None

    def guidance(self, i, e_u, e_t, edits, guidance_scale):
        """The step's guidance term (added to e_u): CFG plus semantic guidance."""
        g = guidance_scale * (e_t - e_u)
        b = g.shape[0]
        if self.mom is None:
            self.mom = torch.zeros_like(g)
        w = torch.zeros(self.k, b, dtype=g.dtype, device=g.device)
        ge = torch.zeros((self.k,) + tuple(g.shape), dtype=g.dtype, device=g.device)
        warm = []
        for c, e_c in enumerate(edits):
            if i >= self.warm[c]:
                warm.append(c)
            if i >= self.cool[c]:
                continue  # this concept's direction is zero from its cool-down on
            d = (e_c - e_u) * (-1.0 if self.rev[c] else 1.0) * self.scale[c]
            w[c] = self.weight[c]
            flat = d.abs().reshape(b, -1, d.shape[-1])  # [b, positions, channels]
            q = torch.quantile(flat, self.thr[c], dim=1)  # [b, channels]
            ge[c] = torch.where(d.abs() >= q.view(b, *([1] * (d.dim() - 2)), -1), d, torch.zeros_like(d))
        if 0 < len(warm) < self.k:  # some concepts still warm up: the others, re-weighted, now
            idx = torch.tensor(warm, device=g.device)
            wt = w.index_select(0, idx).clamp(min=0)
            wt = wt / wt.sum(0)
            g = g + torch.einsum("cb,cb...->b...", wt, ge.index_select(0, idx))
        w = torch.nan_to_num(w.clamp(min=0))
        edit = torch.einsum("cb,cb...->b...", w, ge) + self.mom_scale * self.mom
        self.mom = self.mom_beta * self.mom + (1 - self.mom_beta) * edit
        if len(warm) == self.k:
            g = g + edit
        return g


def sega_denoise(pipe, x, sched, cross_kv, guidance, added, generator, edit_kv, state: SegaState):
    """SEGA loop: CFG batch [uncond, cond, edit_1, ..., edit_k] per step."""
    b, k = x.shape[0], state.k
    kvk = [torch.cat([kv] + [e[j] for e in edit_kv], 0) for j, kv in enumerate(cross_kv)]
    pipe._kv_static = False  # the UNet copies this (2 + k)-way K/V, it is not the text graph's output
    i = 0
    while sched.step_index < sched.n:
        xi = (x * sched.current_scale()).to(pipe.dtype)
        e = pipe._unet_eval(torch.cat([xi] * (2 + k), 0), sched.current_t(), kvk, added).float()
        e_u, e_t = e[:b], e[b:2 * b]
        edits = [e[(2 + c) * b:(3 + c) * b] for c in range(k)]
        x = sched.step(e_u + state.guidance(i, e_u, e_t, edits, guidance), x, generator)
        i += 1
    return x


def ae_gauss_kernel(kernel_size=3, sigma=0.5):
    """The prompt-to-prompt GaussianSmoothing kernel diffusers' A&E uses:
    exp(-((x - mu) / (2 sigma))^2) per axis (its quirk: 2 sigma, not 2 sigma^2),
    outer product, normalised to sum 1."""
    g = torch.arange(kernel_size, dtype=torch.float32) - (kernel_size - 1) / 2
    g = torch.exp(-((g / (2 * sigma)) ** 2)) / (sigma * math.sqrt(2 * math.pi))
    k = g[:, None] * g[None, :]
    return k / k.sum()


def ae_max_attention(maps, indices, res):
    """Per token index, the max over the (res x res) map of the smoothed,
    token-softmaxed cross-attention (diffusers 0.16.1
    _compute_max_attention_per_index on AttentionStore.aggregate_attention)."""
    a = torch.cat([m.reshape(-1, res, res, m.shape[-1]) for m in maps], 0)
    a = a.sum(0) / a.shape[0]
    t = torch.softmax(a[:, :, 1:-1] * 100, dim=-1)
    ker = ae_gauss_kernel().to(t)[None, None]
    out = []
    for i in indices:
        img = F.pad(t[:, :, int(i) - 1][None, None], (1, 1, 1, 1), mode="reflect")
        out.append(F.conv2d(img, ker)[0, 0].max())
    return out


def ae_loss(maxes):
    return torch.stack([torch.clamp(1.0 - m, min=0.0) for m in maxes]).max()


@contextlib.contextmanager
def _reference_ops():
    from .. import ops

    prev = ops.get_mode()
    ops.set_mode("reference")
    try:
        yield
    finally:
        ops.set_mode(prev)


def _ae_maxes(pipe, x, t, kv_cond, indices, res):
    """One text-conditioned UNet pass with autograd from ``x`` (leaf with
    grad): the maxima per token index, in the graph."""
    from ..models.layers import Attention

    mods = [m for m in pipe.unet.modules() if isinstance(m, Attention) and m.is_cross]
    store: list = []
    for m in mods:
        m._store_probs = store
    try:
        with torch.enable_grad(), _reference_ops():
            tt = torch.tensor([float(t)], device=x.device, dtype=torch.float32)
            pipe.unet(x.to(pipe.dtype), tt, cross_kv=kv_cond, added_cond=None)
    finally:
        for m in mods:
            m.__dict__.pop("_store_probs", None)
    maps = [p for p in store if p.shape[-2] == res * res]
    if not maps:
        raise ValueError(f"{AE}: no cross-attention maps at {res} x {res} (attn_res) for this image size")
    with torch.enable_grad():
        return ae_max_attention(maps, indices, res)


def _ae_step(x, loss, step):
    g, = torch.autograd.grad(loss, [x])
    return (x - step * g).detach().requires_grad_(True)


def ae_denoise(pipe, x, sched, cross_kv, guidance, added, generator, token_indices, max_iter_to_alter=25,
               thresholds=None, scale_factor=20.0, attn_res=16, max_refinement_steps=20):
    """Attend-and-Excite loop (diffusers 0.16.1 __call__ / _perform_iterative_refinement_step)."""
    import numpy as np

    thresholds = {0: 0.05, 10: 0.5, 20: 0.8} if thresholds is None else {int(k): float(v)
                                                                         for k, v in thresholds.items()}
    b = x.shape[0]
    cfg = guidance > 1.0
    kv_cond = [kv[b:] if cfg else kv for kv in cross_kv]
    steps = scale_factor * np.sqrt(np.linspace(1.0, 0.5, sched.n))
    i = 0
    while sched.step_index < sched.n:
        t = sched.current_t()
        if i < max_iter_to_alter:
            with torch.enable_grad():  # (the pipeline's denoise runs under no_grad)
                xg = x.detach().requires_grad_(True)
                maxes = _ae_maxes(pipe, xg, t, kv_cond, token_indices, attn_res)
                loss = ae_loss(maxes)
                if i in thresholds and loss.item() > 1.0 - thresholds[i]:
                    target, it = max(0.0, 1.0 - thresholds[i]), 0
                    while loss.item() > target:
                        it += 1
                        xg = xg.detach().requires_grad_(True)
                        loss = ae_loss(_ae_maxes(pipe, xg, t, kv_cond, token_indices, attn_res))
                        if loss.item() != 0:
                            xg = _ae_step(xg, loss, float(steps[i]))
                        if it >= max_refinement_steps:
                            break
                    xg = xg.detach().requires_grad_(True)  # one more pass: the loss the step below uses
                    maxes = _ae_maxes(pipe, xg, t, kv_cond, token_indices, attn_res)
                loss = ae_loss(maxes)
                if loss.item() != 0:
                    xg = _ae_step(xg, loss, float(steps[i]))
            x = xg.detach()
        xi = (x * sched.current_scale()).to(pipe.dtype)
        e = pipe._unet_eval(torch.cat([xi, xi], 0) if cfg else xi, t, cross_kv, added).float()
        if cfg:
            e_u, e_t = e.chunk(2)
            e = e_u + guidance * (e_t - e_u)
        x = sched.step(e, x, generator)
        i += 1
    return x


@contextlib.contextmanager
def _override(pipe, denoise, decode=None):
    pipe._denoise_override = denoise
    if decode is not None:
        pipe.decode = decode
    try:
        yield
    finally:
        pipe._denoise_override = None
        pipe.__dict__.pop("decode", None)


def _check(pipe, cls, kwargs):
    if pipe.family.is_xl or pipe.family.is_pix2pix or pipe.family.is_depth or pipe.unet.cfg.in_channels != 4:
        raise ValueError(f"{cls} runs plain Stable Diffusion checkpoints, not {pipe.family.name}")
    bad = sorted(k for k in ("image", "mask_image", "strength", "image_guidance_scale", "depth_map",
                             "controlnet_conditioning_scale", "cfg_split") if k in kwargs)
    if bad:
        raise TypeError(f"{cls}.__call__() got unexpected keyword arguments {bad}")
    if getattr(pipe, "controlnet", None) is not None:
        raise ValueError(f"{cls} does not take a ControlNet")


def run_panorama(pipe, height=None, width=None, view_batch_size=1, circular_padding=False, **kwargs):
    """``StableDiffusionPanoramaPipeline.__call__`` (diffusers defaults 512 x 2048)."""
    _check(pipe, PANORAMA, kwargs)
    if int(view_batch_size) < 1:
        raise ValueError("view_batch_size must be >= 1")
    circ = bool(circular_padding)

    def denoise(p, x, sched, cross_kv, guidance, added, generator, **_):
        return panorama_denoise(p, x, sched, cross_kv, guidance, added, generator, circular=circ)

    decode = None
    if circ:
        plain = pipe.decode

        def decode(latents, to_host=True):  # wrap-around columns on both sides, cropped after the VAE
            pad = min(CIRC_PAD, window_for(pipe)[0] // 2)  # 8 latent columns (test-size families: fewer)
            z = torch.cat([latents[:, :, -pad:], latents, latents[:, :, :pad]], dim=2)
            img = plain(z, to_host=False)
            px = pad * 8
            img = img[:, :, px:img.shape[2] - px].contiguous()
            return img.cpu() if to_host else img

    w = window_for(pipe)[0] * 8
    with _override(pipe, denoise, decode):
        return pipe(height=height or w, width=width or 4 * w, **kwargs)


def run_sag(pipe, sag_scale=0.75, **kwargs):
    """``StableDiffusionSAGPipeline.__call__``."""
    _check(pipe, SAG, kwargs)
    s = float(sag_scale)

    def denoise(p, x, sched, cross_kv, guidance, added, generator, **_):
        return sag_denoise(p, x, sched, cross_kv, guidance, added, generator, sag_scale=s)

    with _override(pipe, denoise):
        return pipe(**kwargs)


def run_safe(pipe, sld_guidance_scale=1000, sld_warmup_steps=10, sld_threshold=0.01, sld_momentum_scale=0.3,
             sld_mom_beta=0.4, safety_concept=None, **kwargs):
    """``StableDiffusionPipelineSafe.__call__``: safety guidance runs when
    ``sld_guidance_scale > 1`` and classifier-free guidance is on; otherwise
    the plain loop."""
    _check(pipe, SAFE, kwargs)
    concept = SAFETY_CONCEPT if safety_concept is None else str(safety_concept)
    if not (float(sld_guidance_scale) > 1.0 and float(kwargs.get("guidance_scale", 7.5)) > 1.0):
        return pipe(**kwargs)
    n = max(1, int(kwargs.get("num_images_per_prompt", 1) or 1))
    prompt = kwargs.get("prompt", "")
    b = (len(prompt) if isinstance(prompt, list) else 1) * n
    _, _, skv = pipe.encode([concept] * b, [""] * b, cfg=False)
    skv = [t.clone() for t in skv]  # (the text graph's static outputs are rewritten by the next encode)
    opts = dict(sld_guidance_scale=float(sld_guidance_scale), sld_warmup_steps=int(sld_warmup_steps),
                sld_threshold=float(sld_threshold), sld_momentum_scale=float(sld_momentum_scale),
                sld_mom_beta=float(sld_mom_beta))

    def denoise(p, x, sched, cross_kv, guidance, added, generator, **_):
        return sld_denoise(p, x, sched, cross_kv, guidance, added, generator, skv, **opts)

    with _override(pipe, denoise):
        out = pipe(**kwargs)
    out.applied_safety_concept = concept
    return out


def run_sega(pipe, editing_prompt=None, editing_prompt_embeddings=None, reverse_editing_direction=False,
             edit_guidance_scale=5, edit_warmup_steps=10, edit_cooldown_steps=None, edit_threshold=0.9,
             edit_momentum_scale=0.1, edit_mom_beta=0.4, edit_weights=None, sem_guidance=None, **kwargs):
    """``SemanticStableDiffusionPipeline.__call__``: with no editing prompt (or
    no classifier-free guidance) the plain loop."""
    _check(pipe, SEGA, kwargs)
    if editing_prompt_embeddings is not None or sem_guidance is not None:
        raise TypeError(f"{SEGA}: editing_prompt_embeddings / sem_guidance (tensors) are not accepted in a job")
    concepts = [editing_prompt] if isinstance(editing_prompt, str) else list(editing_prompt or [])
    if not concepts or not float(kwargs.get("guidance_scale", 7.5)) > 1.0:
        return pipe(**kwargs)
    n = max(1, int(kwargs.get("num_images_per_prompt", 1) or 1))
    prompt = kwargs.get("prompt", "")
    b = (len(prompt) if isinstance(prompt, list) else 1) * n
    edit_kv = []
    for c in concepts:
        _, _, kv = pipe.encode([str(c)] * b, [""] * b, cfg=False)
        edit_kv.append([t.clone() for t in kv])  # (the text graph's static outputs are rewritten by the next encode)
    steps = int(kwargs.get("num_inference_steps", 50))
    opts = dict(edit_guidance_scale=edit_guidance_scale, edit_warmup_steps=edit_warmup_steps,
                edit_cooldown_steps=edit_cooldown_steps, edit_threshold=edit_threshold,
                reverse_editing_direction=reverse_editing_direction, edit_weights=edit_weights,
                edit_momentum_scale=edit_momentum_scale, edit_mom_beta=edit_mom_beta)
    SegaState(len(concepts), steps, **opts)  # option errors before any UNet work

    def denoise(p, x, sched, cross_kv, guidance, added, generator, **_):
        return sega_denoise(p, x, sched, cross_kv, guidance, added, generator, edit_kv,
                            SegaState(len(concepts), steps, **opts))

    with _override(pipe, denoise):
        return pipe(**kwargs)


def run_attend_and_excite(pipe, token_indices=None, max_iter_to_alter=25, thresholds=None, scale_factor=20,
                          attn_res=16, **kwargs):
    """``StableDiffusionAttendAndExcitePipeline.__call__`` (one prompt, one image,
    as diffusers 0.16.1 runs it: its gradient pass takes prompt_embeds[1])."""
    _check(pipe, AE, kwargs)
    if token_indices is None or not list(token_indices):
        raise TypeError(f"{AE}.__call__() missing required argument 'token_indices'")
    idx = [int(i) for i in token_indices]
    if min(idx) < 1 or max(idx) > 75:
        raise ValueError(f"{AE}: token_indices must lie in 1..75 (prompt tokens after the start token)")
    prompt = kwargs.get("prompt", "")
    if isinstance(prompt, list) and len(prompt) != 1 or int(kwargs.get("num_images_per_prompt", 1) or 1) != 1:
        raise ValueError(f"{AE} runs one prompt and one image per call")
    opts = dict(token_indices=idx, max_iter_to_alter=int(max_iter_to_alter), thresholds=thresholds,
                scale_factor=float(scale_factor), attn_res=int(attn_res))

    def denoise(p, x, sched, cross_kv, guidance, added, generator, **_):
        return ae_denoise(p, x, sched, cross_kv, guidance, added, generator, **opts)

    with _override(pipe, denoise):
        return pipe(**kwargs)


def run(cls, pipe, **kwargs):
    if cls == AE:
        return run_attend_and_excite(pipe, **kwargs)
    if cls == PANORAMA:
        return run_panorama(pipe, **kwargs)
    if cls == SAFE:
        return run_safe(pipe, **kwargs)
    if cls == SEGA:
        return run_sega(pipe, **kwargs)
    return run_sag(pipe, **kwargs)
