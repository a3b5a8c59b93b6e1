"""Diffusion upscalers.

* ``LatentUpscaler`` — the ``upscale: true`` option of txt2img/img2img jobs
  (reference: swarm/diffusion/upscale.py:6-32, stabilityai/sd-x2-latent-upscaler,
  20 steps, guidance 0).  Images are VAE-encoded; the k-diffusion K-UNet
  (``models.kunet``) denoises at twice the latent resolution conditioned on the
  nearest-upsampled low-res latents, the pooled CLIP-L text (mapping network)
  and the pre-final-LayerNorm CLIP-L hidden states (cross-attention), with the
  Karras preconditioning (c_noise = log(sigma)/4, x0 = x/(s^2+1) +
  s/sqrt(s^2+1) F, Euler); the VAE decodes at 2x.  Unlike the reference (which
  returned only ``images[0]``) every image is upscaled, as one batch.
* ``X4Upscaler`` — stabilityai/stable-diffusion-x4-upscaler, the third stage
  of DeepFloyd IF (reference: swarm/diffusion/diffusion_func_if.py:36-40,
  :63-65): 7-channel UNet (4 latent + 3 noised low-res RGB) with the noise
  level as a class embedding, v-prediction, OpenCLIP-H text context, f=4 VAE.

Both replay their UNet step from a hipGraph (``graphs.GraphCache``) and use
the same fused sampler-step kernel as the SD path.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from PIL import Image

from .. import ops
from ..models import clip as clip_mod
from ..models.layers import init_random_fast_, prepare_model
from ..models.tokenizer import CLIPTokenizer
from ..models.weights import tokenizer_dir
from ..models.kunet import LATENT_X2_K, TINY_X2_K, KUNet2DConditionModel
from ..models.unet import TINY_X4, X4_UPSCALER, UNet2DConditionModel
from ..models.vae import SD_VAE, TINY_VAE, AutoencoderKL, VAEConfig
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights
from ..schedulers import get_scheduler
from .graphs import GraphCache

X4_VAE = VAEConfig(block_out_channels=(128, 256, 512), scaling_factor=0.08333)
TINY_X4_VAE = VAEConfig(block_out_channels=(32, 32, 32), layers_per_block=1, scaling_factor=0.08333)


def _to_nhwc(images, device) -> torch.Tensor:
    """PIL list or NHWC [-1, 1] tensor -> NHWC fp32 [-1, 1] on device."""
    if torch.is_tensor(images):
        return images.to(device).float()
    arr = np.stack([np.asarray(im.convert("RGB"), dtype=np.float32) for im in images]) / 127.5 - 1.0
    return torch.from_numpy(arr).to(device)


def _to_pil(img_u8: torch.Tensor) -> list[Image.Image]:
    return [Image.fromarray(a.numpy()) for a in img_u8]


class _Base:
    def _init(self, mods, seed, weights_dir, parts):
        for i, m in enumerate(mods):
            m.eval().requires_grad_(False)
            init_random_fast_(m, seed=seed + i)
        self.weights_source = "random-init"
        if weights_dir:
            from ..models.weights import _VAE_RENAMES, load_component

            reps = [load_component(m, weights_dir, sub, _VAE_RENAMES if sub == "vae" else None) for sub, m in parts]
            if any(r is not None for r in reps):
                self.weights_source = str(weights_dir)
        for m in mods:
            prepare_model(m)

    def _unet_fn(self, x, t, kv, class_labels=None):
        return self.unet(x, t, cross_kv=list(kv), class_labels=class_labels)

    def _encode_text(self, prompts):
        ids = self.tokenizer(prompts).to(self.device)
        last, _, _, _ = self.text_encoder(ids)
        return self.unet.encode_context(last)

    def _denoise(self, x, sched, kv, guidance, cond_img, class_labels, generator):
        cfg = guidance > 1.0
        t_dev = torch.zeros(1, device=self.device, dtype=torch.float32)
        cond = torch.cat([cond_img, cond_img], 0) if cfg else cond_img
        cl = class_labels
        if cl is not None and cfg:
            cl = torch.cat([cl, cl], 0)
        while sched.step_index < sched.n:
            xi = (x * sched.current_scale()).to(self.dtype)
            x_in = torch.cat([torch.cat([xi, xi], 0) if cfg else xi, cond.to(self.dtype)], -1)
            t_dev.fill_(float(sched.current_t()))
            extra = {"class_labels": cl} if cl is not None else {}
            e = self._graphs(self.device, x=x_in, t=t_dev, kv=tuple(kv), **extra)
            coeffs = sched.fused_coeffs()
            if coeffs is not None and ops.use_hip(x):
                nz = (torch.randn(x.shape, generator=generator, device=x.device, dtype=torch.float32)
                      if coeffs.D != 0.0 else None)
                x = ops.sched_step(e, x, sched, coeffs, guidance if cfg else None, nz)
            else:
                if cfg:
                    e_u, e_c = e.float().chunk(2)
                    eg = e_u + guidance * (e_c - e_u)
                else:
                    eg = e.float()
                x = sched.step(eg, x, generator)
        return x


class LatentUpscaler(_Base):
    def __init__(self, device="cpu", tiny=False, seed=11, weights_dir=None):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        tcfg = clip_mod.TINY_TEXT if tiny else clip_mod.CLIP_L
        with torch.device(self.device):
            self.unet = KUNet2DConditionModel(TINY_X2_K if tiny else LATENT_X2_K).to(self.dtype)
            self.vae = AutoencoderKL(TINY_VAE if tiny else SD_VAE).to(self.dtype)
            self.text_encoder = clip_mod.CLIPTextModel(tcfg).to(self.dtype)
        self._init([self.unet, self.vae, self.text_encoder], seed, weights_dir,
                   [("unet", self.unet), ("vae", self.vae), ("text_encoder", self.text_encoder)])
        self.tokenizer = CLIPTokenizer(tokenizer_dir(weights_dir), 77, vocab_size=tcfg.vocab_size)
        self._graphs = GraphCache(self._kunet_fn)
        self.f = 2 ** (len(self.vae.cfg.block_out_channels) - 1)

    def _kunet_fn(self, x, c, cond, kv):
        return self.unet(x, c, cond, cross_kv=list(kv))

    def _text(self, prompts):
        """(cross-attention K/V of the pre-final-LN hidden states, pooled) per prompt."""
        ids = self.tokenizer(prompts).to(self.device)
        hidden, pooled = self.text_encoder.encode_pre_ln(ids)
        return self.unet.encode_context(hidden), pooled

    @torch.no_grad()
    def __call__(self, prompt, images, num_inference_steps=20, guidance_scale=0.0, generator=None, latents=None,
                 negative_prompt=None):
        """images: PIL list (or SD latents via ``latents`` [B, h, w, 4], scaled) -> 2x PIL images."""
        if latents is None:
            x = _to_nhwc(images, self.device)
            latents = self.vae.encode(x.to(self.dtype), generator=generator, sample=True) * self.vae.cfg.scaling_factor
        b, h, w, c = latents.shape
        prompts = prompt if isinstance(prompt, list) else [prompt] * b
        cfg = guidance_scale > 1.0
        negs = negative_prompt if isinstance(negative_prompt, list) else [negative_prompt or ""] * b
        kv, pooled = self._text((negs + prompts) if cfg else prompts)
        nb = pooled.shape[0]
        # low-res noise level 0: inv_noise_level 1 and Fourier(log1p(0)) = [cos 0 | sin 0]
        half = (self.unet.cfg.time_cond_proj_dim - pooled.shape[-1]) // 2
        cond_vec = torch.cat([torch.ones(nb, half, device=self.device), torch.zeros(nb, half, device=self.device),
                              pooled.float()], -1).to(self.dtype)
        low = latents.float().repeat_interleave(2, 1).repeat_interleave(2, 2)  # nearest x2
        low = (torch.cat([low, low], 0) if cfg else low).to(self.dtype)
        sched = get_scheduler("EulerDiscreteScheduler", use_karras_sigmas=False, prediction_type="k_denoiser")
        sched.set_timesteps(num_inference_steps)
        noise = torch.randn((b, c, 2 * h, 2 * w), generator=generator, device=self.device, dtype=torch.float32)
        x = noise.permute(0, 2, 3, 1).contiguous() * sched.init_noise_sigma
        c_dev = torch.zeros(nb, device=self.device, dtype=torch.float32)
        while sched.step_index < sched.n:
            xi = (x * sched.current_scale()).to(self.dtype)
            x_in = torch.cat([torch.cat([xi, xi], 0) if cfg else xi, low], -1)
            c_dev.fill_(math.log(max(sched.eval_sigma(), 1e-10)) * 0.25)
            e = self._graphs(self.device, x=x_in, c=c_dev, cond=cond_vec, kv=tuple(kv))
            coeffs = sched.fused_coeffs()
            if ops.use_hip(x):
                x = ops.sched_step(e, x, sched, coeffs, guidance_scale if cfg else None, None)
            else:
                if cfg:
                    e_u, e_c = e.float().chunk(2)
                    eg = e_u + guidance_scale * (e_c - e_u)
                else:
                    eg = e.float()
                x = sched.step(eg, x, generator)
        img = self.vae.decode((x / self.vae.cfg.scaling_factor).to(self.dtype))
        return _to_pil(ops.vae_postprocess(img).cpu())


class X4Upscaler(_Base):
    def __init__(self, device="cpu", tiny=False, seed=21, weights_dir=None):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        tcfg = clip_mod.TINY_TEXT if tiny else clip_mod.OPENCLIP_H
        with torch.device(self.device):
            self.unet = UNet2DConditionModel(TINY_X4 if tiny else X4_UPSCALER).to(self.dtype)
            self.vae = AutoencoderKL(TINY_X4_VAE if tiny else X4_VAE, with_encoder=False).to(self.dtype)
            self.text_encoder = clip_mod.CLIPTextModel(tcfg).to(self.dtype)
        self._init([self.unet, self.vae, self.text_encoder], seed, weights_dir,
                   [("unet", self.unet), ("vae", self.vae), ("text_encoder", self.text_encoder)])
        self.tokenizer = CLIPTokenizer(tokenizer_dir(weights_dir), 77, pad_with_eos=False, vocab_size=tcfg.vocab_size)
        self._graphs = GraphCache(self._unet_fn)
        # low_res_scheduler: DDPM linear betas 1e-4 .. 2e-2
        betas = np.linspace(1e-4, 0.02, 1000, dtype=np.float64)
        self.low_res_acp = np.cumprod(1.0 - betas)
        # the denoising scheduler's training schedule: the checkpoint's
        # scheduler/scheduler_config.json, else the published x4 config
        # (DDIM, scaled_linear 1e-4 .. 2e-2, v-prediction, leading + offset 1)
        self._sched_cfg = {"beta_start": 0.0001, "beta_end": 0.02, "beta_schedule": "scaled_linear",
                           "prediction_type": "v_prediction", "steps_offset": 1}
        if weights_dir:
            import json
            import os

            from ..models.hf_config import scheduler_kwargs

            f = os.path.join(weights_dir, "scheduler", "scheduler_config.json")
            if os.path.exists(f):
                with open(f) as fh:
                    self._sched_cfg.update(scheduler_kwargs(json.load(fh)))

    def scheduler_kwargs(self) -> dict:
        return dict(self._sched_cfg)

    @torch.no_grad()
    def __call__(self, prompt, image, num_inference_steps=75, guidance_scale=9.0, noise_level=20,
                 negative_prompt=None, generator=None, scheduler=None):
        """image: PIL list or NHWC [-1, 1] tensor [B, h, w, 3] -> 4x PIL images."""
        img = _to_nhwc(image if isinstance(image, (list, torch.Tensor)) else [image], self.device)
        b, h, w, _ = img.shape
        prompts = prompt if isinstance(prompt, list) else [prompt] * b
        negs = negative_prompt if isinstance(negative_prompt, list) else [negative_prompt or ""] * b
        cfg = guidance_scale > 1.0
        kv = self._encode_text((negs + prompts) if cfg else prompts)
        acp = float(self.low_res_acp[int(noise_level)])
        nz = torch.randn(img.shape, generator=generator, device=self.device, dtype=torch.float32)
        cond = img * acp ** 0.5 + nz * (1 - acp) ** 0.5
        labels = torch.full((b,), int(noise_level), device=self.device, dtype=torch.long)
        sched = scheduler or get_scheduler("DDIMScheduler", use_karras_sigmas=False, **self.scheduler_kwargs())
        sched.prediction_type = self._sched_cfg.get("prediction_type", "v_prediction")
        sched.set_timesteps(num_inference_steps)
        noise = torch.randn((b, 4, h, w), generator=generator, device=self.device, dtype=torch.float32)
        x = noise.permute(0, 2, 3, 1).contiguous() * sched.init_noise_sigma
        x = self._denoise(x, sched, kv, guidance_scale, cond, labels, generator)
        out = self.vae.decode((x / self.vae.cfg.scaling_factor).to(self.dtype))
        return _to_pil(ops.vae_postprocess(out).cpu())


def load_latent_upscaler(device: str, model_name: str = "stabilityai/sd-x2-latent-upscaler") -> LatentUpscaler:
    tiny = model_name.startswith("tiny")
    return cache().get(("x2", model_name, str(device)),
                       lambda: LatentUpscaler(device, tiny=tiny, weights_dir=ensure_weights(model_name)))


def load_x4_upscaler(device: str, model_name: str = "stabilityai/stable-diffusion-x4-upscaler",
                     tiny: bool | None = None) -> X4Upscaler:
    tiny = model_name.startswith("tiny") if tiny is None else tiny
    return cache().get(("x4", model_name, str(device), tiny),
                       lambda: X4Upscaler(device, tiny=tiny, weights_dir=ensure_weights(model_name)))


def upscale_images(images, device_identifier, prompt, generator=None, num_inference_steps=20,
                   model_name="stabilityai/sd-x2-latent-upscaler"):
    """The ``upscale: true`` job option: every image x2 (one batched call)."""
    up = load_latent_upscaler(device_identifier, model_name)
    gen = generator if generator is not None else torch.Generator(device=up.device).manual_seed(0)
    return up([prompt] * len(images), images, num_inference_steps=num_inference_steps, guidance_scale=0.0,
              generator=gen)
