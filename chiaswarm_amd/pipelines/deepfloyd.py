"""DeepFloyd IF three-stage cascade (reference:
swarm/diffusion/diffusion_func_if.py:14-92).

  stage I   T5-XXL prompt embedding -> 64x64 pixel diffusion (IF-I-*)
  stage II  64 -> 256 pixel super-resolution conditioned on the noised,
            upsampled stage-I image and its noise level (IF-II-L)
  stage III 256 -> 1024 with the SD x4 upscaler (noise_level 100)

Differences by design (SURVEY §2.13 fixes): the negative prompt is the
job's ``negative_prompt`` (the reference passed the prompt itself,
diffusion_func_if.py:44); nothing is written to the CWD (:66); the NSFW flag
comes from the checker's output.  All three stages stay resident (no CPU
offload, 288 GB HBM) and every UNet step replays from a hipGraph.

Stage I/II sample with DDPM-family schedulers on the epsilon half of the
6-channel UNet output (the learned-variance half is dropped: fixed-variance
sampling) with IF's ``squaredcos_cap_v2`` noise schedule and Imagen dynamic
thresholding of the x0 prediction (``Scheduler.threshold_x0``).  Geometry and sampler
details are parity-unpinned (no IF checkpoint in this image).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..models.if_unet import IF_I_XL, IF_II_L, TINY_IF_I, TINY_IF_II, IFUNet
from ..models.layers import init_random_fast_, prepare_model
from ..models.t5 import T5_XXL, TINY_T5, T5Encoder, T5Tokenizer
from ..output.processor import OutputProcessor
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights
from ..schedulers import get_scheduler
from .graphs import GraphCache
from .upscale import load_x4_upscaler

# IF-I / IF-II scheduler_config: cosine betas, epsilon half of the learned-range
# output, Imagen dynamic thresholding (ratio 0.95, sample_max_value 1.5)
IF_SCHED = dict(beta_schedule="squaredcos_cap_v2", use_karras_sigmas=False, prediction_type="epsilon",
                thresholding=True, dynamic_thresholding_ratio=0.95, sample_max_value=1.5)


def _cos_acp(n=1000):
    from ..schedulers import _betas

    return np.cumprod(1 - _betas(n, schedule="squaredcos_cap_v2"))


class IFCascade:
    def __init__(self, device="cpu", tiny=False, seed=5, weights_dir=None, stage2_dir=None):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        with torch.device(self.device):
            self.t5 = T5Encoder(TINY_T5 if tiny else T5_XXL).to(self.dtype)
            self.stage1 = IFUNet(TINY_IF_I if tiny else IF_I_XL).to(self.dtype)
            self.stage2 = IFUNet(TINY_IF_II if tiny else IF_II_L).to(self.dtype)
        mods = [self.t5, self.stage1, self.stage2]
        for i, m in enumerate(mods):
            m.eval().requires_grad_(False)
            init_random_fast_(m, seed=seed + i)
        self.weights_source = "random-init"
        self._load(weights_dir, stage2_dir)
        for m in mods:
            prepare_model(m)
        from ..models.weights import CheckpointMismatch, tokenizer_dir

        if self.weights_source != "random-init" and tokenizer_dir(weights_dir) is None:
            # real T5 weights fed hash-fallback ids would condition on a random prompt
            raise CheckpointMismatch(f"{weights_dir}: tokenizer/spiece.model missing beside real T5 weights")
        self.tokenizer = T5Tokenizer(tokenizer_dir(weights_dir), 77, vocab=self.t5.cfg.vocab)
        self.tiny = tiny
        self.acp = _cos_acp()
        self._g1 = GraphCache(self._s1)
        self._g2 = GraphCache(self._s2)

    def _load(self, d1, d2):

        from ..models.weights import load_component

        from ..models.weights import CheckpointMismatch

        got = []
        for d, parts in ((d1, (("text_encoder", self.t5), ("unet", self.stage1))), (d2, (("unet", self.stage2),))):
            for sub, m in parts if d else ():
                if load_component(m, d, sub) is not None:
                    got.append(f"{'stage1' if d is d1 else 'stage2'}/{sub}")
        if got and len(got) != 3:
            # stage I with a random stage II (or T5) would still emit an image
            raise CheckpointMismatch(f"IF cascade: only {got} of stage1/text_encoder, stage1/unet, stage2/unet "
                                     "have weights; refusing a partial load")
        if got:
            self.weights_source = str(d1)

    def _s1(self, x, t, kv, temb):
        return self.stage1(x, t, list(kv), temb)

    def _s2(self, x, t, kv, temb, nl):
        return self.stage2(x, t, list(kv), temb, noise_level=nl)

    @torch.no_grad()
    def encode_prompt(self, prompts, negatives):
        ids, mask = self.tokenizer(negatives + prompts)
        return self.t5(ids.to(self.device), mask.to(self.device))

    def _sample(self, unet, graphs, x, states, steps, guidance, generator, cond=None, noise_level=None):
        kv, temb = unet.encode_context(states)
        sched = get_scheduler("DDPMScheduler", **IF_SCHED)
        sched.set_timesteps(steps)
        t_dev = torch.zeros(1, device=self.device, dtype=torch.float32)
        b = x.shape[0]
        nl = None
        if noise_level is not None:
            nl = torch.full((2 * b,), float(noise_level), device=self.device)
        while sched.step_index < sched.n:
            xi = (x * sched.current_scale()).to(self.dtype)
            x_in = torch.cat([xi, xi], 0)
            if cond is not None:
                x_in = torch.cat([x_in, torch.cat([cond, cond], 0).to(self.dtype)], -1)
            t_dev.fill_(float(sched.current_t()))
            extra = {"nl": nl} if nl is not None else {}
            out = graphs(self.device, x=x_in, t=t_dev, kv=tuple(kv), temb=temb, **extra)
            e = out[..., :3]
            e_u, e_c = e.float().chunk(2)
            x = sched.step(e_u + guidance * (e_c - e_u), x, generator)
        return x.clamp(-1, 1)

    @torch.no_grad()
    def __call__(self, prompt="", negative_prompt=None, num_images_per_prompt=1, generator=None,
                 stage1_steps=100, stage2_steps=50, stage3_steps=75, guidance_scale=7.0, stage2_guidance=4.0,
                 stage3_guidance=9.0, noise_level_2=250, noise_level_3=100, **unused):
        prompts = [prompt] * num_images_per_prompt if isinstance(prompt, str) else list(prompt)
        b = len(prompts)
        neg = negative_prompt or ""
        negs = [neg] * b if isinstance(neg, str) else list(neg)
        states = self.encode_prompt(prompts, negs)
        s1 = self.stage1.cfg.sample_size
        x = torch.randn((b, 3, s1, s1), generator=generator, device=self.device).permute(0, 2, 3, 1).contiguous()
        img64 = self._sample(self.stage1, self._g1, x, states, stage1_steps, guidance_scale, generator)
        # stage II: upsample + noise the low-res image at noise_level_2
        s2 = self.stage2.cfg.sample_size
        up = F.interpolate(img64.permute(0, 3, 1, 2), (s2, s2), mode="bilinear", align_corners=True)
        up = up.permute(0, 2, 3, 1).contiguous()
        a = float(self.acp[noise_level_2])
        up = up * a ** 0.5 + torch.randn(up.shape, generator=generator, device=self.device) * (1 - a) ** 0.5
        x = torch.randn((b, 3, s2, s2), generator=generator, device=self.device).permute(0, 2, 3, 1).contiguous()
        img256 = self._sample(self.stage2, self._g2, x, states, stage2_steps, stage2_guidance, generator,
                              cond=up, noise_level=noise_level_2)
        # stage III: SD x4 upscaler
        x4 = load_x4_upscaler(str(self.device), tiny=self.tiny)
        return x4(prompts, img256, num_inference_steps=stage3_steps, guidance_scale=stage3_guidance,
                  noise_level=noise_level_3, negative_prompt=negs, generator=generator)


def load_if(model_name: str, device: str) -> IFCascade:
    tiny = model_name.lower().startswith("tiny")
    return cache().get(("if", model_name, device),
                       lambda: IFCascade(device, tiny=tiny, weights_dir=ensure_weights(model_name),
                                         stage2_dir=ensure_weights("DeepFloyd/IF-II-L-v1.0")))


def diffusion_if_callback(device_identifier, model_name, **kwargs):
    pipe = load_if(model_name, device_identifier)
    gen = kwargs.pop("generator", None)
    if gen is None:
        gen = torch.Generator(device=pipe.device).manual_seed(int(kwargs.pop("seed", 0) or 0))
    op = OutputProcessor(kwargs.pop("outputs", ["primary"]), kwargs.pop("content_type", "image/jpeg"))
    steps = kwargs.pop("num_inference_steps", None)
    if steps:
        kwargs.setdefault("stage1_steps", int(steps))
        kwargs.setdefault("stage2_steps", max(1, int(steps) // 2))
        kwargs.setdefault("stage3_steps", int(steps))
    images = pipe(prompt=kwargs.pop("prompt", ""), negative_prompt=kwargs.pop("negative_prompt", None),
                  num_images_per_prompt=int(kwargs.pop("num_images_per_prompt", 1)), generator=gen,
                  guidance_scale=float(kwargs.pop("guidance_scale", 7.0)),
                  **{k: v for k, v in kwargs.items() if k.startswith("stage") or k.startswith("noise_level")})
    op.add_outputs(images)
    return op.get_results(), {"_class_name": "IFPipeline", "_framework": "chiaswarm_amd",
                              "stages": ["IF-I", "IF-II", "x4-upscaler"], "weights": pipe.weights_source,
                              "ops": ops.get_mode()}
