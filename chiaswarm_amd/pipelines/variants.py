"""The reflection-reachable SD pipeline classes beyond txt2img / img2img /
inpaint (reference: the hive names any diffusers class in
``parameters.pipeline_type`` and the worker builds it by reflection,
swarm/job_arguments.py:143-145, swarm/type_helpers.py:1-3,
swarm/diffusion/diffusion_func.py:41-46):

* ``StableDiffusionDepth2ImgPipeline`` (stabilityai/stable-diffusion-2-depth):
  a 5-channel UNet whose extra input is the depth of the start image at latent
  size, normalised to [-1, 1] per image (diffusers ``prepare_depth_map``);
  img2img otherwise (strength, noised init latents).  The depth comes from the
  job's ``depth_map`` or from a DPT depth estimator: the checkpoint's own
  ``depth_estimator/`` when it is a plain ViT DPT, else the shared ControlNet
  depth annotator (Intel/dpt-large, controlnet/annotators.py) — the published
  checkpoint ships DPT-hybrid (BiT backbone), which is not built here, so the
  depth network differs from diffusers' there (parity unpinned, documented).
* ``StableDiffusionImageVariationPipeline`` (lambdalabs/sd-image-variations-
  diffusers): no text encoder; the CLIP ViT-L/14 image embedding of the start
  image (``CLIPVisionModelWithProjection.image_embeds``, CLIP preprocessing)
  is the single context token, its zeros the unconditional one.  The vision
  tower is the safety checker's (models/safety.py) — pinned against
  transformers in tests/test_variants.py.

* ``StableUnCLIPImg2ImgPipeline`` (stabilityai/stable-diffusion-2-1-unclip):
  the SD2.1-v UNet with a "projection" class embedding fed the noised CLIP
  ViT-H/14 image embedding of the start image plus its noise level; the
  prompt still conditions through cross-attention.

All run on the resident StableDiffusion bundle (UNet hipGraph step, fused
sampler loop, VAE decode kernels).
"""
from __future__ import annotations

import json
import logging
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from PIL import Image

from ..models.layers import Linear
from ..models.safety import CLIP_L14, MEAN, STD, SafetyConfig, _HF_RENAMES
from ..models.transformer import ViT
from .sd import StableDiffusion


# ---------------------------------------------------------------------------
# Depth2Img
# ---------------------------------------------------------------------------
_DEPTH_CACHE: dict = {}


def _dpt_from_dir(d: str, device, dtype):
    """A DPTForDepthEstimation checkpoint directory -> (model, input size) or
    None when it is a hybrid (BiT-backbone) DPT."""
    from ..controlnet.annotators import DPTDepth
    from ..models.weights import _read_dir, load_into

    with open(os.path.join(d, "config.json")) as f:
        cfg = json.load(f)
    if cfg.get("is_hybrid"):
        return None
    size = int(cfg.get("image_size", 384))
    m = DPTDepth(c=int(cfg.get("hidden_size", 1024)), heads=int(cfg.get("num_attention_heads", 16)),
                 mlp=int(cfg.get("intermediate_size", 4096)), n=int(cfg.get("num_hidden_layers", 24)),
                 patch=int(cfg.get("patch_size", 16)), image=size,
                 out_indices=tuple(cfg.get("backbone_out_indices", (5, 11, 17, 23))),
                 neck_sizes=tuple(cfg.get("neck_hidden_sizes", (256, 512, 1024, 1024))),
                 factors=tuple(cfg.get("reassemble_factors", (4, 2, 1, 0.5))),
                 fusion=int(cfg.get("fusion_hidden_size", 256)))
    load_into(m, _read_dir(d), allow_unexpected=True, name="depth_estimator")
    return m.to(device, dtype).eval().requires_grad_(False), size


def depth_estimator(pipe: StableDiffusion):
    """(model, input size) of the pipe's depth network (cached per pipe)."""
    key = id(pipe)
    hit = _DEPTH_CACHE.get(key)
    if hit is not None:
        return hit
    dt = torch.bfloat16 if pipe.device.type == "cuda" else torch.float32
    wd = getattr(pipe, "weights_dir", None)
    got = None
    if wd and os.path.exists(os.path.join(wd, "depth_estimator", "config.json")):
        got = _dpt_from_dir(os.path.join(wd, "depth_estimator"), pipe.device, dt)
        if got is None:
            logging.warning("depth_estimator: DPT-hybrid (BiT) is not built here; using the DPT-large "
                            "depth annotator for Depth2Img")
    if got is None:
        from ..controlnet.annotators import DPTDepth, _build

        m = _build("depth", DPTDepth)
        got = (m, 384)
    _DEPTH_CACHE[key] = got
    return got


@torch.no_grad()
def depth_latents(pipe: StableDiffusion, images: list, lh: int, lw: int, depth_map=None) -> torch.Tensor:
    """[B, lh, lw, 1] depth in [-1, 1] (diffusers StableDiffusionDepth2ImgPipeline
    .prepare_depth_map): DPT prediction (or the given ``depth_map`` [B, H, W] /
    [H, W]) -> bicubic resize to the latent grid -> per-image min-max to [-1, 1]."""
    if depth_map is not None:
        d = torch.as_tensor(np.asarray(depth_map) if not torch.is_tensor(depth_map) else depth_map).float()
        if d.dim() == 2:
            d = d[None]
        d = d.to(pipe.device)
        if d.shape[0] != len(images):
            d = d[:1].expand(len(images), *d.shape[1:])
    else:
        m, size = depth_estimator(pipe)
        p = next(m.parameters())
        arr = np.stack([np.asarray(im.convert("RGB").resize((size, size), Image.Resampling.BICUBIC))
                        for im in images]).astype(np.float32)
        x = torch.from_numpy((arr / 255.0 - 0.5) / 0.5).to(p.device).permute(0, 3, 1, 2).to(p.dtype)
        d = m(x).float()
    d = F.interpolate(d[:, None], size=(lh, lw), mode="bicubic", align_corners=False)
    lo = d.amin(dim=(1, 2, 3), keepdim=True)
    hi = d.amax(dim=(1, 2, 3), keepdim=True)
    d = 2.0 * (d - lo) / (hi - lo).clamp_min(1e-12) - 1.0
    return d.permute(0, 2, 3, 1).contiguous()


# ---------------------------------------------------------------------------
# ImageVariation
# ---------------------------------------------------------------------------
class CLIPImageEncoder(nn.Module):
    """transformers ``CLIPVisionModelWithProjection``: the CLIP vision tower
    (pre-LN, quick-GELU) + ``visual_projection`` of the post-LN CLS token."""

    def __init__(self, cfg: SafetyConfig = CLIP_L14):
        super().__init__()
        self.cfg = cfg
        self.vision_model = ViT(cfg.image_size, cfg.patch, cfg.dim, cfg.depth, cfg.heads, cfg.mlp, eps=1e-5,
                                act=cfg.act, pre_norm=True, patch_bias=False)
        self.visual_projection = Linear(cfg.dim, cfg.proj, bias=False)

    def preprocess(self, images: list) -> torch.Tensor:
        """PIL images -> CLIPImageProcessor pixels, NHWC (shortest side -> 224
        bicubic, centre crop, /255, CLIP mean/std)."""
        s = self.cfg.image_size
        out = []
        for im in images:
            im = im.convert("RGB")
            w, h = im.size
            r = s / min(w, h)
            nw, nh = max(s, round(w * r)), max(s, round(h * r))
            im = im.resize((nw, nh), Image.Resampling.BICUBIC)
            t, l = (nh - s) // 2, (nw - s) // 2
            out.append(np.asarray(im.crop((l, t, l + s, t + s)), dtype=np.float32) / 255.0)
        x = (np.stack(out) - np.array(MEAN, np.float32)) / np.array(STD, np.float32)
        p = self.visual_projection.weight
        return torch.from_numpy(x).to(p.device, p.dtype)

    def forward(self, pixels_nhwc: torch.Tensor) -> torch.Tensor:
        return self.visual_projection(self.vision_model(pixels_nhwc)[:, 0])


def image_encoder_config(d: str) -> SafetyConfig:
    with open(os.path.join(d, "config.json")) as f:
        raw = json.load(f)
    v = raw.get("vision_config") or raw
    base = CLIP_L14
    return SafetyConfig(image_size=int(v.get("image_size", base.image_size)), patch=int(v.get("patch_size", base.patch)),
                        dim=int(v.get("hidden_size", base.dim)), depth=int(v.get("num_hidden_layers", base.depth)),
                        heads=int(v.get("num_attention_heads", base.heads)),
                        mlp=int(v.get("intermediate_size", base.mlp)),
                        proj=int(raw.get("projection_dim", v.get("projection_dim", base.proj))),
                        act=str(v.get("hidden_act", base.act)))


def load_image_encoder(device, weights_dir: str | None, cfg: SafetyConfig | None = None, seed: int = 0):
    from ..models.layers import init_random_fast_, prepare_model
    from ..models.weights import _read_dir, load_into

    d = os.path.join(weights_dir, "image_encoder") if weights_dir else None
    if cfg is None:
        cfg = image_encoder_config(d) if d and os.path.exists(os.path.join(d, "config.json")) else CLIP_L14
    dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
    with torch.device(device):
        m = CLIPImageEncoder(cfg).to(dt).eval().requires_grad_(False)
    init_random_fast_(m, seed=seed)
    src = "random-init"
    if d and os.path.isdir(d):
        load_into(m, _read_dir(d, m.visual_projection.weight.device), _HF_RENAMES, name="image_encoder")
        src = d
    m.weights_source = src
    return prepare_model(m)


class ImageVariation(StableDiffusion):
    """``StableDiffusionImageVariationPipeline``: the context is the start
    image's CLIP image embedding [B, 1, 768] (zeros for the unconditional CFG
    half); no prompt."""

    def __init__(self, family, device="cpu", dtype=None, seed=0, weights_dir=None, image_encoder_cfg=None):
        super().__init__(family, device=device, dtype=dtype, seed=seed, weights_dir=weights_dir)
        d = os.path.join(weights_dir, "image_encoder") if weights_dir else None
        if image_encoder_cfg is None and not (d and os.path.exists(os.path.join(d, "config.json"))):
            xd = self.family.unet.cross_attention_dim
            # no checkpoint: ViT-L/14 for the real geometry, a tiny tower for test-size UNets
            image_encoder_cfg = CLIP_L14 if xd == CLIP_L14.proj else SafetyConfig(
                image_size=28, patch=14, dim=64, depth=2, heads=2, mlp=128, proj=int(xd))
        self.image_encoder = load_image_encoder(self.device, weights_dir, image_encoder_cfg, seed=seed + 17)
        self._img_ctx = None
        self.config["image_encoder"] = ["chiaswarm_amd", "CLIPVisionModelWithProjection"]
        self.config.pop("text_encoder", None)
        self.config.pop("tokenizer", None)

    @torch.no_grad()
    def image_embeds(self, images: list) -> torch.Tensor:
        return self.image_encoder(self.image_encoder.preprocess(images))

    def encode(self, prompts, negatives, cfg, with_kv=True):  # the image embedding replaces the text context
        emb = self._img_ctx
        if emb is None:
            raise ValueError("StableDiffusionImageVariationPipeline needs an input image")
        ctx = emb[:, None, :].to(self.dtype)
        if cfg:
            ctx = torch.cat([torch.zeros_like(ctx), ctx], 0)
        kv = tuple(self.unet.encode_context(ctx)) if with_kv else ()
        return ctx, None, kv

    @torch.no_grad()
    def __call__(self, image=None, height=None, width=None, num_inference_steps=50, guidance_scale=7.5,
                 num_images_per_prompt=1, generator=None, eta=0.0, latents=None, output_type="pil", scheduler=None,
                 prompt=None, negative_prompt=None, **unexpected):
        # (prompt / negative_prompt: the router's defaults; the diffusers class has no text input)
        if unexpected:
            raise TypeError(f"StableDiffusionImageVariationPipeline.__call__() got unexpected keyword arguments "
                            f"{sorted(unexpected)}")
        if image is None:
            raise ValueError("StableDiffusionImageVariationPipeline needs an input image (start_image_uri)")
        images = image if isinstance(image, list) else [image]
        emb = self.image_embeds(images)
        self._img_ctx = emb.repeat_interleave(num_images_per_prompt, 0)
        try:
            return super().__call__(prompt=[""] * len(images), negative_prompt=None,
                                    num_inference_steps=num_inference_steps, guidance_scale=guidance_scale,
                                    num_images_per_prompt=num_images_per_prompt,
                                    height=height or self.family.default_size, width=width or self.family.default_size,
                                    generator=generator, eta=eta, latents=latents, output_type=output_type,
                                    scheduler=scheduler)
        finally:
            self._img_ctx = None


# ---------------------------------------------------------------------------
# StableUnCLIPImg2Img
# ---------------------------------------------------------------------------
def _unclip_extras(weights_dir: str | None, dim: int, device):
    """(mean, std) of the checkpoint's ``image_normalizer`` ([1, dim] fp32;
    0 / 1 without one) and the ``image_noising_scheduler``'s alpha-bar table
    (its scheduler_config.json; diffusers' squaredcos_cap_v2 DDPM default)."""
    from ..schedulers import _betas

    mean = torch.zeros(1, dim, dtype=torch.float32, device=device)
    std = torch.ones(1, dim, dtype=torch.float32, device=device)
    cfg = {"num_train_timesteps": 1000, "beta_schedule": "squaredcos_cap_v2", "beta_start": 0.00085,
           "beta_end": 0.012}
    if weights_dir:
        nd = os.path.join(weights_dir, "image_normalizer")
        if os.path.isdir(nd):
            from ..models.weights import _read_dir

            sd = _read_dir(nd)
            mean = sd["mean"].reshape(1, -1).float().to(device)
            std = sd["std"].reshape(1, -1).float().to(device)
        sp = os.path.join(weights_dir, "image_noising_scheduler", "scheduler_config.json")
        if os.path.exists(sp):
            with open(sp) as f:
                cfg.update({k: v for k, v in json.load(f).items() if k in cfg})
    betas = _betas(int(cfg["num_train_timesteps"]), float(cfg["beta_start"]), float(cfg["beta_end"]),
                   str(cfg["beta_schedule"]))
    return mean, std, np.cumprod(1.0 - np.asarray(betas, dtype=np.float64))


class UnCLIPImg2Img(StableDiffusion):
    """``StableUnCLIPImg2ImgPipeline`` (stabilityai/stable-diffusion-2-1-unclip):
    the start image's CLIP ViT-H/14 image embedding, normalised, noised to
    ``noise_level`` by the checkpoint's image-noising schedule, un-normalised
    and concatenated with the level's sinusoidal embedding, is the UNet's
    ``projection`` class embedding (zeros for the unconditional CFG half); the
    prompt conditions through cross-attention as usual and the latents start
    from pure noise.  The class labels ride in the UNet's added conditioning,
    so the step stays one hipGraph replay (the device-resident loop)."""

    def __init__(self, family, device="cpu", dtype=None, seed=0, weights_dir=None, image_encoder_cfg=None):
        from ..models.safety import CLIP_H14

        super().__init__(family, device=device, dtype=dtype, seed=seed, weights_dir=weights_dir)
        d = os.path.join(weights_dir, "image_encoder") if weights_dir else None
        if image_encoder_cfg is None and not (d and os.path.exists(os.path.join(d, "config.json"))):
            pd = self.family.unet.projection_class_embeddings_input_dim // 2
            image_encoder_cfg = CLIP_H14 if pd == CLIP_H14.proj else SafetyConfig(
                image_size=28, patch=14, dim=64, depth=2, heads=2, mlp=128, proj=int(pd), act="gelu")
        self.image_encoder = load_image_encoder(self.device, weights_dir, image_encoder_cfg, seed=seed + 19)
        dim = self.image_encoder.cfg.proj
        if 2 * dim != self.family.unet.projection_class_embeddings_input_dim:
            raise ValueError(f"unCLIP: image embedding {dim} x 2 != the UNet's class input "
                             f"{self.family.unet.projection_class_embeddings_input_dim}")
        self.norm_mean, self.norm_std, self.noise_abar = _unclip_extras(weights_dir, dim, self.device)
        self._class = None
        self.config["image_encoder"] = ["chiaswarm_amd", "CLIPVisionModelWithProjection"]
        self.config["image_normalizer"] = ["chiaswarm_amd", "StableUnCLIPImageNormalizer"]
        self.config["image_noising_scheduler"] = ["chiaswarm_amd", "DDPMScheduler"]

    @torch.no_grad()
    def image_embeds(self, images: list) -> torch.Tensor:
        return self.image_encoder(self.image_encoder.preprocess(images))

    def noise_image_embeds(self, emb: torch.Tensor, noise_level: int, generator=None) -> torch.Tensor:
        """diffusers ``noise_image_embeddings``: [B, 2 D] = [unscale(add_noise(scale(emb))) | sinusoid(level)]."""
        from ..models.layers import timestep_embedding
        from ..schedulers import batch_randn

        lvl = int(noise_level)
        if not 0 <= lvl < len(self.noise_abar):
            raise ValueError(f"noise_level must be in [0, {len(self.noise_abar) - 1}], got {noise_level}")
        b, dim = emb.shape
        noise = batch_randn((b, dim), generator, emb.device)
        x = (emb.float() - self.norm_mean) / self.norm_std
        a = float(self.noise_abar[lvl])
        x = math.sqrt(a) * x + math.sqrt(1.0 - a) * noise
        x = x * self.norm_std + self.norm_mean
        t = torch.full((b,), float(lvl), dtype=torch.float32, device=emb.device)
        return torch.cat([x, timestep_embedding(t, dim).float()], 1)

    def encode(self, prompts, negatives, cfg, with_kv=True):
        ctx, _, kv = super().encode(prompts, negatives, cfg, with_kv)
        cl = self._class
        if cl is None:
            raise ValueError("StableUnCLIPImg2ImgPipeline needs an input image (or image_embeds)")
        cl = cl.to(self.dtype)
        if cfg:
            cl = torch.cat([torch.zeros_like(cl), cl], 0)
        return ctx, {"class_labels": cl}, kv

    @torch.no_grad()
    def __call__(self, image=None, prompt="", height=None, width=None, num_inference_steps=20, guidance_scale=10.0,
                 negative_prompt=None, num_images_per_prompt=1, eta=0.0, generator=None, latents=None,
                 output_type="pil", scheduler=None, noise_level=0, image_embeds=None, **unexpected):
        if unexpected:
            raise TypeError(f"StableUnCLIPImg2ImgPipeline.__call__() got unexpected keyword arguments "
                            f"{sorted(unexpected)}")
        prompts = prompt if isinstance(prompt, list) else [prompt]
        b = len(prompts) * num_images_per_prompt
        if image_embeds is None:
            if image is None:
                raise ValueError("StableUnCLIPImg2ImgPipeline needs an input image (start_image_uri)")
            images = image if isinstance(image, list) else [image]
            emb = self.image_embeds(images)
        else:
            emb = torch.as_tensor(image_embeds).to(self.device)
            emb = emb.reshape(-1, emb.shape[-1])
        if emb.shape[0] == 1:
            emb = emb.expand(b, -1)
        elif emb.shape[0] == len(prompts):
            emb = emb.repeat_interleave(num_images_per_prompt, 0)
        elif emb.shape[0] != b:
            raise ValueError(f"{emb.shape[0]} image embeddings for {b} images")
        self._class = self.noise_image_embeds(emb, noise_level, generator)
        try:
            return super().__call__(prompt=prompts, negative_prompt=negative_prompt,
                                    num_inference_steps=num_inference_steps, guidance_scale=guidance_scale,
                                    num_images_per_prompt=num_images_per_prompt,
                                    height=height or self.family.default_size, width=width or self.family.default_size,
                                    generator=generator, eta=eta, latents=latents, output_type=output_type,
                                    scheduler=scheduler)
        finally:
            self._class = None
