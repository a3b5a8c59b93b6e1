"""NSFW safety checker (CompVis/stable-diffusion-safety-checker semantics: the
component every diffusers SD pipeline the reference loads runs after decode,
swarm/diffusion/diffusion_func.py:96-111 reads its ``nsfw_content_detected``).

CLIP ViT-L/14 vision tower (pre-LN, quick-GELU, 224² input) -> visual
projection 768 -> cosine similarity against 17 concept and 3 "special care"
embeddings with per-concept thresholds; a special-care hit lowers every concept
threshold by 0.01.  Flagged images are blacked out, as diffusers does.

MI355X path: the tower runs on the shared transformer kernels (fused-QKV MFMA
GEMM, flash attention, LayerNorm, quick-GELU epilogue), patch embedding is the
implicit-GEMM conv; preprocessing (resize/crop/normalise) happens on the uint8
images already on the device.  Without checkpoint weights the thresholds are
set so nothing is flagged (a random tower must not censor output).
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn
import torch.nn.functional as F

from .layers import Linear
from .transformer import ViT

MEAN = (0.48145466, 0.4578275, 0.40821073)
STD = (0.26862954, 0.26130258, 0.27577711)


@dataclasses.dataclass
class SafetyConfig:
    image_size: int = 224
    patch: int = 14
    dim: int = 1024
    depth: int = 24
    heads: int = 16
    mlp: int = 4096
    proj: int = 768
    act: str = "quick_gelu"  # transformers hidden_act (OpenCLIP ViT-H/14 image encoders: "gelu")


CLIP_L14 = SafetyConfig()
# OpenCLIP ViT-H/14 image tower (stabilityai/stable-diffusion-2-1-unclip image_encoder/)
CLIP_H14 = SafetyConfig(dim=1280, depth=32, heads=16, mlp=5120, proj=1024, act="gelu")
TINY_SAFETY = SafetyConfig(image_size=28, patch=14, dim=64, depth=2, heads=2, mlp=128, proj=32)


class SafetyChecker(nn.Module):
    def __init__(self, cfg: SafetyConfig = CLIP_L14):
        super().__init__()
        self.cfg = cfg
        self.vision_model = ViT(cfg.image_size, cfg.patch, cfg.dim, cfg.depth, cfg.heads, cfg.mlp, eps=1e-5,
                                act="quick_gelu", pre_norm=True, patch_bias=False)
        self.visual_projection = Linear(cfg.dim, cfg.proj, bias=False)
        self.concept_embeds = nn.Parameter(torch.zeros(17, cfg.proj))
        self.special_care_embeds = nn.Parameter(torch.zeros(3, cfg.proj))
        # random-init default: thresholds above any cosine similarity -> never flags
        self.concept_embeds_weights = nn.Parameter(torch.full((17,), 2.0))
        self.special_care_embeds_weights = nn.Parameter(torch.full((3,), 2.0))

    def preprocess(self, images_u8: torch.Tensor) -> torch.Tensor:
        """uint8 NHWC [B, H, W, 3] -> normalised NHWC [B, S, S, 3] (shortest-side
        resize + centre crop, CLIP mean/std)."""
        s = self.cfg.image_size
        x = images_u8.permute(0, 3, 1, 2).float() / 255.0
        h, w = x.shape[-2:]
        r = s / min(h, w)
        nh, nw = max(s, round(h * r)), max(s, round(w * r))
        x = F.interpolate(x, size=(nh, nw), mode="bicubic", align_corners=False, antialias=True)
        t, l = (nh - s) // 2, (nw - s) // 2
        x = x[:, :, t:t + s, l:l + s]
        mean = torch.tensor(MEAN, device=x.device)[None, :, None, None]
        std = torch.tensor(STD, device=x.device)[None, :, None, None]
        return ((x - mean) / std).permute(0, 2, 3, 1).contiguous()

    def image_embeds(self, x: torch.Tensor) -> torch.Tensor:
        """Normalised NHWC pixels -> projected CLS embedding (CLIPVisionModelWithProjection.image_embeds)."""
        return self.visual_projection(self.vision_model(x)[:, 0])

    def flags(self, emb: torch.Tensor) -> torch.Tensor:
        """Per-image NSFW decision from projected embeddings [B, proj]; scores are
        rounded to 3 decimals before the > 0 test, as diffusers does."""
        emb = F.normalize(emb.float(), dim=-1)
        special = emb @ F.normalize(self.special_care_embeds.float(), dim=-1).t()
        concept = emb @ F.normalize(self.concept_embeds.float(), dim=-1).t()
        special_scores = torch.round((special - self.special_care_embeds_weights.float()) * 1000) / 1000
        adj = (special_scores > 0).any(dim=1, keepdim=True).float() * 0.01
        concept_scores = torch.round((concept - self.concept_embeds_weights.float() + adj) * 1000) / 1000
        return (concept_scores > 0).any(dim=1)

    @torch.no_grad()
    def forward(self, images_u8: torch.Tensor):
        """Returns (nsfw flags list[bool], images with flagged ones blacked out)."""
        dt = self.visual_projection.weight.dtype
        x = self.preprocess(images_u8.to(self.visual_projection.weight.device)).to(dt)
        flags = self.flags(self.image_embeds(x))
        out = images_u8.clone()
        if bool(flags.any()):
            out[flags.to(out.device)] = 0
        return [bool(f) for f in flags.cpu()], out


_HF_RENAMES = {"vision_model.embeddings.patch_embedding.": "vision_model.patch_embedding.",
               "vision_model.embeddings.class_embedding": "vision_model.class_embedding",
               "vision_model.embeddings.position_embedding.weight": "vision_model.position_embedding",
               "vision_model.pre_layrnorm.": "vision_model.pre_ln.",
               "vision_model.post_layernorm.": "vision_model.post_ln.",
               "vision_model.encoder.layers.": "vision_model.layers.",
               ".self_attn.q_proj.": ".attn.q.", ".self_attn.k_proj.": ".attn.k.",
               ".self_attn.v_proj.": ".attn.v.", ".self_attn.out_proj.": ".attn.o.",
               ".layer_norm1.": ".ln1.", ".layer_norm2.": ".ln2.", ".mlp.fc1.": ".fc1.", ".mlp.fc2.": ".fc2."}


def config_from_dir(weights_dir) -> SafetyConfig | None:
    """The checker's geometry from its ``config.json`` (a transformers
    ``CLIPConfig``: ``vision_config`` + ``projection_dim``; fields it omits take
    the ViT-L/14 defaults), or None without one."""
    import json
    import os

    path = os.path.join(weights_dir, "config.json") if weights_dir else None
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        raw = json.load(f)
    v = raw.get("vision_config") or raw.get("vision_config_dict") or {}
    d = CLIP_L14
    return SafetyConfig(image_size=int(v.get("image_size", d.image_size)), patch=int(v.get("patch_size", d.patch)),
                        dim=int(v.get("hidden_size", d.dim)), depth=int(v.get("num_hidden_layers", d.depth)),
                        heads=int(v.get("num_attention_heads", d.heads)),
                        mlp=int(v.get("intermediate_size", d.mlp)),
                        proj=int(raw.get("projection_dim", v.get("projection_dim", d.proj))))


def load_safety_checker(device, weights_dir=None, tiny=False) -> SafetyChecker:
    from .layers import init_random_fast_, prepare_model

    dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
    cfg = TINY_SAFETY if tiny else (config_from_dir(weights_dir) or CLIP_L14)
    with torch.device(device):
        m = SafetyChecker(cfg).to(dt).eval().requires_grad_(False)
    keep = {k: v.clone() for k, v in m.state_dict().items() if "embeds" in k}
    init_random_fast_(m, seed=99)
    m.load_state_dict({**m.state_dict(), **keep})  # random tower, never-flag thresholds
    if weights_dir:
        from .weights import _read_dir, load_into

        # StableDiffusionSafetyChecker nests CLIPVisionModel: vision_model.vision_model.*
        load_into(m, _read_dir(weights_dir), _HF_RENAMES, prefix_strip="vision_model.")
    return prepare_model(m)
