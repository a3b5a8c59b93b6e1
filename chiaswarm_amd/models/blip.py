"""BLIP image captioning (ViT image encoder + BERT decoder with cross-attention,
greedy autoregressive decode).  Reference: the transformers
``BlipProcessor`` / ``BlipForConditionalGeneration`` pair chosen by the hive at
swarm/captioning/caption_image.py:11-29 (conditional captioning when a prompt
is given, unconditional otherwise).

Decode is a causal re-run of the (short, <= 40 token) prefix each step through
the flash-attention kernel with causal masking; the image K/V of every
cross-attention layer are computed once.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch
import torch.nn as nn
from PIL import Image

from .layers import LayerNorm, Linear
from .transformer import PostLNBlock, ViT


@dataclasses.dataclass
class BlipConfig:
    image_size: int = 384
    vision_dim: int = 768
    vision_depth: int = 12
    vision_heads: int = 12
    text_dim: int = 768
    text_depth: int = 12
    text_heads: int = 12
    vocab: int = 30524
    max_pos: int = 512
    bos_id: int = 30522  # [DEC]
    sep_id: int = 102
    pad_id: int = 0


BLIP_BASE = BlipConfig()
BLIP_LARGE = BlipConfig(vision_dim=1024, vision_depth=24, vision_heads=16)
TINY_BLIP = BlipConfig(image_size=64, vision_dim=64, vision_depth=2, vision_heads=2, text_dim=64, text_depth=2,
                       text_heads=2, vocab=1000, bos_id=998, sep_id=999)

MEAN = np.array([0.48145466, 0.4578275, 0.40821073], np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], np.float32)


class BlipCaptioner(nn.Module):
    def __init__(self, cfg: BlipConfig = BLIP_BASE):
        super().__init__()
        self.cfg = cfg
        self.vision_model = ViT(cfg.image_size, 16, cfg.vision_dim, cfg.vision_depth, cfg.vision_heads,
                                4 * cfg.vision_dim)
        self.word_embeddings = nn.Embedding(cfg.vocab, cfg.text_dim)
        self.position_embeddings = nn.Embedding(cfg.max_pos, cfg.text_dim)
        self.emb_ln = LayerNorm(cfg.text_dim, eps=1e-12)
        self.layers = nn.ModuleList([PostLNBlock(cfg.text_dim, cfg.text_heads, 4 * cfg.text_dim,
                                                 cross_dim=cfg.vision_dim) for _ in range(cfg.text_depth)])
        self.head_transform = Linear(cfg.text_dim, cfg.text_dim)
        self.head_ln = LayerNorm(cfg.text_dim, eps=1e-12)
        self.head_bias = nn.Parameter(torch.zeros(cfg.vocab))

    def preprocess(self, image: Image.Image) -> torch.Tensor:
        s = self.cfg.image_size
        a = np.asarray(image.convert("RGB").resize((s, s), Image.Resampling.BICUBIC), np.float32) / 255.0
        a = (a - MEAN) / STD
        return torch.from_numpy(a)[None]

    @torch.no_grad()
    def generate(self, image: Image.Image, prefix_ids: list[int], max_new_tokens=30) -> list[int]:
        dev = self.head_bias.device
        dt = self.word_embeddings.weight.dtype
        img = self.preprocess(image).to(dev)
        vis = self.vision_model(img.to(dt))
        kvs = [blk.cross.kv_of(vis) for blk in self.layers]
        ids = [self.cfg.bos_id] + list(prefix_ids)
        out = []
        for _ in range(max_new_tokens):
            t = torch.tensor([ids], device=dev)
            x = self.word_embeddings(t) + self.position_embeddings.weight[: t.shape[1]][None]
            x = self.emb_ln(x)
            for blk, kv in zip(self.layers, kvs):
                x = blk.ln1(blk.attn(x, residual=x, causal=True))
                x = blk.ln_x(blk.cross(x, kv=kv, residual=x))
                x = blk.ln2(blk.fc2(blk.fc1(x, act="gelu"), residual=x))
            h = self.head_ln(self.head_transform(x[:, -1:], act="gelu"))
            logits = h.float() @ self.word_embeddings.weight.float().t() + self.head_bias.float()
            nxt = int(logits[0, -1].argmax())
            if nxt == self.cfg.sep_id:
                break
            ids.append(nxt)
            out.append(nxt)
        return list(prefix_ids) + out
