"""Generic transformer blocks on the shared kernels (fused-QKV GEMM, flash
attention, LayerNorm, GEMM epilogues with bias/act/residual) for the non-SD
model families: ViT / BERT (BLIP captioning), GPT (Bark), T5 (DeepFloyd IF),
RoBERTa (CLAP for AudioLDM) and the CLIP vision tower (safety checker).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops
from .layers import LayerNorm, Linear, Prepared


class MHA(Prepared):
    """Multi-head attention with separate q/k/v/o Linear modules (packed QKV at
    prepare time).  ``kv_dim`` != None -> cross-attention."""

    def __init__(self, dim, heads, kv_dim=None, bias=True, out_bias=True, head_dim=None, scale=None):
        super().__init__()
        self.heads = heads
        self.dh = head_dim or dim // heads
        inner = self.heads * self.dh
        self.cross = kv_dim is not None
        self.q = Linear(dim, inner, bias=bias)
        self.k = Linear(kv_dim or dim, inner, bias=bias)
        self.v = Linear(kv_dim or dim, inner, bias=bias)
        self.o = Linear(inner, dim, bias=out_bias)
        self.scale = scale if scale is not None else 1.0 / math.sqrt(self.dh)

    def prepare(self):
        ws = [self.k.weight, self.v.weight] if self.cross else [self.q.weight, self.k.weight, self.v.weight]
        self.w_in = torch.cat(ws, 0).detach()
        if self.q.bias is not None:
            bs = [self.k.bias, self.v.bias] if self.cross else [self.q.bias, self.k.bias, self.v.bias]
            self.b_in = torch.cat(bs, 0).detach()
        else:
            self.b_in = None

    def _ensure(self):
        w = getattr(self, "w_in", None)
        if w is None or w.device != self.q.weight.device or w.dtype != self.q.weight.dtype:
            self.prepare()

    def kv_of(self, ctx):
        self._ensure()
        b, s, _ = ctx.shape
        return ops.gemm(ctx, self.w_in, self.b_in).view(b, s, 2, self.heads, self.dh)

    def forward(self, x, ctx=None, kv=None, residual=None, causal=False):
        self._ensure()
        b, s, _ = x.shape
        if self.cross:
            q = self.q(x).view(b, s, self.heads, self.dh)
            kv = kv if kv is not None else self.kv_of(ctx)
            k, v = kv[:, :, 0], kv[:, :, 1]
        else:
            qkv = ops.gemm(x, self.w_in, self.b_in).view(b, s, 3, self.heads, self.dh)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        o = ops.attention(q, k, v, self.scale, causal=causal)
        return self.o(o.reshape(b, s, self.heads * self.dh), residual=residual)


class PreLNBlock(nn.Module):
    """x += attn(LN(x)); [x += cross(LN(x), ctx)]; x += mlp(LN(x))   (ViT/GPT/CLIP style)."""

    def __init__(self, dim, heads, mlp_dim, act="gelu", cross_dim=None, bias=True, eps=1e-5):
        super().__init__()
        self.ln1 = LayerNorm(dim, eps=eps)
        self.attn = MHA(dim, heads, bias=bias)
        self.cross = None
        if cross_dim is not None:
            self.ln_x = LayerNorm(dim, eps=eps)
            self.cross = MHA(dim, heads, kv_dim=cross_dim, bias=bias)
        self.ln2 = LayerNorm(dim, eps=eps)
        self.fc1 = Linear(dim, mlp_dim, bias=bias)
        self.fc2 = Linear(mlp_dim, dim, bias=bias)
        self.act = act

    def forward(self, x, ctx=None, causal=False):
        x = self.attn(self.ln1(x), residual=x, causal=causal)
        if self.cross is not None:
            x = self.cross(self.ln_x(x), ctx=ctx, residual=x)
        return self.fc2(self.fc1(self.ln2(x), act=self.act), residual=x)


class PostLNBlock(nn.Module):
    """BERT style: x = LN(x + attn(x)); [x = LN(x + cross(x))]; x = LN(x + mlp(x))."""

    def __init__(self, dim, heads, mlp_dim, cross_dim=None, eps=1e-12):
        super().__init__()
        self.attn = MHA(dim, heads)
        self.ln1 = LayerNorm(dim, eps=eps)
        self.cross = MHA(dim, heads, kv_dim=cross_dim) if cross_dim else None
        self.ln_x = LayerNorm(dim, eps=eps) if cross_dim else None
        self.fc1 = Linear(dim, mlp_dim)
        self.fc2 = Linear(mlp_dim, dim)
        self.ln2 = LayerNorm(dim, eps=eps)

    def forward(self, x, ctx=None, causal=False):
        x = self.ln1(self.attn(x, residual=x, causal=causal))
        if self.cross is not None:
            x = self.ln_x(self.cross(x, ctx=ctx, residual=x))
        return self.ln2(self.fc2(self.fc1(x, act="gelu"), residual=x))


class ViT(nn.Module):
    """Patch-embedding vision transformer (pre-LN), NHWC image input."""

    def __init__(self, image_size=384, patch=16, dim=768, depth=12, heads=12, mlp=3072, eps=1e-5,
                 act="gelu", pre_norm=False, patch_bias=True):
        super().__init__()
        self.patch, self.image_size = patch, image_size
        from .layers import Conv2d

        # CLIP's patch embedding has no bias, BLIP's has one
        self.patch_embedding = Conv2d(3, dim, patch, stride=patch, padding=0, bias=patch_bias)
        self.class_embedding = nn.Parameter(torch.zeros(dim))
        self.position_embedding = nn.Parameter(torch.zeros(1 + (image_size // patch) ** 2, dim))
        self.pre_ln = LayerNorm(dim, eps=eps) if pre_norm else None
        self.layers = nn.ModuleList([PreLNBlock(dim, heads, mlp, act=act, eps=eps) for _ in range(depth)])
        self.post_ln = LayerNorm(dim, eps=eps)

    def forward(self, img):
        """img: NHWC [B, H, W, 3] normalised -> tokens [B, 1 + P, dim]."""
        p = self.patch_embedding(img.to(self.class_embedding.dtype))  # [B, h, w, dim]
        b = p.shape[0]
        p = p.reshape(b, -1, p.shape[-1])
        cls = self.class_embedding.expand(b, 1, -1)
        x = torch.cat([cls, p], 1) + self.position_embedding[None, : p.shape[1] + 1]
        if self.pre_ln is not None:
            x = self.pre_ln(x)
        for layer in self.layers:
            x = layer(x)
        return self.post_ln(x)
