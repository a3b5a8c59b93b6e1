"""T5 v1.1 encoder (DeepFloyd IF text encoder, T5-XXL: 24 layers, d_model
4096, 64 heads, gated-GELU FFN 10240) with the transformers parameter names
(``shared``, ``encoder.block.{i}.layer.{0,1}...``), so an IF
``text_encoder/*.safetensors`` loads without renames.  Reached by the
reference via ``stage_1.encode_prompt`` (swarm/diffusion/diffusion_func_if.py:43-45).

MI355X path: Q/K/V/O and the gated FFN are MFMA GEMMs (tanh-GELU of wi_0
fused into its epilogue, the residual adds fused into wo / o).  The attention
core (77 tokens, per-head relative-position bias, key-padding mask) is a few
batched torch matmuls: at 77 tokens it is launch-bound either way, and it runs
once per request.
"""
from __future__ import annotations

import dataclasses
import hashlib
import math
import os

import torch
import torch.nn as nn

from .layers import Linear


@dataclasses.dataclass
class T5Config:
    vocab: int = 32128
    d_model: int = 4096
    d_kv: int = 64
    heads: int = 64
    d_ff: int = 10240
    layers: int = 24
    buckets: int = 32
    max_distance: int = 128
    eps: float = 1e-6


T5_XXL = T5Config()
TINY_T5 = T5Config(vocab=1000, d_model=64, d_kv=16, heads=4, d_ff=128, layers=2)


class T5RMSNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return (y * self.weight.float()).to(x.dtype)


def relative_position_bucket(rel: torch.Tensor, num_buckets=32, max_distance=128) -> torch.Tensor:
    """Bidirectional T5 bucketing of (key - query) offsets."""
    num_buckets //= 2
    out = (rel > 0).long() * num_buckets
    n = rel.abs()
    max_exact = num_buckets // 2
    large = max_exact + (torch.log(n.float().clamp_min(1) / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).long()
    large = large.clamp_max(num_buckets - 1)
    return out + torch.where(n < max_exact, n, large)


class _SelfAttention(nn.Module):
    def __init__(self, c: T5Config, has_bias: bool):
        super().__init__()
        inner = c.heads * c.d_kv
        self.c = c
        self.q = Linear(c.d_model, inner, bias=False)
        self.k = Linear(c.d_model, inner, bias=False)
        self.v = Linear(c.d_model, inner, bias=False)
        self.o = Linear(inner, c.d_model, bias=False)
        if has_bias:
            self.relative_attention_bias = nn.Embedding(c.buckets, c.heads)

    def position_bias(self, s, device):
        pos = torch.arange(s, device=device)
        rel = pos[None, :] - pos[:, None]
        bucket = relative_position_bucket(rel, self.c.buckets, self.c.max_distance)
        return self.relative_attention_bias(bucket).permute(2, 0, 1).float()  # [H, S, S]


class _AttnLayer(nn.Module):
    def __init__(self, c, has_bias):
        super().__init__()
        self.SelfAttention = _SelfAttention(c, has_bias)
        self.layer_norm = T5RMSNorm(c.d_model, c.eps)

    def forward(self, x, bias, mask):
        a = self.SelfAttention
        b, s, _ = x.shape
        h = self.layer_norm(x)
        q, k, v = (m(h).view(b, s, a.c.heads, a.c.d_kv).transpose(1, 2).float() for m in (a.q, a.k, a.v))
        scores = q @ k.transpose(-1, -2) + bias[None]  # T5: no 1/sqrt(d) scaling
        if mask is not None:
            scores = scores.masked_fill(~mask[:, None, None, :], float("-inf"))
        o = (torch.softmax(scores, -1) @ v).transpose(1, 2).reshape(b, s, -1).to(x.dtype)
        return a.o(o, residual=x)


class _FFLayer(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.DenseReluDense = nn.Module()
        self.DenseReluDense.wi_0 = Linear(c.d_model, c.d_ff, bias=False)
        self.DenseReluDense.wi_1 = Linear(c.d_model, c.d_ff, bias=False)
        self.DenseReluDense.wo = Linear(c.d_ff, c.d_model, bias=False)
        self.layer_norm = T5RMSNorm(c.d_model, c.eps)

    def forward(self, x):
        d = self.DenseReluDense
        h = self.layer_norm(x)
        g = d.wi_0(h, act="gelu_tanh")
        return d.wo(g * d.wi_1(h), residual=x)


class _Block(nn.Module):
    def __init__(self, c, has_bias):
        super().__init__()
        self.layer = nn.ModuleList([_AttnLayer(c, has_bias), _FFLayer(c)])


class T5Encoder(nn.Module):
    def __init__(self, c: T5Config = T5_XXL):
        super().__init__()
        self.cfg = c
        self.shared = nn.Embedding(c.vocab, c.d_model)
        self.encoder = nn.Module()
        self.encoder.block = nn.ModuleList([_Block(c, i == 0) for i in range(c.layers)])
        self.encoder.final_layer_norm = T5RMSNorm(c.d_model, c.eps)
        self.checkpoint_ignore = ("encoder.embed_tokens.",)  # tied to ``shared`` in transformers checkpoints

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, mask: torch.Tensor | None = None) -> torch.Tensor:
        dt = self.shared.weight.dtype
        x = self.shared(ids).to(dt)
        bias = self.encoder.block[0].layer[0].SelfAttention.position_bias(ids.shape[1], ids.device)
        for blk in self.encoder.block:
            x = blk.layer[0](x, bias, mask)
            x = blk.layer[1](x)
        return self.encoder.final_layer_norm(x)


class T5Tokenizer:
    """SentencePiece (``spiece.model``) when present; deterministic hash
    fallback otherwise.  Appends ``</s>`` (id 1), pads with 0 to max_length."""

    def __init__(self, model_dir: str | None = None, max_length: int = 77, vocab: int = 32128):
        self.max_length, self.vocab = max_length, vocab
        self.sp = None
        path = os.path.join(model_dir, "spiece.model") if model_dir else None
        if path and os.path.exists(path):
            import sentencepiece

            self.sp = sentencepiece.SentencePieceProcessor(model_file=path)

    def encode(self, text: str) -> list[int]:
        # IFPipeline without bs4/ftfy caption cleaning: lower-case + strip
        text = text.lower().strip()
        if self.sp is not None:
            return list(self.sp.encode(text))
        return [int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little") % (self.vocab - 100) + 3
                for w in text.lower().split()]

    def __call__(self, texts: list[str]):
        ids, masks = [], []
        for t in texts:
            x = self.encode(t)[: self.max_length - 1] + [1]
            masks.append([1] * len(x) + [0] * (self.max_length - len(x)))
            ids.append(x + [0] * (self.max_length - len(x)))
        return torch.tensor(ids), torch.tensor(masks, dtype=torch.bool)
