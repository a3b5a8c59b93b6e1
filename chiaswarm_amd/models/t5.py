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


def relative_position_bucket(rel: torch.Tensor, num_buckets=32, max_distance=128, bidirectional=True) -> torch.Tensor:
    """T5 bucketing of (key - query) offsets; the decoder's self-attention is
    unidirectional (only offsets <= 0, all buckets for the past)."""
    if bidirectional:
        num_buckets //= 2
        out = (rel > 0).long() * num_buckets
        n = rel.abs()
    else:
        out = torch.zeros_like(rel)
        n = (-rel).clamp_min(0)
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

    def position_bias(self, s, device, bidirectional=True):
        pos = torch.arange(s, device=device)
        rel = pos[None, :] - pos[:, None]
        bucket = relative_position_bucket(rel, self.c.buckets, self.c.max_distance, bidirectional)
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


def _attend(a: "_SelfAttention", h, kv_src, bias, mask):
    """softmax(q k^T + bias [+ key mask]) v for one T5 attention (no 1/sqrt(d))."""
    b, s, _ = h.shape
    t = kv_src.shape[1]
    q = a.q(h).view(b, s, a.c.heads, a.c.d_kv).transpose(1, 2).float()
    k = a.k(kv_src).view(b, t, a.c.heads, a.c.d_kv).transpose(1, 2).float()
    v = a.v(kv_src).view(b, t, a.c.heads, a.c.d_kv).transpose(1, 2).float()
    scores = q @ k.transpose(-1, -2)
    if bias is not None:
        scores = scores + bias[None]
    if mask is not None:
        scores = scores.masked_fill(~mask[:, None, None, :], float("-inf"))
    return (torch.softmax(scores, -1) @ v).transpose(1, 2).reshape(b, s, -1)


class _DecSelfLayer(nn.Module):
    def __init__(self, c, has_bias):
        super().__init__()
        self.SelfAttention = _SelfAttention(c, has_bias)
        self.layer_norm = T5RMSNorm(c.d_model, c.eps)

    def forward(self, x, bias):
        h = self.layer_norm(x)
        return self.SelfAttention.o(_attend(self.SelfAttention, h, h, bias, None).to(x.dtype), residual=x)


class _CrossLayer(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.EncDecAttention = _SelfAttention(c, False)
        self.layer_norm = T5RMSNorm(c.d_model, c.eps)

    def forward(self, x, enc, enc_mask):
        h = self.layer_norm(x)
        return self.EncDecAttention.o(_attend(self.EncDecAttention, h, enc, None, enc_mask).to(x.dtype), residual=x)


class _DecBlock(nn.Module):
    def __init__(self, c, has_bias):
        super().__init__()
        self.layer = nn.ModuleList([_DecSelfLayer(c, has_bias), _CrossLayer(c), _FFLayer(c)])


class T5Seq2Seq(nn.Module):
    """T5 v1.1 / Flan-T5 encoder-decoder (transformers ``T5ForConditionalGeneration``
    parameter names: ``shared``, ``encoder.*``, ``decoder.*``, ``lm_head``), for
    BLIP-2's Flan-T5 language models.  The encoder takes input EMBEDDINGS (BLIP-2
    puts the projected image queries ahead of the prompt); the decoder re-runs
    its (short) prefix each greedy step with the causal relative-position bias
    and cross-attention over the encoder output."""

    def __init__(self, c: T5Config, dec_layers: int | None = None, tie_embeddings: bool = False):
        super().__init__()
        self.cfg = c
        self.tie = tie_embeddings
        self.shared = nn.Embedding(c.vocab, c.d_model)
        self.encoder = nn.Module()
        self.encoder.block = nn.ModuleList([_Block(c, i == 0) for i in range(c.layers)])
        self.encoder.final_layer_norm = T5RMSNorm(c.d_model, c.eps)
        self.decoder = nn.Module()
        self.decoder.block = nn.ModuleList([_DecBlock(c, i == 0) for i in range(dec_layers or c.layers)])
        self.decoder.final_layer_norm = T5RMSNorm(c.d_model, c.eps)
        self.lm_head = Linear(c.d_model, c.vocab, bias=False)
        self.checkpoint_ignore = ("encoder.embed_tokens.", "decoder.embed_tokens.")

    @torch.no_grad()
    def encode(self, x: torch.Tensor, mask: torch.Tensor | None = None) -> torch.Tensor:
        bias = self.encoder.block[0].layer[0].SelfAttention.position_bias(x.shape[1], x.device)
        for blk in self.encoder.block:
            x = blk.layer[0](x, bias, mask)
            x = blk.layer[1](x)
        return self.encoder.final_layer_norm(x)

    @torch.no_grad()
    def decode_logits(self, enc: torch.Tensor, ids: list[int], enc_mask=None) -> torch.Tensor:
        """Next-token logits [vocab] after decoder ids (starting with the
        decoder start token)."""
        dt = self.shared.weight.dtype
        x = self.shared(torch.tensor([ids], device=enc.device)).to(dt)
        s = x.shape[1]
        bias = self.decoder.block[0].layer[0].SelfAttention.position_bias(s, x.device, bidirectional=False)
        bias = bias.masked_fill(torch.ones(s, s, dtype=torch.bool, device=x.device).triu(1)[None], float("-inf"))
        for blk in self.decoder.block:
            x = blk.layer[0](x, bias)
            x = blk.layer[1](x, enc, enc_mask)
            x = blk.layer[2](x)
        h = self.decoder.final_layer_norm(x[:, -1:])
        if self.tie:  # tied head (original T5): transformers rescales by d_model^-0.5
            h = (h.float() * self.cfg.d_model ** -0.5).to(h.dtype)
        return self.lm_head(h).float()[0, -1]


class T5Tokenizer:
    """SentencePiece (``spiece.model``) when present; deterministic hash
    fallback otherwise.  Appends ``</s>`` (id 1), pads with 0 to max_length."""

    def __init__(self, model_dir: str | None = None, max_length: int = 77, vocab: int = 32128, lower: bool = True):
        self.max_length, self.vocab, self.lower = max_length, vocab, lower
        self.sp = None
        path = os.path.join(model_dir, "spiece.model") if model_dir else None
        if path and os.path.exists(path):
            import sentencepiece

            self.sp = sentencepiece.SentencePieceProcessor(model_file=path)

    def encode(self, text: str) -> list[int]:
        # IFPipeline without bs4/ftfy caption cleaning: lower-case + strip
        # (lower=False: the plain tokenizer, e.g. BLIP-2's Flan-T5 prompts)
        text = (text.lower() if self.lower else text).strip()
        if self.sp is not None:
            return list(self.sp.encode(text))
        return [int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little") % (self.vocab - 100) + 3
                for w in text.split()]

    def decode(self, ids: list[int]) -> str:
        """Text of ``ids`` without pad / eos (``skip_special_tokens``)."""
        ids = [int(i) for i in ids if int(i) not in (0, 1)]
        if self.sp is not None:
            return self.sp.decode(ids)
        return " ".join(f"w{i}" for i in ids)

    def __call__(self, texts: list[str]):
        ids, masks = [], []
        for t in texts:
            x = self.encode(t)[: self.max_length - 1] + [1]
            masks.append([1] * len(x) + [0] * (self.max_length - len(x)))
            ids.append(x + [0] * (self.max_length - len(x)))
        return torch.tensor(ids), torch.tensor(masks, dtype=torch.bool)
