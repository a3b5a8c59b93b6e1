"""LLaMA / Vicuna decoder (transformers ``LlamaForCausalLM`` parameter names:
``model.embed_tokens``, ``model.layers.{i}.self_attn.{q,k,v,o}_proj``,
``mlp.{gate,up,down}_proj``, ``input_layernorm`` / ``post_attention_layernorm``,
``model.norm``, ``lm_head``) for InstructBLIP's Vicuna language models.

Pre-RMSNorm blocks; rotary position embedding (rotate-half form, default
theta 10000) on q / k; grouped K/V heads expanded to the query heads; SwiGLU
MLP (SiLU of gate_proj fused into its GEMM epilogue, the residual adds fused
into o_proj / down_proj).  Input embeddings may be given directly (the image
query embeddings precede the prompt); greedy decode re-runs the short
sequence (the GEMMs stream their weights once per step either way).
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn

from .. import ops
from .layers import Linear


@dataclasses.dataclass
class LlamaConfig:
    vocab: int = 32000
    dim: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 32
    ffn: int = 11008
    eps: float = 1e-6
    theta: float = 10000.0
    bos_id: int = 1
    eos_id: int = 2

    @classmethod
    def from_hf(cls, t: dict) -> "LlamaConfig":
        rope = t.get("rope_parameters") or t.get("rope_scaling") or {}
        if rope.get("rope_type", rope.get("type", "default")) not in ("default", None):
            raise ValueError(f"img2txt: LLaMA rope type {rope.get('rope_type')!r} is not supported")
        return cls(vocab=t.get("vocab_size", 32000), dim=t.get("hidden_size", 4096),
                   layers=t.get("num_hidden_layers", 32), heads=t.get("num_attention_heads", 32),
                   kv_heads=t.get("num_key_value_heads") or t.get("num_attention_heads", 32),
                   ffn=t.get("intermediate_size", 11008), eps=t.get("rms_norm_eps", 1e-6),
                   theta=rope.get("rope_theta", t.get("rope_theta", 10000.0)), bos_id=t.get("bos_token_id", 1),
                   eos_id=t.get("eos_token_id", 2))


class RMSNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        return (self.weight.float() * (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps))).to(x.dtype)


def _rotate_half(x):
    h = x.shape[-1] // 2
    return torch.cat((-x[..., h:], x[..., :h]), -1)


class _Attn(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.c, self.hd = c, c.dim // c.heads
        self.q_proj = Linear(c.dim, c.heads * self.hd, bias=False)
        self.k_proj = Linear(c.dim, c.kv_heads * self.hd, bias=False)
        self.v_proj = Linear(c.dim, c.kv_heads * self.hd, bias=False)
        self.o_proj = Linear(c.heads * self.hd, c.dim, bias=False)

    def forward(self, h, x, cos, sin):
        b, s, _ = h.shape
        q = self.q_proj(h).view(b, s, self.c.heads, self.hd)
        k = self.k_proj(h).view(b, s, self.c.kv_heads, self.hd)
        v = self.v_proj(h).view(b, s, self.c.kv_heads, self.hd)
        qf, kf = q.float(), k.float()
        q = (qf * cos + _rotate_half(qf) * sin).to(h.dtype)
        k = (kf * cos + _rotate_half(kf) * sin).to(h.dtype)
        if self.c.kv_heads != self.c.heads:
            rep = self.c.heads // self.c.kv_heads
            k, v = k.repeat_interleave(rep, 2), v.repeat_interleave(rep, 2)
        o = ops.attention(q.contiguous(), k.contiguous(), v.contiguous(), self.hd ** -0.5, causal=True)
        return self.o_proj(o.reshape(b, s, -1), residual=x)


class _MLP(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.gate_proj = Linear(c.dim, c.ffn, bias=False)
        self.up_proj = Linear(c.dim, c.ffn, bias=False)
        self.down_proj = Linear(c.ffn, c.dim, bias=False)

    def forward(self, h, x):
        return self.down_proj(self.gate_proj(h, act="silu") * self.up_proj(h), residual=x)


class _Layer(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.self_attn = _Attn(c)
        self.mlp = _MLP(c)
        self.input_layernorm = RMSNorm(c.dim, c.eps)
        self.post_attention_layernorm = RMSNorm(c.dim, c.eps)


class LlamaLM(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.cfg = c
        self.model = nn.Module()
        self.model.embed_tokens = nn.Embedding(c.vocab, c.dim)
        self.model.layers = nn.ModuleList([_Layer(c) for _ in range(c.layers)])
        self.model.norm = RMSNorm(c.dim, c.eps)
        self.lm_head = Linear(c.dim, c.vocab, bias=False)

    def _rope(self, s, device):
        hd = self.cfg.dim // self.cfg.heads
        inv = 1.0 / (self.cfg.theta ** (torch.arange(0, hd, 2, dtype=torch.float32, device=device) / hd))
        f = torch.arange(s, dtype=torch.float32, device=device)[:, None] * inv[None]
        emb = torch.cat((f, f), -1)
        return emb.cos()[None, :, None], emb.sin()[None, :, None]  # [1, S, 1, hd]

    @torch.no_grad()
    def last_logits(self, x: torch.Tensor) -> torch.Tensor:
        """Next-token logits [vocab] after input embeddings x [1, S, dim]."""
        cos, sin = self._rope(x.shape[1], x.device)
        for lyr in self.model.layers:
            x = lyr.self_attn(lyr.input_layernorm(x), x, cos, sin)
            x = lyr.mlp(lyr.post_attention_layernorm(x), x)
        return self.lm_head(self.model.norm(x[:, -1:])).float()[0, -1]
