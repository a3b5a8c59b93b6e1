"""CLIP text encoders (CLIP-L/14, OpenCLIP-H/14, OpenCLIP-bigG/14) and the
CLIP ViT vision tower used by the safety checker (K14, K19).

transformers-compatible key layout (``text_model.encoder.layers.N.self_attn.
q_proj`` ...).  Runs once per request (not per step), so it uses the same GEMM /
attention / LayerNorm kernels as the UNet with a causal mask.
Reference call sites: prompt encoding inside the diffusers pipeline call at
swarm/diffusion/diffusion_func.py:96 and the safety checker (:98-111).
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn

from .. import ops
from .layers import LayerNorm, Linear, Prepared


@dataclasses.dataclass
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 1024
    intermediate_size: int = 4096
    num_layers: int = 23
    num_heads: int = 16
    max_position: int = 77
    act: str = "gelu"  # "quick_gelu" for OpenAI CLIP-L
    projection_dim: int | None = None  # CLIPTextModelWithProjection
    eos_token_id: int = 49407


CLIP_L = CLIPTextConfig(hidden_size=768, intermediate_size=3072, num_layers=12, num_heads=12, act="quick_gelu")
OPENCLIP_H = CLIPTextConfig()  # SD2.x text encoder (23 layers kept)
OPENCLIP_BIGG = CLIPTextConfig(hidden_size=1280, intermediate_size=5120, num_layers=32, num_heads=20,
                               projection_dim=1280)
TINY_TEXT = CLIPTextConfig(vocab_size=1000, hidden_size=32, intermediate_size=64, num_layers=2, num_heads=2)
TINY_TEXT_G = dataclasses.replace(TINY_TEXT, projection_dim=32)  # second (pooled) encoder of tiny-xl


class _SelfAttn(Prepared):
    def __init__(self, d, heads):
        super().__init__()
        self.heads, self.dh = heads, d // heads
        self.q_proj, self.k_proj, self.v_proj, self.out_proj = (Linear(d, d) for _ in range(4))

    def prepare(self):
        self.w_qkv = torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0).detach()
        self.b_qkv = torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias], 0).detach()

    def forward(self, x, residual, causal=True):
        w = getattr(self, "w_qkv", None)
        if w is None or w.device != self.q_proj.weight.device or w.dtype != self.q_proj.weight.dtype:
            self.prepare()
        b, s, d = x.shape
        qkv = ops.gemm(x, self.w_qkv, self.b_qkv).view(b, s, 3, self.heads, self.dh)
        o = ops.attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], causal=causal)
        return self.out_proj(o.reshape(b, s, d), residual=residual)


class _MLP(nn.Module):
    def __init__(self, d, inner, act):
        super().__init__()
        self.fc1, self.fc2, self.act = Linear(d, inner), Linear(inner, d), act

    def forward(self, x, residual):
        return self.fc2(self.fc1(x, act=self.act), residual=residual)


class _Layer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.self_attn = _SelfAttn(cfg.hidden_size, cfg.num_heads)
        self.layer_norm1 = LayerNorm(cfg.hidden_size)
        self.mlp = _MLP(cfg.hidden_size, cfg.intermediate_size, cfg.act)
        self.layer_norm2 = LayerNorm(cfg.hidden_size)

    def forward(self, x, causal=True):
        x = self.self_attn(self.layer_norm1(x), residual=x, causal=causal)
        return self.mlp(self.layer_norm2(x), residual=x)


class _Embeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.token_embedding = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = nn.Embedding(cfg.max_position, cfg.hidden_size)

    def forward(self, ids):
        s = ids.shape[1]
        return self.token_embedding(ids) + self.position_embedding.weight[:s][None]


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layers = nn.ModuleList([_Layer(cfg) for _ in range(cfg.num_layers)])


class _TextTransformer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.final_layer_norm = LayerNorm(cfg.hidden_size)


class CLIPTextModel(Prepared):
    """Returns (last_hidden_state, penultimate_hidden_state, pooled[, projected])."""

    def __init__(self, cfg: CLIPTextConfig = OPENCLIP_H):
        super().__init__()
        self.cfg = cfg
        self.text_model = _TextTransformer(cfg)
        self.checkpoint_alias_prefix = "text_model."  # transformers>=5 saves CLIPTextModel without it
        if cfg.projection_dim:
            self.text_projection = nn.Linear(cfg.hidden_size, cfg.projection_dim, bias=False)

    def _encode(self, input_ids):
        """(output of the last encoder layer before final_layer_norm, penultimate
        hidden state, final_layer_norm output)."""
        tm = self.text_model
        x = tm.embeddings(input_ids)
        penult = x
        n = len(tm.encoder.layers)
        for i, layer in enumerate(tm.encoder.layers):
            if i == n - 1:
                penult = x
            x = layer(x)
        if n == 1:
            penult = x
        return x, penult, tm.final_layer_norm(x)

    def _pool(self, last, input_ids):
        # pooled = hidden state at the EOS token (highest id in CLIP vocab order)
        eos_pos = (input_ids == self.cfg.eos_token_id).int().argmax(dim=-1)
        return last[torch.arange(last.shape[0], device=last.device), eos_pos]

    @torch.no_grad()
    def encode_pre_ln(self, input_ids: torch.Tensor):
        """(last encoder layer output BEFORE final_layer_norm, pooled output):
        transformers' ``hidden_states[-1]`` / ``pooler_output``, the latent x2
        upscaler's text conditioning."""
        x, _, last = self._encode(input_ids)
        return x, self._pool(last, input_ids)

    @torch.no_grad()
    def forward(self, input_ids: torch.Tensor):
        _, penult, last = self._encode(input_ids)
        pooled = self._pool(last, input_ids)
        proj = None
        if self.cfg.projection_dim:
            proj = pooled @ self.text_projection.weight.t().to(pooled.dtype)
        return last, penult, pooled, proj
