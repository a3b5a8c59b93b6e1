"""CLAP text tower (RoBERTa encoder + pooler + 2-layer projection) for AudioLDM.

AudioLDM conditions its UNet on the L2-normalised CLAP text embedding of the
prompt (one 512-d vector per prompt, fed through the UNet's
``simple_projection`` class embedding).  Geometry is the public
``ClapTextModelWithProjection`` config (RoBERTa-base, 12 post-LN layers,
projection 768 -> 512 -> 512 with ReLU), reached by the reference via
``AudioLDMPipeline`` at swarm/audio/audioldm.py:12-24.

MI355X path: every projection is the MFMA GEMM with fused bias / GELU /
residual epilogues, attention is the flash kernel.  Prompts are encoded
unpadded (one sequence per prompt), which is exactly equivalent to the padded +
attention-masked HF computation for the pooled first-token output and needs no
key-padding mask in the attention kernel.
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn as nn

from .layers import LayerNorm, Linear
from .transformer import PostLNBlock


@dataclasses.dataclass
class ClapTextConfig:
    vocab: int = 50265
    dim: int = 768
    depth: int = 12
    heads: int = 12
    mlp: int = 3072
    max_pos: int = 514
    pad_id: int = 1
    eps: float = 1e-12
    projection_dim: int = 512


CLAP_TEXT = ClapTextConfig()
TINY_CLAP = ClapTextConfig(vocab=1000, dim=64, depth=2, heads=2, mlp=128, max_pos=80, projection_dim=32)

# transformers key -> our module names (substring renames, applied in order)
HF_RENAMES = {
    "text_model.embeddings.": "", "text_model.encoder.layer.": "layers.",
    ".attention.self.query.": ".attn.q.", ".attention.self.key.": ".attn.k.",
    ".attention.self.value.": ".attn.v.", ".attention.output.dense.": ".attn.o.",
    ".attention.output.LayerNorm.": ".ln1.", ".intermediate.dense.": ".fc1.",
    ".output.dense.": ".fc2.", ".output.LayerNorm.": ".ln2.", "text_model.pooler.dense.": "pooler.",
    "LayerNorm.": "emb_ln.",
}


class ClapTextEncoder(nn.Module):
    def __init__(self, cfg: ClapTextConfig = CLAP_TEXT):
        super().__init__()
        self.cfg = cfg
        self.word_embeddings = nn.Embedding(cfg.vocab, cfg.dim)
        self.position_embeddings = nn.Embedding(cfg.max_pos, cfg.dim)
        self.token_type_embeddings = nn.Embedding(1, cfg.dim)
        self.emb_ln = LayerNorm(cfg.dim, eps=cfg.eps)
        self.layers = nn.ModuleList([PostLNBlock(cfg.dim, cfg.heads, cfg.mlp, eps=cfg.eps) for _ in range(cfg.depth)])
        self.pooler = Linear(cfg.dim, cfg.dim)
        self.text_projection = nn.Module()
        self.text_projection.linear1 = Linear(cfg.dim, cfg.projection_dim)
        self.text_projection.linear2 = Linear(cfg.projection_dim, cfg.projection_dim)

    @torch.no_grad()
    def forward(self, ids_list: list[list[int]]) -> torch.Tensor:
        """Unpadded token-id lists -> L2-normalised text embeddings [B, projection_dim] (fp32)."""
        dev = self.word_embeddings.weight.device
        dt = self.word_embeddings.weight.dtype
        outs = []
        for ids in ids_list:
            ids = ids[: self.cfg.max_pos - 2]
            t = torch.tensor([ids], device=dev)
            # RoBERTa positions start after padding_idx (no padding in an unpadded sequence)
            pos = torch.arange(len(ids), device=dev)[None] + self.cfg.pad_id + 1
            x = self.word_embeddings(t) + self.position_embeddings(pos) + self.token_type_embeddings.weight[0]
            x = self.emb_ln(x.to(dt))
            for layer in self.layers:
                x = layer(x)
            pooled = torch.tanh(self.pooler(x[:, 0]).float()).to(dt)
            h = self.text_projection.linear1(pooled, act="relu")
            outs.append(self.text_projection.linear2(h).float())
        e = torch.cat(outs, 0)
        return e / e.norm(dim=-1, keepdim=True).clamp_min(1e-12)
