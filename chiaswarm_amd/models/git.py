"""GIT image captioning (GenerativeImage2Text: CLIP ViT image encoder ->
projection -> a BERT-style post-LN decoder over [image tokens; text tokens]).
Reference: the transformers ``GitForCausalLM`` / ``GitProcessor`` (or
``AutoProcessor``) pair a hive job may name at
swarm/captioning/caption_image.py:11-29; greedy ``generate`` from [CLS] with
transformers' default ``max_length=20``, stopping at [SEP].

Attention layout (transformers' GIT mask): the image tokens attend to each
other bidirectionally and never to text; each text token attends to every
image token and causally to the text before it.  So the image half of every
layer is independent of the text: it runs ONCE per image and each layer keeps
its image K/V; a decode step runs only the text tokens, attending over
[image K/V; text K/V] with the bottom-right-aligned causal mask of the shared
flash-attention kernel (the image keys precede every query).
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch
import torch.nn as nn
from PIL import Image

from .. import ops
from .layers import LayerNorm, Linear
from .transformer import PostLNBlock, ViT

MEAN = np.array([0.48145466, 0.4578275, 0.40821073], np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], np.float32)


@dataclasses.dataclass
class GitConfig:
    image_size: int = 224
    patch: int = 16
    vision_dim: int = 768
    vision_depth: int = 12
    vision_heads: int = 12
    vision_mlp: int = 3072
    vision_eps: float = 1e-5
    dim: int = 768
    depth: int = 6
    heads: int = 12
    mlp: int = 3072
    eps: float = 1e-12
    vocab: int = 30522
    max_pos: int = 1024
    bos_id: int = 101  # [CLS]
    eos_id: int = 102  # [SEP]

    @classmethod
    def from_hf(cls, cfg: dict) -> "GitConfig":
        """A transformers ``GitConfig`` config.json."""
        v = cfg.get("vision_config") or {}
        return cls(image_size=v.get("image_size", 224), patch=v.get("patch_size", 16),
                   vision_dim=v.get("hidden_size", 768), vision_depth=v.get("num_hidden_layers", 12),
                   vision_heads=v.get("num_attention_heads", 12), vision_mlp=v.get("intermediate_size", 3072),
                   vision_eps=v.get("layer_norm_eps", 1e-5), dim=cfg.get("hidden_size", 768),
                   depth=cfg.get("num_hidden_layers", 6), heads=cfg.get("num_attention_heads", 12),
                   mlp=cfg.get("intermediate_size", 3072), eps=cfg.get("layer_norm_eps", 1e-12),
                   vocab=cfg.get("vocab_size", 30522), max_pos=cfg.get("max_position_embeddings", 1024),
                   bos_id=cfg.get("bos_token_id", 101), eos_id=cfg.get("eos_token_id", 102))


GIT_BASE = GitConfig()  # microsoft/git-base(-coco/-textcaps): CLIP ViT-B/16
GIT_LARGE = GitConfig(patch=14, vision_dim=1024, vision_depth=24, vision_heads=16, vision_mlp=4096)  # ViT-L/14
TINY_GIT = GitConfig(image_size=32, patch=16, vision_dim=32, vision_depth=2, vision_heads=2, vision_mlp=64, dim=32,
                     depth=2, heads=2, mlp=64, vocab=100, max_pos=64, bos_id=1, eos_id=2)


def convert_hf_git(sd: dict) -> dict:
    """transformers ``GitForCausalLM`` state dict -> this module's keys."""
    vis = {"embeddings.patch_embedding.": "patch_embedding.", "embeddings.class_embedding": "class_embedding",
           "embeddings.position_embedding.weight": "position_embedding", "pre_layrnorm.": "pre_ln.",
           "post_layernorm.": "post_ln.", "encoder.layers.": "layers.", ".self_attn.q_proj.": ".attn.q.",
           ".self_attn.k_proj.": ".attn.k.", ".self_attn.v_proj.": ".attn.v.", ".self_attn.out_proj.": ".attn.o.",
           ".layer_norm1.": ".ln1.", ".layer_norm2.": ".ln2.", ".mlp.fc1.": ".fc1.", ".mlp.fc2.": ".fc2."}
    txt = {".attention.self.query.": ".attn.q.", ".attention.self.key.": ".attn.k.",
           ".attention.self.value.": ".attn.v.", ".attention.output.dense.": ".attn.o.",
           ".attention.output.LayerNorm.": ".ln1.", ".intermediate.dense.": ".fc1.", ".output.dense.": ".fc2.",
           ".output.LayerNorm.": ".ln2."}
    out = {}
    for k, v in sd.items():
        if k.endswith("position_ids"):
            continue
        if k.startswith("git.image_encoder.vision_model."):
            r = k[len("git.image_encoder.vision_model."):]
            for a, b in vis.items():
                r = r.replace(a, b)
            out["image_encoder." + r] = v
        elif k.startswith("git.visual_projection.visual_projection."):
            r = k[len("git.visual_projection.visual_projection."):]
            out[("proj." if r.startswith("0.") else "proj_ln.") + r[2:]] = v
        elif k.startswith("git.embeddings."):
            r = k[len("git.embeddings."):].replace("LayerNorm.", "emb_ln.")
            out[r] = v
        elif k.startswith("git.encoder.layer."):
            r = "layers." + k[len("git.encoder.layer."):]
            for a, b in txt.items():
                r = r.replace(a, b)
            out[r] = v
        elif k.startswith("output."):
            out[k] = v
        else:
            out[k] = v  # unknown keys surface as a CheckpointMismatch in load_into
    return out


class GitCaptioner(nn.Module):
    def __init__(self, cfg: GitConfig = GIT_BASE):
        super().__init__()
        self.cfg = cfg
        self.image_encoder = ViT(cfg.image_size, cfg.patch, cfg.vision_dim, cfg.vision_depth, cfg.vision_heads,
                                 cfg.vision_mlp, eps=cfg.vision_eps, act="quick_gelu", pre_norm=True,
                                 patch_bias=False)
        self.proj = Linear(cfg.vision_dim, cfg.dim)
        self.proj_ln = LayerNorm(cfg.dim, eps=cfg.vision_eps)
        self.word_embeddings = nn.Embedding(cfg.vocab, cfg.dim)
        self.position_embeddings = nn.Embedding(cfg.max_pos, cfg.dim)
        self.emb_ln = LayerNorm(cfg.dim, eps=cfg.eps)
        self.layers = nn.ModuleList([PostLNBlock(cfg.dim, cfg.heads, cfg.mlp, eps=cfg.eps)
                                     for _ in range(cfg.depth)])
        self.output = Linear(cfg.dim, cfg.vocab)

    def preprocess(self, image: Image.Image) -> torch.Tensor:
        """CLIPImageProcessor: shortest side -> image_size (bicubic), centre crop,
        CLIP mean / std; NHWC [1, S, S, 3]."""
        s = self.cfg.image_size
        im = image.convert("RGB")
        w, h = im.size
        r = s / min(w, h)
        im = im.resize((max(s, round(w * r)), max(s, round(h * r))), Image.Resampling.BICUBIC)
        w, h = im.size
        left, top = (w - s) // 2, (h - s) // 2
        a = np.asarray(im.crop((left, top, left + s, top + s)), np.float32) / 255.0
        return torch.from_numpy((a - MEAN) / STD)[None]

    def _layer(self, blk, x, kv_prefix=None):
        """One post-LN layer on x [1, T, D]; with ``kv_prefix`` (the image K/V of
        this layer) the queries attend over [prefix; x] causally (text), else
        bidirectionally over x (image).  Returns (x', (k, v) of x)."""
        attn = blk.attn
        attn._ensure()
        b, t, _ = x.shape
        qkv = ops.gemm(x, attn.w_in, attn.b_in).view(b, t, 3, attn.heads, attn.dh)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        if kv_prefix is None:
            o = ops.attention(q, k, v, attn.scale)
        else:
            o = ops.attention(q, torch.cat([kv_prefix[0], k], 1), torch.cat([kv_prefix[1], v], 1), attn.scale,
                              causal=True)
        x = blk.ln1(attn.o(o.reshape(b, t, attn.heads * attn.dh), residual=x))
        x = blk.ln2(blk.fc2(blk.fc1(x, act="gelu"), residual=x))
        return x, (k.contiguous(), v.contiguous())

    @torch.no_grad()
    def image_kv(self, pixels: torch.Tensor):
        """Per-layer image K/V: the image half of the [image; text] sequence,
        computed once (it never attends to text)."""
        dt = self.output.weight.dtype
        h = self.proj_ln(self.proj(self.image_encoder(pixels.to(dt))))
        kvs = []
        for blk in self.layers:
            h, kv = self._layer(blk, h)
            kvs.append(kv)
        return kvs

    @torch.no_grad()
    def text_logits(self, kvs, ids: list[int]) -> torch.Tensor:
        """Next-token logits [vocab] after ``ids`` (text positions 0..T-1)."""
        dev = self.output.weight.device
        t = torch.tensor([ids], device=dev)
        x = self.emb_ln(self.word_embeddings(t) + self.position_embeddings.weight[: t.shape[1]][None])
        for blk, kv in zip(self.layers, kvs):
            x, _ = self._layer(blk, x, kv)
        return self.output(x[:, -1:]).float()[0, -1]

    @torch.no_grad()
    def generate(self, image: Image.Image, prefix_ids: list[int], max_new_tokens: int | None = None,
                 max_length: int = 20) -> list[int]:
        """Greedy decode from ``[CLS] + prefix`` (transformers' default
        ``max_length=20`` total tokens); returns prefix + generated ids."""
        if max_new_tokens is None:
            max_new_tokens = max(0, max_length - 1 - len(prefix_ids))
        kvs = self.image_kv(self.preprocess(image).to(self.output.weight.device))
        ids = [self.cfg.bos_id] + list(prefix_ids)
        out = []
        for _ in range(max_new_tokens):
            nxt = int(self.text_logits(kvs, ids).argmax())
            if nxt == self.cfg.eos_id:
                break
            ids.append(nxt)
            out.append(nxt)
        return list(prefix_ids) + out
