"""ViT -> GPT-2 image captioning (transformers ``VisionEncoderDecoderModel`` with a
``ViTModel`` encoder and a cross-attending ``GPT2LMHeadModel`` decoder, e.g.
``nlpconnect/vit-gpt2-image-captioning``; ``ViTImageProcessor`` +
``GPT2Tokenizer``).  Reference: the hive names the model / processor classes
at swarm/captioning/caption_image.py:11-29 and the reference instantiates the
class it is given.

Both halves run on the shared kernels: the encoder is the package ViT
(post-LN on every token), the decoder is pre-LN GPT-2 blocks with
cross-attention (fused-QKV GEMM, flash attention with the causal mask,
tanh-GELU MLP, residual adds in the GEMM epilogues).  The image K/V of every
cross-attention layer are computed once per image; greedy decode from the
decoder start token (GPT-2's ``<|endoftext|>``) re-runs the short prefix each
step (transformers' default ``max_length=20``), stopping at eos.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch
import torch.nn as nn
from PIL import Image

from .layers import LayerNorm, Linear
from .transformer import PreLNBlock, ViT


@dataclasses.dataclass
class VitGpt2Config:
    image_size: int = 224
    patch: int = 16
    enc_dim: int = 768
    enc_depth: int = 12
    enc_heads: int = 12
    enc_mlp: int = 3072
    enc_eps: float = 1e-12
    dim: int = 768
    depth: int = 12
    heads: int = 12
    mlp: int = 3072
    eps: float = 1e-5
    vocab: int = 50257
    max_pos: int = 1024
    start_id: int = 50256
    eos_id: int = 50256
    pad_id: int = 50256
    mean: tuple = (0.5, 0.5, 0.5)
    std: tuple = (0.5, 0.5, 0.5)

    @classmethod
    def from_hf(cls, cfg: dict, preprocessor: dict | None = None) -> "VitGpt2Config":
        """A transformers ``VisionEncoderDecoderConfig`` config.json (ViT encoder,
        GPT-2 decoder); ``preprocessor``: preprocessor_config.json (mean / std)."""
        e, d = cfg.get("encoder") or {}, cfg.get("decoder") or {}
        if e.get("model_type", "vit") != "vit" or d.get("model_type", "gpt2") != "gpt2":
            raise ValueError(f"img2txt: VisionEncoderDecoderModel {e.get('model_type')!r} -> "
                             f"{d.get('model_type')!r} is not supported (vit -> gpt2)")
        p = preprocessor or {}
        eos = d.get("eos_token_id", 50256)
        return cls(image_size=e.get("image_size", 224), patch=e.get("patch_size", 16), enc_dim=e.get("hidden_size", 768),
                   enc_depth=e.get("num_hidden_layers", 12), enc_heads=e.get("num_attention_heads", 12),
                   enc_mlp=e.get("intermediate_size", 3072), enc_eps=e.get("layer_norm_eps", 1e-12),
                   dim=d.get("n_embd", 768), depth=d.get("n_layer", 12), heads=d.get("n_head", 12),
                   mlp=d.get("n_inner") or 4 * d.get("n_embd", 768), eps=d.get("layer_norm_epsilon", 1e-5),
                   vocab=d.get("vocab_size", 50257), max_pos=d.get("n_positions", 1024),
                   start_id=cfg.get("decoder_start_token_id") or d.get("bos_token_id", 50256), eos_id=eos,
                   pad_id=cfg.get("pad_token_id") or eos,
                   mean=tuple(p.get("image_mean", (0.5, 0.5, 0.5))), std=tuple(p.get("image_std", (0.5, 0.5, 0.5))))


VIT_GPT2 = VitGpt2Config()
TINY_VIT_GPT2 = VitGpt2Config(image_size=32, patch=16, enc_dim=32, enc_depth=2, enc_heads=2, enc_mlp=64, dim=32,
                              depth=2, heads=2, mlp=64, vocab=100, max_pos=64, start_id=1, eos_id=2, pad_id=2)

# ViT layer names: hub checkpoints (encoder.encoder.layer.N.attention.attention.query ...)
# and newer transformers' own (encoder.layers.N.attention.q_proj ...)
_VIT = {"layernorm_before": "ln1", "attention.attention.query": "attn.q", "attention.attention.key": "attn.k",
        "attention.attention.value": "attn.v", "attention.output.dense": "attn.o", "layernorm_after": "ln2",
        "intermediate.dense": "fc1", "output.dense": "fc2", "attention.q_proj": "attn.q", "attention.k_proj": "attn.k",
        "attention.v_proj": "attn.v", "attention.o_proj": "attn.o", "mlp.fc1": "fc1", "mlp.fc2": "fc2"}


def _conv1d(v):
    """GPT-2 Conv1D weight [in, out] -> Linear [out, in]."""
    return v.t().contiguous() if v.dim() == 2 else v


def convert_hf_vit_gpt2(sd: dict) -> dict:
    """transformers ``VisionEncoderDecoderModel`` (ViT -> GPT-2) state dict ->
    this module's keys: Conv1D weights transposed, GPT-2's fused c_attn split
    into q / k / v (cross-attention: q_attn + the k / v pair), the LM head tied
    to ``wte``."""
    out: dict = {}
    for k, v in sd.items():
        if k.endswith(("attn.bias", "attn.masked_bias")) and v.dim() == 4:
            continue  # causal-mask buffers of old checkpoints
        if k.startswith("encoder.pooler.") or k == "decoder.lm_head.weight":
            continue
        if k.startswith("encoder.embeddings."):
            r = k.removeprefix("encoder.embeddings.")
            if r == "cls_token":
                out["encoder.class_embedding"] = v.reshape(-1)
            elif r == "position_embeddings":
                out["encoder.position_embedding"] = v.reshape(v.shape[-2], v.shape[-1])
            elif r.startswith("patch_embeddings.projection."):
                out["encoder.patch_embedding." + r.rsplit(".", 1)[1]] = v
            else:
                out[k] = v
        elif k.startswith("encoder.layernorm."):
            out["encoder.post_ln." + k.rsplit(".", 1)[1]] = v
        elif k.startswith(("encoder.encoder.layer.", "encoder.layers.")):
            n, rest = k.removeprefix("encoder.encoder.layer.").removeprefix("encoder.layers.").split(".", 1)
            for a, b in _VIT.items():
                if rest.startswith(a + "."):
                    out[f"encoder.layers.{n}.{b}{rest[len(a):]}"] = v
                    break
            else:
                out[k] = v
        elif k.startswith("decoder.transformer."):
            r = k.removeprefix("decoder.transformer.")
            if r in ("wte.weight", "wpe.weight"):
                out[r] = v
            elif r.startswith("ln_f."):
                out["ln_f." + r.rsplit(".", 1)[1]] = v
            elif r.startswith("h."):
                n, rest = r.removeprefix("h.").split(".", 1)
                pre = f"layers.{n}."
                kind = rest.rsplit(".", 1)[1]
                if rest.startswith("attn.c_attn."):
                    parts = _conv1d(v).chunk(3, 0)
                    for nm, part in zip("qkv", parts):
                        out[pre + f"attn.{nm}.{kind}"] = part.contiguous()
                elif rest.startswith("crossattention.c_attn."):
                    parts = _conv1d(v).chunk(2, 0)
                    for nm, part in zip("kv", parts):
                        out[pre + f"cross.{nm}.{kind}"] = part.contiguous()
                else:
                    m = {"attn.c_proj": "attn.o", "crossattention.q_attn": "cross.q",
                         "crossattention.c_proj": "cross.o", "mlp.c_fc": "fc1", "mlp.c_proj": "fc2", "ln_1": "ln1",
                         "ln_2": "ln2", "ln_cross_attn": "ln_x"}
                    for a, b in m.items():
                        if rest.startswith(a + "."):
                            out[pre + b + "." + kind] = _conv1d(v) if not a.startswith("ln") else v
                            break
                    else:
                        out[k] = v
            else:
                out[k] = v
        else:
            out[k] = v  # unknown keys surface as a CheckpointMismatch in load_into
    return out


class VitGpt2Captioner(nn.Module):
    def __init__(self, cfg: VitGpt2Config = VIT_GPT2):
        super().__init__()
        self.cfg = cfg
        self.encoder = ViT(cfg.image_size, cfg.patch, cfg.enc_dim, cfg.enc_depth, cfg.enc_heads, cfg.enc_mlp,
                           eps=cfg.enc_eps)
        # encoder width != decoder width: transformers inserts a projection
        self.enc_to_dec_proj = Linear(cfg.enc_dim, cfg.dim) if cfg.enc_dim != cfg.dim else None
        self.wte = nn.Embedding(cfg.vocab, cfg.dim)
        self.wpe = nn.Embedding(cfg.max_pos, cfg.dim)
        self.layers = nn.ModuleList([PreLNBlock(cfg.dim, cfg.heads, cfg.mlp, act="gelu_tanh", cross_dim=cfg.dim,
                                                eps=cfg.eps) for _ in range(cfg.depth)])
        self.ln_f = LayerNorm(cfg.dim, eps=cfg.eps)

    def preprocess(self, image: Image.Image) -> torch.Tensor:
        """ViTImageProcessor: bilinear resize to image_size², /255, mean / std; NHWC."""
        s = self.cfg.image_size
        a = np.asarray(image.convert("RGB").resize((s, s), Image.Resampling.BILINEAR), np.float32) / 255.0
        a = (a - np.array(self.cfg.mean, np.float32)) / np.array(self.cfg.std, np.float32)
        return torch.from_numpy(a)[None]

    @torch.no_grad()
    def image_kv(self, pixels: torch.Tensor):
        """Per-layer cross-attention K/V of the encoder tokens (computed once)."""
        enc = self.encoder(pixels.to(self.wte.weight.dtype))
        if self.enc_to_dec_proj is not None:
            enc = self.enc_to_dec_proj(enc)
        return [blk.cross.kv_of(enc) for blk in self.layers]

    @torch.no_grad()
    def logits(self, kvs, ids: list[int]) -> torch.Tensor:
        """Next-token logits [vocab] after decoder ids."""
        dev = self.wte.weight.device
        t = torch.tensor([ids], device=dev)
        x = self.wte(t) + self.wpe.weight[: t.shape[1]][None]
        for blk, kv in zip(self.layers, kvs):
            x = blk.attn(blk.ln1(x), residual=x, causal=True)
            x = blk.cross(blk.ln_x(x), kv=kv, residual=x)
            x = blk.fc2(blk.fc1(blk.ln2(x), act=blk.act), residual=x)
        h = self.ln_f(x[:, -1:])
        return (h.float() @ self.wte.weight.float().t())[0, -1]

    @torch.no_grad()
    def generate(self, image: Image.Image, prefix_ids: list[int], max_new_tokens: int | None = None,
                 max_length: int = 20) -> list[int]:
        """Greedy decode from ``start + prefix``; returns prefix + generated ids."""
        if max_new_tokens is None:
            max_new_tokens = max(0, max_length - 1 - len(prefix_ids))
        kvs = self.image_kv(self.preprocess(image).to(self.wte.weight.device))
        ids = [self.cfg.start_id] + list(prefix_ids)
        out = []
        for _ in range(max_new_tokens):
            nxt = int(self.logits(kvs, ids).argmax())
            if nxt == self.cfg.eos_id:
                break
            ids.append(nxt)
            out.append(nxt)
        return list(prefix_ids) + out
