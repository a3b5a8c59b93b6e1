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

_HF_TEXT = {"attention.self.query": "attn.q", "attention.self.key": "attn.k", "attention.self.value": "attn.v",
            "attention.output.dense": "attn.o", "attention.output.LayerNorm": "ln1",
            "crossattention.self.query": "cross.q", "crossattention.self.key": "cross.k",
            "crossattention.self.value": "cross.v", "crossattention.output.dense": "cross.o",
            "crossattention.output.LayerNorm": "ln_x", "intermediate.dense": "fc1", "output.dense": "fc2",
            "output.LayerNorm": "ln2"}
_HF_VIS = {"self_attn.projection": "attn.o", "layer_norm1": "ln1", "layer_norm2": "ln2", "mlp.fc1": "fc1",
           "mlp.fc2": "fc2"}


def convert_hf_blip(sd: dict) -> dict:
    """transformers ``BlipForConditionalGeneration`` state dict -> this module's
    keys (fused vision qkv split into q/k/v; the LM head decoder weight is tied
    to the word embeddings and its bias duplicates ``cls.predictions.bias``)."""
    out = {}
    for k, v in sd.items():
        if k.startswith("text_decoder.cls.predictions.decoder."):
            continue
        if k == "text_decoder.cls.predictions.bias":
            out["head_bias"] = v
            continue
        m = k.removeprefix("text_decoder.")
        if m.startswith("cls.predictions.transform."):
            r = m.removeprefix("cls.predictions.transform.")
            out[("head_transform." if r.startswith("dense.") else "head_ln.") + r.split(".", 1)[1]] = v
            continue
        if m.startswith("bert.embeddings."):
            r = m.removeprefix("bert.embeddings.")
            out[r.replace("LayerNorm.", "emb_ln.")] = v
            continue
        if m.startswith("bert.encoder.layer."):
            n, rest = m.removeprefix("bert.encoder.layer.").split(".", 1)
            for a, b in _HF_TEXT.items():
                if rest.startswith(a + "."):
                    out[f"layers.{n}.{b}.{rest[len(a) + 1:]}"] = v
                    break
            else:
                out[k] = v  # surfaces as an unexpected key
            continue
        if k.startswith("vision_model.embeddings."):
            r = k.removeprefix("vision_model.embeddings.")
            if r == "class_embedding":
                v = v.reshape(-1)
            elif r == "position_embedding":
                v = v.reshape(v.shape[-2], v.shape[-1])
            out["vision_model." + r] = v
            continue
        if k.startswith("vision_model.post_layernorm."):
            out["vision_model.post_ln." + k.rsplit(".", 1)[1]] = v
            continue
        if k.startswith("vision_model.encoder.layers."):
            n, rest = k.removeprefix("vision_model.encoder.layers.").split(".", 1)
            pre = f"vision_model.layers.{n}."
            if rest.startswith("self_attn.qkv."):
                for name, part in zip("qkv", v.chunk(3, 0)):
                    out[pre + f"attn.{name}." + rest.rsplit(".", 1)[1]] = part.contiguous()
                continue
            for a, b in _HF_VIS.items():
                if rest.startswith(a + "."):
                    out[pre + b + rest[len(a):]] = v
                    break
            else:
                out[k] = v
            continue
        out[k] = v
    return out


def _convert_text_stack(rest: str, dst: str, v, out: dict, k: str):
    """One BERT-stack key (after its ``embeddings.`` / ``encoder.layer.`` prefix
    was split off by the caller) -> this package's names under ``dst``."""
    if rest.startswith("embeddings."):
        r = rest.removeprefix("embeddings.")
        out[dst + r.replace("LayerNorm.", "emb_ln.")] = v
        return
    if rest.startswith("encoder.layer."):
        n, tail = rest.removeprefix("encoder.layer.").split(".", 1)
        for a, b in _HF_TEXT.items():
            if tail.startswith(a + "."):
                out[f"{dst}layers.{n}.{b}.{tail[len(a) + 1:]}"] = v
                return
    out[k] = v  # surfaces as an unexpected key


def convert_hf_blip_vqa(sd: dict) -> dict:
    """transformers ``BlipForQuestionAnswering`` state dict -> ``BlipVQA`` keys:
    ``text_encoder.*`` (BERT over the question, cross-attending to the image)
    -> ``encoder.*``; ``text_decoder.bert.*`` -> ``decoder.*``; the LM head as in
    the captioner; the vision tower shared with ``convert_hf_blip``."""
    out, vis = {}, {}
    for k, v in sd.items():
        if k.startswith("text_encoder."):
            r = k.removeprefix("text_encoder.")
            if r.startswith("pooler."):
                continue  # add_pooling_layer=False in the reference model; harmless if present
            _convert_text_stack(r, "encoder.", v, out, k)
        elif k.startswith("text_decoder.cls.predictions.decoder."):
            continue
        elif k == "text_decoder.cls.predictions.bias":
            out["head_bias"] = v
        elif k.startswith("text_decoder.cls.predictions.transform."):
            r = k.removeprefix("text_decoder.cls.predictions.transform.")
            out[("head_transform." if r.startswith("dense.") else "head_ln.") + r.split(".", 1)[1]] = v
        elif k.startswith("text_decoder.bert."):
            _convert_text_stack(k.removeprefix("text_decoder.bert."), "decoder.", v, out, k)
        else:
            vis[k] = v
    out.update(convert_hf_blip(vis))
    return out


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


    patch: int = 16
    cross_dim: int | None = None  # text_config.encoder_hidden_size (None: vision_dim)
    cls_id: int = 101

    @classmethod
    def from_hf(cls, cfg: dict) -> "BlipConfig":
        """A transformers ``BlipConfig`` config.json (text_config / vision_config)."""
        t, v = cfg.get("text_config") or {}, cfg.get("vision_config") or {}
        return cls(image_size=v.get("image_size", 384), vision_dim=v.get("hidden_size", 768),
                   vision_depth=v.get("num_hidden_layers", 12), vision_heads=v.get("num_attention_heads", 12),
                   text_dim=t.get("hidden_size", 768), text_depth=t.get("num_hidden_layers", 12),
                   text_heads=t.get("num_attention_heads", 12), vocab=t.get("vocab_size", 30524),
                   max_pos=t.get("max_position_embeddings", 512), bos_id=t.get("bos_token_id", 30522),
                   sep_id=t.get("sep_token_id", 102), pad_id=t.get("pad_token_id", 0),
                   patch=v.get("patch_size", 16), cross_dim=t.get("encoder_hidden_size"))


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
        self.vision_model = ViT(cfg.image_size, cfg.patch, cfg.vision_dim, cfg.vision_depth, cfg.vision_heads,
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
    def generate(self, image: Image.Image, prefix_ids: list[int], max_new_tokens: int | None = None,
                 max_length: int = 20) -> list[int]:
        """Greedy decode from ``[DEC] + prefix``.  Default length cap: transformers'
        ``generate`` default ``max_length=20`` total tokens, which the reference
        call (swarm/captioning/caption_image.py:29, no length kwargs) runs with."""
        if max_new_tokens is None:
            max_new_tokens = max(0, max_length - 1 - len(prefix_ids))
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


class _TextStack(nn.Module):
    """BERT embeddings + post-LN layers with cross-attention (BlipTextModel)."""

    def __init__(self, cfg: BlipConfig, cross_dim: int):
        super().__init__()
        self.word_embeddings = nn.Embedding(cfg.vocab, cfg.text_dim)
        self.position_embeddings = nn.Embedding(cfg.max_pos, cfg.text_dim)
        self.emb_ln = LayerNorm(cfg.text_dim, eps=1e-12)
        self.layers = nn.ModuleList([PostLNBlock(cfg.text_dim, cfg.text_heads, 4 * cfg.text_dim, cross_dim=cross_dim)
                                     for _ in range(cfg.text_depth)])

    def run(self, ids: list[int], kvs, causal: bool):
        dev = self.word_embeddings.weight.device
        t = torch.tensor([ids], device=dev)
        x = self.emb_ln(self.word_embeddings(t) + self.position_embeddings.weight[: t.shape[1]][None])
        for blk, kv in zip(self.layers, kvs):
            x = blk.ln1(blk.attn(x, residual=x, causal=causal))
            x = blk.ln_x(blk.cross(x, kv=kv, residual=x))
            x = blk.ln2(blk.fc2(blk.fc1(x, act="gelu"), residual=x))
        return x


class BlipVQA(nn.Module):
    """BLIP visual question answering (transformers ``BlipForQuestionAnswering``,
    the VQA branch of swarm/captioning/caption_image.py:21-29): the question is
    encoded by a bidirectional BERT that cross-attends to the image, and the
    answer is decoded greedily from [DEC] by a causal BERT that cross-attends
    to the question encoding."""

    def __init__(self, cfg: BlipConfig = BLIP_BASE):
        super().__init__()
        self.cfg = cfg
        xd = cfg.cross_dim or cfg.vision_dim
        self.vision_model = ViT(cfg.image_size, cfg.patch, cfg.vision_dim, cfg.vision_depth, cfg.vision_heads,
                                4 * cfg.vision_dim)
        self.encoder = _TextStack(cfg, xd)
        self.decoder = _TextStack(cfg, xd)
        self.head_transform = Linear(cfg.text_dim, cfg.text_dim)
        self.head_ln = LayerNorm(cfg.text_dim, eps=1e-12)
        self.head_bias = nn.Parameter(torch.zeros(cfg.vocab))

    preprocess = BlipCaptioner.preprocess

    @torch.no_grad()
    def answer(self, image: Image.Image, question_ids: list[int], max_length: int = 20) -> list[int]:
        """Greedy answer tokens (transformers ``generate`` defaults: at most
        ``max_length`` tokens including [DEC], stop at [SEP]).  ``question_ids``:
        the BERT-tokenised question WITH [CLS] ... [SEP]."""
        dev = self.head_bias.device
        dt = self.encoder.word_embeddings.weight.dtype
        vis = self.vision_model(self.preprocess(image).to(dev).to(dt))
        q = self.encoder.run(list(question_ids), [blk.cross.kv_of(vis) for blk in self.encoder.layers], causal=False)
        kvs = [blk.cross.kv_of(q) for blk in self.decoder.layers]
        ids = [self.cfg.bos_id]
        out = []
        for _ in range(max(0, max_length - 1)):
            x = self.decoder.run(ids, kvs, causal=True)
            h = self.head_ln(self.head_transform(x[:, -1:], act="gelu"))
            logits = h.float() @ self.decoder.word_embeddings.weight.float().t() + self.head_bias.float()
            nxt = int(logits[0, -1].argmax())
            if nxt == self.cfg.sep_id:
                break
            ids.append(nxt)
            out.append(nxt)
        return out
