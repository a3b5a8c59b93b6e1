"""AltDiffusion's text encoder: XLM-RoBERTa + a linear transformation
(diffusers ``RobertaSeriesModelWithTransformation``, the ``text_encoder`` of
``AltDiffusionPipeline`` / ``AltDiffusionImg2ImgPipeline`` — diffusers 0.16.1,
the reference's pin, reaches them by class name like every pipeline class:
swarm/job_arguments.py:143-145, swarm/type_helpers.py:1-3) and its
sentencepiece tokenizer (transformers ``XLMRobertaTokenizer``).

MI355X path: the post-LN RoBERTa blocks run on the MFMA GEMM (packed QKV,
fused bias / GELU / residual epilogues) and the flash attention kernel.  The
tokenizer pads to 77 and the encoder masks the padding keys; here every prompt
runs as its 77 queries against only its real (non-pad) keys — the masked
computation exactly, with no key-padding mask in the attention kernel.

``projection_state`` = transformation(last hidden state), or with
``has_pre_transformation`` (AltDiffusion-m9) transformation_pre(pre_LN(hidden
state of the second-to-last layer)).
"""
from __future__ import annotations

import dataclasses
import hashlib
import os

import torch
import torch.nn as nn

from .. import ops
from .layers import LayerNorm, Linear
from .transformer import PostLNBlock


@dataclasses.dataclass
class XLMRConfig:
    vocab_size: int = 250002
    hidden_size: int = 1024
    num_layers: int = 24
    num_heads: int = 16
    intermediate_size: int = 4096
    max_position: int = 514
    layer_norm_eps: float = 1e-5
    pad_token_id: int = 1
    project_dim: int = 768
    pre_transformation: bool = False
    use_attention_mask: bool = True


XLMR_LARGE = XLMRConfig()  # BAAI/AltDiffusion
TINY_XLMR = XLMRConfig(vocab_size=1000, hidden_size=32, num_layers=2, num_heads=2, intermediate_size=64,
                       max_position=80, project_dim=32)


def xlmr_text_config(cfg: dict, what: str = "text_encoder") -> XLMRConfig:
    """``RobertaSeriesModelWithTransformation`` config.json -> ``XLMRConfig``."""
    from .hf_config import UnsupportedConfig

    if cfg.get("hidden_act", "gelu") != "gelu":
        raise UnsupportedConfig(f"{what}: hidden_act={cfg.get('hidden_act')!r} is not supported")
    if cfg.get("type_vocab_size", 1) != 1:
        raise UnsupportedConfig(f"{what}: type_vocab_size={cfg.get('type_vocab_size')} is not supported")
    return XLMRConfig(vocab_size=cfg.get("vocab_size", 250002), hidden_size=cfg.get("hidden_size", 1024),
                      num_layers=cfg.get("num_hidden_layers", 24), num_heads=cfg.get("num_attention_heads", 16),
                      intermediate_size=cfg.get("intermediate_size", 4096),
                      max_position=cfg.get("max_position_embeddings", 514),
                      layer_norm_eps=cfg.get("layer_norm_eps", 1e-5), pad_token_id=cfg.get("pad_token_id", 1),
                      project_dim=cfg.get("project_dim", 768),
                      pre_transformation=bool(cfg.get("has_pre_transformation", False)),
                      use_attention_mask=bool(cfg.get("use_attention_mask", True)))


def is_xlmr_config(cfg: dict) -> bool:
    return "RobertaSeriesModelWithTransformation" in (cfg.get("architectures") or []) or \
        cfg.get("model_type") in ("roberta", "xlm-roberta")


class XLMRobertaSeries(nn.Module):
    """State dict = diffusers' (roberta.* + transformation.*), through ``hf_renames``."""

    hf_renames = {
        "roberta.embeddings.LayerNorm.": "emb_ln.", "roberta.embeddings.": "", "roberta.encoder.layer.": "layers.",
        ".attention.self.query.": ".attn.q.", ".attention.self.key.": ".attn.k.",
        ".attention.self.value.": ".attn.v.", ".attention.output.dense.": ".attn.o.",
        ".attention.output.LayerNorm.": ".ln1.", ".intermediate.dense.": ".fc1.",
        ".output.dense.": ".fc2.", ".output.LayerNorm.": ".ln2.", "roberta.pooler.dense.": "pooler.",
        "pre_LN.": "pre_ln.",
    }

    def __init__(self, cfg: XLMRConfig = XLMR_LARGE):
        super().__init__()
        self.cfg = cfg
        d = cfg.hidden_size
        self.word_embeddings = nn.Embedding(cfg.vocab_size, d)
        self.position_embeddings = nn.Embedding(cfg.max_position, d)
        self.token_type_embeddings = nn.Embedding(1, d)
        self.emb_ln = LayerNorm(d, eps=cfg.layer_norm_eps)
        self.layers = nn.ModuleList([PostLNBlock(d, cfg.num_heads, cfg.intermediate_size, eps=cfg.layer_norm_eps)
                                     for _ in range(cfg.num_layers)])
        self.pooler = Linear(d, d)  # (in the checkpoint; unused by the pipeline)
        self.transformation = Linear(d, cfg.project_dim)
        if cfg.pre_transformation:
            self.transformation_pre = Linear(d, cfg.project_dim)
            self.pre_ln = LayerNorm(d, eps=cfg.layer_norm_eps)

    def _layer(self, blk: PostLNBlock, x, n):
        """Post-LN block with the keys / values cut to the first ``n`` (real) tokens."""
        a = blk.attn
        a._ensure()
        b, s, _ = x.shape
        qkv = ops.gemm(x, a.w_in, a.b_in).view(b, s, 3, a.heads, a.dh)
        o = ops.attention(qkv[:, :, 0], qkv[:, :n, 1], qkv[:, :n, 2], a.scale)
        x = blk.ln1(a.o(o.reshape(b, s, a.heads * a.dh), residual=x))
        return blk.ln2(blk.fc2(blk.fc1(x, act="gelu"), residual=x))

    def forward(self, ids: torch.Tensor):
        """ids [B, S] (padded with pad_token_id) -> (projection_state [B, S, project_dim],
        None, None, None): the CLIPTextModel tuple layout the SD pipeline reads."""
        cfg = self.cfg
        dt = self.word_embeddings.weight.dtype
        outs = []
        for r in range(ids.shape[0]):
            t = ids[r:r + 1]
            real = t != cfg.pad_token_id
            n = int(real.sum()) if cfg.use_attention_mask else t.shape[1]
            # RoBERTa create_position_ids_from_input_ids: real tokens count from pad + 1, pads sit at pad
            pos = (torch.cumsum(real.int(), 1) * real.int() + cfg.pad_token_id).long()
            x = self.word_embeddings(t) + self.position_embeddings(pos) + self.token_type_embeddings.weight[0]
            x = self.emb_ln(x.to(dt))
            hidden = [x]
            for blk in self.layers:
                x = self._layer(blk, x, max(n, 1))
                hidden.append(x)
            if cfg.pre_transformation:
                outs.append(self.transformation_pre(self.pre_ln(hidden[-2])))
            else:
                outs.append(self.transformation(x))
        return torch.cat(outs, 0), None, None, None


class XLMRTokenizer:
    """transformers ``XLMRobertaTokenizer`` (slow) on the checkpoint's
    ``sentencepiece.bpe.model``: fairseq ids (<s> 0, <pad> 1, </s> 2, <unk> 3,
    sentencepiece ids + 1), ``<s> ... </s>`` truncated and padded to
    ``max_length``.  Hash ids without the model file (random-init runs)."""

    def __init__(self, model_dir: str | None = None, max_length: int = 77, vocab_size: int = 250002):
        self.max_length = max_length
        self.vocab_size = vocab_size
        self.sp = None
        self.source = "hash-fallback"
        self.added_tokens: dict = {}
        f = os.path.join(model_dir, "sentencepiece.bpe.model") if model_dir else None
        if f and os.path.exists(f):
            import sentencepiece as spm

            self.sp = spm.SentencePieceProcessor(model_file=f)
            self.source = model_dir
        self.bos, self.pad, self.eos, self.unk = 0, 1, 2, 3

    @property
    def loaded(self) -> bool:
        return self.sp is not None

    def encode(self, text: str) -> list[int]:
        if self.sp is None:
            return [int.from_bytes(hashlib.blake2b(w.encode(), digest_size=8).digest(), "little")
                    % (self.vocab_size - 5) + 4 for w in text.split()]
        out = []
        for piece in self.sp.encode(text, out_type=str):
            i = self.sp.piece_to_id(piece)
            out.append(i + 1 if i else self.unk)
        return out

    def __call__(self, texts) -> torch.Tensor:
        if isinstance(texts, str):
            texts = [texts]
        rows = []
        for t in texts:
            ids = [self.bos] + self.encode(t)[: self.max_length - 2] + [self.eos]
            rows.append(ids + [self.pad] * (self.max_length - len(ids)))
        return torch.tensor(rows, dtype=torch.long)
