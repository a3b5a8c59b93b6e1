"""BLIP-2 / InstructBLIP image captioning / prompted VQA (OPT, Flan-T5 or Vicuna-LLaMA language models)
(transformers ``Blip2ForConditionalGeneration`` + ``Blip2Processor``, the
``Salesforce/blip2-opt-*`` and ``blip2-flan-t5-*`` checkpoints).  Reference: the hive names the
processor / model classes at swarm/captioning/caption_image.py:11-29 and the
reference instantiates whatever transformers class it is given.

Three stages, all on the shared kernels (fused-QKV GEMMs, flash attention,
LayerNorm, GEMM epilogues):

* vision: ViT (post-LN on every token; EVA ViT-g/14 geometry by default,
  q/v biases with a zero k bias);
* Q-Former: 32 learned query tokens through a BERT-style post-LN stack that
  cross-attends to the image tokens every ``cross_attention_frequency``
  layers (query FFN only: captioning feeds no text to the Q-Former);
* language model, either
  - OPT (``blip2-opt-*``): pre-LN decoder, ReLU MLP, learned positions with
    offset 2, LM head tied to the token embeddings, over
    ``[projected queries; </s>; prompt]``; or
  - Flan-T5 (``blip2-flan-t5-*``, ``models/t5.py::T5Seq2Seq``): the encoder
    reads ``[projected queries; prompt; </s>]``, the decoder generates from the
    decoder start token (pad, 0) with cross-attention over it;
  - Vicuna / LLaMA (``instructblip-vicuna-*``, ``models/llama.py``) after
    ``[projected queries; <s> prompt]``.
* InstructBLIP (``InstructBlipForConditionalGeneration``): the instruction, in
  the Q-Former's own WordPiece tokens, joins the 32 queries in the Q-Former's
  self-attention (the instruction rows take the text FFN).

Greedy decode with transformers' default ``max_length=20`` (OPT: counted on the
text part, ``</s>`` + prompt + generated; T5: decoder tokens), stopping at the
eos token.  Every step re-runs the (short) decoder sequence: at that size each
GEMM streams its weights once either way, so a KV cache would save no HBM
traffic.  The original-T5 (ReLU FFN) language models are refused.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch
import torch.nn as nn
from PIL import Image

from .layers import LayerNorm, Linear
from .llama import LlamaConfig, LlamaLM
from .t5 import T5Config, T5Seq2Seq
from .transformer import PostLNBlock, PreLNBlock, ViT

MEAN = np.array([0.48145466, 0.4578275, 0.40821073], np.float32)
STD = np.array([0.26862954, 0.26130258, 0.27577711], np.float32)


@dataclasses.dataclass
class Blip2Config:
    image_size: int = 224
    patch: int = 14
    vision_dim: int = 1408
    vision_depth: int = 39
    vision_heads: int = 16
    vision_mlp: int = 6144
    vision_eps: float = 1e-6
    q_dim: int = 768
    q_depth: int = 12
    q_heads: int = 12
    q_mlp: int = 3072
    q_eps: float = 1e-12
    cross_freq: int = 2
    num_query: int = 32
    lm_dim: int = 2560
    lm_depth: int = 32
    lm_heads: int = 32
    lm_ffn: int = 10240
    lm_eps: float = 1e-5
    vocab: int = 50272
    max_pos: int = 2048
    bos_id: int = 2
    eos_id: int = 2
    pad_id: int = 1
    lm_type: str = "opt"
    t5: T5Config | None = None  # lm_type "t5": the Flan-T5 geometry (lm_dim = t5.d_model)
    t5_dec_layers: int = 0
    t5_tied: bool = False
    llama: LlamaConfig | None = None  # lm_type "llama" (InstructBLIP's Vicuna)
    instruct: bool = False  # InstructBLIP: the Q-Former also reads the instruction text
    q_vocab: int = 30522
    q_max_pos: int = 512
    q_cls_id: int = 101  # the Q-Former tokenizer's [CLS] / [SEP] (bert-base-uncased)
    q_sep_id: int = 102

    @classmethod
    def from_hf(cls, cfg: dict) -> "Blip2Config":
        """A transformers ``Blip2Config`` config.json (vision / qformer / text
        sub-configs; the text model is OPT or (Flan-)T5 v1.1)."""
        v, q, t = cfg.get("vision_config") or {}, cfg.get("qformer_config") or {}, cfg.get("text_config") or {}
        lm = t.get("model_type", "opt")
        instruct = cfg.get("model_type") == "instructblip" or bool(q.get("vocab_size") and "instructblip" in
                                                                     str(cfg.get("architectures", "")).lower())
        if lm == "llama" and instruct:
            base = cls._vision_qformer(cfg, v, q)
            lc = LlamaConfig.from_hf(t)
            return dataclasses.replace(base, lm_type="llama", llama=lc, lm_dim=lc.dim, vocab=lc.vocab,
                                       bos_id=lc.bos_id, eos_id=lc.eos_id, pad_id=t.get("pad_token_id") or 0)
        if lm not in ("opt", "t5"):
            raise ValueError(f"img2txt: BLIP-2 with a {lm!r} language model is not supported (OPT, Flan-T5)")
        if lm == "t5":
            proj = t.get("feed_forward_proj", "relu")
            if "gated" not in proj:
                raise ValueError(f"img2txt: BLIP-2 t5 language model with feed_forward_proj={proj!r} is not supported "
                                 "(gated-gelu: T5 v1.1 / Flan-T5)")
            t5 = T5Config(vocab=t.get("vocab_size", 32128), d_model=t.get("d_model", 2048), d_kv=t.get("d_kv", 64),
                          heads=t.get("num_heads", 32), d_ff=t.get("d_ff", 5120), layers=t.get("num_layers", 24),
                          buckets=t.get("relative_attention_num_buckets", 32),
                          max_distance=t.get("relative_attention_max_distance", 128),
                          eps=t.get("layer_norm_epsilon", 1e-6))
            base = cls._vision_qformer(cfg, v, q)
            return dataclasses.replace(base, lm_type="t5", t5=t5, lm_dim=t5.d_model, vocab=t5.vocab,
                                       t5_dec_layers=t.get("num_decoder_layers") or t5.layers,
                                       # original T5 scales the decoder output by d_model^-0.5 before
                                       # the (tied) head; v1.1 / Flan-T5 configs say
                                       # tie_word_embeddings=false (newer transformers:
                                       # scale_decoder_outputs)
                                       t5_tied=bool(t.get("scale_decoder_outputs",
                                                          t.get("tie_word_embeddings", True) is not False)),
                                       bos_id=t.get("decoder_start_token_id", 0), eos_id=t.get("eos_token_id", 1),
                                       pad_id=t.get("pad_token_id", 0))
        if t.get("word_embed_proj_dim", t.get("hidden_size", 2560)) != t.get("hidden_size", 2560):
            raise ValueError("img2txt: OPT with word_embed_proj_dim != hidden_size is not supported")
        return dataclasses.replace(
            cls._vision_qformer(cfg, v, q), lm_dim=t.get("hidden_size", 2560), lm_depth=t.get("num_hidden_layers", 32),
            lm_heads=t.get("num_attention_heads", 32), lm_ffn=t.get("ffn_dim", 10240),
            vocab=t.get("vocab_size", 50272), max_pos=t.get("max_position_embeddings", 2048),
            bos_id=t.get("bos_token_id", 2), eos_id=t.get("eos_token_id", 2), pad_id=t.get("pad_token_id", 1))

    @classmethod
    def _vision_qformer(cls, cfg, v, q) -> "Blip2Config":
        instruct = cfg.get("model_type") == "instructblip" or "instructblip" in str(cfg.get("architectures", "")).lower()
        return cls(instruct=instruct, q_vocab=q.get("vocab_size", 30522), q_max_pos=q.get("max_position_embeddings", 512),
                   image_size=v.get("image_size", 224), patch=v.get("patch_size", 14),
                   vision_dim=v.get("hidden_size", 1408), vision_depth=v.get("num_hidden_layers", 39),
                   vision_heads=v.get("num_attention_heads", 16), vision_mlp=v.get("intermediate_size", 6144),
                   vision_eps=v.get("layer_norm_eps", 1e-6), q_dim=q.get("hidden_size", 768),
                   q_depth=q.get("num_hidden_layers", 12), q_heads=q.get("num_attention_heads", 12),
                   q_mlp=q.get("intermediate_size", 3072), q_eps=q.get("layer_norm_eps", 1e-12),
                   cross_freq=q.get("cross_attention_frequency", 2), num_query=cfg.get("num_query_tokens", 32))


BLIP2_OPT_2_7B = Blip2Config()
BLIP2_OPT_6_7B = Blip2Config(lm_dim=4096, lm_ffn=16384)
_FLAN_T5_XL = T5Config(d_model=2048, d_kv=64, heads=32, d_ff=5120, layers=24)
BLIP2_FLAN_T5_XL = Blip2Config(lm_type="t5", t5=_FLAN_T5_XL, lm_dim=2048, vocab=32128, t5_dec_layers=24,
                               bos_id=0, eos_id=1, pad_id=0)
TINY_BLIP2 = Blip2Config(image_size=28, patch=14, vision_dim=32, vision_depth=2, vision_heads=2, vision_mlp=64,
                         q_dim=32, q_depth=2, q_heads=2, q_mlp=64, num_query=4, lm_dim=32, lm_depth=2, lm_heads=2,
                         lm_ffn=64, vocab=100, max_pos=64)

_Q = {"attention.attention.query": "attn.q", "attention.attention.key": "attn.k",
      "attention.attention.value": "attn.v", "attention.output.dense": "attn.o", "attention.output.LayerNorm": "ln1",
      "crossattention.attention.query": "cross.q", "crossattention.attention.key": "cross.k",
      "crossattention.attention.value": "cross.v", "crossattention.output.dense": "cross.o",
      "crossattention.output.LayerNorm": "ln_x", "intermediate_query.dense": "fc1", "output_query.dense": "fc2",
      "output_query.LayerNorm": "ln2"}
_V = {"self_attn.projection": "attn.o", "layer_norm1": "ln1", "layer_norm2": "ln2", "mlp.fc1": "fc1",
      "mlp.fc2": "fc2"}
_LM = {"self_attn.q_proj": "attn.q", "self_attn.k_proj": "attn.k", "self_attn.v_proj": "attn.v",
       "self_attn.out_proj": "attn.o", "self_attn_layer_norm": "ln1", "final_layer_norm": "ln2", "fc1": "fc1",
       "fc2": "fc2"}


def _sub(rest: str, table: dict) -> str | None:
    for a, b in table.items():
        if rest.startswith(a + "."):
            return b + rest[len(a):]
    return None


def convert_hf_blip2(sd: dict, instruct: bool | None = None) -> dict:
    """transformers ``Blip2ForConditionalGeneration`` (OPT) state dict -> this
    module's keys.  Vision attention biases come either as the fused
    ``qkv.bias`` or as the original checkpoints' ``q_bias`` / ``v_bias`` (k bias
    zero); the Q-Former's text FFN (``intermediate.`` / ``output.``, unused
    without Q-Former text input) is dropped; the LM head is tied."""
    out: dict = {}
    if instruct is None:  # InstructBLIP: the Q-Former has its own text embeddings
        instruct = "qformer.embeddings.word_embeddings.weight" in sd
    llama = "language_model.model.embed_tokens.weight" in sd
    for k, v in sd.items():
        if k.endswith("position_ids"):
            continue
        if k == "language_model.lm_head.weight":
            if "language_model.shared.weight" in sd:  # T5: own (or tied-and-saved) head
                out["t5.lm_head.weight"] = v
            elif llama:
                out["llama.lm_head.weight"] = v
            continue  # OPT: tied to the token embeddings
        if k == "query_tokens":
            out[k] = v.reshape(v.shape[-2], v.shape[-1])
        elif k.startswith("vision_model.embeddings."):
            r = k.removeprefix("vision_model.embeddings.")
            if r == "class_embedding":
                v = v.reshape(-1)
            elif r == "position_embedding":
                v = v.reshape(v.shape[-2], v.shape[-1])
            out["vision_model." + r] = v
        elif k.startswith("vision_model.post_layernorm."):
            out["vision_model.post_ln." + k.rsplit(".", 1)[1]] = v
        elif k.startswith("vision_model.encoder.layers."):
            n, rest = k.removeprefix("vision_model.encoder.layers.").split(".", 1)
            pre = f"vision_model.layers.{n}.attn."
            if rest == "self_attn.qkv.weight" or rest == "self_attn.qkv.bias":
                for name, part in zip("qkv", v.chunk(3, 0)):
                    out[pre + f"{name}." + rest.rsplit(".", 1)[1]] = part.contiguous()
            elif rest == "self_attn.q_bias":
                out[pre + "q.bias"] = v
                out.setdefault(pre + "k.bias", torch.zeros_like(v))
            elif rest == "self_attn.v_bias":
                out[pre + "v.bias"] = v
            else:
                s = _sub(rest, _V)
                out[f"vision_model.layers.{n}.{s}" if s else k] = v
        elif k.startswith("qformer.layernorm.") or k.startswith("qformer.embeddings.layernorm."):
            out["qformer_ln." + k.rsplit(".", 1)[1]] = v
        elif k == "qformer.embeddings.word_embeddings.weight" and instruct:
            out["q_word.weight"] = v
        elif k == "qformer.embeddings.position_embeddings.weight" and instruct:
            out["q_pos.weight"] = v
        elif k.startswith("qformer.encoder.layer."):
            n, rest = k.removeprefix("qformer.encoder.layer.").split(".", 1)
            if rest.startswith(("intermediate.", "output.")):
                if instruct:  # the instruction tokens' FFN (InstructBLIP)
                    t = {"intermediate.dense": "fc1", "output.dense": "fc2", "output.LayerNorm": "ln"}
                    s = _sub(rest, t)
                    out[f"qtext.{n}.{s}" if s else k] = v
                continue
            s = _sub(rest, _Q)
            out[f"qformer.{n}.{s}" if s else k] = v
        elif k.startswith("language_model.model.") and not k.startswith("language_model.model.decoder.") and \
                "language_model.model.embed_tokens.weight" in sd:  # LLaMA (InstructBLIP Vicuna)
            out["llama." + k.removeprefix("language_model.")] = v
        elif k.startswith("language_projection."):
            out[k] = v
        elif k.startswith("language_model.") and not k.startswith("language_model.model.") and \
                not k.startswith("language_model.lm_head"):
            r = k.removeprefix("language_model.")
            if not r.endswith("embed_tokens.weight"):
                out["t5." + r] = v  # T5ForConditionalGeneration names (models/t5.py::T5Seq2Seq)
        elif k.startswith("language_model.model.decoder."):
            r = k.removeprefix("language_model.model.decoder.")
            if r.startswith("layers."):
                n, rest = r.removeprefix("layers.").split(".", 1)
                s = _sub(rest, _LM)
                out[f"lm.{n}.{s}" if s else k] = v
            elif r.startswith("final_layer_norm."):
                out["lm_ln." + r.rsplit(".", 1)[1]] = v
            elif r == "embed_tokens.weight":
                out["embed_tokens.weight"] = v
            elif r == "embed_positions.weight":
                out["embed_positions.weight"] = v
            else:
                out[k] = v
        else:
            out[k] = v  # unknown keys surface as a CheckpointMismatch in load_into
    if "language_model.shared.weight" in sd and "t5.lm_head.weight" not in out:
        out["t5.lm_head.weight"] = sd["language_model.shared.weight"]  # tied head not saved
    return out


class Blip2Captioner(nn.Module):
    def __init__(self, cfg: Blip2Config = BLIP2_OPT_2_7B):
        super().__init__()
        self.cfg = cfg
        self.vision_model = ViT(cfg.image_size, cfg.patch, cfg.vision_dim, cfg.vision_depth, cfg.vision_heads,
                                cfg.vision_mlp, eps=cfg.vision_eps)
        self.query_tokens = nn.Parameter(torch.zeros(cfg.num_query, cfg.q_dim))
        self.qformer_ln = LayerNorm(cfg.q_dim, eps=cfg.q_eps)
        self.qformer = nn.ModuleList([
            PostLNBlock(cfg.q_dim, cfg.q_heads, cfg.q_mlp, cross_dim=cfg.vision_dim if i % cfg.cross_freq == 0 else None,
                        eps=cfg.q_eps) for i in range(cfg.q_depth)])
        if cfg.instruct:  # InstructBLIP: instruction tokens enter the Q-Former too
            self.q_word = nn.Embedding(cfg.q_vocab, cfg.q_dim)
            self.q_pos = nn.Embedding(cfg.q_max_pos, cfg.q_dim)
            self.qtext = nn.ModuleList([_TextFFN(cfg) for _ in range(cfg.q_depth)])
        self.language_projection = Linear(cfg.q_dim, cfg.lm_dim)
        if cfg.lm_type == "llama":
            self.llama = LlamaLM(cfg.llama)
            return
        if cfg.lm_type == "t5":
            self.t5 = T5Seq2Seq(cfg.t5, cfg.t5_dec_layers or cfg.t5.layers, tie_embeddings=cfg.t5_tied)
            return
        self.embed_tokens = nn.Embedding(cfg.vocab, cfg.lm_dim)
        self.embed_positions = nn.Embedding(cfg.max_pos + 2, cfg.lm_dim)
        self.lm = nn.ModuleList([PreLNBlock(cfg.lm_dim, cfg.lm_heads, cfg.lm_ffn, act="relu", eps=cfg.lm_eps)
                                 for _ in range(cfg.lm_depth)])
        self.lm_ln = LayerNorm(cfg.lm_dim, eps=cfg.lm_eps)

    @property
    def _emb(self) -> nn.Embedding:
        if self.cfg.lm_type == "llama":
            return self.llama.model.embed_tokens
        return self.t5.shared if self.cfg.lm_type == "t5" else self.embed_tokens

    def preprocess(self, image: Image.Image) -> torch.Tensor:
        """BlipImageProcessor: bicubic resize to image_size², CLIP mean / std; NHWC."""
        s = self.cfg.image_size
        a = np.asarray(image.convert("RGB").resize((s, s), Image.Resampling.BICUBIC), np.float32) / 255.0
        return torch.from_numpy((a - MEAN) / STD)[None]

    @torch.no_grad()
    def image_prefix(self, pixels: torch.Tensor, qtext_ids: list[int] | None = None) -> torch.Tensor:
        """Projected Q-Former query outputs [1, num_query, lm_dim]: the language
        model's input embeddings ahead of the text.  InstructBLIP: the
        instruction's Q-Former tokens ([CLS] ... [SEP]) follow the queries through
        the self-attention (cross-attention and the query FFN on the query rows,
        the text FFN on the instruction rows)."""
        dt = self._emb.weight.dtype
        img = self.vision_model(pixels.to(dt))
        q = self.query_tokens[None].to(dt)
        if not self.cfg.instruct:
            q = self.qformer_ln(q)
            for blk in self.qformer:
                q = blk(q, ctx=img)
            return self.language_projection(q)
        ids = torch.tensor([list(qtext_ids or [])], device=q.device, dtype=torch.long)
        t = self.q_word(ids).to(dt) + self.q_pos.weight[: ids.shape[1]][None].to(dt)
        h = self.qformer_ln(torch.cat([q, t], 1))
        nq = q.shape[1]
        for blk, tf in zip(self.qformer, self.qtext):
            h = blk.ln1(blk.attn(h, residual=h))
            qp, tp = h[:, :nq], h[:, nq:]
            if blk.cross is not None:
                qp = blk.ln_x(blk.cross(qp, ctx=img, residual=qp))
            qp = blk.ln2(blk.fc2(blk.fc1(qp, act="gelu"), residual=qp))
            if tp.shape[1]:
                tp = tf.ln(tf.fc2(tf.fc1(tp, act="gelu"), residual=tp))
            h = torch.cat([qp, tp], 1)
        return self.language_projection(h[:, :nq])

    @torch.no_grad()
    def text_logits(self, prefix: torch.Tensor, ids: list[int]) -> torch.Tensor:
        """Next-token logits [vocab] for [prefix embeddings; embed(ids)]."""
        dev = self.embed_tokens.weight.device
        t = torch.tensor([ids], device=dev)
        x = torch.cat([prefix, self.embed_tokens(t)], 1)
        x = x + self.embed_positions.weight[2: 2 + x.shape[1]][None]
        for blk in self.lm:
            x = blk(x, causal=True)
        h = self.lm_ln(x[:, -1:])
        return (h.float() @ self.embed_tokens.weight.float().t())[0, -1]

    @torch.no_grad()
    def generate(self, image: Image.Image, prefix_ids: list[int], max_new_tokens: int | None = None,
                 max_length: int = 20, qtext_ids: list[int] | None = None) -> list[int]:
        """Greedy decode from ``</s> + prefix`` after the image queries; returns
        prefix + generated ids (without the leading ``</s>``)."""
        if self.cfg.lm_type == "t5":
            return self._generate_t5(image, prefix_ids, max_new_tokens, max_length, qtext_ids)
        if self.cfg.lm_type == "llama":
            return self._generate_llama(image, prefix_ids, max_new_tokens, max_length, qtext_ids)
        if max_new_tokens is None:
            max_new_tokens = max(0, max_length - 1 - len(prefix_ids))
        prefix = self.image_prefix(self.preprocess(image).to(self.embed_tokens.weight.device))
        ids = [self.cfg.bos_id] + list(prefix_ids)
        out = []
        for _ in range(max_new_tokens):
            nxt = int(self.text_logits(prefix, ids).argmax())
            if nxt == self.cfg.eos_id:
                break
            ids.append(nxt)
            out.append(nxt)
        return list(prefix_ids) + out

    @torch.no_grad()
    def t5_encoder_states(self, prefix: torch.Tensor, prompt_ids: list[int]) -> torch.Tensor:
        """Flan-T5 encoder over [projected queries; prompt; </s>]."""
        t5 = self.t5
        ids = torch.tensor([list(prompt_ids) + [self.cfg.eos_id]], device=prefix.device)
        return t5.encode(torch.cat([prefix, t5.shared(ids).to(prefix.dtype)], 1))

    def _generate_t5(self, image, prompt_ids, max_new_tokens, max_length, qtext_ids=None) -> list[int]:
        """Greedy decode from the decoder start token; returns the generated ids
        (the prompt lives in the encoder)."""
        if max_new_tokens is None:
            max_new_tokens = max(0, max_length - 1)
        prefix = self.image_prefix(self.preprocess(image).to(self.t5.shared.weight.device), qtext_ids)
        enc = self.t5_encoder_states(prefix, prompt_ids)
        ids = [self.cfg.bos_id]
        for _ in range(max_new_tokens):
            nxt = int(self.t5.decode_logits(enc, ids).argmax())
            if nxt == self.cfg.eos_id:
                break
            ids.append(nxt)
        return ids[1:]

    def _generate_llama(self, image, prompt_ids, max_new_tokens, max_length, qtext_ids=None) -> list[int]:
        """InstructBLIP (Vicuna): greedy decode after [queries; <s> prompt];
        returns the generated ids."""
        if max_new_tokens is None:
            max_new_tokens = max(0, max_length - 1)
        emb = self.llama.model.embed_tokens
        prefix = self.image_prefix(self.preprocess(image).to(emb.weight.device), qtext_ids)
        ids = [self.cfg.bos_id] + list(prompt_ids)
        out = []
        for _ in range(max_new_tokens):
            x = torch.cat([prefix, emb(torch.tensor([ids], device=prefix.device)).to(prefix.dtype)], 1)
            nxt = int(self.llama.last_logits(x).argmax())
            if nxt == self.cfg.eos_id:
                break
            ids.append(nxt)
            out.append(nxt)
        return out


class _TextFFN(nn.Module):
    """InstructBLIP Q-Former FFN of the instruction tokens (post-LN)."""

    def __init__(self, cfg: Blip2Config):
        super().__init__()
        self.fc1 = Linear(cfg.q_dim, cfg.q_mlp)
        self.fc2 = Linear(cfg.q_mlp, cfg.q_dim)
        self.ln = LayerNorm(cfg.q_dim, eps=cfg.q_eps)
