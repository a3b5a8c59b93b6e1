"""Bark text-to-speech (suno/bark): three GPT stages + the EnCodec 24 kHz
decoder (reference: swarm/audio/bark.py:11-39, which calls the ``bark``
package's ``generate_audio``).

Stages (geometry and token conventions of the public Bark release):
  1. semantic GPT (causal): BERT-cased text ids (+10048 offset, 256 slots)
     summed with a 256-slot semantic history, then autoregressive sampling of
     ~50 Hz semantic tokens (temperature 0.7, early stop on the EOS logit);
  2. coarse GPT (causal): semantic -> 2 interleaved EnCodec codebooks at 75 Hz,
     generated in sliding windows of 60 tokens over a 630-token history;
  3. fine GPT (non-causal): completes codebooks 2..7 in 1024-frame windows;
  4. EnCodec decoder: codebook embeddings -> causal SEANet decoder (weight-norm
     folded at load, reflect padding, ELU, 2-layer LSTM) -> 24 kHz waveform.

MI355X path: all GPT projections are the MFMA GEMM with fused bias/GELU/
residual epilogues; prefill and KV-cached decode both run the flash-attention
kernel on strided views of a preallocated per-layer KV cache (no concatenation
per token); decoder convs are the implicit-GEMM conv kernel with ELU fused
into the epilogue and transposed convs in polyphase form.  The LSTM runs in
fp32 through torch (MIOpen RNN).
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .layers import Conv1d, ConvTranspose1d, LayerNorm, Linear, init_random_fast_, prepare_model
from ..utils import stable_seed

# token conventions (Bark generation constants)
CONTEXT_WINDOW = 1024
SEMANTIC_RATE_HZ = 49.9
SEMANTIC_VOCAB = 10_000
CODEBOOK_SIZE = 1024
N_COARSE = 2
N_FINE = 8
COARSE_RATE_HZ = 75
SAMPLE_RATE = 24_000
TEXT_OFFSET = 10_048
SEMANTIC_PAD = 10_000
TEXT_PAD = 129_595
SEMANTIC_INFER = 129_599
COARSE_SEMANTIC_PAD = 12_048
COARSE_INFER = 12_050


@dataclasses.dataclass
class GPTConfig:
    in_vocab: int
    out_vocab: int
    n_layer: int = 24
    n_head: int = 16
    n_embd: int = 1024
    block_size: int = 1024
    bias: bool = False
    causal: bool = True
    n_codes_total: int = 8  # fine model only
    n_codes_given: int = 1


def bark_configs_from_hf(raw: dict):
    """GPT + EnCodec geometry from a transformers ``BarkConfig`` dict
    (``semantic_config`` / ``coarse_acoustics_config`` / ``fine_acoustics_config``
    / ``codec_config``) — the config.json beside suno/bark's safetensors."""
    def gpt(c, causal=True):
        g = GPTConfig(int(c["input_vocab_size"]), int(c["output_vocab_size"]), int(c["num_layers"]),
                      int(c["num_heads"]), int(c["hidden_size"]), int(c["block_size"]), bool(c.get("bias", False)),
                      causal)
        if not causal:
            g.n_codes_total, g.n_codes_given = int(c.get("n_codes_total", 8)), int(c.get("n_codes_given", 1))
        return g

    cc = raw.get("codec_config") or {}
    fine = gpt(raw["fine_acoustics_config"], causal=False)
    codec = EncodecConfig(dim=int(cc.get("hidden_size", 128)), n_filters=int(cc.get("num_filters", 32)),
                          ratios=tuple(cc.get("upsampling_ratios", (8, 5, 4, 2))), n_q=fine.n_codes_total,
                          bins=int(cc.get("codebook_size", 1024)), lstm_layers=int(cc.get("num_lstm_layers", 2)),
                          compress=int(cc.get("compress", 2)), kernel=int(cc.get("kernel_size", 7)),
                          residual_kernel=int(cc.get("residual_kernel_size", 3)),
                          last_kernel=int(cc.get("last_kernel_size", 7)))
    unsupported = [k for k, ok in (("num_residual_layers", cc.get("num_residual_layers", 1) == 1),
                                   ("use_causal_conv", cc.get("use_causal_conv", True)),
                                   ("pad_mode", cc.get("pad_mode", "reflect") == "reflect"),
                                   ("use_conv_shortcut", cc.get("use_conv_shortcut", True)),
                                   ("audio_channels", cc.get("audio_channels", 1) == 1)) if not ok]
    if unsupported:
        from .hf_config import UnsupportedConfig

        raise UnsupportedConfig(f"bark codec_config: unsupported {', '.join(unsupported)}")
    return gpt(raw["semantic_config"]), gpt(raw["coarse_acoustics_config"]), fine, codec


def bark_configs(size: str = "large"):
    dims = {"large": (24, 16, 1024), "small": (12, 12, 768), "tiny": (2, 2, 64)}[size]
    ln, nh, ne = dims
    blk = 1024 if size != "tiny" else 1200
    return (GPTConfig(129_600, 10_048, ln, nh, ne, blk),
            GPTConfig(12_096, 12_096, ln, nh, ne, blk),
            GPTConfig(1056, 1056, ln, nh, ne, blk, causal=False))


class _Attn(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        self.nh, self.dh = c.n_head, c.n_embd // c.n_head
        self.att_proj = Linear(c.n_embd, 3 * c.n_embd, bias=c.bias)
        self.out_proj = Linear(c.n_embd, c.n_embd, bias=c.bias)

    def decode(self, x, residual, cache, pos_t, len_t):
        """One-token step with device-side position / length (graph-capturable)."""
        b = x.shape[0]
        qkv = self.att_proj(x).view(b, 1, 3, self.nh, self.dh)
        kc, vc = cache
        kc.index_copy_(1, pos_t, qkv[:, :, 1])
        vc.index_copy_(1, pos_t, qkv[:, :, 2])
        o = ops.attention(qkv[:, :, 0], kc, vc, 1.0 / math.sqrt(self.dh), kv_len=len_t)
        return self.out_proj(o.reshape(b, 1, -1), residual=residual)

    def forward(self, x, residual, causal, cache=None, pos=0):
        b, s, _ = x.shape
        qkv = self.att_proj(x).view(b, s, 3, self.nh, self.dh)
        q = qkv[:, :, 0]
        if cache is not None:
            kc, vc = cache  # [B, block, H, D]
            kc[:, pos:pos + s].copy_(qkv[:, :, 1])
            vc[:, pos:pos + s].copy_(qkv[:, :, 2])
            k, v = kc[:, :pos + s], vc[:, :pos + s]
            # with a cache, new queries see every cached key (causal within the new block only)
            causal = causal and s > 1
        else:
            k, v = qkv[:, :, 1], qkv[:, :, 2]
        o = ops.attention(q, k, v, 1.0 / math.sqrt(self.dh), causal=causal)
        return self.out_proj(o.reshape(b, s, -1), residual=residual)


class _Block(nn.Module):
    def __init__(self, c: GPTConfig):
        super().__init__()
        ln_bias = c.bias or not c.causal  # the fine (non-causal) model always has LayerNorm biases
        self.layernorm_1 = LayerNorm(c.n_embd, elementwise_affine=True, bias=ln_bias)
        self.attn = _Attn(c)
        self.layernorm_2 = LayerNorm(c.n_embd, elementwise_affine=True, bias=ln_bias)
        self.mlp = nn.Module()
        self.mlp.in_proj = Linear(c.n_embd, 4 * c.n_embd, bias=c.bias)
        self.mlp.out_proj = Linear(4 * c.n_embd, c.n_embd, bias=c.bias)

    def forward(self, x, causal, cache=None, pos=0):
        x = self.attn(self.layernorm_1(x), x, causal, cache, pos)
        return self.mlp.out_proj(self.mlp.in_proj(self.layernorm_2(x), act="gelu"), residual=x)

    def decode(self, x, cache, pos_t, len_t):
        x = self.attn.decode(self.layernorm_1(x), x, cache, pos_t, len_t)
        return self.mlp.out_proj(self.mlp.in_proj(self.layernorm_2(x), act="gelu"), residual=x)


class BarkCausalGPT(nn.Module):
    """Semantic / coarse GPT (HF ``BarkCausalModel`` parameter names)."""

    def __init__(self, c: GPTConfig):
        super().__init__()
        self.cfg = c
        self.input_embeds_layer = nn.Embedding(c.in_vocab, c.n_embd)
        self.position_embeds_layer = nn.Embedding(c.block_size, c.n_embd)
        self.layers = nn.ModuleList([_Block(c) for _ in range(c.n_layer)])
        self.layernorm_final = LayerNorm(c.n_embd, bias=c.bias)
        self.lm_head = Linear(c.n_embd, c.out_vocab, bias=False)
        self.cache = None

    def new_cache(self, batch=1):
        """(Re)use the persistent per-layer KV buffers (allocated once, so a
        captured decode graph stays valid across generations)."""
        c = self.cfg
        p = self.lm_head.weight
        shape = (batch, c.block_size, c.n_head, c.n_embd // c.n_head)
        kv = getattr(self, "_kv", None)
        if kv is None or kv[0][0].shape != shape or kv[0][0].device != p.device or kv[0][0].dtype != p.dtype:
            self._kv = [(torch.empty(shape, device=p.device, dtype=p.dtype),
                         torch.empty(shape, device=p.device, dtype=p.dtype)) for _ in range(c.n_layer)]
            self._graph = None
        self.cache = self._kv

    @torch.no_grad()
    def _decode_fn(self, ids, pos_t, len_t):
        x = self.input_embeds_layer(ids) + self.position_embeds_layer.weight.index_select(0, pos_t)[None]
        x = x.to(self.lm_head.weight.dtype)
        for i, layer in enumerate(self.layers):
            x = layer.decode(x, self.cache[i], pos_t, len_t)
        return self.lm_head(self.layernorm_final(x[:, -1])).float()

    @torch.no_grad()
    def decode_step(self, token: int, pos: int):
        """Logits after appending ``token`` at position ``pos`` of the KV cache.
        On the GPU the whole step (every layer) replays from one hipGraph."""
        dev = self.lm_head.weight.device
        st = getattr(self, "_dstate", None)
        if st is None or st[0].device != dev:
            st = (torch.zeros(1, 1, dtype=torch.long, device=dev), torch.zeros(1, dtype=torch.long, device=dev),
                  torch.zeros(1, dtype=torch.int32, device=dev))
            self._dstate = st
        ids, pos_t, len_t = st
        ids.fill_(int(token))
        pos_t.fill_(int(pos))
        len_t.fill_(int(pos) + 1)
        from ..pipelines.graphs import CapturedCall, graphs_enabled

        if not graphs_enabled(dev):
            return self._decode_fn(ids, pos_t, len_t)
        g = getattr(self, "_graph", None)
        if g is None:
            g = CapturedCall(self._decode_fn, ids=ids, pos_t=pos_t, len_t=len_t)
            self._graph = g
        return g.run(ids=ids, pos_t=pos_t, len_t=len_t)

    @torch.no_grad()
    def forward(self, ids=None, embeds=None, pos=0, last_only=True):
        """ids [B, S] (or precomputed embeds [B, S, C]); with a cache, ``pos`` is
        the number of tokens already cached.  Returns fp32 logits of the last
        position [B, out_vocab] (or all positions)."""
        x = self.input_embeds_layer(ids) if embeds is None else embeds
        s = x.shape[1]
        x = x + self.position_embeds_layer.weight[pos:pos + s]
        x = x.to(self.lm_head.weight.dtype)
        for i, layer in enumerate(self.layers):
            x = layer(x, self.cfg.causal, self.cache[i] if self.cache is not None else None, pos)
        if last_only:
            x = x[:, -1]
        return self.lm_head(self.layernorm_final(x)).float()


class BarkFineGPT(nn.Module):
    """Non-causal fine model (HF ``BarkFineModel`` names)."""

    def __init__(self, c: GPTConfig):
        super().__init__()
        self.cfg = c
        self.input_embeds_layers = nn.ModuleList([nn.Embedding(c.in_vocab, c.n_embd) for _ in range(c.n_codes_total)])
        self.position_embeds_layer = nn.Embedding(c.block_size, c.n_embd)
        self.layers = nn.ModuleList([_Block(c) for _ in range(c.n_layer)])
        self.layernorm_final = LayerNorm(c.n_embd, bias=True)
        self.lm_heads = nn.ModuleList([Linear(c.n_embd, c.out_vocab, bias=False)
                                       for _ in range(c.n_codes_given, c.n_codes_total)])

    @torch.no_grad()
    def forward(self, pred_idx: int, codes: torch.Tensor):
        """codes [B, T, 8] -> logits [B, T, out_vocab] for codebook ``pred_idx``."""
        t = codes.shape[1]
        x = sum(self.input_embeds_layers[i](codes[:, :, i]) for i in range(pred_idx + 1))
        x = (x + self.position_embeds_layer.weight[:t]).to(self.lm_heads[0].weight.dtype)
        for layer in self.layers:
            x = layer(x, False)
        return self.lm_heads[pred_idx - self.cfg.n_codes_given](self.layernorm_final(x)).float()


# ----------------------------------------------------------------------------
# EnCodec 24 kHz decoder
# ----------------------------------------------------------------------------
@dataclasses.dataclass
class EncodecConfig:
    dim: int = 128
    n_filters: int = 32
    ratios: tuple = (8, 5, 4, 2)
    n_q: int = 8
    bins: int = 1024
    lstm_layers: int = 2
    compress: int = 2
    kernel: int = 7
    residual_kernel: int = 3
    last_kernel: int = 7

    @property
    def hop(self):
        return int(np.prod(self.ratios))


TINY_ENCODEC = EncodecConfig(dim=16, n_filters=8, ratios=(4, 2), n_q=8, bins=1024)


def _reflect_left(x, p):
    """Left reflect-pad [B, T, C] by p (EnCodec causal conv padding)."""
    if p == 0:
        return x
    t = x.shape[1]
    if t <= p:  # HF _pad1d: zero-extend first so reflect is defined
        x = torch.cat([x, x.new_zeros(x.shape[0], p - t + 1, x.shape[2])], 1)
    return torch.cat([x[:, 1:p + 1].flip(1), x], 1)[:, : t + p]


class _CausalConv(nn.Module):
    def __init__(self, cin, cout, k, dilation=1):
        super().__init__()
        self.conv = Conv1d(cin, cout, k, dilation=dilation)
        self.pad = (k - 1) * dilation

    def forward(self, x, act=None, residual=None):
        return self.conv(_reflect_left(x, self.pad), act=act, residual=residual, padding=0)


class _CausalConvT(nn.Module):
    def __init__(self, cin, cout, ratio):
        super().__init__()
        self.conv = ConvTranspose1d(cin, cout, 2 * ratio, stride=ratio)
        self.trim = ratio  # padding_total = k - stride, all trimmed on the right (causal)

    def forward(self, x):
        y = self.conv(x)
        return y[:, : y.shape[1] - self.trim].contiguous()


class _ResBlock(nn.Module):
    def __init__(self, dim, compress, k):
        super().__init__()
        hid = dim // compress
        self.block = nn.ModuleList([nn.Identity(), _CausalConv(dim, hid, k), nn.Identity(), _CausalConv(hid, dim, 1)])
        self.shortcut = _CausalConv(dim, dim, 1)

    def forward(self, x):
        sc = self.shortcut(x)
        h = self.block[1](ops.act(x, "elu"), act="elu")
        return self.block[3](h, residual=sc)


class _LSTM(nn.Module):
    def __init__(self, dim, layers):
        super().__init__()
        self.lstm = nn.LSTM(dim, dim, layers)

    def forward(self, x):
        xf = x.float().transpose(0, 1)  # [T, B, C]
        y, _ = self.lstm(xf)
        return (y + xf).transpose(0, 1).to(x.dtype).contiguous()


class EncodecDecoder(nn.Module):
    def __init__(self, cfg: EncodecConfig = EncodecConfig()):
        super().__init__()
        self.cfg = cfg
        self.codebooks = nn.Parameter(torch.zeros(cfg.n_q, cfg.bins, cfg.dim))
        scale = 2 ** len(cfg.ratios)
        layers: list[nn.Module] = [_CausalConv(cfg.dim, scale * cfg.n_filters, cfg.kernel),
                                   _LSTM(scale * cfg.n_filters, cfg.lstm_layers)]
        for r in cfg.ratios:
            c = scale * cfg.n_filters
            layers += [nn.ELU(), _CausalConvT(c, c // 2, r), _ResBlock(c // 2, cfg.compress, cfg.residual_kernel)]
            scale //= 2
        layers += [nn.ELU(), _CausalConv(cfg.n_filters, 1, cfg.last_kernel)]
        self.layers = nn.ModuleList(layers)

    @torch.no_grad()
    def forward(self, codes: torch.Tensor) -> torch.Tensor:
        """codes [n_q, T] int -> waveform [T * hop] fp32."""
        emb = sum(self.codebooks[i][codes[i]] for i in range(codes.shape[0]))  # [T, dim]
        x = emb[None].to(self.layers[0].conv.weight.dtype).contiguous()
        pending_elu = False
        for m in self.layers:
            if isinstance(m, nn.ELU):
                pending_elu = True
                continue
            if pending_elu:
                x = ops.act(x, "elu")
                pending_elu = False
            x = m(x)
        return x[0, :, 0].float()


def fold_weight_norm(sd: dict) -> dict:
    """{name.weight_g, name.weight_v} (or parametrizations.weight.original0/1) -> name.weight."""
    out = dict(sd)
    for k in list(sd):
        for g_suf, v_suf in ((".weight_g", ".weight_v"),
                             (".parametrizations.weight.original0", ".parametrizations.weight.original1")):
            if k.endswith(g_suf):
                base = k[: -len(g_suf)]
                g, v = sd[k].float(), sd[base + v_suf].float()
                norm = v.flatten(1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))
                out[base + ".weight"] = g * v / norm
                out.pop(k, None)
                out.pop(base + v_suf, None)
    return out


# ----------------------------------------------------------------------------
# generation
# ----------------------------------------------------------------------------
def _sample(logits: torch.Tensor, temp: float, gen) -> int:
    p = torch.softmax(logits.float() / temp, -1)
    return int(torch.multinomial(p, 1, generator=gen).item())


class Bark:
    sample_rate = SAMPLE_RATE

    def __init__(self, device="cpu", size="large", seed=0, weights_dir=None):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        import os

        raw = None
        if weights_dir and os.path.exists(os.path.join(weights_dir, "config.json")):
            from .hf_config import read_json

            raw = read_json(os.path.join(weights_dir, "config.json"))
        if raw and "semantic_config" in raw:
            sc, cc, fc, ec = bark_configs_from_hf(raw)
        else:
            sc, cc, fc = bark_configs(size)
            ec = TINY_ENCODEC if size == "tiny" else EncodecConfig()
        with torch.device(self.device):
            self.semantic = BarkCausalGPT(sc).to(self.dtype)
            self.coarse = BarkCausalGPT(cc).to(self.dtype)
            self.fine = BarkFineGPT(fc).to(self.dtype)
            self.codec = EncodecDecoder(ec).to(self.dtype)
        self.codec.layers[1].float()  # LSTM in fp32
        mods = [self.semantic, self.coarse, self.fine, self.codec]
        for i, m in enumerate(mods):
            m.eval().requires_grad_(False)
            init_random_fast_(m, seed=seed + i)
        with torch.no_grad():
            self.codec.codebooks.normal_(0, 1.0)
        self.weights_source = "random-init"
        if weights_dir and self._load(weights_dir):
            self.weights_source = str(weights_dir)
        for m in mods:
            prepare_model(m)
        from .wordpiece import WordPiece

        tdir = weights_dir if weights_dir and os.path.exists(os.path.join(weights_dir, "vocab.txt")) else None
        self.tokenizer = WordPiece(tdir, vocab_size=119_547, lower=False)

    def _load(self, d) -> bool:
        """transformers ``BarkModel`` safetensors: the three GPTs (strict), the
        EnCodec decoder (weight norm folded; the encoder is not needed to
        synthesise) and the first n_q quantizer codebooks."""
        import os

        from .weights import CheckpointMismatch, _read_dir, load_into

        if not os.path.isdir(d):
            return False
        sd = fold_weight_norm(_read_dir(d))
        if not sd:
            return False
        fine = self.fine.cfg
        for i in range(fine.n_codes_total - fine.n_codes_given):
            # the fine model ties lm_heads[i] to input_embeds_layers[i + n_codes_given];
            # safetensors exports keep only one of each tied pair
            a, b = f"fine_acoustics.lm_heads.{i}.weight", f"fine_acoustics.input_embeds_layers.{i + fine.n_codes_given}.weight"
            if a in sd and b not in sd:
                sd[b] = sd[a]
            elif b in sd and a not in sd:
                sd[a] = sd[b]
        for pre, mod in (("semantic.", self.semantic), ("coarse_acoustics.", self.coarse),
                         ("fine_acoustics.", self.fine)):
            # "<layer>.attn.bias" is transformers' causal-mask buffer, not a parameter
            load_into(mod, {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre) and not k.endswith(".attn.bias")},
                      name=pre[:-1])
        pre = "codec_model.decoder."
        dec = {k[len(pre):]: v for k, v in sd.items() if k.startswith(pre)}
        cb = [sd.get(f"codec_model.quantizer.layers.{i}.codebook.embed") for i in range(self.codec.cfg.n_q)]
        if any(c is None for c in cb):
            raise CheckpointMismatch(f"bark: {d} lacks codec_model.quantizer codebooks 0..{self.codec.cfg.n_q - 1}")
        dec["codebooks"] = torch.stack(cb)
        load_into(self.codec, dec, name="codec_model.decoder")
        return True

    # -- stage 1 -----------------------------------------------------------
    @torch.no_grad()
    def text_to_semantic(self, text: str, gen, temp=0.7, min_eos_p=0.2, max_tokens=768) -> np.ndarray:
        ids = (np.array(self.tokenizer.encode(text), dtype=np.int64) + TEXT_OFFSET)[:256]
        ids = np.pad(ids, (0, 256 - len(ids)), constant_values=TEXT_PAD)
        hist = np.full(256, SEMANTIC_PAD, dtype=np.int64)
        dev = self.device
        m = self.semantic
        m.new_cache()
        wte = m.input_embeds_layer
        t_ids = torch.from_numpy(ids).to(dev)[None]
        h_ids = torch.from_numpy(hist).to(dev)[None]
        # merge_context: text and history embeddings are summed position-wise
        e = torch.cat([wte(t_ids) + wte(h_ids), wte(torch.tensor([[SEMANTIC_INFER]], device=dev))], 1)
        max_tokens = min(max_tokens, m.cfg.block_size - e.shape[1])
        logits = m(embeds=e, pos=0)[0]
        pos = e.shape[1]
        out: list[int] = []
        for _ in range(max_tokens):
            rel = torch.cat([logits[:SEMANTIC_VOCAB], logits[SEMANTIC_PAD:SEMANTIC_PAD + 1]])
            probs = torch.softmax(rel / temp, -1)
            nxt = int(torch.multinomial(probs, 1, generator=gen).item())
            if nxt == SEMANTIC_VOCAB or float(probs[-1]) >= min_eos_p:
                break
            out.append(nxt)
            logits = m.decode_step(nxt, pos)[0]
            pos += 1
        return np.array(out, dtype=np.int64)

    # -- stage 2 -----------------------------------------------------------
    @torch.no_grad()
    def semantic_to_coarse(self, sem: np.ndarray, gen, temp=0.7, window=60, max_hist=630) -> np.ndarray:
        ratio = COARSE_RATE_HZ / SEMANTIC_RATE_HZ * N_COARSE
        max_sem_hist = int(np.floor(max_hist / ratio))
        n_steps = int(round(np.floor(len(sem) * ratio / N_COARSE) * N_COARSE))
        m = self.coarse
        dev = self.device
        coarse: list[int] = []
        n_step = 0
        for _ in range(int(np.ceil(n_steps / window))):
            si = int(round(n_step / ratio))
            x_sem = sem[max(0, si - max_sem_hist):][:256]
            x_sem = np.pad(x_sem, (0, 256 - len(x_sem)), constant_values=COARSE_SEMANTIC_PAD)
            ctx = np.concatenate([x_sem, [COARSE_INFER], np.array(coarse[-max_hist:], dtype=np.int64)])
            m.new_cache()
            logits = m(torch.from_numpy(ctx.astype(np.int64)).to(dev)[None], pos=0)[0]
            pos = len(ctx)
            for _ in range(window):
                if n_step >= n_steps or pos >= m.cfg.block_size:
                    break
                major = n_step % 2 == 0
                lo = SEMANTIC_VOCAB + (0 if major else CODEBOOK_SIZE)
                nxt = _sample(logits[lo:lo + CODEBOOK_SIZE], temp, gen) + lo
                coarse.append(nxt)
                n_step += 1
                logits = m.decode_step(nxt, pos)[0]
                pos += 1
        arr = np.array(coarse, dtype=np.int64).reshape(-1, N_COARSE).T - SEMANTIC_VOCAB
        for n in range(1, N_COARSE):
            arr[n] -= n * CODEBOOK_SIZE
        return np.clip(arr, 0, CODEBOOK_SIZE - 1)

    # -- stage 3 -----------------------------------------------------------
    @torch.no_grad()
    def coarse_to_fine(self, coarse: np.ndarray, gen, temp=0.5) -> np.ndarray:
        win = min(1024, self.fine.cfg.block_size)
        n = coarse.shape[1]
        arr = np.full((N_FINE, max(n, win)), CODEBOOK_SIZE, dtype=np.int64)
        arr[:N_COARSE, :n] = coarse
        arr = arr.T.copy()  # [T, 8]
        total = arr.shape[0]
        n_loops = max(0, int(np.ceil((n - win) / (win // 2)))) + 1
        for i in range(n_loops):
            start = min(i * (win // 2), total - win)
            fill = min(i * (win // 2), total - win // 2)
            rel = fill - start
            buf = torch.from_numpy(arr[start:start + win]).to(self.device)[None]
            for cb in range(N_COARSE, N_FINE):
                logits = self.fine(cb, buf)[0, rel:, :CODEBOOK_SIZE]
                if temp is None:
                    pred = logits.argmax(-1)
                else:
                    pred = torch.multinomial(torch.softmax(logits / temp, -1), 1, generator=gen)[:, 0]
                buf[0, rel:, cb] = pred
            arr[start + rel:start + win] = buf[0, rel:].cpu().numpy()
        return arr.T[:, :n]

    @torch.no_grad()
    def generate_audio(self, text: str, seed=None, max_semantic_tokens=768) -> np.ndarray:
        gen = torch.Generator(device=self.device)
        gen.manual_seed(int(seed) if seed is not None else 0)
        sem = self.text_to_semantic(text, gen, max_tokens=max_semantic_tokens)
        if len(sem) < 2:
            sem = np.array([0, 0], dtype=np.int64)
        coarse = self.semantic_to_coarse(sem, gen)
        fine = self.coarse_to_fine(coarse, gen)
        codes = torch.from_numpy(fine).to(self.device)
        return self.codec(codes).cpu().numpy()


def load_bark(model_name: str, device: str) -> Bark:
    from ..runtime.model_cache import cache
    from ..runtime.provision import ensure_weights

    name = model_name.lower()
    size = "tiny" if name.startswith("tiny") else ("small" if "small" in name else "large")
    return cache().get(("bark", model_name, device),
                       lambda: Bark(device, size=size, weights_dir=ensure_weights(model_name),
                                    seed=stable_seed(model_name)))
