"""UNet2DConditionModel (SD1.5 / SD2.x / SDXL configs) on NHWC bf16.

Covers the denoiser reached by the reference's txt2img / img2img / inpaint /
ControlNet / pix2pix / upscaler calls (swarm/diffusion/diffusion_func.py:96,
swarm/diffusion/upscale.py:22, swarm/video/pix2pix.py:142).  Geometry from the
public model configs (SURVEY.md §2.3 "Model geometry").

MI355X-specific structure:
  * all ResNet time projections of a step are ONE batched GEMM
    (``prepare_self`` concatenates every ``time_emb_proj``), then each block
    receives its [B, Cout] slice as a per-sample bias fused into conv1's
    epilogue;
  * cross-attention K/V of the (fixed) prompt context are computed once per
    request by ``encode_context`` and re-used for every denoising step (K8);
  * ControlNet residuals are added where the skip tensors are produced.
"""
from __future__ import annotations

import dataclasses
from typing import Sequence

import torch
import torch.nn as nn

from .. import ops
from .layers import (Conv2d, Downsample2D, GroupNorm, Linear, Prepared, ResnetBlock2D,
                     TimestepEmbedding, Transformer2D, Upsample2D, timestep_embedding)


@dataclasses.dataclass
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: Sequence[int] = (320, 640, 1280, 1280)
    layers_per_block: int = 2
    down_block_types: Sequence[str] = ("CrossAttnDownBlock2D",) * 3 + ("DownBlock2D",)
    up_block_types: Sequence[str] = ("UpBlock2D",) + ("CrossAttnUpBlock2D",) * 3
    num_heads: Sequence[int] | int = (5, 10, 20, 20)  # diffusers "attention_head_dim"
    cross_attention_dim: int = 1024
    use_linear_projection: bool = True
    transformer_layers_per_block: Sequence[int] | int = 1
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    addition_embed_type: str | None = None  # "text_time" for SDXL
    addition_time_embed_dim: int = 256
    projection_class_embeddings_input_dim: int = 2816
    prediction_type: str = "epsilon"
    sample_size: int = 64
    # sd-x2-latent-upscaler / x4 upscaler style extra conditioning
    num_class_embeds: int | None = None
    class_embed_type: str | None = None
    class_embeddings_concat: bool = False

    def per_block(self, v, n):
        return list(v) if isinstance(v, (list, tuple)) else [v] * n


SD15 = UNetConfig(num_heads=8, cross_attention_dim=768, use_linear_projection=False)
SD21 = UNetConfig()  # stabilityai/stable-diffusion-2-1-base (512^2, epsilon)
SD21_V = dataclasses.replace(SD21, prediction_type="v_prediction", sample_size=96)
SDXL = UNetConfig(
    block_out_channels=(320, 640, 1280),
    down_block_types=("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D"),
    up_block_types=("CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"),
    num_heads=(5, 10, 20), transformer_layers_per_block=(1, 2, 10),
    cross_attention_dim=2048, addition_embed_type="text_time", sample_size=128)
PIX2PIX = dataclasses.replace(SD15, in_channels=8)
INPAINT_SD2 = dataclasses.replace(SD21, in_channels=9)
INPAINT_SD15 = dataclasses.replace(SD15, in_channels=9)
# tiny config for CPU plumbing tests (same topology, small widths)
TINY = UNetConfig(block_out_channels=(32, 64), layers_per_block=1,
                  down_block_types=("CrossAttnDownBlock2D", "DownBlock2D"),
                  up_block_types=("UpBlock2D", "CrossAttnUpBlock2D"),
                  num_heads=(2, 2), cross_attention_dim=32, sample_size=8)
# stabilityai/stable-diffusion-xl-refiner-1.0: bigG context only (1280), pooled
# 1280 + 5 aesthetic-score time ids x 256 = 2560
SDXL_REFINER = UNetConfig(
    block_out_channels=(384, 768, 1536, 1536),
    down_block_types=("DownBlock2D", "CrossAttnDownBlock2D", "CrossAttnDownBlock2D", "DownBlock2D"),
    up_block_types=("UpBlock2D", "CrossAttnUpBlock2D", "CrossAttnUpBlock2D", "UpBlock2D"),
    num_heads=(6, 12, 24, 24), transformer_layers_per_block=4, cross_attention_dim=1280,
    addition_embed_type="text_time", projection_class_embeddings_input_dim=2560, sample_size=128)
# SDXL structure at test size: text_time add-embedding, two text encoders
# (32 + 32 context, pooled projection 32), deeper transformer stack below
TINY_XL = UNetConfig(block_out_channels=(32, 64), layers_per_block=1,
                     down_block_types=("DownBlock2D", "CrossAttnDownBlock2D"),
                     up_block_types=("CrossAttnUpBlock2D", "UpBlock2D"),
                     num_heads=(2, 2), transformer_layers_per_block=(1, 2), cross_attention_dim=64,
                     addition_embed_type="text_time", addition_time_embed_dim=8,
                     projection_class_embeddings_input_dim=32 + 6 * 8, sample_size=8)
TINY_XL_REFINER = dataclasses.replace(TINY_XL, cross_attention_dim=32, projection_class_embeddings_input_dim=32 + 5 * 8)

# AudioLDM (cvssp/audioldm-*): 8-channel mel latents, CLAP embedding as a
# concatenated class embedding, attention blocks whose "cross" attention runs on
# the hidden states themselves (no text sequence)
AUDIOLDM = UNetConfig(
    in_channels=8, out_channels=8, block_out_channels=(128, 256, 384, 640),
    down_block_types=("DownBlock2D",) + ("CrossAttnDownBlock2D",) * 3,
    up_block_types=("CrossAttnUpBlock2D",) * 3 + ("UpBlock2D",),
    num_heads=8, cross_attention_dim=(128, 256, 384, 640), use_linear_projection=False,
    class_embed_type="simple_projection", projection_class_embeddings_input_dim=512,
    class_embeddings_concat=True, sample_size=128)
TINY_AUDIOLDM = UNetConfig(
    in_channels=8, out_channels=8, block_out_channels=(32, 64), layers_per_block=1,
    down_block_types=("DownBlock2D", "CrossAttnDownBlock2D"), up_block_types=("CrossAttnUpBlock2D", "UpBlock2D"),
    num_heads=2, cross_attention_dim=(32, 64), class_embed_type="simple_projection",
    projection_class_embeddings_input_dim=32, class_embeddings_concat=True, sample_size=8)

# stabilityai/stable-diffusion-x4-upscaler: 4 latent + 3 low-res RGB channels,
# noise level as a class embedding, OpenCLIP-H context
X4_UPSCALER = UNetConfig(
    in_channels=7, out_channels=4, block_out_channels=(256, 512, 512, 1024),
    down_block_types=("DownBlock2D",) + ("CrossAttnDownBlock2D",) * 3,
    up_block_types=("CrossAttnUpBlock2D",) * 3 + ("UpBlock2D",),
    num_heads=8, cross_attention_dim=1024, num_class_embeds=1000, sample_size=128)
TINY_X4 = dataclasses.replace(TINY, in_channels=7, num_class_embeds=1000)
# stabilityai/stable-diffusion-2-1-unclip: SD2.1-v UNet + "projection" class
# embedding of [noised ViT-H/14 image embedding (1024) | noise-level sinusoid (1024)]
SD21_UNCLIP = dataclasses.replace(SD21_V, class_embed_type="projection", projection_class_embeddings_input_dim=2048)
TINY_UNCLIP = dataclasses.replace(TINY, class_embed_type="projection", projection_class_embeddings_input_dim=64)
# stabilityai/stable-diffusion-2-depth: latents + 1 depth channel (512 px, epsilon)
DEPTH_SD2 = dataclasses.replace(SD21, in_channels=5)
TINY_DEPTH = dataclasses.replace(TINY, in_channels=5)

CONFIGS = {"sd15": SD15, "sd21": SD21, "sd21-v": SD21_V, "sdxl": SDXL, "pix2pix": PIX2PIX,
           "sd2-inpaint": INPAINT_SD2, "sd15-inpaint": INPAINT_SD15, "tiny": TINY}


class _Block(nn.Module):
    def __init__(self, resnets, attentions, sampler_attr, sampler):
        super().__init__()
        self.resnets = nn.ModuleList(resnets)
        self.attentions = nn.ModuleList(attentions) if attentions else None
        if sampler is not None:
            setattr(self, sampler_attr, nn.ModuleList([sampler]))
        else:
            setattr(self, sampler_attr, None)


class UNet2DConditionModel(Prepared):
    def __init__(self, cfg: UNetConfig = SD21):
        super().__init__()
        self.cfg = cfg
        ch = list(cfg.block_out_channels)
        nb = len(ch)
        heads = cfg.per_block(cfg.num_heads, nb)
        tlayers = cfg.per_block(cfg.transformer_layers_per_block, nb)
        temb_dim = ch[0] * 4
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        xdims = cfg.per_block(cfg.cross_attention_dim, nb)

        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch[0], temb_dim)
        if cfg.addition_embed_type == "text_time":
            self.add_embedding = TimestepEmbedding(cfg.projection_class_embeddings_input_dim, temb_dim)
        if cfg.class_embed_type == "timestep":
            self.class_embedding = TimestepEmbedding(ch[0], temb_dim)
        elif cfg.class_embed_type == "simple_projection":  # AudioLDM: CLAP embedding -> temb
            self.class_embedding = Linear(cfg.projection_class_embeddings_input_dim, temb_dim)
        elif cfg.class_embed_type == "projection":  # SD2.1-unCLIP: noised CLIP image embedding + level -> temb
            self.class_embedding = TimestepEmbedding(cfg.projection_class_embeddings_input_dim, temb_dim)
        elif cfg.num_class_embeds is not None:  # x4 upscaler: noise level as a class id
            self.class_embedding = nn.Embedding(cfg.num_class_embeds, temb_dim)
        rtemb = temb_dim * (2 if cfg.class_embeddings_concat else 1)

        def resnet(ci, co):
            return ResnetBlock2D(ci, co, rtemb, g, eps)

        def xformer(c, i):
            return Transformer2D(c, heads[i], xdims[i], tlayers[i], cfg.use_linear_projection, g)

        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i, btype in enumerate(cfg.down_block_types):
            cin, cout = cout, ch[i]
            final = i == nb - 1
            res = [resnet(cin if j == 0 else cout, cout) for j in range(cfg.layers_per_block)]
            att = ([xformer(cout, i) for _ in range(cfg.layers_per_block)]
                   if btype.startswith("CrossAttn") else None)
            self.down_blocks.append(_Block(res, att, "downsamplers", None if final else Downsample2D(cout)))

        self.mid_block = _Block([resnet(ch[-1], ch[-1]), resnet(ch[-1], ch[-1])],
                                [xformer(ch[-1], nb - 1)], "upsamplers", None)

        rch = list(reversed(ch))
        rheads = list(reversed(heads))
        rtl = list(reversed(tlayers))
        rxd = list(reversed(xdims))
        self.up_blocks = nn.ModuleList()
        out_c = rch[0]
        for i, btype in enumerate(cfg.up_block_types):
            prev_c, out_c = out_c, rch[i]
            in_c = rch[min(i + 1, nb - 1)]
            final = i == nb - 1
            nl = cfg.layers_per_block + 1
            res = []
            for j in range(nl):
                skip = in_c if j == nl - 1 else out_c
                rin = prev_c if j == 0 else out_c
                res.append(resnet(rin + skip, out_c))
            att = None
            if btype.startswith("CrossAttn"):
                att = [Transformer2D(out_c, rheads[i], rxd[i], rtl[i],
                                     cfg.use_linear_projection, g) for _ in range(nl)]
            self.up_blocks.append(_Block(res, att, "upsamplers", None if final else Upsample2D(out_c)))

        self.conv_norm_out = GroupNorm(g, ch[0], eps=eps)
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3, padding=1)

    # ------------------------------------------------------------------
    def _resnets(self):
        out = []
        for blk in list(self.down_blocks) + [self.mid_block] + list(self.up_blocks):
            out.extend(blk.resnets)
        return out

    def prepare_self(self):
        """Concatenate every ResNet's time_emb_proj into one [sum Cout, Temb] GEMM."""
        rs = self._resnets()
        self._temb_w = torch.cat([r.time_emb_proj.weight for r in rs], 0).detach()
        self._temb_b = torch.cat([r.time_emb_proj.bias for r in rs], 0).detach()
        self._temb_splits = [r.out_channels for r in rs]

    def _temb_projs(self, temb):
        w = getattr(self, "_temb_w", None)
        if w is None or w.device != temb.device or w.dtype != self.conv_in.weight.dtype:
            self.prepare_self()
        proj = ops.gemm(ops.silu(temb), self._temb_w, self._temb_b)
        return list(torch.split(proj, self._temb_splits, dim=-1))

    @torch.no_grad()
    def temb_table(self, ts: torch.Tensor) -> torch.Tensor:
        """[n, sum Cout] batched ResNet time projections for every timestep of
        ``ts`` (fp32 [n]) — the whole time-embedding chain (sinusoid, MLP, SiLU,
        projection GEMM) for a request's schedule in one pass, so the sampler
        loop's step graph only gathers its row (``forward(temb_proj=...)``)."""
        dtype = self.conv_in.weight.dtype
        ts = ts.reshape(-1).float()
        temb = self.time_embed(ts, ts.numel(), dtype)
        w = getattr(self, "_temb_w", None)
        if w is None or w.device != temb.device or w.dtype != dtype:
            self.prepare_self()
        return ops.gemm(ops.silu(temb), self._temb_w, self._temb_b)

    def cross_attention_modules(self):
        mods = []
        for blk in list(self.down_blocks) + [self.mid_block] + list(self.up_blocks):
            if blk.attentions is not None:
                for t in blk.attentions:
                    mods.extend(t.cross_modules())
        return mods

    @torch.no_grad()
    def encode_context(self, ctx: torch.Tensor):
        """Per-request cache of every cross-attention K/V (constant over steps)."""
        return [m.context_kv(ctx) for m in self.cross_attention_modules()]

    # ------------------------------------------------------------------
    def add_emb(self, added_cond, dtype=None):
        """SDXL ``text_time`` addition embedding (pooled text embeds + the
        sinusoidal size / crop ids through ``add_embedding``): constant over a
        request's denoising steps."""
        dtype = dtype or self.conv_in.weight.dtype
        text_embeds = added_cond["text_embeds"]
        tid = timestep_embedding(added_cond["time_ids"].reshape(-1), self.cfg.addition_time_embed_dim)
        tid = tid.reshape(text_embeds.shape[0], -1)
        add_in = torch.cat([text_embeds.float(), tid], dim=-1).to(dtype)
        return self.add_embedding(add_in)

    def time_embed(self, timestep, batch, dtype, added_cond=None, class_labels=None):
        t = timestep
        if not torch.is_tensor(t):
            t = torch.tensor([t], dtype=torch.float32, device=self.conv_in.weight.device)
        t = t.reshape(-1).float()
        if ops.use_hip(t) and dtype == torch.bfloat16:
            from ..ops import hip_ops  # one kernel instead of ~12 small torch ops per step

            emb = hip_ops.timestep_embedding(t, batch, self.cfg.block_out_channels[0])
        else:
            emb = timestep_embedding(t.expand(batch) if t.numel() == 1 else t,
                                     self.cfg.block_out_channels[0]).to(dtype)
        temb = self.time_embedding(emb)
        if self.cfg.addition_embed_type == "text_time":
            ae = added_cond.get("add_emb")  # precomputed once per request (pipelines.sd._UNetGraph)
            temb = temb + (ae if ae is not None else self.add_emb(added_cond, dtype))
        if class_labels is None and added_cond is not None:  # per-request labels carried with the added cond
            class_labels = added_cond.get("class_labels")
        if self.cfg.class_embed_type == "timestep" and class_labels is not None:
            cl = timestep_embedding(class_labels.reshape(-1).float(), self.cfg.block_out_channels[0])
            temb = temb + self.class_embedding(cl.to(dtype))
        elif self.cfg.class_embed_type == "simple_projection" and class_labels is not None:
            cemb = self.class_embedding(class_labels.to(dtype))
            temb = torch.cat([temb, cemb], -1) if self.cfg.class_embeddings_concat else temb + cemb
        elif self.cfg.class_embed_type == "projection" and class_labels is not None:
            temb = temb + self.class_embedding(class_labels.to(dtype))
        elif self.cfg.num_class_embeds is not None and class_labels is not None:
            temb = temb + self.class_embedding(class_labels.reshape(-1).long()).to(dtype).expand_as(temb)
        return temb

    def forward(self, *args, **kwargs):
        """``_forward`` inside the model's tuning context (SDXL: its own tile
        choices for shape keys it shares with SD2.1, ops/tuning.py::context)."""
        ctx = "sdxl" if self.cfg.addition_embed_type == "text_time" else None
        if ctx is None:
            return self._forward(*args, **kwargs)
        from ..ops import tuning

        with tuning.context(ctx):
            return self._forward(*args, **kwargs)

    def _forward(self, sample, timestep, encoder_hidden_states=None, cross_kv=None,
                 added_cond=None, down_residuals=None, mid_residual=None, class_labels=None, control=None,
                 cfg_dup=False, temb_proj=None):
        """sample: NHWC [B, H, W, Cin]; returns NHWC [B, H, W, Cout].

        ``control``: a ControlNet's pre-zero-conv features
        (``pipelines.controlnet.ControlFeatures``): each skip and the mid-block
        output are merged as ``skip + scale * zero_conv(feature)`` inside the
        zero conv's GEMM epilogue (no separate add pass); ``down_residuals`` /
        ``mid_residual`` (ready-made residuals, diffusers style) are added.

        ``cfg_dup``: the caller guarantees ``sample[:B/2] == sample[B/2:]`` and a
        per-sample-identical time embedding (classifier-free guidance duplicates
        the latents; the reference's ``torch.cat([latents] * 2)`` in diffusers'
        pipelines behind swarm/diffusion/diffusion_func.py:96).  Everything up to
        the first cross-attention — conv_in, the first ResNet, the first
        transformer's GroupNorm / proj_in / self-attention and its cross-attention
        query projection — is then bit-identical for both halves, so it runs once
        at half batch and is duplicated where the halves start to differ
        (common-subexpression elimination, not an approximation).

        ``temb_proj``: precomputed [B, sum Cout] ResNet time projections (a row
        of ``temb_table``); ``timestep`` is then unused."""
        b = sample.shape[0]
        dtype = self.conv_in.weight.dtype
        x = sample.to(dtype)
        if temb_proj is not None:
            if getattr(self, "_temb_splits", None) is None:
                self.prepare_self()
            tprojs = iter(torch.split(temb_proj, self._temb_splits, dim=-1))
        else:
            temb = self.time_embed(timestep, b, dtype, added_cond, class_labels)
            tprojs = iter(self._temb_projs(temb))
        kv_iter = iter(cross_kv) if cross_kv is not None else None
        ctx = encoder_hidden_states
        half = b // 2 if (cfg_dup and b % 2 == 0) else 0

        def run_attn(t, h, dup=False):
            kvs = None
            if kv_iter is not None:
                kvs = [next(kv_iter) for _ in t.transformer_blocks]
            if dup:
                return t(h, ctx=ctx, kvs=kvs, dup=True)
            return t(h, ctx=ctx, kvs=kvs)

        dup2 = ops.dup2  # [B/2, ...] -> [B, ...] (both CFG halves)

        if half:
            h = self.conv_in(x[:half], gn_stats=True)  # the first ResNet's norm1 statistics
            skips = [dup2(h)]
        else:
            h = self.conv_in(x, gn_stats=True)
            skips = [h]
        for blk in self.down_blocks:
            for j, r in enumerate(blk.resnets):
                tp = next(tprojs)
                h = r(h, tp[:half] if half else tp)
                if blk.attentions is not None:
                    h = run_attn(blk.attentions[j], h, dup=bool(half))
                    half = 0
                skips.append(dup2(h) if half else h)
            if blk.downsamplers is not None:
                h = blk.downsamplers[0](h)
                skips.append(dup2(h) if half else h)
        if half:  # no cross-attention in the down path
            h = dup2(h)

        if control is not None:
            skips = [control.merge_skip(i, s) for i, s in enumerate(skips)]
        elif down_residuals is not None:
            skips = [s + r.to(s.dtype) for s, r in zip(skips, down_residuals)]

        h = self.mid_block.resnets[0](h, next(tprojs))
        h = run_attn(self.mid_block.attentions[0], h)
        h = self.mid_block.resnets[1](h, next(tprojs))
        if control is not None:
            h = control.merge_mid(h)
        elif mid_residual is not None:
            h = h + mid_residual.to(h.dtype)

        for blk in self.up_blocks:
            for j, r in enumerate(blk.resnets):
                s = skips.pop()
                h = r.forward_cat(h, s, next(tprojs))
                if blk.attentions is not None:
                    h = run_attn(blk.attentions[j], h)
            if blk.upsamplers is not None:
                h = blk.upsamplers[0](h, size=skips[-1].shape[1:3] if skips else None)

        h = self.conv_norm_out(h, silu=True)
        return self.conv_out(h)
