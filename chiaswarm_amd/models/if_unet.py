"""Pixel-space cascade UNet of DeepFloyd IF (stage I 64x64, stage II 256x256).

Structure follows diffusers' IF UNet (``UNet2DConditionModel`` with
``ResnetDownsampleBlock2D`` / ``SimpleCrossAttn*`` blocks):
  * ResNets with ``scale_shift`` time conditioning — GroupNorm, then
    ``h * (1 + scale) + shift`` from the time projection, then SiLU — and
    resampling *inside* the ResNet (avg-pool down / nearest up of both the
    main path and the shortcut), which is how IF down/upsamples;
  * ``SimpleCrossAttention`` (AttnAddedKV): GroupNorm'd pixels give Q and
    self K/V; the T5 tokens give extra K/V (``add_k_proj``/``add_v_proj``)
    that are concatenated in front of the self K/V, one attention call;
  * the T5 states go through ``encoder_hid_proj`` and a pooled projection of
    them is added to the time embedding (``addition_embed_type="text"``);
  * stage II conditions on the noise level of its upscaled input through a
    timestep-style class embedding.
The UNet predicts 6 channels (epsilon + learned-variance interpolation); the
pipeline uses the epsilon half.

Geometry: IF checkpoints are not in this image (no network), so per-stage
widths are the published orders of magnitude (IF-I-XL 4.3B, IF-II-L 1.2B)
rather than verified configs — parity unpinned, documented in
``pipelines/deepfloyd.py``.

MI355X path: every conv is the implicit-GEMM conv kernel (nearest-up fused
into conv1's input addressing for up-ResNets; shortcut added in conv2's
epilogue), GroupNorm(+SiLU) is the fused norm kernel with the per-sample
scale/shift folded into its affine, attention is the flash kernel with the
text K/V cached per request.
"""
from __future__ import annotations

import dataclasses
from typing import Sequence

import torch
import torch.nn as nn

from .. import ops
from .layers import (Conv2d, GroupNorm, LayerNorm, Linear, Prepared, TimestepEmbedding, timestep_embedding)


@dataclasses.dataclass
class IFUNetConfig:
    in_channels: int = 3
    out_channels: int = 6
    block_out_channels: Sequence[int] = (512, 1024, 1536, 2048)
    attn_levels: Sequence[bool] = (False, True, True, True)
    layers_per_block: int = 3
    head_dim: int = 64
    encoder_hid_dim: int = 4096
    cross_dim: int = 2048
    groups: int = 32
    noise_level_cond: bool = False  # stage II
    sample_size: int = 64


IF_I_XL = IFUNetConfig()
IF_II_L = IFUNetConfig(in_channels=6, block_out_channels=(128, 256, 512, 1024, 1536),
                       attn_levels=(False, False, False, True, True), layers_per_block=2, cross_dim=1536,
                       noise_level_cond=True, sample_size=256)
TINY_IF_I = IFUNetConfig(block_out_channels=(32, 64), attn_levels=(False, True), layers_per_block=1, head_dim=16,
                         encoder_hid_dim=64, cross_dim=64, sample_size=16)
TINY_IF_II = dataclasses.replace(TINY_IF_I, in_channels=6, noise_level_cond=True, sample_size=32)


def _avg_pool2(x):
    b, h, w, c = x.shape
    return x.view(b, h // 2, 2, w // 2, 2, c).float().mean((2, 4)).to(x.dtype)


def _nearest_up2(x):
    return x.repeat_interleave(2, 1).repeat_interleave(2, 2)


class ScaleShiftResnet(nn.Module):
    def __init__(self, cin, cout, temb_dim, groups=32, up=False, down=False):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps=1e-5)
        self.conv1 = Conv2d(cin, cout, 3, padding=1)
        self.time_emb_proj = Linear(temb_dim, 2 * cout)
        self.norm2 = GroupNorm(groups, cout, eps=1e-5)
        self.conv2 = Conv2d(cout, cout, 3, padding=1)
        self.conv_shortcut = Conv2d(cin, cout, 1, padding=0) if cin != cout else None
        self.up, self.down = up, down
        self.out_channels = cout

    def forward(self, x, temb):
        h = self.norm1(x, silu=True)
        if self.down:
            h, x = _avg_pool2(h), _avg_pool2(x)
        h = self.conv1(h, up2x=self.up)
        if self.up:
            x = _nearest_up2(x)
        ss = self.time_emb_proj(ops.silu(temb)).float()
        scale, shift = ss.chunk(2, dim=-1)
        # GroupNorm affine with the per-sample (1 + scale), shift folded in
        g = self.norm2.weight.float()[None] * (1 + scale)
        bt = self.norm2.bias.float()[None] * (1 + scale) + shift
        h = ops.group_norm(h, g.to(h.dtype), bt.to(h.dtype), self.norm2.num_groups, self.norm2.eps, silu=True)
        sc = x if self.conv_shortcut is None else self.conv_shortcut(x)
        return self.conv2(h, residual=sc)


class SimpleCrossAttention(Prepared):
    def __init__(self, dim, head_dim, cross_dim, groups=32):
        super().__init__()
        self.heads, self.dh = dim // head_dim, head_dim
        self.group_norm = GroupNorm(groups, dim, eps=1e-5)
        self.to_q = Linear(dim, dim)
        self.to_k = Linear(dim, dim)
        self.to_v = Linear(dim, dim)
        self.add_k_proj = Linear(cross_dim, dim)
        self.add_v_proj = Linear(cross_dim, dim)
        self.to_out = nn.ModuleList([Linear(dim, dim)])

    def prepare(self):
        self.w_qkv = torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight], 0).detach()
        self.b_qkv = torch.cat([self.to_q.bias, self.to_k.bias, self.to_v.bias], 0).detach()
        self.w_add = torch.cat([self.add_k_proj.weight, self.add_v_proj.weight], 0).detach()
        self.b_add = torch.cat([self.add_k_proj.bias, self.add_v_proj.bias], 0).detach()

    def _ensure(self):
        w = getattr(self, "w_qkv", None)
        if w is None or w.device != self.to_q.weight.device or w.dtype != self.to_q.weight.dtype:
            self.prepare()

    def context_kv(self, ctx):
        """Text K/V [B, S, 2, H, D] (cached per request)."""
        self._ensure()
        b, s, _ = ctx.shape
        return ops.gemm(ctx, self.w_add, self.b_add).view(b, s, 2, self.heads, self.dh)

    def forward(self, x, text_kv):
        self._ensure()
        b, hh, ww, c = x.shape
        n = hh * ww
        h = self.group_norm(x).view(b, n, c)
        qkv = ops.gemm(h, self.w_qkv, self.b_qkv).view(b, n, 3, self.heads, self.dh)
        k = torch.cat([text_kv[:, :, 0], qkv[:, :, 1]], 1)
        v = torch.cat([text_kv[:, :, 1], qkv[:, :, 2]], 1)
        o = ops.attention(qkv[:, :, 0], k, v, self.dh ** -0.5)
        return self.to_out[0](o.reshape(b, n, c), residual=x.view(b, n, c)).view(b, hh, ww, c)


class TextPool(nn.Module):
    """addition_embed_type="text": LayerNorm -> masked mean pool -> proj -> LayerNorm."""

    def __init__(self, enc_dim, temb_dim):
        super().__init__()
        self.norm1 = LayerNorm(enc_dim)
        self.proj = Linear(enc_dim, temb_dim)
        self.norm2 = LayerNorm(temb_dim)

    def forward(self, enc):
        h = self.norm1(enc).float().mean(1).to(enc.dtype)
        return self.norm2(self.proj(h))


class IFUNet(Prepared):
    def __init__(self, cfg: IFUNetConfig = IF_I_XL):
        super().__init__()
        self.cfg = cfg
        ch = list(cfg.block_out_channels)
        nb = len(ch)
        temb = ch[0] * 4
        g = cfg.groups
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch[0], temb)
        self.encoder_hid_proj = Linear(cfg.encoder_hid_dim, cfg.cross_dim)
        self.add_embedding = TextPool(cfg.cross_dim, temb)
        if cfg.noise_level_cond:
            self.class_embedding = TimestepEmbedding(ch[0], temb)

        def res(ci, co, **kw):
            return ScaleShiftResnet(ci, co, temb, g, **kw)

        def att(c):
            return SimpleCrossAttention(c, cfg.head_dim, cfg.cross_dim, g)

        self.down = nn.ModuleList()
        cout = ch[0]
        for i in range(nb):
            cin, cout = cout, ch[i]
            blk = nn.Module()
            blk.resnets = nn.ModuleList([res(cin if j == 0 else cout, cout) for j in range(cfg.layers_per_block)])
            blk.attentions = (nn.ModuleList([att(cout) for _ in range(cfg.layers_per_block)])
                              if cfg.attn_levels[i] else None)
            blk.downsampler = res(cout, cout, down=True) if i < nb - 1 else None
            self.down.append(blk)
        self.mid = nn.Module()
        self.mid.resnets = nn.ModuleList([res(ch[-1], ch[-1]), res(ch[-1], ch[-1])])
        self.mid.attention = att(ch[-1])
        self.up = nn.ModuleList()
        rch = list(reversed(ch))
        ratt = list(reversed(cfg.attn_levels))
        out_c = rch[0]
        for i in range(nb):
            prev_c, out_c = out_c, rch[i]
            skip_c = rch[min(i + 1, nb - 1)]
            blk = nn.Module()
            nl = cfg.layers_per_block + 1
            blk.resnets = nn.ModuleList([res((prev_c if j == 0 else out_c) + (skip_c if j == nl - 1 else out_c), out_c)
                                         for j in range(nl)])
            blk.attentions = nn.ModuleList([att(out_c) for _ in range(nl)]) if ratt[i] else None
            blk.upsampler = res(out_c, out_c, up=True) if i < nb - 1 else None
            self.up.append(blk)
        self.conv_norm_out = GroupNorm(g, ch[0], eps=1e-5)
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3, padding=1)

    def attention_modules(self):
        mods = []
        for blk in self.down:
            if blk.attentions is not None:
                mods.extend(blk.attentions)
        mods.append(self.mid.attention)
        for blk in self.up:
            if blk.attentions is not None:
                mods.extend(blk.attentions)
        return mods

    @torch.no_grad()
    def encode_context(self, t5_states: torch.Tensor):
        """T5 states [B, 77, 4096] -> (per-attention text K/V list, pooled text embedding)."""
        ctx = self.encoder_hid_proj(t5_states.to(self.conv_in.weight.dtype))
        return [m.context_kv(ctx) for m in self.attention_modules()], self.add_embedding(ctx)

    def forward(self, x, t, text_kv, text_emb, noise_level=None):
        dt = self.conv_in.weight.dtype
        b = x.shape[0]
        tt = t.reshape(-1).float().expand(b) if t.numel() == 1 else t.reshape(-1).float()
        temb = self.time_embedding(timestep_embedding(tt, self.cfg.block_out_channels[0]).to(dt))
        temb = temb + text_emb.to(dt)
        if self.cfg.noise_level_cond and noise_level is not None:
            nl = noise_level.reshape(-1).float().expand(b) if noise_level.numel() == 1 else noise_level.reshape(-1)
            temb = temb + self.class_embedding(timestep_embedding(nl.float(), self.cfg.block_out_channels[0]).to(dt))
        kv = iter(text_kv)
        h = self.conv_in(x.to(dt))
        skips = [h]
        for blk in self.down:
            for j, r in enumerate(blk.resnets):
                h = r(h, temb)
                if blk.attentions is not None:
                    h = blk.attentions[j](h, next(kv))
                skips.append(h)
            if blk.downsampler is not None:
                h = blk.downsampler(h, temb)
                skips.append(h)
        h = self.mid.resnets[0](h, temb)
        h = self.mid.attention(h, next(kv))
        h = self.mid.resnets[1](h, temb)
        for blk in self.up:
            for j, r in enumerate(blk.resnets):
                h = r(torch.cat([h, skips.pop()], -1), temb)
                if blk.attentions is not None:
                    h = blk.attentions[j](h, next(kv))
            if blk.upsampler is not None:
                h = blk.upsampler(h, temb)
        h = self.conv_norm_out(h, silu=True)
        return self.conv_out(h)
