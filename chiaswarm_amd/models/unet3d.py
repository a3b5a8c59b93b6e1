"""UNet3DConditionModel (ModelScope text-to-video, damo-vilab/text-to-video-ms-1.7b)
on NHWC bf16 frames.  Reference call site: the txt2vid pipeline at
swarm/video/tx2vid.py:24-55.

Layout: video latents are [B*F, h, w, C] (frames folded into the batch), so
every spatial op (ResNet convs, GroupNorm, spatial transformer) is the image
kernel unchanged.  Temporal ops reuse them by re-viewing the same memory:
  * TemporalConvLayer (Conv3d (3,1,1)) = the implicit-GEMM conv on the
    [B, F, h*w, C] view with a 3x1 kernel (no copy);
  * TransformerTemporalModel = GroupNorm over [B, F*h*w, C] + attention over
    the F frames of every pixel ([B*h*w, F, C] tokens).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import (BasicTransformerBlock, Conv2d, Downsample2D, GroupNorm, Linear, Prepared, ResnetBlock2D,
                     TimestepEmbedding, Transformer2D, Upsample2D, timestep_embedding)
from .unet import UNetConfig

T2V = UNetConfig(num_heads=(5, 10, 20, 20), cross_attention_dim=1024, use_linear_projection=False,
                 down_block_types=("CrossAttnDownBlock3D",) * 3 + ("DownBlock3D",),
                 up_block_types=("UpBlock3D",) + ("CrossAttnUpBlock3D",) * 3)
TINY_T2V = UNetConfig(block_out_channels=(32, 64), layers_per_block=1, num_heads=(2, 2), cross_attention_dim=32,
                      use_linear_projection=False,
                      down_block_types=("CrossAttnDownBlock3D", "DownBlock3D"),
                      up_block_types=("UpBlock3D", "CrossAttnUpBlock3D"))


class TemporalConvLayer(nn.Module):
    def __init__(self, cin, cout=None, groups=32):
        super().__init__()
        cout = cout or cin
        self.conv1 = nn.ModuleList([GroupNorm(groups, cin), nn.Identity(), Conv2d(cin, cout, (3, 1), padding=0)])
        self.conv2 = nn.ModuleList([GroupNorm(groups, cout), nn.Identity(), Conv2d(cout, cout, (3, 1), padding=0)])
        self.conv3 = nn.ModuleList([GroupNorm(groups, cout), nn.Identity(), Conv2d(cout, cout, (3, 1), padding=0)])
        self.conv4 = nn.ModuleList([GroupNorm(groups, cout), nn.Identity(), Conv2d(cout, cout, (3, 1), padding=0)])

    def forward(self, x, frames):
        bf, h, w, c = x.shape
        b = bf // frames
        v = x.view(b, frames, h * w, c)  # temporal view: "image" of height F, width h*w
        hcur = v
        for i, blk in enumerate((self.conv1, self.conv2, self.conv3, self.conv4)):
            n = blk[0](hcur.reshape(b, frames * h * w, -1), silu=True).view(b, frames, h * w, -1)
            hcur = blk[2](n, padding=(1, 0, 1, 0), residual=v if i == 3 else None)
        return hcur.view(bf, h, w, c)


class TransformerTemporal(nn.Module):
    def __init__(self, channels, heads, dim_head=64, groups=32, layers=1):
        super().__init__()
        inner = heads * dim_head
        self.norm = GroupNorm(groups, channels, eps=1e-6)
        self.proj_in = Linear(channels, inner)
        self.transformer_blocks = nn.ModuleList([_TemporalBlock(inner, heads, dim_head) for _ in range(layers)])
        self.proj_out = Linear(inner, channels)

    def forward(self, x, frames):
        bf, h, w, c = x.shape
        b = bf // frames
        n = self.norm(x.view(b, frames * h * w, c))
        t = n.view(b, frames, h * w, c).transpose(1, 2).reshape(b * h * w, frames, c)
        t = self.proj_in(t)
        for blk in self.transformer_blocks:
            t = blk(t)
        t = self.proj_out(t)
        t = t.view(b, h * w, frames, c).transpose(1, 2).reshape(bf, h, w, c)
        return ops.add(t.contiguous(), x)


class _TemporalBlock(BasicTransformerBlock):
    """attn1 and attn2 both self-attention over frames (double_self_attention)."""

    def __init__(self, dim, heads, dim_head):
        super().__init__(dim, heads, dim_head, cross_dim=None)
        from .layers import Attention

        self.attn2 = Attention(dim, heads, dim_head)

    def forward(self, x, ctx=None, kv=None, row_stats=None):
        x = self.attn1(self.norm1(x), residual=x)
        x = self.attn2(self.norm2(x), residual=x)
        return self.ff(self.norm3(x), residual=x)


class _Block3D(nn.Module):
    def __init__(self, resnets, temp_convs, attentions, temp_attentions, sampler_attr, sampler):
        super().__init__()
        self.resnets = nn.ModuleList(resnets)
        self.temp_convs = nn.ModuleList(temp_convs)
        self.attentions = nn.ModuleList(attentions) if attentions else None
        self.temp_attentions = nn.ModuleList(temp_attentions) if temp_attentions else None
        setattr(self, sampler_attr, nn.ModuleList([sampler]) if sampler is not None else None)


class UNet3DConditionModel(Prepared):
    def __init__(self, cfg: UNetConfig = T2V):
        super().__init__()
        self.cfg = cfg
        ch = list(cfg.block_out_channels)
        nb = len(ch)
        temb_dim = ch[0] * 4
        g = cfg.norm_num_groups
        heads = cfg.per_block(cfg.num_heads, nb)
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch[0], temb_dim)
        self.transformer_in = TransformerTemporal(ch[0], max(1, ch[0] // 64), 64, g)

        def cross(c, i):
            return Transformer2D(c, heads[i], cfg.cross_attention_dim, 1, cfg.use_linear_projection, g)

        def temporal(c):
            return TransformerTemporal(c, max(1, c // 64), 64, g)

        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i, bt in enumerate(cfg.down_block_types):
            cin, cout = cout, ch[i]
            attn = bt.startswith("CrossAttn")
            n = cfg.layers_per_block
            self.down_blocks.append(_Block3D(
                [ResnetBlock2D(cin if j == 0 else cout, cout, temb_dim, g) for j in range(n)],
                [TemporalConvLayer(cout) for _ in range(n)],
                [cross(cout, i) for _ in range(n)] if attn else None,
                [temporal(cout) for _ in range(n)] if attn else None,
                "downsamplers", None if i == nb - 1 else Downsample2D(cout)))
        c = ch[-1]
        self.mid_block = _Block3D([ResnetBlock2D(c, c, temb_dim, g), ResnetBlock2D(c, c, temb_dim, g)],
                                  [TemporalConvLayer(c), TemporalConvLayer(c)], [cross(c, nb - 1)], [temporal(c)],
                                  "upsamplers", None)
        rch = list(reversed(ch))
        rheads = list(reversed(heads))
        self.up_blocks = nn.ModuleList()
        out_c = rch[0]
        for i, bt in enumerate(cfg.up_block_types):
            prev, out_c = out_c, rch[i]
            in_c = rch[min(i + 1, nb - 1)]
            n = cfg.layers_per_block + 1
            attn = bt.startswith("CrossAttn")
            res = [ResnetBlock2D((prev if j == 0 else out_c) + (in_c if j == n - 1 else out_c), out_c, temb_dim, g)
                   for j in range(n)]
            self.up_blocks.append(_Block3D(
                res, [TemporalConvLayer(out_c) for _ in range(n)],
                [Transformer2D(out_c, rheads[i], cfg.cross_attention_dim, 1, cfg.use_linear_projection, g)
                 for _ in range(n)] if attn else None,
                [temporal(out_c) for _ in range(n)] if attn else None,
                "upsamplers", None if i == nb - 1 else Upsample2D(out_c)))
        self.conv_norm_out = GroupNorm(g, ch[0], eps=1e-5)
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3, padding=1)

    def cross_attention_modules(self):
        mods = []
        for blk in list(self.down_blocks) + [self.mid_block] + list(self.up_blocks):
            if blk.attentions is not None:
                for t in blk.attentions:
                    mods.extend(t.cross_modules())
        return mods

    @torch.no_grad()
    def encode_context(self, ctx, frames):
        """ctx [B, 77, D] -> per-layer K/V repeated for every frame."""
        ctx_f = ctx.repeat_interleave(frames, dim=0)
        return [m.context_kv(ctx_f) for m in self.cross_attention_modules()]

    def forward(self, sample, timestep, frames, cross_kv):
        """sample: [B*F, h, w, C]."""
        bf = sample.shape[0]
        dtype = self.conv_in.weight.dtype
        t = timestep.reshape(-1).float()
        t = t.expand(bf) if t.numel() == 1 else t.repeat_interleave(frames)
        temb = ops.silu(self.time_embedding(timestep_embedding(t, self.cfg.block_out_channels[0]).to(dtype)))
        kv_iter = iter(cross_kv)

        def attn(blk, j, h):
            if blk.attentions is None:
                return h
            h = blk.attentions[j](h, kvs=[next(kv_iter)])
            return blk.temp_attentions[j](h, frames)

        h = self.conv_in(sample.to(dtype))
        h = self.transformer_in(h, frames)
        skips = [h]
        for blk in self.down_blocks:
            for j, r in enumerate(blk.resnets):
                h = r(h, r.time_emb_proj(temb))
                h = blk.temp_convs[j](h, frames)
                h = attn(blk, j, h)
                skips.append(h)
            if blk.downsamplers is not None:
                h = blk.downsamplers[0](h)
                skips.append(h)
        m = self.mid_block
        h = m.resnets[0](h, m.resnets[0].time_emb_proj(temb))
        h = m.temp_convs[0](h, frames)
        h = attn(m, 0, h)
        h = m.resnets[1](h, m.resnets[1].time_emb_proj(temb))
        h = m.temp_convs[1](h, frames)
        for blk in self.up_blocks:
            for j, r in enumerate(blk.resnets):
                h = r(torch.cat([h, skips.pop()], dim=-1), r.time_emb_proj(temb))
                h = blk.temp_convs[j](h, frames)
                h = attn(blk, j, h)
            if blk.upsamplers is not None:
                h = blk.upsamplers[0](h)
        h = self.conv_norm_out(h, silu=True)
        return self.conv_out(h)
