"""ControlNetModel (SD1.5 / SD2.x geometry) on NHWC bf16.

Reference: ControlNetModel.from_pretrained at swarm/diffusion/diffusion_func.py:29-34
and the StableDiffusionControlNetPipeline call at :96.  diffusers key layout:
``controlnet_cond_embedding.{conv_in,blocks.N,conv_out}``, the UNet-encoder copy
(``conv_in``, ``time_embedding``, ``down_blocks``, ``mid_block``), and the zero
1x1 convs ``controlnet_down_blocks.N`` / ``controlnet_mid_block``.

The 13 zero-conv residuals are returned already multiplied by the
conditioning scale (folded into one GEMM epilogue scale: the zero-conv weights
and bias are pre-scaled once per job instead of scaling every step's tensors).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .layers import Conv2d, Downsample2D, Prepared, ResnetBlock2D, TimestepEmbedding, Transformer2D, timestep_embedding
from .unet import SD15, UNetConfig, _Block
from .. import ops


def _spatial_mean(x):
    """NHWC [B, H, W, C] -> [B, 1, 1, C] (fp32 accumulation)."""
    return x.float().mean(dim=(1, 2), keepdim=True).to(x.dtype).contiguous()


class CondEmbedding(nn.Module):
    def __init__(self, out_ch=320, channels=(16, 32, 96, 256), cin=3):
        super().__init__()
        self.conv_in = Conv2d(cin, channels[0], 3, padding=1)
        blocks = []
        for i in range(len(channels) - 1):
            blocks.append(Conv2d(channels[i], channels[i], 3, padding=1))
            blocks.append(Conv2d(channels[i], channels[i + 1], 3, padding=1, stride=2))
        self.blocks = nn.ModuleList(blocks)
        self.conv_out = Conv2d(channels[-1], out_ch, 3, padding=1)

    def forward(self, x):
        h = ops.silu(self.conv_in(x))
        for b in self.blocks:
            h = ops.silu(b(h))
        return self.conv_out(h)


class ControlNetModel(Prepared):
    """``cond_channels`` / ``cond_in`` / ``bgr`` / ``global_pool``: the
    checkpoint config's ``conditioning_embedding_out_channels``,
    ``conditioning_channels``, ``controlnet_conditioning_channel_order`` and
    ``global_pool_conditions`` (shuffle ControlNets average every residual over
    the image, diffusers ControlNetModel.forward)."""

    def __init__(self, cfg: UNetConfig = SD15, cond_channels=(16, 32, 96, 256), cond_in: int = 3,
                 bgr: bool = False, global_pool: bool = False):
        super().__init__()
        self.cfg = cfg
        self.bgr, self.global_pool = bgr, global_pool
        ch = list(cfg.block_out_channels)
        nb = len(ch)
        heads = cfg.per_block(cfg.num_heads, nb)
        tl = cfg.per_block(cfg.transformer_layers_per_block, nb)
        temb_dim = ch[0] * 4
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch[0], temb_dim)
        self.controlnet_cond_embedding = CondEmbedding(ch[0], tuple(cond_channels), cond_in)
        self.down_blocks = nn.ModuleList()
        zero = [Conv2d(ch[0], ch[0], 1, padding=0)]
        cout = ch[0]
        for i, bt in enumerate(cfg.down_block_types):
            cin, cout = cout, ch[i]
            final = i == nb - 1
            res = [ResnetBlock2D(cin if j == 0 else cout, cout, temb_dim, g, eps) for j in range(cfg.layers_per_block)]
            att = ([Transformer2D(cout, heads[i], cfg.cross_attention_dim, tl[i], cfg.use_linear_projection, g)
                    for _ in range(cfg.layers_per_block)] if bt.startswith("CrossAttn") else None)
            self.down_blocks.append(_Block(res, att, "downsamplers", None if final else Downsample2D(cout)))
            zero.extend(Conv2d(cout, cout, 1, padding=0) for _ in range(cfg.layers_per_block))
            if not final:
                zero.append(Conv2d(cout, cout, 1, padding=0))
        self.controlnet_down_blocks = nn.ModuleList(zero)
        self.mid_block = _Block([ResnetBlock2D(ch[-1], ch[-1], temb_dim, g, eps),
                                 ResnetBlock2D(ch[-1], ch[-1], temb_dim, g, eps)],
                                [Transformer2D(ch[-1], heads[-1], cfg.cross_attention_dim, tl[-1],
                                               cfg.use_linear_projection, g)], "upsamplers", None)
        self.controlnet_mid_block = Conv2d(ch[-1], ch[-1], 1, padding=0)

    def zero_init_(self):
        with torch.no_grad():
            for m in list(self.controlnet_down_blocks) + [self.controlnet_mid_block]:
                m.weight.zero_()
                m.bias.zero_()

    def cross_attention_modules(self):
        mods = []
        for blk in list(self.down_blocks) + [self.mid_block]:
            if blk.attentions is not None:
                for t in blk.attentions:
                    mods.extend(t.cross_modules())
        return mods

    @torch.no_grad()
    def encode_context(self, ctx):
        return [m.context_kv(ctx) for m in self.cross_attention_modules()]

    def embed_cond(self, cond):
        """cond: NHWC [B, H, W, 3] in [0, 1] -> [B, H/8, W/8, C0] (constant per job)."""
        if self.bgr:
            cond = cond.flip(-1)
        return self.controlnet_cond_embedding(cond.to(self.conv_in.weight.dtype))

    def features(self, sample, timestep, cond_emb, cross_kv=None, ctx=None):
        """The ControlNet encoder copy up to (not including) its zero convs:
        (the 12 skip features, the mid-block output)."""
        return self._encode(sample, timestep, cond_emb, cross_kv, ctx)

    def merge_skip(self, i, feat, unet_skip, scale: float = 1.0):
        """UNet skip i + scale * zero_conv_i(feat) in ONE GEMM: the residual add
        and the conditioning scale ride in the 1x1 conv's epilogue (which also
        emits the GroupNorm statistics the consuming up-block ResNet needs).
        Global pooling: mean(zero_conv(f)) = zero_conv(mean(f)) (a 1x1 conv is
        affine), so the [B, 1, 1, C] residual broadcasts over the skip."""
        if self.global_pool:
            return unet_skip + scale * self.controlnet_down_blocks[i](_spatial_mean(feat)).to(unet_skip.dtype)
        return self.controlnet_down_blocks[i](feat, residual=unet_skip, out_scale=scale, gn_stats=True)

    def merge_mid(self, feat, unet_h, scale: float = 1.0):
        if self.global_pool:
            return unet_h + scale * self.controlnet_mid_block(_spatial_mean(feat)).to(unet_h.dtype)
        return self.controlnet_mid_block(feat, residual=unet_h, out_scale=scale, gn_stats=True)

    def forward(self, sample, timestep, cond_emb, cross_kv=None, ctx=None, scale: float = 1.0):
        """Residual tensors (diffusers ControlNetModel output: down residuals, mid residual)."""
        skips, h = self._encode(sample, timestep, cond_emb, cross_kv, ctx)
        if self.global_pool:
            skips, h = [_spatial_mean(s) for s in skips], _spatial_mean(h)
        downs = [zc(s) for zc, s in zip(self.controlnet_down_blocks, skips)]
        mid = self.controlnet_mid_block(h)
        if scale != 1.0:
            downs = [d * scale for d in downs]
            mid = mid * scale
        return downs, mid

    def _encode(self, sample, timestep, cond_emb, cross_kv=None, ctx=None):
        b = sample.shape[0]
        dtype = self.conv_in.weight.dtype
        t = timestep.reshape(-1).float()
        if t.numel() == 1:
            t = t.expand(b)
        temb = self.time_embedding(timestep_embedding(t, self.cfg.block_out_channels[0]).to(dtype))
        temb_s = ops.silu(temb)
        kv_iter = iter(cross_kv) if cross_kv is not None else None
        h = self.conv_in(sample.to(dtype), residual=cond_emb, gn_stats=True)
        skips = [h]
        for blk in self.down_blocks:
            for j, r in enumerate(blk.resnets):
                h = r(h, r.time_emb_proj(temb_s))
                if blk.attentions is not None:
                    t2 = blk.attentions[j]
                    kvs = [next(kv_iter) for _ in t2.transformer_blocks] if kv_iter else None
                    h = t2(h, ctx=ctx, kvs=kvs)
                skips.append(h)
            if blk.downsamplers is not None:
                h = blk.downsamplers[0](h)
                skips.append(h)
        m = self.mid_block
        h = m.resnets[0](h, m.resnets[0].time_emb_proj(temb_s))
        t2 = m.attentions[0]
        kvs = [next(kv_iter) for _ in t2.transformer_blocks] if kv_iter else None
        h = t2(h, ctx=ctx, kvs=kvs)
        h = m.resnets[1](h, m.resnets[1].time_emb_proj(temb_s))
        return skips, h
