"""K-diffusion UNet of stabilityai/sd-x2-latent-upscaler on NHWC bf16.

The latent upscaler the reference runs for the ``upscale`` job option
(swarm/diffusion/upscale.py:8-30, diffusers ``StableDiffusionLatentUpscalePipeline``)
is Katherine Crowson's k-diffusion ``image_v1`` denoiser, published in diffusers
as a ``UNet2DConditionModel`` built from K blocks.  Architecture (k-diffusion
semantics, which are what the weights were trained as):

  * conditioning: Fourier features of ``c_noise = log(sigma) / 4`` plus a
    bias-free projection of the 896-d mapping condition (128-d low-res noise
    embedding + 768-d pooled CLIP-L text), then a 2-layer GELU MLP
    (``time_embedding``: cond_proj, linear_1, linear_2, post-GELU);
  * every normalisation is an AdaGroupNorm: GroupNorm with ``C / 32`` groups
    and a per-sample affine ``x * (1 + scale) + shift`` predicted from the
    mapping output;
  * ResnetBlockCondNorm2D: AdaGN, GELU, 3x3 conv, AdaGN, GELU, 3x3 conv, plus a
    bias-free 1x1 shortcut when the width changes;
  * KAttentionBlock: optional AdaGN self-attention, then AdaGN cross-attention
    on LayerNorm'd text states (``attn2.norm_cross``), head size 64, biased
    projections;
  * K down/upsampling: a fixed depthwise [1, 3, 3, 1]/8 binomial filter with
    reflect padding (no parameters);
  * down levels 384 / 384 / 768 with 2 / 4 / 4 layers (cross-attention on the
    two lower levels, self-attention on the lowest), mirrored up levels fed
    with the pre-downsample skips of the two upper levels, 1x1 conv_in (8 = 4
    noisy + 4 low-res latent channels) and conv_out (4 + 1 variance channel,
    dropped).

MI355X structure: every AdaGN mapper of a step is ONE batched GEMM (its "+1"
folded into the bias) whose [B, 2C] row slices feed the GroupNorm kernel's
per-sample affine in place; GN + affine + GELU is one kernel; conv residuals
are fused into conv2's epilogue; cross-attention K/V of the fixed prompt are
computed once per request (``encode_context``).

Checkpoint key layout follows diffusers' K-block naming (``down_blocks.N.
resnets.M.norm1.linear``, ``attentions.M.attn2.norm_cross`` ...) as far as it
can be reconstructed offline; the published checkpoint is not available here,
so key-level parity with it is unpinned — ``load_into`` is strict and reports
any mismatch loudly.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from .layers import Attention, Conv2d, LayerNorm, Linear, Prepared


@dataclasses.dataclass
class KUNetConfig:
    in_channels: int = 8
    out_channels: int = 5  # 4 + the unused variance channel
    block_out_channels: Sequence[int] = (384, 384, 768)
    layers_per_block: Sequence[int] = (2, 4, 4)
    cross_attn: Sequence[bool] = (False, True, True)
    self_attn: Sequence[bool] = (False, False, True)
    attention_head_dim: int = 64
    cross_attention_dim: int = 768
    time_cond_proj_dim: int = 896
    group_size: int = 32
    eps: float = 1e-5
    sample_size: int = 96

    @property
    def temb_dim(self):
        return 2 * self.block_out_channels[0]


LATENT_X2_K = KUNetConfig()
TINY_X2_K = KUNetConfig(block_out_channels=(32, 32, 64), layers_per_block=(1, 2, 2), attention_head_dim=16,
                        cross_attention_dim=32, time_cond_proj_dim=64 + 32, group_size=8, sample_size=8)


class AdaGroupNorm(nn.Module):
    """GroupNorm whose affine comes from the time embedding (key ``linear``).
    The model computes every mapper at once; ``forward`` receives this norm's
    [B, 2C] row block (scale + 1 | shift)."""

    def __init__(self, temb_dim, channels, groups, eps):
        super().__init__()
        self.linear = Linear(temb_dim, 2 * channels)
        self.channels, self.groups, self.eps = channels, groups, eps

    def forward(self, x, ss, act="gelu"):
        c = self.channels
        return ops.group_norm(x, ss[:, :c], ss[:, c:], self.groups, self.eps, silu=act)


class ResnetBlockCondNorm2D(nn.Module):
    def __init__(self, cin, cmid, cout, temb_dim, group_size, eps):
        super().__init__()
        self.norm1 = AdaGroupNorm(temb_dim, cin, max(1, cin // group_size), eps)
        self.conv1 = Conv2d(cin, cmid, 3, padding=1)
        self.norm2 = AdaGroupNorm(temb_dim, cmid, max(1, cmid // group_size), eps)
        self.conv2 = Conv2d(cmid, cout, 3, padding=1)
        self.conv_shortcut = Conv2d(cin, cout, 1, bias=False) if cin != cout else None

    def norms(self):
        return [self.norm1, self.norm2]

    def forward(self, x, ss):
        h = self.norm1(x, next(ss))
        h = self.conv1(h, gn_stats=True)
        h = self.norm2(h, next(ss))
        sc = x if self.conv_shortcut is None else self.conv_shortcut(x)
        return self.conv2(h, residual=sc, gn_stats=True)


class _NormedCrossAttention(Attention):
    """Cross-attention whose context goes through ``norm_cross`` (LayerNorm)."""

    def __init__(self, dim, heads, dim_head, cross_dim):
        super().__init__(dim, heads, dim_head, cross_dim=cross_dim, bias=True)
        self.norm_cross = LayerNorm(cross_dim)

    def context_kv(self, ctx):
        return super().context_kv(self.norm_cross(ctx))


class KAttentionBlock(nn.Module):
    def __init__(self, dim, dim_head, cross_dim, temb_dim, group_size, eps, self_attn):
        super().__init__()
        heads = max(1, dim // dim_head)
        groups = max(1, dim // group_size)
        self.add_self_attention = self_attn
        if self_attn:
            self.norm1 = AdaGroupNorm(temb_dim, dim, groups, eps)
            self.attn1 = Attention(dim, heads, dim_head, bias=True)
        self.norm2 = AdaGroupNorm(temb_dim, dim, groups, eps)
        self.attn2 = _NormedCrossAttention(dim, heads, dim_head, cross_dim)

    def norms(self):
        return ([self.norm1] if self.add_self_attention else []) + [self.norm2]

    def forward(self, x, ss, kv, ctx=None):
        b, hh, ww, c = x.shape
        if self.add_self_attention:
            hn = self.norm1(x, next(ss), act=None).view(b, hh * ww, c)
            x = self.attn1(hn, residual=x.view(b, hh * ww, c)).view(b, hh, ww, c)
        hn = self.norm2(x, next(ss), act=None).view(b, hh * ww, c)
        a2 = self.attn2
        out = a2.attend_q(a2.to_q(hn), kv, ctx, residual=x.view(b, hh * ww, c))
        return out.view(b, hh, ww, c)


def _binomial_kernel(c, scale=1.0):
    k1 = torch.tensor([1.0, 3.0, 3.0, 1.0]) / 8.0 * scale
    return (k1[:, None] * k1[None, :]).expand(c, 1, 4, 4).contiguous()


class KDownsample2D(nn.Module):
    """Depthwise [1,3,3,1]/8 binomial filter, reflect pad 1, stride 2 (no
    checkpoint params; the filter is a non-persistent buffer so it moves with
    the model and never needs a host copy inside a captured graph).  A fixed
    16-tap depthwise filter: MIOpen's grouped conv, not worth an MFMA tile."""

    def __init__(self, channels):
        super().__init__()
        self.register_buffer("kernel", _binomial_kernel(channels), persistent=False)

    def forward(self, x):
        c = x.shape[-1]
        xn = F.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect")
        y = F.conv2d(xn, self.kernel.to(x.dtype), stride=2, groups=c)
        return y.permute(0, 2, 3, 1).contiguous()


class KUpsample2D(nn.Module):
    """Transposed depthwise binomial filter (x2 gain), reflect pad 1, stride 2."""

    def __init__(self, channels):
        super().__init__()
        self.register_buffer("kernel", _binomial_kernel(channels, 2.0), persistent=False)

    def forward(self, x):
        c = x.shape[-1]
        xn = F.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1), mode="reflect")
        y = F.conv_transpose2d(xn, self.kernel.to(x.dtype), stride=2, padding=3, groups=c)
        return y.permute(0, 2, 3, 1).contiguous()


class KTimestepEmbedding(nn.Module):
    """Mapping network: (fourier(c_noise) + cond_proj(cond)) -> Linear-GELU-Linear-GELU."""

    def __init__(self, dim, cond_dim):
        super().__init__()
        self.cond_proj = Linear(cond_dim, dim, bias=False)
        self.linear_1 = Linear(dim, dim)
        self.linear_2 = Linear(dim, dim)

    def forward(self, emb, cond):
        h = self.cond_proj(cond, residual=emb)
        return self.linear_2(self.linear_1(h, act="gelu"), act="gelu")


class GaussianFourierProjection(nn.Module):
    def __init__(self, size):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(size), requires_grad=False)

    def forward(self, t):
        f = t.float()[:, None] * self.weight.float()[None, :] * (2 * math.pi)
        return torch.cat([torch.cos(f), torch.sin(f)], dim=-1)


class _KBlock(nn.Module):
    def __init__(self, resnets, attentions, sampler_attr, sampler):
        super().__init__()
        self.resnets = nn.ModuleList(resnets)
        self.attentions = nn.ModuleList(attentions) if attentions else None
        setattr(self, sampler_attr, nn.ModuleList([sampler]) if sampler is not None else None)


class KUNet2DConditionModel(Prepared):
    def __init__(self, cfg: KUNetConfig = LATENT_X2_K):
        super().__init__()
        self.cfg = cfg
        ch = list(cfg.block_out_channels)
        n = len(ch)
        td, gs, eps = cfg.temb_dim, cfg.group_size, cfg.eps

        def res(ci, cm, co):
            return ResnetBlockCondNorm2D(ci, cm, co, td, gs, eps)

        def att(c, i):
            if not cfg.cross_attn[i]:
                return None
            return KAttentionBlock(c, cfg.attention_head_dim, cfg.cross_attention_dim, td, gs, eps,
                                   cfg.self_attn[i])

        self.conv_in = Conv2d(cfg.in_channels, ch[0], 1)
        self.time_proj = GaussianFourierProjection(td // 2)
        self.time_embedding = KTimestepEmbedding(td, cfg.time_cond_proj_dim)

        # down: level i runs at ch[i]; the downsample that k-diffusion puts at the
        # START of level i+1 sits at the END of block i (diffusers layout)
        self.down_blocks = nn.ModuleList()
        for i in range(n):
            cin = ch[max(0, i - 1)]
            rs = [res(cin if j == 0 else ch[i], ch[i], ch[i]) for j in range(cfg.layers_per_block[i])]
            ats = [att(ch[i], i) for _ in rs] if cfg.cross_attn[i] else None
            self.down_blocks.append(_KBlock(rs, ats, "downsamplers", KDownsample2D(ch[i]) if i < n - 1 else None))

        # up (lowest level first): level i takes [h | skip_i] except the first,
        # mid width ch[i], last layer narrows to ch[i-1]
        self.up_blocks = nn.ModuleList()
        for k, i in enumerate(reversed(range(n))):
            cin = ch[i] if k == 0 else 2 * ch[i]
            cout = ch[max(0, i - 1)]
            nl = cfg.layers_per_block[i]
            rs, ats = [], []
            for j in range(nl):
                last = j == nl - 1
                rs.append(res(cin if j == 0 else ch[i], ch[i], cout if last else ch[i]))
                ats.append(att(cout if last else ch[i], i))
            self.up_blocks.append(_KBlock(rs, ats if cfg.cross_attn[i] else None, "upsamplers",
                                          KUpsample2D(cout) if i > 0 else None))
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 1)

    # ------------------------------------------------------------------
    def _norms(self):
        out = []
        for blk in list(self.down_blocks) + list(self.up_blocks):
            for j, r in enumerate(blk.resnets):
                out.extend(r.norms())
                if blk.attentions is not None:
                    out.extend(blk.attentions[j].norms())
        return out

    def prepare_self(self):
        """All AdaGN mappers of a step as one [sum 2C, Temb] GEMM; the "+1" of
        ``1 + scale`` is folded into its bias."""
        norms = self._norms()
        self._ada_w = torch.cat([m.linear.weight for m in norms], 0).detach()
        bs = []
        for m in norms:
            b = m.linear.bias.detach().float().clone()
            b[:m.channels] += 1.0
            bs.append(b)
        self._ada_b = torch.cat(bs).to(self._ada_w.dtype)
        self._ada_splits = [2 * m.channels for m in norms]

    def _ada(self, temb):
        w = getattr(self, "_ada_w", None)
        if w is None or w.device != temb.device or w.dtype != self.conv_in.weight.dtype:
            self.prepare_self()
        proj = ops.gemm(temb, self._ada_w, self._ada_b)
        return iter(torch.split(proj, self._ada_splits, dim=-1))

    def cross_attention_modules(self):
        mods = []
        for blk in list(self.down_blocks) + list(self.up_blocks):
            if blk.attentions is not None:
                mods.extend(a.attn2 for a in blk.attentions)
        return mods

    @torch.no_grad()
    def encode_context(self, ctx: torch.Tensor):
        """Per-request K/V of every cross-attention (constant over steps)."""
        return [m.context_kv(ctx) for m in self.cross_attention_modules()]

    def time_embed(self, c_noise, cond):
        dtype = self.conv_in.weight.dtype
        emb = self.time_proj(c_noise).to(dtype)
        return self.time_embedding(emb, cond.to(dtype))

    def forward(self, sample, c_noise, cond, cross_kv=None, encoder_hidden_states=None, drop_variance=True):
        """sample: NHWC [B, H, W, 8] (scaled noisy latents | low-res latents);
        ``c_noise``: [B] = log(sigma) / 4; ``cond``: [B, 896] mapping condition.
        Returns the NHWC network output F (k-diffusion; the caller applies the
        Karras preconditioning): [B, H, W, 4], or all 5 channels (with the
        unused variance channel, which is otherwise never computed)."""
        dtype = self.conv_in.weight.dtype
        x = sample.to(dtype)
        ss = self._ada(self.time_embed(c_noise.reshape(-1).expand(x.shape[0]), cond))
        kv_iter = iter(cross_kv) if cross_kv is not None else None
        ctx = encoder_hidden_states

        def attn(a, h):
            return a(h, ss, next(kv_iter) if kv_iter is not None else None, ctx)

        h = self.conv_in(x)
        skips = []
        for blk in self.down_blocks:
            for j, r in enumerate(blk.resnets):
                h = r(h, ss)
                if blk.attentions is not None:
                    h = attn(blk.attentions[j], h)
            skips.append(h)
            if blk.downsamplers is not None:
                h = blk.downsamplers[0](h)
        for k, blk in enumerate(self.up_blocks):
            skip = skips.pop()
            if k > 0:
                h = ops.cat_channels(h, skip)
            for j, r in enumerate(blk.resnets):
                h = r(h, ss)
                if blk.attentions is not None:
                    h = attn(blk.attentions[j], h)
            if blk.upsamplers is not None:
                h = blk.upsamplers[0](h)
        if not drop_variance:
            return self.conv_out(h)
        co = self.conv_out
        n = self.cfg.out_channels - 1
        return ops.gemm(h, co.weight[:n].reshape(n, -1), co.bias[:n])
