"""AutoencoderKL (SD VAE, f=8) on NHWC bf16.

Decoder = the single largest kernel sequence after the denoise loop (SURVEY
§3.2, K15/K16); the encoder serves img2img / inpaint / pix2pix image latents
(K17, swarm/job_arguments.py:112-131).  Post-processing to uint8 HWC is fused
into one kernel (``ops.hip_ops.vae_postprocess``) so only uint8 crosses PCIe.
"""
from __future__ import annotations

import dataclasses
from typing import Sequence

import torch
import torch.nn as nn

from .layers import Conv2d, Downsample2D, GroupNorm, Prepared, ResnetBlock2D, SpatialSelfAttention, Upsample2D


@dataclasses.dataclass
class VAEConfig:
    in_channels: int = 3
    out_channels: int = 3
    latent_channels: int = 4
    block_out_channels: Sequence[int] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    scaling_factor: float = 0.18215


SD_VAE = VAEConfig()
SDXL_VAE = dataclasses.replace(SD_VAE, scaling_factor=0.13025)
TINY_VAE = VAEConfig(block_out_channels=(32, 32, 32, 32), layers_per_block=1)
# AudioLDM mel-spectrogram VAE: 1 channel in/out, 8 latent channels, f=4
AUDIOLDM_VAE = VAEConfig(in_channels=1, out_channels=1, latent_channels=8, block_out_channels=(128, 256, 512),
                         scaling_factor=0.9227914)
TINY_AUDIO_VAE = VAEConfig(in_channels=1, out_channels=1, latent_channels=8, block_out_channels=(32, 32, 32),
                           layers_per_block=1, scaling_factor=0.9227914)


class _MidBlock(nn.Module):
    def __init__(self, c, g):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(c, c, None, g, 1e-6), ResnetBlock2D(c, c, None, g, 1e-6)])
        self.attentions = nn.ModuleList([SpatialSelfAttention(c, g, 1e-6)])

    def forward(self, x):
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class _UpDecBlock(nn.Module):
    def __init__(self, cin, cout, n, g, upsample):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, None, g, 1e-6) for i in range(n)])
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if upsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class _DownEncBlock(nn.Module):
    def __init__(self, cin, cout, n, g, downsample):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, None, g, 1e-6) for i in range(n)])
        self.downsamplers = nn.ModuleList([Downsample2D(cout, padding=0)]) if downsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
        return x


class Decoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch = list(cfg.block_out_channels)
        g = cfg.norm_num_groups
        self.conv_in = Conv2d(cfg.latent_channels, ch[-1], 3, padding=1)
        self.mid_block = _MidBlock(ch[-1], g)
        rch = list(reversed(ch))
        self.up_blocks = nn.ModuleList()
        cout = rch[0]
        for i in range(len(ch)):
            cin, cout = cout, rch[i]
            self.up_blocks.append(_UpDecBlock(cin, cout, cfg.layers_per_block + 1, g, i != len(ch) - 1))
        self.conv_norm_out = GroupNorm(g, ch[0], eps=1e-6)
        self.conv_out = Conv2d(ch[0], cfg.out_channels, 3, padding=1)

    def forward(self, z):
        h = self.conv_in(z, gn_stats=True)  # the mid-block norm1 statistics
        h = self.mid_block(h)
        for blk in self.up_blocks:
            h = blk(h)
        h = self.conv_norm_out(h, silu=True)
        return self.conv_out(h)


class Encoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch = list(cfg.block_out_channels)
        g = cfg.norm_num_groups
        self.conv_in = Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i in range(len(ch)):
            cin, cout = cout, ch[i]
            self.down_blocks.append(_DownEncBlock(cin, cout, cfg.layers_per_block, g, i != len(ch) - 1))
        self.mid_block = _MidBlock(ch[-1], g)
        self.conv_norm_out = GroupNorm(g, ch[-1], eps=1e-6)
        self.conv_out = Conv2d(ch[-1], 2 * cfg.latent_channels, 3, padding=1)

    def forward(self, x):
        h = self.conv_in(x)
        for blk in self.down_blocks:
            h = blk(h)
        h = self.mid_block(h)
        h = self.conv_norm_out(h, silu=True)
        return self.conv_out(h)


class AutoencoderKL(Prepared):
    def __init__(self, cfg: VAEConfig = SD_VAE, with_encoder=True):
        super().__init__()
        self.cfg = cfg
        self.decoder = Decoder(cfg)
        self.post_quant_conv = Conv2d(cfg.latent_channels, cfg.latent_channels, 1, padding=0)
        if with_encoder:
            self.encoder = Encoder(cfg)
            self.quant_conv = Conv2d(2 * cfg.latent_channels, 2 * cfg.latent_channels, 1, padding=0)
        else:  # decoder-only: a full checkpoint's encoder tensors are expected extras
            self.checkpoint_ignore = ("encoder.", "quant_conv.")

    # Output pixels per decode call above which the decoder runs one sample at a
    # time (slicing) and in overlapping spatial tiles (tiling) — the reference
    # turns diffusers' enable_vae_slicing / enable_vae_tiling on for low-memory
    # GPUs (swarm/diffusion/diffusion_func.py:89-92).  With 288 GB of HBM a
    # whole 4 x 2048^2 decode fits, so only larger outputs take this path.
    SLICE_PIXELS = 4 * 2048 * 2048
    TILE_PIXELS = 4096 * 4096

    @property
    def upscale(self) -> int:
        return 2 ** (len(self.cfg.block_out_channels) - 1)

    def _decode_full(self, z):
        z = z.to(self.post_quant_conv.weight.dtype)
        return self.decoder(self.post_quant_conv(z))

    def decode(self, z):
        """z: NHWC latents (already divided by scaling_factor) -> NHWC [-1, 1] image."""
        B, h, w = z.shape[0], z.shape[1], z.shape[2]
        px = h * w * self.upscale * self.upscale
        if px > self.TILE_PIXELS:
            return torch.cat([self.tiled_decode(z[i:i + 1]) for i in range(B)])
        if B > 1 and B * px > self.SLICE_PIXELS:
            return torch.cat([self._decode_full(z[i:i + 1]) for i in range(B)])
        return self._decode_full(z)

    def tiled_decode(self, z, tile: int = 64, overlap: float = 0.25):
        """Decode in ``tile``-latent tiles overlapping by ``overlap``: each tile
        is linearly cross-faded into its upper and left neighbours over the
        overlap and cropped to the stride (diffusers' tiled VAE decode
        semantics, NHWC).  Bounded memory for arbitrarily large outputs."""
        f = self.upscale
        stride = max(1, int(tile * (1 - overlap)))
        blend = int(tile * f * overlap)
        keep = tile * f - blend
        H, W = z.shape[1], z.shape[2]
        rows = [[self._decode_full(z[:, i:i + tile, j:j + tile]) for j in range(0, W, stride)]
                for i in range(0, H, stride)]
        out_rows = []
        for i, row in enumerate(rows):
            res = []
            for j, t in enumerate(row):
                # in place, as diffusers: a tile's neighbours below / to the right
                # blend against its already cross-faded pixels
                if i > 0:
                    _blend_(rows[i - 1][j], t, blend, dim=1)
                if j > 0:
                    _blend_(row[j - 1], t, blend, dim=2)
                res.append(t[:, :keep, :keep])
            out_rows.append(torch.cat(res, dim=2))
        return torch.cat(out_rows, dim=1)[:, :H * f, :W * f]

    def encode(self, x, generator=None, sample=True):
        """x: NHWC [-1, 1] image -> NHWC latents (NOT yet scaled)."""
        h = self.encoder(x.to(self.quant_conv.weight.dtype))
        moments = self.quant_conv(h).float()
        c = self.cfg.latent_channels
        mean, logvar = moments[..., :c], moments[..., c:].clamp(-30.0, 20.0)
        if not sample:
            return mean
        std = torch.exp(0.5 * logvar)
        noise = torch.randn(mean.shape, generator=generator, device=mean.device, dtype=torch.float32)
        return mean + std * noise


def _blend_(a, b, extent, dim):
    """In place: the first ``extent`` rows (dim 1) / columns (dim 2) of b
    cross-faded from the trailing ``extent`` of its neighbour ``a`` (weight
    y / extent on b)."""
    e = min(a.shape[dim], b.shape[dim], extent)
    if e <= 0:
        return b
    w = torch.arange(e, device=b.device, dtype=torch.float32) / e
    shape = [1, 1, 1, 1]
    shape[dim] = e
    w = w.view(shape)
    tail = a.narrow(dim, a.shape[dim] - e, e).float()
    head = b.narrow(dim, 0, e).float()
    b.narrow(dim, 0, e).copy_((tail * (1 - w) + head * w).to(b.dtype))
    return b
