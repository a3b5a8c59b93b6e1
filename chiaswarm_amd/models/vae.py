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

    def decode(self, z):
        """z: NHWC latents (already divided by scaling_factor) -> NHWC [-1, 1] image."""
        z = z.to(self.post_quant_conv.weight.dtype)
        return self.decoder(self.post_quant_conv(z))

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
