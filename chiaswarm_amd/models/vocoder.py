"""HiFi-GAN vocoder (mel spectrogram -> 16 kHz waveform) for AudioLDM.

Geometry is the public ``SpeechT5HifiGan`` config shipped with
cvssp/audioldm (64 mel bins, upsample 5x4x2x2x2 = 160 samples per frame,
multi-receptive-field residual blocks with kernels 3/7/11 and dilations 1/3/5);
reached by the reference through ``AudioLDMPipeline`` (swarm/audio/audioldm.py:25).

MI355X path, all on token-layout [B, T, C] bf16 tensors:
  * every Conv1d is the implicit-GEMM conv kernel on the [B, 1, T, C] view
    (dilated taps are plain address offsets), with the LeakyReLU that follows
    it fused into its epilogue and the block residual fused as the epilogue's
    residual operand;
  * each ConvTranspose1d upsampler runs as ``stride`` polyphase convolutions
    that write interleaved output directly (``ops.pack_conv_transpose1d``);
  * the multi-receptive-field average and the LeakyReLU before the next
    upsampler are one fused ``axpby_nhwc`` pass; tanh is fused into conv_post.
"""
from __future__ import annotations

import dataclasses
from typing import Sequence

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv1d, ConvTranspose1d


@dataclasses.dataclass
class HifiGanConfig:
    model_in_dim: int = 64
    sampling_rate: int = 16000
    upsample_initial_channel: int = 1024
    upsample_rates: Sequence[int] = (5, 4, 2, 2, 2)
    upsample_kernel_sizes: Sequence[int] = (16, 16, 8, 4, 4)
    resblock_kernel_sizes: Sequence[int] = (3, 7, 11)
    resblock_dilation_sizes: Sequence[Sequence[int]] = ((1, 3, 5), (1, 3, 5), (1, 3, 5))
    normalize_before: bool = True

    @property
    def hop(self) -> int:
        h = 1
        for r in self.upsample_rates:
            h *= r
        return h


AUDIOLDM_HIFIGAN = HifiGanConfig()
TINY_HIFIGAN = HifiGanConfig(model_in_dim=16, upsample_initial_channel=64, upsample_rates=(4, 2),
                             upsample_kernel_sizes=(8, 4), resblock_kernel_sizes=(3, 5),
                             resblock_dilation_sizes=((1, 3), (1, 3)))


class HifiGanResidualBlock(nn.Module):
    def __init__(self, ch, k, dilations):
        super().__init__()
        self.convs1 = nn.ModuleList([Conv1d(ch, ch, k, dilation=d, padding=d * (k - 1) // 2) for d in dilations])
        self.convs2 = nn.ModuleList([Conv1d(ch, ch, k, dilation=1, padding=(k - 1) // 2) for _ in dilations])

    def forward(self, x, x_act):
        """x: block input; x_act = lrelu(x, 0.1) (shared by the parallel blocks)."""
        for i, (c1, c2) in enumerate(zip(self.convs1, self.convs2)):
            xa = x_act if i == 0 else ops.act(x, "lrelu0.1")
            h = c1(xa, act="lrelu0.1")
            x = c2(h, residual=x)
        return x


class HifiGan(nn.Module):
    def __init__(self, cfg: HifiGanConfig = AUDIOLDM_HIFIGAN):
        super().__init__()
        self.cfg = cfg
        uic = cfg.upsample_initial_channel
        self.conv_pre = Conv1d(cfg.model_in_dim, uic, 7, padding=3)
        self.upsampler = nn.ModuleList()
        self.resblocks = nn.ModuleList()
        ch = uic
        for u, k in zip(cfg.upsample_rates, cfg.upsample_kernel_sizes):
            self.upsampler.append(ConvTranspose1d(ch, ch // 2, k, stride=u, padding=(k - u) // 2))
            ch //= 2
            for rk, rd in zip(cfg.resblock_kernel_sizes, cfg.resblock_dilation_sizes):
                self.resblocks.append(HifiGanResidualBlock(ch, rk, rd))
        self.conv_post = Conv1d(ch, 1, 7, padding=3)
        self.register_buffer("mean", torch.zeros(cfg.model_in_dim))
        self.register_buffer("scale", torch.ones(cfg.model_in_dim))

    @torch.no_grad()
    def forward(self, mel: torch.Tensor) -> torch.Tensor:
        """mel [B, T, model_in_dim] -> waveform [B, ~T * hop] (fp32; the transposed convs
        add a few tail samples, trimmed by the caller)."""
        dt = self.conv_pre.weight.dtype
        x = mel.float()
        if self.cfg.normalize_before:
            x = (x - self.mean.float()) / self.scale.float()
        x = self.conv_pre(x.to(dt).contiguous(), act="lrelu0.1")  # lrelu before upsampler[0]
        nk = len(self.cfg.resblock_kernel_sizes)
        last = len(self.upsampler) - 1
        for i, up in enumerate(self.upsampler):
            x = up(x).contiguous()
            x_act = ops.act(x, "lrelu0.1")
            acc = None
            for j in range(nk):
                r = self.resblocks[i * nk + j](x, x_act)
                if j == 0:
                    acc = r
                elif j < nk - 1:
                    acc = ops.axpby_nhwc(acc, r, 1.0, 1.0, acc)
                else:
                    # mean over the parallel blocks fused with the next LeakyReLU
                    nxt = "lrelu0.1" if i < last else "lrelu0.01"
                    acc = ops.axpby_nhwc(acc, r, 1.0 / nk, 1.0 / nk, acc, act=nxt)
            if nk == 1:
                acc = ops.act(acc, "lrelu0.1" if i < last else "lrelu0.01")
            x = acc
        y = self.conv_post(x, act="tanh")
        return y[..., 0].float()
