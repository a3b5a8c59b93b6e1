"""Real-ESRGAN RRDBNet x4 (north-star config #5; SURVEY K22 — not in the
reference, whose roadmap leaves it unchecked at README.md:34).

basicsr key layout: conv_first, body.N.rdb{1,2,3}.conv{1..5}, conv_body,
conv_up1, conv_up2, conv_hr, conv_last.

MI355X structure — every conv is the implicit-GEMM MFMA kernel with its
epilogue doing the elementwise work:
  * dense blocks are zero-copy: each RDB owns one NHWC buffer of
    nf + 4*gc = 192 channels; conv_i reads the first nf + i*gc channels as a
    strided view and writes its gc output channels straight into the next
    slice (no torch.cat);
  * LeakyReLU(0.2) fused in conv1..4, "conv5 * 0.2 + x" fused in conv5
    (out_scale + residual); in the third block the RRDB's own "* 0.2 + x"
    folds into the same epilogue: x + 0.2 (c + 0.2 conv5) = 0.04 conv5 +
    0.2 c + x, written over x in place (two residuals: no axpby pass);
  * the two nearest-x2 upsamples are fused into conv_up1 / conv_up2 addressing.
The 3x3 convs with 32 / 64 / 3 outputs run the persistent halo-tile kernel
(csrc/kernels/conv_tile.hip, incl. the up-convs and the RGB conv_last).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import ops
from .layers import Conv2d


class RDB(nn.Module):
    def __init__(self, nf=64, gc=32):
        super().__init__()
        self.nf, self.gc = nf, gc
        for i in range(4):
            setattr(self, f"conv{i + 1}", Conv2d(nf + i * gc, gc, 3, padding=1))
        self.conv5 = Conv2d(nf + 4 * gc, nf, 3, padding=1)

    def forward(self, buf, out, outer=None):
        """buf: [B,H,W,nf+4gc] with x in [..., :nf]; writes x + 0.2*conv5 into
        ``out`` — or, with ``outer`` (the enclosing RRDB's input, may alias
        ``out``), outer + 0.2 * (x + 0.2*conv5)."""
        nf, gc = self.nf, self.gc
        for i in range(4):
            conv = getattr(self, f"conv{i + 1}")
            c0 = nf + i * gc
            conv(buf[..., :c0], act="lrelu", out=buf[..., c0:c0 + gc])
        if outer is None:
            self.conv5(buf, out_scale=0.2, residual=buf[..., :nf], out=out)
        else:
            self.conv5(buf, out_scale=0.04, residual=buf[..., :nf], res_scale=0.2, residual2=outer, out=out)
        return out


class RRDB(nn.Module):
    def __init__(self, nf=64, gc=32):
        super().__init__()
        self.rdb1, self.rdb2, self.rdb3 = RDB(nf, gc), RDB(nf, gc), RDB(nf, gc)

    def forward(self, a, b, c):
        """x in a[..., :nf]; result written back into a[..., :nf]."""
        nf = self.rdb1.nf
        self.rdb1(a, b[..., :nf])
        self.rdb2(b, c[..., :nf])
        self.rdb3(c, a[..., :nf], outer=a[..., :nf])


class RRDBNet(nn.Module):
    def __init__(self, in_ch=3, out_ch=3, nf=64, nb=23, gc=32, scale=4):
        super().__init__()
        self.nf, self.gc, self.scale = nf, gc, scale
        self.conv_first = Conv2d(in_ch, nf, 3, padding=1)
        self.body = nn.ModuleList([RRDB(nf, gc) for _ in range(nb)])
        self.conv_body = Conv2d(nf, nf, 3, padding=1)
        self.conv_up1 = Conv2d(nf, nf, 3, padding=1)
        self.conv_up2 = Conv2d(nf, nf, 3, padding=1)
        self.conv_hr = Conv2d(nf, nf, 3, padding=1)
        self.conv_last = Conv2d(nf, out_ch, 3, padding=1)

    @torch.no_grad()
    def forward(self, x, u8_out=False):
        """x: NHWC [B, H, W, 3] in [0, 1] (or uint8 pixels) -> [B, 4H, 4W, 3]
        (``u8_out``: uint8 pixels, round(clamp(y, 0, 1) * 255), stored by
        conv_last's epilogue)."""
        dt = self.conv_first.weight.dtype
        x = x.to(dt) * (1.0 / 255.0) if x.dtype == torch.uint8 else x.to(dt)
        b, h, w, _ = x.shape
        C = self.nf + 4 * self.gc
        bufs = [torch.empty(b, h, w, C, dtype=dt, device=x.device) for _ in range(3)]
        feat = self.conv_first(x)
        bufs[0][..., :self.nf].copy_(feat)
        for blk in self.body:
            blk(*bufs)
        fea = self.conv_body(bufs[0][..., :self.nf], residual=feat)
        fea = self.conv_up1(fea, up2x=True, act="lrelu")
        fea = self.conv_up2(fea, up2x=True, act="lrelu")
        fea = self.conv_hr(fea, act="lrelu")
        if u8_out:
            return ops.conv2d(fea, self.conv_last._wp(), self.conv_last.bias, 1, 1, out_u8=True)
        return self.conv_last(fea)


TINY_RRDB = dict(nf=16, nb=2, gc=8)
