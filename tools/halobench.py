#!/usr/bin/env python
"""Halo 3x3 conv (conv_halo.hip) vs the tuned implicit-GEMM conv on the SD2.1
UNet ResNet shapes (CFG batch 8 by default), with and without the fused
GroupNorm+SiLU prologue (the baseline then includes the GroupNorm apply pass):

    python tools/halobench.py [--batch 8] [--iters 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402

SHAPES = [(64, 320, 320), (64, 640, 320), (64, 960, 320), (32, 640, 640), (32, 1280, 640), (32, 1920, 640),
          (32, 320, 640), (16, 1280, 1280), (16, 2560, 1280), (16, 640, 1280)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    B = a.batch
    for hw, cin, cout in SHAPES:
        x0 = (torch.randn(B, hw, hw, cin, device=dev)).bfloat16()
        wsrc = ops.pack_conv_weight((torch.randn(cin, cin, 3, 3, device=dev) * (9 * cin) ** -0.5).bfloat16())
        x = hip_ops.conv2d(x0, wsrc, None, 1, 1, None, False, None, gn_stats=True)  # carries _csk_gn
        wp = ops.pack_conv_weight((torch.randn(cout, cin, 3, 3, device=dev) * (9 * cin) ** -0.5).bfloat16())
        g, bt = torch.ones(cin, device=dev).bfloat16(), torch.zeros(cin, device=dev).bfloat16()
        fl = 2.0 * B * hw * hw * cout * 9 * cin
        if not hip_ops.conv_halo_ok(x, wp):
            print(f"{hw}x{hw} {cin}->{cout}: halo unsupported")
            continue
        t_conv = timeit(lambda: hip_ops.conv2d(x, wp, None, 1, 1, None, False, None, gn_stats=True), a.iters)
        t_gn = timeit(lambda: hip_ops.group_norm(x, g, bt, 32, 1e-5, True), a.iters)
        t_halo = timeit(lambda: hip_ops.conv_halo(x, wp), a.iters)
        t_fin = timeit(lambda: hip_ops.gn_finalize(x, 32, 1e-5), a.iters)
        st = hip_ops.gn_finalize(x, 32, 1e-5)
        t_halo_gn = timeit(lambda: hip_ops.conv_halo(x, wp, gn=(st, g, bt, 32, True)), a.iters)
        print(f"B{B} {hw}x{hw} {cin}->{cout}: conv {t_conv:7.1f} us ({fl / t_conv / 1e6:6.1f} TF/s)  +GN apply "
              f"{t_gn:6.1f}  | halo {t_halo:7.1f} us ({fl / t_halo / 1e6:6.1f} TF/s)  halo+GN {t_halo_gn:7.1f}  "
              f"finalize {t_fin:5.1f}  | fused saves {t_conv + t_gn - t_halo_gn - t_fin:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
