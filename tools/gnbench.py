#!/usr/bin/env python
"""GroupNorm(+SiLU) on the UNet's shapes, isolated: the full path (statistics
pass + apply) and the apply-only path fed by a producer's fused epilogue
statistics, in us and GB/s (bytes = read x + write y):

    python tools/gnbench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import hip_ops  # noqa: E402

SHAPES = [(8, 64, 64, 320), (8, 64, 64, 640), (8, 32, 32, 640), (8, 32, 32, 1280), (8, 16, 16, 1280),
          (8, 16, 16, 2560), (8, 8, 8, 1280), (8, 8, 8, 2560)]


def timed(fn, reps=20):
    """GPU time per call: ``reps`` calls captured in one hipGraph and replayed
    (eager back-to-back calls measure the ~25 us host cost of the wrapper)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (5 * reps) * 1000.0


def main():
    ops._lib.load()
    dev = torch.device("cuda", 0)
    for B, H, W, C in SHAPES:
        x = torch.randn(B, H, W, 64, device=dev).bfloat16()
        wp = ops.pack_conv_weight((torch.randn(C, 64, 1, 1, device=dev) * 0.125).bfloat16())
        y = hip_ops.conv2d(x, wp, None, 1, 0, None, False, None, gn_stats=True)
        g, bt = torch.ones(C, device=dev).bfloat16(), torch.zeros(C, device=dev).bfloat16()
        yplain = y.clone()
        full = timed(lambda: hip_ops.group_norm(yplain, g, bt, 32, 1e-5, True))
        fused = timed(lambda: hip_ops.group_norm(y, g, bt, 32, 1e-5, True)) if getattr(y, "_csk_gn", None) else None
        gb = 2 * y.numel() * 2 / 1e9
        line = f"gn {B}x{H}x{W}x{C:<5d} full {full:7.1f} us {gb / full * 1e6:7.0f} GB/s"
        if fused is not None:
            line += f"   apply-from-epilogue-stats {fused:7.1f} us {gb / fused * 1e6:7.0f} GB/s"
        print(line, flush=True)


if __name__ == "__main__":
    main()
