#!/usr/bin/env python
"""Time the RRDB dense-block convs (3x3, Cout 32, input / output channel slices
of a 192-channel buffer) on the persistent halo-tile kernel vs the tuned
implicit-GEMM path: python tools/convtilebench.py [--hw 512]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hw", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    buf = torch.randn(1, a.hw, a.hw, 224, device=dev).to(torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for cin in (64, 96, 128, 160):
        wp = ops.pack_conv_weight((torch.randn(32, cin, 3, 3, device=dev) * (9 * cin) ** -0.5).to(torch.bfloat16))
        b = torch.randn(32, device=dev).to(torch.bfloat16)
        res = {}
        for tile in (True, False):
            hip_ops.CONV_TILE = tile
            run = lambda: ops.conv2d(buf[..., :cin], wp, b, act="lrelu", out=buf[..., 192:224])  # noqa: E731
            run()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                ev[0].record()
                for _ in range(a.iters):
                    run()
                ev[1].record()
                ev[1].synchronize()
                best = min(best, ev[0].elapsed_time(ev[1]) * 1e3 / a.iters)
            res[tile] = best
        fl = 2.0 * a.hw * a.hw * 32 * 9 * cin
        print(f"conv {a.hw}x{a.hw} {cin}->32: halo-tile {res[True]:7.1f} us ({fl / res[True] / 1e6:6.1f} TF/s)   "
              f"implicit GEMM {res[False]:7.1f} us ({fl / res[False] / 1e6:6.1f} TF/s)", flush=True)
    hip_ops.CONV_TILE = True


if __name__ == "__main__":
    main()
