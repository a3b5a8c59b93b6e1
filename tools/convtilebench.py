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
    ap.add_argument("--rw", action="store_true", help="also time the per-unit weight DMA, 8-row tile variant (switch 3)")
    ap.add_argument("--switch", default="", help="','-separated extra csk_set_conv_tile_no_rw values to time (bit 0: per-unit weight DMA, bit 1: 8-row tiles)")
    ap.add_argument("--shapes", default="", help="';'-separated hw,cin,cout (default: the four Cout = 32 convs)")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    shapes = ([tuple(map(int, t.split(","))) for t in a.shapes.split(";")] if a.shapes
              else [(a.hw, c, 32) for c in (64, 96, 128, 160)])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    hip_ops.CONV_TILE64 = True
    for hw, cin, cout in shapes:
        buf = torch.randn(1, hw, hw, 192 + cout, device=dev).to(torch.bfloat16)
        wp = ops.pack_conv_weight((torch.randn(cout, cin, 3, 3, device=dev) * (9 * cin) ** -0.5).to(torch.bfloat16))
        b = torch.randn(cout, device=dev).to(torch.bfloat16)
        res = {}
        extra = [int(v) for v in a.switch.split(",") if v]
        arms = [(True, 0), (False, 0)] + ([(True, 3)] if a.rw else []) + [(True, v) for v in extra]
        for tile, no_rw in arms:
            hip_ops.CONV_TILE = tile
            _lib.call("csk_set_conv_tile_no_rw", no_rw)
            run = lambda: ops.conv2d(buf[..., :cin], wp, b, act="lrelu", out=buf[..., 192:192 + cout])  # noqa: E731
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
            res[(tile, no_rw)] = best
        del buf
        fl = 2.0 * hw * hw * cout * 9 * cin
        t, g = res[(True, 0)], res[(False, 0)]
        extra_s = (f"   per-unit weight DMA, 8-row tiles {res[(True, 3)]:7.1f} us" if a.rw else "")
        extra_s += "".join(f"   switch {v}: {res[(True, v)]:7.1f} us" for v in extra)
        print(f"conv {hw}x{hw} {cin}->{cout}: halo-tile {t:7.1f} us ({fl / t / 1e6:6.1f} TF/s)   "
              f"implicit GEMM {g:7.1f} us ({fl / g / 1e6:6.1f} TF/s){extra_s}", flush=True)
    _lib.call("csk_set_conv_tile_no_rw", 0)
    hip_ops.CONV_TILE = True
    hip_ops.CONV_TILE64 = False


if __name__ == "__main__":
    main()
