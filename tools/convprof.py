#!/usr/bin/env python
"""Run one conv / GEMM shape with an explicit (tile, ksplit) for PMC profiling:

    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU ... -- python tools/convprof.py --tile 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib  # noqa: E402
from chiaswarm_amd.ops.hip_ops import _p, _s  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="2,6,11,12,14,15")
    ap.add_argument("--shape", default="8,64,64,320,320")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    B, H, W, Ci, Co = map(int, a.shape.split(","))
    _lib.load()
    x = torch.randn(B, H, W, Ci, device="cuda").bfloat16()
    wp = ops.pack_conv_weight((torch.randn(Co, Ci, 3, 3, device="cuda") * (9 * Ci) ** -0.5).bfloat16())
    y = torch.empty(B, H, W, Co, device="cuda", dtype=torch.bfloat16)
    for tile in [int(t) for t in a.tiles.split(",")]:
        def run():
            _lib.call("csk_conv2d", _p(y), _p(x), _p(wp), None, None, None, B, H, W, Ci, Co, 3, 3, 1, 1, 1, H, W, 0,
                      Ci, Co, 0, 0, 1.0, 1, None, tile, 1, None, _s())
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tf = 2 * B * H * W * Co * 9 * Ci / ms / 1e9
        print(f"tile {tile:3d}: {ms * 1000:8.1f} us  {tf:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
