#!/usr/bin/env python
"""Sweep every (tile, ksplit) of the MFMA GEMM on given shapes (for tuning
work and PMC runs):

    python tools/gemmprof.py --shapes 32768x320x320,32768x320x2560:geglu --tiles 11,12,14,18,19,20
    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA ... -- python tools/gemmprof.py --iters 3
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib  # noqa: E402
from chiaswarm_amd.ops.hip_ops import ACT, _p, _s  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="32768x320x320,32768x320x960,32768x320x2560:geglu,32768x1280x320,"
                                       "8192x640x640,2048x1280x1280")
    ap.add_argument("--tiles", default="2,11,12,13,14,17,18,19,20,23")
    ap.add_argument("--splits", default="1")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    _lib.load()
    for spec in a.shapes.split(","):
        dims, _, act = spec.partition(":")
        M, K, N = map(int, dims.split("x"))
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).bfloat16()
        code = ACT[act or None]
        if act == "geglu":
            w, _ = ops.pack_geglu(w, None)
        n_out = N // 2 if code == 3 else N
        y = torch.empty(M, n_out, device="cuda", dtype=torch.bfloat16)
        best = None
        for tile in [int(t) for t in a.tiles.split(",")]:
            for split in [int(s) for s in a.splits.split(",")]:
                ws = torch.empty(split * M * N, device="cuda") if split > 1 else None

                def run():
                    _lib.call("csk_gemm", _p(y), _p(x), _p(w), None, None, None, M, N, K, K, K, n_out, n_out, 1,
                              code, 1.0, None, tile, split, _p(ws), _s())

                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / a.iters * 1000
                tf = 2 * M * N * K / us / 1e6
                print(f"{spec:24s} tile {tile:3d} split {split}: {us:8.1f} us {tf:7.1f} TF/s", flush=True)
                if best is None or us < best[0]:
                    best = (us, tile, split)
        print(f"{spec:24s} BEST tile {best[1]} split {best[2]}: {best[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
