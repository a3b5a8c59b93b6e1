#!/usr/bin/env python
"""One implicit-GEMM conv (or plain GEMM) shape in a loop, fixed tile / split,
for PMC counter runs and tile A/Bs:

    python tools/convbench.py --shape 8,64,64,320,320 --tiles 11,19,25 --iters 50
    python tools/convbench.py --gemm 32768,1280,320 --tiles 11,25
    rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA ... -- python3 tools/convbench.py --tiles 11 --iters 5
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
    ap.add_argument("--shape", default="8,64,64,320,320", help="B,H,W,Cin,Cout (3x3, pad 1)")
    ap.add_argument("--gemm", default="", help="M,N,K (plain GEMM instead of the conv)")
    ap.add_argument("--tiles", default="11")
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--act", type=int, default=0, help="GEMM epilogue activation code (3 = GEGLU, N = 2 x out)")
    a = ap.parse_args()
    _lib.load()
    dev = "cuda"
    if a.gemm:
        M, N, K = map(int, a.gemm.split(","))
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * K ** -0.5).bfloat16()
        No = N // 2 if a.act == 3 else N
        y = torch.empty(M, No, dtype=torch.bfloat16, device=dev)
        flops = 2 * M * N * K
        ws = torch.empty(a.split * M * N, dtype=torch.float32, device=dev)

        def run(tile):
            _lib.call("csk_gemm", _p(y), _p(x), _p(w), None, None, None, M, N, K, K, K, No, No, 1, a.act, 1.0, None,
                      tile, a.split, _p(ws), _s())

        def ref():
            r = x.float() @ w.float().t()
            if a.act == 3:  # packed (hidden, gate) 16-column pairs
                r = r.view(M, N // 32, 2, 16)
                r = (r[:, :, 0] * torch.nn.functional.gelu(r[:, :, 1])).reshape(M, No)
            return r
    else:
        B, H, W, Cin, Cout = map(int, a.shape.split(","))
        x = torch.randn(B, H, W, Cin, device=dev).bfloat16()
        wp = ops.pack_conv_weight((torch.randn(Cout, Cin, 3, 3, device=dev) * (9 * Cin) ** -0.5).bfloat16())
        y = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device=dev)
        flops = 2 * B * H * W * Cout * Cin * 9
        ws = torch.empty(a.split * B * H * W * Cout, dtype=torch.float32, device=dev)

        def run(tile):
            _lib.call("csk_conv2d", _p(y), _p(x), _p(wp), None, None, None, B, H, W, Cin, Cout, 3, 3, 1, 1, 1, H, W, 0,
                      Cin, Cout, 0, 0, 1.0, 1, None, tile, a.split, _p(ws), _s())

        def ref():
            return ops._ref_conv2d(x.float(), wp.float(), None, 1, 1, None, False, None)
    for tile in map(int, a.tiles.split(",")):
        for _ in range(3):
            run(tile)
        torch.cuda.synchronize()
        if a.check:
            r = ref()
            err = ((y.float() - r).norm() / r.norm()).item()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run(tile)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        extra = f"  rel_err {err:.2e}" if a.check else ""
        print(f"tile {tile:2d} split {a.split}: {ms * 1000:8.1f} us  {flops / ms / 1e9:7.1f} TF/s{extra}", flush=True)


if __name__ == "__main__":
    main()
