#!/usr/bin/env python
"""The fused feed-forward (csrc/kernels/ff.hip) on the SD2.1 64x64-level shape
(C = 320, M = batch x 4096) with its profiling probes (csk_set_ff_probe: 1 no
MFMAs, 2 no GEGLU math, 4 no weight DMA after the prologue), against the
production unfused chain (LN-fused GEGLU GEMM -> [M, 1280] in HBM ->
down-projection GEMM + residual):

    python tools/ffbench.py [--batch 8,2] [--iters 30]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.models.layers import BasicTransformerBlock, init_random_fast_, prepare_model  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


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
    ap.add_argument("--batch", default="8,2")
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--probes", default="0,1,2,4")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    C = 320
    with torch.device(dev):
        blk = BasicTransformerBlock(C, C // 64, 64, 1024).to(torch.bfloat16).eval()
    init_random_fast_(blk, seed=1)
    prepare_model(blk)
    ff, n3 = blk.ff, blk.norm3
    w1p, b1p, w2p = ff.fused_weights()
    g = ff.net[0]
    g.ensure()
    eye = torch.eye(C, device=dev).bfloat16()
    for batch in [int(b) for b in a.batch.split(",")]:
        S = a.hw * a.hw
        M = batch * S
        x0 = torch.randn(batch, S, C, device=dev).bfloat16()
        x = ops.gemm(x0, eye, row_stats=True)  # the producer's row statistics, as in the block
        fl = 2.0 * M * C * (2 * ff.inner) + 2.0 * M * ff.inner * C

        def unfused():
            hdn = ops.layer_norm_gemm(x, n3, g.wp, g.bp, blk._fold("ff", g.wp, g.bp, n3), act="geglu")
            return ff.net[2](hdn, residual=x)

        t_ref = timeit(unfused, a.iters)
        print(f"B{batch} M{M}: unfused GEGLU GEMM + down GEMM {t_ref:7.1f} us ({fl / t_ref / 1e6:6.1f} TF/s)")
        ref = unfused()
        for probe in [int(p) for p in a.probes.split(",")]:
            _lib.call("csk_set_ff_probe", probe)
            t = timeit(lambda: hip_ops.ff_geglu(x, n3.weight, n3.bias, w1p, b1p, w2p, ff.net[2].bias, n3.eps),
                       a.iters)
            line = f"B{batch} M{M}: fused probe {probe:2d} {t:7.1f} us ({fl / t / 1e6:6.1f} TF/s)"
            if probe == 0:
                y = hip_ops.ff_geglu(x, n3.weight, n3.bias, w1p, b1p, w2p, ff.net[2].bias, n3.eps)
                err = ((y.float() - ref.float()).norm() / ref.float().norm()).item()
                line += f"  rel err vs unfused {err:.2e}  speedup {t_ref / t:.2f}x"
            print(line, flush=True)
        _lib.call("csk_set_ff_probe", 0)


if __name__ == "__main__":
    main()
