#!/usr/bin/env python
"""Fused transformer input (csrc/kernels/xin.hip) vs the unfused chain it
replaces (GroupNorm apply -> proj_in GEMM with LN1 row statistics -> LN-folded
QKV GEMM), graph-replayed at the SD2.1 64x64 level (C = 320):

    python tools/xinbench.py --batch 8
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.models.layers import Transformer2D, init_random_  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters)
    return best * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--side", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--probes", type=lambda v: [int(x) for x in v.split(",") if x], default=[1, 2, 4, 7])
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    t = Transformer2D(320, 5, 1024).to(dev)
    init_random_(t, seed=0)
    t = t.bfloat16()
    P = a.side * a.side
    x = torch.randn(a.batch, P, 320, device=dev).bfloat16()
    xs = x.float().reshape(-1, 64, 320)
    mean = xs.mean(1)
    x._csk_gn = (torch.stack([mean, ((xs - mean[:, None]) ** 2).sum(1)], -1).reshape(-1).contiguous(), 64)
    blk = t.transformer_blocks[0]
    a1 = blk.attn1
    a1._ensure()
    packed = t._xin_weights()
    fold = blk._fold("qkv", a1.w_qkv, a1.b_qkv, blk.norm1)

    def fused():
        st = hip_ops.gn_stats(x, 32, t.norm.eps)
        return hip_ops.xin_qkv(x, st, t.norm.weight, t.norm.bias, *packed, blk.norm1.eps)

    def kernel_only(st=hip_ops.gn_stats(x, 32, t.norm.eps)):
        return hip_ops.xin_qkv(x, st, t.norm.weight, t.norm.bias, *packed, blk.norm1.eps)

    def unfused():
        h = t.norm(x)
        h = t.proj_in(h, row_stats=True)
        w2, cs, b2 = fold
        return hip_ops.gemm(h.reshape(-1, 320), w2, b2, ln=(h._csk_rows, cs, float(blk.norm1.eps)))

    M = a.batch * P
    flop = 2.0 * M * 320 * (320 + 960)
    for name, fn in (("unfused", unfused), ("fused", fused), ("xin kernel", kernel_only)):
        us = timed(fn, a.iters)
        print(f"B{a.batch} {a.side}x{a.side} {name:11s} {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s", flush=True)
    # probes (wrong results): 1 no stores, 2 no MFMAs, 4 no weight DMA after the prologue, 7 all three
    for pr in a.probes:
        _lib.call("csk_set_xin_probe", pr)
        us = timed(kernel_only, a.iters)
        print(f"B{a.batch} {a.side}x{a.side} probe {pr}     {us:8.1f} us", flush=True)
    _lib.call("csk_set_xin_probe", 0)


if __name__ == "__main__":
    main()
