#!/usr/bin/env python
"""The fused cross-attention sub-block (xattn.hip) on the SD2.1 64x64-level
shape, with its profiling probes (csk_set_xattn_probe: 1 no Q-projection MFMAs,
2 no attention, 4 no out-projection MFMAs, 8 no per-head DMA, 15 all) for the
4-wave and 8-wave workgroups (csk_set_xattn_waves), against
the unfused chain (LN-fused Q GEMM + attn_shortkv + out-projection GEMM):

    python tools/xattnbench.py [--batch 8] [--iters 30]
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
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--hw", type=int, default=64)
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    C = 320
    with torch.device(dev):
        blk = BasicTransformerBlock(C, C // 64, 64, 1024).to(torch.bfloat16).eval()
    init_random_fast_(blk, seed=1)
    prepare_model(blk)
    S = a.hw * a.hw
    x = torch.randn(a.batch, S, C, device=dev).bfloat16()
    kv = blk.attn2.context_kv(torch.randn(a.batch, 77, 1024, device=dev).bfloat16())
    a2 = blk.attn2
    w2, colsum, b2 = blk._fold("q", a2.to_q.weight, a2.to_q.bias, blk.norm2)
    wo, bo = a2.to_out[0].weight, a2.to_out[0].bias
    fl = 2.0 * a.batch * S * C * C * 2 + 4.0 * a.batch * S * 77 * C
    ref = None
    for waves in (4, 8):
        hip_ops.XATTN_WAVES = waves  # applied by the next xattn_block call
        for probe in (0, 1, 2, 4, 8, 15):
            _lib.call("csk_set_xattn_probe", probe)
            t = timeit(lambda: hip_ops.xattn_block(x, w2, colsum, b2, kv, wo, bo, 1e-5, a2.scale, S), a.iters)
            print(f"xattn {waves} waves probe {probe:2d}: {t:7.1f} us  {fl / t / 1e6:6.1f} TF/s", flush=True)
        _lib.call("csk_set_xattn_probe", 0)
        y = hip_ops.xattn_block(x, w2, colsum, b2, kv, wo, bo, 1e-5, a2.scale, S).float()
        if ref is None:
            ref = y
        else:
            print(f"  {waves} waves vs 4 waves: max abs diff {(y - ref).abs().max().item():.3e}", flush=True)
    hip_ops.XATTN_WAVES = 4
    xr = ops.row_stats_wanted(x)
    x1 = ops.gemm(x, blk.attn1.to_out[0].weight, None, row_stats=xr)  # a producer carrying row statistics

    def chain():
        q = ops.layer_norm_gemm(x1, blk.norm2, a2.to_q.weight, a2.to_q.bias, (w2, colsum, b2))
        return a2.attend_q(q, kv, None, residual=x1, row_stats=True)

    t = timeit(chain, a.iters)
    print(f"unfused chain (Q GEMM + attn_shortkv + out GEMM): {t:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
