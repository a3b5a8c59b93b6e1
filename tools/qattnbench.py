#!/usr/bin/env python
"""The cross-attention query projection with the attention epilogue
(hip_ops.gemm_attn) on tiles 19 / 12 against the unfused query GEMM +
short-KV attention, on the SD2.1 / SDXL shapes (graph-replayed, us per call):

    python tools/qattnbench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402

SHAPES = [(8, 1024, 640), (8, 256, 1280), (2, 1024, 1280), (2, 4096, 640)]


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000


def main():
    _lib.load()
    dev = torch.device("cuda", 0)
    for B, S, C in SHAPES:
        M = B * S
        x = torch.randn(M, C, device=dev).bfloat16()
        w = (torch.randn(C, C, device=dev) * C ** -0.5).bfloat16()
        bias = torch.randn(C, device=dev).bfloat16()
        kv = torch.randn(B, 77, 2, C // 64, 64, device=dev).bfloat16()
        line = f"B{B} S{S} C{C}:"
        for tile in (19, 12):
            us = timed(lambda: hip_ops.gemm_attn(x, w, bias, kv, 0.125, S, tile=tile))
            line += f"  qattn tile {tile} {us:6.1f} us"
        q3 = x.view(B, S, C)

        def unfused():
            q = ops.gemm(q3, w, bias)
            return ops.attention(q.view(B, S, C // 64, 64), kv[:, :, 0], kv[:, :, 1], 0.125)

        line += f"  unfused {timed(unfused):6.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
