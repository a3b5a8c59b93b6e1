#!/usr/bin/env python
"""Per-kernel fixed cost inside a hipGraph on this GPU: N dependent launches of
(a) a 64-element axpby, (b) the 64x64 LDS-DMA GEMM at M = 64, N = 64, K = 64
(one workgroup, one K-step), (c) the same GEMM at M = 2, N = 1280, K = 1280,
each captured into one graph and replayed; prints microseconds per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


def per_launch(fn, n=200, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / n)
    return best


def main():
    _lib.load()
    dev = torch.device("cuda", 0)
    x = torch.randn(64, device=dev).to(torch.bfloat16)
    y = torch.randn(64, device=dev).to(torch.bfloat16)
    o = torch.empty_like(x)
    print(f"axpby 64 elements          {per_launch(lambda: hip_ops.axpby(x, y, 1.0, 1.0, o)):6.2f} us/launch", flush=True)
    for M, N, K in ((64, 64, 64), (2, 1280, 1280), (512, 1280, 1280)):
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        for tile in (14, 18):
            def run(a=a, w=w, c=c, M=M, N=N, K=K, tile=tile):
                _lib.call("csk_gemm", c.data_ptr(), a.data_ptr(), w.data_ptr(), None, None, None, M, N, K, K, K, N, N, 1,
                          0, 1.0, None, tile, 1, None, _lib.stream_ptr())
            print(f"gemm M{M} N{N} K{K} tile {tile:2d}  {per_launch(run):6.2f} us/launch", flush=True)


if __name__ == "__main__":
    main()
