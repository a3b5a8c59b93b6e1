#!/usr/bin/env python
"""Per-op A/B microbenchmark on the exact SD2.1-512 (batch 4 -> CFG 8) UNet and
VAE shapes: hand-written HIP kernel vs the PyTorch reference op (hipBLASLt /
MIOpen / SDPA / native), interleaved in one process (cdna_hip_programming.md
§5.4 rule 24), random data.  Prints a table and writes JSON.

    python tools/opbench.py [--out profiles/opbench.json] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def r(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).bfloat16()


def _attn_variant(q, k, v, var):
    from chiaswarm_amd.ops import hip_ops

    if not ops.use_hip(q):
        return ops.attention(q, k, v)
    old, hip_ops.ATTN_VARIANT = hip_ops.ATTN_VARIANT, var
    try:
        return ops.attention(q, k, v)
    finally:
        hip_ops.ATTN_VARIANT = old


def cases():
    B = 8
    out = []
    # conv 3x3 (UNet)
    for (H, Ci, Co) in [(64, 320, 320), (64, 640, 320), (64, 960, 320), (32, 640, 640), (32, 1920, 640),
                        (16, 1280, 1280), (16, 2560, 1280), (8, 1280, 1280), (64, 4, 320), (64, 320, 4)]:
        x, w = r(B, H, H, Ci), ops.pack_conv_weight(r(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5))
        bias = r(Co)
        flops = 2 * B * H * H * Co * 9 * Ci
        out.append((f"conv3x3 B{B} {H}x{H} {Ci}->{Co}", flops, lambda x=x, w=w, b=bias: ops.conv2d(x, w, b, 1, 1)))
    # VAE decoder convs (B=4)
    for (H, Ci, Co) in [(64, 512, 512), (128, 512, 512), (256, 512, 256), (256, 256, 256), (512, 256, 128),
                        (512, 128, 128), (512, 128, 3)]:
        x, w = r(4, H, H, Ci), ops.pack_conv_weight(r(Co, Ci, 3, 3, scale=(9 * Ci) ** -0.5))
        flops = 2 * 4 * H * H * Co * 9 * Ci
        out.append((f"vae conv3x3 B4 {H}x{H} {Ci}->{Co}", flops, lambda x=x, w=w: ops.conv2d(x, w, None, 1, 1)))
    # GEMMs (UNet transformer at 64x64, 32x32)
    for (M, K, N, act) in [(B * 4096, 320, 960, None), (B * 4096, 320, 2560, "geglu"), (B * 4096, 1280, 320, None),
                           (B * 4096, 320, 320, None), (B * 1024, 640, 5120, "geglu"), (B * 256, 1280, 10240, "geglu"),
                           (B * 1024, 2560, 640, None)]:
        a, w = r(M, K), r(N, K, scale=K ** -0.5)
        if act == "geglu":
            w, _ = ops.pack_geglu(w, None)
        out.append((f"gemm {M}x{K}x{N} {act or ''}", 2 * M * N * K, lambda a=a, w=w, act=act: ops.gemm(a, w, act=act)))
    # attention
    for (S, Skv, Hh, D) in [(4096, 4096, 5, 64), (4096, 77, 5, 64), (1024, 1024, 10, 64), (256, 256, 20, 64),
                            (1024, 77, 10, 64)]:
        q, k, v = r(B, S, Hh, D), r(B, Skv, Hh, D), r(B, Skv, Hh, D)
        out.append((f"attn B{B} S{S} Skv{Skv} H{Hh} D{D}", 4 * B * Hh * S * Skv * D,
                    lambda q=q, k=k, v=v: ops.attention(q, k, v)))
        for var in (5, 6, 7):
            out.append((f"attn B{B} S{S} Skv{Skv} H{Hh} D{D} variant{var}", 4 * B * Hh * S * Skv * D,
                        lambda q=q, k=k, v=v, var=var: _attn_variant(q, k, v, var)))
    q, k, v = r(4, 4096, 1, 512), r(4, 4096, 1, 512), r(4, 4096, 1, 512)
    out.append(("vae attn B4 S4096 D512", 4 * 4 * 4096 * 4096 * 512, lambda: ops.attention(q, k, v)))
    # norms
    for shp in [(B, 64, 64, 320), (B, 64, 64, 960), (B, 16, 16, 2560), (4, 512, 512, 128), (4, 256, 256, 256)]:
        x, g, b = r(*shp), r(shp[-1]), r(shp[-1])
        nbytes = 2 * 2 * math.prod(shp)
        out.append((f"groupnorm+silu {shp}", -nbytes, lambda x=x, g=g, b=b: ops.group_norm(x, g, b, 32, 1e-5, True)))
    for (M, C) in [(B * 4096, 320), (B * 1024, 640), (B * 77, 1024)]:
        x, g, b = r(M, C), r(C), r(C)
        out.append((f"layernorm {M}x{C}", -4 * M * C, lambda x=x, g=g, b=b: ops.layer_norm(x, g, b)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/opbench.json")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    ops._lib.load()
    rows = []
    print(f"{'op':48s} {'hip ms':>9s} {'ref ms':>9s} {'speedup':>8s} {'hip TF/s|GB/s':>14s}")
    for name, work, fn in cases():
        if a.filter and a.filter not in name:
            continue
        with ops.ops_mode("hip"):
            th = bench(fn, a.iters)
        with ops.ops_mode("reference"):
            tr = bench(fn, a.iters)
        rate = (work / th / 1e9) if work > 0 else (-work / th / 1e6)
        print(f"{name:48s} {th:9.3f} {tr:9.3f} {tr / th:8.2f} {rate:14.1f}", flush=True)
        rows.append({"op": name, "hip_ms": th, "ref_ms": tr, "speedup": tr / th,
                     "hip_rate": rate, "rate_unit": "TFLOP/s" if work > 0 else "GB/s"})
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
