#!/usr/bin/env python
"""Whole-model timing on SD2.1-512 shapes: one UNet step (CFG batch 8, 64x64
latents; HIP kernels + hipGraph vs PyTorch reference eager), VAE decode (batch 4
-> 512x512), OpenCLIP-H prompt encode (batch 8 x 77).  Median of N runs.

    python tools/modelbench.py [--iters 10] [--only unet]
"""
from __future__ import annotations

import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402


def timeit(fn, iters):
    for _ in range(2):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--out", default="gpurun_out/modelbench.json")
    a = ap.parse_args()
    from chiaswarm_amd.pipelines.sd import StableDiffusion, _UNetGraph

    dev = torch.device("cuda", 0)
    ops._lib.load()
    p = StableDiffusion("sd21", device=dev, seed=0)
    B, L = a.batch, a.res // 8
    res = {}
    x = torch.randn(2 * B, L, L, 4, device=dev).bfloat16()
    ctx = torch.randn(2 * B, 77, 1024, device=dev).bfloat16()
    t = torch.tensor([500.0], device=dev)
    if not a.only or a.only == "unet":
        kv = p.unet.encode_context(ctx)
        with ops.ops_mode("reference"):
            res["unet_step_reference_ms"] = timeit(lambda: p.unet(x, t, encoder_hidden_states=ctx), a.iters)
        res["unet_step_hip_eager_ms"] = timeit(lambda: p.unet(x, t, cross_kv=kv), a.iters)
        g = _UNetGraph(p.unet, x, kv, None)
        res["unet_step_hip_graph_ms"] = timeit(lambda: g.run(x, 500.0, kv, None, None), a.iters)
    if not a.only or a.only == "vae":
        z = torch.randn(B, L, L, 4, device=dev)
        with ops.ops_mode("reference"):
            res["vae_decode_reference_ms"] = timeit(lambda: p.vae.decode(z), max(3, a.iters // 2))
        res["vae_decode_hip_ms"] = timeit(lambda: p.vae.decode(z), max(3, a.iters // 2))
    if not a.only or a.only == "text":
        ids = torch.randint(0, 49000, (2 * B, 77), device=dev)
        te = p.text_encoders[0]
        with ops.ops_mode("reference"):
            res["text_encode_reference_ms"] = timeit(lambda: te(ids), a.iters)
        res["text_encode_hip_ms"] = timeit(lambda: te(ids), a.iters)
    for k, v in res.items():
        print(f"{k:32s} {v:9.3f}")
    from chiaswarm_amd.ops import tuning

    if os.environ.get("CSK_AUTOTUNE") == "1":
        tuning.save_user()
        print("tuning table entries:", len(tuning.table()))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
