#!/usr/bin/env python
"""Attention throughput per head dim (UNet 40/64/80/160, VAE 512) at the
SD shapes, interleaved rounds in one process; JSON to --out:

    python tools/attndims.py --out gpurun_out/attn_dims.json
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402

SHAPES = [  # (label, B, S, H, D)
    ("sd21-64x64 self", 8, 4096, 5, 64), ("sd15-64x64 self", 8, 4096, 8, 40), ("sd15-32x32 self", 8, 1024, 8, 80),
    ("sd15-16x16 self", 8, 256, 8, 160), ("vae-512^2 mid", 4, 4096, 1, 512), ("vae-1024^2 mid", 1, 16384, 1, 512),
    ("sd21-1024^2 self", 2, 16384, 5, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    rows = []
    for label, B, S, H, D in SHAPES:
        q, k, v = (torch.randn(B, S, H, D, device=dev).to(torch.bfloat16) for _ in range(3))
        fl = 4.0 * B * H * S * S * D
        hip_ops.attention(q, k, v, D ** -0.5)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                hip_ops.attention(q, k, v, D ** -0.5)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / a.iters)
        us = statistics.median(ts)
        rows.append({"shape": label, "B": B, "S": S, "H": H, "D": D, "us": round(us, 1),
                     "tflops": round(fl / us / 1e6, 1)})
        print(json.dumps(rows[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
