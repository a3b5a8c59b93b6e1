#!/usr/bin/env python
"""A/B of the SD VAE decode (4 x 512^2, the bench job's decode) over runtime
knobs, arms interleaved in one process:

    python tools/decode_ab.py --arms narrow0,narrow1 --rounds 5
"""
import os as _os

_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import statistics
import sys

sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


def apply_arm(arm):
    if arm in ("narrow0", "narrow1"):  # Cout <= 16 3x3 convs on the halo-tile kernel (conv_out 128 -> 3)
        hip_ops.CONV_TILE_NARROW_MIN_PX = (1 << 18) if arm == "narrow1" else (1 << 62)
    elif arm != "base":
        raise SystemExit(f"unknown arm {arm}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="narrow0,narrow1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    _lib.load()
    dev = torch.device("cuda", 0)
    p = StableDiffusion("sd21", device=dev, seed=0)
    z = torch.randn(a.batch, 64, 64, 4, device=dev) * p.vae.cfg.scaling_factor
    arms = a.arms.split(",")
    res = {arm: [] for arm in arms}
    outs = {}
    for _ in range(a.rounds):
        for arm in arms:
            apply_arm(arm)
            outs[arm] = p.decode(z, to_host=False)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                p.decode(z, to_host=False)
            e1.record()
            torch.cuda.synchronize()
            res[arm].append(e0.elapsed_time(e1) / a.iters)
    base = outs[arms[0]].float()
    for arm, ts in res.items():
        d = (outs[arm].float() - base).abs().max().item()
        print(f"{arm:10s} median {statistics.median(ts):7.3f} ms  min {min(ts):7.3f}  max|d uint8| vs {arms[0]} {d:.0f}"
              f"  all {[round(t, 3) for t in ts]}", flush=True)


if __name__ == "__main__":
    main()
