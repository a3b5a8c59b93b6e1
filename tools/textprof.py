#!/usr/bin/env python
"""Time the text-encoding phase (text encoders + every cross-attention K/V
projection, one graph replay) of a family: python tools/textprof.py sdxl [--eager]"""
import os
import statistics
import sys
import time

os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
os.environ.setdefault("SDAAS_OFFLINE", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.pipelines.sd import StableDiffusion  # noqa: E402


def main():
    fam = sys.argv[1] if len(sys.argv) > 1 else "sdxl"
    p = StableDiffusion(fam, device=torch.device("cuda", 0))
    if "--eager" in sys.argv:
        p.use_graphs = False
    for _ in range(3):
        p.encode(["a fox"], [""], cfg=True)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        t = time.perf_counter()
        p.encode(["a fox"], [""], cfg=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    t = time.perf_counter()
    for _ in range(20):
        p._text_fn(tuple(tok(["", "a fox"]).to(p.device) for tok in p.tokenizers), False)
    torch.cuda.synchronize()
    print(f"{fam}: encode (text encoders + K/V, {'eager' if '--eager' in sys.argv else 'graph'}) median "
          f"{1000 * statistics.median(ts):.2f} ms; text encoders only (eager) {(time.perf_counter() - t) * 50:.2f} ms")


if __name__ == "__main__":
    main()
