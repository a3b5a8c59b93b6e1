#!/usr/bin/env python
"""The bench job's non-UNet phases alone, for kernel traces and PMC passes:
SD VAE decode of 4 512x512 latents (bf16, HIP kernels) and the OpenCLIP-H text
encoder on a CFG batch of 8 prompts.

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/decodeprof.py --iters 3
    rocprofv3 --pmc SQ_WAVES ... -- python3 tools/decodeprof.py --iters 1
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.models import clip, vae  # noqa: E402
from chiaswarm_amd.models.layers import init_random_fast_, prepare_model  # noqa: E402
from chiaswarm_amd.ops import _lib  # noqa: E402


def build(cls, cfg, dev):
    with torch.device(dev):
        m = cls(cfg).to(torch.bfloat16).eval().requires_grad_(False)
    init_random_fast_(m, seed=1)
    return prepare_model(m)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--only", default="vae,text")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    z = torch.randn(4, 64, 64, 4, device=dev)
    ids = torch.randint(0, 49000, (8, 77), device=dev)
    vm = build(vae.AutoencoderKL, vae.SD_VAE, dev) if "vae" in a.only else None
    tm = build(clip.CLIPTextModel, clip.OPENCLIP_H, dev) if "text" in a.only else None
    with torch.no_grad():
        for name, fn in (("vae_decode_4x512", (lambda: vm.decode(z)) if vm else None),
                         ("openclip_h_encode_8x77", (lambda: tm(ids)) if tm else None)):
            if fn is None:
                continue
            fn()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.iters):
                fn()
            torch.cuda.synchronize()
            print(f"{name}: {(time.perf_counter() - t) / a.iters * 1000:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
