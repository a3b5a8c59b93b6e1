#!/usr/bin/env python
"""Which GroupNorm calls of one SD2.1 UNet step (CFG batch 8, 64x64) get their
statistics from the producer's epilogue (one apply pass) and which need the
separate statistics pass, by shape:

    python tools/gnsites.py
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import hip_ops  # noqa: E402


def main():
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    ops._lib.load()
    dev = torch.device("cuda", 0)
    p = StableDiffusion("sd21", device=dev, seed=0)
    x = torch.randn(8, 64, 64, 4, device=dev).bfloat16()
    ctx = torch.randn(8, 77, 1024, device=dev).bfloat16()
    kv = p.unet.encode_context(ctx)
    sites = collections.Counter()
    gn, gnc = hip_ops.group_norm, hip_ops.group_norm_cat

    def rec_gn(x, *a, **k):
        sites[("gn", tuple(x.shape), getattr(x, "_csk_gn", None) is not None)] += 1
        return gn(x, *a, **k)

    def rec_cat(a, b, *r, **k):
        y = gnc(a, b, *r, **k)
        sites[("gn_cat", tuple(a.shape), tuple(b.shape), y is not None,
               getattr(a, "_csk_gn", None) is not None, getattr(b, "_csk_gn", None) is not None)] += 1
        return y

    hip_ops.group_norm, hip_ops.group_norm_cat = rec_gn, rec_cat
    with torch.no_grad():
        p.unet(x, torch.tensor([500.0], device=dev), cross_kv=kv)
    torch.cuda.synchronize()
    for k, v in sorted(sites.items(), key=lambda kv: str(kv[0])):
        print(v, k)


if __name__ == "__main__":
    main()
