"""List the GroupNorms of one SD2.1 UNet step (CFG-shared prefix on) that
still run the statistics pass (no fused producer partials), with shapes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from chiaswarm_amd.models import unet  # noqa: E402
from chiaswarm_amd.models.layers import init_random_fast_, prepare_model
from chiaswarm_amd.ops import hip_ops


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8, help="UNet batch (CFG: 2 x images)")
    a = ap.parse_args()
    dev = "cuda"
    with torch.device(dev):
        m = unet.UNet2DConditionModel(unet.SD21).to(torch.bfloat16).eval().requires_grad_(False)
    init_random_fast_(m, seed=1)
    m = prepare_model(m)
    orig_gn, orig_cat = hip_ops.group_norm, hip_ops.group_norm_cat

    def gn(x, *a, **k):
        if getattr(x, "_csk_gn", None) is None:
            print("group_norm stats pass", tuple(x.shape))
        return orig_gn(x, *a, **k)

    def cat(a, b, *r, **k):
        sa, sb = getattr(a, "_csk_gn", None), getattr(b, "_csk_gn", None)
        if sa is None or sb is None or sa[1] != sb[1]:
            print("group_norm_cat stats pass", tuple(a.shape), tuple(b.shape),
                  None if sa is None else sa[1], None if sb is None else sb[1])
        return orig_cat(a, b, *r, **k)

    hip_ops.group_norm, hip_ops.group_norm_cat = gn, cat
    xh = torch.randn(a.batch // 2, 64, 64, 4, device=dev).bfloat16()
    x = torch.cat([xh, xh])
    ctx = torch.randn(a.batch, 77, 1024, device=dev).bfloat16()
    with torch.no_grad():
        kv = m.encode_context(ctx)
        m(x, torch.tensor([500.0], device=dev), cross_kv=kv, cfg_dup=True)
        torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
