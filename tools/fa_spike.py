"""Repeat the rescale-spike case of tests/test_attn_fa_gpu.py under several
kernel probes / worker counts and print the error of each run (race hunting)."""
import sys

import torch

sys.path.insert(0, ".")
from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402

lib = _lib.load()
lib.csk_set_attn_fa_min_skv(128)
gpu = torch.device("cuda", 0)
B, S, H = 1, 1024, 2
torch.manual_seed(7)
q, k, v = (torch.randn(B, S, H, 64, device=gpu).bfloat16() for _ in range(3))
k[0, 100, 0] = q[0, 5, 0] * 8
k[0, 130, 0] = q[0, 5, 0] * 12
k[0, 700, 0] = q[0, 5, 0] * 16
k[0, 200, 1] = q[0, 70, 1] * 10
k[0, 333, 1] = q[0, 70, 1] * 16
k[0, 1000, 1] = q[0, 300, 1] * 14
ref = ops._ref_attention(q.float().cpu(), k.float().cpu(), v.float().cpu(), 0.125, False)
for probe in [int(x) for x in sys.argv[1].split(",")]:
    lib.csk_set_attn_fa_probe(probe)
    for workers in (0, 3, 11):
        hip_ops.ATTN_FA_WORKERS = workers
        errs = []
        for _ in range(5):
            y = hip_ops.attention(q, k, v, 0.125).float().cpu()
            e = ((y - ref).norm() / ref.norm()).item()
            d = (y - ref).abs().amax(dim=-1)[0]  # [S, H]
            bad = (d > 0.05).nonzero().tolist()
            errs.append((round(e, 4), bad[:6]))
        print("probe", probe, "workers", workers, errs, flush=True)
        for (r, h) in errs[-1][1][:3]:  # which reference row does a bad row hold?
            dist = (ref[0, :, h] - y[0, r, h]).norm(dim=-1)
            print("   row", r, "head", h, "closest ref row", int(dist.argmin()), round(float(dist.min()), 4),
                  "own", round(float(dist[r]), 4), "out", y[0, r, h, :4].tolist(), "ref", ref[0, r, h, :4].tolist())
