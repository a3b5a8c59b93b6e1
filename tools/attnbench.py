#!/usr/bin/env python
"""Attention-only loop on the SD2.1 64x64-level self-attention shape (for PMC
counter runs and variant timing):

    python tools/attnbench.py --variant 3 --iters 50
    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA ... -- python3 tools/attnbench.py --iters 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shape", default="8,4096,4096,5,64")
    ap.add_argument("--short-kv", type=int, default=-1, help="Skv <= 128 kernel: 1 plain, 2 pipelined, 3 K/V-resident")
    ap.add_argument("--kv-rows", type=int, default=0, help="K/V-resident kernel rows per workgroup (0 auto)")
    ap.add_argument("--attn32", type=int, default=1, help="csk_set_attn32 value (0 off, 1 default)")
    ap.add_argument("--split", type=int, default=0, help="force this many key splits (attention_split); 0: the op's rule")
    ap.add_argument("--fa", type=int, default=1, help="persistent stream-K d=64 kernel (attn_fa.hip) on / off")
    ap.add_argument("--workers", type=int, default=0, help="attn_fa workers (0: one per CU)")
    ap.add_argument("--probe", type=int, default=0, help="attn_fa profiling probe (wrong results): 1 exp 2 waits 4 PV 8 QK 16 barrier")
    ap.add_argument("--logits", default="randn",
                    help="query/key statistics (the lazy-rescale fast path of attn_fa depends on them): randn "
                         "(unit logits), scale:S (logit std S, trained-model-like spread), rising:S (key norms grow "
                         "along the sequence so every key block raises the running row max: the rescale worst case)")
    a = ap.parse_args()
    _lib.load()
    if a.short_kv >= 0:
        _lib.call("csk_set_short_kv_variant", a.short_kv)
    _lib.call("csk_set_short_kv_rows", a.kv_rows)
    _lib.call("csk_set_attn32", a.attn32)
    hip_ops.set_attn_fa(bool(a.fa))
    hip_ops.ATTN_FA_WORKERS = a.workers
    _lib.load().csk_set_attn_fa_probe(a.probe)
    _lib.load().csk_set_attn_fa_min_skv(128)
    B, Sq, Skv, H, D = map(int, a.shape.split(","))
    q, k, v = (torch.randn(B, s, H, D, device="cuda") for s in (Sq, Skv, Skv))
    kind, _, arg = a.logits.partition(":")
    if kind == "scale":  # q.k / sqrt(D) has std = S
        q = q * float(arg)
    elif kind == "rising":  # a shared direction u: logit(q, k_j) ~ S j / Skv + N(0, 1), rising along the keys
        u = torch.nn.functional.normalize(torch.randn(D, device="cuda"), dim=0)
        ramp = float(arg) * torch.arange(Skv, device="cuda", dtype=torch.float32) / Skv
        q = q + D ** 0.5 * u
        k = k + ramp[None, :, None, None] * u
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    hip_ops.ATTN_VARIANT = a.variant
    def run():
        if a.split > 1:
            return hip_ops.attention_split(q, k, v, D ** -0.5, a.split)
        return hip_ops.attention(q, k, v, D ** -0.5)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    if a.probe == 128:
        import ctypes
        n = 256 * 8 * 8
        buf = (ctypes.c_ulonglong * n)()
        _lib.load().csk_attn_fa_dbg(buf, n)
        import numpy as np
        arr = np.frombuffer(buf, dtype=np.uint64).reshape(256, 8, 8).astype(np.float64)
        units = arr[:, 0, 7].sum()
        names = ["vmcnt-wait", "barrier", "dma-issue", "qk+exp+pack", "pv-wait+mfma", "rowmax+rescale"]
        tot = arr[:, :, :6].sum(axis=(0, 1))
        per = tot / (units * 8)
        print("phase cycles per unit per wave:", {k: round(v, 1) for k, v in zip(names, per)},
              "sum", round(per.sum(), 1), "seg ends", arr[:, 0, 6].sum())
    print(f"fa {a.fa} probe {a.probe} w {a.workers} attn32 {a.attn32} variant {a.variant} split {a.split} short_kv {a.short_kv} rows {a.kv_rows} {a.shape}: "
          f"logits {a.logits}: {ms * 1000:.1f} us  "
          f"{4 * B * H * Sq * Skv * D / ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
