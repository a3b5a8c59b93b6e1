#!/usr/bin/env python
"""A/B the hipGraph-replayed SD2.1 UNet step (CFG batch 8, 64x64 latents) over
runtime kernel knobs, each arm captured in its own graph, arms interleaved:

    python tools/abstep.py --arms gn0,gn1024,gnmax --rounds 5
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402


def apply_arm(arm):
    if arm in ("side0", "side1"):  # ResNet shortcuts on a forked side stream (1) or inline (0)
        ops.SIDE_STREAM = arm == "side1"
    elif arm in ("swodd0", "swodd1"):  # 160-wide tiles: LDS (0) / direct row-layout (1) epilogue
        _lib.call("csk_set_sw_odd", int(arm == "swodd1"))
    elif arm in ("nt0", "nt1", "nt2"):  # direct epilogue: plain / non-temporal C stores (/ + residual loads);
        # measured: nt1 +0.23 ms, nt2 +0.30 ms per CFG-8 step (the consumer's reads miss the MALL), default 0
        _lib.call("csk_set_epi_nt", int(arm[2:]))
    elif arm in ("band0", "band1"):  # LDS-staged epilogue: generic loop (0) / compile-time band path (1)
        _lib.call("csk_set_epi_band", int(arm == "band1"))
    elif arm in ("gnd0", "gnd1"):  # GN statistics in the direct (gnd0) / LDS (gnd1) epilogue
        _lib.call("csk_set_gn_lds", int(arm == "gnd1"))
    elif arm.startswith("gnwg"):
        hip_ops.GN_TARGET_WG = int(arm[4:])
    elif arm in ("gnfine", "gntile"):
        hip_ops.set_gn_fine(arm == "gnfine")
    elif arm.startswith("gn"):
        v = arm[2:]
        _lib.call("csk_set_gn_prologue_max", (1 << 30) if v == "max" else int(v))
    elif arm.startswith("asw"):  # split-KV attention: workgroup count below which the key range is split
        hip_ops.ATTN_SPLIT_WG = int(arm[3:])
    elif arm.startswith("gcs"):  # channel-blocked GN apply: small-grid fallback on (1) / off (0)
        _lib.call("csk_set_gn_cb_small", int(arm[3:]))
    elif arm.startswith("gcm"):  # channel-blocked GN apply: block width in lcm(8, C/G) units
        _lib.call("csk_set_gn_cb_mult", int(arm[3:]))
    elif arm.startswith("gcb"):  # channel-blocked GN apply merging its own partials: target workgroups (0 = off)
        _lib.call("csk_set_gn_cb", int(arm[3:]))
    elif arm.startswith("gfw"):  # GN finalize: a workgroup per group above this many partials
        _lib.call("csk_set_gn_finalize_wg", int(arm[3:]))
    elif arm.startswith("kvr"):  # short-KV kernel rows per workgroup (0 = auto), variant 3
        _lib.call("csk_set_short_kv_variant", 3)
        _lib.call("csk_set_short_kv_rows", int(arm[3:]))
    elif arm.startswith("xkv"):
        _lib.call("csk_set_short_kv_variant", int(arm[3:]))
    elif arm.startswith("attn"):
        hip_ops.ATTN_VARIANT = int(arm[4:])
    elif arm in ("skgn0", "skgn1"):
        hip_ops.SPLITK_GN = arm == "skgn1"
    elif arm.startswith("skr"):  # split-K reduces: partial splits loaded per memory round trip (1 / 4 / 8)
        _lib.call("csk_set_skr_unroll", int(arm[3:]))
    elif arm.startswith("xw"):  # fused cross-attention: minimum grid (workgroups) for the fused kernel
        hip_ops.XATTN_MIN_WG = int(arm[2:])
    elif arm in ("xa0", "xa1"):  # C = 320 cross-attention: unfused chain (0) / one fused kernel (1)
        hip_ops.XATTN_FUSED = arm == "xa1"
    elif arm in ("ff0", "ff1"):  # C = 320 feed-forward: two GEMMs (0) / one fused kernel (1, ff.hip)
        hip_ops.FF_FUSED = arm == "ff1"
    elif arm in ("xin0", "xin1"):  # C = 320 transformer input: GN + proj_in + QKV GEMMs (0) / one kernel (1, xin.hip)
        hip_ops.XIN_FUSED = arm == "xin1"
    elif arm in ("lnoff", "lnon"):
        ops.LN_FUSE = arm == "lnon"
    elif arm in ("lnk0", "lnk1"):  # fused-LN row statistics: merge kernel (0) / in the consumer prologue (1)
        _lib.call("csk_set_ln_in_kernel", int(arm == "lnk1"))
    elif arm.startswith("a32t"):  # attn32 on/off: csk_set_attn32 value (0 off, 1 default)
        _lib.call("csk_set_attn32", int(arm[4:]))
    elif arm in ("a32off", "a32on"):  # D = 64 self-attention: 16x16x32 pipelined / 32x32x16 kernel
        hip_ops.set_attn32(arm == "a32on")
    elif arm in ("dup0", "dup1"):  # CFG-shared prefix off / on (UNet forward cfg_dup)
        pass
    elif arm != "base":
        raise SystemExit(f"unknown arm {arm}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="base")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="UNet batch (CFG: 2 x images); 2 = batch-1 jobs")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-cfg", action="store_true",
                    help="--batch images without CFG duplication: one CFG-parallel half (batch 1 = the CFG-1 step)")
    a = ap.parse_args()
    from chiaswarm_amd.pipelines.sd import StableDiffusion, _UNetGraph

    ops._lib.load()
    dev = torch.device("cuda", 0)
    p = StableDiffusion("sd21", device=dev, seed=0)
    if a.no_cfg:
        x = torch.randn(a.batch, 64, 64, 4, device=dev).bfloat16()
    else:
        x = torch.randn(a.batch // 2, 64, 64, 4, device=dev).bfloat16()
        x = torch.cat([x, x])  # identical CFG halves, as in the product loop
    ctx = torch.randn(a.batch, 77, 1024, device=dev).bfloat16()
    kv = p.unet.encode_context(ctx)
    graphs = {}
    for arm in a.arms.split(","):
        for sub in arm.split("+"):  # combined knobs, e.g. gcm2+gcb1024 (settings persist into later arms)
            apply_arm(sub)
        graphs[arm] = _UNetGraph(p.unet, x, kv, None, cfg_dup=arm != "dup0" and not a.no_cfg)
    res = {arm: [] for arm in graphs}
    for _ in range(a.rounds):
        for arm, g in graphs.items():
            g.run(x, 500.0, kv, None, None)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                g.graph.replay()
            e1.record()
            torch.cuda.synchronize()
            res[arm].append(e0.elapsed_time(e1) / a.iters)
    for arm, ts in res.items():
        print(f"{arm:10s} median {statistics.median(ts):7.3f} ms  min {min(ts):7.3f}  all {[round(t, 3) for t in ts]}",
              flush=True)


if __name__ == "__main__":
    main()
