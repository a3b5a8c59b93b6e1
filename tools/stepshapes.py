#!/usr/bin/env python
"""Per-shape time and TFLOP/s of every GEMM / conv / attention launch of one
SD2.1 UNet step (CFG batch 8, 64x64 latents), eager, each launch timed with
events (synchronised, so launch gaps are excluded):

    python tools/stepshapes.py [--batch 8] [--iters 3] [--json out.json]
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import collections
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd.ops import _lib  # noqa: E402


def flops_of(name, a):
    if name == "csk_gemm" or name == "csk_gemm_ln":
        M, N, K, code = a[6], a[7], a[8], a[14]
        return f"gemm M{M} N{N} K{K}" + (" geglu" if code == 3 else ""), 2.0 * M * N * K, a[-4]
    if name == "csk_conv2d_ex":
        B, H, W, Cin, Cout, kh, kw, stride = a[7:15]
        Ho, Wo, up = a[17], a[18], a[19]
        return (f"conv B{B} {H}x{W}{' up2x' if up else ''} s{stride} {Cin}->{Cout} k{kh}",
                2.0 * B * Ho * Wo * Cout * kh * kw * Cin, a[-4])
    if name == "csk_attention":
        B, H, Sq, Skv, D = a[5:10]
        return f"attn B{B} H{H} Sq{Sq} Skv{Skv} D{D}", 4.0 * B * H * Sq * Skv * D, None
    if name == "csk_attention_fa":  # persistent stream-K attention (attn_fa.hip)
        B, H, Sq, Skv, D = a[5:10]
        return f"attn-fa B{B} H{H} Sq{Sq} Skv{Skv} D{D}", 4.0 * B * H * Sq * Skv * D, None
    if name == "csk_xattn_block":
        M, C, rpb, Bc, Skv = a[9:14]
        return (f"xattn block M{M} C{C} Skv{Skv}", 2.0 * M * C * C * 2 + 4.0 * M * Skv * C, None)
    if name == "csk_conv_tile":  # persistent halo-tile 3x3 conv (conv_tile.hip)
        B, H, W, Cin, Cout = a[5:10]
        return f"conv-tile B{B} {H}x{W} s1 {Cin}->{Cout} k3", 2.0 * B * H * W * Cout * 9 * Cin, None
    if name == "csk_conv_tile2":  # ... with the fused x2 upsample / second residual / narrow outputs
        B, H, W, Cin, Cout = a[6:11]
        tags = (" up2x" if a[18] else "") + (" res2" if a[5] else "") + (" u8" if a[19] else "")
        return (f"conv-tile B{B} {H}x{W}{tags} s1 {Cin}->{Cout} k3", 2.0 * B * H * W * Cout * 9 * Cin,
                None)
    if name == "csk_ff_geglu":  # fused feed-forward (ff.hip)
        M, C, inner = a[8:11]
        return f"ff fused M{M} C{C} I{inner}", 2.0 * M * C * 2 * inner + 2.0 * M * inner * C, None
    return name, 0.0, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    from chiaswarm_amd.models import unet as unet_mod
    from chiaswarm_amd.models.layers import init_random_fast_, prepare_model

    _lib.load()
    dev = torch.device("cuda", 0)
    with torch.device(dev):
        m = unet_mod.UNet2DConditionModel(unet_mod.SD21).to(torch.bfloat16).eval().requires_grad_(False)
    init_random_fast_(m, seed=0)
    prepare_model(m)
    x = torch.randn(a.batch, 64, 64, 4, device=dev).to(torch.bfloat16)
    ctx = torch.randn(a.batch, 77, 1024, device=dev).to(torch.bfloat16)
    kv = m.encode_context(ctx)
    t = torch.tensor([500.0], device=dev)
    with torch.no_grad():
        m(x, t, cross_kv=kv)  # tuning-table lookups, allocations
    torch.cuda.synchronize()

    rec = collections.defaultdict(list)
    orig = _lib.call

    def timed(name, *args):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(name, *args)
        e1.record()
        e1.synchronize()
        rec[(name,) + tuple(x for x in args if isinstance(x, (int, float)) and not isinstance(x, bool))].append(
            e0.elapsed_time(e1) * 1e3)
        timed.seq.append((name, args, e0.elapsed_time(e1) * 1e3))

    timed.seq = []
    _lib.call = timed
    with torch.no_grad():
        for _ in range(a.iters):
            timed.seq.clear()
            m(x, t, cross_kv=kv)
    _lib.call = orig
    agg = collections.OrderedDict()
    for name, args, us in timed.seq:
        label, fl, tile = flops_of(name, args)
        key = (label, tile)
        r = agg.setdefault(key, [0, 0.0, fl])
        r[0] += 1
        r[1] += us
    total = sum(r[1] for r in agg.values())
    print(f"step (sum of synchronised launches): {total / 1e3:.2f} ms over {len(timed.seq)} launches")
    rows = []
    for (label, tile), (n, us, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tf = fl * n / (us * 1e-6) / 1e12 if fl else 0.0
        rows.append({"op": label, "tile": tile, "calls": n, "us_total": round(us, 1), "us_each": round(us / n, 1),
                     "tflops": round(tf, 1)})
        print(f"{us:9.1f} us {n:3d}x {us / n:8.1f} us  {tf:7.1f} TF/s  tile {tile}  {label}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"total_us": total, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
