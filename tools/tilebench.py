#!/usr/bin/env python
"""Same-process A/B of GEMM / conv tiles on the SD2.1 UNet step's hot shapes
(interleaved rounds, random operands, median us and TFLOP/s per tile):

    python tools/tilebench.py --tiles 11,26,31,32 --rounds 5
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import _lib, hip_ops  # noqa: E402
from chiaswarm_amd.ops.hip_ops import _p, _s  # noqa: E402

CONVS = ["8,64,64,320,320", "8,64,64,640,320", "8,64,64,960,320", "8,32,32,640,640", "8,32,32,1280,640",
         "8,32,32,1920,640", "8,16,16,1280,1280", "8,16,16,2560,1280", "8,32,32,320,640", "8,16,16,640,1280"]
GEMMS = ["32768,320,320", "32768,960,320", "32768,2560,320:geglu", "32768,320,1280", "8192,640,640",
         "8192,5120,640:geglu", "8192,640,2560", "2048,1280,1280", "2048,10240,1280:geglu", "2048,1280,5120"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="11,26,31,32")
    ap.add_argument("--splits", default="1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="", help="conv|gemm")
    ap.add_argument("--probe", action="store_true", help="GEMMs also without their epilogue (act 99)")
    ap.add_argument("--res", action="store_true", help="GEMMs also with a residual input (epilogue load)")
    ap.add_argument("--nt", type=int, default=0, help="csk_set_epi_nt for this run (non-temporal direct-epilogue stores)")
    ap.add_argument("--graph", action="store_true",
                    help="time hipGraph replays of --iters launches (no host launch cost: small kernels)")
    ap.add_argument("--gemms", default="", help="';'-separated 'M,N,K' list overriding the GEMM shapes")
    ap.add_argument("--convs", default="", help="';'-separated 'B,H,W,Cin,Cout' list overriding the conv shapes")
    ap.add_argument("--gn", action="store_true", help="convs also emitting fused GroupNorm statistics (64-row segments)")
    ap.add_argument("--swodd", default="", help="comma list of csk_set_sw_odd values to A/B (160-wide tile epilogue)")
    ap.add_argument("--probe-halo", action="store_true",
                    help="convs also without epilogue (act 99) and without the kx != 0 A DMA (act 98, 2-stage tiles)")
    a = ap.parse_args()
    _lib.load()
    dev = torch.device("cuda", 0)
    _lib.load()
    _lib.call("csk_set_epi_nt", a.nt)
    tiles = [int(t) for t in a.tiles.split(",")]
    splits = [int(s) for s in a.splits.split(",")]
    jobs = []
    if a.only != "gemm":
        for spec in (a.convs.split(";") if a.convs else CONVS):
            up = int(spec.endswith("u"))  # "B,H,W,Cin,Cout u": nearest-x2 upsample fused into the conv input
            B, H, W, Cin, Cout = map(int, spec.rstrip("u").split(","))
            Ho, Wo = H << up, W << up
            x = (torch.randn(B, H, W, Cin, device=dev)).to(torch.bfloat16)
            wp = ops.pack_conv_weight((torch.randn(Cout, Cin, 3, 3, device=dev) * (9 * Cin) ** -0.5).to(torch.bfloat16))
            y = torch.empty(B, Ho, Wo, Cout, dtype=torch.bfloat16, device=dev)
            fl = 2.0 * B * Ho * Wo * Cout * 9 * Cin

            gpart = torch.empty(B * Ho * Wo // 64 * Cout * 2, dtype=torch.float32, device=dev)
            variants = [(0, False, None)]
            if a.gn:
                variants.append((0, True, None))
            for sw in [int(v) for v in a.swodd.split(",") if v]:
                variants.append((0, a.gn, sw))
            if a.probe_halo:
                variants += [(97, False, None), (99, False, None), (98, False, None)]
            for act, gn, sw in variants:
                def run(tile, split, x=x, wp=wp, y=y, B=B, H=H, W=W, Cin=Cin, Cout=Cout, act=act, gn=gn, sw=sw,
                        gpart=gpart, up=up, Ho=Ho, Wo=Wo):
                    if sw is not None:
                        _lib.call("csk_set_sw_odd", sw)
                    ws = hip_ops._ws(split, B * Ho * Wo, Cout, dev)
                    _lib.call("csk_conv2d", _p(y), _p(x), _p(wp), None, None, None, B, H, W, Cin, Cout, 3, 3, 1, 1, 1,
                              Ho, Wo, up, Cin, Cout, 0, act, 1.0, 1, _p(gpart) if gn else None, tile, split, _p(ws),
                              _s())
                    if sw is not None:
                        _lib.call("csk_set_sw_odd", 0)
                tag = {0: "", 97: " nostore", 99: " noepi", 98: " noepi-noA"}[act] + (" gn" if gn else "") + \
                    ("" if sw is None else f" swodd{sw}")
                jobs.append((f"conv {spec}{tag}", fl, run))
    if a.only != "conv":
        for spec in (a.gemms.split(";") if a.gemms else GEMMS):
            geglu = spec.endswith(":geglu")
            M, N, K = map(int, spec.split(":")[0].split(","))
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
            no = N // 2 if geglu else N
            y = torch.empty(M, no, dtype=torch.bfloat16, device=dev)
            yfull = torch.empty(M, N, dtype=torch.bfloat16, device=dev)  # probe runs: act 99 is not GEGLU
            fl = 2.0 * M * N * K

            r = torch.randn(M, no, device=dev).to(torch.bfloat16)
            variants = [(False, False)] + ([(True, False)] if a.probe else []) + ([(False, True)] if a.res else [])
            for probe, res in variants:
                def run(tile, split, x=x, w=w, y=y, yfull=yfull, M=M, N=N, K=K, no=no, geglu=geglu, probe=probe, res=res,
                        r=r):
                    ws = hip_ops._ws(split, M, N, dev)
                    # a probe is not a GEGLU epilogue: full-width output buffer and row stride
                    out, ldo = (yfull, N) if probe else (y, no)
                    _lib.call("csk_gemm", _p(out), _p(x), _p(w), None, None, _p(r) if (res and not probe) else None, M,
                              N, K, K, K, ldo, ldo, 1, 99 if probe else (3 if geglu else 0), 1.0, None, tile, split,
                              _p(ws), _s())
                jobs.append((f"gemm {spec}" + (" noepi" if probe else "") + (" res" if res else ""), fl, run))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for name, fl, run in jobs:
        res = {}
        arms = []
        for t, s in [(t, s) for t in tiles for s in splits]:
            try:  # a tile that rejects the shape (e.g. the B-stationary K limit) is skipped
                run(t, s)
                arms.append((t, s))
            except Exception as e:  # noqa: BLE001
                print(f"  {name}: tile {t} split {s} unsupported ({str(e)[:60]})", flush=True)
        torch.cuda.synchronize()
        graphs = {}
        if a.graph:
            for t, s in arms:
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    run(t, s)
                torch.cuda.current_stream().wait_stream(st)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(a.iters):
                        run(t, s)
                graphs[(t, s)] = g
            torch.cuda.synchronize()
        for _ in range(a.rounds):
            for t, s in arms:
                ev[0].record()
                if a.graph:
                    graphs[(t, s)].replay()
                else:
                    for _ in range(a.iters):
                        run(t, s)
                ev[1].record()
                ev[1].synchronize()
                res.setdefault((t, s), []).append(ev[0].elapsed_time(ev[1]) * 1e3 / a.iters)
        line = "  ".join(f"t{t}/s{s}: {statistics.median(v):7.1f}us {fl / statistics.median(v) / 1e6:6.0f}TF"
                         for (t, s), v in res.items())
        print(f"{name:28s} {line}", flush=True)


if __name__ == "__main__":
    main()
