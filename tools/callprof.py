#!/usr/bin/env python
"""Exact per-call kernel time of one SD2.1 UNet step (CFG batch 8, 64x64; or
``--model sdxl --batch 2``: the SDXL 1024-px CFG-batch-2 step; ``--model
controlnet``: SD1.5 + ControlNet at 64x64, config #4):
every libcsk call is followed by a 1-element int32 fill, so in a rocprofv3
kernel trace the separator kernels split the dispatch stream into calls; the
calls' shapes are recorded on the host in the same order.  No host syncs, so
the kernels run back to back as in the hipGraph (durations are device time).

    rocprofv3 --kernel-trace -d OUT -o cp -- python tools/callprof.py --record OUT/calls.json
    python tools/callprof.py --db OUT/.../cp_results.db --calls OUT/calls.json
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import collections
import glob
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def record(path, batch, iters, dup=True, model="sd21"):
    import torch

    from chiaswarm_amd.models import unet as unet_mod
    from chiaswarm_amd.models.layers import init_random_fast_, prepare_model
    from chiaswarm_amd.ops import _lib
    from stepshapes import flops_of

    _lib.load()
    dev = torch.device("cuda", 0)
    if model == "esrgan":  # Real-ESRGAN x4plus 512 -> 2048 (config #5): one upscale per "step"
        from chiaswarm_amd.models.rrdbnet import RRDBNet

        with torch.device(dev):
            net = RRDBNet().to(torch.bfloat16).eval().requires_grad_(False)
        init_random_fast_(net, seed=0)
        prepare_model(net)
        img = torch.rand(1, 512, 512, 3, device=dev)
        return _record_steps(path, iters, lambda: net(img), flops_of, _lib)
    sdxl = model == "sdxl"
    cn = model == "controlnet"
    cfg, lat, cdim = ((unet_mod.SDXL, 128, 2048) if sdxl else (unet_mod.SD15, 64, 768) if cn
                      else (unet_mod.SD21, 64, 1024))
    with torch.device(dev):
        m = unet_mod.UNet2DConditionModel(cfg).to(torch.bfloat16).eval().requires_grad_(False)
    init_random_fast_(m, seed=0)
    prepare_model(m)
    dup = dup and not sdxl and not cn  # SDXL's halves differ in the pooled text embedding; ControlNet: no prefix
    x = torch.randn(batch // 2 if dup else batch, lat, lat, 4, device=dev).to(torch.bfloat16)
    if dup:  # identical CFG halves and the shared prefix, as in the product loop
        x = torch.cat([x, x])
    ctx = torch.randn(batch, 77, cdim, device=dev).to(torch.bfloat16)
    kv = m.encode_context(ctx)
    t = torch.tensor([500.0], device=dev)
    kw = {"cfg_dup": dup}
    step = None
    if cn:  # SD1.5 + ControlNet (config #4): the encoder copy + zero convs merged into the skips
        from chiaswarm_amd.models.controlnet import ControlNetModel
        from chiaswarm_amd.pipelines.controlnet import ControlFeatures

        with torch.device(dev):
            cnm = ControlNetModel(cfg).to(torch.bfloat16).eval().requires_grad_(False)
        init_random_fast_(cnm, seed=1)
        prepare_model(cnm)
        with torch.no_grad():
            cond_emb = cnm.embed_cond(torch.rand(batch, 8 * lat, 8 * lat, 3, device=dev))
            cn_kv = cnm.encode_context(ctx)

        def step():
            feats, mid = cnm.features(x, t, cond_emb, cross_kv=cn_kv)
            return m(x, t, cross_kv=kv, control=ControlFeatures(cnm, feats, mid, 1.0), **kw)
    if sdxl:
        kw["added_cond"] = {"text_embeds": torch.randn(batch, 1280, device=dev).to(torch.bfloat16),
                            "time_ids": torch.tensor([[1024.0, 1024, 0, 0, 1024, 1024]] * batch, device=dev)}
    if step is None:
        def step():
            return m(x, t, cross_kv=kv, **kw)
    return _record_steps(path, iters, step, flops_of, _lib)


def _record_steps(path, iters, step, flops_of, _lib):
    import torch

    dev = torch.device("cuda", 0)
    with torch.no_grad():
        for _ in range(2):
            step()
    torch.cuda.synchronize()
    sep = torch.zeros(1, dtype=torch.int32, device=dev)
    orig = _lib.call
    seq = []

    def wrapped(name, *args):
        orig(name, *args)
        sep.fill_(len(seq))
        label, fl, tile = flops_of(name, args)
        seq.append([label, fl, tile])

    _lib.call = wrapped
    with torch.no_grad():
        for _ in range(iters):
            step()
    torch.cuda.synchronize()
    _lib.call = orig
    with open(path, "w") as f:
        json.dump({"iters": iters, "calls": seq}, f)
    print(f"recorded {len(seq)} calls")


def analyse(db, calls_path, out_json=""):
    with open(calls_path) as f:
        meta = json.load(f)
    calls = meta["calls"]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    is_sep = [("FillFunctor<int>" in r[0]) for r in rows]
    sep_idx = [i for i, s in enumerate(is_sep) if s]
    n = len(calls)
    if len(sep_idx) < n:
        raise SystemExit(f"{len(sep_idx)} separators for {n} calls")
    sep_idx = sep_idx[-n:]  # the recorded calls are the last n separated groups
    agg = collections.OrderedDict()
    per_kernel = collections.defaultdict(float)
    torch_kernels = collections.defaultdict(float)
    prev = sep_idx[0] - 1
    # the group of call k: the kernels between separator k-1 and separator k
    first = sep_idx[0]
    j = first - 1
    while j >= 0 and not is_sep[j]:
        j -= 1
    bounds = [j] + sep_idx
    total = 0.0
    for k in range(n):
        ks = [r for r in rows[bounds[k] + 1:bounds[k + 1]] if "FillFunctor<int>" not in r[0]]
        us = sum(e - s for _, s, e in ks) / 1e3
        total += us
        label, fl, tile = calls[k]
        key = (label, tile)
        a = agg.setdefault(key, [0, 0.0, fl, collections.Counter()])
        a[0] += 1
        a[1] += us
        for nm, s, e in ks:
            short = nm.split("(")[0][:60]
            if "at::native" in nm:  # torch kernels between libcsk calls: name them fully
                short = nm.replace("(anonymous namespace)::", "")[:160]
                torch_kernels[(label, short)] += (e - s) / 1e3
            a[3][short] += 1
            per_kernel[nm.split("(")[0][:70]] += (e - s) / 1e3
    iters = meta.get("iters", 1)
    print(f"{n} calls over {iters} step(s): {total / iters / 1e3:.3f} ms device time per step")
    out = []
    for (label, tile), (cnt, us, fl, kn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        tf = fl * cnt / (us * 1e-6) / 1e12 if fl and us else 0.0
        print(f"{us / iters:9.1f} us {cnt // iters:3d}x {us / cnt:8.1f} us {tf:7.1f} TF/s  tile {tile}  {label}  "
              f"[{', '.join(f'{k}' for k in kn)}]")
        out.append({"op": label, "tile": tile, "calls_per_step": cnt // iters, "us_each": round(us / cnt, 2),
                    "us_per_step": round(us / iters, 1), "tflops": round(tf, 1), "kernels": list(kn)})
    if torch_kernels:
        print("torch (at::native) kernels launched before these libcsk calls (us per step):")
        for (label, nm), us in sorted(torch_kernels.items(), key=lambda kv: -kv[1]):
            print(f"  {us / iters:8.1f} us  before {label}:  {nm}")
    if out_json:
        with open(out_json, "w") as f:
            json.dump({"ms_per_step": total / iters / 1e3, "rows": out}, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--record", default="")
    ap.add_argument("--db", default="")
    ap.add_argument("--calls", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--no-cfg-dup", action="store_true")
    ap.add_argument("--model", default="sd21", choices=("sd21", "sdxl", "controlnet", "esrgan"),
                    help="sdxl: 128x128 latents (1024 px); controlnet: SD1.5 + ControlNet (config #4)")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if a.record:
        record(a.record, a.batch, a.iters, not a.no_cfg_dup, a.model)
    if a.db:
        dbs = glob.glob(a.db) or [a.db]
        analyse(dbs[0], a.calls, a.json)


if __name__ == "__main__":
    main()
