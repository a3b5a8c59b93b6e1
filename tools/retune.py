#!/usr/bin/env python
"""Re-measure part of the per-shape GEMM/conv table on this GPU.

Drops the shipped entries whose key matches --drop (regex), runs the given
models once with CSK_AUTOTUNE=1 (every miss is timed over all (tile, split)
candidates, outside graph capture) and writes the merged table:

    python tools/retune.py --drop '^g:.*:3$' --models sd21 --out gpurun_out/tune_gfx950.json
"""
import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["CSK_AUTOTUNE"] = "1"

import torch  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402
from chiaswarm_amd.ops import tuning  # noqa: E402


def run_model(name, dev):
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    if name in ("sd21", "sd15", "sdxl"):
        size = 1024 if name == "sdxl" else 512
        batch = 1 if name == "sdxl" else 4
        p = StableDiffusion(name, device=dev, seed=0)
        p.use_graphs = False
        g = torch.Generator(device=dev).manual_seed(0)
        p(prompt="tune", num_inference_steps=2, height=size, width=size, num_images_per_prompt=batch, generator=g)
    elif name == "esrgan":  # Real-ESRGAN x4plus, 512 -> 2048 (config #5): RRDB convs at 512^2, up-convs
        import numpy as np
        from PIL import Image

        from chiaswarm_amd.pipelines.esrgan import load_esrgan, upscale_x4

        net = load_esrgan("xinntao/RealESRGAN_x4plus", str(dev))
        img = Image.fromarray((np.random.default_rng(0).random((512, 512, 3)) * 255).astype(np.uint8))
        upscale_x4(net, img)
    elif name == "controlnet":  # SD1.5 + ControlNet-canny 512^2 (config #4), batch 1 and 4
        import numpy as np
        from PIL import Image

        from chiaswarm_amd.controlnet.preprocess import image_to_canny
        from chiaswarm_amd.pipelines.controlnet import load_controlnet
        from chiaswarm_amd.pipelines.sd import StableDiffusion

        p = StableDiffusion("sd15", device=dev, seed=0)
        p.controlnet = load_controlnet("lllyasviel/control_v11p_sd15_canny", p, str(dev))
        p.use_graphs = False
        img = image_to_canny(Image.fromarray((np.random.default_rng(0).random((512, 512, 3)) * 255).astype(np.uint8)))
        g = torch.Generator(device=dev)
        for n in (1, 4):
            p(prompt="tune", image=img, num_inference_steps=2, num_images_per_prompt=n, generator=g.manual_seed(0))
    else:
        raise SystemExit(f"unknown model {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--drop", default="", help="regex of table keys to re-measure")
    ap.add_argument("--models", default="sd21")
    ap.add_argument("--out", default="gpurun_out/tune_gfx950.json")
    a = ap.parse_args()
    ops._lib.load()
    t = tuning.table()
    dropped = {}
    if a.drop:
        rx = re.compile(a.drop)
        for k in [k for k in t if rx.search(k)]:
            dropped[k] = t.pop(k)
            print("re-measure", k, dropped[k], flush=True)
    before = set(t)
    dev = torch.device("cuda", 0)
    for m in a.models.split(","):
        run_model(m, dev)
    for k in sorted(set(t) - before):
        print("measured", k, t[k], "was", dropped.get(k), flush=True)
    for k, v in dropped.items():  # entries of models not run this time stay as they were
        t.setdefault(k, v)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(t, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()
