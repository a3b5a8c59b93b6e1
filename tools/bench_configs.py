#!/usr/bin/env python
"""Secondary BASELINE.json configs on one MI355X (random weights, synthetic inputs):

  sdxl      SDXL-base 1024x1024, 30 steps, batch 1 per GPU (config #3's per-GPU share)
  controlnet ControlNet-canny on SD1.5 512x512 (config #4), batch 1 and 4
  x2up      sd-x2-latent-upscaler K-UNet 512 -> 1024, 20 steps (the ``upscale`` option)
  esrgan    Real-ESRGAN x4 512 -> 2048 (config #5)
  sd21-b1   SD2.1 512x512 50 steps batch 1 (latency)
  audioldm  AudioLDM-S 10 s clip, 25 steps (txt2audio default)
  bark      Bark (large) ~ one sentence

    python tools/bench_configs.py --only sdxl,esrgan [--impl hip|reference]
Prints one JSON line per config (images/s, p50 latency ms).
"""
from __future__ import annotations

import os as _os

# synthetic (random-init) weights of the real architectures: there are no
# checkpoints on the bench / profiling boxes (runtime/provision.py)
_os.environ.setdefault("SDAAS_ALLOW_RANDOM", "1")
_os.environ.setdefault("SDAAS_OFFLINE", "1")

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from chiaswarm_amd import ops  # noqa: E402


LAST_PHASES: dict = {}


def timed(fn, reps, warm=1):
    """Wall latencies of ``reps`` calls; the pipelines' own phase timings
    (text encode / prepare / denoise / decode, device-synchronised) are kept
    as per-phase medians in LAST_PHASES."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    lat, ph = [], {}
    for _ in range(reps):
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
        for k, v in (getattr(out, "timings", None) or {}).items():
            ph.setdefault(k, []).append(v)
    LAST_PHASES.clear()
    LAST_PHASES.update({k: round(1000 * statistics.median(v), 2) for k, v in ph.items()})
    return lat


def emit(name, imgs_per_call, lat, extra=None):
    p50 = statistics.median(lat)
    rec = {"config": name, "images_per_s": round(imgs_per_call / p50, 4), "p50_latency_ms": round(1000 * p50, 1),
           "impl": ops.get_mode(), "reps": len(lat)}
    rec.update(extra or {})
    if LAST_PHASES:
        rec["phase_ms_median"] = dict(LAST_PHASES)
    print(json.dumps(rec), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="sdxl,controlnet,esrgan,sd21-b1")
    ap.add_argument("--impl", default="hip")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    ops.set_mode(a.impl)
    ops._lib.load()
    dev = torch.device("cuda", 0)
    todo = a.only.split(",")
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.schedulers import get_scheduler

    if "sd21-b1" in todo:
        p = StableDiffusion("sd21", device=dev)
        g = torch.Generator(device=dev)
        lat = timed(lambda: p(prompt="a fox", num_inference_steps=50, height=512, width=512, generator=g.manual_seed(0),
                              scheduler=get_scheduler("DPMSolverMultistepScheduler")), a.reps)
        emit("sd21-512-50step-batch1", 1, lat)
        del p
    if "sdxl" in todo:
        p = StableDiffusion("sdxl", device=dev)
        g = torch.Generator(device=dev)
        lat = timed(lambda: p(prompt="a fox", num_inference_steps=30, height=1024, width=1024,
                              generator=g.manual_seed(0), scheduler=get_scheduler("EulerDiscreteScheduler")), a.reps)
        emit("sdxl-1024-30step-batch1", 1, lat, {"scheduler": "EulerDiscreteScheduler"})
        del p
    if "controlnet" in todo:
        from chiaswarm_amd.controlnet.preprocess import image_to_canny
        from chiaswarm_amd.pipelines.controlnet import load_controlnet

        p = StableDiffusion("sd15", device=dev)
        p.controlnet = load_controlnet("lllyasviel/control_v11p_sd15_canny", p, str(dev))
        rng = np.random.default_rng(0)
        img = Image.fromarray((rng.random((512, 512, 3)) * 255).astype(np.uint8))
        g = torch.Generator(device=dev)

        for n in (1, 4):
            def run(n=n):
                cond = image_to_canny(img)
                p(prompt="a house", image=cond, num_inference_steps=30, generator=g.manual_seed(0),
                  num_images_per_prompt=n, scheduler=get_scheduler("DPMSolverMultistepScheduler"))

            lat = timed(run, a.reps)
            emit(f"controlnet-canny-sd15-512-30step{'' if n == 1 else '-batch4'}", n, lat)
        del p
    if "x2up" in todo:
        from chiaswarm_amd.pipelines.upscale import LatentUpscaler

        up = LatentUpscaler(str(dev))
        rng = np.random.default_rng(0)
        ims = [Image.fromarray((rng.random((512, 512, 3)) * 255).astype(np.uint8))]
        g = torch.Generator(device=dev)
        lat = timed(lambda: up(["a fox"], ims, num_inference_steps=20, generator=g.manual_seed(0)), a.reps)
        emit("latent-x2-upscaler-512to1024-20step", 1, lat)
        del up
    if "audioldm" in todo:
        from chiaswarm_amd.pipelines.audio import AudioLDM

        p = AudioLDM(str(dev))
        g = torch.Generator(device=dev)
        lat = timed(lambda: p(prompt="rain on a tin roof", num_inference_steps=25, audio_length_in_s=10.0,
                              generator=g.manual_seed(0)), a.reps)
        emit("audioldm-10s-25step", 1, lat, {"phases_ms": {k: round(v * 1000, 1) for k, v in p.timings.items()}})
        del p
    if "bark" in todo:
        from chiaswarm_amd.models.bark import Bark

        bk = Bark(str(dev), size="large")
        lat = timed(lambda: bk.generate_audio("Hello, this is a test of the speech model.", seed=0,
                                              max_semantic_tokens=256), a.reps, warm=0)
        emit("bark-large-256-semantic-tokens", 1, lat)
        del bk
    if "esrgan" in todo:
        from chiaswarm_amd.pipelines.esrgan import load_esrgan, upscale_x4

        net = load_esrgan("xinntao/RealESRGAN_x4plus", str(dev))
        rng = np.random.default_rng(0)
        img = Image.fromarray((rng.random((512, 512, 3)) * 255).astype(np.uint8))
        lat = timed(lambda: upscale_x4(net, img), a.reps)
        emit("realesrgan-x4-512to2048", 1, lat)


if __name__ == "__main__":
    main()
