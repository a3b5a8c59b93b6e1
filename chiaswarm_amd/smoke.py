"""Manual smoke jobs (reference: swarm/test.py:7-77 — canned job dicts run
through the real ``do_work`` on device 0; prints "ok" or the error).

    python -m swarm.test [sd|txt2audio|vid2vid|txt2vid|bark|if|tiny] [--cpu] [--synthetic]

Models are provisioned like any job (fetched on a miss, runtime/provision.py);
``--synthetic`` runs seeded random-init weights of the same architecture
instead (SDAAS_ALLOW_RANDOM=1, no fetch) — a plumbing check on a box without
checkpoints.  The "tiny" job always runs synthetic.
"""
from __future__ import annotations

import argparse
import asyncio

NEG = "ugly, duplicate, morbid, mutilated, extra fingers, blurry, bad anatomy"

JOBS = {
    "sd": {"id": "__test__", "model_name": "stabilityai/stable-diffusion-2-1", "prompt": "spoons",
           "num_inference_steps": 10, "outputs": ["primary", "inference_image_strip"]},
    "tiny": {"id": "__test__", "model_name": "tiny/sd", "prompt": "spoons", "num_inference_steps": 4,
             "height": 64, "width": 64, "outputs": ["primary"]},
    "txt2audio": {"id": "__test__", "model_name": "cvssp/audioldm", "workflow": "txt2audio",
                  "prompt": "Techno music with a strong, upbeat tempo", "num_inference_steps": 10,
                  "outputs": ["primary"]},
    "vid2vid": {"id": "__test__", "model_name": "timbrooks/instruct-pix2pix", "prompt": "make it sunny",
                "negative_prompt": NEG, "num_inference_steps": 10, "workflow": "vid2vid",
                "video_uri": "https://example.invalid/video.mp4", "outputs": ["primary"]},
    "txt2vid": {"id": "__test__", "model_name": "damo-vilab/text-to-video-ms-1.7b", "prompt": "dogs dancing",
                "negative_prompt": NEG, "num_inference_steps": 10, "workflow": "txt2vid", "outputs": ["primary"]},
    "bark": {"id": "__test__", "model_name": "suno/bark", "prompt": "Hola, mi nombre es Pepe", "workflow": "txt2audio",
             "outputs": ["primary"]},
    "if": {"id": "__test__", "model_name": "DeepFloyd/IF-II-L-v1.0", "prompt": "a green frog", "workflow": "txt2img",
           "outputs": ["primary"]},
}


async def run_test(job, cpu=False):
    from .runtime.device import Device
    from .runtime.generator import do_work

    result = await do_work(dict(job), Device("cpu" if cpu else 0))
    if "error" in result["pipeline_config"]:
        print(result["pipeline_config"]["error"])
    else:
        print("ok")
    return result


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("job", nargs="?", default="sd", choices=sorted(JOBS))
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--synthetic", action="store_true", help="random-init weights, no fetch")
    a = ap.parse_args(argv)
    if a.synthetic or a.job == "tiny":
        import os

        os.environ["SDAAS_ALLOW_RANDOM"] = "1"
        os.environ["SDAAS_OFFLINE"] = "1"
    asyncio.run(run_test(JOBS[a.job], a.cpu))


if __name__ == "__main__":
    main()
