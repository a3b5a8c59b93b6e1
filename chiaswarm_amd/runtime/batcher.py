"""Request coalescing (SURVEY §7.1 ``batcher.py``): compatible txt2img jobs that
are queued for the same GPU run as ONE UNet batch.

The reference ran exactly one job per GPU at a time (swarm/worker.py:40-44);
on an MI355X a single 512² job (CFG batch 2) leaves most of the 256 CUs idle,
while a CFG batch of 8-16 runs near the kernels' efficient regime.  Jobs are
compatible when everything that shapes the UNet call matches (model, size,
steps, scheduler, guidance) and none of them carries per-job conditioning the
batched path does not split (init image, mask, ControlNet, LoRA, textual
inversion, upscale).  Every job keeps its own seed: its initial noise is drawn
from its own generator, so with a deterministic sampler (DPM-Solver++ 2M,
Euler, DDIM, ...) a batched job returns exactly the images it would alone.
"""
from __future__ import annotations

import logging
import time

from .. import __version__

# kwargs (after jobs.router.format_args) that must be equal across a batch
KEY_FIELDS = ("model_name", "revision", "pipeline_type", "scheduler_type", "num_inference_steps", "guidance_scale",
              "height", "width", "content_type", "eta")
# kwargs that make a job unbatchable
SOLO_FIELDS = ("image", "mask_image", "controlnet_model_name", "lora", "textual_inversion", "latents",
               "prompt_embeds", "negative_prompt_embeds")


def batch_key(fn, kwargs) -> tuple | None:
    if getattr(fn, "__name__", "") != "diffusion_callback":
        return None
    if any(kwargs.get(k) is not None for k in SOLO_FIELDS) or kwargs.get("upscale"):
        return None
    if not isinstance(kwargs.get("prompt", ""), str):
        return None
    return tuple(str(kwargs.get(k)) for k in KEY_FIELDS)


def images_of(kwargs) -> int:
    return max(1, int(kwargs.get("num_images_per_prompt", 1) or 1))


def run_jobs(jobs: list[dict], device, max_images: int = 8) -> list[dict]:
    """Execute queued jobs on one device, coalescing compatible txt2img jobs.
    Returns one result envelope per job, in input order."""
    from ..jobs.router import format_args
    from .generator import _error_result, synchronous_do_work_function

    results: dict = {}
    groups: dict = {}
    order = []
    for job in jobs:
        jid = job.get("id")
        order.append(jid)
        try:
            fn, kwargs = format_args(dict((k, v) for k, v in job.items() if k != "id"))
        except Exception as e:  # routing errors are fatal, as in the single-job path
            logging.exception(e)
            results[jid] = _error_result(jid, e, job.get("content_type", "image/jpeg"), True)
            continue
        key = batch_key(fn, kwargs)
        if key is None:
            results[jid] = synchronous_do_work_function(job, device)
            continue
        groups.setdefault(key, []).append((jid, job, kwargs))
    for members in groups.values():
        # split into batches of <= max_images images
        batch, n = [], 0
        chunks = []
        for m in members:
            k = images_of(m[2])
            if batch and n + k > max_images:
                chunks.append(batch)
                batch, n = [], 0
            batch.append(m)
            n += k
        if batch:
            chunks.append(batch)
        for chunk in chunks:
            if len(chunk) == 1:
                jid, job, _ = chunk[0]
                results[jid] = synchronous_do_work_function(job, device)
                continue
            results.update(_run_batch(chunk, device))
    return [results[j] for j in order]


def _run_batch(chunk, device) -> dict:
    from ..pipelines.diffusion import diffusion_batch
    from .generator import synchronous_do_work_function

    t0 = time.perf_counter()
    try:
        outs = device.run_batch(diffusion_batch, [kw for _, _, kw in chunk])
    except Exception as e:  # fall back to one-by-one (gets the per-job error classes right)
        logging.exception(e)
        return {jid: synchronous_do_work_function(job, device) for jid, job, _ in chunk}
    res = {}
    for (jid, _, _), (artifacts, cfg) in zip(chunk, outs):
        cfg["batched_with"] = len(chunk)
        if isinstance(cfg.get("timings"), dict):
            cfg["timings"]["total"] = round(time.perf_counter() - t0, 4)
        res[jid] = {"id": jid, "artifacts": artifacts, "nsfw": cfg.get("nsfw", False),
                    "worker_version": __version__, "pipeline_config": cfg}
    return res
