"""One OS process per GPU: the reference ran every GPU as a
thread of one Python process (swarm/generator.py:13-14, one shared GIL); here
each GPU gets its own process that owns its HBM-resident model cache and runs
jobs.  Results are encoded (grid, JPEG, thumbnail, base64, sha256) by a small
pool of encoder processes this process starts BEFORE it touches the GPU
(output/encoder.py): the GPU thread hands over uint8 pixels and goes straight on
to the next job; a finisher thread resolves the encodings and posts results.

This module must not import torch at import time: the child selects its GPU via
HIP_VISIBLE_DEVICES *before* torch initialises.
"""
from __future__ import annotations

import os
import traceback


def gpu_main(gpu_index, inbox, outbox, env: dict | None = None):
    """Child entry point.  inbox: job dicts (None = stop); outbox: (gpu, job_id, result|None, err)."""
    if gpu_index != "cpu":
        os.environ["HIP_VISIBLE_DEVICES"] = str(gpu_index)
        os.environ["CUDA_VISIBLE_DEVICES"] = str(gpu_index)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k, v in (env or {}).items():
        os.environ[k] = v
    # encoder processes first: spawning is only safe before this process initialises HIP
    from ..output.encoder import EncoderPool
    from ..output.processor import resolve_artifacts, set_encoder_pool

    encoders = EncoderPool() if gpu_index != "cpu" else None
    if encoders is not None and encoders.kind == "process":
        set_encoder_pool(encoders)
    import concurrent.futures as cf

    finisher = cf.ThreadPoolExecutor(max_workers=1)

    def post(jid, result):
        """Resolve deferred artifacts off the GPU thread, then hand the result over."""
        def run():
            try:
                outbox.put((gpu_index, jid, resolve_artifacts(result), None))
            except BaseException as e:
                outbox.put((gpu_index, jid, None, f"result encoding failed: {e}\n{traceback.format_exc()}"))
        finisher.submit(run)

    from ..log_setup import setup_logging
    from ..settings import load_settings, resolve_path
    from .device import Device
    from .generator import synchronous_do_work_function

    settings = load_settings()
    try:
        setup_logging(resolve_path(settings.log_filename), settings.log_level, suffix=f"gpu{gpu_index}")
    except Exception:
        pass
    device = Device("cpu" if gpu_index == "cpu" else 0)
    outbox.put((gpu_index, "__ready__", None, device.descriptor()))
    while True:
        job = inbox.get()
        if job is None:
            break
        if isinstance(job, list):  # a coalesced batch (runtime.batcher)
            from .batcher import run_jobs

            try:
                for res in run_jobs(job, device, max(1, settings.max_batch)):
                    post(res["id"], res)
            except BaseException as e:
                for j in job:
                    outbox.put((gpu_index, j.get("id"), None, f"{e}\n{traceback.format_exc()}"))
            continue
        jid = job.get("id")
        try:
            result = synchronous_do_work_function(job, device)
            post(jid, result)
        except BaseException as e:  # never let the loop die silently
            outbox.put((gpu_index, jid, None, f"{e}\n{traceback.format_exc()}"))
    finisher.shutdown(wait=True)  # every pending result is posted before the process exits
    if encoders is not None:
        encoders.shutdown()
