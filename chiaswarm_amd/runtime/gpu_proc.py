"""One OS process per GPU: the reference ran every GPU as a
thread of one Python process (swarm/generator.py:13-14, one shared GIL); here
each GPU gets its own process that owns its HBM-resident model cache and runs
jobs.  Results are encoded (grid, JPEG, thumbnail, base64, sha256) by a small
pool of encoder processes this process starts BEFORE it touches the GPU
(output/encoder.py): the GPU thread hands over uint8 pixels and goes straight on
to the next job; a finisher thread resolves the encodings and posts results.

With ``WORLD_SIZE`` > 1 in its environment (set by the supervisor) the child
joins the node's process group — RCCL over xGMI (``nccl`` backend), gloo for
CPU children — before any GPU work.  The group is used for collective model
preloads: every child reads 1/N of each checkpoint's bytes and an all_gather
assembles the rest (parallel/sharded.py).  Job-triggered loads stay local.

This module must not import torch at import time: the child selects its GPU via
HIP_VISIBLE_DEVICES *before* torch initialises.
"""
from __future__ import annotations

import os
import traceback


def _join_group(gpu_index) -> str:
    """Join the node's process group (RANK / WORLD_SIZE / MASTER_* in the env).
    Returns a status string; a failure leaves the child working rank-local."""
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return "single"
    os.environ["LOCAL_RANK"] = "0"  # this child sees exactly one GPU (HIP_VISIBLE_DEVICES)
    from ..parallel import comm

    backend = "gloo" if gpu_index == "cpu" else os.environ.get("CSK_DIST_BACKEND", "nccl")
    try:
        comm.init_distributed(backend=backend, timeout_s=int(os.environ.get("CSK_DIST_TIMEOUT", "600")))
        return f"{backend} rank {os.environ.get('RANK')}/{os.environ.get('WORLD_SIZE')}"
    except Exception as e:  # pragma: no cover - depends on the node
        import logging

        logging.exception(e)
        return f"no group ({e})"


def _preload(names: list, device_id: str) -> dict:
    """Collective preload of SD-family models (every child, same list, same order)."""
    from ..parallel import comm
    from ..pipelines.diffusion import load_sd

    done = {}
    with comm.collective_loading():
        for name in names:
            pipe = load_sd(name, device_id)
            done[name] = pipe.config.get("weights", "random-init")
    return done


def _test_hook(job):
    """CSK_TEST_HOOKS=1 only: deterministic crash / hang for the watchdog tests."""
    if os.environ.get("CSK_TEST_HOOKS") != "1" or not isinstance(job, dict):
        return
    what = job.get("_test")
    if what == "exit":
        os._exit(3)
    if what == "hang":
        import time

        time.sleep(3600)


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
    group = _join_group(gpu_index)
    device = Device("cpu" if gpu_index == "cpu" else 0)
    outbox.put((gpu_index, "__ready__", None, f"{device.descriptor()} [{group}]"))
    while True:
        job = inbox.get()
        if job is None:
            break
        if isinstance(job, dict) and "__preload__" in job:
            try:
                res = _preload(list(job["__preload__"]), device.identifier())
                outbox.put((gpu_index, "__preloaded__", res, None))
            except BaseException as e:
                outbox.put((gpu_index, "__preloaded__", None, f"{e}\n{traceback.format_exc()}"))
            continue
        for j in (job if isinstance(job, list) else [job]):
            _test_hook(j)
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
