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

GPU visibility: by default every child sees ALL of the node's GPUs and binds
its own with ``torch.cuda.set_device(i)`` (LOCAL_RANK = i), so RCCL can see its
peers and take the P2P / xGMI paths (a child isolated with HIP_VISIBLE_DEVICES
sees no peer device, which leaves RCCL only host-memory transports);
``SDAAS_GPU_ISOLATION=1`` restores the one-visible-GPU child.

The process group's rendezvous store lives in the SUPERVISOR (runtime/worker.py)
so no GPU child's death takes it down; ``__regroup__`` re-forms the group (a new
store generation) after a child was restarted.

This module must not import torch at import time: an isolated child selects its
GPU via HIP_VISIBLE_DEVICES *before* torch initialises.
"""
from __future__ import annotations

import os
import traceback


def _isolated() -> bool:
    return os.environ.get("SDAAS_GPU_ISOLATION", "0") == "1"


def _local_index(gpu_index) -> int:
    """The torch device index of this child's GPU."""
    return 0 if (gpu_index == "cpu" or _isolated()) else int(gpu_index)


def _join_group(gpu_index) -> dict:
    """Join the node's process group (RANK / WORLD_SIZE / SDAAS_STORE_* /
    SDAAS_GROUP_GEN in the env).  Returns the group status the supervisor
    checks before it issues any collective: {"gen", "rank", "world"} when
    joined, {"error": ...} on failure (the child then works rank-local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return {"world": 1}
    os.environ["LOCAL_RANK"] = str(_local_index(gpu_index))
    from ..parallel import comm

    backend = "gloo" if gpu_index == "cpu" else os.environ.get("CSK_DIST_BACKEND", "nccl")
    try:
        comm.init_distributed(backend=backend, timeout_s=int(os.environ.get("CSK_DIST_TIMEOUT", "600")))
        return {"gen": int(os.environ.get("SDAAS_GROUP_GEN", "0")), "rank": int(os.environ["RANK"]),
                "world": world, "backend": backend}
    except Exception as e:  # pragma: no cover - depends on the node
        import logging

        logging.exception(e)
        comm.leave_group()
        return {"error": f"{type(e).__name__}: {e}"}


def _regroup(gpu_index, spec: dict) -> dict:
    """Leave the current group (aborting its communicators: a peer may be dead)
    and join generation ``spec['gen']`` as ``spec['rank']`` of ``spec['world']``."""
    from ..parallel import comm

    comm.leave_group()
    os.environ.update({"RANK": str(spec["rank"]), "WORLD_SIZE": str(spec["world"]),
                       "SDAAS_GROUP_GEN": str(spec["gen"]), "SDAAS_STORE_PORT": str(spec["store_port"])})
    return _join_group(gpu_index)


def _preload(names: list, device_id: str, collective: bool = True) -> dict:
    """Preload of SD-family models.  ``collective``: every child of the group
    loads the same list in the same order, reading 1/N of the bytes each
    (the supervisor sends it only when every child reported the same group)."""
    import contextlib

    from ..parallel import comm
    from ..pipelines.diffusion import load_sd

    done = {}
    with comm.collective_loading() if collective else contextlib.nullcontext():
        for name in names:
            if name == "__test_exit__" and os.environ.get("CSK_TEST_HOOKS") == "1":
                if os.environ.get("RANK") == os.environ.get("CSK_TEST_EXIT_RANK", "1"):
                    os._exit(3)  # a rank dying inside a collective preload (tests/test_worker_procs.py)
                continue
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


def _watch_parent(period_s: float = 1.0) -> None:
    """The child is not daemonic (it owns encoder processes): end it when the
    supervisor process is gone (re-parented), whatever killed the supervisor."""
    import threading
    import time

    parent = os.getppid()

    def run():
        while True:
            time.sleep(period_s)
            if os.getppid() != parent:
                os._exit(3)

    threading.Thread(target=run, daemon=True, name="csk-parent-watch").start()


def gpu_main(gpu_index, inbox, outbox, env: dict | None = None):
    """Child entry point.  inbox: job dicts (None = stop); outbox: (gpu, job_id, result|None, err)."""
    _watch_parent()
    if gpu_index != "cpu" and _isolated():
        os.environ["HIP_VISIBLE_DEVICES"] = str(gpu_index)
        os.environ["CUDA_VISIBLE_DEVICES"] = str(gpu_index)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    for k, v in (env or {}).items():
        os.environ[k] = v
    # encoder processes first: spawning is only safe before this process initialises HIP
    from ..output.encoder import EncoderPool
    from ..output.processor import resolve_artifacts, set_encoder_pool

    # (cpu children: only when asked, tests/test_worker_procs.py)
    encoders = EncoderPool() if gpu_index != "cpu" or os.environ.get("CSK_CHILD_ENCODERS") == "1" else None
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
    if gpu_index != "cpu":
        import torch

        torch.cuda.set_device(_local_index(gpu_index))  # before any allocation: this child's GPU
    group = _join_group(gpu_index)
    device = Device("cpu" if gpu_index == "cpu" else _local_index(gpu_index))
    outbox.put((gpu_index, "__ready__", None, {"desc": device.descriptor(), "group": group,
                                               "encoders": "none" if encoders is None else encoders.kind}))
    while True:
        job = inbox.get()
        if job is None:
            break
        if isinstance(job, dict) and "__preload__" in job:
            try:
                res = _preload(list(job["__preload__"]), device.identifier(), bool(job.get("collective", True)))
                outbox.put((gpu_index, "__preloaded__", res, None))
            except BaseException as e:
                outbox.put((gpu_index, "__preloaded__", None, f"{e}\n{traceback.format_exc()}"))
            continue
        if isinstance(job, dict) and "__regroup__" in job:
            try:
                outbox.put((gpu_index, "__regrouped__", _regroup(gpu_index, job["__regroup__"]), None))
            except BaseException as e:
                outbox.put((gpu_index, "__regrouped__", None, f"{e}\n{traceback.format_exc()}"))
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
            # the device part is done: the supervisor may hand over the next job
            # while this one's envelope is still being encoded (post)
            outbox.put((gpu_index, f"__gpu_done__:{jid}", None, None))
            post(jid, result)
        except BaseException as e:  # never let the loop die silently
            outbox.put((gpu_index, jid, None, f"{e}\n{traceback.format_exc()}"))
    finisher.shutdown(wait=True)  # every pending result is posted before the process exits
    if encoders is not None:
        encoders.shutdown()
