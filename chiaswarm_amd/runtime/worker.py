"""The worker daemon (reference: swarm/worker.py:34-195).

asyncio supervisor: poll the hive -> bounded work queue (depth = #devices) ->
one executor per device -> result queue -> POST results.  Poll cadence, queue
depth, error backoff and hive endpoints are the reference's.

MI355X-first changes:
  * ``ProcessExecutor``: one OS process per GPU (HIP_VISIBLE_DEVICES=i), so
    the eight GPUs of a node do not share a GIL and each keeps its own resident
    models; results are encoded in the GPU's process.
  * per-GPU watchdog: a crashed / hung child is restarted and its in-flight job
    is reported as a NON-fatal error (the hive may retry it), SURVEY §5.3.
  * the GPU children form one process group (RCCL over xGMI): models listed in
    ``settings.preload`` are read once across the node — each GPU reads 1/N of
    the checkpoint bytes, one all_gather per dtype fills every GPU
    (parallel/sharded.py).  A restarted child leaves the group (rank-local).
  * split jobs: a multi-image txt2img job may run on several idle GPUs at once
    (image j always uses seed + j, so the images do not depend on the split);
    the supervisor assembles the images in order and builds the one envelope.
  * ``ThreadExecutor`` (reference-style, in-process) for CPU plumbing runs and
    tests.
"""
from __future__ import annotations

import asyncio
import logging
import multiprocessing as mp
import os
import threading
import time

from .. import __version__
from ..hive.client import HiveClient
from ..settings import load_settings, resolve_path


def visible_gpus(settings) -> list:
    if settings.gpus:
        return [int(x) for x in str(settings.gpus).split(",") if x.strip() != ""]
    try:
        import torch  # counting devices does not initialise HIP on this image

        return list(range(torch.cuda.device_count()))
    except Exception:
        return []


class ThreadExecutor:
    def __init__(self, device_id="cpu"):
        from .device import Device

        self.device = Device(device_id)
        self.name = self.device.descriptor()

    async def run(self, job):
        from .generator import do_work

        return await do_work(job, self.device)

    async def run_batch(self, jobs, max_images=8):
        from .batcher import run_jobs

        loop = asyncio.get_running_loop()
        return await loop.run_in_executor(None, run_jobs, jobs, self.device, max_images)

    def close(self):
        pass


class ProcessExecutor:
    def __init__(self, gpu_index, env=None, job_timeout_s: float = 1800.0):
        self.gpu_index = gpu_index
        self.env = dict(env or {})
        self.job_timeout_s = job_timeout_s
        self.ctx = mp.get_context("spawn")
        self.name = f"gpu{gpu_index}"
        self.pending: dict = {}
        self.loop = None
        self.restarts = 0
        self.ready = threading.Event()
        self.ready_info = ""
        self._start()

    def _start(self):
        from .gpu_proc import gpu_main

        self.inbox = self.ctx.Queue()
        self.outbox = self.ctx.Queue()
        self.proc = self.ctx.Process(target=gpu_main, args=(self.gpu_index, self.inbox, self.outbox, self.env),
                                     daemon=True, name=f"chiaswarm-gpu{self.gpu_index}")
        self.proc.start()
        self.reader = threading.Thread(target=self._read, args=(self.outbox,), daemon=True)
        self.reader.start()

    def _read(self, outbox):
        while True:
            try:
                item = outbox.get()
            except (EOFError, OSError):
                return
            if item is None:
                return
            _, jid, result, err = item
            if jid == "__ready__":
                self.ready_info = str(err)
                self.ready.set()
                print(f"Started device {err}")
                continue
            fut = self.pending.pop(jid, None)
            if fut is not None and self.loop is not None:
                self.loop.call_soon_threadsafe(_resolve, fut, (result, err))

    def _restart(self):
        try:
            self.proc.kill()
        except Exception:
            pass
        self.proc.join(timeout=10)
        # the process group cannot re-admit a rank: the fresh child works rank-local
        self.env["WORLD_SIZE"] = "1"
        self.restarts += 1
        self._start()

    async def preload(self, names, timeout_s: float = 3600.0):
        """Collective model preload (every executor of the group, same list)."""
        self.loop = asyncio.get_running_loop()
        fut = self.loop.create_future()
        self.pending["__preloaded__"] = fut
        self.inbox.put({"__preload__": list(names)})
        result, err = await asyncio.wait_for(fut, timeout_s)
        if err:
            raise RuntimeError(f"{self.name} preload failed: {err}")
        return result

    async def run(self, job):
        from .generator import _error_result

        self.loop = asyncio.get_running_loop()
        fut = self.loop.create_future()
        jid = job.get("id")
        self.pending[jid] = fut
        self.inbox.put(job)
        t0 = time.monotonic()
        while True:
            done, _ = await asyncio.wait({fut}, timeout=2.0)
            if done:
                result, err = fut.result()
                if result is not None:
                    return result
                return _error_result(jid, RuntimeError(f"worker error: {err}"), job.get("content_type", "image/jpeg"),
                                     False)
            if not self.proc.is_alive() or time.monotonic() - t0 > self.job_timeout_s:
                why = "crashed" if not self.proc.is_alive() else "timed out"
                logging.error(f"{self.name} {why} on job {jid}; restarting")
                self.pending.pop(jid, None)
                self._restart()
                return _error_result(jid, RuntimeError(f"GPU worker {why}"), job.get("content_type", "image/jpeg"),
                                     False)

    async def run_batch(self, jobs, max_images=8):
        """Send compatible jobs as one list; the child coalesces them."""
        from .generator import _error_result

        self.loop = asyncio.get_running_loop()
        futs = {}
        for j in jobs:
            fut = self.loop.create_future()
            self.pending[j.get("id")] = fut
            futs[j.get("id")] = fut
        self.inbox.put(list(jobs))
        t0 = time.monotonic()
        why = "failed"
        while True:
            done, _ = await asyncio.wait(set(futs.values()), timeout=2.0)
            if len(done) == len(futs):
                break
            if not self.proc.is_alive() or time.monotonic() - t0 > self.job_timeout_s * len(jobs):
                why = "crashed" if not self.proc.is_alive() else "timed out"
                logging.error(f"{self.name} {why} on a batch of {len(jobs)}; restarting")
                for jid in futs:
                    self.pending.pop(jid, None)
                self._restart()
                break
        out = []
        for j in jobs:
            fut = futs[j.get("id")]
            if fut.done():
                result, err = fut.result()
                if result is not None:
                    out.append(result)
                    continue
                out.append(_error_result(j.get("id"), RuntimeError(f"worker error: {err}"),
                                         j.get("content_type", "image/jpeg"), False))
            else:
                out.append(_error_result(j.get("id"), RuntimeError(f"GPU worker {why}"),
                                         j.get("content_type", "image/jpeg"), False))
        return out

    def close(self):
        try:
            self.inbox.put(None)
            self.proc.join(timeout=10)
        finally:
            if self.proc.is_alive():
                self.proc.kill()


def _raw_key(job):
    """Batch-compatibility key of a raw hive job (None: run alone)."""
    if job.get("workflow") not in (None, "txt2img") or job.get("start_image_uri") or job.get("mask_image_uri"):
        return None
    p = job.get("parameters") or {}
    if any(p.get(k) for k in ("controlnet", "lora", "textual_inversion", "upscale")):
        return None
    if str(job.get("model_name", "")).startswith("DeepFloyd/"):
        return None
    return (job.get("model_name"), job.get("height"), job.get("width"), job.get("num_inference_steps"),
            job.get("guidance_scale"), p.get("scheduler_type"), p.get("pipeline_type"), job.get("content_type"),
            job.get("revision"))


def splittable(job) -> int:
    """Number of images of a job that may be split across GPUs (0: not splittable)."""
    if _raw_key(job) is None or not str(job.get("content_type", "image/jpeg")).startswith("image/"):
        return 0
    n = int(job.get("num_images_per_prompt", 1) or 1)
    return n if n >= 2 else 0


def _ranges(n, k):
    q, r = divmod(n, k)
    out, lo = [], 0
    for i in range(k):
        hi = lo + q + (1 if i < r else 0)
        out.append((lo, hi))
        lo = hi
    return out


def _resolve(fut, value):
    if not fut.done():
        fut.set_result(value)


class Supervisor:
    def __init__(self, settings=None, executors=None, hive=None):
        self.settings = settings or load_settings()
        self.hive = hive or HiveClient(self.settings)
        self.executors = executors if executors is not None else self._default_executors()
        n = max(1, len(self.executors))
        # batching: each device may hold up to max_batch queued jobs (max_batch <= 1:
        # the reference's queue depth of one job per device)
        self.batch_jobs = max(1, int(getattr(self.settings, "max_batch", 1) or 1))
        self.work_queue: asyncio.Queue = asyncio.Queue(maxsize=n * self.batch_jobs)
        self.result_queue: asyncio.Queue = asyncio.Queue()
        self.busy = 0
        self.results_submitted = 0
        self.splits = 0
        self.stop = asyncio.Event()
        self.locks = {id(ex): asyncio.Lock() for ex in self.executors}

    def _default_executors(self):
        gpus = visible_gpus(self.settings)
        if not gpus:
            return [ThreadExecutor("cpu")]
        # (re)build the kernel library HERE, before any child initialises HIP:
        # GPU children only check it (ops/_lib.py::check_fresh) and never run hipcc
        from ..ops._lib import ensure_built

        ensure_built()
        return [ProcessExecutor(g, env=e) for g, e in zip(gpus, group_envs(len(gpus), self.settings))]

    # ------------------------------------------------------------------ split jobs
    async def _claim_helpers(self, job, ex) -> list:
        """Idle executors for a split (an uncontended asyncio.Lock.acquire never
        suspends, so check-and-take is atomic on the event loop)."""
        if not getattr(self.settings, "split_jobs", True) or len(self.executors) < 2:
            return []
        n = splittable(job)
        if n < 2:
            return []
        helpers = []
        for other in self.executors:
            if len(helpers) + 1 >= n:
                break
            lk = self.locks[id(other)]
            if other is not ex and not lk.locked():
                await lk.acquire()
                helpers.append(other)
        return helpers

    async def _run_split(self, job, exs) -> dict:
        import random

        from .generator import _error_result

        jid = job.get("id")
        n = splittable(job)
        seed = job.get("seed")
        if seed is None:
            seed = random.SystemRandom().randrange(0, 2 ** 63 - 1)
        subs = []
        for i, (lo, hi) in enumerate(_ranges(n, len(exs))):
            subs.append(dict(job, id=f"{jid}#{i}", seed=seed, num_images_per_prompt=hi - lo,
                             _image_range=[lo, hi], _return_images=True))
        results = await asyncio.gather(*(e.run(sj) for e, sj in zip(exs, subs)))
        for r in results:
            cfg = r.get("pipeline_config", {})
            if "_images" not in cfg:  # a part failed: report it for the whole job
                out = dict(r, id=jid)
                return out
        loop = asyncio.get_running_loop()
        content_type = job.get("content_type", "image/jpeg")

        def assemble():
            import numpy as np
            from PIL import Image

            from ..output.processor import OutputProcessor, resolve_artifacts

            images = [Image.fromarray(np.asarray(a)) for r in results for a in r["pipeline_config"]["_images"]]
            op = OutputProcessor(job.get("outputs", ["primary"]), content_type)
            op.add_outputs(images)
            return resolve_artifacts({"artifacts": op.get_results()})["artifacts"]

        try:
            artifacts = await loop.run_in_executor(None, assemble)
        except Exception as e:
            return _error_result(jid, e, content_type, False)
        cfg = {k: v for k, v in results[0]["pipeline_config"].items() if k != "_images"}
        cfg["seed"] = seed
        cfg["split"] = len(exs)
        nsfw = any(r.get("nsfw", False) for r in results)
        self.splits += 1
        from .. import __version__

        return {"id": jid, "artifacts": artifacts, "nsfw": nsfw, "worker_version": __version__,
                "pipeline_config": cfg}

    async def preload(self, names):
        """Every executor loads the same models together (sharded reads + all_gather)."""
        names = [n for n in names if n]
        if not names:
            return []
        return await asyncio.gather(*(ex.preload(names) for ex in self.executors if hasattr(ex, "preload")))

    def _drain_compatible(self, first) -> list:
        """Take queued jobs that can share ``first``'s UNet batch (cheap raw-job
        check; runtime.batcher re-validates after routing)."""
        batch = [first]
        if self.batch_jobs <= 1 or not hasattr(self.executors[0], "run_batch"):
            return batch
        keep = []
        while not self.work_queue.empty() and len(batch) < self.batch_jobs:
            j = self.work_queue.get_nowait()
            if _raw_key(j) is not None and _raw_key(j) == _raw_key(first):
                batch.append(j)
            else:
                keep.append(j)
            self.work_queue.task_done()
        for j in keep:
            self.work_queue.put_nowait(j)
        return batch

    async def device_worker(self, ex):
        lock = self.locks[id(ex)]
        while True:
            job = await self.work_queue.get()
            batch = self._drain_compatible(job)
            self.busy += len(batch)
            helpers = []
            try:
                async with lock:  # a split job may hold this executor as a helper
                    if len(batch) == 1:
                        helpers = await self._claim_helpers(job, ex)
                        if helpers:
                            self.busy += len(helpers)
                            results = [await self._run_split(job, [ex] + helpers)]
                        else:
                            results = [await ex.run(job)]
                    else:
                        results = await ex.run_batch(batch, max(1, int(self.settings.max_batch)))
                for result in results:
                    await self.result_queue.put(result)
            except Exception as e:
                logging.exception(e)
                print(f"device_worker {e}")
            finally:
                for h in helpers:
                    self.locks[id(h)].release()
                self.busy -= len(batch) + len(helpers)
                self.work_queue.task_done()

    async def result_worker(self):
        while True:
            result = await self.result_queue.get()
            try:
                print("Result complete")
                await self.hive.submit_result(result)
                self.results_submitted += 1
            except Exception as e:
                logging.exception(e)
                print(f"result_worker {e}")
            finally:
                self.result_queue.task_done()

    async def run(self, max_polls: int | None = None):
        logging.info(f"worker {__version__}")
        pre = [n.strip() for n in str(getattr(self.settings, "preload", "") or "").split(",") if n.strip()]
        if pre:
            try:
                await self.preload(pre)
            except Exception as e:  # a failed preload leaves models to load on demand
                logging.exception(e)
                print(f"preload failed: {e}")
        tasks = [asyncio.create_task(self.device_worker(ex)) for ex in self.executors]
        tasks.append(asyncio.create_task(self.result_worker()))
        polls = 0
        try:
            while not self.stop.is_set():
                while (self.work_queue.full() or
                       self.busy + self.work_queue.qsize() >= len(self.executors) * self.batch_jobs) \
                        and not self.stop.is_set():
                    await asyncio.sleep(0.05 if max_polls else 1)
                jobs, sleep_s = await self.hive.ask_for_work()
                for job in jobs:
                    await self.work_queue.put(job)
                polls += 1
                if max_polls is not None and polls >= max_polls:
                    break
                try:
                    await asyncio.wait_for(self.stop.wait(), timeout=sleep_s)
                except asyncio.TimeoutError:
                    pass
            await self.work_queue.join()
            await self.result_queue.join()
        finally:
            for t in tasks:
                t.cancel()


def group_envs(n: int, settings=None, port: int | None = None) -> list:
    """Per-child process-group environment (RANK, WORLD_SIZE, MASTER_*)."""
    if n <= 1 or (settings is not None and not getattr(settings, "distributed", True)):
        return [{} for _ in range(n)]
    if port is None:
        import socket

        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
    return [{"RANK": str(i), "WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
             "HSA_ENABLE_IPC_MODE_LEGACY": "0"} for i in range(n)]


def startup(settings=None, require_gpu=True):
    from ..log_setup import setup_logging

    s = settings or load_settings()
    setup_logging(resolve_path(s.log_filename), s.log_level)
    logging.info(f"Version {__version__}")
    if require_gpu and not visible_gpus(s) and not os.environ.get("SDAAS_ALLOW_CPU"):
        raise Exception("No GPU present (set SDAAS_ALLOW_CPU=1 for a CPU plumbing run). Quitting.")
    return s


async def run_worker(max_polls=None):
    s = startup()
    sup = Supervisor(s)
    print(f"Found {len(sup.executors)} devices")
    try:
        await sup.run(max_polls=max_polls)
    finally:
        for ex in sup.executors:
            ex.close()


def main():
    asyncio.run(run_worker())


if __name__ == "__main__":
    main()
