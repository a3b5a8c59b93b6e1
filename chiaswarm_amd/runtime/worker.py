"""The worker daemon (reference: swarm/worker.py:34-195).

asyncio supervisor: poll the hive -> bounded work queue (depth = #devices) ->
one executor per device -> result queue -> POST results.  Poll cadence, queue
depth, error backoff and hive endpoints are the reference's.

MI355X-first changes:
  * ``ProcessExecutor``: one OS process per GPU (torch.cuda.set_device(i), all
    GPUs visible so RCCL sees its peers), so the eight GPUs of a node do not
    share a GIL and each keeps its own resident models; results are encoded in
    the GPU's process.
  * per-GPU watchdog: a crashed / hung child is restarted and its in-flight job
    is reported as a NON-fatal error (the hive may retry it), SURVEY §5.3.
  * the GPU children form one process group (RCCL over xGMI) whose rendezvous
    store (a TCPStore) lives HERE in the supervisor, so a child's death never
    takes the store with it.  Collectives are issued only while every child
    reports the same group generation; a restarted child comes back rank-local
    and the next idle moment re-forms the group (a new generation).
  * preload: models listed in ``settings.preload`` are read once across the
    node — each GPU reads 1/N of the checkpoint bytes, one all_gather per
    dtype fills every GPU (parallel/sharded.py); a child dying mid-preload
    restarts every group child (the others may be wedged in the collective).
  * split jobs: a multi-image txt2img job may run on several idle GPUs at once
    (image j always uses seed + j, so the images do not depend on the split);
    with a healthy group the helpers send their uint8 images device-to-device
    to the leading GPU (RCCL point-to-point over xGMI), which builds the one
    envelope; without one the supervisor assembles pickled images.
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
        self.gpu_done: dict = {}  # job id -> asyncio.Event set when the child's device part is done
        self.loop = None
        self.restarts = 0
        self.ready = threading.Event()
        self.ready_info = ""
        self.group: dict = {}  # the child's process-group status ({"gen", "rank", "world"} when joined)
        self.encoders = "none"  # the child's result encoders: "process" | "thread" | "none" (cpu children)
        self._start()

    def _start(self):
        from .gpu_proc import gpu_main

        self.ready.clear()
        self.group = {}
        self.inbox = self.ctx.Queue()
        self.outbox = self.ctx.Queue()
        # NOT daemonic: a daemonic process may not start children, and the GPU
        # child starts its JPEG encoder processes (output/encoder.py) — as a
        # daemon it silently fell back to encoding on its GPU thread (30.8 ms
        # per 4-image job, profiles/bench_sup_phases_r6d.json).  gpu_main exits
        # by itself when this process disappears (parent watchdog).
        self.proc = self.ctx.Process(target=gpu_main, args=(self.gpu_index, self.inbox, self.outbox, self.env),
                                     daemon=False, name=f"chiaswarm-gpu{self.gpu_index}")
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
                info = err if isinstance(err, dict) else {"desc": str(err), "group": {}}
                self.group = dict(info.get("group") or {})
                self.encoders = info.get("encoders", "none")
                self.ready_info = f"{info.get('desc')} [{_group_str(self.group)}]"
                self.ready.set()
                print(f"Started device {self.ready_info}")
                continue
            if isinstance(jid, str) and jid.startswith("__gpu_done__:"):
                ev = self.gpu_done.pop(jid[len("__gpu_done__:"):], None)
                if ev is not None and self.loop is not None:
                    self.loop.call_soon_threadsafe(ev.set)
                continue
            if jid == "__regrouped__" and result is not None:
                self.group = dict(result)
            fut = self.pending.pop(jid, None)
            if fut is not None and self.loop is not None:
                self.loop.call_soon_threadsafe(_resolve, fut, (result, err))

    def _restart(self):
        try:
            self.proc.kill()
        except Exception:
            pass
        self.proc.join(timeout=10)
        # a live process group cannot re-admit a rank: the fresh child starts
        # rank-local and joins the next generation when the supervisor regroups
        self.env["WORLD_SIZE"] = "1"
        self.restarts += 1
        # everything in flight dies with the child: control messages AND jobs
        # (a job sent during a regroup that then timed out would otherwise wait
        # out job_timeout_s on a fresh child that never saw it)
        for jid, fut in list(self.pending.items()):
            self.pending.pop(jid, None)
            if self.loop is not None:
                self.loop.call_soon_threadsafe(_resolve, fut, (None, "GPU worker restarted"))
        self._start()

    def kill(self):
        """Kill the child (its pending run() notices within 2 s and restarts it)."""
        try:
            self.proc.kill()
        except Exception:
            pass

    async def _control(self, key: str, reply: str, msg: dict, timeout_s: float):
        """Send a control message and await its reply, watching the child: a
        child that dies or outlives ``timeout_s`` is restarted and the call
        raises (a plain wait would block forever on a dead child)."""
        self.loop = asyncio.get_running_loop()
        fut = self.loop.create_future()
        self.pending[reply] = fut
        self.inbox.put(msg)
        t0 = time.monotonic()
        while True:
            done, _ = await asyncio.wait({fut}, timeout=1.0)
            if done:
                result, err = fut.result()
                if err:
                    raise RuntimeError(f"{self.name} {key} failed: {err}")
                return result
            if not self.proc.is_alive() or time.monotonic() - t0 > timeout_s:
                why = "died" if not self.proc.is_alive() else "timed out"
                self.pending.pop(reply, None)
                self._restart()
                raise RuntimeError(f"{self.name} {why} during {key}")

    async def preload(self, names, timeout_s: float = 3600.0, collective: bool = True):
        """Model preload (collective: every executor of the group, same list)."""
        return await self._control("preload", "__preloaded__",
                                   {"__preload__": list(names), "collective": collective}, timeout_s)

    async def regroup(self, spec: dict, timeout_s: float = 300.0):
        """Leave the current process group and join generation ``spec``."""
        self.env.update({"RANK": str(spec["rank"]), "WORLD_SIZE": str(spec["world"]),
                         "SDAAS_GROUP_GEN": str(spec["gen"]), "SDAAS_STORE_PORT": str(spec["store_port"])})
        res = await self._control("regroup", "__regrouped__", {"__regroup__": dict(spec)}, timeout_s)
        self.group = dict(res or {})
        return self.group

    async def run(self, job, gpu_done: asyncio.Event | None = None):
        """Run one job; ``gpu_done`` (optional) is set as soon as the child's
        device part has finished (its envelope may still be encoding)."""
        from .generator import _error_result

        self.loop = asyncio.get_running_loop()
        fut = self.loop.create_future()
        jid = job.get("id")
        self.pending[jid] = fut
        if gpu_done is not None:
            self.gpu_done[jid] = gpu_done
        self.inbox.put(job)
        t0 = time.monotonic()
        while True:
            done, _ = await asyncio.wait({fut}, timeout=2.0)
            if done:
                self.gpu_done.pop(jid, None)
                if gpu_done is not None:
                    gpu_done.set()
                result, err = fut.result()
                if result is not None:
                    return result
                return _error_result(jid, RuntimeError(f"worker error: {err}"), job.get("content_type", "image/jpeg"),
                                     False)
            if not self.proc.is_alive() or time.monotonic() - t0 > self.job_timeout_s:
                why = "crashed" if not self.proc.is_alive() else "timed out"
                logging.error(f"{self.name} {why} on job {jid}; restarting")
                self.pending.pop(jid, None)
                self.gpu_done.pop(jid, None)
                if gpu_done is not None:
                    gpu_done.set()
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
    from ..jobs.router import GUIDED_PIPELINES

    if p.get("pipeline_type") in GUIDED_PIPELINES:
        return None  # their own sampling loops (pipelines/guided.py): never batched or split
    return (job.get("model_name"), job.get("height"), job.get("width"), job.get("num_inference_steps"),
            job.get("guidance_scale"), p.get("scheduler_type"), p.get("pipeline_type"), job.get("content_type"),
            job.get("revision"), job.get("eta"))


def splittable(job) -> int:
    """Number of images of a job that may be split across GPUs (0: not splittable)."""
    if _raw_key(job) is None or not str(job.get("content_type", "image/jpeg")).startswith("image/"):
        return 0
    n = int(job.get("num_images_per_prompt", 1) or 1)
    return n if n >= 2 else 0


def cfg_splittable(job) -> bool:
    """A one-image CFG txt2img job whose two CFG halves may run on two idle
    GPUs (CFG-parallel, SURVEY §2.6: lower latency for the common batch-1 job)."""
    if _raw_key(job) is None or not str(job.get("content_type", "image/jpeg")).startswith("image/"):
        return False
    if int(job.get("num_images_per_prompt", 1) or 1) != 1:
        return False
    p = job.get("parameters") or {}
    if "pix2pix" in str(p.get("pipeline_type", "")).lower():
        return False
    return float(job.get("guidance_scale", 7.5) or 0.0) > 1.0


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


def _group_str(g: dict) -> str:
    if g.get("error"):
        return f"no group ({g['error']})"
    if "rank" in g:
        return f"{g.get('backend', '?')} rank {g['rank']}/{g['world']} gen {g.get('gen', 0)}"
    return "single"


class GroupStore:
    """The node process group's rendezvous: a TCPStore hosted by the
    supervisor (is_master), with generations — each (re)formed group uses its
    own key prefix, so a regroup never reads a dead generation's keys."""

    def __init__(self, host: str = "127.0.0.1"):
        import datetime

        import torch.distributed as dist

        self.host = host
        self.store = dist.TCPStore(host, 0, is_master=True, wait_for_workers=False,
                                   timeout=datetime.timedelta(seconds=600))
        self.port = self.store.port
        self.gen = 0

    def next_gen(self) -> int:
        self.gen += 1
        return self.gen


_STORES: list = []  # keep every hosted store alive for the life of the process


class Supervisor:
    def __init__(self, settings=None, executors=None, hive=None):
        self.settings = settings or load_settings()
        self.hive = hive or HiveClient(self.settings)
        self.executors = executors if executors is not None else self._default_executors()
        self.store = next((s for s in _STORES if any(getattr(e, "env", {}).get("SDAAS_STORE_PORT") == str(s.port)
                                                       for e in self.executors)), None)
        self._last_regroup = 0.0
        self._regroup_task = None  # a background regroup (never awaited by the poll loop)
        self.regroups = 0
        n = max(1, len(self.executors))
        # batching: each device may hold up to max_batch queued jobs (max_batch <= 1:
        # the reference's queue depth of one job per device)
        self.batch_jobs = max(1, int(getattr(self.settings, "max_batch", 1) or 1))
        self.work_queue: asyncio.Queue = asyncio.Queue(maxsize=n * self.batch_jobs)
        self.result_queue: asyncio.Queue = asyncio.Queue()
        self.busy = 0
        self.results_submitted = 0
        self.splits = 0
        self.cfg_splits = 0  # one-image jobs run CFG-parallel on two GPUs
        self.stop = asyncio.Event()
        self.locks = {id(ex): asyncio.Lock() for ex in self.executors}
        # executors whose device_worker is parked on the work queue: only these
        # may be claimed as split helpers (their lock has no waiter, so taking it
        # never suspends; ADVICE r2: probing lk.locked() alone could stall)
        self.idle: set = set()

    def _default_executors(self):
        gpus = visible_gpus(self.settings)
        if not gpus:
            return [ThreadExecutor("cpu")]
        # (re)build the kernel library HERE, before any child initialises HIP:
        # GPU children only check it (ops/_lib.py::check_fresh) and never run hipcc
        from ..ops._lib import ensure_built

        ensure_built()
        return [ProcessExecutor(g, env=e) for g, e in zip(gpus, group_envs(len(gpus), self.settings))]

    # ------------------------------------------------------------------ process group
    def group_ok(self) -> bool:
        """Every executor reports the SAME live group generation with distinct
        ranks 0..N-1: only then are collectives / point-to-point sends issued
        (a half-formed group would leave the joined ranks waiting forever)."""
        gs = [getattr(e, "group", None) or {} for e in self.executors]
        if len(self.executors) < 2 or not all("rank" in g for g in gs):
            return False
        gens = {g.get("gen") for g in gs}
        return len(gens) == 1 and sorted(g["rank"] for g in gs) == list(range(len(gs))) and \
            all(g["world"] == len(gs) for g in gs)

    async def regroup(self, timeout_s: float = 300.0) -> bool:
        """Re-form the process group as a new store generation (after a child
        restart left it degraded).  Call only while every executor is idle."""
        if self.store is None or len(self.executors) < 2:
            return False
        gen = self.store.next_gen()
        self._last_regroup = time.monotonic()
        self.regroups += 1
        specs = [{"gen": gen, "rank": i, "world": len(self.executors), "store_port": self.store.port}
                 for i in range(len(self.executors))]
        res = await asyncio.gather(*(e.regroup(sp, timeout_s) for e, sp in zip(self.executors, specs)),
                                   return_exceptions=True)
        ok = self.group_ok()
        if not ok:
            logging.error(f"regroup to generation {gen} failed: {res}")
        return ok

    async def _maybe_regroup(self):
        """Start a regroup in the background when the group is degraded and the
        node idle: the hive poll loop never waits on it (a wedged child would
        otherwise stall polling for the whole per-executor control timeout)."""
        if self._regroup_task is not None and not self._regroup_task.done():
            return
        if (self.store is not None and not self.group_ok() and self.busy == 0 and self.work_queue.empty()
                and all(hasattr(e, "regroup") for e in self.executors) and len(self.executors) > 1
                and time.monotonic() - self._last_regroup > float(os.environ.get("SDAAS_REGROUP_S", "60"))):
            self._regroup_task = asyncio.ensure_future(
                self.regroup(timeout_s=float(os.environ.get("SDAAS_REGROUP_TIMEOUT_S", "60"))))

    # ------------------------------------------------------------------ split jobs
    async def _claim_helpers(self, job, ex) -> list:
        """Idle executors for a split, claimed synchronously: an executor in
        ``self.idle`` has no waiter on its lock, so ``acquire`` returns at once."""
        if len(self.executors) < 2:
            return []
        n = splittable(job)
        if n >= 2 and not getattr(self.settings, "split_jobs", True):
            return []
        if n < 2:  # one image: its two CFG halves on two GPUs (needs the process group)
            if not (getattr(self.settings, "cfg_parallel", True) and cfg_splittable(job) and self.group_ok()
                    and hasattr(ex, "kill")):
                return []
            n = 2
        helpers = []
        for other in self.executors:
            if len(helpers) + 1 >= n:
                break
            lk = self.locks[id(other)]
            if other is not ex and other in self.idle and not lk.locked():
                self.idle.discard(other)
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
        if n < 2:  # claimed for CFG-parallel (_claim_helpers)
            return await self._run_cfg_split(job, exs[:2], seed)
        if self.group_ok() and all(hasattr(e, "kill") for e in exs):
            return await self._run_split_group(job, exs, n, seed)
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

    async def _run_split_group(self, job, exs, n, seed) -> dict:
        """Split over the process group: the leader (exs[0]) renders images
        [0, n0) and receives every helper's uint8 images over RCCL (gloo on
        CPU children), then encodes the one envelope itself.  A part whose child
        dies leaves its peers blocked in a transfer, so the other parts' children
        are killed too (each restarts; the group re-forms when idle)."""
        jid = job.get("id")
        rngs = _ranges(n, len(exs))
        ranks = [e.group["rank"] for e in exs]
        subs = [dict(job, id=jid, seed=seed, num_images_per_prompt=rngs[0][1] - rngs[0][0], _image_range=list(rngs[0]),
                     _split={"role": "leader", "peers": ranks[1:]})]
        for i in range(1, len(exs)):
            lo, hi = rngs[i]
            subs.append(dict(job, id=f"{jid}#{i}", seed=seed, num_images_per_prompt=hi - lo, _image_range=[lo, hi],
                             _split={"role": "helper", "leader": ranks[0]}))
        return await self._await_parts(job, exs, subs, seed)

    async def _run_cfg_split(self, job, exs, seed) -> dict:
        """CFG-parallel: both parts run the whole job with the same seed; part 0
        evaluates the unconditional half of every UNet step, part 1 the
        conditional half, and they swap predictions each step over the process
        group (pipelines.sd._denoise_cfg_split).  Part 0 decodes and answers."""
        jid = job.get("id")
        r0, r1 = (e.group["rank"] for e in exs)
        subs = [dict(job, id=jid, seed=seed, _split={"role": "cfg", "peer": r1, "half": 0}),
                dict(job, id=f"{jid}#cfg", seed=seed, _split={"role": "cfg", "peer": r0, "half": 1})]
        # lockstep: a part that failed mid-loop leaves its peer blocked in the
        # per-step exchange, so the survivor is killed at once (no grace)
        out = await self._await_parts(job, exs, subs, seed, lockstep=True)
        if out.get("artifacts"):
            self.cfg_splits += 1
        return out

    async def _await_parts(self, job, exs, subs, seed, lockstep: bool = False) -> dict:
        """Run the parts of a group split; the first part answers the job, the
        others must return a ``_split_ack``.  ``lockstep``: the parts exchange
        data every step (CFG-parallel), so once one part has failed the others
        can only be waiting on it: they are killed without a grace period."""
        from .generator import _error_result

        jid = job.get("id")
        restarts0 = [e.restarts for e in exs]
        tasks = [asyncio.ensure_future(e.run(sj)) for e, sj in zip(exs, subs)]
        pending = set(tasks)
        failed_at = None  # when a part first returned an error result
        # a part that FAILED released its peers (pipelines.diffusion._split_failed):
        # the others finish their own images and return, so the grace only
        # catches a peer wedged in the transfer — long enough for a healthy
        # leader still rendering (a crashed part is handled at once below)
        grace = float(os.environ.get("SDAAS_SPLIT_GRACE_S", "300"))
        while pending:
            done, pending = await asyncio.wait(pending, timeout=grace if failed_at is not None else None,
                                               return_when=asyncio.FIRST_COMPLETED)
            for t in done:
                i = tasks.index(t)
                cfg = t.result().get("pipeline_config") or {}
                if "error" in cfg or (i > 0 and "_split_ack" not in cfg):
                    failed_at = failed_at if failed_at is not None else time.monotonic()
            crashed = any(e.restarts != r0 for e, r0 in zip(exs, restarts0))
            # a crashed part never sends; a part that failed released its peers
            # (pipelines.diffusion._split_failed), so survivors still pending
            # after the grace period are wedged on the transfer: restart them
            # rather than leave queued sends a later split could match
            if crashed or (failed_at is not None and pending and
                           (lockstep or time.monotonic() - failed_at >= grace)):
                for e, t in zip(exs, tasks):
                    if not t.done():
                        e.kill()
        results = [t.result() for t in tasks]
        lead = results[0]
        helper_ok = all("_split_ack" in (r.get("pipeline_config") or {}) for r in results[1:])
        if lead.get("artifacts") and helper_ok and "error" not in (lead.get("pipeline_config") or {}):
            self.splits += 1
            lead["pipeline_config"]["seed"] = seed
            return lead
        bad = next((r for r in results if "error" in (r.get("pipeline_config") or {})), lead)
        return dict(bad, id=jid) if bad.get("pipeline_config") else \
            _error_result(jid, RuntimeError("split job failed"), job.get("content_type", "image/jpeg"), False)

    async def preload(self, names):
        """Every executor loads the same models: collectively (sharded reads +
        all_gather) while the group is healthy, otherwise each on its own.  A
        child dying mid-collective restarts every group child (the survivors may
        be blocked in the collective) and the preload is abandoned."""
        names = [n for n in names if n]
        exs = [ex for ex in self.executors if hasattr(ex, "preload")]
        if not names or not exs:
            return []
        collective = self.group_ok()
        if not collective and any(getattr(e, "group", {}).get("error") for e in exs):
            logging.warning("process group incomplete: " + "; ".join(getattr(e, "ready_info", "") for e in exs))
        tasks = [asyncio.ensure_future(ex.preload(names, collective=collective)) for ex in exs]
        pending = set(tasks)
        killed = False
        while pending:
            done, pending = await asyncio.wait(pending, return_when=asyncio.FIRST_COMPLETED)
            if collective and not killed and any(t.cancelled() or t.exception() is not None for t in done):
                killed = True
                for ex, t in zip(exs, tasks):  # peers of a dead rank are stuck in the all_gather
                    if not t.done():
                        ex.kill()
        failed = [asyncio.CancelledError("preload cancelled") if t.cancelled() else t.exception() for t in tasks
                  if t.cancelled() or t.exception() is not None]
        if failed:
            raise RuntimeError(f"preload failed on {len(failed)} device(s): {failed[0]}")
        return [t.result() for t in tasks]

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
            self.idle.add(ex)
            try:
                job = await self.work_queue.get()
            finally:
                self.idle.discard(ex)
            rt = self._regroup_task
            if rt is not None and not rt.done():  # no job into a child that is mid-regroup
                try:
                    await asyncio.shield(rt)
                except Exception as e:  # a failed regroup restarted the children; run anyway
                    logging.warning(f"regroup failed before a job: {e}")
            batch = self._drain_compatible(job)
            self.busy += len(batch)
            helpers = []
            deferred = None  # a single job whose envelope is still encoding in the child
            try:
                async with lock:  # a split job may hold this executor as a helper
                    if len(batch) == 1:
                        helpers = await self._claim_helpers(job, ex)
                        if helpers:
                            self.busy += len(helpers)
                            results = [await self._run_split(job, [ex] + helpers)]
                        elif isinstance(ex, ProcessExecutor):
                            # pipelined: the next job goes to the child as soon as this
                            # one's device part is done; its envelope (JPEG / base64 /
                            # sha256, encoder processes) finishes meanwhile
                            ev = asyncio.Event()
                            deferred = asyncio.ensure_future(ex.run(job, gpu_done=ev))
                            waiter = asyncio.ensure_future(ev.wait())
                            await asyncio.wait({deferred, waiter}, return_when=asyncio.FIRST_COMPLETED)
                            waiter.cancel()
                            results = []
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
                if deferred is None:
                    self.busy -= len(batch) + len(helpers)
                    self.work_queue.task_done()
                else:
                    asyncio.ensure_future(self._finish_deferred(deferred, job))

    async def _finish_deferred(self, task, job):
        """Queue the result of a pipelined job once its envelope is ready."""
        from .generator import _error_result

        try:
            try:
                result = await task
            except Exception as e:
                logging.exception(e)
                result = _error_result(job.get("id"), e, job.get("content_type", "image/jpeg"), False)
            await self.result_queue.put(result)
        finally:
            self.busy -= 1
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
                await self._maybe_regroup()
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


def group_envs(n: int, settings=None, store: GroupStore | None = None) -> list:
    """Per-child process-group environment (RANK, WORLD_SIZE and the
    supervisor-hosted store's port / generation); hosts the store if none given."""
    if n <= 1 or (settings is not None and not getattr(settings, "distributed", True)):
        return [{} for _ in range(n)]
    if store is None:
        store = GroupStore()
        _STORES.append(store)
    return [{"RANK": str(i), "WORLD_SIZE": str(n), "SDAAS_STORE_HOST": store.host, "SDAAS_STORE_PORT": str(store.port),
             "SDAAS_GROUP_GEN": str(store.gen), "MASTER_ADDR": store.host, "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
            for i in range(n)]


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
