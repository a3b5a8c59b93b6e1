"""Result encoding off the GPU process's interpreter.

The reference encodes results (grid, JPEG ``optimize+progressive``, thumbnail,
base64, sha256 — swarm/output_processor.py:10-58, :90-136) inline, after the
forward pass, on the same thread that drives the GPU.  At 4 images of 512²
that is ~30 ms of CPU per job.  Here the GPU-driving thread only hands the
uint8 pixels to a small pool of encoder *processes* and immediately starts the
next job; the encoding runs in parallel with the next job's denoising instead
of being serialized in front of it.  (An in-process thread is not enough: the
encoder holds the GIL for long stretches — base64, grid paste, PIL glue — and
delays the next job's host-side launch work by ~30 ms, measured with
tools/phaseprof.py jobs.)

The pool must be created BEFORE the process initialises the GPU: the workers
are started with the ``spawn`` method (fork+exec of a fresh interpreter), and
no process that has touched HIP may exec.  ``EncoderPool`` checks this and
falls back to a thread pool when the GPU is already up.
"""
from __future__ import annotations

import concurrent.futures as cf
import multiprocessing as mp
import os
import sys


class BrokenEncoderPool(RuntimeError):
    """No encoder process is alive to take (or finish) a task."""


def _worker_main(inq, outq, parent=None):
    """Encoder process: run (task id, fn, args) items until a None arrives (or
    the owning process is gone: re-parented after a SIGKILL of the GPU child)."""
    import queue

    while True:
        try:
            item = inq.get(timeout=1.0)
        except queue.Empty:
            if parent is not None and os.getppid() != parent:
                return
            continue
        if item is None:
            return
        tid, fn, args = item
        try:
            outq.put((tid, True, fn(*args)))
        except BaseException as e:  # reported on the task's future
            outq.put((tid, False, e))


class _ProcessPool:
    """A fixed set of spawned encoder processes, all started at construction
    (this process may not spawn once it has initialised the GPU, so nothing is
    ever respawned), each with its own task queue; tasks go round-robin to live
    workers.  A monitor thread fails the pending tasks of a worker that died
    (``BrokenEncoderPool``) and takes it out of rotation.  Only public
    multiprocessing / concurrent.futures APIs are used."""

    def __init__(self, n: int, ctx):
        import threading

        self.outq = ctx.Queue()
        self.workers = []  # [process, task queue, pending task ids]
        for _ in range(n):
            inq = ctx.Queue()
            proc = ctx.Process(target=_worker_main, args=(inq, self.outq, os.getpid()), daemon=True)
            proc.start()
            self.workers.append([proc, inq, set()])
        self.futs: dict = {}
        self.lock = threading.Lock()
        self.next_id = 0
        self.rr = 0
        self.closed = False
        self.reader = threading.Thread(target=self._read, daemon=True)
        self.reader.start()
        self.monitor = threading.Thread(target=self._watch, daemon=True)
        self.monitor.start()

    def pids(self) -> list:
        return [w[0].pid for w in self.workers]

    def alive(self) -> int:
        return sum(1 for w in self.workers if w[0].is_alive())

    def submit(self, fn, *args) -> cf.Future:
        fut: cf.Future = cf.Future()
        with self.lock:
            live = [i for i, w in enumerate(self.workers) if w[0].is_alive()]
            if self.closed or not live:
                raise BrokenEncoderPool("no live encoder process")
            wi = live[self.rr % len(live)]
            self.rr += 1
            tid = self.next_id
            self.next_id += 1
            self.futs[tid] = (fut, wi)
            self.workers[wi][2].add(tid)
            self.workers[wi][1].put((tid, fn, args))
        return fut

    def _read(self):
        while True:
            try:
                item = self.outq.get()
            except Exception:  # noqa: BLE001 - queue torn down (EOF / OSError, or interpreter exit)
                return
            if item is None:
                return
            tid, ok, value = item
            with self.lock:
                fut, wi = self.futs.pop(tid, (None, None))
                if wi is not None:
                    self.workers[wi][2].discard(tid)
            if fut is not None and not fut.done():
                (fut.set_result if ok else fut.set_exception)(value)

    def _watch(self):
        import time

        while not self.closed:
            time.sleep(0.25)
            with self.lock:
                dead = [(wi, w) for wi, w in enumerate(self.workers) if not w[0].is_alive() and w[2]]
                lost = []
                for wi, w in dead:
                    for tid in list(w[2]):
                        fut, _ = self.futs.pop(tid, (None, None))
                        if fut is not None:
                            lost.append(fut)
                    w[2].clear()
            for fut in lost:
                if not fut.done():
                    fut.set_exception(BrokenEncoderPool("the encoder process running this task died"))

    def shutdown(self, wait: bool = True):
        self.closed = True
        for proc, inq, _ in self.workers:
            if proc.is_alive():
                inq.put(None)
        if wait:
            for proc, _, _ in self.workers:
                proc.join(timeout=30)
        self.outq.put(None)
        if wait:  # let the reader drain and return before interpreter teardown
            self.reader.join(timeout=5)


def encode_arrays(arrays, content_type: str = "image/jpeg", output_list=("primary",)) -> dict:
    """uint8 HWC arrays -> the result envelope's artifacts dict (runs in a worker)."""
    from PIL import Image

    from .processor import OutputProcessor

    op = OutputProcessor(list(output_list), content_type)
    op.add_outputs([Image.fromarray(a) for a in arrays])
    return op.get_results()


def encode_artifact(arrays, content_type: str = "image/jpeg") -> dict:
    """uint8 HWC arrays -> ONE artifact (grid, encode, thumbnail, base64, sha256)."""
    from PIL import Image

    from .processor import image_to_buffer, make_result, post_process

    img = post_process([Image.fromarray(a) for a in arrays])
    return make_result(image_to_buffer(img, content_type), img, content_type)


def _gpu_initialised() -> bool:
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return False


class EncoderPool:
    """``submit(arrays, content_type) -> Future[dict]``.

    processes: worker processes (0 -> threads; default ``$CSK_ENCODER_PROCS`` or 2).
    """

    def __init__(self, processes: int | None = None):
        if processes is None:
            processes = int(os.environ.get("CSK_ENCODER_PROCS", "2"))
        self.kind = "thread"
        self._pool: cf.Executor | _ProcessPool
        if processes > 0 and not _gpu_initialised():
            try:
                # every worker starts now, while this process has not touched the GPU
                self._pool = _ProcessPool(processes, mp.get_context("spawn"))
                self.kind = "process"
                return
            except Exception:
                pass
        self._pool = cf.ThreadPoolExecutor(max_workers=max(1, processes or 2))

    def pids(self) -> list:
        return self._pool.pids() if isinstance(self._pool, _ProcessPool) else []

    def _submit(self, fn, *args) -> cf.Future:
        try:
            return self._pool.submit(fn, *args)
        except BrokenEncoderPool:
            # every worker died (OOM kill, crash) and this process may not spawn
            # replacements once the GPU is up: degrade to encoder threads instead
            # of failing every job
            self._pool.shutdown(wait=False)
            self._pool = cf.ThreadPoolExecutor(max_workers=2)
            self.kind = "thread"
            return self._pool.submit(fn, *args)

    def submit(self, arrays, content_type: str = "image/jpeg", output_list=("primary",)) -> cf.Future:
        return self._submit(encode_arrays, list(arrays), content_type, tuple(output_list))

    def submit_artifact(self, arrays, content_type: str = "image/jpeg") -> cf.Future:
        return self._submit(encode_artifact, list(arrays), content_type)

    def shutdown(self):
        self._pool.shutdown(wait=True)
