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


def _noop(_=None) -> int:
    import time

    time.sleep(0.05)  # keep each worker busy so every submit below starts a new one
    return os.getpid()


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
        self._pool: cf.Executor
        if processes > 0 and not _gpu_initialised():
            try:
                self._pool = cf.ProcessPoolExecutor(max_workers=processes, mp_context=mp.get_context("spawn"))
                # start every worker now, while this process has not touched the GPU
                # (the executor only spawns on submit; a later spawn would exec from
                # a GPU process)
                list(self._pool.map(_noop, range(processes)))
                procs = getattr(self._pool, "_processes", None)
                while procs is not None and len(procs) < processes and hasattr(self._pool, "_spawn_process"):
                    self._pool._spawn_process()
                self.kind = "process"
                return
            except Exception:
                pass
        self._pool = cf.ThreadPoolExecutor(max_workers=max(1, processes or 2))

    def _submit(self, fn, *args) -> cf.Future:
        try:
            return self._pool.submit(fn, *args)
        except cf.process.BrokenProcessPool:
            # a worker died (OOM kill, crash): the process pool refuses all further
            # work and this process may not spawn replacements once the GPU is up,
            # so the pool degrades to encoder threads instead of failing every job
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
