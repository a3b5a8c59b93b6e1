"""Per-GPU device wrapper (reference: swarm/gpu/device.py:6-50).

Semantics kept: >= 8 GB admission check, non-blocking mutex ("busy" if
re-entered), seed = job seed or a fresh random one, a seeded torch.Generator on
the device injected as ``generator``, and ``pipeline_config["seed"]`` echoed.
``idenitifier`` (sic) is kept as an alias of ``identifier`` for drop-in
compatibility.  A ``cpu`` device is supported for plumbing tests (BASELINE
config #1).
"""
from __future__ import annotations

import logging
import random
from threading import Lock

MIN_BYTES = 8_000_000_000


class Device:
    def __init__(self, device_id: int | str = 0) -> None:
        import torch

        self.is_cpu = device_id == "cpu" or not torch.cuda.is_available()
        self.device_id = 0 if self.is_cpu else int(device_id)
        if not self.is_cpu:
            total = torch.cuda.get_device_properties(self.device_id).total_memory
            if total < MIN_BYTES:
                raise Exception(f"Not enough memory on device {self.device_id}. At least 8GB VRAM is required")
        self.mutex = Lock()

    def descriptor(self) -> str:
        return f"{self.identifier()}:{self.name()}"

    def identifier(self) -> str:
        return "cpu" if self.is_cpu else f"cuda:{self.device_id}"

    idenitifier = identifier  # reference spelling

    def name(self) -> str:
        if self.is_cpu:
            return "cpu"
        import torch

        return torch.cuda.get_device_name(self.device_id)

    def __call__(self, func, **kwargs):
        import torch

        if not self.mutex.acquire(False):
            logging.error(f"Device {self.device_id} is busy but got invoked.")
            raise Exception("busy")
        try:
            logging.debug(f"Using device# {self.descriptor()}")
            model_name = kwargs.pop("model_name")
            seed = kwargs.pop("seed", None)
            if seed is None:
                seed = random.SystemRandom().randrange(0, 2 ** 63 - 1)
            seed = int(seed)
            kwargs["generator"] = torch.Generator(device=self.identifier()).manual_seed(seed)
            artifacts, pipeline_config = func(self.identifier(), model_name, **kwargs)
            self._health_check()
            pipeline_config["seed"] = seed
            return artifacts, pipeline_config
        finally:
            self.mutex.release()

    def _health_check(self):
        """Fail the job (non-fatal: the hive reissues it) when a kernel's
        in-launch hand-off protocol reported a timeout during it (the
        persistent attention's merge, csrc/kernels/attn_fa.hip): the kernel is
        off for this process from now on and every resident model — whose
        captured graphs still launch it — is dropped."""
        if self.is_cpu:
            return
        from ..ops import _lib

        if _lib._LIB is None:  # the HIP library never ran in this process
            return
        from ..ops import hip_ops

        if not hip_ops.attn_fa_health():
            from .model_cache import cache

            cache().clear()
            raise RuntimeError("persistent attention merge timed out on this GPU; the kernel is disabled for this "
                               "process and the job must be retried")

    def run_batch(self, func, kwargs_list):
        """Batched variant (runtime.batcher): every job gets its own seeded
        generator; ``func(identifier, kwargs_list) -> [(artifacts, config)]``."""
        import torch

        if not self.mutex.acquire(False):
            raise Exception("busy")
        try:
            jobs, seeds = [], []
            for kw in kwargs_list:
                kw = dict(kw)
                seed = kw.pop("seed", None)
                if seed is None:
                    seed = random.SystemRandom().randrange(0, 2 ** 63 - 1)
                seed = int(seed)
                seeds.append(seed)
                kw["generator"] = torch.Generator(device=self.identifier()).manual_seed(seed)
                jobs.append(kw)
            outs = func(self.identifier(), jobs)
            self._health_check()
            for (_, cfg), seed in zip(outs, seeds):
                cfg["seed"] = seed
            return outs
        finally:
            self.mutex.release()
