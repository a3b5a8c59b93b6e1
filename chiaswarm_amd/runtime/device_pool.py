"""Thread-safe pool of idle devices (reference: swarm/gpu/device_pool.py:1-34,
dead code there; here the supervisor can use it to lend a GPU to a one-off
task such as a model warm-up).  Acquisition has a timeout instead of the
reference's unchecked ``mutex.acquire(True, 1)`` return value."""
from __future__ import annotations

import threading

from .device import Device

_lock = threading.Lock()
available: list[Device] = []


def get_available_gpu_count() -> int:
    with _lock:
        return len(available)


def add_device_to_pool(device: Device) -> None:
    with _lock:
        available.append(device)


def remove_device_from_pool() -> Device:
    with _lock:
        if available:
            return available.pop(0)
    raise RuntimeError("busy")
