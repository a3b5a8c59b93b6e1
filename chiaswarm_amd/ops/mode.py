"""Execution-mode switch for the op layer.

* ``hip``       (default): CUDA tensors go to the hand-written gfx950 kernels in
                 libcsk.so; a missing library/kernel is a hard error.
* ``reference``: every op runs its plain-PyTorch definition.  Used by the
                 numerics tests (HIP vs torch fp32 reference of the same op) and
                 by ``bench.py --impl reference`` to measure the
                 "reference-on-MI355X" comparison point (diffusers-style eager
                 PyTorch: MIOpen convs, hipBLASLt GEMMs, SDPA).

CPU tensors always take the reference path (BASELINE config #1: CPU fp32
plumbing run).
"""
from __future__ import annotations

import contextlib
import os
import threading

_state = threading.local()
_DEFAULT = os.environ.get("CSWARM_OPS", "hip")


def get_mode() -> str:
    return getattr(_state, "mode", _DEFAULT)


def set_mode(mode: str) -> None:
    assert mode in ("hip", "reference"), mode
    _state.mode = mode


@contextlib.contextmanager
def ops_mode(mode: str):
    old = get_mode()
    set_mode(mode)
    try:
        yield
    finally:
        set_mode(old)


def use_hip(t) -> bool:
    return t.is_cuda and get_mode() == "hip"
