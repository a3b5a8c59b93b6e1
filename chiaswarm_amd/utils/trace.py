"""roctx ranges around the phases of a job (SURVEY §5.1 "roctx ranges around
UNet, VAE and text-encoder calls").

Enabled with ``CSK_ROCTX=1``; then ``rocprofv3 --marker-trace --kernel-trace``
shows every job's text-encode / denoise / decode / encode ranges above its
kernels.  Disabled (the default) a range is a no-op context manager: nothing
is loaded and nothing is called on the hot path.  Ranges are host-side markers:
inside a hipGraph replay they bracket the replay call, not individual kernels.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_LIB = None
_ENABLED = os.environ.get("CSK_ROCTX") == "1"


def _lib():
    global _LIB, _ENABLED
    if _LIB is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4", "libroctx64.so"):
            for d in ("", "/opt/rocm/lib/"):
                try:
                    lib = ctypes.CDLL(d + name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                    _LIB = lib
                    return _LIB
                except OSError:
                    continue
        _ENABLED = False
    return _LIB


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED or _lib() is None:
        yield
        return
    _LIB.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        _LIB.roctxRangePop()


def mark(name: str) -> None:
    if _ENABLED and _lib() is not None:
        _LIB.roctxMarkA(name.encode())
