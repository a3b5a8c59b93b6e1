"""Loader for the in-tree HIP kernel library (``chiaswarm_amd/lib/libcsk.so``).

The kernels live in ``csrc/kernels/*.hip`` and are compiled for gfx950 by
``chiaswarm_amd/_build.py`` (``hipcc --offload-arch=gfx950 -shared``).  Every
launcher is an ``extern "C"`` function taking raw device pointers, sizes and a
``hipStream_t``; we call them through ctypes with torch's *current* stream so
they are captured by ``torch.cuda.CUDAGraph`` (= hipGraph on ROCm) like any
other kernel.

Policy (see README "no silent fallback"): on a GPU box the library MUST load;
if it does not, every GPU op raises.  The torch reference implementations in
``ops/*`` are used only for CPU tensors (plumbing tests, BASELINE config #1) or
when a caller explicitly selects ``reference`` mode for A/B numerics.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_LIB = None
_LOCK = threading.Lock()
_LOAD_ERR: Exception | None = None

LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib")
# CSK_LIB_PATH: load another build (same-box A/B of two builds: tools/gpu/lib_ab.sh; set
# CSK_ALLOW_STALE=1 with it, the staleness stamp belongs to the in-tree build).
# CSK_DEBUG=1: the bounds-checking build (python -m chiaswarm_amd._build --debug)
DEBUG = os.environ.get("CSK_DEBUG", "") not in ("", "0")
LIB_PATH = os.environ.get("CSK_LIB_PATH") or os.path.join(LIB_DIR, "libcsk_debug.so" if DEBUG else "libcsk.so")
# translation units that export csk_debug_read_<tu> / csk_debug_clear_<tu> in debug builds
DEBUG_TUS = ("gemm", "gemm_glds", "gemm8p", "attention", "attention_wide", "xattn")

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_float = ctypes.c_float
c_int64 = ctypes.c_int64

# name -> argtypes.  Every launcher returns int (hipError_t).
_SIGS: dict[str, list] = {}


def sig(name: str, *argtypes):
    _SIGS[name] = list(argtypes)


class StaleLibraryError(RuntimeError):
    pass


def check_fresh():
    """Raise if libcsk.so was built from other kernel sources than the ones in
    this tree (a stale launcher signature would be called with the wrong
    arguments).  Content digest, not mtimes (a copied tree reorders mtimes).

    Never rebuilds here: this runs inside GPU worker processes that have
    already initialised HIP, where fork+exec of hipcc is unsafe and N
    children would race on the same output files.  Build at install time or
    in the supervisor before any GPU work (``ensure_built``)."""
    src_dir = os.path.normpath(os.path.join(os.path.dirname(LIB_DIR), "..", "csrc", "kernels"))
    if not os.path.isdir(src_dir) or os.environ.get("CSK_ALLOW_STALE"):
        return
    from .. import _build

    want = _build.source_digest(DEBUG)
    try:
        with open(LIB_PATH + ".src") as f:
            have = f.read().strip()
    except OSError:
        have = None
    if have != want:
        raise StaleLibraryError(
            f"{LIB_PATH} is stale or unstamped (built from {have}, sources are {want}): "
            "run `python -m chiaswarm_amd._build` before starting GPU work")


def ensure_built():
    """Build the library if it is missing or stale.  Only for processes that
    have NOT initialised the GPU (the supervisor, install scripts, tests)."""
    try:
        if os.path.exists(LIB_PATH):
            check_fresh()
            return
    except StaleLibraryError:
        pass
    from .. import _build

    _build.build(verbose=False, debug=DEBUG)


def load():
    """Load libcsk.so (idempotent).  Raises if it is missing or broken."""
    global _LIB, _LOAD_ERR
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        if not os.path.exists(LIB_PATH):
            _LOAD_ERR = FileNotFoundError(
                f"{LIB_PATH} not built: run `python -m chiaswarm_amd._build`"
            )
            raise _LOAD_ERR
        check_fresh()
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, args in _SIGS.items():
            if os.environ.get("CSK_LIB_PATH") and os.environ.get("CSK_ALLOW_STALE") and not hasattr(lib, name):
                continue  # same-box A/B against an older build: entry points it lacks fail when called
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
        if hasattr(lib, "csk_init"):
            lib.csk_init.restype = c_int
            err = lib.csk_init()  # zero page for LDS-DMA padding (allocated outside any graph capture)
            if err != 0:
                raise RuntimeError(f"csk_init failed with hipError {err}")
        _LIB = lib
        return lib


def debug_records(clear: bool = True) -> list:
    """Bounds violations recorded by a CSK_DEBUG build since the last clear:
    [(tu, count, site, block_x, thread, value, limit, block_y)].  Call after a
    synchronise.  Empty for release builds (no records are compiled in)."""
    lib = load()
    out = []
    for tu in DEBUG_TUS:
        rd = getattr(lib, f"csk_debug_read_{tu}", None)
        if rd is None:
            continue
        buf = (ctypes.c_uint * 8)()
        rd.argtypes = [c_void_p]
        rd.restype = c_int
        if rd(ctypes.cast(buf, c_void_p)) != 0:
            raise RuntimeError(f"csk_debug_read_{tu} failed")
        if buf[0]:
            val = buf[4] | (buf[5] << 32)
            if val >= 1 << 63:
                val -= 1 << 64
            out.append((tu, buf[0], buf[1], buf[2], buf[3], val, buf[6], buf[7]))
            if clear:
                getattr(lib, f"csk_debug_clear_{tu}")()
    return out


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


_BOUND: dict = {}


def call(name: str, *args):
    fn = _BOUND.get(name)
    if fn is None:
        lib = load()
        fn = getattr(lib, name)
        fn.argtypes = _SIGS[name]
        fn.restype = c_int
        _BOUND[name] = fn
    err = fn(*args)
    if err != 0:
        raise RuntimeError(f"HIP kernel launcher {name} failed with hipError {err}")


def call_int(name: str, *args) -> int:
    """A library query that returns a value (not a hipError_t), e.g. a support check."""
    fn = _BOUND.get(name)
    if fn is None:
        lib = load()
        fn = getattr(lib, name)
        fn.argtypes = _SIGS[name]
        fn.restype = c_int
        _BOUND[name] = fn
    return int(fn(*args))


def ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()
