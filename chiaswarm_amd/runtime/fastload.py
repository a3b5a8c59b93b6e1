"""Fast safetensors reads through the native reader (``csrc/host/csk_io.cpp``,
built into ``chiaswarm_amd/lib/libcskio.so``).

The reference loads every model with ``from_pretrained`` in every job
(swarm/diffusion/diffusion_func.py:41-46).  Here a model is read once per
worker process, so the read itself is the cold-start cost of every model-cache
miss and every worker start.  A safetensors file is one JSON header followed by
one contiguous data region, so the whole region is moved in ONE native call —
threaded ``pread`` from the page cache into a pinned staging ring and
``hipMemcpyAsync`` to one device buffer — and every tensor is a zero-copy view
of that buffer (``safetensors.torch.load_file`` instead does one pageable
host tensor per entry and a per-tensor H2D copy in ``load_into``).

``read_range`` is the primitive the sharded loader (parallel/sharded.py) uses
for each rank's 1/N byte range.  Without the native library (not built) the
same byte ranges are read with Python ``readinto`` — same results, slower.
"""
from __future__ import annotations

import ctypes
import json
import os
import struct
import threading
import time

import torch

_DT = {"F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
       "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
       "BOOL": torch.bool}

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libcskio.so")
_LIB = None
_LOCK = threading.Lock()
THREADS = int(os.environ.get("CSK_IO_THREADS", "8"))

# per-process totals (bench / logs): bytes, wall seconds inside the reader
STATS = {"bytes": 0, "seconds": 0.0, "calls": 0}


def lib():
    """The native reader, or None when it is not built (pure-Python fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB or None
    with _LOCK:
        if _LIB is None:
            if os.environ.get("CSK_IO_NATIVE", "1") == "0" or not os.path.exists(LIB_PATH):
                _LIB = False
            else:
                lb = ctypes.CDLL(LIB_PATH)
                lb.csk_io_read.argtypes = [ctypes.c_char_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.POINTER(ctypes.c_double)]
                lb.csk_io_read.restype = ctypes.c_int
                lb.csk_io_release.restype = ctypes.c_int
                _LIB = lb
    return _LIB or None


def read_header(path: str) -> tuple[int, dict]:
    """(data start offset, {name: (dtype, shape, (begin, end))}) of a safetensors file."""
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        hdr = json.loads(f.read(n))
    hdr.pop("__metadata__", None)
    return 8 + n, {k: (v["dtype"], tuple(v["shape"]), tuple(v["data_offsets"])) for k, v in hdr.items()}


def read_metadata(path: str) -> dict:
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        return json.loads(f.read(n)).get("__metadata__", {}) or {}


def read_range(path: str, offset: int, out: torch.Tensor) -> None:
    """Fill the contiguous uint8 tensor ``out`` (host or device) with
    ``out.numel()`` bytes of ``path`` starting at ``offset``."""
    assert out.dtype == torch.uint8 and out.is_contiguous()
    n = out.numel()
    if n == 0:
        return
    t0 = time.perf_counter()
    lb = lib()
    on_dev = out.device.type == "cuda"
    if lb is not None:
        stats = (ctypes.c_double * 3)()
        stream = torch.cuda.current_stream(out.device).cuda_stream if on_dev else None
        rc = lb.csk_io_read(os.fsencode(path), int(offset), int(n), ctypes.c_void_p(out.data_ptr()), int(on_dev),
                            THREADS, ctypes.c_void_p(stream) if stream else None, stats)
        if rc < 0:
            raise OSError(-rc, f"csk_io_read({path}, {offset}, {n}): {os.strerror(-rc)}")
        if rc > 0:
            raise RuntimeError(f"csk_io_read({path}): hipError {rc}")
    else:
        host = out if not on_dev else torch.empty(n, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        mv = memoryview(host.numpy()).cast("B")
        with open(path, "rb") as f:
            f.seek(offset)
            got = f.readinto(mv)
        if got != n:
            raise OSError(f"{path}: short read {got} < {n} at {offset}")
        if on_dev:
            out.copy_(host, non_blocking=False)
    STATS["bytes"] += n
    STATS["seconds"] += time.perf_counter() - t0
    STATS["calls"] += 1


def views(buf: torch.Tensor, hdr: dict, base: int = 0) -> dict:
    """{name: tensor} views into the uint8 buffer holding a data region
    (``base``: the region's offset inside ``buf``).  A tensor whose byte offset
    is not a multiple of its element size is copied out (never for files
    written by the safetensors library, which aligns the region)."""
    out = {}
    for name, (dt, shape, (b, e)) in hdr.items():
        tdt = _DT[dt]
        raw = buf[base + b:base + e]
        esz = torch.empty(0, dtype=tdt).element_size()
        if (raw.storage_offset() % esz) != 0:
            raw = raw.clone()
        out[name] = raw.view(tdt).view(shape) if e > b else torch.empty(shape, dtype=tdt, device=buf.device)
    return out


def load_file(path: str, device="cpu") -> dict:
    """Drop-in for ``safetensors.torch.load_file``: the whole data region in one
    native read onto ``device``, tensors as views of it (bitwise identical)."""
    start, hdr = read_header(path)
    size = os.path.getsize(path) - start
    buf = torch.empty(size, dtype=torch.uint8, device=device)
    read_range(path, start, buf)
    return views(buf, hdr)
