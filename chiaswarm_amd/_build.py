"""Build the in-tree HIP kernel library for gfx950.

    python -m chiaswarm_amd._build [--force] [-j N] [--debug]

Compiles every ``csrc/kernels/*.hip`` with ``hipcc --offload-arch=gfx950 -O3``
into objects under ``build/`` (content-hash cached) and links them into
``chiaswarm_amd/lib/libcsk.so``.  No torch headers are involved, so a full
rebuild takes seconds; the library is loaded with ctypes (``ops/_lib.py``).

``--debug`` builds ``libcsk_debug.so`` with ``-DCSK_DEBUG=1``: device-side
bounds checks on every LDS-DMA source / destination and the attention K/V
ring indices, recorded per translation unit (``csrc/kernels/common.h``) and
read back by ``ops/_lib.debug_records``; ``CSK_DEBUG=1`` makes the loader
pick that library.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "kernels")
BUILD = os.path.join(ROOT, "build", "csk")
OUT = os.path.join(ROOT, "chiaswarm_amd", "lib", "libcsk.so")
OUT_DEBUG = os.path.join(ROOT, "chiaswarm_amd", "lib", "libcsk_debug.so")
ARCH = os.environ.get("CSK_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wno-unused-result"]
DEBUG_FLAGS = ["-DCSK_DEBUG=1"]


def flags(debug: bool = False) -> list:
    return FLAGS + (DEBUG_FLAGS if debug else [])


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _digest(path: str, extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    with open(path, "rb") as f:
        h.update(f.read())
    for hdr in sorted(glob.glob(os.path.join(SRC, "*.h"))):
        with open(hdr, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def source_digest(debug: bool = False) -> str:
    """Digest of every kernel source + header + the compile flags: the identity
    of the library they build (stored next to it as ``libcsk.so.src``)."""
    h = hashlib.sha256(" ".join(flags(debug)).encode())
    for f in sorted(glob.glob(os.path.join(SRC, "*.hip")) + glob.glob(os.path.join(SRC, "*.h"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _compile(src: str, force: bool, debug: bool = False) -> str:
    name = os.path.splitext(os.path.basename(src))[0]
    fl = flags(debug)
    dig = _digest(src, " ".join(fl))
    obj = os.path.join(BUILD, f"{name}.{dig}.o")
    if os.path.exists(obj) and not force:
        return obj
    cmd = [hipcc(), *fl, "-I", SRC, "-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(force: bool = False, jobs: int = 8, verbose: bool = True, debug: bool = False) -> str:
    out = OUT_DEBUG if debug else OUT
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(SRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, debug), srcs))
    key = hashlib.sha256("".join(objs).encode()).hexdigest()[:16]
    stamp = out + ".stamp"
    if os.path.exists(out) and not force and os.path.exists(stamp) and open(stamp).read() == key:
        os.utime(out)
        with open(out + ".src", "w") as f:
            f.write(source_digest(debug))
        if verbose:
            print(f"[csk] up to date: {out}")
        return out
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(key)
    with open(out + ".src", "w") as f:
        f.write(source_digest(debug))
    if verbose:
        print(f"[csk] built {out} from {len(srcs)} sources")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true", help="libcsk_debug.so with device-side bounds records")
    a = ap.parse_args(argv)
    build(a.force, a.j, debug=a.debug)


if __name__ == "__main__":
    sys.exit(main())
