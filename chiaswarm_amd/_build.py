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
import re
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


# ---- assembly lint: hazards hipcc does not pad around inline asm ----------
# A transcendental VALU op (v_exp / v_log / v_rcp / v_rsq / v_sqrt) needs one
# wait state before a VALU reads its result (CDNA3/4 trans forwarding hazard).
# hipcc pads its own readers, not an inline-asm reader (common.h vadd / vmax3),
# and a schedule that puts one right behind the v_exp reads the pre-exp value:
# the persistent attention's row sums went wrong this way in one build.
_TRANS = re.compile(r"^\s*(v_(?:exp|log|rcp|rsq|sqrt)_f(?:32|16)\w*)\s+(v\d+)")
# profiling variants (wrong results by design) are exempt
_LINT_EXEMPT = (re.compile(r"attn_fa_kernelILi[1-9]"), re.compile(r"attn32_kernelILi1ELi[1-9]"))


def lint_asm(text: str) -> list:
    """(function, line, trans op, reader) of every trans result read by the
    very next instruction."""
    out, func, prev = [], "", None
    for n, line in enumerate(text.split("\n"), 1):
        t = line.strip()
        if re.match(r"^_Z\w*:", line):
            func, prev = line.split(":")[0], None
            continue
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        if prev is not None and t.startswith("v_"):
            parts = t.split(None, 1)
            srcs = parts[1].split(",")[1:] if len(parts) > 1 else []
            if any(re.search(r"\b%s\b" % prev[1], x) for x in srcs):
                out.append((func, n, prev[0], t))
        m = _TRANS.match(line)
        prev = (t, m.group(2)) if m else None
    return [h for h in out if not any(e.search(h[0]) for e in _LINT_EXEMPT)]


def _lint(src: str, fl: list, dig: str) -> None:
    name = os.path.splitext(os.path.basename(src))[0]
    ok = os.path.join(BUILD, f"{name}.{dig}.lint")
    if os.path.exists(ok):
        return
    asm = os.path.join(BUILD, f"{name}.{dig}.s")
    cmd = [hipcc(), *[f for f in fl if f != "-fPIC"], "-I", SRC, "-S", "--cuda-device-only", src, "-o", asm]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc -S failed for {src}:\n{r.stderr}")
    with open(asm) as f:
        hits = lint_asm(f.read())
    os.remove(asm)
    if hits:
        msg = "\n".join(f"  {fn} (.s line {n}): {a}  ->  {b}" for fn, n, a, b in hits[:10])
        raise RuntimeError(f"{src}: transcendental result read by the next (inline-asm) instruction — "
                           f"use vadd_t / an s_nop:\n{msg}")
    open(ok, "w").close()


def _compile(src: str, force: bool, debug: bool = False) -> str:
    name = os.path.splitext(os.path.basename(src))[0]
    fl = flags(debug)
    dig = _digest(src, " ".join(fl))
    obj = os.path.join(BUILD, f"{name}.{dig}.o")
    if os.path.exists(obj) and not force:
        _lint(src, fl, dig)
        return obj
    cmd = [hipcc(), *fl, "-I", SRC, "-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    _lint(src, fl, dig)
    return obj


HOST_SRC = os.path.join(ROOT, "csrc", "host")
OUT_IO = os.path.join(ROOT, "chiaswarm_amd", "lib", "libcskio.so")


def io_digest() -> str:
    h = hashlib.sha256(b"cskio-v1")
    for f in sorted(glob.glob(os.path.join(HOST_SRC, "*.cpp"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_io(force: bool = False, verbose: bool = True) -> str:
    """``libcskio.so``: the host-side native checkpoint reader
    (``csrc/host/csk_io.cpp``: threaded pread into a pinned staging ring +
    hipMemcpyAsync).  Plain host C++ against the HIP runtime, built with g++."""
    dig = io_digest()
    stamp = OUT_IO + ".src"
    if os.path.exists(OUT_IO) and not force and os.path.exists(stamp) and open(stamp).read().strip() == dig:
        return OUT_IO
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cxx = shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no host C++ compiler for csrc/host")
    srcs = sorted(glob.glob(os.path.join(HOST_SRC, "*.cpp")))
    cmd = [cxx, "-D__HIP_PLATFORM_AMD__", f"-I{rocm}/include", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           *srcs, "-o", OUT_IO + ".tmp", f"-L{rocm}/lib", "-lamdhip64", "-lpthread", f"-Wl,-rpath,{rocm}/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"host library build failed:\n{r.stderr}")
    os.replace(OUT_IO + ".tmp", OUT_IO)
    with open(stamp, "w") as f:
        f.write(dig)
    if verbose:
        print(f"[csk] built {OUT_IO} from {len(srcs)} host sources")
    return OUT_IO


def build(force: bool = False, jobs: int = 8, verbose: bool = True, debug: bool = False) -> str:
    build_io(force, verbose)
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
