"""Per-shape kernel configuration table (the ``cudnn.benchmark`` analogue the
reference turned on at swarm/worker.py:180; SURVEY §5.4 "tuned-kernel table on
disk").

For every GEMM / implicit-GEMM conv shape we pick (tile, ksplit):
  tile   1:128x128  2:128x64  3:64x128  4:64x64  5:128x32  6:128x64(4x1 waves)
  ksplit split-K factor (fp32 partials + reduce kernel) for small-M/large-K
         shapes (UNet 16x16 / 8x8 levels) that would otherwise not fill 256 CUs.

Lookup order: in-memory -> user table ($SDAAS_ROOT/csk_tune.json) -> shipped
table (chiaswarm_amd/lib/tune_gfx950.json, measured on MI355X) -> heuristic;
inside ``context("sdxl")`` (the SDXL UNet) an "sdxl|<key>" entry wins over the
plain key.
With CSK_AUTOTUNE=1 a miss is measured on the spot (outside graph capture)
with hip events over every candidate and the winner is recorded.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading

import torch

SHIPPED = os.environ.get("CSK_TUNE_FILE") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "tune_gfx950.json")
_TABLE: dict | None = None
_LOCK = threading.Lock()
TILES = {1: (128, 128), 2: (128, 64), 3: (64, 128), 4: (64, 64), 5: (128, 32), 6: (128, 64),
         # LDS-DMA multi-stage variants (gemm_glds.hip)
         11: (128, 128), 12: (128, 64), 13: (64, 128), 14: (64, 64), 15: (128, 128), 16: (128, 32), 17: (128, 64),
         18: (64, 64), 19: (128, 64), 20: (64, 128),
         # one 256x160 workgroup per CU (3-stage, 156 KB LDS): least L2->LDS traffic per output
         25: (256, 160), 26: (128, 160),
         # 4-stage rings (3 K-steps in flight) for latency-bound low-M / long-K shapes
         27: (128, 128), 28: (64, 128), 29: (128, 64),
         # 8-wave 256-row phased tiles (gemm8p.hip): half the L2->LDS bytes per FLOP of 128x128
         31: (256, 256), 32: (256, 128),
         # 8-wave 256x160 3-stage ring (gemm8p.hip gemm8r_kernel): 0.0102 B/FLOP, 256 tiles at the 64x64 level
         33: (256, 160), 34: (256, 128),
         # 64x160 2-stage (fewest L2->LDS bytes per output of the 64-row tiles)
         36: (64, 160)}
GLDS = frozenset(range(11, 30)) | {36}  # gemm_glds.hip tiles (in-kernel split-K fixup)
# waves along M of the tiles whose epilogue stages one wave-row band at a time
# (gemm_common.h epi_passes: BM > 128 or BN == 160); the GN-statistics segment
# cannot exceed that band (hip_ops._gn_seg mirrors gemm_common.h gn_seg_for)
EPI_WM = {25: 2, 26: 2, 31: 2, 32: 2, 33: 4, 34: 4, 36: 2}


def _user_path():
    root = os.environ.get("SDAAS_ROOT") or os.path.expanduser("~/.sdaas")
    return os.path.join(root, "csk_tune.json")


def table() -> dict:
    global _TABLE
    if _TABLE is None:
        t = {}
        for p in (() if os.environ.get("CSK_RETUNE") == "1" else (SHIPPED, _user_path())):
            try:
                with open(p) as f:
                    t.update(json.load(f))
            except (FileNotFoundError, json.JSONDecodeError):
                pass
        _TABLE = t
    return _TABLE


def save_user():
    p = _user_path()
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p, "w") as f:
        json.dump(table(), f, indent=0, sort_keys=True)


def heuristic(M, N, K) -> tuple[int, int]:
    """Untuned shapes, from the MI355X sweeps (tools/gemmprof.py, the tuned
    table): LDS-DMA tiles everywhere; short K (<= 1280, latency/bandwidth
    bound) prefers the small-LDS 2-stage tiles (3-5 workgroups per CU), long K
    (3x3 convs) the 128x128 tile; split-K only when the grid cannot fill 256 CUs."""
    if N <= 32:
        return 16, 1
    tiles128 = -(-M // 128) * -(-N // 128)
    tiles12864 = -(-M // 128) * -(-N // 64)
    tiles64 = -(-M // 64) * -(-N // 64)
    if K <= 1280:
        if N <= 1280 and tiles12864 >= 256:
            return 19, 1
        if tiles64 >= 256:
            return 18, 1
    elif tiles128 >= 384:
        return 11, 1
    elif tiles64 >= 384:
        return 14, 1
    split = 1
    while tiles64 * split < 384 and K // 64 >= 4 * split * 2 and split < 8:
        split *= 2
    return 18, split


def candidates(M, N, K):
    out = []
    for tile, (bm, bn) in TILES.items():
        if tile in (5, 16) and N > 32:
            continue
        if tile in (2, 6, 12, 17, 19, 22, 24, 29) and N > 1280:
            continue
        if tile >= 31 and K % 64:
            continue
        ntiles = -(-M // bm) * -(-N // bn)
        for split in (1, 2, 4, 8, 16):  # 16: the 8x8-level convs (M = 512 rows, K = 11520 / 23040)
            if split > 1 and (ntiles >= 512 or K // 64 < 4 * split):
                continue
            if split == 16 and ntiles > 64:
                continue
            out.append((tile, split))
            if split > 1 and tile in GLDS:
                out.append((tile, -split))  # the same split with the in-kernel fixup (no reduce launch)
    return out


def _time(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


_CTX = threading.local()


@contextlib.contextmanager
def context(name: str | None):
    """Tuning context of the calls inside (e.g. "sdxl": the SDXL UNet): a shape
    key shared by two models' steps (M2048 N1280 K1280 is both SD2.1's CFG-8
    16x16 level and SDXL's CFG-2 32x32 level) may take a different tile in each;
    ``choose`` looks up "<context>|<key>" first, then the plain key."""
    prev = getattr(_CTX, "name", None)
    _CTX.name = name
    try:
        yield
    finally:
        _CTX.name = prev


def current_context() -> str | None:
    return getattr(_CTX, "name", None)


def choose(key: str, M: int, N: int, K: int, runner) -> tuple[int, int]:
    """runner(tile, ksplit) launches the kernel once (used only when tuning)."""
    t = table()
    ctx = getattr(_CTX, "name", None)
    hit = t.get(f"{ctx}|{key}") if ctx else None
    if hit is None:
        hit = t.get(key)
    if hit is not None:
        return int(hit[0]), int(hit[1])
    if os.environ.get("CSK_AUTOTUNE") == "1" and not torch.cuda.is_current_stream_capturing():
        with _LOCK:
            best, best_ms = None, float("inf")
            for tile, split in candidates(M, N, K):
                try:
                    ms = _time(lambda: runner(tile, split))
                except RuntimeError:
                    continue
                if ms < best_ms:
                    best, best_ms = (tile, split), ms
            if best is not None:
                t[key] = [best[0], best[1], round(best_ms * 1000, 2)]
                return best
    return heuristic(M, N, K)
