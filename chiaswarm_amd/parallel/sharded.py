"""Sharded checkpoint loading over the node's process group (SURVEY §2.7
"Recommended weight-distribution scheme").

The reference loads every model from disk in every job on every GPU
(swarm/diffusion/diffusion_func.py:41-46).  Here, when the per-GPU worker
processes form a process group (RCCL over xGMI on the GPU box, gloo in tests),
a model that all ranks preload is read ONCE across the node:

  1. every rank reads only the safetensors *headers* of the checkpoint files;
     their data regions, concatenated in file order, form one byte stream of
     ``total`` bytes;
  2. the stream is cut into ``world`` equal byte ranges (the last one short);
     rank r reads ONLY range r — one or a few contiguous ``pread`` runs through
     the native reader (runtime/fastload.py, csrc/host/csk_io.cpp) straight into
     its device shard buffer, so its PCIe / page-cache traffic is 1/world of the
     model and runs at link speed;
  3. ONE ``all_gather_into_tensor`` of the raw bytes (uint8) gives every rank
     the whole stream — no per-dtype buckets, no host-side casts;
  4. every tensor is a view of the gathered buffer (the strict loader
     ``models/weights.load_into`` casts it into the module on the device).

Collective: every rank of the group must call it with the same file list in
the same order.  ``models/weights.load_component`` uses it only inside
``comm.collective_loading()`` (the supervisor's preload broadcast); model loads
triggered by an individual job stay rank-local.
"""
from __future__ import annotations

import os
import time

import torch

from ..runtime import fastload

_DT = fastload._DT
read_header = fastload.read_header
ALIGN = 4096  # shard boundaries (bytes)


LAST_READER = None  # the reader of the latest sharded_state_dict call (tests inspect it)


class _Reader:
    """Records what a rank read: (file, begin, end) byte ranges of the files,
    bytes, and the time split between reading and the all_gather."""

    def __init__(self):
        self.ranges: list[tuple[str, int, int]] = []
        self.read_bytes = 0
        self.read_s = 0.0    # this rank's byte-range reads (+ H2D copies), device-synchronised
        self.gather_s = 0.0  # the all_gather (device-synchronised on GPUs)


def shard_bounds(total: int, world: int, rank: int) -> tuple[int, int, int]:
    """(begin, end, shard) of rank ``rank``'s byte range of a ``total``-byte stream."""
    shard = -(-total // world)
    shard = -(-shard // ALIGN) * ALIGN
    b = min(total, rank * shard)
    return b, min(total, b + shard), shard


def sharded_state_dict(files: list[str], dtype: torch.dtype | None, device, reader: _Reader | None = None,
                       group=None) -> dict:
    """Collective: every rank returns the full ``{name: tensor}`` of ``files``
    (views of one gathered byte buffer on ``device``, in the files' own dtypes;
    ``dtype`` is accepted for the old signature and ignored — the consumer
    casts) having read only its own 1/world byte range."""
    import torch.distributed as dist

    global LAST_READER
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    reader = reader or _Reader()
    LAST_READER = reader
    segs = []  # (path, data start in file, data bytes, offset in the stream, header)
    total = 0
    for p in sorted(files):
        start, hdr = read_header(p)
        n = os.path.getsize(p) - start
        segs.append((p, start, n, total, hdr))
        total += n
    b0, b1, shard = shard_bounds(total, world, rank)
    on_gpu = torch.device(device).type == "cuda"
    t0 = time.perf_counter()
    mine = torch.empty(shard, dtype=torch.uint8, device=device)
    for p, start, n, so, _ in segs:
        lo, hi = max(b0, so), min(b1, so + n)
        if lo >= hi:
            continue
        fastload.read_range(p, start + lo - so, mine[lo - b0:hi - b0])
        reader.ranges.append((p, start + lo - so, start + hi - so))
        reader.read_bytes += hi - lo
    full = torch.empty(shard * world, dtype=torch.uint8, device=device)
    if on_gpu:
        torch.cuda.synchronize(device)
    t1 = time.perf_counter()
    dist.all_gather_into_tensor(full, mine, group=group)
    if on_gpu:
        torch.cuda.synchronize(device)
    reader.read_s += t1 - t0
    reader.gather_s += time.perf_counter() - t1
    out = {}
    for _, _, _, so, hdr in segs:
        out.update(fastload.views(full, hdr, base=so))
    return out


def safetensors_files(d: str) -> list[str]:
    fs = sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".safetensors"))
    fp16 = [f for f in fs if ".fp16." in os.path.basename(f)]
    if fp16 and len(fp16) < len(fs):
        fs = [f for f in fs if f not in fp16]
    return fs
