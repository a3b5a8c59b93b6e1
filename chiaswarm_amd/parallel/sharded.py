"""Sharded checkpoint loading over the node's process group (SURVEY §2.7
"Recommended weight-distribution scheme").

The reference loads every model from disk in every job on every GPU
(swarm/diffusion/diffusion_func.py:41-46).  Here, when the per-GPU worker
processes form a process group (RCCL over xGMI on the GPU box, gloo in tests),
a model that all ranks preload is read ONCE across the node:

  1. every rank reads only the safetensors *headers* (names, dtypes, shapes,
     byte ranges) of the checkpoint files;
  2. the tensors are split into ``world`` contiguous groups of about equal byte
     size; rank r reads ONLY the byte ranges of group r from the file (its own
     PCIe / page-cache traffic is 1/world of the model);
  3. each rank packs its group (cast to the model dtype) into one flat buffer,
     and a single ``all_gather_into_tensor`` per dtype bucket gives every rank
     every group;
  4. the gathered buffer is unpacked into a regular ``{name: tensor}`` state
     dict, which the strict loader (``models/weights.load_into``) consumes.

Collective: every rank of the group must call it with the same file list in
the same order.  ``models/weights.load_component`` uses it only inside
``comm.collective_loading()`` (the supervisor's preload broadcast); model loads
triggered by an individual job stay rank-local.
"""
from __future__ import annotations

import json
import os
import struct

import torch

_DT = {"F64": torch.float64, "F32": torch.float32, "F16": torch.float16, "BF16": torch.bfloat16,
       "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
       "BOOL": torch.bool}


def read_header(path: str) -> tuple[int, dict]:
    """(data start offset, {name: (dtype, shape, (begin, end))}) of a safetensors file."""
    with open(path, "rb") as f:
        n = struct.unpack("<Q", f.read(8))[0]
        hdr = json.loads(f.read(n))
    hdr.pop("__metadata__", None)
    out = {k: (v["dtype"], tuple(v["shape"]), tuple(v["data_offsets"])) for k, v in hdr.items()}
    return 8 + n, out


def plan(entries: list[tuple[str, int]], world: int) -> list[list[str]]:
    """Split (name, nbytes) entries, in order, into ``world`` contiguous groups
    of about equal total bytes (greedy on the running prefix sum)."""
    total = sum(b for _, b in entries)
    groups: list[list[str]] = [[] for _ in range(world)]
    acc = 0
    for name, nb in entries:
        # the group whose byte range [r*total/world, (r+1)*total/world) holds this tensor's midpoint
        mid = acc + nb / 2.0
        r = min(world - 1, int(mid * world / max(total, 1)))
        groups[r].append(name)
        acc += nb
    return groups


LAST_READER = None  # the reader of the latest sharded_state_dict call (tests inspect it)


class _Reader:
    """Reads single tensors by byte range (never the whole file); records what
    it read so tests can check that a rank touched only its own group."""

    def __init__(self):
        self.read_names: list[str] = []
        self.read_bytes = 0
        self.read_s = 0.0    # host time in this rank's byte-range reads + H2D copies
        self.gather_s = 0.0  # time in the all_gather (device-synchronised on GPUs)

    def read(self, path: str, start: int, meta) -> torch.Tensor:
        dt, shape, (b, e) = meta
        with open(path, "rb") as f:
            f.seek(start + b)
            buf = bytearray(f.read(e - b))
        self.read_bytes += e - b
        t = torch.frombuffer(buf, dtype=_DT[dt]) if e > b else torch.empty(0, dtype=_DT[dt])
        return t.reshape(shape)


def sharded_state_dict(files: list[str], dtype: torch.dtype, device, reader: _Reader | None = None,
                       group=None) -> dict:
    """Collective: every rank returns the full ``{name: tensor}`` of ``files``
    (cast to ``dtype`` for floating tensors) having read only its own share."""
    import torch.distributed as dist

    global LAST_READER
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    reader = reader or _Reader()
    LAST_READER = reader
    metas = []
    for p in sorted(files):
        start, hdr = read_header(p)
        for name in sorted(hdr):
            metas.append((p, start, name, hdr[name]))
    entries = [(name, m[2][1] - m[2][0]) for _, _, name, m in metas]
    groups = plan(entries, world)
    owner = {name: r for r, g in enumerate(groups) for name in g}

    def out_dtype(dt):
        return dtype if _DT[dt].is_floating_point else _DT[dt]

    # one flat buffer per output dtype; element counts per rank known to all ranks
    by_dtype: dict = {}
    for p, start, name, meta in metas:
        by_dtype.setdefault(out_dtype(meta[0]), []).append((p, start, name, meta))
    out = {}
    for odt, items in by_dtype.items():
        counts = [0] * world
        for _, _, name, meta in items:
            counts[owner[name]] += int(torch.Size(meta[1]).numel())
        shard = max(counts) if counts else 0
        if shard == 0:
            for _, _, name, meta in items:
                out[name] = torch.empty(meta[1], dtype=odt, device=device)
            continue
        import time

        on_gpu = getattr(torch.device(device), "type", "cpu") == "cuda"
        t0 = time.perf_counter()
        mine = torch.zeros(shard, dtype=odt, device=device)
        off = 0
        for p, start, name, meta in items:
            if owner[name] != rank:
                continue
            t = reader.read(p, start, meta).to(device=device, dtype=odt).reshape(-1)
            mine[off:off + t.numel()] = t
            reader.read_names.append(name)
            off += t.numel()
        full = torch.empty(shard * world, dtype=odt, device=device)
        if on_gpu:
            torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        dist.all_gather_into_tensor(full, mine, group=group)
        if on_gpu:
            torch.cuda.synchronize(device)
        reader.read_s += t1 - t0
        reader.gather_s += time.perf_counter() - t1
        offs = [r * shard for r in range(world)]
        for _, _, name, meta in items:
            r = owner[name]
            n = int(torch.Size(meta[1]).numel())
            out[name] = full[offs[r]:offs[r] + n].view(meta[1])
            offs[r] += n
    return out


def safetensors_files(d: str) -> list[str]:
    fs = sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(".safetensors"))
    fp16 = [f for f in fs if ".fp16." in os.path.basename(f)]
    if fp16 and len(fp16) < len(fs):
        fs = [f for f in fs if f not in fp16]
    return fs
