"""Intra-node RCCL communication (torch.distributed backend "nccl" == RCCL on
ROCm) over xGMI.  The reference has no collectives at all (all its
parallelism is one job per GPU); these are the north-star additions:

  * ``allgather_module``: every rank holds/loads 1/N of a model's bytes and one
    ``all_gather_into_tensor`` per dtype-bucket assembles the full copy on all
    GPUs (each GPU reads only 1/N over its own PCIe link; xGMI does the rest);
  * ``broadcast_module``: rank-0-loads fallback, bucketed;
  * ``all_gather_tensor``: split-job latent / image assembly.

Buckets are large (default 512 MiB): with 288 GB HBM per GPU there is no
reason to chunk finely, and fewer, larger collectives keep each xGMI link busy.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

BUCKET_BYTES = 512 << 20


def env_rank():
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def init_distributed(backend: str | None = None, timeout_s: int = 600, force: bool = False):
    """Initialise the process group from torchrun env vars (one rank per GPU).

    With ``SDAAS_STORE_PORT`` set (the worker's GPU children) the rendezvous is
    the TCPStore the SUPERVISOR hosts (runtime/worker.py), namespaced by the
    group generation ``SDAAS_GROUP_GEN``: the store outlives any GPU child, so
    a crashed rank 0 takes no surviving rank's store with it, and a re-formed
    group (a new generation) never reads a stale key of the old one.
    ``force``: form the group even at world size 1 (the GPU test of the RCCL
    paths, tests/test_rccl_gpu.py)."""
    rank, local_rank, world = env_rank()
    if world <= 1 and not force:
        return rank, local_rank, world
    if dist.is_initialized():
        return rank, local_rank, world
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", local_rank)
    timeout = datetime.timedelta(seconds=timeout_s)
    if os.environ.get("SDAAS_STORE_PORT"):
        kw["store"] = group_store(timeout)
    dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=timeout, **kw)
    return rank, local_rank, world


def group_store(timeout=datetime.timedelta(seconds=600)):
    """Client of the supervisor-hosted TCPStore, prefixed by the group generation."""
    base = dist.TCPStore(os.environ.get("SDAAS_STORE_HOST", "127.0.0.1"), int(os.environ["SDAAS_STORE_PORT"]),
                         is_master=False, timeout=timeout)
    return dist.PrefixStore(f"gen{os.environ.get('SDAAS_GROUP_GEN', '0')}/", base)


def leave_group():
    """Drop this process's process group without waiting on its peers (a dead
    peer would make a graceful destroy block): abort the communicators."""
    if not dist.is_initialized():
        return
    try:
        from torch.distributed.distributed_c10d import _abort_process_group

        _abort_process_group()
    except Exception:  # pragma: no cover - older torch / already torn down
        try:
            dist.destroy_process_group()
        except Exception:
            pass


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


_COLLECTIVE_LOAD = False


class collective_loading:
    """Within this context every rank of the process group loads the SAME
    models in the SAME order, so checkpoint reads may be sharded across ranks
    (parallel/sharded.py).  Outside it, loads are rank-local (a job-triggered
    load on one GPU must never wait on the others)."""

    def __enter__(self):
        global _COLLECTIVE_LOAD
        self._prev = _COLLECTIVE_LOAD
        _COLLECTIVE_LOAD = is_dist()
        return self

    def __exit__(self, *exc):
        global _COLLECTIVE_LOAD
        _COLLECTIVE_LOAD = self._prev
        return False


def collective_load_active() -> bool:
    return _COLLECTIVE_LOAD and is_dist()


def barrier():
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _buckets(tensors, limit=BUCKET_BYTES):
    """Group tensors by dtype into buckets of <= limit bytes (order preserved)."""
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for _, ts in by_dtype.items():
        cur, size = [], 0
        for t in ts:
            nb = t.numel() * t.element_size()
            if cur and size + nb > limit:
                yield cur
                cur, size = [], 0
            cur.append(t)
            size += nb
        if cur:
            yield cur


def _state_tensors(module):
    return [p.data for p in module.parameters()] + [b for b in module.buffers()]


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0, bucket_bytes=BUCKET_BYTES):
    if not is_dist():
        return module
    for bucket in _buckets(_state_tensors(module), bucket_bytes):
        flat = torch.cat([t.reshape(-1) for t in bucket])
        dist.broadcast(flat, src)
        off = 0
        for t in bucket:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n
    return module


@torch.no_grad()
def allgather_module(module: torch.nn.Module, bucket_bytes=BUCKET_BYTES):
    """Sharded distribution: rank r contributes elements [r*L, (r+1)*L) of each
    flattened bucket (the part it loaded from host); one all_gather per bucket
    rebuilds the full bucket on every rank."""
    if not is_dist():
        return module
    world, rank = dist.get_world_size(), dist.get_rank()
    for bucket in _buckets(_state_tensors(module), bucket_bytes):
        flat = torch.cat([t.reshape(-1) for t in bucket])
        n = flat.numel()
        shard = (n + world - 1) // world
        padded = torch.zeros(shard * world, dtype=flat.dtype, device=flat.device)
        padded[:n] = flat
        mine = padded[rank * shard:(rank + 1) * shard].clone()
        dist.all_gather_into_tensor(padded, mine)
        off = 0
        for t in bucket:
            k = t.numel()
            t.copy_(padded[off:off + k].view_as(t))
            off += k
    return module


def all_gather_tensor(x: torch.Tensor) -> torch.Tensor:
    """Concatenate equal-shaped per-rank tensors along dim 0 on every rank."""
    if not is_dist():
        return x
    world = dist.get_world_size()
    out = torch.empty((world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous())
    return out


def max_over_ranks(value: float) -> float:
    if not is_dist():
        return value
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def module_checksum(module: torch.nn.Module) -> float:
    s = 0.0
    for t in _state_tensors(module):
        s += float(t.float().sum().item())
    return s


def send_tensor(x: torch.Tensor, dst: int):
    """Point-to-point transfer (RCCL over xGMI between GPU children; gloo on CPU)."""
    dist.send(x.contiguous(), dst)


def recv_tensor(shape, dtype, src: int, device) -> torch.Tensor:
    out = torch.empty(tuple(shape), dtype=dtype, device=device)
    dist.recv(out, src)
    return out


def group_device():
    """Where this rank's collective tensors live: its GPU under RCCL, host under gloo."""
    if dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


# -- split-job image transfer (runtime/worker.py splits a multi-image job over
#    idle GPUs; every part's uint8 images go to the leader rank over the group)
def send_images(images: torch.Tensor | None, dst: int, nsfw: bool = False):
    """Helper side: header [n, H, W, C, nsfw] then the uint8 NHWC payload; ``None``
    sends an error header (n = -1) so the leader never waits on a failed part."""
    dev = group_device()
    if images is None:
        send_tensor(torch.tensor([-1, 0, 0, 0, 0], dtype=torch.int64, device=dev), dst)
        return
    n, h, w, c = images.shape
    send_tensor(torch.tensor([n, h, w, c, int(bool(nsfw))], dtype=torch.int64, device=dev), dst)
    send_tensor(images.to(dev, torch.uint8), dst)


def recv_images(src: int):
    """Leader side: (uint8 [n, H, W, C] on the group device, nsfw) or (None, False)
    when the part failed."""
    dev = group_device()
    hdr = recv_tensor((5,), torch.int64, src, dev).tolist()
    if hdr[0] < 0:
        return None, False
    return recv_tensor(tuple(hdr[:4]), torch.uint8, src, dev), bool(hdr[4])


# -- CFG-parallel (runtime/worker.py: a one-image CFG job on two idle GPUs; each
#    rank evaluates one CFG half of the UNet batch and they swap predictions)
def cfg_handshake(peer: int, ok: bool = True) -> bool:
    """Both parts of a CFG-parallel job exchange a ready flag before the first
    step; a part that failed before its denoise loop sends ``ok=False``
    (pipelines.diffusion._split_failed) so its peer raises instead of waiting
    on predictions that never come.  Returns the peer's flag."""
    dev = group_device()
    mine = torch.tensor([1 if ok else -1], dtype=torch.int64, device=dev)
    other = torch.empty_like(mine)
    for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, mine, peer), dist.P2POp(dist.irecv, other, peer)]):
        r.wait()
    return int(other.item()) > 0


def exchange_cfg_half_into(e_full: torch.Tensor, peer: int, half: int):
    """In-place form for the graph-resident CFG-parallel loop: ``e_full``
    [2B, ...] holds this rank's half in rows [half*B, (half+1)*B); the peer's
    half is received into the other rows.  On RCCL the send / receive are
    enqueued on the current stream (their ``wait`` orders the stream, the host
    never blocks); on gloo the halves go through the host."""
    b = e_full.shape[0] // 2
    mine, other = e_full[half * b:(half + 1) * b], e_full[(1 - half) * b:(2 - half) * b]
    dev = group_device()
    if dev.type == e_full.device.type:
        ops = [dist.P2POp(dist.isend, mine, peer), dist.P2POp(dist.irecv, other, peer)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        return
    m, o = mine.to(dev).contiguous(), torch.empty(other.shape, dtype=other.dtype, device=dev)
    for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, m, peer), dist.P2POp(dist.irecv, o, peer)]):
        r.wait()
    other.copy_(o)


def exchange_cfg_half(e: torch.Tensor, peer: int, half: int) -> torch.Tensor:
    """This rank's noise prediction for its CFG half <-> the peer's (one
    send + one receive, posted together): returns [uncond; cond] on e's device.
    SD 512 px batch 1: 32 KB per step over xGMI."""
    dev = group_device()
    mine = e.contiguous() if e.device == dev else e.to(dev).contiguous()
    other = torch.empty_like(mine)
    for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, mine, peer), dist.P2POp(dist.irecv, other, peer)]):
        r.wait()
    full = torch.cat((mine, other) if half == 0 else (other, mine), 0)
    return full if full.device == e.device else full.to(e.device)
