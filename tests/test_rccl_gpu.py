"""RCCL and the native reader on a real MI355X.

Every collective path of the worker had only run under gloo.  Here one spawned
process forms a real ``nccl`` (= RCCL) process group at world size 1 — the
only size a one-GPU box allows — with ``init_process_group(device_id=...)``
exactly as ``parallel/comm.init_distributed`` does on an 8-GPU node, and runs
the production code paths on GPU tensors:

* the sharded checkpoint load (parallel/sharded.py): native byte-range read
  into the device shard + ``all_gather_into_tensor`` of the raw bytes;
* the CFG-parallel prediction exchange (``comm.exchange_cfg_half``:
  ``batch_isend_irecv``, here to itself) and the handshake;
* ``comm.barrier`` (``barrier(device_ids=...)``);
* a captured hipGraph of a HIP-library GEMM replayed between collectives.

``HSA_ENABLE_IPC_MODE_LEGACY=0`` is inherited from the box's environment.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_main(port, d, q):
    os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from chiaswarm_amd import ops
    from chiaswarm_amd.parallel import comm, sharded
    from chiaswarm_amd.runtime import fastload

    out = {}
    try:
        comm.init_distributed(backend="nccl", timeout_s=120, force=True)
        out["backend"] = dist.get_backend()
        dev = torch.device("cuda", 0)
        ops._lib.load()
        # a graph captured before the collectives run ...
        x = torch.randn(256, 320, device=dev).bfloat16()
        w = torch.randn(640, 320, device=dev).bfloat16()
        ref = ops.gemm(x, w)
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ops.gemm(x, w)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = ops.gemm(x, w)
        g.replay()
        # ... the sharded load: native read of this rank's byte range + RCCL all_gather
        files = sharded.safetensors_files(d)
        sd = sharded.sharded_state_dict(files, None, dev)
        plain = {}
        for f in files:
            plain.update(fastload.load_file(f, device="cpu"))
        out["sharded_equal"] = set(sd) == set(plain) and all(
            sd[k].device.type == "cuda" and torch.equal(sd[k].cpu(), plain[k]) for k in plain)
        out["read_bytes"] = sharded.LAST_READER.read_bytes
        g.replay()
        # CFG-parallel exchange: batch_isend_irecv (to itself at world 1)
        assert comm.cfg_handshake(0, ok=True)
        e = torch.randn(1, 64, 64, 4, device=dev).bfloat16()
        full = comm.exchange_cfg_half(e, peer=0, half=0)
        out["exchange_ok"] = full.device == e.device and torch.equal(full, torch.cat((e, e), 0))
        comm.barrier()  # barrier(device_ids=[0]) on RCCL
        g.replay()
        t = torch.full((4,), 3.0, device=dev)
        dist.all_reduce(t)
        out["all_reduce_ok"] = bool((t == 3.0).all())
        torch.cuda.synchronize()
        out["graph_equal"] = torch.equal(y, ref)
        dist.destroy_process_group()
    except Exception as ex:  # reported to the parent, which fails the test with it
        out["error"] = f"{type(ex).__name__}: {ex}"
    q.put(out)


def _write_checkpoint(d):
    from safetensors.torch import save_file

    g = torch.Generator().manual_seed(3)
    save_file({"a.weight": torch.randn(1000, 77, generator=g), "b.bias": torch.randn(33, generator=g).half(),
               "c.ids": torch.arange(5)}, os.path.join(d, "x.safetensors"))
    save_file({"d.weight": torch.randn(4096, 129, generator=g).bfloat16()}, os.path.join(d, "y.safetensors"))


def test_rccl_world1_production_collectives(tmp_path):
    d = str(tmp_path)
    _write_checkpoint(d)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_main, args=(_free_port(), d, q))
    p.start()
    p.join(180)
    if p.is_alive():
        p.kill()
        p.join(10)
        pytest.fail("RCCL world-1 process did not finish in 180 s")
    assert p.exitcode == 0
    out = q.get(timeout=10)
    assert "error" not in out, out.get("error")
    assert out["backend"] == "nccl"
    assert out["sharded_equal"] and out["read_bytes"] > 0
    assert out["exchange_ok"] and out["all_reduce_ok"] and out["graph_equal"]


def test_fastload_device_bitwise_and_rate(tmp_path):
    """The native reader's device path (pinned ring + hipMemcpyAsync) returns
    exactly safetensors' tensors, and moves a 1 GiB file from the page cache at
    well over the pageable-copy rate (prints the GB/s)."""
    import time

    from safetensors.torch import load_file, save_file

    from chiaswarm_amd.runtime import fastload

    assert fastload.lib() is not None, "libcskio.so not built"
    g = torch.Generator().manual_seed(1)
    sd = {f"w{i}": torch.randn(32 << 20, generator=g).bfloat16() for i in range(16)}  # 16 x 64 MiB
    sd["odd"] = torch.randn(7, 3, generator=g)
    path = str(tmp_path / "big.safetensors")
    save_file(sd, path)
    with open(path, "rb") as f:  # page cache warm, as on a preloaded worker
        while f.read(1 << 26):
            pass
    dev = torch.device("cuda", 0)
    got = fastload.load_file(path, device=dev)  # (first call allocates the pinned ring)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = fastload.load_file(path, device=dev)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    size = os.path.getsize(path)
    print(f"fastload device: {size / dt / 1e9:.1f} GB/s ({size / 1e9:.2f} GB in {dt * 1e3:.1f} ms)")
    ref = load_file(path)
    for k in ref:
        assert got[k].device.type == "cuda" and torch.equal(got[k].cpu(), ref[k]), k
    assert size / dt > 8e9  # pageable per-tensor copies ran at ~3 GB/s
