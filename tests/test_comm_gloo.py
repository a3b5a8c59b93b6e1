"""Multi-process distribution paths on CPU (gloo, world_size 2 and 4): sharded
all_gather of module weights is bitwise identical to the source, broadcast,
split-job tensor all-gather (the bench's rank spawning: tests/test_bench_cpu.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from chiaswarm_amd.models import unet
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.parallel import comm

    comm.init_distributed(backend="gloo")
    try:
        # every rank builds the model; only rank 0 has the "true" weights
        m = unet.UNet2DConditionModel(unet.TINY)
        init_random_(m, seed=123 if rank == 0 else 999 + rank)
        ref = [p.detach().clone() for p in m.parameters()]
        # broadcast from rank 0 -> everyone equals rank 0
        comm.broadcast_module(m, src=0, bucket_bytes=1 << 16)
        cs = comm.module_checksum(m)
        # sharded all_gather: after broadcast all shards agree, result unchanged bitwise
        comm.allgather_module(m, bucket_bytes=1 << 15)
        same = all(torch.equal(a, b) for a, b in zip(ref, m.parameters())) if rank == 0 else None
        x = torch.full((2, 3), float(rank))
        g = comm.all_gather_tensor(x)
        mx = comm.max_over_ranks(float(rank))
        q.put((rank, cs, same, g[:, 0].tolist(), mx))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_weight_distribution(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort()
    checks = {o[1] for o in out}
    assert len(checks) == 1  # identical weights everywhere
    assert out[0][2] is True  # rank 0 weights unchanged by broadcast + sharded gather
    for o in out:
        assert o[3] == [float(r) for r in range(world) for _ in range(2)]
        assert o[4] == world - 1
