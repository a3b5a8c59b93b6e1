"""Sharded checkpoint distribution over a process group (gloo on CPU here,
RCCL on the GPU node): every rank reads only its byte ranges, one all_gather
assembles the model, and every rank ends with bitwise-identical weights equal
to a plain full read.  World sizes 2 and 4."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from safetensors.torch import save_file


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_checkpoint(d):
    from chiaswarm_amd.models import clip
    from chiaswarm_amd.models.layers import init_random_

    m = clip.CLIPTextModel(clip.TINY_TEXT)
    init_random_(m, seed=5)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    keys = sorted(sd)
    os.makedirs(os.path.join(d, "text_encoder"), exist_ok=True)
    # two shard files, one of them fp16 (cast on load), like real multi-file checkpoints
    save_file({k: sd[k] for k in keys[: len(keys) // 2]}, os.path.join(d, "text_encoder", "a.safetensors"))
    save_file({k: sd[k].half() for k in keys[len(keys) // 2:]}, os.path.join(d, "text_encoder", "b.safetensors"))
    ref = {k: (sd[k] if i < len(keys) // 2 else sd[k].half().float()) for i, k in enumerate(keys)}
    return ref


def _worker(rank, world, port, d, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from chiaswarm_amd.models import clip
        from chiaswarm_amd.models.weights import load_component
        from chiaswarm_amd.parallel import comm, sharded

        m = clip.CLIPTextModel(clip.TINY_TEXT)
        with comm.collective_loading():
            rep = load_component(m, d, "text_encoder")
        rd = sharded.LAST_READER
        q.put((rank, rep.complete, sorted(rd.read_names), rd.read_bytes,
               {k: v.float().numpy().copy() for k, v in m.state_dict().items()}))  # by value, not shared fds
        # outside the context the same call is rank-local (no collective)
        m2 = clip.CLIPTextModel(clip.TINY_TEXT)
        sharded.LAST_READER = None
        load_component(m2, d, "text_encoder")
        assert sharded.LAST_READER is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_load_reads_only_own_share(tmp_path, world):
    d = str(tmp_path)
    ref = _make_checkpoint(d)
    total = sum(os.path.getsize(os.path.join(d, "text_encoder", f)) for f in os.listdir(os.path.join(d, "text_encoder")))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, d, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    names = [set(r[2]) for r in res]
    assert all(r[1] for r in res)
    for i in range(world):  # disjoint shares that together cover every tensor
        for j in range(i + 1, world):
            assert not names[i] & names[j]
    assert set().union(*names) == set(ref)
    assert all(len(n) > 0 for n in names)
    assert max(r[3] for r in res) < 0.75 * total  # nobody read (close to) the whole checkpoint
    for r in res:  # bitwise equal on every rank, and equal to a plain full read
        for k, v in r[4].items():
            assert torch.equal(torch.from_numpy(v), ref[k].float()), k
