"""Sharded checkpoint distribution over a process group (gloo on CPU here,
RCCL on the GPU node): every rank reads only its 1/world byte range of the
checkpoint's data regions (the native reader, runtime/fastload.py), one
all_gather of the raw bytes assembles the model, and every rank ends with
bitwise-identical weights equal to a plain full read.  World sizes 2 and 4.
Also: ``fastload.load_file`` is bitwise equal to ``safetensors.load_file``."""
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
        q.put((rank, rep.complete, list(rd.ranges), rd.read_bytes,
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
    assert all(r[1] for r in res)
    # the ranks' byte ranges are disjoint and together cover every data byte of every file
    from chiaswarm_amd.runtime.fastload import read_header

    covered = {}
    for r in res:
        for path, b, e in r[2]:
            covered.setdefault(path, []).append((b, e))
    for path, rngs in covered.items():
        rngs.sort()
        start, _ = read_header(path)
        assert rngs[0][0] == start and rngs[-1][1] == os.path.getsize(path)
        for (_, e0), (b1, _) in zip(rngs, rngs[1:]):
            assert e0 == b1
    assert len(covered) == 2
    assert all(r[3] > 0 for r in res)
    assert sum(r[3] for r in res) < total  # headers are never part of a share
    assert max(r[3] for r in res) < 0.75 * total  # nobody read (close to) the whole checkpoint
    for r in res:  # bitwise equal on every rank, and equal to a plain full read
        for k, v in r[4].items():
            assert torch.equal(torch.from_numpy(v), ref[k].float()), k


@pytest.mark.parametrize("native", ["1", "0"])
def test_fastload_bitwise_equal_to_safetensors(tmp_path, monkeypatch, native):
    """The native reader (and its pure-Python fallback) returns exactly the
    tensors safetensors.load_file does, mixed dtypes and odd sizes included,
    for files larger than one 16 MiB staging chunk."""
    from safetensors.torch import load_file

    from chiaswarm_amd.runtime import fastload

    monkeypatch.setattr(fastload, "_LIB", None)
    monkeypatch.setenv("CSK_IO_NATIVE", native)
    g = torch.Generator().manual_seed(0)
    sd = {"big": torch.randn(5 << 20, generator=g),  # 20 MiB fp32: two chunks
          "odd_bf16": torch.randn(7, 13, generator=g).bfloat16(),
          "half": torch.randn(3, 5, generator=g).half(),
          "ids": torch.arange(11, dtype=torch.int64),
          "flag": torch.tensor([True, False, True]),
          "empty": torch.empty(0, 4)}
    path = str(tmp_path / "m.safetensors")
    save_file(sd, path)
    ref = load_file(path)
    got = fastload.load_file(path)
    assert (fastload.lib() is not None) == (native == "1" and os.path.exists(fastload.LIB_PATH))
    assert set(got) == set(ref)
    for k in ref:
        assert got[k].dtype == ref[k].dtype and got[k].shape == ref[k].shape, k
        assert torch.equal(got[k], ref[k]), k
    # a byte range straight into a host tensor
    start, hdr = fastload.read_header(path)
    b, e = hdr["big"][2]
    out = torch.empty(e - b, dtype=torch.uint8)
    fastload.read_range(path, start + b, out)
    assert torch.equal(out.view(torch.float32), sd["big"])
