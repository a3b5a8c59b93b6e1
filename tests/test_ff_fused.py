"""Fused feed-forward (csrc/kernels/ff.hip; SURVEY K10 + K11): x + FF(LN3(x))
of an SD transformer block at C = 320 in one kernel, the [M, 1280] GEGLU
intermediate never leaving the chip.

CPU: the packing round-trips (the fp32 reference built from the packed weights
equals the unfused LayerNorm -> GEGLU -> down-projection composition of the
module).  GPU: the HIP kernel against that fp32 composition on full and ragged
grids, with and without biases, and the transformer block with the fused path
against the unfused one."""
import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.models.layers import BasicTransformerBlock, init_random_


def _unfused(x, blk):
    ff = blk.ff
    h = torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), blk.norm3.weight.float(), blk.norm3.bias.float(),
                                       blk.norm3.eps)
    p = ff.net[0].proj
    vg = torch.nn.functional.linear(h, p.weight.float(), None if p.bias is None else p.bias.float())
    inner = vg.shape[-1] // 2
    hid = vg[..., :inner] * torch.nn.functional.gelu(vg[..., inner:])
    d = ff.net[2]
    return x.float() + torch.nn.functional.linear(hid, d.weight.float(), None if d.bias is None else d.bias.float())


def _setup(dev, dtype, B=2, S=256, C=320, seed=0):
    torch.manual_seed(seed)
    blk = BasicTransformerBlock(C, C // 64, 64, 1024).to(dev)
    init_random_(blk, seed=seed)
    with torch.no_grad():  # non-trivial LayerNorm affine and biases
        blk.norm3.weight.uniform_(0.5, 1.5)
        blk.norm3.bias.normal_(0, 0.2)
        blk.ff.net[0].proj.bias.normal_(0, 0.3)
        blk.ff.net[2].bias.normal_(0, 0.3)
    blk = blk.to(dtype)
    x = (torch.randn(B, S, C, device=dev) * 2 + 0.5).to(dtype)
    return blk, x


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / ref.norm()).item()


def test_pack_roundtrip_cpu():
    blk, x = _setup("cpu", torch.float32)
    w1p, b1p, w2p = blk.ff.fused_weights()
    assert w1p.shape == (80, 5, 32, 64) and b1p.shape == (80, 32) and w2p.shape == (40, 10, 32, 32)
    w1, b1, w2 = ops.unpack_ff_fused(w1p, b1p, w2p)
    p = blk.ff.net[0].proj
    assert torch.equal(w1, p.weight) and torch.equal(b1, p.bias) and torch.equal(w2, blk.ff.net[2].weight)
    y = ops._ref_ff_fused(x, blk.norm3.weight, blk.norm3.bias, w1p, b1p, w2p, blk.ff.net[2].bias, blk.norm3.eps)
    ref = _unfused(x, blk)
    assert torch.allclose(y, ref, atol=1e-4, rtol=1e-4), (y - ref).abs().max()


def test_ff_fused_off_cpu_and_other_widths():
    """Not a HIP path on CPU; only C = 320 blocks carry the packed weights."""
    blk, x = _setup("cpu", torch.float32)
    assert not ops.ff_fusable(x, blk.ff.inner)
    blk640 = BasicTransformerBlock(640, 10, 64, 1024)
    assert blk640.ff.fused_weights() == (None, None, None)


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,bias", [(8, 4096, True), (2, 300, True), (1, 128, False), (3, 77, True)])
def test_ff_kernel_matches_fp32(gpu, B, S, bias):
    from chiaswarm_amd.ops import hip_ops

    blk, x = _setup(gpu, torch.bfloat16, B=B, S=S)
    if not bias:
        with torch.no_grad():
            blk.ff.net[0].proj.bias = None
            blk.ff.net[2].bias = None
        blk.ff.prepare()
    w1p, b1p, w2p = blk.ff.fused_weights()
    y = hip_ops.ff_geglu(x, blk.norm3.weight, blk.norm3.bias, w1p, b1p, w2p, blk.ff.net[2].bias, blk.norm3.eps)
    torch.cuda.synchronize()
    ref = _unfused(x.cpu().float(), blk.cpu().float())
    assert torch.isfinite(y.float()).all()
    assert rel_err(y.cpu(), ref) < 1.2e-2


@pytest.mark.gpu
def test_ff_kernel_deterministic_and_graph_replay(gpu):
    from chiaswarm_amd.ops import hip_ops

    blk, x = _setup(gpu, torch.bfloat16, B=2, S=1024)
    w = blk.ff.fused_weights()
    args = (blk.norm3.weight, blk.norm3.bias, *w, blk.ff.net[2].bias, blk.norm3.eps)
    a = hip_ops.ff_geglu(x, *args)
    b = hip_ops.ff_geglu(x, *args)
    assert torch.equal(a, b)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hip_ops.ff_geglu(x, *args)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        c = hip_ops.ff_geglu(x, *args)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(c, a)


@pytest.mark.gpu
def test_block_with_fused_ff_matches_unfused(gpu, monkeypatch):
    """The transformer block takes the fused FF on the CFG-batch-8 64x64 grid and
    agrees with the unfused GEMM chain."""
    from chiaswarm_amd.ops import hip_ops

    blk, x = _setup(gpu, torch.bfloat16, B=8, S=4096)
    ctx = torch.randn(8, 77, 1024, device=gpu).bfloat16()
    kv = blk.attn2.context_kv(ctx)
    calls = []
    orig = hip_ops.ff_geglu
    monkeypatch.setattr(hip_ops, "ff_geglu", lambda *a, **k: calls.append(1) or orig(*a, **k))
    y_fused = blk(x, kv=kv, row_stats=False)
    assert calls == [1]
    monkeypatch.setattr(hip_ops, "FF_FUSED", False)
    y_ref = blk(x, kv=kv, row_stats=False)
    assert calls == [1]
    torch.cuda.synchronize()
    assert rel_err(y_fused, y_ref) < 1e-2
