"""Fused transformer input (csrc/kernels/xin.hip; SURVEY K6 + K9 + K11):
GroupNorm apply + proj_in + block 0's LayerNorm1 + QKV projection of an SD
transformer at C = 320 in one kernel.

CPU: the packing round-trips, and the fp32 reference built from the packed
weights equals the module's unfused composition (GroupNorm -> proj_in ->
LayerNorm -> to_q / to_k / to_v).  GPU: the HIP kernel against that fp32
composition (statistics from a producer GEMM's epilogue, as in the UNet), graph
replay, and the whole Transformer2D with the fused path against the unfused
chain."""
import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.models.layers import Transformer2D, init_random_


def _setup(dev, dtype, seed=0, linear=True):
    torch.manual_seed(seed)
    t = Transformer2D(320, 5, 1024, layers=1, linear_proj=linear).to(dev)
    init_random_(t, seed=seed)
    with torch.no_grad():  # non-trivial affines and biases
        t.norm.weight.uniform_(0.5, 1.5)
        t.norm.bias.normal_(0, 0.2)
        t.proj_in.bias.normal_(0, 0.3)
        blk = t.transformer_blocks[0]
        blk.norm1.weight.uniform_(0.5, 1.5)
        blk.norm1.bias.normal_(0, 0.2)
    return t.to(dtype)


def _unfused(x, t):
    """fp32 GroupNorm -> proj_in -> LayerNorm1 -> Wq / Wk / Wv of the module."""
    B, C = x.shape[0], x.shape[-1]
    xf = x.float().reshape(B, -1, C)
    g = torch.nn.functional.group_norm(xf.transpose(1, 2), t.norm.num_groups, t.norm.weight.float(),
                                       t.norm.bias.float(), t.norm.eps).transpose(1, 2)
    wi = t.proj_in.weight.float().reshape(C, C)
    h = g @ wi.t() + t.proj_in.bias.float()
    blk = t.transformer_blocks[0]
    n = torch.nn.functional.layer_norm(h, (C,), blk.norm1.weight.float(), blk.norm1.bias.float(), blk.norm1.eps)
    a1 = blk.attn1
    q, k, v = (n @ m.weight.float().t() for m in (a1.to_q, a1.to_k, a1.to_v))
    return h.reshape(-1, C), torch.cat([q, k, v], -1).reshape(-1, 3 * C)


def _lib_ok(hip_ops, x):
    B, C = x.shape[0], x.shape[-1]
    M = x.numel() // C
    return hip_ops._lib.call_int("csk_xin_qkv_ok", M, C, M // B, 32) == 1


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / ref.norm()).item()


@pytest.mark.parametrize("linear", [True, False])
def test_pack_roundtrip_and_reference_cpu(linear):
    t = _setup("cpu", torch.float32, linear=linear)
    packed = t._xin_weights()
    w, bi, colsum, bq = packed
    assert w.shape == (40, 5, 32, 64) and bi.shape == (320,) and colsum.shape == (960,) and bq.shape == (960,)
    wi, wq = ops.unpack_xin_qkv(w)
    assert torch.equal(wi, t.proj_in.weight.reshape(320, 320))
    blk = t.transformer_blocks[0]
    w2, cs2, _ = blk._fold("qkv", blk.attn1.w_qkv, blk.attn1.b_qkv, blk.norm1)
    assert torch.equal(wq, w2) and torch.equal(colsum, cs2)
    x = torch.randn(2, 8, 8, 320) * 2 + 0.3
    h, qkv = ops._ref_xin_qkv(x, t.norm.weight, t.norm.bias, t.norm.num_groups, t.norm.eps, packed, blk.norm1.eps)
    rh, rq = _unfused(x, t)
    assert torch.allclose(h, rh, atol=1e-4, rtol=1e-4), (h - rh).abs().max()
    assert torch.allclose(qkv, rq, atol=2e-4, rtol=2e-4), (qkv - rq).abs().max()
    assert not t._xin_ok(x)  # CPU: the unfused path


def _producer(x, gpu, seg=64):
    """x with fused GroupNorm statistics attached in the producer-epilogue format
    (gemm_common.h gn_part: per (seg-row segment, channel) (mean, M2)), as the
    ResNet output the UNet hands to a transformer carries them."""
    B, P, C = x.shape
    xs = x.float().reshape(B * P // seg, seg, C)
    mean = xs.mean(1)
    m2 = ((xs - mean[:, None]) ** 2).sum(1)
    x._csk_gn = (torch.stack([mean, m2], -1).reshape(-1).contiguous(), seg)
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("B,P", [(8, 4096), (2, 1024), (1, 256)])
def test_xin_kernel_matches_fp32(gpu, B, P):
    from chiaswarm_amd.ops import hip_ops

    t = _setup(gpu, torch.bfloat16)
    x = _producer((torch.randn(B, P, 320, device=gpu) * 2 + 0.5).bfloat16(), gpu)
    assert _lib_ok(hip_ops, x)
    stat = hip_ops.gn_stats(x, 32, t.norm.eps)
    # the finalized statistics against torch's on the same tensor
    g = x.float().reshape(B, P, 32, 10)
    assert torch.allclose(stat[..., 0], g.mean(dim=(1, 3)), atol=2e-3, rtol=1e-3)
    want_rstd = torch.rsqrt(g.var(dim=(1, 3), unbiased=False) + t.norm.eps)
    assert torch.allclose(stat[..., 1], want_rstd, atol=1e-3, rtol=2e-3)
    w, bi, cs, bq = t._xin_weights()
    h, qkv = hip_ops.xin_qkv(x, stat, t.norm.weight, t.norm.bias, w, bi, cs, bq, t.transformer_blocks[0].norm1.eps)
    torch.cuda.synchronize()
    rh, rq = _unfused(x.cpu().float(), t.cpu().float())
    assert torch.isfinite(h.float()).all() and torch.isfinite(qkv.float()).all()
    assert rel_err(h.cpu(), rh) < 8e-3
    assert rel_err(qkv.cpu(), rq) < 1.2e-2


@pytest.mark.gpu
def test_xin_kernel_deterministic_and_graph_replay(gpu):
    from chiaswarm_amd.ops import hip_ops

    t = _setup(gpu, torch.bfloat16)
    x = _producer(torch.randn(2, 4096, 320, device=gpu).bfloat16(), gpu)
    stat = hip_ops.gn_stats(x, 32, t.norm.eps)
    args = (stat, t.norm.weight, t.norm.bias, *t._xin_weights(), t.transformer_blocks[0].norm1.eps)
    a = hip_ops.xin_qkv(x, *args)
    b = hip_ops.xin_qkv(x, *args)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        hip_ops.xin_qkv(x, *args)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        c = hip_ops.xin_qkv(x, *args)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(c[0], a[0]) and torch.equal(c[1], a[1])


@pytest.mark.gpu
@pytest.mark.parametrize("linear", [True, False])
def test_transformer_with_fused_input_matches_unfused(gpu, monkeypatch, linear):
    """Transformer2D takes the fused input kernel on the 64x64 grid (SD2.x
    linear / SD1.x 1x1-conv proj_in) and agrees with the unfused chain."""
    from chiaswarm_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "XIN_FUSED", True)
    t = _setup(gpu, torch.bfloat16, linear=linear)
    x = _producer((torch.randn(4, 4096, 320, device=gpu) * 1.5).bfloat16(), gpu)
    x4 = x.view(4, 64, 64, 320)
    x4._csk_gn = x._csk_gn
    ctx = torch.randn(4, 77, 1024, device=gpu).bfloat16()
    kvs = [m.context_kv(ctx) for m in t.cross_modules()]
    calls = []
    orig = hip_ops.xin_qkv
    monkeypatch.setattr(hip_ops, "xin_qkv", lambda *a, **k: calls.append(1) or orig(*a, **k))
    y_fused = t(x4, kvs=kvs)
    assert calls == [1]
    monkeypatch.setattr(hip_ops, "XIN_FUSED", False)
    y_ref = t(x4, kvs=kvs)
    assert calls == [1]
    torch.cuda.synchronize()
    assert rel_err(y_fused, y_ref) < 1e-2
