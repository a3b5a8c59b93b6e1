"""The persistent stream-K d = 64 / 40 attention (csrc/kernels/attn_fa.hip) against
the fp32 PyTorch reference: ragged query blocks, every merge shape the
stream-K split can produce (forced with small worker counts: one block cut into
2..many pieces, pieces of 1 tile), strided fused-QKV views, the deferred
rescale (logits far above the lazy reference) and far-negative rows."""
import math
import ctypes

import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.ops import hip_ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _short_kv_too(gpu):
    """Take the kernel down to Skv = 128 (the library default keeps S < 512 on attn32)."""
    from chiaswarm_amd.ops import _lib

    _lib.load().csk_set_attn_fa_min_skv(128)
    yield
    _lib.load().csk_set_attn_fa_min_skv(512)


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / (ref.norm() + 1e-12)).item()


def _ref(q, k, v, scale):
    return ops._ref_attention(q.float().cpu(), k.float().cpu(), v.float().cpu(), scale, False)


def _run(q, k, v, scale, workers=0):
    B, Sq, H, D = q.shape
    assert hip_ops.attn_fa_ok(B, H, Sq, k.shape[1], D)
    old = hip_ops.ATTN_FA_WORKERS
    hip_ops.ATTN_FA_WORKERS = workers
    try:
        return hip_ops.attention(q, k, v, scale)
    finally:
        hip_ops.ATTN_FA_WORKERS = old


@pytest.mark.parametrize("B,Sq,Skv,H", [(2, 1024, 1024, 5), (1, 4096, 4096, 2), (1, 320, 256, 3), (2, 256, 1024, 4),
                                        (1, 128, 128, 1), (3, 640, 192, 2), (1, 1000, 512, 2)])
@pytest.mark.parametrize("workers", [0, 7, 33, 100])
def test_attn_fa_shapes_and_cuts(gpu, B, Sq, Skv, H, workers):
    torch.manual_seed(B * 1000 + Sq + Skv + H + workers)
    q, k, v = (torch.randn(B, s, H, 64, device=gpu).bfloat16() for s in (Sq, Skv, Skv))
    y = _run(q, k, v, 0.125, workers)
    assert torch.isfinite(y.float()).all()
    assert rel_err(y.cpu(), _ref(q, k, v, 0.125)) < 1.5e-2
    assert hip_ops.attn_fa_errors() == 0


@pytest.mark.parametrize("B,Sq,Skv,H", [(2, 1024, 1024, 8), (1, 4096, 4096, 2), (1, 320, 256, 3), (1, 1000, 512, 2)])
@pytest.mark.parametrize("workers", [0, 7, 33])
def test_attn_fa_d40_shapes_and_cuts(gpu, B, Sq, Skv, H, workers):
    """Head dim 40 (SD1.5 / ControlNet 64x64 level) on the zero-padded d = 64 images."""
    torch.manual_seed(B * 1000 + Sq + Skv + H + workers + 40)
    q, k, v = (torch.randn(B, s, H, 40, device=gpu).bfloat16() for s in (Sq, Skv, Skv))
    scale = 40 ** -0.5
    y = _run(q, k, v, scale, workers)
    assert y.shape == (B, Sq, H, 40)
    assert torch.isfinite(y.float()).all()
    assert rel_err(y.cpu(), _ref(q, k, v, scale)) < 1.5e-2
    assert hip_ops.attn_fa_errors() == 0


@pytest.mark.parametrize("workers", [0, 5])
def test_attn_fa_d40_fused_qkv_strides(gpu, workers):
    """SD1.5's fused QKV: [B, S, 3, 8, 40] views (80-byte head offsets), output
    the head offsets are 80 bytes (16-byte aligned, not 128)."""
    B, S, H = 2, 1024, 8
    qkv = torch.randn(B, S, 3, H, 40, device=gpu).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    y = _run(q, k, v, 40 ** -0.5, workers)
    assert rel_err(y.cpu(), _ref(q, k, v, 40 ** -0.5)) < 1.5e-2


@pytest.mark.parametrize("workers", [0, 5])
def test_attn_fa_fused_qkv_strides(gpu, workers):
    B, S, H = 2, 768, 10
    qkv = torch.randn(B, S, 3, H, 64, device=gpu).bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    y = _run(q, k, v, 0.125, workers)
    assert rel_err(y.cpu(), _ref(q, k, v, 0.125)) < 1.5e-2


@pytest.mark.parametrize("workers", [0, 3, 11])
def test_attn_fa_rescale_spikes(gpu, workers):
    # logits of 90-180 (log2 units) in later tiles, above the lazy reference's
    # 64 margin: the deferred rescale of O / l and the subtract path must fire,
    # incl. in consecutive tiles and on both sides of a stream-K cut
    B, S, H = 1, 1024, 2
    torch.manual_seed(7)
    q, k, v = (torch.randn(B, S, H, 64, device=gpu).bfloat16() for _ in range(3))
    k[0, 100, 0] = q[0, 5, 0] * 8
    k[0, 130, 0] = q[0, 5, 0] * 12
    k[0, 700, 0] = q[0, 5, 0] * 16
    k[0, 200, 1] = q[0, 70, 1] * 10
    k[0, 333, 1] = q[0, 70, 1] * 16
    k[0, 1000, 1] = q[0, 300, 1] * 14
    y = _run(q, k, v, 0.125, workers)
    assert torch.isfinite(y.float()).all()
    assert rel_err(y.cpu(), _ref(q, k, v, 0.125)) < 1.5e-2


@pytest.mark.parametrize("workers", [0, 4])
def test_attn_fa_far_negative_logits(gpu, workers):
    # every score near -290 (log2 units): the first tile moves the reference down
    B, S, H, D = 1, 384, 1, 64
    u = torch.nn.functional.normalize(torch.randn(D, device=gpu), dim=0)
    q = (u * 40 + 0.3 * torch.randn(B, S, H, D, device=gpu)).bfloat16()
    k = (-u * 40 + 0.3 * torch.randn(B, S, H, D, device=gpu)).bfloat16()
    v = torch.randn(B, S, H, D, device=gpu).bfloat16()
    y = _run(q, k, v, 0.125, workers)
    assert torch.isfinite(y.float()).all()
    assert rel_err(y.cpu(), _ref(q, k, v, 0.125)) < 1.5e-2


def test_attn_fa_repeat_is_deterministic(gpu):
    # the merge order is fixed (owner + its contributors in worker order): two
    # launches give identical bits; flags are reset by their consumers
    q, k, v = (torch.randn(2, 1024, 5, 64, device=gpu).bfloat16() for _ in range(3))
    a = _run(q, k, v, 0.125, 37)
    b = _run(q, k, v, 0.125, 37)
    assert torch.equal(a, b)
    assert hip_ops.attn_fa_errors() == 0


def test_attn_fa_graph_replay(gpu):
    q, k, v = (torch.randn(2, 1024, 5, 64, device=gpu).bfloat16() for _ in range(3))
    ref = _run(q, k, v, 0.125)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        _run(q, k, v, 0.125)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = _run(q, k, v, 0.125)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_attn_fa_timeout_disables_kernel_and_fails_job(gpu):
    """A merge spin that gave up (simulated: csk_attn_fa_inject_errors) turns the
    kernel off for the process, zeroes its flags and fails the job through
    the device wrapper (a stale flag must never be merged later)."""
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.runtime.device import Device

    q, k, v = (torch.randn(1, 1024, 2, 64, device=gpu).bfloat16() for _ in range(3))
    assert hip_ops.attn_fa_ok(1, 2, 1024, 1024, 64)
    assert hip_ops.attn_fa_health()
    lib = _lib.load()
    try:
        assert lib.csk_attn_fa_inject_errors(ctypes.c_uint(3)) == 0
        dev = Device(0)
        with pytest.raises(RuntimeError, match="persistent attention"):
            dev(lambda ident, name, **kw: ({}, {}), model_name="x", seed=1)
        assert not hip_ops.attn_fa_ok(1, 2, 1024, 1024, 64)
        assert hip_ops.attn_fa_errors() == 0
        y = hip_ops.attention(q, k, v, 0.125)  # the fallback kernel serves the shape
        assert rel_err(y.cpu(), _ref(q, k, v, 0.125)) < 1.5e-2
    finally:
        hip_ops.set_attn_fa(True)
    assert hip_ops.attn_fa_ok(1, 2, 1024, 1024, 64)
