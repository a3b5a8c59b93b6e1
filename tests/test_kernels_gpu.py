"""Numerics of every HIP kernel against a plain-PyTorch fp32 reference of the
same op (run on the MI355X box: ``pytest -m gpu``)."""
import math

import pytest
import torch
import torch.nn.functional as F

from chiaswarm_amd import ops
from chiaswarm_amd.ops import hip_ops
from chiaswarm_amd.schedulers import StepCoeffs

pytestmark = pytest.mark.gpu


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / (ref.norm() + 1e-12)).item()


def rnd(*shape, dev, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*shape, device=dev) * scale).to(dtype)


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (1000, 320, 320), (77 * 8, 1024, 1024), (8, 1280, 320),
                                   (4096 * 2, 640, 1280), (130, 48, 40), (33, 4, 16), (512, 2560, 640)])
@pytest.mark.parametrize("act", [None, "gelu", "silu"])
def test_gemm(gpu, M, N, K, act):
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    r = rnd(M, N, dev=gpu)
    y = hip_ops.gemm(a, w, b, r, act)
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), act)
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("tile", [1, 2, 3, 4, 5, 6, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 25, 26, 27, 28, 29, 36])
@pytest.mark.parametrize("split", [1, 3, 13])  # 13: 10 / 7 effective splits (8+1+1 / 4+1+1+1 load batches)
def test_gemm_conv_every_tile_and_splitk(gpu, tile, split):
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.ops.hip_ops import _p, _s

    M, N, K = 200, 96, 640
    a, w, b, r = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu), rnd(M, N, dev=gpu)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    ws = torch.empty(split * M * N, dtype=torch.float32, device=gpu)
    _lib.call("csk_gemm", _p(out), _p(a), _p(w), _p(b), None, _p(r), M, N, K, K, K, N, N, 1, 2, 1.0, None, tile, split,
              _p(ws), _s())
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), "silu")
    assert rel_err(out.cpu(), ref) < 1e-2
    # implicit-GEMM conv, K split across taps
    B, H, W, Cin, Cout = 2, 10, 12, 96, 48
    x = rnd(B, H, W, Cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
    b2 = rnd(B, Cout, dev=gpu)
    y = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device=gpu)
    ws = torch.empty(split * B * H * W * Cout, dtype=torch.float32, device=gpu)
    _lib.call("csk_conv2d", _p(y), _p(x), _p(wp), None, _p(b2), None, B, H, W, Cin, Cout, 3, 3, 1, 1, 1, H, W, 0,
              Cin, Cout, 0, 0, 1.0, 1, None, tile, split, _p(ws), _s())
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), None, 1, 1, None, False, b2.float().cpu())
    assert rel_err(y.cpu(), ref) < 1e-2


def test_gemm_strided_a_and_geglu(gpu):
    M, K, F_ = 300, 320, 1280
    big = rnd(M, 3 * K, dev=gpu)
    a = big[:, K:2 * K]  # row stride 3K
    w, b = rnd(2 * F_, K, dev=gpu, scale=K ** -0.5), rnd(2 * F_, dev=gpu)
    wp, bp = ops.pack_geglu(w, b)
    y = hip_ops.gemm(a, wp, bp, None, "geglu")
    h, g = (a.float() @ w.float().t() + b.float()).chunk(2, dim=-1)
    ref = h * F.gelu(g)
    assert y.shape == (M, F_)
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("tile", [1, 3, 11, 12, 13, 14, 15, 17, 18, 19, 20, 25, 26, 27, 28, 29, 36])
def test_geglu_every_tile(gpu, tile):
    """GEGLU pairs (hidden, gate) 16-column tiles inside each wave's columns: every
    tile must produce the same gated output."""
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.ops.hip_ops import _p, _s

    M, K, F_ = 333, 320, 640
    a = rnd(M, K, dev=gpu)
    w, b = rnd(2 * F_, K, dev=gpu, scale=K ** -0.5), rnd(2 * F_, dev=gpu)
    wp, bp = ops.pack_geglu(w, b)
    y = torch.empty(M, F_, dtype=torch.bfloat16, device=gpu)
    _lib.call("csk_gemm", _p(y), _p(a), _p(wp), _p(bp), None, None, M, 2 * F_, K, K, K, F_, F_, 1, 3, 1.0, None,
              tile, 1, None, _s())
    h, g = (a.float() @ w.float().t() + b.float()).chunk(2, dim=-1)
    assert rel_err(y, h * F.gelu(g)) < 1e-2


@pytest.mark.parametrize("B,H,W,Cin,Cout,k,stride,pad,up", [
    (2, 16, 16, 320, 320, 3, 1, 1, False), (2, 16, 16, 64, 128, 3, 2, 1, False), (1, 8, 8, 128, 64, 3, 1, 1, True),
    (2, 9, 7, 32, 32, 3, 1, 1, False), (1, 16, 16, 4, 320, 3, 1, 1, False), (1, 16, 16, 320, 4, 3, 1, 1, False),
    (1, 16, 16, 64, 64, 3, 2, (0, 0, 1, 1), False), (2, 8, 8, 96, 32, 3, 1, 1, False), (1, 12, 12, 3, 64, 3, 1, 1, False),
    (2, 32, 32, 960, 640, 3, 1, 1, False)])
def test_conv2d(gpu, B, H, W, Cin, Cout, k, stride, pad, up):
    x = rnd(B, H, W, Cin, dev=gpu)
    wt = rnd(Cout, Cin, k, k, dev=gpu, scale=(Cin * k * k) ** -0.5)
    wp = ops.pack_conv_weight(wt)
    bias = rnd(Cout, dev=gpu)
    Ho, Wo = ops.conv_out_size(H, W, k, k, stride, pad, up)
    res = rnd(B, Ho, Wo, Cout, dev=gpu)
    b2 = rnd(B, Cout, dev=gpu)
    y = hip_ops.conv2d(x, wp, bias, stride, pad, res, up, b2)
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), bias.float().cpu(), stride, pad, res.float().cpu(), up,
                          b2.float().cpu())
    assert y.shape == ref.shape
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("shape,G,silu", [((2, 16, 16, 320), 32, True), ((2, 64, 64, 128), 32, False),
                                          ((2, 8, 8, 2560), 32, True), ((1, 32, 32, 1920), 32, True),
                                          ((3, 77, 640), 32, False), ((1, 128, 128, 256), 32, True),
                                          # Cg = 5 (an 8-channel vector spans 3 groups), 6, 7
                                          ((2, 16, 16, 160), 32, True), ((1, 8, 8, 320), 64, False),
                                          ((1, 8, 8, 192), 32, True), ((1, 8, 8, 224), 32, False)])
def test_group_norm(gpu, shape, G, silu):
    x = rnd(*shape, dev=gpu, scale=3.0) + 2.0
    g, b = rnd(shape[-1], dev=gpu), rnd(shape[-1], dev=gpu)
    y = hip_ops.group_norm(x, g, b, G, 1e-5, silu)
    ref = ops._ref_group_norm(x.float().cpu(), g.float().cpu(), b.float().cpu(), G, 1e-5, silu)
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("shape,G", [((2, 32, 32, 384), 12), ((3, 16, 16, 768), 24), ((2, 8, 8, 64), 8)])
@pytest.mark.parametrize("act", [None, "gelu"])
def test_group_norm_adaptive_strided_affine(gpu, shape, G, act):
    """AdaGroupNorm (K-UNet): per-sample affine taken in place from row slices
    of one wider batched projection [B, sum 2C] (row stride > C), + fused GELU."""
    B, C = shape[0], shape[-1]
    x = rnd(*shape, dev=gpu, scale=2.0) + 1.0
    proj = rnd(B, 3 * C + 40, dev=gpu)
    g, b = proj[:, 40:40 + C], proj[:, 40 + C:40 + 2 * C]
    assert g.stride(0) == 3 * C + 40
    y = hip_ops.group_norm(x, g, b, G, 1e-5, act)
    ref = ops._ref_group_norm(x.float().cpu(), g.float().cpu(), b.float().cpu(), G, 1e-5, act)
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("C", [320, 768, 1024, 1280, 2048])
def test_layer_norm(gpu, C):
    x = rnd(3, 50, C, dev=gpu, scale=2.0) + 1.0
    g, b = rnd(C, dev=gpu), rnd(C, dev=gpu)
    y = hip_ops.layer_norm(x, g, b, 1e-5)
    ref = F.layer_norm(x.float(), (C,), g.float(), b.float(), 1e-5)
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("rows,C", [(32768, 320), (4099, 640), (4101, 512), (5000, 96), (8191, 1280), (77, 1024),
                                    (1001, 768), (333, 2048), (130, 4096), (65, 8), (99, 56)])
def test_layer_norm_multirow(gpu, rows, C):
    """UNet-sized row counts (64/LPR rows per wave, lane groups of LPR per row), incl. ragged tails
    and every vectors-per-lane instantiation."""
    x = rnd(rows, C, dev=gpu, scale=2.0) + 1.0
    g, b = rnd(C, dev=gpu), rnd(C, dev=gpu)
    y = hip_ops.layer_norm(x, g, b, 1e-5)
    ref = F.layer_norm(x.float(), (C,), g.float(), b.float(), 1e-5)
    assert rel_err(y, ref) < 1e-2


def _attn_ref(q, k, v, scale, causal):
    return ops._ref_attention(q.float().cpu(), k.float().cpu(), v.float().cpu(), scale, causal)


@pytest.mark.parametrize("B,Sq,Skv,H,D,causal", [(2, 1024, 1024, 5, 64, False), (2, 4096, 77, 5, 64, False),
                                                  (1, 256, 256, 8, 40, False), (1, 300, 300, 8, 80, False),
                                                  (1, 64, 64, 8, 160, False), (2, 77, 77, 16, 64, True),
                                                  (1, 200, 130, 2, 64, False), (1, 77, 77, 12, 64, True)])
def test_attention(gpu, B, Sq, Skv, H, D, causal):
    q, k, v = (rnd(B, s, H, D, dev=gpu) for s in (Sq, Skv, Skv))
    scale = 1 / math.sqrt(D)
    y = hip_ops.attention(q, k, v, scale, causal)
    assert rel_err(y.cpu(), _attn_ref(q, k, v, scale, causal)) < 1.5e-2


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7, 20])
@pytest.mark.parametrize("B,Sq,Skv,H,D,causal", [(2, 1024, 1024, 5, 64, False), (1, 300, 517, 3, 64, False),
                                                  (1, 333, 333, 2, 40, True), (2, 4096, 77, 5, 64, False)])
def test_attention_variants(gpu, variant, B, Sq, Skv, H, D, causal):
    q, k, v = (rnd(B, s, H, D, dev=gpu) for s in (Sq, Skv, Skv))
    old = hip_ops.ATTN_VARIANT
    hip_ops.ATTN_VARIANT = variant
    try:
        y = hip_ops.attention(q, k, v, 1 / math.sqrt(D), causal)
    finally:
        hip_ops.ATTN_VARIANT = old
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 1 / math.sqrt(D), causal)) < 1.5e-2


@pytest.mark.parametrize("short_kv", [1, 2, 3])
@pytest.mark.parametrize("B,Sq,Skv,H,D", [(2, 4096, 77, 5, 64), (2, 1024, 77, 10, 64), (2, 64, 77, 20, 64),
                                          (1, 300, 128, 3, 64), (1, 1000, 1, 2, 64), (2, 333, 77, 8, 40),
                                          (1, 70, 17, 4, 64)])
def test_attention_short_kv_kernels(gpu, short_kv, B, Sq, Skv, H, D):
    """Cross-attention shapes (Skv <= 128): the K/V-resident one-pass kernel (3)
    and the earlier plain (1) / pipelined (2) choices, incl. ragged query tails,
    a single key, head dim 40 and fused-projection (strided) K / V."""
    q = rnd(B, Sq, H, D, dev=gpu)
    kv = rnd(B, Skv, 2, H, D, dev=gpu, scale=2.0)
    k, v = kv[:, :, 0], kv[:, :, 1]
    _lib_call = __import__("chiaswarm_amd.ops._lib", fromlist=["call"]).call
    _lib_call("csk_set_short_kv_variant", short_kv)
    try:
        y = hip_ops.attention(q, k, v, 1 / math.sqrt(D))
    finally:
        _lib_call("csk_set_short_kv_variant", 3)
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 1 / math.sqrt(D), False)) < 1.5e-2


def test_attention_fused_qkv_strides(gpu):
    B, S, H, D = 2, 333, 10, 64
    qkv = rnd(B, S, 3, H, D, dev=gpu)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    y = hip_ops.attention(q, k, v, 0.125)
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 0.125, False)) < 1.5e-2


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 20])
def test_attention_spike_rescale(gpu, variant):
    # forces the online-softmax rescale: growing logits appear in later KV blocks,
    # including consecutive blocks (the pipelined kernels issue block kb+1's
    # scores before block kb's rescale decision)
    B, S, H, D = 1, 512, 2, 64
    q, k, v = (rnd(B, S, H, D, dev=gpu) for _ in range(3))
    k[0, 100, 0] = q[0, 5, 0] * 8
    k[0, 130, 0] = q[0, 5, 0] * 12
    k[0, 200, 1] = q[0, 70, 1] * 10
    k[0, 333, 1] = q[0, 70, 1] * 16
    old = hip_ops.ATTN_VARIANT
    hip_ops.ATTN_VARIANT = variant
    try:
        y = hip_ops.attention(q, k, v, 0.125)
    finally:
        hip_ops.ATTN_VARIANT = old
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 0.125, False)) < 1.5e-2


@pytest.mark.parametrize("a32", [1])
@pytest.mark.parametrize("B,Sq,Skv,H,D,causal,spike", [(2, 1024, 1024, 5, 64, False, False),
                                                        (1, 300, 517, 3, 64, False, True),
                                                        (2, 77, 77, 4, 64, True, False)])
def test_attn32_kernel(gpu, a32, B, Sq, Skv, H, D, causal, spike):
    """The 32x32x16 attention kernel (variant 20) against fp32, incl. a causal
    mask and rescale spikes."""
    from chiaswarm_amd.ops import _lib

    q, k, v = (rnd(B, s, H, D, dev=gpu) for s in (Sq, Skv, Skv))
    if spike:
        k[0, 100, 0] = q[0, 5, 0] * 8
        k[0, 260, 1] = q[0, 70, 1] * 14
    old = hip_ops.ATTN_VARIANT
    hip_ops.ATTN_VARIANT = 20
    _lib.call("csk_set_attn32", a32)
    try:
        y = hip_ops.attention(q, k, v, 1 / math.sqrt(D), causal)
    finally:
        _lib.call("csk_set_attn32", 1)
        hip_ops.ATTN_VARIANT = old
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 1 / math.sqrt(D), causal)) < 1.5e-2


@pytest.mark.parametrize("variant", [2, 3, 5, 20])
def test_attention_far_negative_logits(gpu, variant):
    # every score far below 0 (softmax is shift-invariant): the running-max offset
    # must follow the logits down, not start from 0
    B, S, H, D = 1, 300, 1, 64
    u = torch.nn.functional.normalize(torch.randn(D, device=gpu), dim=0)
    q = (u * 40 + 0.3 * torch.randn(B, S, H, D, device=gpu)).bfloat16()
    k = (-u * 40 + 0.3 * torch.randn(B, S, H, D, device=gpu)).bfloat16()
    v = rnd(B, S, H, D, dev=gpu)
    old = hip_ops.ATTN_VARIANT
    hip_ops.ATTN_VARIANT = variant
    try:
        y = hip_ops.attention(q, k, v, 0.125)
    finally:
        hip_ops.ATTN_VARIANT = old
    assert torch.isfinite(y.float()).all()
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 0.125, False)) < 1.5e-2


def test_attention_vae_d512(gpu):
    q, k, v = (rnd(2, 256, 1, 512, dev=gpu) for _ in range(3))
    y = hip_ops.attention(q, k, v, 512 ** -0.5)
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 512 ** -0.5, False)) < 1.5e-2


def test_elementwise(gpu):
    x, y = rnd(4, 64, 64, 8, dev=gpu), rnd(4, 64, 64, 8, dev=gpu)
    assert rel_err(hip_ops.silu(x), F.silu(x.float())) < 1e-2
    assert rel_err(hip_ops.add(x, y), x.float() + y.float()) < 1e-2
    img = rnd(2, 32, 32, 3, dev=gpu, scale=0.8)
    u8 = hip_ops.vae_postprocess(img)
    ref = ((img.float() / 2 + 0.5).clamp(0, 1) * 255).round().to(torch.uint8)
    assert (u8.int() - ref.int()).abs().max().item() <= 1


@pytest.mark.parametrize("cfg,prev,noise", [(True, True, False), (False, False, True), (True, False, False)])
def test_sched_step(gpu, cfg, prev, noise):
    n = 2 * 64 * 64 * 4
    x = torch.randn(2, 64, 64, 4, device=gpu)
    e = rnd(2 * (2 if cfg else 1), 64, 64, 4, dev=gpu)
    x0p = torch.randn_like(x) if prev else None
    nz = torch.randn_like(x) if noise else None
    c = StepCoeffs(1.3, -0.7, 0.9, 0.2, 0.05 if prev else 0.0, 0.3 if noise else 0.0)
    g = 7.5 if cfg else None
    out, x0 = hip_ops.sched_step(e, x, x0p, c, g, nz)
    ro, rx0 = ops._ref_sched_step(e, x, x0p, c, g, nz)
    assert rel_err(out, ro) < 1e-5 and rel_err(x0, rx0) < 1e-5
    assert n == x.numel()


@pytest.mark.parametrize("tile", [25, 26, 36])
def test_big_tiles_many_tiles_per_workgroup_grid(gpu, tile):
    """The 256x160 / 128x160 / 64x160 tiles on a 64x64-level shape (GEMM and conv)."""
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.ops.hip_ops import _p, _s

    M, N, K = 32768, 320, 320
    a, w, b, r = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu), rnd(M, N, dev=gpu)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    _lib.call("csk_gemm", _p(out), _p(a), _p(w), _p(b), None, _p(r), M, N, K, K, K, N, N, 1, 2, 1.0, None, tile, 1,
              None, _s())
    ref = ops._ref_gemm(a.float(), w.float(), b.float(), r.float(), "silu")
    assert rel_err(out, ref) < 1e-2
    B, H, W, Cin, Cout = 8, 64, 64, 128, 192
    x = rnd(B, H, W, Cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
    y = torch.empty(B, H, W, Cout, dtype=torch.bfloat16, device=gpu)
    _lib.call("csk_conv2d", _p(y), _p(x), _p(wp), None, None, None, B, H, W, Cin, Cout, 3, 3, 1, 1, 1, H, W, 0,
              Cin, Cout, 0, 0, 1.0, 1, None, tile, 1, None, _s())
    refc = ops._ref_conv2d(x.float(), wp.float(), None, 1, 1, None, False, None)
    assert rel_err(y, refc) < 1e-2


@pytest.mark.parametrize("tile", [1, 2, 4, 11, 12, 14, 16, 17, 25, 26, 27, 28, 29, 36])
def test_fused_group_norm_stats(gpu, tile):
    """GroupNorm fed by conv-epilogue statistics == GroupNorm with its own stats pass."""
    from chiaswarm_amd.ops import tuning

    B, H, W, Cin, Cout = 2, 16, 16, 64, 320
    x = rnd(B, H, W, Cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
    res = rnd(B, H, W, Cout, dev=gpu) + 1.0
    g, b = rnd(Cout, dev=gpu), rnd(Cout, dev=gpu)
    key = f"c:{B}:{H}:{W}:{Cin}:{Cout}:3:1:0"
    t = tuning.table()
    old = t.get(key)
    t[key] = [tile, 1, 0.0]
    try:
        y = hip_ops.conv2d(x, wp, None, 1, 1, res, False, None, gn_stats=True)
    finally:
        if old is None:
            t.pop(key, None)
        else:
            t[key] = old
    assert getattr(y, "_csk_gn", None) is not None
    fused = hip_ops.group_norm(y, g, b, 32, 1e-5, True)
    plain = hip_ops.group_norm(y.clone(), g, b, 32, 1e-5, True)
    ref = ops._ref_group_norm(y.float().cpu(), g.float().cpu(), b.float().cpu(), 32, 1e-5, True)
    assert rel_err(fused.cpu(), ref) < 1e-2
    assert rel_err(fused, plain) < 1e-2
    # channel concat keeps the statistics (UNet skip connections)
    y2 = hip_ops.conv2d(x, wp, None, 1, 1, None, False, None, gn_stats=True)
    cat = ops.cat_channels(y, y2)
    if getattr(y2, "_csk_gn", (None, -1))[1] == y._csk_gn[1]:
        assert getattr(cat, "_csk_gn", None) is not None
    g2, b2 = rnd(2 * Cout, dev=gpu), rnd(2 * Cout, dev=gpu)
    yc = hip_ops.group_norm(cat, g2, b2, 32, 1e-5, False)
    refc = ops._ref_group_norm(cat.float().cpu(), g2.float().cpu(), b2.float().cpu(), 32, 1e-5, False)
    assert rel_err(yc.cpu(), refc) < 1e-2


@pytest.mark.parametrize("cbwg,mult", [(512, 1), (64, 1), (0, 1), (512, 2), (512, 4)])
@pytest.mark.parametrize("H,Cin,C", [(64, 64, 320), (32, 64, 640), (16, 128, 960), (8, 128, 2560)])
def test_group_norm_channel_blocked_apply(gpu, cbwg, mult, H, Cin, C):
    """norm.hip gn_apply_cb_kernel: each workgroup merges its own <= 4 groups'
    epilogue partials (no finalize launch); == the fp32 reference GN, for the
    UNet's group widths (10, 20, 30, 80 channels), plain and concat inputs."""
    from chiaswarm_amd.ops import _lib

    x = rnd(2, H, H, Cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(C, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
    g, b = rnd(C, dev=gpu), rnd(C, dev=gpu)
    try:
        _lib.call("csk_set_gn_cb", cbwg)
        _lib.call("csk_set_gn_cb_mult", mult)
        y = hip_ops.conv2d(x, wp, None, 1, 1, None, False, None, gn_stats=True)
        assert getattr(y, "_csk_gn", None) is not None
        out = hip_ops.group_norm(y, g, b, 32, 1e-5, True)
        ref = ops._ref_group_norm(y.float().cpu(), g.float().cpu(), b.float().cpu(), 32, 1e-5, True)
        assert rel_err(out.cpu(), ref) < 1e-2
        # per-sample affine rows (the ResNet time-embedding path uses [B, C])
        g2, b2 = rnd(2, C, dev=gpu), rnd(2, C, dev=gpu)
        out2 = hip_ops.group_norm(y, g2, b2, 32, 1e-5, False)
        for i in range(2):
            r = ops._ref_group_norm(y[i:i + 1].float().cpu(), g2[i].float().cpu(), b2[i].float().cpu(), 32, 1e-5,
                                    False)
            assert rel_err(out2[i:i + 1].cpu(), r) < 1e-2
        # concat [y | y'] with both producers' partials read in place
        h = C // 2 if C != 960 else 640
        wa = ops.pack_conv_weight(rnd(h, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
        wb = ops.pack_conv_weight(rnd(C - h, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
        a = hip_ops.conv2d(x, wa, None, 1, 1, None, False, None, gn_stats=True)
        bb = hip_ops.conv2d(x * 0.5 + 1.0, wb, None, 1, 1, None, False, None, gn_stats=True)
        yc = hip_ops.group_norm_cat(a, bb, g, b, 32, 1e-5, True)
        refc = ops._ref_group_norm(torch.cat([a, bb], -1).float().cpu(), g.float().cpu(), b.float().cpu(), 32, 1e-5,
                                   True)
        assert rel_err(yc.cpu(), refc) < 1e-2
    finally:
        _lib.call("csk_set_gn_cb", 512)
        _lib.call("csk_set_gn_cb_mult", 2)  # library default


@pytest.mark.parametrize("H,C", [(256, 128), (256, 256)])
def test_fused_group_norm_stats_large_vae_maps(gpu, H, C):
    """VAE-sized maps: thousands of epilogue partials per group take the
    workgroup-per-group finalize (norm.hip gn_finalize_part_wg_kernel)."""
    x = rnd(1, H, H, C, dev=gpu)
    wp = ops.pack_conv_weight(rnd(C, C, 3, 3, dev=gpu, scale=(9 * C) ** -0.5))
    y = hip_ops.conv2d(x, wp, None, 1, 1, None, False, None, gn_stats=True)
    assert getattr(y, "_csk_gn", None) is not None
    part, seg = y._csk_gn
    assert (H * H // seg) * (C // 32) > 1024  # the large-map finalize path
    g, b = rnd(C, dev=gpu), rnd(C, dev=gpu)
    fused = hip_ops.group_norm(y, g, b, 32, 1e-6, True)
    plain = hip_ops.group_norm(y.clone(), g, b, 32, 1e-6, True)
    ref = ops._ref_group_norm(y.float().cpu(), g.float().cpu(), b.float().cpu(), 32, 1e-6, True)
    assert rel_err(fused.cpu(), ref) < 1e-2
    assert rel_err(fused, plain) < 1e-2


@pytest.mark.parametrize("tile", [1, 11, 14, 26, 31, 32, 33, 34])
@pytest.mark.parametrize("split", [2, 4, 7, 16])  # 7 -> 6, 16 -> 9 effective: 4- and 8-split load batches
def test_fused_group_norm_stats_split_k(gpu, tile, split):
    """Split-K producers emit GN statistics from the reduce kernel
    (splitk_reduce8_gn_kernel, 64-row segments): fused GN == own-stats GN, and
    the partials match the fp32 segment moments of the output."""
    from chiaswarm_amd.ops import tuning

    B, H, W, Cin, Cout = 2, 16, 16, 128, 320
    x = rnd(B, H, W, Cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
    res = rnd(B, H, W, Cout, dev=gpu) + 1.0
    g, b = rnd(Cout, dev=gpu), rnd(Cout, dev=gpu)
    key = f"c:{B}:{H}:{W}:{Cin}:{Cout}:3:1:0"
    t = tuning.table()
    old = t.get(key)
    t[key] = [tile, split, 0.0]
    try:
        y = hip_ops.conv2d(x, wp, None, 1, 1, res, False, None, gn_stats=True)
    finally:
        if old is None:
            t.pop(key, None)
        else:
            t[key] = old
    part, seg = y._csk_gn
    assert seg == hip_ops.SPLITK_GN_SEG
    yv = y.float().reshape(-1, seg, Cout)
    pm = part.view(-1, Cout, 2)
    assert torch.allclose(pm[..., 0], yv.mean(1), atol=2e-2)
    assert rel_err(pm[..., 1], yv.var(1, unbiased=False) * seg) < 2e-2
    fused = hip_ops.group_norm(y, g, b, 32, 1e-5, True)
    ref = ops._ref_group_norm(y.float().cpu(), g.float().cpu(), b.float().cpu(), 32, 1e-5, True)
    assert rel_err(fused.cpu(), ref) < 1e-2


@pytest.mark.parametrize("size", [(512, 512), (97, 131)])
def test_canny_matches_numpy(gpu, size):
    import numpy as np

    from chiaswarm_amd.controlnet.preprocess import canny_np

    rng = np.random.default_rng(0)
    H, W = size
    yy, xx = np.mgrid[0:H, 0:W]
    img = (127 + 100 * np.sin(xx / 9.0) * np.cos(yy / 13.0) + rng.normal(0, 8, (H, W))).clip(0, 255).astype(np.uint8)
    ref = canny_np(img, 100.0, 200.0)
    got = hip_ops.canny(torch.from_numpy(img).to(gpu), 100.0, 200.0).cpu().numpy()
    # direction quantisation at exact 22.5-degree boundaries may differ (f32 atan2 vs f64)
    assert (got != ref).mean() < 2e-3
    # RGB input (the reference runs cv2.Canny on the RGB array): per-pixel max-gradient channel
    rgb = np.stack([img, np.roll(img, 7, axis=1), (255 - img) // 2], axis=-1).copy()
    ref3 = canny_np(rgb, 100.0, 200.0)
    got3 = hip_ops.canny(torch.from_numpy(rgb).to(gpu), 100.0, 200.0).cpu().numpy()
    assert (got3 != ref3).mean() < 2e-3 and (ref3 != ref).mean() > 1e-3


def test_timestep_embedding_kernel(gpu):
    from chiaswarm_amd.models.layers import timestep_embedding

    for t in (torch.tensor([999.0], device=gpu), torch.tensor([0.0, 1.5, 500.25, 981.0], device=gpu)):
        y = hip_ops.timestep_embedding(t, 4, 320)
        ref = timestep_embedding(t.expand(4) if t.numel() == 1 else t, 320)
        assert y.shape == (4, 320) and y.dtype == torch.bfloat16
        assert (y.float() - ref).abs().max().item() < 1e-2


def test_conv_bias2d_row_stride(gpu):
    """A column slice of the batched time-embedding GEMM as per-sample conv bias (no copy)."""
    B, H, W, Cin, Cout = 2, 8, 8, 64, 96
    x = rnd(B, H, W, Cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
    big = rnd(B, 3 * Cout, dev=gpu)
    b2 = big[:, Cout:2 * Cout]
    y = hip_ops.conv2d(x, wp, None, 1, 1, None, False, b2)
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), None, 1, 1, None, False, b2.float().cpu())
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("ink", [1, 0])
@pytest.mark.parametrize("N,act", [(960, None), (320, None), (2 * 1280, "geglu")])
@pytest.mark.parametrize("tile", [None, 11, 13, 14, 19, 20, 25, 26, 27, 29, 31, 32, 33, 34, 36])
def test_layer_norm_fused_into_gemm(gpu, N, act, tile, ink, monkeypatch):
    """Producer GEMM emits per-row statistics; the consumer GEMM applies the
    LayerNorm in its epilogue with gamma/beta folded into its weights.
    ``tile`` forces producer and consumer onto one tile: the row-layout direct
    epilogue (glds tiles) and the LDS epilogue (heuristic tiles)
    both.  ``ink``: the consumer merges the producer's row partials in its own
    prologue (1, LDS-DMA tiles) or reads them from the merge kernel (0)."""
    from types import SimpleNamespace

    from chiaswarm_amd.ops import _lib, tuning

    monkeypatch.setattr(ops, "LN_FUSE", True)
    _lib.call("csk_set_ln_in_kernel", ink)
    try:
        _ln_fused_case(gpu, N, act, tile, monkeypatch, tuning)
    finally:
        _lib.call("csk_set_ln_in_kernel", 1)


def _ln_fused_case(gpu, N, act, tile, monkeypatch, tuning):
    from types import SimpleNamespace

    M, C, Kp = 1000, 320, 640
    if tile is not None:
        t = tuning.table()
        for key in (f"g:{M}:{C}:{Kp}:0", f"g:{M}:{N}:{C}:{3 if act == 'geglu' else 0}"):
            monkeypatch.setitem(t, key, [tile, 1, 0.0])
    a = rnd(M, Kp, dev=gpu)
    wp_, res = rnd(C, Kp, dev=gpu, scale=Kp ** -0.5), rnd(M, C, dev=gpu, scale=3.0) + 1.5
    x = ops.gemm(a, wp_, None, residual=res, row_stats=True)  # residual stream with an offset
    xr = ops._ref_gemm(a.float().cpu(), wp_.float().cpu(), None, res.float().cpu(), None)
    assert rel_err(x.cpu(), xr) < 1e-2
    assert getattr(x, "_csk_rows", None) is not None
    norm = SimpleNamespace(weight=rnd(C, dev=gpu) + 1.0, bias=rnd(C, dev=gpu), eps=1e-5)
    w, b = rnd(N, C, dev=gpu, scale=C ** -0.5), rnd(N, dev=gpu)
    if act == "geglu":
        w, b = ops.pack_geglu(w, b)
    y = ops.layer_norm_gemm(x, norm, w, b, ops.fold_layer_norm(w, b, norm.weight, norm.bias), act=act)
    xn = F.layer_norm(x.float(), (C,), norm.weight.float(), norm.bias.float(), 1e-5)
    ref = ops._ref_gemm(xn.cpu(), w.float().cpu(), b.float().cpu(), None, act)
    assert y.shape == ref.shape
    assert rel_err(y.cpu(), ref) < 1.5e-2


def test_group_norm_of_concat_in_place(gpu):
    """GroupNorm of [a | b] read from the two tensors (UNet skip concat) == GN of torch.cat."""
    B, H, W, Ca, Cb, K = 2, 32, 32, 320, 320, 256
    xa, xb = rnd(B, H, W, K, dev=gpu), rnd(B, H, W, K, dev=gpu)
    wa, wb = rnd(Ca, K, dev=gpu, scale=K ** -0.5), rnd(Cb, K, dev=gpu, scale=K ** -0.5)
    a = ops.gemm(xa, wa, gn_rows=H * W)  # producers emit fused GN statistics
    b = ops.gemm(xb, wb, gn_rows=H * W)
    assert getattr(a, "_csk_gn", None) is not None and getattr(b, "_csk_gn", None) is not None
    g, bt = rnd(Ca + Cb, dev=gpu), rnd(Ca + Cb, dev=gpu)
    y = hip_ops.group_norm_cat(a, b, g, bt, 32, 1e-5, True)
    if y is None:
        pytest.skip("segment heights differ")
    ref = ops._ref_group_norm(torch.cat([a, b], -1).float().cpu(), g.float().cpu(), bt.float().cpu(), 32, 1e-5, True)
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("Ca,Cb", [(640, 320), (1280, 1280)])
def test_group_norm_of_concat_without_fused_stats(gpu, Ca, Cb):
    """Concat inputs without epilogue statistics (split-K producers): the
    statistics pass reads both tensors in place too."""
    a, b = rnd(2, 16, 16, Ca, dev=gpu, scale=2.0) + 1.0, rnd(2, 16, 16, Cb, dev=gpu)
    g, bt = rnd(Ca + Cb, dev=gpu), rnd(Ca + Cb, dev=gpu)
    y = hip_ops.group_norm_cat(a, b, g, bt, 32, 1e-5, True)
    ref = ops._ref_group_norm(torch.cat([a, b], -1).float().cpu(), g.float().cpu(), bt.float().cpu(), 32, 1e-5, True)
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("tile", [31, 32, 33, 34])
@pytest.mark.parametrize("split", [1, 3])
def test_phased_256_tiles_gemm_conv(gpu, tile, split):
    """8-wave 256-row phased kernels (gemm8p.hip): ragged M / N edges, split-K,
    and the implicit-GEMM conv FAST staging (stride 1 / 2, fused nearest-x2)."""
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.ops.hip_ops import _p, _s

    M, N, K = 600, 320, 640  # M and N not multiples of the tile
    a, w, b, r = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu), rnd(M, N, dev=gpu)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    ws = torch.empty(split * M * N, dtype=torch.float32, device=gpu)
    _lib.call("csk_gemm", _p(out), _p(a), _p(w), _p(b), None, _p(r), M, N, K, K, K, N, N, 1, 2, 1.0, None, tile, split,
              _p(ws), _s())
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), "silu")
    assert rel_err(out.cpu(), ref) < 1e-2
    for (B, H, W, Cin, Cout, stride, up) in ((2, 20, 24, 128, 192, 1, 0), (2, 17, 16, 64, 320, 2, 0),
                                             (1, 9, 12, 128, 64, 1, 1)):
        x = rnd(B, H, W, Cin, dev=gpu)
        wp = ops.pack_conv_weight(rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5))
        b2 = rnd(B, Cout, dev=gpu)
        Ho, Wo = ops.conv_out_size(H, W, 3, 3, stride, 1, bool(up))
        y = torch.empty(B, Ho, Wo, Cout, dtype=torch.bfloat16, device=gpu)
        ws = torch.empty(split * B * Ho * Wo * Cout, dtype=torch.float32, device=gpu)
        _lib.call("csk_conv2d", _p(y), _p(x), _p(wp), None, _p(b2), None, B, H, W, Cin, Cout, 3, 3, stride, 1, 1, Ho,
                  Wo, up, Cin, Cout, 0, 0, 1.0, 1, None, tile, split, _p(ws), _s())
        ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), None, stride, 1, None, bool(up), b2.float().cpu())
        assert rel_err(y.cpu(), ref) < 1e-2, (B, H, W, Cin, Cout, stride, up)


@pytest.mark.parametrize("tile", [31, 32, 33, 34])
def test_phased_256_tiles_geglu_and_gn_stats(gpu, tile):
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.ops.hip_ops import _p, _s

    M, K, F_ = 700, 320, 640
    a = rnd(M, K, dev=gpu)
    w, b = rnd(2 * F_, K, dev=gpu, scale=K ** -0.5), rnd(2 * F_, dev=gpu)
    wp, bp = ops.pack_geglu(w, b)
    y = torch.empty(M, F_, dtype=torch.bfloat16, device=gpu)
    _lib.call("csk_gemm", _p(y), _p(a), _p(wp), _p(bp), None, None, M, 2 * F_, K, K, K, F_, F_, 1, 3, 1.0, None,
              tile, 1, None, _s())
    h, g = (a.float() @ w.float().t() + b.float()).chunk(2, dim=-1)
    assert rel_err(y, h * F.gelu(g)) < 1e-2
    # conv producing fused GroupNorm statistics of its output (64x64 UNet level shape, small batch)
    from chiaswarm_amd.ops import tuning

    x = rnd(2, 32, 32, 128, dev=gpu)
    wt = rnd(256, 128, 3, 3, dev=gpu, scale=(9 * 128) ** -0.5)
    wp = ops.pack_conv_weight(wt)
    key = "c:2:32:32:128:256:3:1:0"
    t = tuning.table()
    old = t.get(key)
    t[key] = [tile, 1, 0.0]
    try:
        yc = hip_ops.conv2d(x, wp, None, 1, 1, None, False, None, gn_stats=True)
        gamma, beta = rnd(256, dev=gpu), rnd(256, dev=gpu)
        gn = hip_ops.group_norm(yc, gamma, beta, 32, 1e-5, silu=True)
    finally:
        if old is None:
            t.pop(key, None)
        else:
            t[key] = old
    ref = F.silu(F.group_norm(yc.float().permute(0, 3, 1, 2), 32, gamma.float(), beta.float(), 1e-5)).permute(0, 2, 3, 1)
    assert rel_err(gn, ref) < 1e-2


def _attn_ref_chunked(q, k, v, scale, chunk=1024):
    """fp32 reference on the GPU, query-chunked (never an S x S matrix of the full size)."""
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))  # [B, H, S, D]
    out = torch.empty_like(qf)
    for s0 in range(0, qf.shape[2], chunk):
        sc = torch.matmul(qf[:, :, s0:s0 + chunk], kf.transpose(-1, -2)) * scale
        out[:, :, s0:s0 + chunk] = torch.matmul(torch.softmax(sc, -1), vf)
    return out.permute(0, 2, 1, 3)


@pytest.mark.parametrize("B,S,H,D", [(1, 4096, 8, 40), (1, 2048, 8, 80), (1, 1024, 8, 160), (2, 4096, 5, 64),
                                     (1, 16384, 1, 64), (1, 16384, 1, 512), (2, 4096, 1, 512), (1, 1000, 1, 512),
                                     (1, 4100, 2, 160)])
def test_attention_head_dims_long_sequences(gpu, B, S, H, D):
    """Every UNet / VAE head dim (SD1.5 40/80/160, SD2/XL 64, VAE 512) up to
    S = 16384 (SD2.1 at 1024^2); the d = 512 flash kernel allocates nothing of
    size S x S (checked with the allocator's peak)."""
    q, k, v = (rnd(B, S, H, D, dev=gpu) for _ in range(3))
    scale = D ** -0.5
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    y = hip_ops.attention(q, k, v, scale)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    split = hip_ops.attn_kv_split(B, H, S, S, D)
    ws = split * B * H * S * 66 * 4 if split > 1 else 0  # split-KV fp32 partials: O(S * D), not S x S
    assert peak <= y.numel() * 2 + ws + (1 << 20), peak  # the output, nothing S x S
    assert rel_err(y, _attn_ref_chunked(q, k, v, scale)) < 1.5e-2


def test_attention_d512_strided_heads(gpu):
    """d = 512 over strided [B, S, H, D] views (fused QKV layout) and a ragged key tail."""
    qkv = rnd(1, 777, 3, 512, dev=gpu)
    q, k, v = qkv[:, :, 0:1], qkv[:, :, 1:2], qkv[:, :, 2:3]
    y = hip_ops.attention(q, k, v, 512 ** -0.5)
    assert rel_err(y, _attn_ref_chunked(q, k, v, 512 ** -0.5)) < 1.5e-2


@pytest.mark.parametrize("tile", [33, 34])
@pytest.mark.parametrize("cin", [64, 32])
def test_ring_256x160_gn_stats_and_fallback(gpu, cin, tile):
    """Tile 33 (8-wave 256x160 ring, 64-row GN segments).  Cin = 32 fails its FAST
    staging condition: the library falls back to tile 26, whose 64-row band
    matches the segment the host sized the statistics buffer for."""
    from chiaswarm_amd.ops import tuning

    B, H, W, Cout = 2, 16, 32, 320
    x = rnd(B, H, W, cin, dev=gpu)
    wp = ops.pack_conv_weight(rnd(Cout, cin, 3, 3, dev=gpu, scale=(9 * cin) ** -0.5))
    res = rnd(B, H, W, Cout, dev=gpu)
    key = f"c:{B}:{H}:{W}:{cin}:{Cout}:3:1:0"
    t = tuning.table()
    old = t.get(key)
    t[key] = [tile, 1, 0.0]
    try:
        y = hip_ops.conv2d(x, wp, None, 1, 1, res, False, None, gn_stats=True)
    finally:
        if old is None:
            t.pop(key, None)
        else:
            t[key] = old
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), None, 1, 1, res.float().cpu(), False, None)
    assert rel_err(y.cpu(), ref) < 1e-2
    part, seg = y._csk_gn
    assert seg == 64
    yf = y.float().reshape(-1, seg, Cout)
    want = torch.stack([yf.mean(1), ((yf - yf.mean(1, keepdim=True)) ** 2).sum(1)], -1)
    got = part.reshape(-1, Cout, 2)
    assert torch.allclose(got[..., 0], want[..., 0], atol=2e-2, rtol=2e-2)
    assert torch.allclose(got[..., 1], want[..., 1], atol=0.5, rtol=2e-2)


def test_debug_build_records_violations(gpu):
    """CSK_DEBUG=1 (libcsk_debug.so): a deliberate violation from the self-test
    kernel lands in the device record with its site / value / limit and is
    cleared on read; release builds export no record at all."""
    from chiaswarm_amd.ops import _lib

    lib = _lib.load()
    if not _lib.DEBUG:
        assert not hasattr(lib, "csk_debug_read_gemm_glds")
        pytest.skip("release build (run with CSK_DEBUG=1 for the debug library)")
    assert _lib.LIB_PATH.endswith("libcsk_debug.so")
    torch.cuda.synchronize()
    assert _lib.debug_records() == []
    _lib.call("csk_debug_selftest", 7, _lib.stream_ptr())
    torch.cuda.synchronize()
    recs = _lib.debug_records()
    assert len(recs) == 1 and recs[0][0] == "gemm_glds", recs
    tu, count, site, bx, tid, val, lim, by = recs[0]
    assert count == 64 and site == 99 and val == 7 and lim == 3, recs  # one wave, every lane fails
    assert _lib.debug_records() == []  # cleared


@pytest.mark.parametrize("shape", [(2, 64, 64, 320), (1, 4096, 320), (3, 5, 8)])
def test_dup2_batch(gpu, shape):
    """[x; x] in one kernel (the CFG-shared UNet prefix duplication)."""
    x = rnd(*shape, dev=gpu)
    y = hip_ops.dup2(x)
    assert y.shape == (2 * shape[0],) + tuple(shape[1:])
    assert torch.equal(y[: shape[0]], x) and torch.equal(y[shape[0]:], x)


def test_row_bcast(gpu):
    """The sampler-loop step graph's gather of its time-projection row."""
    tab = rnd(7, 20160, dev=gpu)
    dst = torch.empty(8, 20160, dtype=torch.bfloat16, device=gpu)
    for i in (0, 3, 6):
        hip_ops.row_bcast(dst, tab, torch.tensor([i], dtype=torch.int32, device=gpu))
        assert torch.equal(dst, tab[i].expand(8, -1))


@pytest.mark.parametrize("B,S,H,split", [(2, 4096, 5, 2), (1, 4096, 5, 4), (2, 1024, 10, 4), (1, 1000, 3, 2),
                                         (1, 700, 2, 4)])
def test_attention_split_kv(gpu, B, S, H, split):
    """Split-KV attn32 (fp32 partials + combine) for small grids, incl. ragged
    key / query tails and splits that get no key block."""
    q, k, v = (rnd(B, S, H, 64, dev=gpu) for _ in range(3))
    y = hip_ops.attention_split(q, k, v, 0.125, split)
    assert rel_err(y.cpu(), _attn_ref(q, k, v, 0.125, False)) < 1.5e-2
    if hip_ops.attn_kv_split(B, H, S, S, 64) > 1:  # the default path takes the split itself
        assert rel_err(hip_ops.attention(q, k, v, 0.125).cpu(), _attn_ref(q, k, v, 0.125, False)) < 1.5e-2


@pytest.mark.parametrize("tile", [1, 4, 31, 32, 33, 34])
def test_profiling_probe_act_rejected_outside_lds_dma_tiles(gpu, tile):
    """act 97-99 (tilebench probes) exist only in the LDS-DMA tiles; any other
    kernel would run them as a plain full-width epilogue (an out-of-bounds write
    into a GEGLU-sized output), so the library refuses them before launching."""
    from chiaswarm_amd.ops import _lib
    from chiaswarm_amd.ops.hip_ops import _p, _s

    M, N, K = 256, 256, 128
    a, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu)
    y = torch.zeros(M, N // 2, dtype=torch.bfloat16, device=gpu)
    with pytest.raises(RuntimeError):
        _lib.call("csk_gemm", _p(y), _p(a), _p(w), None, None, None, M, N, K, K, K, N // 2, N // 2, 1, 99, 1.0, None,
                  tile, 1, None, _s())
    torch.cuda.synchronize()
    assert int(torch.count_nonzero(y)) == 0
