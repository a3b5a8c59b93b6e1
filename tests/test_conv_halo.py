"""Halo-tiled 3x3 conv with the input GroupNorm(+SiLU) applied in its LDS halo
(csrc/kernels/conv_halo.hip; SURVEY K1 + K6) against plain-PyTorch fp32
references: the conv alone (bias, per-sample bias, residual), the fused
GroupNorm + SiLU prologue fed by a producer's epilogue statistics, the channel
concat [a | b] input of the up-block ResNets, the statistics it emits for the
next GroupNorm, and whole ResNet blocks on the halo path."""
import copy

import pytest
import torch
import torch.nn.functional as F

from chiaswarm_amd import ops

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _halo_on(monkeypatch):
    """The path is off by default (measured slower, ops/hip_ops.py CONV_HALO):
    the numerics tests switch it on."""
    from chiaswarm_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "CONV_HALO", True)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def rnd(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def ref_conv(x, w, bias=None, bias2d=None, residual=None):
    y = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, padding=1).permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    if bias2d is not None:
        y = y + bias2d.float()[:, None, None, :]
    if residual is not None:
        y = y + residual.float()
    return y


def ref_gn_silu(x, gamma, beta, groups, eps):
    xf = x.float().permute(0, 3, 1, 2)
    return F.silu(F.group_norm(xf, groups, gamma.float(), beta.float(), eps)).permute(0, 2, 3, 1)


def with_stats(x_src, dev):
    """x produced by a HIP conv with fused GroupNorm statistics (x._csk_gn)."""
    from chiaswarm_amd.ops import hip_ops

    B, H, W, C = x_src.shape
    w = ops.pack_conv_weight(rnd(C, C, 3, 3, dev=dev, scale=(9 * C) ** -0.5))
    y = hip_ops.conv2d(x_src, w, rnd(C, dev=dev), 1, 1, None, False, None, gn_stats=True)
    assert getattr(y, "_csk_gn", None) is not None
    return y


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 64, 64, 320, 320), (2, 32, 32, 640, 640), (2, 16, 16, 1280, 1280),
                                            (1, 32, 32, 320, 640), (2, 16, 16, 640, 1280)])
def test_conv_halo_plain(gpu, B, H, W, Cin, Cout):
    from chiaswarm_amd.ops import hip_ops

    x = rnd(B, H, W, Cin, dev=gpu)
    wt = rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5)
    wp = ops.pack_conv_weight(wt)
    bias, b2, res = rnd(Cout, dev=gpu), rnd(B, Cout, dev=gpu), rnd(B, H, W, Cout, dev=gpu)
    assert hip_ops.conv_halo_ok(x, wp)
    y = hip_ops.conv_halo(x, wp, bias, bias2d=b2, residual=res)
    ref = ref_conv(x.cpu(), wt.cpu(), bias.cpu(), b2.cpu(), res.cpu())
    assert rel(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("B,H,W,C,Cout", [(2, 64, 64, 320, 320), (2, 32, 32, 640, 640), (2, 16, 16, 1280, 1280)])
def test_conv_halo_group_norm_silu_prologue(gpu, B, H, W, C, Cout):
    from chiaswarm_amd.ops import hip_ops

    x = with_stats(rnd(B, H, W, C, dev=gpu, scale=2.0), gpu)
    gamma, beta = rnd(C, dev=gpu), rnd(C, dev=gpu)
    stat = hip_ops.gn_finalize(x, 32, 1e-5)
    xf = x.float().view(B, -1, 32, C // 32)
    mean = xf.mean((1, 3))
    var = xf.var((1, 3), unbiased=False)
    assert torch.allclose(stat[..., 0], mean, atol=1e-3, rtol=1e-3)
    assert torch.allclose(stat[..., 1], torch.rsqrt(var + 1e-5), rtol=2e-3)
    wt = rnd(Cout, C, 3, 3, dev=gpu, scale=(9 * C) ** -0.5)
    bias = rnd(Cout, dev=gpu)
    y = hip_ops.conv_halo(x, ops.pack_conv_weight(wt), bias, gn=(stat, gamma, beta, 32, True))
    ref = ref_conv(ref_gn_silu(x.cpu(), gamma.cpu(), beta.cpu(), 32, 1e-5), wt.cpu(), bias.cpu())
    assert rel(y.cpu(), ref) < 1e-2
    # the statistics it emits describe y for the next GroupNorm
    st2 = hip_ops.gn_finalize(y, 32, 1e-5)
    yf = y.float().view(B, -1, 32, Cout // 32)
    assert torch.allclose(st2[..., 0], yf.mean((1, 3)), atol=2e-3, rtol=2e-3)
    assert torch.allclose(st2[..., 1], torch.rsqrt(yf.var((1, 3), unbiased=False) + 1e-5), rtol=5e-3)


@pytest.mark.parametrize("H,W,Ca,Cb,Cout", [(64, 64, 640, 320, 320), (32, 32, 1280, 640, 640), (16, 16, 1280, 1280, 1280)])
def test_conv_halo_concat_input(gpu, H, W, Ca, Cb, Cout):
    from chiaswarm_amd.ops import hip_ops

    B = 2
    a = with_stats(rnd(B, H, W, Ca, dev=gpu, scale=1.5), gpu)
    b = with_stats(rnd(B, H, W, Cb, dev=gpu), gpu)
    C = Ca + Cb
    gamma, beta = rnd(C, dev=gpu), rnd(C, dev=gpu)
    stat = hip_ops.gn_finalize(a, 32, 1e-5, b)
    assert stat is not None
    wt = rnd(Cout, C, 3, 3, dev=gpu, scale=(9 * C) ** -0.5)
    y = hip_ops.conv_halo(a, ops.pack_conv_weight(wt), None, gn=(stat, gamma, beta, 32, True), x2=b)
    cat = torch.cat([a, b], -1).cpu()
    ref = ref_conv(ref_gn_silu(cat, gamma.cpu(), beta.cpu(), 32, 1e-5), wt.cpu())
    assert rel(y.cpu(), ref) < 1e-2


@torch.no_grad()
@pytest.mark.parametrize("cin,cout,hw", [(320, 320, 64), (320, 640, 32), (1280, 1280, 16)])
def test_resnet_block_halo_path_vs_fp32(gpu, cin, cout, hw):
    from chiaswarm_amd.models.layers import ResnetBlock2D, init_random_fast_, prepare_model
    from chiaswarm_amd.ops import hip_ops

    with torch.device(gpu):
        blk = ResnetBlock2D(cin, cout, 1280).to(torch.bfloat16).eval()
    init_random_fast_(blk, seed=4)
    prepare_model(blk)
    x = with_stats(rnd(2, hw, hw, cin, dev=gpu, scale=2.0), gpu)
    temb = rnd(2, cout, dev=gpu)
    n0 = hip_ops.HALO_STATS[0]
    y = blk(x, temb)
    assert hip_ops.HALO_STATS[0] - n0 == 2  # both GroupNorms fused into the halo convs
    twin = copy.deepcopy(blk).float()
    with ops.ops_mode("reference"):
        ref = twin(x.float(), temb.float())
    assert rel(y, ref) < 2e-2


@torch.no_grad()
def test_resnet_block_concat_halo_path_vs_fp32(gpu):
    from chiaswarm_amd.models.layers import ResnetBlock2D, init_random_fast_, prepare_model
    from chiaswarm_amd.ops import hip_ops

    with torch.device(gpu):
        blk = ResnetBlock2D(960, 320, 1280).to(torch.bfloat16).eval()
    init_random_fast_(blk, seed=5)
    prepare_model(blk)
    a = with_stats(rnd(2, 64, 64, 640, dev=gpu), gpu)
    b = with_stats(rnd(2, 64, 64, 320, dev=gpu, scale=2.0), gpu)
    temb = rnd(2, 320, dev=gpu)
    n0 = hip_ops.HALO_STATS[0]
    y = blk.forward_cat(a, b, temb)
    assert hip_ops.HALO_STATS[0] - n0 == 2
    twin = copy.deepcopy(blk).float()
    with ops.ops_mode("reference"):
        ref = twin(torch.cat([a, b], -1).float(), temb.float())
    assert rel(y, ref) < 2e-2
