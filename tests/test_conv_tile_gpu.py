"""Persistent halo-tile conv (csrc/kernels/conv_tile.hip, 3x3 / stride 1 /
Cout = 32: the Real-ESRGAN dense-block convs) against the fp32 PyTorch
reference: ragged tiles, every Cin chunk count of an RRDB block, channel-slice
input / output views of a dense buffer, bias + leaky ReLU, several images."""
import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.ops import hip_ops

pytestmark = pytest.mark.gpu


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / (ref.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,H,W", [(1, 64, 64), (1, 37, 50), (2, 16, 96), (1, 8, 32), (3, 9, 33)])
@pytest.mark.parametrize("Cin", [32, 64, 96, 160])
@pytest.mark.parametrize("act", [None, "lrelu"])
@pytest.mark.parametrize("Cout", [32, 64])
def test_conv_tile_matches_fp32(gpu, B, H, W, Cin, act, Cout, monkeypatch):
    torch.manual_seed(B * 100 + H + W + Cin + Cout)
    monkeypatch.setattr(hip_ops, "CONV_TILE64", True)
    C = 192  # dense buffer: input = channels [0, Cin), output = channels [C, C + Cout)
    buf = (torch.randn(B, H, W, C + Cout, device=gpu)).to(torch.bfloat16)
    x = buf[..., :Cin]
    out = buf[..., C:C + Cout]
    w = (torch.randn(Cout, Cin, 3, 3, device=gpu) * (9 * Cin) ** -0.5).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w)
    bias = torch.randn(Cout, device=gpu).to(torch.bfloat16)
    keep = buf[..., :C].clone()
    before = hip_ops.CONV_TILE_STATS[0]
    y = ops.conv2d(x, wp, bias, act=act, out=out)
    assert hip_ops.CONV_TILE_STATS[0] == before + 1  # the halo-tile kernel ran
    torch.cuda.synchronize()
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, None, False, None, act)
    assert y.data_ptr() == out.data_ptr()
    assert rel_err(y.cpu(), ref) < 1e-2
    assert torch.equal(buf[..., :C], keep)  # channels outside the output slice are untouched


def test_conv_tile_rrdb_block_matches_gemm_path(gpu):
    """A whole RRDB (3 dense blocks) with the halo-tile convs == the implicit-GEMM path."""
    from chiaswarm_amd.models import rrdbnet
    from chiaswarm_amd.models.layers import init_random_, prepare_model

    torch.manual_seed(0)
    m = rrdbnet.RRDBNet(nb=1).to(gpu).to(torch.bfloat16).eval()
    init_random_(m, seed=3)
    prepare_model(m)
    x = torch.rand(1, 48, 40, 3, device=gpu)
    hip_ops.CONV_TILE = True
    a = m(x)
    hip_ops.CONV_TILE = False
    try:
        b = m(x)
    finally:
        hip_ops.CONV_TILE = True
    assert rel_err(a.cpu(), b.cpu()) < 1e-2


@pytest.mark.parametrize("Cout", [32, 64])
def test_conv_tile_residual_out_scale(gpu, Cout, monkeypatch):
    """RRDB conv5: act-free conv * 0.2 + x (residual a channel slice of the dense buffer)."""
    monkeypatch.setattr(hip_ops, "CONV_TILE64", True)
    torch.manual_seed(Cout)
    B, H, W, Cin = 1, 40, 70, 192
    buf = torch.randn(B, H, W, Cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device=gpu) * (9 * Cin) ** -0.5).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w)
    bias = torch.randn(Cout, device=gpu).to(torch.bfloat16)
    res = buf[..., :Cout]
    out = torch.empty(B, H, W, Cout, device=gpu, dtype=torch.bfloat16)
    before = hip_ops.CONV_TILE_STATS[0]
    y = ops.conv2d(buf, wp, bias, residual=res, out_scale=0.2, out=out)
    assert hip_ops.CONV_TILE_STATS[0] == before + 1
    ref = ops._ref_conv2d(buf.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, res.float().cpu(), False,
                          None, None, 0.2)
    assert rel_err(y.cpu(), ref) < 1e-2


def test_conv_tile64_rrdb_block_matches_gemm_path(gpu, monkeypatch):
    """A whole RRDB with the Cout = 64 instance (conv5 with its fused * 0.2 + x) == the implicit GEMM."""
    monkeypatch.setattr(hip_ops, "CONV_TILE64", True)
    test_conv_tile_rrdb_block_matches_gemm_path(gpu)
