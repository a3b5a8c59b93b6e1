"""Persistent halo-tile conv (csrc/kernels/conv_tile.hip, 3x3 / stride 1 /
Cout = 32 / 64 / <= 16: the Real-ESRGAN convs) against the fp32 PyTorch
reference: ragged tiles, every Cin chunk count of an RRDB block, channel-slice
input / output views of a dense buffer, bias + leaky ReLU, several images, the
fused x2 upsample, the narrow (RGB) outputs and the two-residual epilogue."""
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


@pytest.mark.parametrize("Cout", [32, 64])
@pytest.mark.parametrize("B,H,W", [(1, 24, 40), (2, 9, 33)])
def test_conv_tile_up2x_matches_fp32(gpu, Cout, B, H, W, monkeypatch):
    """Nearest-x2 upsample fused into the halo addressing (Real-ESRGAN conv_up1 / conv_up2):
    the output is 2H x 2W, the halo reads input pixel (y / 2, x / 2)."""
    monkeypatch.setattr(hip_ops, "CONV_TILE64", True)
    torch.manual_seed(Cout + H)
    Cin = 64
    x = torch.randn(B, H, W, Cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device=gpu) * (9 * Cin) ** -0.5).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w)
    bias = torch.randn(Cout, device=gpu).to(torch.bfloat16)
    before = hip_ops.CONV_TILE_STATS[0]
    y = ops.conv2d(x, wp, bias, up2x=True, act="lrelu")
    assert hip_ops.CONV_TILE_STATS[0] == before + 1
    assert y.shape == (B, 2 * H, 2 * W, Cout)
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, None, True, None, "lrelu")
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("Cout", [3, 4, 16])
@pytest.mark.parametrize("B,H,W", [(1, 40, 70), (2, 16, 32)])
def test_conv_tile_narrow_matches_fp32(gpu, Cout, B, H, W, monkeypatch):
    """The 16-wide instance: Cout <= 16 (RGB conv_last), weight rows / bias / stores
    past Cout skipped; the output tensor is exactly [B, H, W, Cout]."""
    monkeypatch.setattr(hip_ops, "CONV_TILE_NARROW_MIN_PX", 1)
    torch.manual_seed(Cout * 7 + H)
    Cin = 64
    x = torch.randn(B, H, W, Cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device=gpu) * (9 * Cin) ** -0.5).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w)
    bias = torch.randn(Cout, device=gpu).to(torch.bfloat16)
    sentinel = torch.full((B * H * W * Cout + 64,), 7.0, device=gpu, dtype=torch.bfloat16)
    out = sentinel[:B * H * W * Cout].view(B, H, W, Cout)
    before = hip_ops.CONV_TILE_STATS[0]
    y = ops.conv2d(x, wp, bias, out=out)
    assert hip_ops.CONV_TILE_STATS[0] == before + 1
    torch.cuda.synchronize()
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, None, False, None, None)
    assert rel_err(y.cpu(), ref) < 1e-2
    assert torch.all(sentinel[B * H * W * Cout:] == 7.0)  # nothing written past the tensor


@pytest.mark.parametrize("Cout", [32, 64])
def test_conv_tile_two_residuals_in_place(gpu, Cout, monkeypatch):
    """y = 0.04 conv + 0.2 res + res2 with the output aliasing res2 (the RRDB's
    third dense block writing over the block input)."""
    monkeypatch.setattr(hip_ops, "CONV_TILE64", True)
    torch.manual_seed(Cout + 1)
    B, H, W, Cin = 1, 24, 50, 192
    buf = torch.randn(B, H, W, Cin, device=gpu).to(torch.bfloat16)
    outer_buf = torch.randn(B, H, W, Cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device=gpu) * (9 * Cin) ** -0.5).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w)
    bias = torch.randn(Cout, device=gpu).to(torch.bfloat16)
    res, res2 = buf[..., :Cout], outer_buf[..., :Cout]
    ref = ops._ref_conv2d(buf.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, res.float().cpu(), False,
                          None, None, 0.04, 1, res2.float().cpu(), 0.2)
    rest = outer_buf[..., Cout:].clone()
    before = hip_ops.CONV_TILE_STATS[0]
    y = ops.conv2d(buf, wp, bias, residual=res, out_scale=0.04, residual2=res2, res_scale=0.2, out=res2)
    assert hip_ops.CONV_TILE_STATS[0] == before + 1
    assert y.data_ptr() == res2.data_ptr()
    torch.cuda.synchronize()
    assert rel_err(y.cpu(), ref) < 1e-2
    assert torch.equal(outer_buf[..., Cout:], rest)
    # the implicit-GEMM fallback (temporary + one combining pass) agrees
    monkeypatch.setattr(hip_ops, "CONV_TILE", False)
    r2 = torch.randn(B, H, W, Cout, device=gpu).to(torch.bfloat16)
    ref2 = ops._ref_conv2d(buf.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, res.float().cpu(), False,
                           None, None, 0.04, 1, r2.float().cpu(), 0.2)
    y2 = ops.conv2d(buf, wp, bias, residual=res, out_scale=0.04, residual2=r2, res_scale=0.2, out=r2)
    torch.cuda.synchronize()
    assert y2.data_ptr() == r2.data_ptr() and rel_err(y2.cpu(), ref2) < 1e-2


def test_conv_tile_narrow_u8_output(gpu, monkeypatch):
    """uint8 image stored by the epilogue: round(clamp(y, 0, 1) * 255) of the fp32 conv."""
    monkeypatch.setattr(hip_ops, "CONV_TILE_NARROW_MIN_PX", 1)
    torch.manual_seed(11)
    B, H, W, Cin = 1, 40, 72, 64
    x = torch.randn(B, H, W, Cin, device=gpu).to(torch.bfloat16)
    w = (torch.randn(3, Cin, 3, 3, device=gpu) * (9 * Cin) ** -0.5 * 0.5).to(torch.bfloat16)
    wp = ops.pack_conv_weight(w)
    bias = torch.full((3,), 0.5, device=gpu).to(torch.bfloat16)
    before = hip_ops.CONV_TILE_STATS[0]
    y = ops.conv2d(x, wp, bias, out_u8=True)
    assert hip_ops.CONV_TILE_STATS[0] == before + 1
    assert y.dtype == torch.uint8 and y.shape == (B, H, W, 3)
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, None, False, None, None)
    ref8 = (ref.clamp(0, 1) * 255).round()
    d = (y.cpu().float() - ref8).abs()
    assert d.max() <= 2 and d.mean() < 0.2
    assert 0 < int((y == 0).sum()) + int((y == 255).sum()) < y.numel()  # clamping exercised, not everywhere


def test_upscale_graph_replay_matches_eager(gpu):
    """upscale_x4's one-replay graph == the eager network, per input (static buffers refreshed)."""
    import numpy as np
    from PIL import Image

    from chiaswarm_amd.models.layers import init_random_, prepare_model
    from chiaswarm_amd.models.rrdbnet import TINY_RRDB, RRDBNet
    from chiaswarm_amd.pipelines.esrgan import upscale_x4

    torch.manual_seed(0)
    with torch.device(gpu):
        net = RRDBNet(**TINY_RRDB).to(torch.bfloat16).eval()
    init_random_(net, seed=5)
    prepare_model(net)
    rng = np.random.default_rng(0)
    for i in range(2):
        arr = (rng.random((40, 56, 3)) * 255).astype(np.uint8)
        got = np.asarray(upscale_x4(net, Image.fromarray(arr)))
        want = net(torch.from_numpy(arr).to(gpu)[None], u8_out=True)[0].cpu().numpy()
        assert got.shape == (160, 224, 3)
        assert np.array_equal(got, want), i
    assert len(net._u8_graphs) == 1
