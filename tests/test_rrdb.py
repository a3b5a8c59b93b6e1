"""RRDBNet (Real-ESRGAN x4) zero-copy dense blocks vs a plain concat-based
PyTorch definition of the same network (CPU), plus the HIP path on the GPU."""
import pytest
import torch
import torch.nn.functional as F

from chiaswarm_amd import ops
from chiaswarm_amd.models.layers import init_random_
from chiaswarm_amd.models.rrdbnet import TINY_RRDB, RRDBNet


def conv(m, x):
    return F.conv2d(x, m.weight.float(), m.bias.float(), padding=1)


def ref_forward(net, x):
    """Textbook RRDBNet in NCHW fp32 with torch.cat dense connections."""
    lr = lambda t: F.leaky_relu(t, 0.2)  # noqa: E731
    x = x.permute(0, 3, 1, 2).float()
    feat = conv(net.conv_first, x)
    h = feat
    for blk in net.body:
        inp = h
        for rdb in (blk.rdb1, blk.rdb2, blk.rdb3):
            x0 = h
            x1 = lr(conv(rdb.conv1, x0))
            x2 = lr(conv(rdb.conv2, torch.cat([x0, x1], 1)))
            x3 = lr(conv(rdb.conv3, torch.cat([x0, x1, x2], 1)))
            x4 = lr(conv(rdb.conv4, torch.cat([x0, x1, x2, x3], 1)))
            x5 = conv(rdb.conv5, torch.cat([x0, x1, x2, x3, x4], 1))
            h = x5 * 0.2 + x0
        h = h * 0.2 + inp
    fea = conv(net.conv_body, h) + feat
    fea = lr(conv(net.conv_up1, F.interpolate(fea, scale_factor=2, mode="nearest")))
    fea = lr(conv(net.conv_up2, F.interpolate(fea, scale_factor=2, mode="nearest")))
    out = conv(net.conv_last, lr(conv(net.conv_hr, fea)))
    return out.permute(0, 2, 3, 1)


def _net(dev, dtype):
    torch.manual_seed(0)
    with torch.device(dev):
        net = RRDBNet(**TINY_RRDB).to(dtype).eval()
    init_random_(net, seed=4)
    return net


def test_rrdb_cpu_matches_concat_reference():
    net = _net("cpu", torch.float32)
    x = torch.rand(1, 12, 10, 3)
    y = net(x)
    assert y.shape == (1, 48, 40, 3)
    ref = ref_forward(net, x)
    assert torch.allclose(y, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_rrdb_gpu_hip_vs_reference(gpu):
    net = _net(gpu, torch.bfloat16)
    x = torch.rand(2, 24, 16, 3, device=gpu)
    y = net(x)
    ref = ref_forward(net, x)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 3e-2
