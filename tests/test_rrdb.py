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


def test_pth_checkpoint_weights_only(tmp_path):
    """Published Real-ESRGAN weights are ``.pth`` files wrapping the state dict
    in ``params_ema``: read with the weights-only unpickler, geometry (block
    count, width, growth) taken from the keys; the original ESRGAN repo's key
    names map onto the same modules; a pickle that is not plain tensors is refused."""
    import pickle

    from chiaswarm_amd.models.weights import CheckpointMismatch, read_pth
    from chiaswarm_amd.pipelines.esrgan import _OLD_ESRGAN_RENAMES, load_esrgan

    src = RRDBNet(**TINY_RRDB).eval()
    init_random_(src, seed=5)
    sd = {k: v.clone() for k, v in src.state_dict().items()}
    f = tmp_path / "RealESRGAN_x4plus_tiny.pth"
    torch.save({"params_ema": sd, "params": {k: torch.zeros_like(v) for k, v in sd.items()}}, f)
    net = load_esrgan(str(f), "cpu")
    assert len(net.body) == TINY_RRDB["nb"] and net.nf == TINY_RRDB["nf"] and net.gc == TINY_RRDB["gc"]
    for k, v in net.state_dict().items():
        assert torch.equal(v, sd[k]), k
    # original ESRGAN naming
    inv = {b: a for a, b in _OLD_ESRGAN_RENAMES.items()}
    old = {}
    for k, v in sd.items():
        for b, a in inv.items():
            k = k.replace(b, a)
        old[k] = v
    assert any(k.startswith("RRDB_trunk.") for k in old)
    g = tmp_path / "old" / "RRDB_ESRGAN_x4.pth"
    g.parent.mkdir()
    torch.save(old, g)
    net2 = load_esrgan(str(g), "cpu")
    for k, v in net2.state_dict().items():
        assert torch.equal(v, sd[k]), k

    class Evil:
        def __reduce__(self):
            return (print, ("executed",))

    h = tmp_path / "evil.pth"
    with open(h, "wb") as fh:
        pickle.dump({"params_ema": Evil()}, fh)
    with pytest.raises(Exception):
        read_pth(str(h))
    torch.save({"params_ema": {"a": 1}}, tmp_path / "notensors.pth")
    with pytest.raises(CheckpointMismatch):
        read_pth(str(tmp_path / "notensors.pth"))


def test_srvgg_checkpoint_is_a_clear_error(tmp_path):
    """A Real-ESRGAN checkpoint of another architecture (SRVGGNetCompact,
    realesr-general-x4v3: ``body.N.weight`` only) is refused with a ValueError
    naming it, not a bare KeyError."""
    from chiaswarm_amd.pipelines.esrgan import load_esrgan

    sd = {f"body.{i}.weight": torch.zeros(64, 64 if i else 3, 3, 3) for i in range(4)}
    f = tmp_path / "realesr-general-x4v3.pth"
    torch.save({"params": sd}, f)
    with pytest.raises(ValueError, match="not an x4 RRDBNet"):
        load_esrgan(str(f), "cpu")
