"""ControlNet neural annotators (controlnet/annotators.py): every detector runs
end to end on the CPU with its seeded random init (no checkpoints offline) and
returns a conditioning image of the input's size; state-dict layouts load back
into themselves (the names the public checkpoints use); the post-processing
(scribble NMS, M-LSD decoding, ADE palette) is checked on constructed inputs.
Parity with the real detectors is unpinned: their checkpoints are not in this
image."""
import numpy as np
import pytest
import torch
from PIL import Image

from chiaswarm_amd.controlnet import annotators as an
from chiaswarm_amd.controlnet.preprocess import preprocess_image


@pytest.fixture(autouse=True)
def _no_weights(tmp_path, monkeypatch):
    monkeypatch.setenv("CSK_ANNOTATOR_DIR", str(tmp_path))
    an._CACHE.clear()
    yield
    an._CACHE.clear()


def _img(w=96, h=80):
    rng = np.random.default_rng(0)
    a = np.zeros((h, w, 3), np.uint8)
    a[20:60, 30:70] = 200
    a += rng.integers(0, 20, a.shape, dtype=np.uint8)
    return Image.fromarray(a)


@pytest.mark.parametrize("kind", ["scribble", "softedge", "lineart", "mlsd"])
def test_conv_annotators_shape(kind):
    out = preprocess_image(_img(), {"preprocess": True, "type": kind})
    assert out.size == (96, 80) and out.mode == "RGB"
    a = np.asarray(out)
    assert a.dtype == np.uint8


def test_depth_dpt_shape():
    out = an.depth(_img(), size=64)  # 4x4 patch grid: position-embedding resize path
    assert out.size == (96, 80)


def test_seg_upernet_palette():
    out = an.segmentation(_img(), res=64)
    a = np.asarray(out).reshape(-1, 3)
    pal = {tuple(c) for c in an.ADE_PALETTE.tolist()}
    assert all(tuple(c) in pal for c in np.unique(a, axis=0).tolist())
    assert an.ADE_PALETTE.shape == (151, 3) and tuple(an.ADE_PALETTE[1]) == (120, 120, 120)


def test_weights_load_from_dir(tmp_path):
    from safetensors.torch import save_file

    m = an.LineartGenerator()
    sd = {k: torch.randn_like(v) if v.is_floating_point() else v for k, v in m.state_dict().items()}
    save_file(sd, str(tmp_path / "lineart.safetensors"))
    an._CACHE.clear()
    g = an._build("lineart", an.LineartGenerator)
    assert g.weights_source.endswith("lineart.safetensors")
    assert torch.allclose(g.state_dict()["model0.1.weight"].float(), sd["model0.1.weight"])


def test_scribble_nms_keeps_thin_ridges():
    x = np.zeros((40, 40), np.uint8)
    x[:, 18:23] = 255  # a 5-px stroke: its blurred ridge is the centre column
    y = an._nms(x, 127, 1.0)
    assert y[:, 20].all() and not y[:, 10].any()


def test_unknown_types_are_fatal():
    with pytest.raises(ValueError):
        preprocess_image(_img(), {"preprocess": True, "type": "no-such-annotator"})


def test_normalbae_end_to_end_shape():
    out = preprocess_image(_img(), {"preprocess": True, "type": "normalbae"})
    assert out.size == (96, 80) and out.mode == "RGB"


def test_normalbae_architecture_and_key_layout():
    """tf_efficientnet_b5 trunk (39 blocks, 2048-ch head) + NNET decoder, with
    the scannet.pt key names; outputs are unit normals at 1/8..1/1 resolution."""
    m = an.NormalBaeNet().eval()
    sd = m.state_dict()
    for k in ("encoder.original_model.conv_stem.weight", "encoder.original_model.blocks.0.0.se.conv_reduce.weight",
              "encoder.original_model.blocks.6.2.conv_pwl.weight", "encoder.original_model.conv_head.weight",
              "decoder.up1._net.0.weight", "decoder.out_conv_res1.6.weight"):
        assert k in sd, k
    assert sum(len(s) for s in m.encoder.original_model.blocks) == 39
    assert sd["encoder.original_model.blocks.1.0.se.conv_reduce.weight"].shape == (6, 144, 1, 1)
    assert sd["decoder.out_conv_res4.0.weight"].shape == (128, 516, 1)
    with torch.no_grad():
        outs = m(torch.randn(1, 3, 64, 96))
    assert [tuple(o.shape[2:]) for o in outs] == [(8, 12), (16, 24), (32, 48), (64, 96)]
    n = outs[-1][0, :3].norm(dim=0)
    assert torch.allclose(n, torch.ones_like(n), atol=1e-4)
    assert (outs[-1][:, 3] > 0).all()  # kappa = elu + 1 + 0.01


def test_normalbae_same_padding_matches_tf():
    """Stride-2 'same' conv pads (k - s) split low/high with the extra row/column high."""
    c = an._Conv2dSame(1, 1, 3, 2, 0, bias=False)
    torch.nn.init.ones_(c.weight)
    y = c(torch.ones(1, 1, 6, 6))
    assert y.shape[2:] == (3, 3)
    # no padding on the low side (first window fully inside); one zero row/column on the high side
    assert y[0, 0, 0, 0].item() == 9.0 and y[0, 0, 2, 2].item() == 4.0 and y[0, 0, 0, 2].item() == 6.0


def test_openpose_end_to_end_shape():
    out = preprocess_image(_img(), {"preprocess": True, "type": "openpose"})
    assert out.size == (96, 80) and out.mode == "RGB"


def test_openpose_checkpoint_key_layout():
    """body_pose_model.pth stores flat layer names (conv1_1.weight, Mconv7_stage6_L2.bias, ...)."""
    m = an.BodyPoseModel()
    flat = {k.split(".", 1)[1]: torch.randn_like(v) for k, v in m.state_dict().items()}
    assert "conv1_1.weight" in flat and "Mconv7_stage6_L2.bias" in flat
    missing, unexpected = m.load_state_dict(flat, strict=False)
    assert not missing and not unexpected
    assert torch.equal(m.model6_2.Mconv7_stage6_L2.bias, flat["Mconv7_stage6_L2.bias"])


def test_openpose_paf_grouping_one_arm():
    """Peaks for neck -> right shoulder -> elbow -> wrist joined by part-affinity
    fields pointing along each limb assemble into one 4-part person."""
    H = W = 64
    heat = np.zeros((H, W, 19), np.float32)
    paf = np.zeros((H, W, 38), np.float32)
    pts = {1: (20, 20), 2: (30, 20), 3: (40, 28), 4: (48, 38)}  # part index (0-based) -> (x, y)
    yy, xx = np.mgrid[0:H, 0:W]
    for p, (x, y) in pts.items():
        heat[:, :, p] = np.exp(-((xx - x) ** 2 + (yy - y) ** 2) / 8.0)
    for k, (a, b) in ((0, (1, 2)), (2, (2, 3)), (3, (3, 4))):
        v = np.subtract(pts[b], pts[a]).astype(np.float32)
        v /= np.linalg.norm(v)
        c0, c1 = [x - 19 for x in an._PAF_IDX[k]]
        paf[:, :, c0], paf[:, :, c1] = v[0], v[1]
    peaks = an._pose_peaks(heat)
    assert [len(peaks[p]) for p in (1, 2, 3, 4)] == [1, 1, 1, 1]
    cands, subset = an._pose_group(peaks, paf, H)
    assert len(subset) == 1 and subset[0][-1] == 4
    canvas = an._draw_pose(H, W, cands, subset)
    assert canvas.shape == (H, W, 3) and canvas.any()


def test_pidinet_pixel_difference_convs_match_definitions():
    """cd: sum_i w_i (x_i - x_c); rd: sum_{i>0} w_i (x_outer_i - x_inner_i) over
    the 8 directions; the folded plain-conv forms reproduce both."""
    torch.manual_seed(0)
    x = torch.randn(1, 2, 9, 9)
    cd = an.PDConv("cd", 2, 3)
    pat = torch.nn.functional.unfold(x, 3, padding=1).view(1, 2, 9, 81)  # [b, c, tap, pix]
    ref = torch.einsum("oct,bctp->bop", cd.weight.view(3, 2, 9), pat - pat[:, :, 4:5]).view(1, 3, 9, 9)
    assert torch.allclose(cd(x), ref, atol=1e-5)
    rd = an.PDConv("rd", 2, 3)
    p5 = torch.nn.functional.unfold(x, 5, padding=2).view(1, 2, 25, 81)
    diff = p5[:, :, an._RD_OUTER] - p5[:, :, an._RD_INNER]
    ref = torch.einsum("oct,bctp->bop", rd.weight.view(3, 2, 9)[:, :, 1:], diff).view(1, 3, 9, 9)
    assert torch.allclose(rd(x), ref, atol=1e-5)
    ad = an.PDConv("ad", 2, 3)
    ref = torch.einsum("oct,bctp->bop", ad.weight.view(3, 2, 9),
                       pat - pat[:, :, [1, 2, 5, 0, 4, 8, 3, 6, 7]]).view(1, 3, 9, 9)
    assert torch.allclose(ad(x), ref, atol=1e-5)


def test_pidinet_checkpoint_layout_and_outputs():
    """table5_pidinet.pth names (module.-prefixed, under 'state_dict') load
    without missing keys; 4 side maps + fused map at input size, in [0, 1]."""
    m = an.PiDiNet().eval()
    sd = m.state_dict()
    for k, shape in (("init_block.weight", (60, 3, 3, 3)), ("block1_1.conv1.weight", (60, 1, 3, 3)),
                     ("block2_1.shortcut.weight", (120, 60, 1, 1)), ("block4_4.conv2.weight", (240, 240, 1, 1)),
                     ("dilations.3.conv2_4.weight", (24, 24, 3, 3)), ("attentions.0.conv1.bias", (4,)),
                     ("conv_reduces.2.conv.weight", (1, 24, 1, 1)), ("classifier.bias", (1,))):
        assert tuple(sd[k].shape) == shape, k
    assert m.block3_2.conv1.kind == "ad" and m.block4_3.conv1.kind == "rd" and m.init_block.kind == "cd"
    wrapped = {"state_dict": {"module." + k: torch.randn_like(v) for k, v in sd.items()}}
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "table5_pidinet.pth")
        torch.save(wrapped, p)
        flat = an.load_checkpoint(p)
    missing, unexpected = m.load_state_dict(flat, strict=True)
    with torch.no_grad():
        outs = m(torch.rand(1, 3, 64, 48))
    assert len(outs) == 5 and all(o.shape == (1, 1, 64, 48) for o in outs)
    assert all(((o >= 0) & (o <= 1)).all() for o in outs)
