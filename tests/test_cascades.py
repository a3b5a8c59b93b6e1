"""DeepFloyd IF cascade, x2 latent / x4 upscalers, T5 pieces and the
per-sample-affine GroupNorm they use (tiny geometries, CPU)."""
import base64
import io

import torch
import torch.nn.functional as F
from PIL import Image

from chiaswarm_amd import ops


def test_group_norm_per_sample_affine():
    torch.manual_seed(0)
    x = torch.randn(2, 5, 6, 64)
    g, b = torch.randn(2, 64), torch.randn(2, 64)
    y = ops.group_norm(x, g, b, 8, 1e-5, silu=True)
    ref = F.group_norm(x.permute(0, 3, 1, 2), 8, None, None, 1e-5) * g[:, :, None, None] + b[:, :, None, None]
    assert torch.allclose(y, F.silu(ref).permute(0, 2, 3, 1), atol=1e-5)


def test_t5_relative_buckets():
    from chiaswarm_amd.models.t5 import relative_position_bucket

    rel = torch.tensor([0, 1, -1, 7, -7, 8, 20, -20, 127, 500, -500])
    got = relative_position_bucket(rel).tolist()
    # bidirectional: 16 buckets per side, 8 exact, log-spaced up to 128
    assert got[:5] == [0, 17, 1, 23, 7]
    assert got[9] == 31 and got[10] == 15
    assert all(16 <= v <= 31 for v, r in zip(got, rel.tolist()) if r > 0)


def test_t5_encoder_mask_invariance():
    from chiaswarm_amd.models.t5 import TINY_T5, T5Encoder, T5Tokenizer

    torch.manual_seed(0)
    enc = T5Encoder(TINY_T5).eval()
    tok = T5Tokenizer(None, 16, vocab=TINY_T5.vocab)
    ids, mask = tok(["a red cube on a table"])
    full = enc(ids, mask)
    n = int(mask.sum())
    short = enc(ids[:, :n], mask[:, :n])
    # masked padding does not change the real tokens' states
    assert torch.allclose(full[:, :n], short, atol=1e-4)


def test_if_cascade_and_callback():
    from chiaswarm_amd.pipelines.deepfloyd import IFCascade, diffusion_if_callback

    p = IFCascade("cpu", tiny=True)
    kw = dict(stage1_steps=3, stage2_steps=2, stage3_steps=2)
    a = p("a red cube", generator=torch.Generator().manual_seed(0), **kw)
    b = p("a red cube", generator=torch.Generator().manual_seed(0), **kw)
    s = p.stage2.cfg.sample_size * 4
    assert a[0].size == (s, s)
    assert a[0].tobytes() == b[0].tobytes()
    res, cfg = diffusion_if_callback("cpu", "tiny-IF", prompt="a cat", num_inference_steps=2)
    img = Image.open(io.BytesIO(base64.b64decode(res["primary"]["blob"])))
    assert img.size == (s, s) and cfg["_class_name"] == "IFPipeline"


def test_upscalers():
    from chiaswarm_amd.pipelines.upscale import LatentUpscaler, X4Upscaler

    ims = [Image.new("RGB", (32, 32), (200, 30, 30)), Image.new("RGB", (32, 32), (30, 30, 200))]
    up = LatentUpscaler("cpu", tiny=True)
    out = up(["a", "b"], ims, num_inference_steps=2, generator=torch.Generator().manual_seed(0))
    assert len(out) == 2 and out[0].size == (64, 64)
    x4 = X4Upscaler("cpu", tiny=True)
    o4 = x4("a", ims[:1], num_inference_steps=2, generator=torch.Generator().manual_seed(0))
    assert o4[0].size == (128, 128)
