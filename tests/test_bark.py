"""Bark: KV-cached decode == full causal forward, EnCodec decoder pieces,
weight-norm folding, and the job callback (reference swarm/audio/bark.py)."""
import base64

import numpy as np
import torch
import torch.nn.functional as F

from chiaswarm_amd.models import bark as bk


def _gpt():
    torch.manual_seed(0)
    sc, _, _ = bk.bark_configs("tiny")
    m = bk.BarkCausalGPT(sc).eval()
    for p in m.parameters():
        p.data.normal_(0, 0.05)
    return m


def test_kv_cache_decode_matches_full_forward():
    m = _gpt()
    ids = torch.randint(0, 1000, (1, 12))
    m.cache = None
    full = m(ids, last_only=False)  # [1, 12, V]
    m.new_cache()
    first = m(ids[:, :5], pos=0)  # prefill 5
    assert torch.allclose(first[0], full[0, 4], atol=1e-4)
    for i in range(5, 12):
        step = m(ids[:, i:i + 1], pos=i)
        assert torch.allclose(step[0], full[0, i], atol=1e-4), i


def test_decode_step_matches_full_forward():
    m = _gpt()
    ids = torch.randint(0, 1000, (1, 10))
    m.cache = None
    full = m(ids, last_only=False)
    m.new_cache()
    m(ids[:, :4], pos=0)
    for i in range(4, 10):
        step = m.decode_step(int(ids[0, i]), i)
        assert torch.allclose(step[0], full[0, i], atol=1e-4), i


def test_fine_model_shapes():
    _, _, fc = bk.bark_configs("tiny")
    m = bk.BarkFineGPT(fc).eval()
    codes = torch.randint(0, 1024, (1, 32, 8))
    assert m(3, codes).shape == (1, 32, fc.out_vocab)


def test_reflect_left_matches_torch():
    x = torch.randn(2, 9, 4)
    ref = F.pad(x.transpose(1, 2), (3, 0), mode="reflect").transpose(1, 2)
    assert torch.equal(bk._reflect_left(x, 3), ref)


def test_fold_weight_norm():
    v, g = torch.randn(6, 4, 3), torch.rand(6, 1, 1) + 0.5
    sd = bk.fold_weight_norm({"c.weight_v": v, "c.weight_g": g, "c.bias": torch.zeros(6)})
    ref = torch.nn.utils.parametrizations.weight_norm(torch.nn.Conv1d(4, 6, 3))
    with torch.no_grad():
        ref.parametrizations.weight.original0.copy_(g)
        ref.parametrizations.weight.original1.copy_(v)
    assert set(sd) == {"c.weight", "c.bias"}
    assert torch.allclose(sd["c.weight"], ref.weight, atol=1e-6)


def test_encodec_decoder_length():
    dec = bk.EncodecDecoder(bk.TINY_ENCODEC).eval()
    codes = torch.randint(0, 1024, (8, 10))
    wav = dec(codes)
    assert wav.shape == (10 * bk.TINY_ENCODEC.hop,)
    assert torch.isfinite(wav).all()


def test_bark_generate_and_callback():
    from chiaswarm_amd.pipelines import audio

    b = bk.Bark("cpu", size="tiny")
    a1 = b.generate_audio("hello world", seed=3, max_semantic_tokens=20)
    a2 = b.generate_audio("hello world", seed=3, max_semantic_tokens=20)
    assert a1.ndim == 1 and len(a1) > 0 and np.array_equal(a1, a2)
    res, cfg = audio.bark_diffusion_callback("cpu", "tiny-bark", prompt="hi there")
    art = res["primary"]
    assert art["content_type"] in ("audio/mpeg", "audio/wav")
    assert len(base64.b64decode(art["blob"])) > 44
    assert cfg == {}
