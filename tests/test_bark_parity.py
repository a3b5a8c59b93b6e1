"""Bark parity against transformers' ``BarkModel`` (reference: swarm/audio/bark.py,
which runs suno's bark package — the same three GPTs + EnCodec): a tiny random
BarkModel is saved with ``save_pretrained`` (safetensors + config.json) and
loaded by ``Bark(weights_dir=...)``; geometry comes from the config, the GPT
logits and the EnCodec waveform must match transformers in fp32."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

from chiaswarm_amd.models import bark as bark_mod  # noqa: E402


def _tiny_hf_bark(tmp_path, tie=True):
    from transformers import BarkConfig, BarkModel

    gpt = dict(block_size=64, num_layers=2, num_heads=2, hidden_size=32, bias=False)
    cfg = BarkConfig(
        semantic_config=dict(gpt, input_vocab_size=300, output_vocab_size=280),
        coarse_acoustics_config=dict(gpt, input_vocab_size=200, output_vocab_size=200),
        fine_acoustics_config=dict(gpt, input_vocab_size=130, output_vocab_size=130, n_codes_total=4,
                                   n_codes_given=1, tie_word_embeddings=tie),
        codec_config=dict(hidden_size=16, num_filters=4, upsampling_ratios=[4, 2], codebook_size=128,
                          codebook_dim=16, num_lstm_layers=2, target_bandwidths=[120.0]))  # 4 quantizers at hop 8
    torch.manual_seed(0)
    ref = BarkModel(cfg).eval()
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for n, p in ref.named_parameters():
            if "weight_g" in n or "original0" in n:
                p.copy_(torch.rand(p.shape, generator=g) + 0.5)
            else:
                p.copy_(torch.randn(p.shape, generator=g) * 0.2)
        for n, b in ref.named_buffers():
            if n.endswith("codebook.embed"):
                b.copy_(torch.randn(b.shape, generator=g))
    ref.save_pretrained(str(tmp_path))
    return ref


def test_bark_gpts_and_codec_match_transformers(tmp_path):
    ref = _tiny_hf_bark(tmp_path)
    mine = bark_mod.Bark("cpu", weights_dir=str(tmp_path))
    assert mine.weights_source == str(tmp_path)
    assert mine.semantic.cfg.n_embd == 32 and mine.fine.cfg.n_codes_total == 4 and mine.codec.cfg.ratios == (4, 2)
    ids = torch.randint(0, 300, (1, 12))
    with torch.no_grad():
        want = ref.semantic(input_ids=ids).logits[:, -1]
        got = mine.semantic(ids)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()
    # KV-cached decode continues the same sequence
    mine.semantic.new_cache()
    with torch.no_grad():
        mine.semantic(ids[:, :-1], pos=0)
        step = mine.semantic.decode_step(int(ids[0, -1]), ids.shape[1] - 1)
    assert torch.allclose(step, want, atol=1e-4, rtol=1e-4)
    mine.semantic.cache = None
    codes = torch.randint(0, 128, (1, 20, 4))
    with torch.no_grad():
        want = ref.fine_acoustics(codebook_idx=2, input_ids=codes).logits
        got = mine.fine(2, codes)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()
    with torch.no_grad():
        want = ref.codec_decode(codes[:, :, :4].transpose(1, 2))[0]
        got = mine.codec(codes[0].T.contiguous())
    assert got.shape == want.shape == (20 * 8,)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()


def test_bark_generate_runs_from_hf_checkpoint(tmp_path):
    _tiny_hf_bark(tmp_path)
    mine = bark_mod.Bark("cpu", weights_dir=str(tmp_path))
    assert np.isfinite(mine.codec(torch.zeros(4, 5, dtype=torch.long)).numpy()).all()
