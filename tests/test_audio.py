"""Audio stack: polyphase transposed conv, HiFi-GAN vocoder vs an independent
PyTorch transcription of the SpeechT5HifiGan forward, CLAP text tower, AudioLDM
end to end + job callback (reference swarm/audio/audioldm.py)."""
import base64

import pytest
import torch
import torch.nn.functional as F

from chiaswarm_amd import ops
from chiaswarm_amd.models.vocoder import TINY_HIFIGAN, HifiGan


@pytest.mark.parametrize("L,cin,cout,k,s,p", [(7, 8, 16, 16, 5, 5), (9, 16, 8, 16, 4, 6), (5, 8, 8, 8, 2, 3),
                                              (6, 8, 8, 4, 2, 1), (4, 8, 8, 3, 2, 0), (5, 8, 8, 5, 3, 1)])
@pytest.mark.parametrize("batch", [1, 2])
def test_polyphase_conv_transpose1d(L, cin, cout, k, s, p, batch):
    torch.manual_seed(0)
    x, w, b = torch.randn(batch, L, cin), torch.randn(cin, cout, k), torch.randn(cout)
    ref = F.conv_transpose1d(x.transpose(1, 2), w, b, stride=s, padding=p).transpose(1, 2)
    lout = ref.shape[1]
    y = ops._conv_transpose1d_polyphase(x, ops.pack_conv_transpose1d(w, s, p), b, s, lout, cout)
    assert y.shape == ref.shape
    assert (y - ref).abs().max().item() < 1e-4


def _hifigan_ref(m: HifiGan, mel):
    """Plain transcription of transformers' SpeechT5HifiGan.forward (NCL layout)."""
    sd = {k: v.float() for k, v in m.state_dict().items()}
    cfg = m.cfg
    x = ((mel - sd["mean"]) / sd["scale"]).transpose(1, 2)
    x = F.conv1d(x, sd["conv_pre.weight"], sd["conv_pre.bias"], padding=3)
    nk = len(cfg.resblock_kernel_sizes)
    for i, (u, k) in enumerate(zip(cfg.upsample_rates, cfg.upsample_kernel_sizes)):
        x = F.leaky_relu(x, 0.1)
        x = F.conv_transpose1d(x, sd[f"upsampler.{i}.weight"], sd[f"upsampler.{i}.bias"], stride=u,
                               padding=(k - u) // 2)
        acc = 0
        for j in range(nk):
            rk, rd = cfg.resblock_kernel_sizes[j], cfg.resblock_dilation_sizes[j]
            h = x
            for n, d in enumerate(rd):
                pre = f"resblocks.{i * nk + j}."
                t = F.leaky_relu(h, 0.1)
                t = F.conv1d(t, sd[pre + f"convs1.{n}.weight"], sd[pre + f"convs1.{n}.bias"], dilation=d,
                             padding=d * (rk - 1) // 2)
                t = F.leaky_relu(t, 0.1)
                t = F.conv1d(t, sd[pre + f"convs2.{n}.weight"], sd[pre + f"convs2.{n}.bias"], padding=(rk - 1) // 2)
                h = t + h
            acc = acc + h
        x = acc / nk
    x = F.leaky_relu(x)
    x = torch.tanh(F.conv1d(x, sd["conv_post.weight"], sd["conv_post.bias"], padding=3))
    return x[:, 0]


def test_hifigan_matches_reference_forward():
    torch.manual_seed(0)
    m = HifiGan(TINY_HIFIGAN).eval()
    for p in m.parameters():
        p.data.normal_(0, 0.15)
    m.mean.normal_()
    m.scale.uniform_(0.5, 2.0)
    mel = torch.randn(2, 24, TINY_HIFIGAN.model_in_dim)
    y = m(mel)
    ref = _hifigan_ref(m, mel)
    assert y.shape == (2, 24 * TINY_HIFIGAN.hop)
    assert (y - ref).abs().max().item() < 1e-4


def test_clap_text_encoder_normalised_and_deterministic():
    from chiaswarm_amd.models.clap import TINY_CLAP, ClapTextEncoder
    from chiaswarm_amd.models.tokenizer import ByteBPETokenizer

    torch.manual_seed(0)
    enc = ClapTextEncoder(TINY_CLAP).eval()
    tok = ByteBPETokenizer(None, vocab_size=TINY_CLAP.vocab)
    ids = tok(["a dog barking", "rain on a tin roof"])
    assert ids[0][0] == 0 and ids[0][-1] == 2
    e = enc(ids)
    assert e.shape == (2, TINY_CLAP.projection_dim)
    assert torch.allclose(e.norm(dim=-1), torch.ones(2), atol=1e-5)
    assert torch.equal(e, enc(ids))
    assert not torch.allclose(e[0], e[1])


def test_byte_bpe_with_vocab(tmp_path):
    import json

    from chiaswarm_amd.models.tokenizer import ByteBPETokenizer

    vocab = {"<s>": 0, "<pad>": 1, "</s>": 2, "a": 3, "Ġ": 4, "d": 5, "o": 6, "g": 7, "do": 8, "dog": 9, "Ġdog": 10}
    (tmp_path / "vocab.json").write_text(json.dumps(vocab))
    (tmp_path / "merges.txt").write_text("#version: 0.2\nd o\ndo g\nĠ dog\n")
    tok = ByteBPETokenizer(str(tmp_path), vocab_size=11)
    assert tok("a dog") == [[0, 3, 10, 2]]


def test_audioldm_pipeline_and_callback():
    from chiaswarm_amd.pipelines import audio

    pipe = audio.AudioLDM("cpu", tiny=True)
    a = pipe(prompt="a dog barking", num_inference_steps=3, audio_length_in_s=0.32,
             generator=torch.Generator().manual_seed(0))
    assert a.shape == (1, int(0.32 * 16000))
    b = pipe(prompt="a dog barking", num_inference_steps=3, audio_length_in_s=0.32,
             generator=torch.Generator().manual_seed(0))
    assert (a == b).all()
    assert abs(a).max() <= 1.0
    res, cfg = audio.txt2audio_diffusion_callback("cpu", "tiny-audioldm", prompt="thunder",
                                                  num_inference_steps=2, audio_length_in_s=0.16)
    art = res["primary"]
    assert art["content_type"] in ("audio/mpeg", "audio/wav")
    blob = base64.b64decode(art["blob"])
    if art["content_type"] == "audio/wav":
        assert blob[:4] == b"RIFF" and len(blob) == 44 + 2 * int(0.16 * 16000)
    assert cfg["_class_name"] == "AudioLDMPipeline"
