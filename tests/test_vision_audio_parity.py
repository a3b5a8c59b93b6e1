"""Parity of the safety checker's CLIP vision tower and the AudioLDM HiFi-GAN
vocoder against transformers (installed here; the checkpoints are not): a
tiny random reference model's state dict goes through OUR checkpoint loaders
unchanged and the outputs must match in fp32.  References:
swarm/diffusion/diffusion_func.py:96-111 (safety checker output),
swarm/audio/audioldm.py:25 (AudioLDMPipeline -> SpeechT5HifiGan)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from chiaswarm_amd.models import safety, vocoder  # noqa: E402


def _randomize(m, seed=0, scale=0.2):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * scale + (1.0 if "norm" in n and n.endswith("weight") else 0.0))


def test_safety_tower_parity_vs_clip_vision_with_projection(tmp_path):
    from safetensors.torch import save_file
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection

    cfg = CLIPVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=2,
                           image_size=28, patch_size=14, projection_dim=32, hidden_act="quick_gelu")
    ref = CLIPVisionModelWithProjection(cfg).eval()
    _randomize(ref)
    # StableDiffusionSafetyChecker layout: CLIPVisionModel nested under vision_model.
    sd = {("vision_model." + k if k.startswith("vision_model.") else k): v for k, v in ref.state_dict().items()}
    sd.update(concept_embeds=torch.randn(17, 32), special_care_embeds=torch.randn(3, 32),
              concept_embeds_weights=torch.rand(17), special_care_embeds_weights=torch.rand(3))
    save_file({k: v.contiguous() for k, v in sd.items()}, str(tmp_path / "model.safetensors"))
    mine = safety.load_safety_checker("cpu", str(tmp_path), tiny=True)
    x = torch.randn(2, 3, 28, 28)
    with torch.no_grad():
        want = ref(pixel_values=x).image_embeds
        got = mine.image_embeds(x.permute(0, 2, 3, 1).contiguous())
    assert torch.allclose(got.float(), want, atol=1e-4, rtol=1e-4), (got - want).abs().max()


def test_safety_flag_rule_matches_diffusers_loop():
    """The vectorised rule equals diffusers' per-image loop (special-care hit
    lowers every concept threshold by 0.01; scores rounded to 3 decimals)."""
    m = safety.SafetyChecker(safety.TINY_SAFETY)
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        m.concept_embeds.copy_(torch.randn(17, 32, generator=g))
        m.special_care_embeds.copy_(torch.randn(3, 32, generator=g))
        m.concept_embeds_weights.fill_(0.2)
        m.special_care_embeds_weights.fill_(0.25)
    emb = torch.randn(64, 32, generator=g)
    got = m.flags(emb)
    e = torch.nn.functional.normalize(emb, dim=-1)
    cos_c = e @ torch.nn.functional.normalize(m.concept_embeds.detach(), dim=-1).t()
    cos_s = e @ torch.nn.functional.normalize(m.special_care_embeds.detach(), dim=-1).t()
    want = []
    for i in range(64):
        adj = 0.0
        for j in range(3):
            if round(float(cos_s[i, j]) - 0.25 + adj, 3) > 0:
                adj = 0.01
        want.append(any(round(float(cos_c[i, j]) - 0.2 + adj, 3) > 0 for j in range(17)))
    assert got.tolist() == want and any(want) and not all(want)


def test_hifigan_parity_vs_speecht5_hifigan():
    from transformers import SpeechT5HifiGan, SpeechT5HifiGanConfig

    hc = vocoder.TINY_HIFIGAN
    cfg = SpeechT5HifiGanConfig(model_in_dim=hc.model_in_dim, sampling_rate=16000,
                                upsample_initial_channel=hc.upsample_initial_channel,
                                upsample_rates=list(hc.upsample_rates), upsample_kernel_sizes=list(hc.upsample_kernel_sizes),
                                resblock_kernel_sizes=list(hc.resblock_kernel_sizes),
                                resblock_dilation_sizes=[list(d) for d in hc.resblock_dilation_sizes],
                                normalize_before=True)
    ref = SpeechT5HifiGan(cfg).eval()
    _randomize(ref, scale=0.3)
    with torch.no_grad():
        ref.mean.copy_(torch.randn(hc.model_in_dim))
        ref.scale.copy_(torch.rand(hc.model_in_dim) + 0.5)
    mine = vocoder.HifiGan(hc).eval()
    missing, unexpected = mine.load_state_dict(ref.state_dict(), strict=True)
    mel = torch.randn(1, 12, hc.model_in_dim)
    with torch.no_grad():
        want = ref(mel)
        got = mine(mel)
    assert got.shape[-1] == want.shape[-1], (got.shape, want.shape)
    assert torch.allclose(got.reshape(want.shape), want, atol=1e-4, rtol=1e-4), (got - want).abs().max()
