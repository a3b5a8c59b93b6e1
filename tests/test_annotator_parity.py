"""Numerical parity of the transformers-backed ControlNet annotators against
transformers itself (installed here; their checkpoints are not): a tiny random
config of each reference class is built, its state dict is loaded into ours
UNCHANGED (same key names as the public safetensors), and the outputs must
match in fp32.  Reference: swarm/controlnet/input_processor.py (depth ->
transformers pipeline("depth-estimation") = DPTForDepthEstimation; seg ->
UperNetForSemanticSegmentation with a ConvNeXt backbone)."""
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")

from chiaswarm_amd.controlnet import annotators as an  # noqa: E402


def _randomize(m, seed=0):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in m.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.2 + (1.0 if n.endswith("layernorm.weight") else 0.0))
        for n, b in m.named_buffers():
            if n.endswith("running_var"):
                b.copy_(torch.rand(b.shape, generator=g) + 0.5)
            elif n.endswith("running_mean"):
                b.copy_(torch.randn(b.shape, generator=g) * 0.1)


def _load(mine, ref, allowed_unexpected=()):
    missing, unexpected = mine.load_state_dict(ref.state_dict(), strict=False)
    assert not missing, missing
    assert all(any(u.startswith(a) for a in allowed_unexpected) for u in unexpected), unexpected


def test_dpt_depth_parity_vs_transformers():
    from transformers import DPTConfig, DPTForDepthEstimation

    cfg = DPTConfig(hidden_size=32, num_hidden_layers=4, num_attention_heads=4, intermediate_size=64,
                    image_size=64, patch_size=16, backbone_out_indices=[0, 1, 2, 3],
                    neck_hidden_sizes=[8, 16, 32, 32], fusion_hidden_size=16, reassemble_factors=[4, 2, 1, 0.5],
                    readout_type="project", is_hybrid=False)
    ref = DPTForDepthEstimation(cfg).eval()
    _randomize(ref)
    mine = an.DPTDepth(c=32, heads=4, mlp=64, n=4, patch=16, image=64, out_indices=(0, 1, 2, 3),
                       neck_sizes=(8, 16, 32, 32), fusion=16).eval()
    _load(mine, ref, ("dpt.layernorm", "dpt.pooler"))
    x = torch.randn(1, 3, 96, 96)  # 6x6 patch grid vs 4x4 trained: exercises the position-embedding resize
    with torch.no_grad():
        want = ref(pixel_values=x).predicted_depth
        got = mine(x)
    assert got.shape == want.shape
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-4), (got - want).abs().max()


def test_upernet_convnext_parity_vs_transformers():
    from transformers import ConvNextConfig, UperNetConfig, UperNetForSemanticSegmentation

    bb = ConvNextConfig(hidden_sizes=[8, 16, 32, 64], depths=[1, 1, 2, 1],
                        out_features=["stage1", "stage2", "stage3", "stage4"])
    cfg = UperNetConfig(backbone_config=bb, hidden_size=32, num_labels=5, pool_scales=[1, 2, 3, 6],
                        use_auxiliary_head=False)
    ref = UperNetForSemanticSegmentation(cfg).eval()
    _randomize(ref)
    mine = an.UperNetConvNext(dims=(8, 16, 32, 64), depths=(1, 1, 2, 1), c=32, num_classes=5).eval()
    _load(mine, ref, ("auxiliary_head",))
    x = torch.randn(1, 3, 64, 96)
    with torch.no_grad():
        want = ref(pixel_values=x).logits
        got = F.interpolate(mine(x), size=x.shape[2:], mode="bilinear", align_corners=False)
    assert got.shape == want.shape
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-4), (got - want).abs().max()
