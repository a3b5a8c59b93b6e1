"""GIT captioning (models/git.py) against transformers' GitForCausalLM on a
tiny random-init configuration (CPU fp32): weight conversion, next-token
logits over the [image; text] sequence with the image K/V computed once, and
greedy generate.  The captioning dispatch accepts GitForCausalLM."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")


def _hf_tiny():
    from transformers import GitConfig as HFConfig
    from transformers import GitForCausalLM

    vis = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2, image_size=32,
               patch_size=16)
    cfg = HFConfig(vision_config=vis, vocab_size=100, hidden_size=32, intermediate_size=64, num_hidden_layers=2,
                   num_attention_heads=2, max_position_embeddings=64, bos_token_id=1, eos_token_id=2, pad_token_id=0)
    torch.manual_seed(0)
    m = GitForCausalLM(cfg).eval()
    with torch.no_grad():  # non-trivial LayerNorms and biases
        for n, p in m.named_parameters():
            if "LayerNorm" in n or "layer_norm" in n or "layrnorm" in n or n.endswith("bias"):
                p.add_(torch.randn_like(p) * 0.1)
    return cfg, m


def _ours(hf_cfg, hf):
    from chiaswarm_amd.models.git import GitCaptioner, GitConfig, convert_hf_git
    from chiaswarm_amd.models.weights import load_into

    cfg = GitConfig.from_hf(hf_cfg.to_dict())
    m = GitCaptioner(cfg).eval()
    load_into(m, convert_hf_git(hf.state_dict()), name="tiny-git")
    return m


def test_git_logits_and_generate_match_transformers():
    from PIL import Image

    hf_cfg, hf = _hf_tiny()
    m = _ours(hf_cfg, hf)
    rng = np.random.default_rng(0)
    img = Image.fromarray((rng.random((40, 48, 3)) * 255).astype(np.uint8))
    px = m.preprocess(img)  # NHWC
    ids = [1, 17, 42, 5]
    with torch.no_grad():
        ref = hf(input_ids=torch.tensor([ids]), pixel_values=px.permute(0, 3, 1, 2)).logits[0, -1]
        got = m.text_logits(m.image_kv(px), ids)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    # greedy decode by re-running transformers' full forward (its cached
    # generate() path handles the image prefix differently in this version and
    # disagrees with its own forward; the forward is the model's definition)
    hf_ids = [hf_cfg.bos_token_id]
    with torch.no_grad():
        while len(hf_ids) < 12:
            nxt = int(hf(input_ids=torch.tensor([hf_ids]), pixel_values=px.permute(0, 3, 1, 2)).logits[0, -1].argmax())
            if nxt == hf_cfg.eos_token_id:
                break
            hf_ids.append(nxt)
    ours = [hf_cfg.bos_token_id] + m.generate(img, [], max_length=12)
    assert ours == hf_ids


def test_caption_dispatch_accepts_git():
    from chiaswarm_amd.pipelines.caption import resolve_task

    assert resolve_task({"model_type": "GitForCausalLM", "processor_type": "GitProcessor"}, "microsoft/git-base") \
        == "git"
    assert resolve_task({"model_type": "GitForCausalLM", "processor_type": "AutoProcessor"}, "x") == "git"
    with pytest.raises(ValueError):
        resolve_task({"model_type": "Kosmos2ForConditionalGeneration"}, "microsoft/kosmos-2-patch14-224")


def test_caption_callback_git_end_to_end():
    """img2txt job with model_type GitForCausalLM on the tiny random-init
    geometry: a text artifact and pipeline_config.caption, no error."""
    from PIL import Image

    from chiaswarm_amd.pipelines.caption import caption_callback

    img = Image.fromarray((np.random.default_rng(1).random((40, 40, 3)) * 255).astype(np.uint8))
    res, cfg = caption_callback("cpu", "tiny-git", image=img, prompt="",
                                parameters={"model_type": "GitForCausalLM", "processor_type": "GitProcessor"})
    assert "error" not in cfg, cfg
    assert isinstance(cfg["caption"], str) and "primary" in res


@pytest.mark.gpu
def test_git_gpu_matches_fp32(gpu):
    """bf16 HIP path (GEMMs + bottom-right causal attention over [image; text])
    against the fp32 CPU model: next-token logits."""
    import copy

    from PIL import Image

    hf_cfg, hf = _hf_tiny()
    m = _ours(hf_cfg, hf)
    g = copy.deepcopy(m).to(gpu).to(torch.bfloat16)
    from chiaswarm_amd.models.layers import prepare_model

    prepare_model(g)
    img = Image.fromarray((np.random.default_rng(2).random((40, 48, 3)) * 255).astype(np.uint8))
    px = m.preprocess(img)
    ids = [1, 17, 42, 5, 9]
    ref = m.text_logits(m.image_kv(px), ids)
    got = g.text_logits(g.image_kv(px.to(gpu)), ids).cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 3e-2
    assert len(g.generate(img, [], max_length=8)) <= 7
