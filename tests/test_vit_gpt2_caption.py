"""ViT -> GPT-2 captioning (models/vit_gpt2.py) against transformers'
VisionEncoderDecoderModel on tiny random-init configurations (CPU fp32):
weight conversion (Conv1D transposes, fused c_attn splits, the encoder-to-
decoder projection when the widths differ), next-token logits and greedy
decode; the img2txt dispatch; bf16 HIP path on the GPU."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")


def _hf_tiny(dec_dim=32):
    from transformers import GPT2Config, ViTConfig, VisionEncoderDecoderConfig, VisionEncoderDecoderModel

    enc = ViTConfig(hidden_size=32, num_hidden_layers=2, num_attention_heads=2, intermediate_size=64, image_size=32,
                    patch_size=16)
    dec = GPT2Config(vocab_size=100, n_positions=64, n_embd=dec_dim, n_layer=2, n_head=2, bos_token_id=1,
                     eos_token_id=2, add_cross_attention=True, is_decoder=True)
    cfg = VisionEncoderDecoderConfig.from_encoder_decoder_configs(enc, dec)
    cfg.decoder_start_token_id = 1
    cfg.pad_token_id = 2
    torch.manual_seed(0)
    m = VisionEncoderDecoderModel(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "ln" in n.lower() or "norm" in n.lower() or n.endswith("bias"):
                p.add_(torch.randn_like(p) * 0.1)
    return cfg, m


def _ours(cfg, sd):
    from chiaswarm_amd.models.vit_gpt2 import VitGpt2Captioner, VitGpt2Config, convert_hf_vit_gpt2
    from chiaswarm_amd.models.weights import load_into

    m = VitGpt2Captioner(VitGpt2Config.from_hf(cfg.to_dict())).eval()
    load_into(m, convert_hf_vit_gpt2(sd), name="tiny-vit-gpt2")
    return m


def _image():
    from PIL import Image

    return Image.fromarray((np.random.default_rng(0).random((40, 48, 3)) * 255).astype(np.uint8))


@pytest.mark.parametrize("dec_dim", [32, 48])
def test_vit_gpt2_logits_and_generate_match_transformers(dec_dim):
    cfg, hf = _hf_tiny(dec_dim)
    m = _ours(cfg, hf.state_dict())
    assert (m.enc_to_dec_proj is not None) == (dec_dim != 32)
    px = m.preprocess(_image())
    ids = [1, 17, 42, 5]
    with torch.no_grad():
        ref = hf(pixel_values=px.permute(0, 3, 1, 2), decoder_input_ids=torch.tensor([ids])).logits[0, -1]
    got = m.logits(m.image_kv(px), ids)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    dec = [1]
    with torch.no_grad():
        while len(dec) < 10:
            nxt = int(hf(pixel_values=px.permute(0, 3, 1, 2), decoder_input_ids=torch.tensor([dec])).logits[0, -1]
                      .argmax())
            if nxt == 2:
                break
            dec.append(nxt)
    assert m.generate(_image(), [], max_length=10) == dec[1:]


def test_vit_gpt2_dispatch_and_callback():
    from chiaswarm_amd.pipelines.caption import caption_callback, resolve_task

    params = {"model_type": "VisionEncoderDecoderModel", "processor_type": "ViTImageProcessor"}
    assert resolve_task(params, "nlpconnect/vit-gpt2-image-captioning") == "vitgpt2"
    assert resolve_task(None, "nlpconnect/vit-gpt2-image-captioning") == "vitgpt2"
    res, cfg = caption_callback("cpu", "tiny/vit-gpt2", image=_image(), prompt="", parameters=params)
    assert "error" not in cfg, cfg
    assert isinstance(cfg["caption"], str)


@pytest.mark.gpu
def test_vit_gpt2_gpu_matches_fp32(gpu):
    import copy

    from chiaswarm_amd.models.layers import prepare_model

    cfg, hf = _hf_tiny(48)
    m = _ours(cfg, hf.state_dict())
    g = copy.deepcopy(m).to(gpu).to(torch.bfloat16)
    prepare_model(g)
    px = m.preprocess(_image())
    ids = [1, 17, 42, 5]
    ref = m.logits(m.image_kv(px), ids)
    got = g.logits(g.image_kv(px.to(gpu)), ids).cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 3e-2
    assert len(g.generate(_image(), [], max_length=8)) <= 7


def test_vit_gpt2_checkpoint_dir(tmp_path, monkeypatch):
    """A VisionEncoderDecoder checkpoint directory (config.json +
    preprocessor_config.json + safetensors) loads strictly through the
    img2txt loader and captions."""
    import json

    from safetensors.torch import save_file

    from chiaswarm_amd.pipelines.caption import caption_callback, load_vitgpt2

    cfg, hf = _hf_tiny(48)
    root = tmp_path / "tiny" / "vit-gpt2-ckpt"
    root.mkdir(parents=True)
    (root / "config.json").write_text(json.dumps(cfg.to_dict()))
    (root / "preprocessor_config.json").write_text(json.dumps({"image_mean": [0.5, 0.5, 0.5],
                                                                "image_std": [0.5, 0.5, 0.5]}))
    save_file({k: v.clone().contiguous() for k, v in hf.state_dict().items()}, str(root / "model.safetensors"))
    monkeypatch.setenv("SDAAS_MODEL_DIR", str(tmp_path))
    m, _ = load_vitgpt2("tiny/vit-gpt2-ckpt", "cpu")
    assert m.weights_source == str(root) and m.enc_to_dec_proj is not None
    res, out = caption_callback("cpu", "tiny/vit-gpt2-ckpt", image=_image(), prompt="",
                                parameters={"model_type": "VisionEncoderDecoderModel",
                                            "processor_type": "ViTImageProcessor"})
    assert "error" not in out, out
