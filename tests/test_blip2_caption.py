"""BLIP-2 (OPT) captioning (models/blip2.py) against transformers'
Blip2ForConditionalGeneration on a tiny random-init configuration (CPU fp32):
weight conversion (fused vision qkv bias and the original q_bias / v_bias
form), next-token logits over [projected queries; </s>; prompt], and greedy
decode against transformers' forward run token by token."""
import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")

NQ, IMG_TOK = 4, 99


def _hf_tiny():
    from transformers import Blip2Config, Blip2ForConditionalGeneration

    vis = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2, image_size=28,
               patch_size=14)
    qf = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2,
              encoder_hidden_size=32, cross_attention_frequency=2)
    txt = dict(model_type="opt", hidden_size=32, ffn_dim=64, num_hidden_layers=2, num_attention_heads=2,
               vocab_size=100, max_position_embeddings=64, word_embed_proj_dim=32, bos_token_id=2, eos_token_id=2,
               pad_token_id=1)
    cfg = Blip2Config(vision_config=vis, qformer_config=qf, text_config=txt, num_query_tokens=NQ,
                      image_token_index=IMG_TOK)
    torch.manual_seed(0)
    m = Blip2ForConditionalGeneration(cfg).eval()
    with torch.no_grad():  # non-trivial LayerNorms, biases and query tokens
        for n, p in m.named_parameters():
            if "norm" in n.lower() or n.endswith("bias") or "query_tokens" in n:
                p.add_(torch.randn_like(p) * 0.1)
            elif p.dim() >= 2 and p.std() < 1e-3:
                p.normal_(0, 0.05)
    return cfg, m


def _ours(hf_cfg, sd):
    from chiaswarm_amd.models.blip2 import Blip2Captioner, Blip2Config, convert_hf_blip2
    from chiaswarm_amd.models.weights import load_into

    m = Blip2Captioner(Blip2Config.from_hf(hf_cfg.to_dict())).eval()
    load_into(m, convert_hf_blip2(sd), name="tiny-blip2")
    return m


def _image():
    from PIL import Image

    return Image.fromarray((np.random.default_rng(0).random((40, 48, 3)) * 255).astype(np.uint8))


def test_blip2_logits_and_generate_match_transformers():
    hf_cfg, hf = _hf_tiny()
    m = _ours(hf_cfg, hf.state_dict())
    img = _image()
    px = m.preprocess(img)
    prompt = [17, 42, 5]

    def hf_logits(text_ids):
        ids = torch.tensor([[IMG_TOK] * NQ + text_ids])
        return hf(pixel_values=px.permute(0, 3, 1, 2), input_ids=ids).logits[0, -1]

    with torch.no_grad():
        ref = hf_logits([2] + prompt)
    got = m.text_logits(m.image_prefix(px), [2] + prompt)
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    ids = [2]
    with torch.no_grad():
        while len(ids) < 10:
            nxt = int(hf_logits(ids).argmax())
            if nxt == 2:
                break
            ids.append(nxt)
    assert m.generate(img, [], max_length=10) == ids[1:]


def test_blip2_original_qv_bias_form():
    """Original hub checkpoints carry q_bias / v_bias instead of a fused qkv bias."""
    hf_cfg, hf = _hf_tiny()
    sd = dict(hf.state_dict())
    for k in [k for k in sd if k.endswith("self_attn.qkv.bias")]:
        q, kb, v = sd.pop(k).chunk(3, 0)
        sd[k.replace("qkv.bias", "q_bias")] = q
        sd[k.replace("qkv.bias", "v_bias")] = v
    m = _ours(hf_cfg, sd)
    ref = _ours(hf_cfg, hf.state_dict())
    px = m.preprocess(_image())
    for blk_a, blk_b in zip(m.vision_model.layers, ref.vision_model.layers):
        assert torch.equal(blk_a.attn.q.bias, blk_b.attn.q.bias) and torch.equal(blk_a.attn.v.bias, blk_b.attn.v.bias)
    # the fused form's k bias is whatever the checkpoint holds; the original form has none
    assert torch.count_nonzero(m.vision_model.layers[0].attn.k.bias) == 0
    assert m.image_prefix(px).shape == (1, NQ, 32)


def test_blip2_other_lm_refused():
    from chiaswarm_amd.models.blip2 import Blip2Config

    with pytest.raises(ValueError, match="llama"):
        Blip2Config.from_hf({"text_config": {"model_type": "llama"}})


@pytest.mark.gpu
@pytest.mark.parametrize("lm", ["opt", "t5", "instruct-llama"])
def test_blip2_gpu_matches_fp32(gpu, lm):
    """bf16 HIP path against the fp32 CPU model: next-token logits (OPT) /
    decoder logits over the encoder states (Flan-T5)."""
    import copy

    from chiaswarm_amd.models.layers import prepare_model

    hf_cfg, hf = _hf_tiny() if lm == "opt" else (_hf_tiny_t5(False) if lm == "t5" else _hf_tiny_instruct("llama"))
    m = _ours(hf_cfg, hf.state_dict())
    g = copy.deepcopy(m).to(gpu).to(torch.bfloat16)
    prepare_model(g)
    px = m.preprocess(_image())
    if lm == "opt":
        ids = [2, 17, 42, 5]
        ref = m.text_logits(m.image_prefix(px), ids)
        got = g.text_logits(g.image_prefix(px.to(gpu)), ids).cpu()
    elif lm == "t5":
        ref = m.t5.decode_logits(m.t5_encoder_states(m.image_prefix(px), [17, 42]), [0, 9, 33])
        got = g.t5.decode_logits(g.t5_encoder_states(g.image_prefix(px.to(gpu)), [17, 42]), [0, 9, 33]).cpu()
    else:
        qids, ids = [3, 11, 25, 4], torch.tensor([[1, 17, 42, 5]])
        ref = m.llama.last_logits(torch.cat([m.image_prefix(px, qids), m.llama.model.embed_tokens(ids)], 1))
        pre = g.image_prefix(px.to(gpu), qids)
        got = g.llama.last_logits(torch.cat([pre, g.llama.model.embed_tokens(ids.to(gpu))], 1)).cpu()
    assert ((got - ref).norm() / ref.norm()).item() < 3e-2
    assert len(g.generate(_image(), [], max_length=8)) <= 8


def test_blip2_dispatch_and_callback():
    """img2txt job naming Blip2ForConditionalGeneration / Blip2Processor on the
    tiny random-init geometry: a caption, no error; GPT-2 BPE decode round trip."""
    from chiaswarm_amd.models.tokenizer import ByteBPETokenizer
    from chiaswarm_amd.pipelines.caption import caption_callback, resolve_task

    params = {"model_type": "Blip2ForConditionalGeneration", "processor_type": "Blip2Processor"}
    assert resolve_task(params, "Salesforce/blip2-opt-2.7b") == "blip2"
    assert resolve_task(None, "Salesforce/blip2-opt-2.7b") == "blip2"
    res, cfg = caption_callback("cpu", "tiny/blip2", image=_image(), prompt="Question: what is it? Answer:",
                                parameters=params)
    assert "error" not in cfg, cfg
    assert isinstance(cfg["caption"], str) and "primary" in res
    assert ByteBPETokenizer(None, bos=2, eos=2, pad=1).decode([2, 7, 9, 2]) == "w7 w9"


def test_gpt2_bpe_decode_roundtrip(tmp_path):
    """decode(encode(text)) == text on a small byte-level vocabulary."""
    import json

    from chiaswarm_amd.models.tokenizer import ByteBPETokenizer, _bytes_to_unicode

    be = _bytes_to_unicode()
    vocab = {c: i + 4 for i, c in enumerate(be.values())}
    vocab.update({"<s>": 0, "<pad>": 1, "</s>": 2, "<unk>": 3})
    merges = ["Ġ t", "h e", "Ġt he"]
    for m in merges:
        vocab.setdefault(m.replace(" ", ""), len(vocab))
    (tmp_path / "vocab.json").write_text(json.dumps(vocab))
    (tmp_path / "merges.txt").write_text("#version: 0.2\n" + "\n".join(merges) + "\n")
    tok = ByteBPETokenizer(str(tmp_path), bos=2, eos=2, pad=1)
    text = "two cats on the couch, café"
    ids = tok.encode(text)
    assert vocab["Ġthe"] in ids
    assert tok.decode([2] + ids) == text


def _hf_tiny_t5(tied=False):
    from transformers import Blip2Config, Blip2ForConditionalGeneration

    vis = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2, image_size=28,
               patch_size=14)
    qf = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2,
              encoder_hidden_size=32, cross_attention_frequency=2)
    txt = dict(model_type="t5", vocab_size=100, d_model=32, d_kv=16, num_heads=2, d_ff=64, num_layers=2,
               num_decoder_layers=3, feed_forward_proj="gated-gelu", tie_word_embeddings=tied,
               decoder_start_token_id=0, eos_token_id=1, pad_token_id=0)
    cfg = Blip2Config(vision_config=vis, qformer_config=qf, text_config=txt, num_query_tokens=NQ,
                      image_token_index=IMG_TOK)
    torch.manual_seed(1)
    m = Blip2ForConditionalGeneration(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n.lower() or n.endswith("bias") or "query_tokens" in n:
                p.add_(torch.randn_like(p) * 0.1)
            elif p.dim() >= 2 and p.std() < 1e-3:
                p.normal_(0, 0.05)
    return cfg, m


@pytest.mark.parametrize("tied", [False, True])
def test_blip2_flan_t5_logits_and_generate_match_transformers(tied):
    """Flan-T5 language model: the encoder over [queries; prompt; </s>], the
    decoder from the start token; logits and greedy decode vs transformers."""
    hf_cfg, hf = _hf_tiny_t5(tied)
    m = _ours(hf_cfg, hf.state_dict())
    assert m.cfg.lm_type == "t5" and m.cfg.t5_tied == tied
    img = _image()
    px = m.preprocess(img)
    prompt = [17, 42, 5]
    enc_ids = torch.tensor([[IMG_TOK] * NQ + prompt + [1]])

    def hf_logits(dec):
        return hf(pixel_values=px.permute(0, 3, 1, 2), input_ids=enc_ids,
                  decoder_input_ids=torch.tensor([dec])).logits[0, -1]

    with torch.no_grad():
        ref = hf_logits([0, 9, 33])
    enc = m.t5_encoder_states(m.image_prefix(px), prompt)
    got = m.t5.decode_logits(enc, [0, 9, 33])
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    dec = [0]
    with torch.no_grad():
        while len(dec) < 10:
            nxt = int(hf_logits(dec).argmax())
            if nxt == 1:
                break
            dec.append(nxt)
    assert m.generate(img, prompt, max_length=10) == dec[1:]


def test_blip2_t5_v10_refused():
    from chiaswarm_amd.models.blip2 import Blip2Config

    with pytest.raises(ValueError, match="feed_forward_proj"):
        Blip2Config.from_hf({"text_config": {"model_type": "t5", "feed_forward_proj": "relu"}})


def test_blip2_flan_t5_callback(tmp_path, monkeypatch):
    """img2txt job on a BLIP-2 Flan-T5 checkpoint directory (config.json of the
    tiny geometry, its weights as safetensors): loads strictly and captions."""
    import json

    from safetensors.torch import save_file

    from chiaswarm_amd.pipelines.caption import caption_callback

    hf_cfg, hf = _hf_tiny_t5(False)
    root = tmp_path / "tiny" / "blip2-flan-t5"
    root.mkdir(parents=True)
    (root / "config.json").write_text(json.dumps(hf_cfg.to_dict()))
    save_file({k: v.clone().contiguous() for k, v in hf.state_dict().items()}, str(root / "model.safetensors"))
    monkeypatch.setenv("SDAAS_MODEL_DIR", str(tmp_path))
    res, cfg = caption_callback("cpu", "tiny/blip2-flan-t5", image=_image(), prompt="",
                                parameters={"model_type": "Blip2ForConditionalGeneration",
                                            "processor_type": "Blip2Processor"})
    assert "error" not in cfg, cfg
    assert isinstance(cfg["caption"], str)
    from chiaswarm_amd.pipelines.caption import load_blip2

    m, _ = load_blip2("tiny/blip2-flan-t5", "cpu")
    assert m.cfg.lm_type == "t5" and m.weights_source == str(root)


def _hf_tiny_instruct(lm):
    from transformers import InstructBlipConfig, InstructBlipForConditionalGeneration

    vis = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2, image_size=28,
               patch_size=14)
    qf = dict(hidden_size=32, intermediate_size=64, num_hidden_layers=2, num_attention_heads=2,
              encoder_hidden_size=32, cross_attention_frequency=2, vocab_size=60, max_position_embeddings=32)
    if lm == "t5":
        txt = dict(model_type="t5", vocab_size=100, d_model=32, d_kv=16, num_heads=2, d_ff=64, num_layers=2,
                   num_decoder_layers=2, feed_forward_proj="gated-gelu", tie_word_embeddings=False,
                   decoder_start_token_id=0, eos_token_id=1, pad_token_id=0)
    else:
        txt = dict(model_type="llama", vocab_size=100, hidden_size=32, intermediate_size=64, num_hidden_layers=2,
                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=64, bos_token_id=1,
                   eos_token_id=2, pad_token_id=0)
    cfg = InstructBlipConfig(vision_config=vis, qformer_config=qf, text_config=txt, num_query_tokens=NQ,
                             image_token_index=IMG_TOK)
    torch.manual_seed(3)
    m = InstructBlipForConditionalGeneration(cfg).eval()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n.lower() or n.endswith("bias") or "query_tokens" in n:
                p.add_(torch.randn_like(p) * 0.1)
            elif p.dim() >= 2 and p.std() < 1e-3:
                p.normal_(0, 0.05)
    return cfg, m


@pytest.mark.parametrize("lm", ["t5", "llama"])
def test_instructblip_logits_and_generate_match_transformers(lm):
    """InstructBLIP (Flan-T5 / Vicuna-LLaMA language model): the instruction's
    Q-Former tokens join the queries; logits and greedy decode vs transformers."""
    cfg, hf = _hf_tiny_instruct(lm)
    m = _ours(cfg, hf.state_dict())
    assert m.cfg.instruct and m.cfg.lm_type == lm
    img = _image()
    px = m.preprocess(img)
    qids = [3, 11, 25, 4]  # Q-Former tokens of the instruction ([CLS] ... [SEP])
    prompt = [17, 42, 5]
    pv = px.permute(0, 3, 1, 2)
    if lm == "t5":
        enc_ids = torch.tensor([[IMG_TOK] * NQ + prompt + [1]])

        def hf_logits(dec):
            return hf(pixel_values=pv, qformer_input_ids=torch.tensor([qids]), input_ids=enc_ids,
                      decoder_input_ids=torch.tensor([dec])).logits[0, -1]

        with torch.no_grad():
            ref = hf_logits([0, 9, 33])
        got = m.t5.decode_logits(m.t5_encoder_states(m.image_prefix(px, qids), prompt), [0, 9, 33])
        start, eos = [0], 1
    else:
        def hf_logits(dec):
            ids = torch.tensor([[IMG_TOK] * NQ + [1] + prompt + dec])
            return hf(pixel_values=pv, qformer_input_ids=torch.tensor([qids]), input_ids=ids).logits[0, -1]

        with torch.no_grad():
            ref = hf_logits([9, 33])
        pre = m.image_prefix(px, qids)
        emb = m.llama.model.embed_tokens
        got = m.llama.last_logits(torch.cat([pre, emb(torch.tensor([[1] + prompt + [9, 33]]))], 1))
        start, eos = [], 2
    assert torch.allclose(got, ref, atol=1e-4, rtol=1e-4), (got - ref).abs().max()
    dec = list(start)
    with torch.no_grad():
        while len(dec) < 8:
            nxt = int(hf_logits(dec).argmax())
            if nxt == eos:
                break
            dec.append(nxt)
    assert m.generate(img, prompt, max_length=8 if lm == "t5" else 9, qtext_ids=qids) == dec[len(start):]


def test_instructblip_vicuna_callback(tmp_path, monkeypatch):
    """img2txt job naming InstructBlipForConditionalGeneration on a Vicuna-LLaMA
    checkpoint directory (config.json + safetensors): strict load, caption."""
    import json

    from safetensors.torch import save_file

    from chiaswarm_amd.pipelines.caption import caption_callback, load_blip2

    cfg, hf = _hf_tiny_instruct("llama")
    root = tmp_path / "tiny" / "instructblip-vicuna"
    root.mkdir(parents=True)
    (root / "config.json").write_text(json.dumps(cfg.to_dict()))
    save_file({k: v.clone().contiguous() for k, v in hf.state_dict().items()}, str(root / "model.safetensors"))
    monkeypatch.setenv("SDAAS_MODEL_DIR", str(tmp_path))
    m, _ = load_blip2("tiny/instructblip-vicuna", "cpu")
    assert m.cfg.instruct and m.cfg.lm_type == "llama" and m.weights_source == str(root)
    res, out = caption_callback("cpu", "tiny/instructblip-vicuna", image=_image(), prompt="what is in the picture?",
                                parameters={"model_type": "InstructBlipForConditionalGeneration",
                                            "processor_type": "InstructBlipProcessor"})
    assert "error" not in out, out
    assert isinstance(out["caption"], str)
