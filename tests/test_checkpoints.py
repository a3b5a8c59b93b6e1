"""Real-checkpoint fidelity on CPU (no network, no downloaded weights).

* Parity: transformers' own ``CLIPTextModel(WithProjection)``, ``T5EncoderModel``,
  ``BlipForConditionalGeneration`` and ``ClapTextModelWithProjection`` are built
  offline from small configs with random init; their state dicts go through
  safetensors into our modules with the STRICT loader, and fp32 outputs must
  match.  This pins the key layout and the numerics of the models the reference
  loads with ``from_pretrained`` (swarm/diffusion/diffusion_func.py:41-46,
  swarm/captioning/caption_image.py:14-17, swarm/audio/audioldm.py:19-21).
  diffusers itself is not importable here: UNet/VAE parity vs diffusers is
  "parity unpinned"; their key layout is pinned by the round-trip tests below.
* Tokenizer: our CLIP BPE against ``transformers.CLIPTokenizer`` on a BPE
  vocabulary trained here with the ``tokenizers`` library (fixture files).
* Round trip: every model family's state_dict -> safetensors -> a fresh,
  differently seeded model loads with 100 % of keys matched, bitwise equal.
"""
import json
import os

import pytest
import torch
from safetensors.torch import save_file

from chiaswarm_amd.models.weights import CheckpointMismatch, load_component, load_into

transformers = pytest.importorskip("transformers")


def _save(sd, d, name="model.safetensors"):
    os.makedirs(d, exist_ok=True)
    save_file({k: v.detach().contiguous().clone() for k, v in sd.items()}, os.path.join(d, name))
    return d


# --------------------------------------------------------------------------- CLIP
@pytest.mark.parametrize("act,proj,layers", [("quick_gelu", None, 3), ("gelu", 48, 2)])
def test_clip_text_parity_vs_transformers(tmp_path, act, proj, layers):
    from transformers import CLIPTextConfig as HFCfg
    from transformers import CLIPTextModel as HFModel
    from transformers import CLIPTextModelWithProjection as HFProj

    from chiaswarm_amd.models import clip

    hcfg = HFCfg(vocab_size=500, hidden_size=64, intermediate_size=128, num_hidden_layers=layers,
                 num_attention_heads=4, max_position_embeddings=77, hidden_act=act, eos_token_id=499,
                 bos_token_id=498, pad_token_id=1, projection_dim=proj or 64)
    torch.manual_seed(0)
    hf = (HFProj(hcfg) if proj else HFModel(hcfg)).eval()
    d = _save(hf.state_dict(), str(tmp_path / "text_encoder"))
    ours = clip.CLIPTextModel(clip.CLIPTextConfig(vocab_size=500, hidden_size=64, intermediate_size=128,
                                                  num_layers=layers, num_heads=4, act=act, projection_dim=proj,
                                                  eos_token_id=499)).eval()
    rep = load_component(ours, str(tmp_path), "text_encoder")
    assert rep.complete and not rep.unexpected
    ids = torch.randint(2, 490, (3, 77))
    ids[:, 0] = 498
    ids[0, 10], ids[1, 40], ids[2, 76] = 499, 499, 499
    with torch.no_grad():
        out = hf(ids, output_hidden_states=True)
        last, penult, pooled, projd = ours(ids)
    ref_last = out.last_hidden_state
    torch.testing.assert_close(last, ref_last, atol=2e-4, rtol=1e-4)
    torch.testing.assert_close(penult, out.hidden_states[-2], atol=2e-4, rtol=1e-4)
    if proj:
        torch.testing.assert_close(projd, out.text_embeds, atol=2e-4, rtol=1e-4)
    else:
        torch.testing.assert_close(pooled, out.pooler_output, atol=2e-4, rtol=1e-4)


def test_strict_loader_rejects_partial_checkpoints(tmp_path):
    from chiaswarm_amd.models import clip

    m = clip.CLIPTextModel(clip.TINY_TEXT)
    sd = dict(m.state_dict())
    sd.pop("text_model.final_layer_norm.weight")
    with pytest.raises(CheckpointMismatch, match="missing"):
        load_into(clip.CLIPTextModel(clip.TINY_TEXT), sd)
    sd = dict(m.state_dict())
    sd["text_model.encoder.layers.0.bogus.weight"] = torch.zeros(1)
    with pytest.raises(CheckpointMismatch, match="unexpected"):
        load_into(clip.CLIPTextModel(clip.TINY_TEXT), sd)
    sd = dict(m.state_dict())
    sd["text_model.final_layer_norm.weight"] = torch.zeros(7)
    with pytest.raises(CheckpointMismatch, match="shape"):
        load_into(clip.CLIPTextModel(clip.TINY_TEXT), sd)
    rep = load_into(clip.CLIPTextModel(clip.TINY_TEXT), sd, strict=False)
    assert not rep.complete and rep.mismatched


# --------------------------------------------------------------------------- T5
def test_t5_encoder_parity_vs_transformers(tmp_path):
    from transformers import T5Config, T5EncoderModel

    from chiaswarm_amd.models.t5 import T5Config as OurCfg
    from chiaswarm_amd.models.t5 import T5Encoder

    hcfg = T5Config(vocab_size=300, d_model=64, d_kv=16, num_heads=4, d_ff=96, num_layers=2,
                    feed_forward_proj="gated-gelu", relative_attention_num_buckets=32,
                    relative_attention_max_distance=128, dropout_rate=0.0)
    torch.manual_seed(0)
    hf = T5EncoderModel(hcfg).eval()
    d = _save(hf.state_dict(), str(tmp_path / "text_encoder"))
    ours = T5Encoder(OurCfg(vocab=300, d_model=64, d_kv=16, heads=4, d_ff=96, layers=2)).eval()
    rep = load_component(ours, str(tmp_path), "text_encoder")
    assert rep.complete, rep.summary()
    ids = torch.randint(2, 300, (2, 77))
    mask = torch.ones(2, 77, dtype=torch.bool)
    mask[1, 30:] = False
    with torch.no_grad():
        ref = hf(input_ids=ids, attention_mask=mask.long()).last_hidden_state
        got = ours(ids, mask)
    torch.testing.assert_close(got[0], ref[0], atol=3e-4, rtol=1e-4)
    torch.testing.assert_close(got[1, :30], ref[1, :30], atol=3e-4, rtol=1e-4)
    assert d


# --------------------------------------------------------------------------- BLIP
def test_blip_captioner_parity_vs_transformers(tmp_path):
    from PIL import Image
    from transformers import BlipConfig, BlipForConditionalGeneration

    from chiaswarm_amd.models.blip import BlipCaptioner, convert_hf_blip
    from chiaswarm_amd.models.blip import BlipConfig as OurCfg

    hcfg = BlipConfig(text_config=dict(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                       intermediate_size=256, encoder_hidden_size=64, bos_token_id=998,
                                       sep_token_id=999, pad_token_id=0, eos_token_id=999),
                      vision_config=dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                         intermediate_size=256, image_size=64, patch_size=16))
    torch.manual_seed(0)
    hf = BlipForConditionalGeneration(hcfg).eval()
    with torch.no_grad():  # a non-trivial LM head so greedy decode is informative
        hf.text_decoder.cls.predictions.bias.normal_(0, 0.5)
    _save(hf.state_dict(), str(tmp_path))
    ours = BlipCaptioner(OurCfg(image_size=64, vision_dim=64, vision_depth=2, vision_heads=2, text_dim=64,
                                text_depth=2, text_heads=2, vocab=1000, bos_id=998, sep_id=999)).eval()
    from chiaswarm_amd.models.weights import _read_dir

    rep = load_into(ours, convert_hf_blip(_read_dir(str(tmp_path))))
    assert rep.complete, rep.summary()
    img = Image.fromarray((torch.rand(64, 64, 3) * 255).byte().numpy())
    pix = ours.preprocess(img).permute(0, 3, 1, 2)  # NCHW for transformers
    with torch.no_grad():
        ref_vis = hf.vision_model(pixel_values=pix).last_hidden_state
        got_vis = ours.vision_model(ours.preprocess(img))
    torch.testing.assert_close(got_vis, ref_vis, atol=3e-4, rtol=1e-4)
    prefix = [17, 42]
    with torch.no_grad():
        ref = hf.generate(pixel_values=pix, input_ids=torch.tensor([[101] + prefix + [999]]), max_length=12,
                          do_sample=False, num_beams=1)[0].tolist()
    got = ours.generate(img, prefix, max_length=12)
    # transformers returns [bos] + prefix + new tokens (+ sep when it stopped there)
    ref_body = [t for t in ref[1:] if t != 999]
    assert got == ref_body[: len(got)] and len(got) >= len(prefix)


def test_blip_vqa_parity_vs_transformers(tmp_path):
    """BlipForQuestionAnswering: question encoder (bidirectional, cross-attends to
    the image) + answer decoder (causal, cross-attends to the question): strict
    load of the transformers state dict, question encoding and greedy answer
    tokens equal to transformers' generate."""
    from PIL import Image
    from transformers import BlipConfig, BlipForQuestionAnswering

    from chiaswarm_amd.models.blip import BlipConfig as OurCfg
    from chiaswarm_amd.models.blip import BlipVQA, convert_hf_blip_vqa
    from chiaswarm_amd.models.weights import _read_dir

    raw = dict(text_config=dict(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                intermediate_size=256, encoder_hidden_size=64, bos_token_id=998, sep_token_id=999,
                                pad_token_id=0, eos_token_id=999),
               vision_config=dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=2, intermediate_size=256,
                                  image_size=64, patch_size=16))
    hcfg = BlipConfig(**raw)
    torch.manual_seed(0)
    hf = BlipForQuestionAnswering(hcfg).eval()
    with torch.no_grad():
        hf.text_decoder.cls.predictions.bias.normal_(0, 0.5)
    _save(hf.state_dict(), str(tmp_path))
    cfg = OurCfg.from_hf(raw)
    assert cfg.vision_dim == 64 and cfg.bos_id == 998 and cfg.sep_id == 999
    ours = BlipVQA(cfg).eval()
    rep = load_into(ours, convert_hf_blip_vqa(_read_dir(str(tmp_path))))
    assert rep.complete, rep.summary()
    img = Image.fromarray((torch.rand(64, 64, 3) * 255).byte().numpy())
    pix = ours.preprocess(img).permute(0, 3, 1, 2)
    q = [101, 17, 42, 300, 102]
    with torch.no_grad():
        vis = hf.vision_model(pixel_values=pix)[0]
        ref_q = hf.text_encoder(input_ids=torch.tensor([q]), encoder_hidden_states=vis,
                                encoder_attention_mask=torch.ones(vis.shape[:-1], dtype=torch.long))[0]
        got_vis = ours.vision_model(ours.preprocess(img))
        got_q = ours.encoder.run(q, [blk.cross.kv_of(got_vis) for blk in ours.encoder.layers], causal=False)
    torch.testing.assert_close(got_q, ref_q, atol=3e-4, rtol=1e-4)
    with torch.no_grad():
        ref = hf.generate(input_ids=torch.tensor([q]), pixel_values=pix, max_length=10, do_sample=False,
                          num_beams=1)[0].tolist()
    got = ours.answer(img, q, max_length=10)
    ref_body = [t for t in ref[1:] if t != 999]  # transformers: [DEC] + answer (+ [SEP])
    assert got == ref_body


def test_img2txt_class_names(tmp_path):
    """processor_type / model_type pick captioning or VQA; any other class is a
    fatal error naming it (the reference instantiated the named class)."""
    from chiaswarm_amd.pipelines.caption import resolve_task

    assert resolve_task({"processor_type": "BlipProcessor", "model_type": "BlipForConditionalGeneration"},
                        "Salesforce/blip-image-captioning-base") == "caption"
    assert resolve_task({"processor_type": "BlipProcessor", "model_type": "BlipForQuestionAnswering"},
                        "Salesforce/blip-vqa-base") == "vqa"
    assert resolve_task(None, "Salesforce/blip-vqa-base") == "vqa"
    assert resolve_task({"processor_type": "AutoProcessor", "model_type": "GitForCausalLM"}, "microsoft/git-base") \
        == "git"
    with pytest.raises(ValueError, match="Kosmos2ForConditionalGeneration"):
        resolve_task({"processor_type": "AutoProcessor", "model_type": "Kosmos2ForConditionalGeneration"}, "x")
    with pytest.raises(ValueError, match="ViltProcessor"):
        resolve_task({"processor_type": "ViltProcessor", "model_type": "BlipForQuestionAnswering"}, "x")


# --------------------------------------------------------------------------- CLAP
def test_clap_text_parity_vs_transformers(tmp_path):
    from transformers import ClapTextConfig, ClapTextModelWithProjection

    from chiaswarm_amd.models.clap import HF_RENAMES, ClapTextEncoder
    from chiaswarm_amd.models.clap import ClapTextConfig as OurCfg

    hcfg = ClapTextConfig(vocab_size=1000, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                          intermediate_size=128, max_position_embeddings=80, projection_dim=32, pad_token_id=1,
                          type_vocab_size=1, projection_hidden_act="relu")
    torch.manual_seed(0)
    hf = ClapTextModelWithProjection(hcfg).eval()
    _save(hf.state_dict(), str(tmp_path / "text_encoder"))
    ours = ClapTextEncoder(OurCfg(vocab=1000, dim=64, depth=2, heads=2, mlp=128, max_pos=80,
                                  projection_dim=32)).eval()
    rep = load_component(ours, str(tmp_path), "text_encoder", HF_RENAMES)
    assert rep.complete, rep.summary()
    seqs = [[0, 5, 9, 77, 2], [0, 300, 2]]
    with torch.no_grad():
        got = ours(seqs)
        ref = []
        for s in seqs:
            e = hf(input_ids=torch.tensor([s])).text_embeds
            ref.append(e / e.norm(dim=-1, keepdim=True))
    torch.testing.assert_close(got, torch.cat(ref), atol=3e-4, rtol=1e-4)


# --------------------------------------------------------------------------- tokenizer
def _train_bpe(d):
    from tokenizers import Regex, Tokenizer, models, normalizers, pre_tokenizers, trainers

    tok = Tokenizer(models.BPE(end_of_word_suffix="</w>", unk_token="<|endoftext|>"))
    tok.normalizer = normalizers.Sequence([normalizers.NFC(), normalizers.Replace(Regex(r"\s+"), " "),
                                           normalizers.Lowercase()])
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|"""
                                   r"""[^\s\p{L}\p{N}]+"""), behavior="removed", invert=True),
        pre_tokenizers.ByteLevel(add_prefix_space=False)])
    corpus = ["a photograph of an astronaut riding a horse on mars, highly detailed, 8k",
              "a red fox in the snow, digital painting by greg rutkowski",
              "the quick brown fox jumps over the lazy dog 1234567890",
              "portrait of a woman's face, studio lighting, bokeh, 35mm"] * 20
    trainer = trainers.BpeTrainer(vocab_size=400, end_of_word_suffix="</w>",
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  special_tokens=["<|startoftext|>", "<|endoftext|>"])
    tok.train_from_iterator(corpus, trainer)
    m = json.loads(tok.to_str())["model"]
    vocab = dict(m["vocab"])
    # CLIP vocab also holds every byte symbol with the word suffix
    for ch in pre_tokenizers.ByteLevel.alphabet():
        vocab.setdefault(ch + "</w>", len(vocab))
    merges = [" ".join(x) if isinstance(x, list) else x for x in m["merges"]]
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f)
    with open(os.path.join(d, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n" + "\n".join(merges) + "\n")
    return vocab, merges


@pytest.mark.parametrize("pad", ["<|endoftext|>", "!"])
def test_clip_tokenizer_matches_transformers(tmp_path, pad):
    from transformers import CLIPTokenizer as HFTok

    from chiaswarm_amd.models.tokenizer import CLIPTokenizer

    d = str(tmp_path / "tokenizer")
    vocab, merges = _train_bpe(d)
    with open(os.path.join(d, "special_tokens_map.json"), "w") as f:
        json.dump({"bos_token": "<|startoftext|>", "eos_token": "<|endoftext|>", "unk_token": "<|endoftext|>",
                   "pad_token": pad}, f)
    with open(os.path.join(d, "tokenizer_config.json"), "w") as f:
        json.dump({"model_max_length": 77}, f)
    hf = HFTok(vocab=vocab, merges=[tuple(m.split()) for m in merges], pad_token=pad)
    ours = CLIPTokenizer(d, 77)
    assert ours.loaded and ours.pad == vocab[pad]
    texts = ["A photograph of an ASTRONAUT riding a horse", "fox 2024, digital   painting!!",
             "woman's face (bokeh) 35mm", "unseen wörds ünïcode ☃", "", "a " * 100]
    got = ours(texts).tolist()
    ref = hf(texts, padding="max_length", max_length=77, truncation=True)["input_ids"]
    assert got == ref


def test_sd_pipeline_reads_tokenizer_dirs(tmp_path):
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    root = tmp_path / "model"
    _train_bpe(str(root / "tokenizer"))
    with open(root / "tokenizer" / "special_tokens_map.json", "w") as f:
        json.dump({"pad_token": "!"}, f)
    pipe = StableDiffusion("tiny", device="cpu", weights_dir=str(root))
    assert pipe.tokenizers[0].loaded and pipe.tokenizers[0].source.endswith("tokenizer")
    assert pipe.weights_source == "random-init"  # no model tensors in that directory


# --------------------------------------------------------------------------- round trips
def _families():
    from chiaswarm_amd.models import (bark, clap, clip, controlnet, if_unet, rrdbnet, safety, t5, unet, unet3d,
                                      vae, vocoder)

    out = {
        "unet-tiny": lambda: unet.UNet2DConditionModel(unet.TINY),
        "unet-audioldm-tiny": lambda: unet.UNet2DConditionModel(unet.TINY_AUDIOLDM),
        "unet-x4-tiny": lambda: unet.UNet2DConditionModel(unet.TINY_X4),
        "vae-tiny": lambda: vae.AutoencoderKL(vae.TINY_VAE),
        "clip-tiny": lambda: clip.CLIPTextModel(clip.TINY_TEXT),
        "t5-tiny": lambda: t5.T5Encoder(t5.TINY_T5),
        "clap-tiny": lambda: clap.ClapTextEncoder(clap.TINY_CLAP),
        "if-unet-tiny": lambda: if_unet.IFUNet(if_unet.TINY_IF_I),
        "if-unet-ii-tiny": lambda: if_unet.IFUNet(if_unet.TINY_IF_II),
    }
    from chiaswarm_amd.models.unet import TINY

    sem, coarse, fine = bark.bark_configs("tiny")
    out.update({
        "controlnet-tiny": lambda: controlnet.ControlNetModel(TINY),
        "unet3d-tiny": lambda: unet3d.UNet3DConditionModel(unet3d.TINY_T2V),
        "rrdbnet-tiny": lambda: rrdbnet.RRDBNet(**rrdbnet.TINY_RRDB),
        "hifigan-tiny": lambda: vocoder.HifiGan(vocoder.TINY_HIFIGAN),
        "safety-tiny": lambda: safety.SafetyChecker(safety.TINY_SAFETY),
        "encodec-tiny": lambda: bark.EncodecDecoder(bark.TINY_ENCODEC),
    })
    if sem is not None:
        out["bark-semantic-tiny"] = lambda: bark.BarkCausalGPT(sem)
        out["bark-fine-tiny"] = lambda: bark.BarkFineGPT(fine)
    return out


@pytest.mark.parametrize("name", sorted(_families()))
def test_state_dict_round_trip(tmp_path, name):
    from chiaswarm_amd.models.layers import init_random_

    make = _families()[name]
    try:
        a = make()
    except TypeError:
        pytest.skip(f"{name}: constructor signature differs")
    init_random_(a, seed=1)
    for n, p in a.named_parameters():  # make norms/biases non-trivial too
        if p.dim() < 2:
            with torch.no_grad():
                p.add_(torch.randn(p.shape, generator=torch.Generator().manual_seed(len(n))) * 0.1)
    _save(a.state_dict(), str(tmp_path / "m"))
    b = make()
    init_random_(b, seed=2)
    rep = load_component(b, str(tmp_path), "m")
    assert rep.complete and not rep.unexpected, rep.summary()
    sa, sb = a.state_dict(), b.state_dict()
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
