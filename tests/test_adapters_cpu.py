"""LoRA / textual-inversion adapters on a resident pipeline (reference:
swarm/diffusion/diffusion_func.py:48-68, which reloads the whole pipeline per job).

Here the resident model is patched for one job and must come back BIT FOR BIT
afterwards, and every captured graph must be dropped on each change."""
import torch
from safetensors.torch import save_file

from chiaswarm_amd.models.lora import (load_lora, load_textual_inversion, unload_lora,
                                       unload_textual_inversion)
from chiaswarm_amd.pipelines.sd import StableDiffusion


def _pipe(dtype=torch.bfloat16):
    return StableDiffusion("tiny", device="cpu", dtype=dtype, seed=3)


def _lora_file(unet, path, rank=2):
    g = torch.Generator().manual_seed(0)
    sd = {}
    for name, mod in unet.named_modules():
        if name.endswith(("attn1.to_q", "attn2.to_v", "attn1.to_out.0")):
            o, i = mod.weight.shape
            sd[f"unet.{name}.lora_A.weight"] = torch.randn(rank, i, generator=g) * 0.3
            sd[f"unet.{name}.lora_B.weight"] = torch.randn(o, rank, generator=g) * 0.3
    save_file(sd, path)
    return len(sd) // 2


def _snapshot(m):
    return {k: v.detach().clone() for k, v in m.state_dict().items()}


def test_lora_unload_restores_bitwise(tmp_path):
    pipe = _pipe()
    f = str(tmp_path / "lora.safetensors")
    n = _lora_file(pipe.unet, f)
    before = _snapshot(pipe.unet)
    pipe._graphs = {"stale": object()}
    assert load_lora(pipe.unet, f, 0.8, pipe=pipe) == n
    assert pipe._graphs == {}, "captured graphs must be invalidated on weight change"
    changed = [k for k, v in pipe.unet.state_dict().items() if not torch.equal(v, before[k])]
    assert len(changed) == n
    # packed buffers follow the merged weights
    for name, mod in pipe.unet.named_modules():
        if name.endswith("attn1"):
            q = mod.to_q.weight
            assert torch.equal(mod.w_qkv[: q.shape[0]], q)
    pipe._graphs = {"stale": object()}
    unload_lora(pipe.unet, pipe=pipe)
    assert pipe._graphs == {}
    for k, v in pipe.unet.state_dict().items():
        assert torch.equal(v, before[k]), k  # bf16: W + d - d would NOT round-trip


def test_lora_job_then_plain_job_matches_fresh(tmp_path):
    pipe = _pipe(torch.float32)
    f = str(tmp_path / "lora.safetensors")
    _lora_file(pipe.unet, f)

    def run():
        g = torch.Generator().manual_seed(11)
        return pipe(prompt="a cat", num_inference_steps=2, height=64, width=64, generator=g,
                    output_type="latent").latents

    ref = run()
    load_lora(pipe.unet, f, 1.0, pipe=pipe)
    with_lora = run()
    unload_lora(pipe.unet, pipe=pipe)
    after = run()
    assert not torch.equal(ref, with_lora)
    assert torch.equal(ref, after)


def test_textual_inversion_is_per_job(tmp_path):
    pipe = _pipe(torch.float32)
    te = pipe.text_encoders[0]
    emb = te.text_model.embeddings.token_embedding
    orig_w, orig_n = emb.weight, emb.weight.shape[0]
    f = str(tmp_path / "ti.safetensors")
    save_file({"<cat-toy>": torch.randn(2, orig_w.shape[1])}, f)

    def ids(text):
        return pipe.tokenizers[0]([text])[0].tolist()

    plain = ids("a <cat-toy> photo")
    tok = load_textual_inversion(pipe, f)
    assert tok == "<cat-toy>"
    assert emb.weight.shape[0] == orig_n + 2
    with_ti = ids("a <cat-toy> photo")
    assert orig_n in with_ti and orig_n + 1 in with_ti
    unload_textual_inversion(pipe)
    assert emb.weight is orig_w and emb.weight.shape[0] == orig_n
    assert ids("a <cat-toy> photo") == plain
    # a second job can register the same token again
    load_textual_inversion(pipe, f)
    unload_textual_inversion(pipe)
