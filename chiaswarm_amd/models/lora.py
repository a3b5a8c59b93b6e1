"""LoRA and textual-inversion adapters (reference: swarm/diffusion/diffusion_func.py:48-68,
``pipeline.unet.load_attn_procs(lora)`` / ``pipeline.load_textual_inversion``).

LoRA weights are merged into the resident UNet (W += scale * up @ down) for the
duration of one job, so the hot path keeps running the plain fused GEMMs — no
per-step adapter cost.  ``unload_lora`` restores the ORIGINAL weights bit for
bit (``copy_`` from saved copies: in bf16, W + d - d != W, so subtracting the
delta again would drift the shared resident model job after job).  Packed
buffers are rebuilt in place (stable pointers), and the owning pipeline's
hipGraphs are invalidated on every adapter change (``_invalidate``).
Textual inversion is per job too: ``unload_textual_inversion`` restores the
original embedding table and removes the placeholder token.
Supported key layouts: diffusers attn-procs (``...attn1.processor.to_q_lora.
{down,up}.weight``), diffusers PEFT (``...attn1.to_q.lora_A/B.weight``) and kohya
(``lora_unet_down_blocks_0_..._to_q.lora_down/up.weight`` + ``.alpha``).
Only safetensors files are read (no pickles).  A name that is not a local
file/dir (hub ids need network) raises -> the job fails as fatal ValueError,
like an incompatible LoRA in the reference.
"""
from __future__ import annotations

import os
import re

import torch


def _resolve(path_or_name: str) -> str:
    from ..runtime.provision import ensure_weights

    if os.path.isfile(path_or_name):
        return path_or_name
    d = path_or_name if os.path.isdir(path_or_name) else ensure_weights(path_or_name)
    if d and os.path.isdir(d):
        for f in sorted(os.listdir(d)):
            if f.endswith(".safetensors"):
                return os.path.join(d, f)
    raise FileNotFoundError(f"adapter weights not found locally: {path_or_name}")


def _read(path):
    from safetensors.torch import load_file

    return load_file(path, device="cpu")


def _linear_index(unet):
    idx = {}
    for name, mod in unet.named_modules():
        if isinstance(mod, torch.nn.Linear):
            idx[name] = mod
            idx[name.replace(".", "_")] = mod
    return idx


def _pairs(sd: dict):
    """Yield (target module name, down, up, alpha or None)."""
    groups: dict = {}
    for k, v in sd.items():
        m = (re.match(r"(.*)\.processor\.(to_[qkv]|to_out)_lora\.(down|up)\.weight$", k)
             or re.match(r"(.*)\.(to_[qkv]|to_out\.0)\.lora_(A|B)\.weight$", k))
        if m:
            base, proj, which = m.group(1), m.group(2), m.group(3)
            proj = "to_out.0" if proj.startswith("to_out") else proj
            target = f"{base}.{proj}".removeprefix("unet.")
            g = groups.setdefault(target, {})
            g["down" if which in ("down", "A") else "up"] = v
            continue
        m = re.match(r"lora_unet_(.*)\.(lora_down|lora_up)\.weight$", k)
        if m:
            g = groups.setdefault("kohya:" + m.group(1), {})
            g["down" if m.group(2) == "lora_down" else "up"] = v
            continue
        m = re.match(r"lora_unet_(.*)\.alpha$", k)
        if m:
            groups.setdefault("kohya:" + m.group(1), {})["alpha"] = float(v)
    for t, g in groups.items():
        if "down" in g and "up" in g:
            yield t, g["down"], g["up"], g.get("alpha")


def load_lora(unet, path_or_name: str, scale: float = 1.0, pipe=None):
    sd = _read(_resolve(path_or_name))
    idx = _linear_index(unet)
    merged = []
    with torch.no_grad():
        try:
            for target, down, up, alpha in _pairs(sd):
                key = target[len("kohya:"):] if target.startswith("kohya:") else target
                mod = idx.get(key)
                if mod is None:
                    raise KeyError(f"LoRA target {key} not in this UNet")
                down2, up2 = down.float().flatten(1), up.float().flatten(1)
                rank = down2.shape[0]
                s = scale * ((alpha / rank) if alpha else 1.0)
                delta = (up2 @ down2) * s
                if delta.shape != mod.weight.shape:
                    raise ValueError(f"LoRA shape {tuple(delta.shape)} != {tuple(mod.weight.shape)} for {key}")
                orig = mod.weight.detach().clone()
                merged.append((mod, orig))
                mod.weight.copy_((orig.float() + delta.to(orig.device)).to(orig.dtype))
        except Exception:
            for mod, orig in merged:  # leave the resident model untouched on failure
                mod.weight.copy_(orig)
            raise
    if not merged:
        raise ValueError("no LoRA weights recognised in file")
    unet._lora_merged = merged
    _reprepare(unet, pipe)
    return len(merged)


def unload_lora(unet, pipe=None):
    merged = getattr(unet, "_lora_merged", None)
    if not merged:
        return
    with torch.no_grad():
        for mod, orig in merged:
            mod.weight.copy_(orig)  # bitwise restore
    unet._lora_merged = None
    _reprepare(unet, pipe)


def _invalidate(pipe):
    from ..utils import has_method

    if pipe is not None and has_method(pipe, "invalidate_graphs"):
        pipe.invalidate_graphs()


def _reprepare(unet, pipe=None):
    from .layers import prepare_model

    prepare_model(unet)
    _invalidate(pipe)


def load_textual_inversion(pipe, path_or_name: str, token: str | None = None):
    """A1111 / diffusers embedding file: {"<token>": [n, D]} or {"emb_params": ...}
    / {"string_to_param": {"*": ...}}.  Appends rows to the token embedding and
    registers the placeholder with the tokenizer."""
    sd = _read(_resolve(path_or_name))
    if "emb_params" in sd:
        vecs = sd["emb_params"]
        tok = token or os.path.splitext(os.path.basename(str(path_or_name)))[0]
    else:
        (tok0, vecs), = [(k, v) for k, v in sd.items() if v.dim() in (1, 2)][:1]
        tok = token or tok0
    if vecs.dim() == 1:
        vecs = vecs[None]
    te = pipe.text_encoders[0]
    emb = te.text_model.embeddings.token_embedding
    if vecs.shape[-1] != emb.weight.shape[1]:
        raise ValueError(f"embedding width {vecs.shape[-1]} != text encoder width {emb.weight.shape[1]}")
    tokz = pipe.tokenizers[0]
    added = getattr(tokz, "added_tokens", None) or {}
    if tok in added:
        raise ValueError(f"token {tok!r} is already registered")
    with torch.no_grad():
        orig = emb.weight
        start = orig.shape[0]
        new = torch.cat([orig, vecs.to(orig)], 0)
        emb.weight = torch.nn.Parameter(new, requires_grad=False)
        emb.num_embeddings = new.shape[0]
    te._ti_orig = getattr(te, "_ti_orig", None) or (orig, start)
    tokz.added_tokens = dict(added)
    tokz.added_tokens[tok] = list(range(start, start + vecs.shape[0]))
    _invalidate(pipe)
    return tok


def unload_textual_inversion(pipe):
    """Drop every per-job embedding row and placeholder token (bitwise the
    original table object comes back)."""
    te = pipe.text_encoders[0]
    saved = getattr(te, "_ti_orig", None)
    if saved is None:
        return
    orig, n = saved
    emb = te.text_model.embeddings.token_embedding
    emb.weight = orig
    emb.num_embeddings = n
    te._ti_orig = None
    pipe.tokenizers[0].added_tokens = {}
    _invalidate(pipe)
