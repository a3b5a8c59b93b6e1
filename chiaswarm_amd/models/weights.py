"""Checkpoint loading (safetensors only — never pickles).

Reads a diffusers-layout model directory (``unet/``, ``vae/``, ``text_encoder/``
[, ``text_encoder_2/``] each holding ``*.safetensors``) into our modules, whose
parameter names follow the diffusers / transformers keys.  Older VAE attention
names (``query/key/value/proj_attn``) are remapped.  Returns False when no
weights are found (the caller keeps its random init and says so in
``pipeline_config.weights``).
"""
from __future__ import annotations

import glob
import os

import torch

_VAE_RENAMES = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}


def _read_dir(d: str) -> dict:
    from safetensors.torch import load_file

    out = {}
    for f in sorted(glob.glob(os.path.join(d, "*.safetensors"))):
        out.update(load_file(f, device="cpu"))
    return out


def load_into(module: torch.nn.Module, sd: dict, renames: dict | None = None, prefix_strip: str = "") -> int:
    own = module.state_dict()
    n = 0
    with torch.no_grad():
        for k, v in sd.items():
            kk = k[len(prefix_strip):] if prefix_strip and k.startswith(prefix_strip) else k
            for a, b in (renames or {}).items():
                kk = kk.replace(a, b)
            if kk in own:
                t = own[kk]
                if t.shape != v.shape and v.numel() == t.numel():
                    v = v.reshape(t.shape)  # e.g. VAE attention 1x1-conv weights
                if t.shape == v.shape:
                    t.copy_(v.to(t.dtype))
                    n += 1
    return n


def load_sd_weights(pipe, weights_dir: str) -> bool:
    if not weights_dir or not os.path.isdir(weights_dir):
        return False
    loaded = 0
    parts = [("unet", pipe.unet, None), ("vae", pipe.vae, _VAE_RENAMES)]
    for i, te in enumerate(pipe.text_encoders):
        parts.append(("text_encoder" if i == 0 else f"text_encoder_{i + 1}", te, None))
    for sub, mod, ren in parts:
        d = os.path.join(weights_dir, sub)
        if os.path.isdir(d):
            loaded += load_into(mod, _read_dir(d), ren)
    return loaded > 0
