"""Checkpoint loading (safetensors; pickled ``.bin`` / ``.pth`` files only
through ``torch.load(weights_only=True)``, which executes nothing from the file).

Reads a diffusers-layout model directory (``unet/``, ``vae/``, ``text_encoder/``
[, ``text_encoder_2/``] each holding ``*.safetensors``) into our modules, whose
parameter names follow the diffusers / transformers keys.  Older VAE attention
names (``query/key/value/proj_attn``) are remapped.

Loading is STRICT: every parameter of the module must be present with the right
shape and every checkpoint tensor must land somewhere (up to a short list of
known-harmless extras such as ``position_ids`` buffers), otherwise
``CheckpointMismatch`` is raised — a partially loaded model would otherwise run
with random layers and produce plausible-looking garbage.  The reference gets
the same guarantee from ``from_pretrained`` (swarm/diffusion/diffusion_func.py:41-46).
Every load returns a ``LoadReport`` (loaded / missing / unexpected / mismatched).
"""
from __future__ import annotations

import dataclasses
import glob
import os

import torch

_VAE_RENAMES = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.", ".proj_attn.": ".to_out.0."}
# checkpoint tensors that legitimately have no parameter here
_HARMLESS = ("position_ids", "token_type_ids", "num_batches_tracked", "logit_scale")


class CheckpointMismatch(ValueError):
    pass


@dataclasses.dataclass
class LoadReport:
    name: str
    loaded: int
    total: int
    missing: list
    unexpected: list
    mismatched: list

    @property
    def complete(self) -> bool:
        return not self.missing and not self.mismatched and self.loaded == self.total

    def __int__(self):
        return self.loaded

    def __radd__(self, other):
        return other + self.loaded

    def summary(self, n=6) -> str:
        def cut(xs):
            return ", ".join(map(str, xs[:n])) + (f" (+{len(xs) - n} more)" if len(xs) > n else "")
        parts = [f"{self.name or 'module'}: {self.loaded}/{self.total} tensors loaded"]
        if self.missing:
            parts.append(f"missing [{cut(self.missing)}]")
        if self.unexpected:
            parts.append(f"unexpected [{cut(self.unexpected)}]")
        if self.mismatched:
            parts.append(f"shape mismatch [{cut(self.mismatched)}]")
        return "; ".join(parts)


# pickled files of a transformers / diffusers repo that hold no model weights
_NON_WEIGHT_BINS = ("training_args.bin", "optimizer.bin", "scheduler.bin", "rng_state.bin", "scaler.bin")


def weight_files(d: str) -> tuple:
    """(kind, files) of a component directory: its ``*.safetensors``, else the
    ``*.bin`` weight files (``pytorch_model.bin`` / ``diffusion_pytorch_model.bin``,
    sharded or not) that ``from_pretrained`` would read; ("", []) if none."""
    st = sorted(glob.glob(os.path.join(d, "*.safetensors")))
    if st:
        return "safetensors", st
    bins = sorted(f for f in glob.glob(os.path.join(d, "*.bin")) if os.path.basename(f) not in _NON_WEIGHT_BINS)
    return ("bin", bins) if bins else ("", [])


def _read_dir(d: str, device="cpu") -> dict:
    """Tensors of a component directory.  Safetensors go through the native
    reader (runtime/fastload.py: one threaded read of each file's data region
    straight to ``device``; tensors are views of it); ``.bin`` files through
    the weights-only unpickler on the host."""
    from ..runtime.fastload import load_file

    out = {}
    kind, files = weight_files(d)
    if kind == "bin":
        fp16 = [f for f in files if ".fp16." in os.path.basename(f)]
        if fp16 and len(fp16) < len(files):
            files = [f for f in files if f not in fp16]
        for f in files:
            out.update(read_pth(f))
        return out
    # diffusers ships fp32 and fp16 variants side by side: take one of each model file
    fp16 = [f for f in files if ".fp16." in os.path.basename(f)]
    if fp16 and len(fp16) < len(files):
        files = [f for f in files if f not in fp16]
    for f in files:
        out.update(load_file(f, device=device))
    return out


def read_pth(path: str) -> dict:
    """A PyTorch ``.pth`` / ``.pt`` checkpoint read with the weights-only
    unpickler (tensors and plain containers only: nothing in the file is
    executed).  Real-ESRGAN / BasicSR checkpoints wrap the state dict as
    ``{"params_ema": ...}`` (or ``"params"``); that wrapper is unwrapped."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, dict):
        for key in ("params_ema", "params", "state_dict", "model"):
            if isinstance(obj.get(key), dict):
                obj = obj[key]
                break
    if not isinstance(obj, dict) or not all(torch.is_tensor(v) for v in obj.values()):
        raise CheckpointMismatch(f"{path}: not a state dict of tensors")
    return obj


def read_weights(path: str) -> dict:
    """State dict of a directory (``*.safetensors``, else a single ``*.pth`` /
    ``*.pt``) or of one file of either format."""
    if os.path.isdir(path):
        kind, files = weight_files(path)
        # safetensors always win; a .pth is read only where there are none
        if kind == "safetensors" or (files and not glob.glob(os.path.join(path, "*.pth"))):
            return _read_dir(path)
        pth = sorted(glob.glob(os.path.join(path, "*.pth")) + glob.glob(os.path.join(path, "*.pt")))
        if len(pth) != 1:
            raise CheckpointMismatch(f"{path}: expected *.safetensors or exactly one *.pth, found {pth}")
        return read_pth(pth[0])
    if path.endswith(".safetensors"):
        from ..runtime.fastload import load_file

        return load_file(path, device="cpu")
    return read_pth(path)


def load_into(module: torch.nn.Module, sd: dict, renames: dict | None = None, prefix_strip: str = "",
              strict: bool = True, allow_unexpected: bool = False, name: str = "") -> LoadReport:
    """Copy ``sd`` into ``module``'s parameters/buffers (cast to their dtype).
    Raises ``CheckpointMismatch`` under ``strict`` unless the match is complete."""
    own = module.state_dict()
    ignore = tuple(getattr(module, "checkpoint_ignore", ()))  # e.g. a decoder-only VAE: encoder.*
    alias = getattr(module, "checkpoint_alias_prefix", "")  # e.g. transformers>=5 drops "text_model."
    done: set = set()
    unexpected, mismatched = [], []
    with torch.no_grad():
        for k, v in sd.items():
            kk = k[len(prefix_strip):] if prefix_strip and k.startswith(prefix_strip) else k
            for a, b in (renames or {}).items():
                kk = kk.replace(a, b)
            if kk not in own and alias and alias + kk in own:
                kk = alias + kk
            if kk not in own:
                if not kk.endswith(_HARMLESS) and not (ignore and kk.startswith(ignore)):
                    unexpected.append(k)
                continue
            t = own[kk]
            if t.shape != v.shape and v.numel() == t.numel() and v.dim() != t.dim():
                v = v.reshape(t.shape)  # e.g. VAE attention 1x1-conv weights
            if t.shape != v.shape:
                mismatched.append(f"{kk} {tuple(v.shape)}!={tuple(t.shape)}")
                continue
            t.copy_(v.to(t.dtype))
            done.add(kk)
    missing = [k for k in own if k not in done and not k.endswith(_HARMLESS)]
    rep = LoadReport(name, len(done), len([k for k in own if not k.endswith(_HARMLESS)]), missing, unexpected,
                     mismatched)
    if strict and (missing or mismatched or (unexpected and not allow_unexpected)):
        raise CheckpointMismatch(rep.summary())
    return rep


def read_checkpoint(d: str, like: torch.nn.Module | None = None) -> dict:
    """All tensors of a directory's safetensors files.  Inside
    ``comm.collective_loading()`` with a process group, each rank reads only
    its 1/world share of the bytes and an all_gather assembles the rest
    (parallel/sharded.py); otherwise a plain local read."""
    from ..parallel import comm

    if comm.collective_load_active() and weight_files(d)[0] == "safetensors":
        from ..parallel.sharded import safetensors_files, sharded_state_dict

        p = next(like.parameters(), None) if like is not None else None
        dt = p.dtype if p is not None else torch.float32
        dev = p.device if p is not None else "cpu"
        if dev is not None and getattr(dev, "type", dev) == "cuda" and torch.distributed.get_backend() == "gloo":
            dev = "cpu"
        return sharded_state_dict(safetensors_files(d), dt, dev)
    p = next(like.parameters(), None) if like is not None else None
    return _read_dir(d, p.device if p is not None else "cpu")


def load_component(module, weights_dir: str, sub: str, renames=None, **kw) -> LoadReport | None:
    """Strict load of ``weights_dir/sub`` (safetensors or weights-only ``.bin``;
    None if that dir is absent)."""
    d = os.path.join(weights_dir, sub) if sub else weights_dir
    if not os.path.isdir(d) or not weight_files(d)[1]:
        return None
    return load_into(module, read_checkpoint(d, module), renames, name=sub or os.path.basename(d), **kw)


def load_sd_weights(pipe, weights_dir: str) -> bool:
    """All SD components of a diffusers directory; True if any was present.
    ``pipe.load_reports`` keeps one ``LoadReport`` per component (or "packed
    cache" when it came from ``runtime/packed_cache.py``); components loaded
    here are also prepared (packed), listed in ``pipe.prepared``."""
    pipe.prepared = set()
    if not weights_dir or not os.path.isdir(weights_dir):
        return False
    import hashlib

    from ..parallel import comm
    from ..runtime import packed_cache
    from .layers import prepare_model

    use_cache = os.environ.get("SDAAS_PACKED_CACHE", "1") != "0" and not comm.collective_load_active()
    key = hashlib.sha1(os.path.abspath(weights_dir).encode()).hexdigest()[:16]
    parts = [("unet", pipe.unet, None), ("vae", pipe.vae, _VAE_RENAMES)]
    fam = getattr(pipe, "family", None)
    tnames = fam.text_components if fam is not None else \
        ["text_encoder" if i == 0 else f"text_encoder_{i + 1}" for i in range(len(pipe.text_encoders))]
    for name, te in zip(tnames, pipe.text_encoders):
        parts.append((name, te, getattr(te, "hf_renames", None)))  # (AltDiffusion's XLM-R: transformers names)
    present = [sub for sub, _, _ in parts if weight_files(os.path.join(weights_dir, sub))[1]]
    if not present:
        return False
    absent = [sub for sub, _, _ in parts if sub not in present]
    if absent:
        # a real UNet beside a random-init VAE / text encoder would produce
        # plausible-looking garbage while reporting the checkpoint as loaded
        raise CheckpointMismatch(f"{weights_dir}: no weights for {absent} (present: {present}); "
                                 "refusing a partial load")
    reports = {}
    for sub, mod, ren in parts:
        src = os.path.join(weights_dir, sub)
        fp = packed_cache.fingerprint(src, mod)
        path = packed_cache.cache_path(key, "main", sub)
        if use_cache and packed_cache.load(mod, path, fp):
            reports[sub] = "packed cache"
            pipe.prepared.add(sub)
            continue
        reports[sub] = load_component(mod, weights_dir, sub, ren)
        prepare_model(mod)
        pipe.prepared.add(sub)
        if use_cache:
            try:
                packed_cache.save(mod, path, fp)
            except OSError:  # read-only store: run without the cache
                pass
    pipe.load_reports = reports
    return bool(reports)


def tokenizer_dir(weights_dir: str | None, sub: str = "tokenizer") -> str | None:
    if not weights_dir:
        return None
    d = os.path.join(weights_dir, sub)
    return d if any(os.path.exists(os.path.join(d, f)) for f in ("vocab.json", "spiece.model",
                                                                  "sentencepiece.bpe.model")) else None
