"""Packed-weight cache (SURVEY §5.4 "model store / caches").

A checkpoint as shipped is fp16/fp32, in the diffusers key layout, with conv
weights [Cout, Cin, kh, kw] — every load casts it and then ``prepare()`` packs
the tensors the kernels read: NHWC ``[Cout, kh, kw, Cin]`` conv weights, fused
QKV / cross K-V weights, interleaved GEGLU projections, and the UNet's batched
time-embedding projection.  The first load of a component writes the result —
parameters in the model dtype plus every packed buffer — to
``$SDAAS_ROOT/packed/<model>/<revision>/<component>.safetensors``; later loads
read that one file straight into place and skip the casts and the packing.

Validity: the file's metadata holds a fingerprint of the source checkpoint
(relative path, size and mtime of each safetensors file), the framework
version, the dtype and the component's class; any mismatch re-packs from the
source.  safetensors only — nothing that can execute code is ever written or read.
"""
from __future__ import annotations

import hashlib
import json
import os
from pathlib import Path

import torch

from .. import __framework_version__

_SKIP = ("_parameters", "_buffers", "_modules")


def cache_path(model_name: str, revision: str, component: str) -> Path:
    from ..settings import get_settings_dir

    safe = model_name.replace("/", "--")
    return get_settings_dir() / "packed" / safe / (revision or "main") / f"{component}.safetensors"


def fingerprint(src_dir: str, module: torch.nn.Module) -> str:
    h = hashlib.sha256()
    h.update(f"{__framework_version__}|{type(module).__name__}".encode())
    p = next(module.parameters(), None)
    h.update(str(p.dtype if p is not None else None).encode())
    for f in sorted(list(Path(src_dir).glob("*.safetensors")) + list(Path(src_dir).glob("*.bin"))):
        st = f.stat()
        h.update(f"{f.name}|{st.st_size}|{st.st_mtime_ns}".encode())
    return h.hexdigest()


def _packed_items(module: torch.nn.Module):
    """(key, tensor) of every prepared buffer (plain tensor attributes, not
    parameters / registered buffers) and (key, int list) of small int lists."""
    tensors, lists = {}, {}
    for name, m in module.named_modules():
        for attr, v in m.__dict__.items():
            if attr in _SKIP:
                continue
            key = f"{name}::{attr}"
            if torch.is_tensor(v):
                tensors[key] = v
            elif isinstance(v, list) and v and all(isinstance(x, int) for x in v):
                lists[key] = v
            elif v is None:  # e.g. a bias-free projection's packed bias
                lists[key] = None
    return tensors, lists


def save(module: torch.nn.Module, path: Path, fp: str) -> None:
    from safetensors.torch import save_file

    tensors, lists = _packed_items(module)
    out = {f"p::{k}": v.detach() for k, v in module.state_dict().items()}
    out.update({f"x::{k}": v.detach() for k, v in tensors.items()})
    # safetensors refuses aliasing tensors: store a contiguous copy of each
    out = {k: v.contiguous().clone().cpu() for k, v in out.items()}
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_suffix(f".tmp{os.getpid()}")
    save_file(out, str(tmp), metadata={"fingerprint": fp, "lists": json.dumps(lists)})
    os.replace(tmp, path)


def load(module: torch.nn.Module, path: Path, fp: str) -> bool:
    """Fill ``module`` from the cache; False (module untouched) if absent/stale."""
    if not path.is_file():
        return False
    from ..models.weights import load_into
    from . import fastload

    p0 = next(module.parameters())
    meta = fastload.read_metadata(str(path))
    if meta.get("fingerprint") != fp:
        return False
    # one native read of the whole file onto the module's device (fastload)
    tensors = fastload.load_file(str(path), device=p0.device)
    params = {k[3:]: v for k, v in tensors.items() if k.startswith("p::")}
    extra = {k[3:]: v for k, v in tensors.items() if k.startswith("x::")}
    load_into(module, params, name=str(path.name))
    mods = dict(module.named_modules())
    for key, t in extra.items():
        name, attr = key.split("::", 1)
        # own storage: a view would pin the whole file buffer (params included) in HBM
        setattr(mods[name], attr, t.clone() if t.device == p0.device else t.to(p0.device))
    for key, v in json.loads(meta.get("lists", "{}")).items():
        name, attr = key.split("::", 1)
        setattr(mods[name], attr, None if v is None else list(v))
    return True
