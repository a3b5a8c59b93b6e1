"""HBM-resident model cache (per GPU process).

The reference re-loaded every pipeline from disk on every job
(swarm/diffusion/diffusion_func.py:41-46 and six other call sites, SURVEY §1
observation 2).  With 288 GB of HBM per MI355X we keep models resident: an LRU
keyed by (kind, model name, revision, device) with a byte budget
(``settings.cache_gb``); eviction frees the least recently used bundle.
"""
from __future__ import annotations

import glob
import os
import threading
from collections import OrderedDict


def _nbytes(obj) -> int:
    import torch

    seen, total = set(), 0
    mods = []
    for attr in ("unet", "vae", "controlnet", "model", "text_encoders", "modules"):
        v = getattr(obj, attr, None)
        if v is None:
            continue
        mods.extend(v if isinstance(v, (list, tuple)) else [v])
    if isinstance(obj, torch.nn.Module):
        mods.append(obj)
    for m in mods:
        if not isinstance(m, torch.nn.Module):
            continue
        for p in list(m.parameters()) + list(m.buffers()):
            if id(p) not in seen:
                seen.add(id(p))
                total += p.numel() * p.element_size()
    return total


class ModelCache:
    def __init__(self, budget_bytes: int):
        self.budget = budget_bytes
        self._items: OrderedDict = OrderedDict()
        self._sizes: dict = {}
        self._lock = threading.Lock()
        self.hits = self.misses = 0

    def get(self, key, factory):
        with self._lock:
            if key in self._items:
                self._items.move_to_end(key)
                self.hits += 1
                return self._items[key]
        self.misses += 1
        obj = factory()
        size = _nbytes(obj)
        with self._lock:
            self._items[key] = obj
            self._sizes[key] = size
            self._evict()
        return obj

    def _evict(self):
        while sum(self._sizes.values()) > self.budget and len(self._items) > 1:
            k, _ = self._items.popitem(last=False)
            self._sizes.pop(k, None)
            try:
                import torch

                if torch.cuda.is_available():
                    torch.cuda.empty_cache()
            except Exception:
                pass

    def keys(self):
        return list(self._items)

    def clear(self):
        """Drop every resident bundle (and with them their captured hipGraphs)."""
        with self._lock:
            self._items.clear()
            self._sizes.clear()
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.empty_cache()
        except Exception:
            pass


_CACHE: ModelCache | None = None


def cache() -> ModelCache:
    global _CACHE
    if _CACHE is None:
        from ..settings import load_settings

        _CACHE = ModelCache(int(load_settings().cache_gb * (1 << 30)))
    return _CACHE


def find_weights(model_name: str, revision: str = "main") -> str | None:
    """Local diffusers-layout directory for ``model_name`` if one exists:
    $SDAAS_MODEL_DIR/<org>/<name>, else the Hugging Face hub cache snapshot."""
    from ..settings import model_store_dir

    d = model_store_dir() / model_name
    if d.is_dir():
        return str(d)
    hub = os.path.expanduser(os.environ.get("HF_HOME", "~/.cache/huggingface"))
    snaps = glob.glob(os.path.join(hub, "hub", "models--" + model_name.replace("/", "--"), "snapshots", "*"))
    return sorted(snaps)[-1] if snaps else None
