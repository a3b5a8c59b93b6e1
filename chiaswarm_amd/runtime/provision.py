"""Model provisioning at job time: never serve random-init weights as a result.

The reference builds every model with ``from_pretrained`` inside the job
(swarm/diffusion/diffusion_func.py:41-46, swarm/video/tx2vid.py:24-30,
swarm/captioning/caption_image.py:14-17, swarm/diffusion/upscale.py:8-13):
a model that is not in the local cache is downloaded on the spot, and a failed
download raises — the job reports an error instead of a picture.

``ensure_weights`` is that contract here:
  * a local copy (``$SDAAS_MODEL_DIR`` or the HF hub cache) is used as is;
  * otherwise the model is fetched like ``python -m swarm.initialize`` does
    (``initialize.fetch``: safetensors first, pickled ``.bin`` only when the
    repo has no safetensors) under a per-model lock, so concurrent jobs of one
    process share one download;
  * if there are still no weights the job fails with ``WeightsMissing`` — a
    RuntimeError, i.e. a NON-fatal error envelope (runtime/generator.py class
    (c)): the hive may hand the job to a provisioned worker.
Seeded random-init weights are allowed only under ``SDAAS_ALLOW_RANDOM=1``
(bench.py, the smoke test and the test suite set it: they run synthetic models
of the real architectures by design).  ``SDAAS_OFFLINE=1`` skips the fetch.
"""
from __future__ import annotations

import glob
import os
import threading
from collections import defaultdict

from .model_cache import find_weights

_LOCKS: dict = defaultdict(threading.Lock)
_LOCKS_GUARD = threading.Lock()

# test hook: a callable with huggingface_hub.snapshot_download's signature
DOWNLOADER = None


class WeightsMissing(RuntimeError):
    """No weights for a model the job needs (non-fatal: retry elsewhere)."""


def allow_random() -> bool:
    return os.environ.get("SDAAS_ALLOW_RANDOM", "0") == "1"


def offline() -> bool:
    return os.environ.get("SDAAS_OFFLINE", "0") == "1"


def has_weights(path: str | None) -> bool:
    """A directory (or file) holding model weights this framework can read:
    safetensors anywhere below it, or pickled .bin / .pth files read with the
    weights-only loader (models/weights.py)."""
    if not path:
        return False
    if os.path.isfile(path):
        return path.endswith((".safetensors", ".bin", ".pth", ".pt"))
    for ext in ("safetensors", "bin", "pth", "pt"):
        if glob.glob(os.path.join(path, f"*.{ext}")) or glob.glob(os.path.join(path, "*", f"*.{ext}")):
            return True
    return False


def _lock(key):
    with _LOCKS_GUARD:
        return _LOCKS[key]


def ensure_weights(model_name: str, revision: str = "main", variant: str | None = None,
                   required: bool = True) -> str | None:
    """Local weights directory of ``model_name``, fetched on a miss.

    Returns None only when the model may run without weights: ``required`` is
    False (an optional component, e.g. a separately provisioned safety
    checker) or ``SDAAS_ALLOW_RANDOM=1``.  Raises ``WeightsMissing`` otherwise."""
    revision = revision or "main"
    w = find_weights(model_name, revision)
    if has_weights(w):
        return w
    err = "offline (SDAAS_OFFLINE=1)" if offline() else None
    if not offline():
        with _lock((model_name, revision)):
            w = find_weights(model_name, revision)
            if has_weights(w):
                return w
            try:
                from ..initialize import fetch
                from ..settings import load_settings

                token = getattr(load_settings(), "huggingface_token", None)
                w = fetch(model_name, revision, variant, token, DOWNLOADER)
            except Exception as e:  # no network, unknown repo, auth
                err = f"{type(e).__name__}: {e}"[:300]
                w = None
            if has_weights(w):
                return w
            if err is None:
                err = "the fetched snapshot holds no weights"
    if not required or allow_random():
        return None
    raise WeightsMissing(f"model {model_name} (revision {revision}) is not provisioned on this worker and could not "
                         f"be fetched: {err}")
