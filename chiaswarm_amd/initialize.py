"""``python -m swarm.initialize [--reset] [--silent] [--offline]`` — worker
provisioning (reference: swarm/initialize.py:19-116).

Prompts for hive URI / token (unless --silent), saves settings, fetches the
model catalogue (``GET /api/models`` -> ``models.json``) and provisions every
``can_preload`` model the way the reference's ``download_diffusers`` did
(swarm/initialize.py:62-94, ``from_pretrained`` with revision / variant): a
``huggingface_hub.snapshot_download`` into the HF cache, restricted to what this
framework reads — safetensors weights (the requested ``variant`` when given),
JSON configs and tokenizer files; a repo without any safetensors is fetched
again for its ``.bin`` weights (read later with the weights-only loader,
never unpickled), never ``.ckpt`` / ``.pth`` single-file checkpoints.
``--offline`` (or no network) only locates local copies (``$SDAAS_MODEL_DIR``
or the HF cache).  The packed bf16 weight cache (``runtime/packed_cache.py``)
is written on each model's first load, not here.
Quirk fixed: the reference's ``settings_exist`` was always true.
"""
from __future__ import annotations

import argparse
import json

from . import __framework_version__, __version__
from .hive.client import HiveClient
from .log_setup import setup_logging
from .settings import (Settings, get_settings_full_path, load_settings, resolve_path, save_file, save_settings,
                       settings_exist)


def init(argv=None):
    print("init_app")
    ap = argparse.ArgumentParser()
    ap.add_argument("--reset", action="store_true", help="overwrite existing settings")
    ap.add_argument("--silent", action="store_true", help="do not prompt for input")
    ap.add_argument("--offline", action="store_true", help="do not contact the hive")
    args = ap.parse_args(argv)

    exists = settings_exist()
    if not args.silent and (not exists or args.reset):
        settings = Settings()
        settings.sdaas_uri = input("chiaSWARM uri (https://chiaswarm.ai): ").strip() or "https://chiaswarm.ai"
        settings.sdaas_token = input("chiaSWARM token: ").strip()
        save_settings(settings)
        print(f"Configuration saved to {get_settings_full_path()}")
    elif not exists:
        save_settings(load_settings())

    settings = load_settings()
    setup_logging(resolve_path(settings.log_filename), settings.log_level)
    print(f"Version {__version__} (chiaswarm_amd {__framework_version__})")
    print("App initialization complete")
    report = prepare_models(settings, offline=args.offline)
    save_file(report, "prepared_models.json")
    print("To be the swarm type 'python -m swarm.worker'")
    return report


# what a snapshot fetch may bring: weights as safetensors only, configs, tokenizers
ALLOW = ["*.json", "*.txt", "*.model", "*.safetensors"]
IGNORE = ["*.bin", "*.ckpt", "*.pt", "*.pth", "*.msgpack", "*.h5", "*.onnx", "*.onnx_data", "*.pb", "*.ot"]


def allow_patterns(variant: str | None) -> list:
    """Weight files of the requested variant only (diffusers names them
    ``<name>.<variant>.safetensors``); config / tokenizer files always."""
    if not variant:
        return ALLOW
    return ["*.json", "*.txt", "*.model", f"*.{variant}.safetensors"]


BIN_ALLOW = ["*.json", "*.txt", "*.model", "*.bin"]


def _has_safetensors(path) -> bool:
    import glob
    import os

    return bool(path) and bool(glob.glob(os.path.join(str(path), "**", "*.safetensors"), recursive=True))


def _components_without_safetensors(path) -> list:
    """Component sub-directories of a fetched repo (those with a config.json,
    or the repo root itself) that hold no safetensors weights: their weights
    exist only as pickled ``.bin`` files, which from_pretrained would read."""
    import glob
    import os

    if not path:
        return []
    root = str(path)
    out = []
    for cfg in sorted(glob.glob(os.path.join(root, "*", "config.json")) + [os.path.join(root, "config.json")]):
        d = os.path.dirname(cfg)
        if os.path.exists(cfg) and not glob.glob(os.path.join(d, "*.safetensors")):
            out.append(os.path.relpath(d, root))
    return out


def fetch(name: str, revision: str = "main", variant: str | None = None, token=None, downloader=None) -> str:
    """Download (or re-validate) one model into the HF cache; returns its path.
    Safetensors first; a repo that ships only pickled ``pytorch_model.bin`` /
    ``diffusion_pytorch_model.bin`` weights (what the reference's
    ``from_pretrained`` reads, swarm/initialize.py:84-89) is fetched again with
    ``*.bin`` allowed."""
    if downloader is None:
        from huggingface_hub import snapshot_download as downloader
    tok = token if isinstance(token, str) and token else None
    path = downloader(name, revision=revision, allow_patterns=allow_patterns(variant), ignore_patterns=IGNORE,
                      token=tok)
    if not _has_safetensors(path):
        path = downloader(name, revision=revision, allow_patterns=BIN_ALLOW,
                          ignore_patterns=[p for p in IGNORE if p != "*.bin"], token=tok)
        return path
    # per component: one that ships only pytorch_model.bin (e.g. a text_encoder
    # beside a safetensors unet) gets its .bin fetched too
    missing = _components_without_safetensors(path)
    if missing:
        pats = [f"{c}/*.bin" if c != "." else "*.bin" for c in missing]
        path = downloader(name, revision=revision, allow_patterns=pats,
                          ignore_patterns=[p for p in IGNORE if p != "*.bin"], token=tok)
    return path


def prepare_models(settings, offline=False, downloader=None) -> list:
    from .runtime.model_cache import find_weights

    models = [] if offline else HiveClient(settings).get_models()
    report = []
    for model in models:
        name = model["model_name"]
        params = model.get("parameters", {}) or {}
        entry = {"model_name": name, "revision": model.get("revision", "main"), "variant": model.get("variant"),
                 "can_preload": params.get("can_preload", True)}
        w = None
        if entry["can_preload"] and not offline:
            try:
                w = fetch(name, entry["revision"], entry["variant"], settings.huggingface_token, downloader)
                entry["fetched"] = True
            except Exception as e:  # no network / unknown repo: fall back to a local copy
                entry["fetch_error"] = f"{type(e).__name__}: {e}"[:300]
                print(f"Failed to fetch {name}/{entry['revision']}: {e}")
        if w is None and entry["can_preload"]:
            w = find_weights(name, entry["revision"])
        entry["weights"] = w or "synthetic (no local checkpoint)"
        print(f"Initializing {name}/{entry['revision']}: {entry['weights']}")
        report.append(entry)
    print("Model preparation complete")
    return report


def main():
    print(json.dumps(init(), indent=1)[:2000])


if __name__ == "__main__":
    main()
