"""``python -m swarm.initialize [--reset] [--silent] [--offline]`` — worker
provisioning (reference: swarm/initialize.py:19-116).

Prompts for hive URI / token (unless --silent), saves settings, fetches the
model catalogue (``GET /api/models`` -> ``models.json``) and prepares every
``can_preload`` model.  The reference downloaded diffusers checkpoints from the
Hugging Face hub; here "prepare" means: locate a local diffusers-layout copy
(``$SDAAS_MODEL_DIR`` or the HF cache) and convert it into the packed NHWC/bf16
cache format, or record that the model will run with synthetic weights.
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


def prepare_models(settings, offline=False) -> list:
    from .runtime.model_cache import find_weights

    models = [] if offline else HiveClient(settings).get_models()
    report = []
    for model in models:
        name = model["model_name"]
        params = model.get("parameters", {}) or {}
        entry = {"model_name": name, "revision": model.get("revision", "main"),
                 "can_preload": params.get("can_preload", True)}
        w = find_weights(name, entry["revision"]) if entry["can_preload"] else None
        entry["weights"] = w or "synthetic (no local checkpoint)"
        print(f"Initializing {name}/{entry['revision']}: {entry['weights']}")
        report.append(entry)
    print("Model preparation complete")
    return report


def main():
    print(json.dumps(init(), indent=1)[:2000])


if __name__ == "__main__":
    main()
