"""Worker settings: defaults -> ``$SDAAS_ROOT/settings.json`` (or ``~/.sdaas``)
-> environment overrides.  Same file, keys and env vars as the reference
(swarm/settings.py:7-73); extra MI355X knobs are additive and optional.

Quirk fixed: ``settings_exist`` really checks for the file (the
reference's ``load_settings() is not None`` was always true).
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Union


class Settings:
    huggingface_token: Union[bool, str] = True
    log_level: str = "WARN"
    log_filename: str = "log/generator.log"
    sdaas_token: str = ""
    sdaas_uri: str = "http://localhost:9511"
    worker_name: str = "worker"
    # --- MI355X additions (env: SDAAS_GPUS, SDAAS_MAX_BATCH, SDAAS_CACHE_GB, SDAAS_MODEL_DIR) ---
    gpus: str = ""              # comma list of visible GPU indices; "" = all
    max_batch: int = 8          # max images coalesced into one UNet batch
    cache_gb: float = 200.0     # HBM budget for resident models per GPU
    model_dir: str = ""         # local diffusers-layout model store ("" -> $SDAAS_ROOT/models)
    preload: str = ""           # comma list of models every GPU loads at startup (sharded RCCL read)
    distributed: bool = True    # per-GPU processes form one process group (RCCL over xGMI)
    split_jobs: bool = True     # a multi-image txt2img job may use several idle GPUs
    cfg_parallel: bool = False  # opt-in: a one-image CFG txt2img job may run its two CFG halves on two idle GPUs (UNet at batch 1 per half: not bit-identical to the solo batch-2 run)

    def __init__(self):
        for k in ("huggingface_token", "log_level", "log_filename", "sdaas_token", "sdaas_uri", "worker_name",
                  "gpus", "max_batch", "cache_gb", "model_dir", "preload", "distributed", "split_jobs",
                  "cfg_parallel"):
            setattr(self, k, getattr(type(self), k))


def load_settings() -> Settings:
    settings = Settings()
    try:
        with open(get_settings_full_path(), "r") as f:
            d = json.load(f)
    except FileNotFoundError:
        d = {}
    except json.JSONDecodeError:
        print("invalid settings file")
        d = {}
    settings.log_level = d.get("log_level", "WARN")
    settings.log_filename = d.get("log_filename", "log/generator.log")
    settings.sdaas_token = d.get("sdaas_token", "")
    settings.sdaas_uri = d.get("sdaas_uri", "http://localhost:9511")
    settings.worker_name = d.get("worker_name", "worker")
    settings.gpus = str(d.get("gpus", ""))
    settings.max_batch = int(d.get("max_batch", 8))
    settings.cache_gb = float(d.get("cache_gb", 200.0))
    settings.model_dir = d.get("model_dir", "")
    settings.preload = str(d.get("preload", ""))
    settings.distributed = bool(d.get("distributed", True))
    settings.split_jobs = bool(d.get("split_jobs", True))
    settings.cfg_parallel = bool(d.get("cfg_parallel", False))

    settings.sdaas_token = os.getenv("SDAAS_TOKEN", settings.sdaas_token)
    settings.sdaas_uri = os.getenv("SDAAS_URI", settings.sdaas_uri)
    settings.worker_name = os.getenv("SDAAS_WORKERNAME", settings.worker_name)
    settings.gpus = os.getenv("SDAAS_GPUS", settings.gpus)
    settings.max_batch = int(os.getenv("SDAAS_MAX_BATCH", settings.max_batch))
    settings.cache_gb = float(os.getenv("SDAAS_CACHE_GB", settings.cache_gb))
    settings.model_dir = os.getenv("SDAAS_MODEL_DIR", settings.model_dir)
    settings.preload = os.getenv("SDAAS_PRELOAD", settings.preload)
    settings.distributed = os.getenv("SDAAS_DIST", "1" if settings.distributed else "0") != "0"
    settings.split_jobs = os.getenv("SDAAS_SPLIT_JOBS", "1" if settings.split_jobs else "0") != "0"
    settings.cfg_parallel = os.getenv("SDAAS_CFG_PARALLEL", "1" if settings.cfg_parallel else "0") != "0"
    return settings


def save_settings(settings: Settings):
    with open(get_settings_full_path(), "w") as f:
        json.dump(dict(settings.__dict__), f, indent=2)


def settings_exist() -> bool:
    return get_settings_full_path().is_file()


def resolve_path(path) -> Path:
    full = get_settings_dir().joinpath(path)
    full.parent.mkdir(parents=True, exist_ok=True)
    return full


def get_settings_dir() -> Path:
    return Path(os.environ.get("SDAAS_ROOT") or "~/.sdaas/").expanduser()


def save_file(data, filename):
    with open(resolve_path(filename), "w") as f:
        json.dump(data, f, indent=2)


def get_settings_full_path() -> Path:
    return resolve_path("settings.json")


def model_store_dir(settings: Settings | None = None) -> Path:
    s = settings or load_settings()
    return Path(s.model_dir).expanduser() if s.model_dir else get_settings_dir() / "models"
