"""Rotating file logging (reference: swarm/log_setup.py:5-29, 50 MiB x 7).

Differences: the level map accepts "WARN" (the reference's map lacked it and
fell back to INFO), and every per-GPU process writes its own
``<name>.gpuN.log`` so rotation never races between processes (the reference
needed concurrent_log_handler for its single multi-threaded process).
Structured per-job JSON lines go through ``log_job``.
"""
from __future__ import annotations

import json
import logging
import logging.handlers
import os

LEVELS = {"CRITICAL": logging.CRITICAL, "ERROR": logging.ERROR, "WARNING": logging.WARNING,
          "WARN": logging.WARNING, "INFO": logging.INFO, "DEBUG": logging.DEBUG}


def setup_logging(log_path, log_level, suffix: str | None = None):
    path = str(log_path)
    if suffix:
        root, ext = os.path.splitext(path)
        path = f"{root}.{suffix}{ext}"
    logger = logging.getLogger()
    logger.setLevel(LEVELS.get(str(log_level).upper(), logging.INFO))
    for h in list(logger.handlers):
        if isinstance(h, logging.handlers.RotatingFileHandler) and getattr(h, "baseFilename", "") == os.path.abspath(path):
            return logger
    handler = logging.handlers.RotatingFileHandler(path, "a", maxBytes=50 * 1024 * 1024, backupCount=7)
    handler.setFormatter(logging.Formatter(fmt="%(asctime)s - %(levelname)s - %(message)s",
                                           datefmt="%Y-%m-%dT%H:%M:%S"))
    logger.addHandler(handler)
    return logger


def log_job(record: dict):
    """One structured JSON line per job (phase timings, GPU, batch, images/s)."""
    logging.getLogger("chiaswarm_amd.jobs").info(json.dumps(record, default=str))
