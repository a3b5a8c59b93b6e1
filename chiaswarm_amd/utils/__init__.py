"""Small reflection helpers (reference: swarm/type_helpers.py:1-7).

``get_type`` resolves a dotted ``module.attr`` lazily (the hive names pipeline
and scheduler classes by string); ``has_method`` is the duck-typing probe the
reference uses before optional pipeline calls.
"""
from __future__ import annotations

import importlib


def get_type(module_name: str, type_name: str):
    """``getattr(import_module(module_name), type_name)``; unlike the reference's
    ``__import__`` this resolves dotted sub-modules too."""
    return getattr(importlib.import_module(module_name), type_name)


def has_method(o, name: str) -> bool:
    return callable(getattr(o, name, None))


def stable_seed(name: str) -> int:
    """Process-independent 31-bit seed of a string (Python's ``hash`` is salted
    per process, so random-init weights would differ between GPU workers)."""
    import zlib

    return zlib.crc32(str(name).encode("utf-8")) & 0x7FFFFFFF
