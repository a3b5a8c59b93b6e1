"""ctypes bindings of the gfx950 kernels in libcsk.so (filled per kernel)."""
from __future__ import annotations
