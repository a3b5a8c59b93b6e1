"""Generic hipGraph capture of a fixed-shape model call.

``CapturedCall(fn, **inputs)`` records ``fn(**static_inputs)`` once into a HIP
graph (after warm-up on a side stream, so the kernel libraries' lazy init and
the per-shape tile choices happen outside capture); ``run(**inputs)`` copies
the new tensor inputs into the static buffers and replays.  Non-tensor inputs
(e.g. a python float timestep) are passed as 1-element device tensors by the
caller; lists/tuples of tensors (per-layer cross-attention K/V) are copied
element-wise.  Used for the denoiser step of every non-SD pipeline (AudioLDM, IF,
latent upscaler); the SD UNet keeps its own wrapper (``sd._UNetGraph``)
because of the per-request cross-attention K/V list.
"""
from __future__ import annotations

import torch

from .. import ops


def graphs_enabled(device: torch.device) -> bool:
    return device.type == "cuda" and ops.get_mode() == "hip" and ops._lib.available()


def _clone(v):
    if torch.is_tensor(v):
        return v.clone()
    if isinstance(v, (list, tuple)):
        return type(v)(_clone(x) for x in v)
    return v


def _copy_into(dst, src):
    if torch.is_tensor(dst):
        if dst.data_ptr() != src.data_ptr():
            dst.copy_(src)
    elif isinstance(dst, (list, tuple)):
        for d, s in zip(dst, src):
            _copy_into(d, s)


def _key(v):
    if torch.is_tensor(v):
        return (tuple(v.shape), v.dtype)
    if isinstance(v, (list, tuple)):
        return tuple(_key(x) for x in v)
    return v


class CapturedCall:
    def __init__(self, fn, warmup: int = 2, **inputs):
        self.fn = fn
        self.static = {k: _clone(v) for k, v in inputs.items()}
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn(**self.static)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn(**self.static)

    def run(self, **inputs):
        for k, v in inputs.items():
            _copy_into(self.static[k], v)
        self.graph.replay()
        return self.out


class GraphCache:
    """Shape-keyed ``CapturedCall`` cache with an eager fallback."""

    def __init__(self, fn):
        self.fn = fn
        self.graphs: dict = {}

    def __call__(self, device, **inputs):
        if not graphs_enabled(device):
            return self.fn(**inputs)
        key = tuple((k, _key(v)) for k, v in sorted(inputs.items()))
        g = self.graphs.get(key)
        if g is None:
            g = CapturedCall(self.fn, **inputs)
            self.graphs[key] = g
        return g.run(**inputs)
