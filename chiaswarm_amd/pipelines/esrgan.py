"""Real-ESRGAN x4 upscaling workflow (north-star extension; the reference only
lists it on its roadmap, README.md:34).

Routed for ``workflow: "upscale"`` or a model name containing "esrgan"; also
used as the pixel-space upscaler option.  Inputs above ``tile`` pixels are
processed in overlapping tiles (output stitched without seams by cropping the
overlap), which keeps the 2048^2+ activations bounded; on a 288 GB MI355X the
default tile is large (1024).
"""
from __future__ import annotations

import io

import numpy as np
import torch
from PIL import Image

from ..models.layers import init_random_fast_, prepare_model
from ..models.rrdbnet import TINY_RRDB, RRDBNet
from ..output.processor import OutputProcessor
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights


# the original ESRGAN repo's RRDB_ESRGAN_x4.pth names -> BasicSR / Real-ESRGAN names
_OLD_ESRGAN_RENAMES = {"RRDB_trunk.": "body.", ".RDB1.": ".rdb1.", ".RDB2.": ".rdb2.", ".RDB3.": ".rdb3.",
                       "trunk_conv.": "conv_body.", "upconv1.": "conv_up1.", "upconv2.": "conv_up2.",
                       "HRconv.": "conv_hr."}


def esrgan_state_dict(path: str) -> dict:
    """Real-ESRGAN x4 weights from a directory or file: ``*.safetensors`` or
    the published ``.pth`` (``params_ema`` wrapper, weights-only unpickler),
    BasicSR key names or the original ESRGAN repo's."""
    from ..models.weights import read_weights

    sd = read_weights(path)
    if any(k.startswith("RRDB_trunk.") for k in sd):
        out = {}
        for k, v in sd.items():
            for a, b in _OLD_ESRGAN_RENAMES.items():
                k = k.replace(a, b)
            out[k] = v
        sd = out
    return sd


def load_esrgan(model_name: str, device: str):
    def make():
        import os
        import re

        tiny = model_name.lower().startswith("tiny")
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        w = model_name if os.path.isfile(model_name) else ensure_weights(model_name)
        sd = esrgan_state_dict(w) if w else None
        kw = dict(TINY_RRDB) if tiny else {}
        if sd is not None and not ("conv_first.weight" in sd and "body.0.rdb1.conv1.weight" in sd):
            # e.g. SRVGGNetCompact (realesr-general-x4v3: body.N.weight, no conv_first)
            raise ValueError(f"{model_name}: not an x4 RRDBNet checkpoint (no conv_first / body.0.rdb1 weights); "
                             "only the RRDBNet Real-ESRGAN architecture is supported")
        if sd is not None:  # geometry from the checkpoint: block count, width, growth
            kw["nb"] = 1 + max(int(m.group(1)) for k in sd for m in [re.match(r"body\.(\d+)\.", k)] if m)
            kw["nf"] = int(sd["conv_first.weight"].shape[0])
            kw["gc"] = int(sd["body.0.rdb1.conv1.weight"].shape[0])
            kw["in_ch"] = int(sd["conv_first.weight"].shape[1])
            if kw["in_ch"] != 3:
                raise ValueError(f"{model_name}: {kw['in_ch']}-channel input (pixel-unshuffled x2/x1 "
                                 "Real-ESRGAN) is not supported; x4 RRDBNet only")
        with torch.device(device):
            net = RRDBNet(**kw).to(dt).eval().requires_grad_(False)
        init_random_fast_(net, seed=77, std_scale=0.5)
        if sd is not None:
            from ..models.weights import load_into

            load_into(net, sd, name=model_name)
        prepare_model(net)
        return net

    return cache().get(("esrgan", model_name, device), make)


_GRAPH_SHAPES = 4  # captured input shapes kept per network (each holds its activations' pool)


def _run_u8(net: RRDBNet, x: torch.Tensor) -> torch.Tensor:
    """uint8 [1, h, w, 3] device pixels -> uint8 [1, 4h, 4w, 3]: the whole
    network as ONE hipGraph replay per input shape (350 launches per 512^2
    upscale otherwise paid on the host), eager on CPU / reference mode."""
    from .graphs import CapturedCall, graphs_enabled

    if not graphs_enabled(x.device):
        return net(x, u8_out=True)
    graphs = net.__dict__.setdefault("_u8_graphs", {})
    key = tuple(x.shape)
    g = graphs.pop(key, None)
    if g is None:
        while len(graphs) >= _GRAPH_SHAPES:
            graphs.pop(next(iter(graphs)))  # least recently used
        g = CapturedCall(lambda x: net(x, u8_out=True), x=x)
    graphs[key] = g  # most recently used last
    return g.run(x=x)


@torch.no_grad()
def upscale_x4(net: RRDBNet, image: Image.Image, tile: int = 1024, overlap: int = 16) -> Image.Image:
    dev = net.conv_first.weight.device
    arr = np.array(image.convert("RGB"))  # (writable: torch.from_numpy)
    h, w = arr.shape[:2]
    x = torch.from_numpy(arr).to(dev, non_blocking=False)[None]  # uint8 upload; scaled on the device
    s = net.scale
    if max(h, w) <= tile:
        y = _run_u8(net, x)
    else:
        y = torch.empty(1, h * s, w * s, 3, device=dev, dtype=torch.uint8)
        for y0 in range(0, h, tile):
            for x0 in range(0, w, tile):
                ys, xs = max(0, y0 - overlap), max(0, x0 - overlap)
                ye, xe = min(h, y0 + tile + overlap), min(w, x0 + tile + overlap)
                out = _run_u8(net, x[:, ys:ye, xs:xe].contiguous())
                oy, ox = (y0 - ys) * s, (x0 - xs) * s
                th, tw = min(tile, h - y0) * s, min(tile, w - x0) * s
                y[:, y0 * s:y0 * s + th, x0 * s:x0 * s + tw] = out[:, oy:oy + th, ox:ox + tw]
    return _to_image(net, y[0])


def _to_image(net: RRDBNet, y: torch.Tensor) -> Image.Image:
    """uint8 [H, W, 3] device pixels -> PIL image through a pinned host buffer
    kept per output shape: a fresh 12 MB pageable ``.cpu()`` buffer per 2048^2
    upscale page-faulted once the process had run another pipeline (d2h 0.28
    -> 0.9 ms, fromarray 1.4 -> 3.4 ms; the upscale through this path stays
    at 17.2 ms after SD2.1 against 17.2 solo: profiles/esrgan_host_r6.txt)."""
    if y.device.type != "cuda":
        return Image.fromarray(y.numpy())
    bufs = net.__dict__.setdefault("_host_bufs", {})
    host = bufs.get(tuple(y.shape))
    if host is None:
        bufs.clear()  # one shape kept
        host = bufs[tuple(y.shape)] = torch.empty(y.shape, dtype=torch.uint8, pin_memory=True)
    host.copy_(y, non_blocking=True)
    torch.cuda.current_stream(y.device).synchronize()
    return Image.fromarray(host.numpy())  # (copies: RGB is not a PIL map mode, so the buffer is free again)

