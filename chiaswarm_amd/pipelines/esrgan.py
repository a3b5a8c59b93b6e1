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
from ..runtime.model_cache import cache, find_weights


def load_esrgan(model_name: str, device: str):
    def make():
        tiny = model_name.lower().startswith("tiny")
        dt = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
        with torch.device(device):
            net = RRDBNet(**(TINY_RRDB if tiny else {})).to(dt).eval().requires_grad_(False)
        init_random_fast_(net, seed=77, std_scale=0.5)
        w = find_weights(model_name)
        if w:
            from ..models.weights import _read_dir, load_into

            load_into(net, _read_dir(w))
        prepare_model(net)
        return net

    return cache().get(("esrgan", model_name, device), make)


@torch.no_grad()
def upscale_x4(net: RRDBNet, image: Image.Image, tile: int = 1024, overlap: int = 16) -> Image.Image:
    dev = net.conv_first.weight.device
    arr = np.asarray(image.convert("RGB"), dtype=np.float32) / 255.0
    h, w = arr.shape[:2]
    x = torch.from_numpy(arr).to(dev)[None]
    s = net.scale
    if max(h, w) <= tile:
        y = net(x)
    else:
        y = torch.empty(1, h * s, w * s, 3, device=dev, dtype=net.conv_first.weight.dtype)
        for y0 in range(0, h, tile):
            for x0 in range(0, w, tile):
                ys, xs = max(0, y0 - overlap), max(0, x0 - overlap)
                ye, xe = min(h, y0 + tile + overlap), min(w, x0 + tile + overlap)
                out = net(x[:, ys:ye, xs:xe].contiguous())
                oy, ox = (y0 - ys) * s, (x0 - xs) * s
                th, tw = min(tile, h - y0) * s, min(tile, w - x0) * s
                y[:, y0 * s:y0 * s + th, x0 * s:x0 * s + tw] = out[:, oy:oy + th, ox:ox + tw]
    img = (y.float().clamp(0, 1) * 255).round().to(torch.uint8)[0].cpu().numpy()
    return Image.fromarray(img)


def esrgan_callback(device_identifier, model_name, **kwargs):
    net = load_esrgan(model_name, device_identifier)
    image = kwargs["image"]
    out = upscale_x4(net, image, tile=int(kwargs.get("tile", 1024)))
    op = OutputProcessor(kwargs.get("outputs", ["primary"]), kwargs.get("content_type", "image/jpeg"))
    op.add_outputs([out])
    return op.get_results(), {"_class_name": "RealESRGANer", "_framework": "chiaswarm_amd",
                              "scale": net.scale, "input_size": list(image.size), "output_size": list(out.size)}
