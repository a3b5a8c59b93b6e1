"""ControlNet conditioning for the SD pipeline (reference: ControlNet load at
swarm/diffusion/diffusion_func.py:29-39; StableDiffusionControlNetPipeline
selected at swarm/job_arguments.py:116-124).

Per job (not per step): the conditioning image is embedded once by the
ControlNet's cond-embedding convs and the prompt K/V of every ControlNet
cross-attention are computed once; per step only the ControlNet encoder copy
runs, and its 13 residuals feed the UNet skip tensors.
"""
from __future__ import annotations

import numpy as np
import torch
from PIL import Image

from ..models.controlnet import ControlNetModel
from ..models.layers import init_random_fast_, prepare_model
from ..runtime.model_cache import cache, find_weights
from ..utils import stable_seed


class ControlNetRunner:
    def __init__(self, model: ControlNetModel, name: str):
        self.model = model
        self.name = name

    def make_fn(self, image, height, width, b, nrep, ctx, scale, dtype):
        im = image[0] if isinstance(image, list) else image
        arr = np.asarray(im.convert("RGB").resize((width, height), Image.Resampling.BICUBIC), dtype=np.float32) / 255.0
        dev = self.model.conv_in.weight.device
        cond = torch.from_numpy(arr).to(dev)[None].expand(b * nrep, -1, -1, -1).contiguous()
        with torch.no_grad():
            cond_emb = self.model.embed_cond(cond)
            kv = self.model.encode_context(ctx)
        scale = float(scale if not isinstance(scale, (list, tuple)) else scale[0])

        def fn(x_in, t):
            tt = torch.tensor([float(t)], device=dev, dtype=torch.float32)
            with torch.no_grad():
                downs, mid = self.model(x_in[..., :self.model.cfg.in_channels], tt, cond_emb, cross_kv=kv,
                                        scale=scale)
            return {"down_residuals": downs, "mid_residual": mid}

        return fn


def load_controlnet(name: str, pipe, device_identifier: str, revision: str = "main") -> ControlNetRunner:
    def make():
        cfg = pipe.unet.cfg
        with torch.device(device_identifier):
            m = ControlNetModel(cfg).to(pipe.dtype).eval().requires_grad_(False)
        init_random_fast_(m, seed=stable_seed(name))
        w = find_weights(name, revision)
        if w:
            from ..models.weights import _read_dir, load_into

            load_into(m, _read_dir(w))
        prepare_model(m)
        return ControlNetRunner(m, name)

    return cache().get(("controlnet", name, revision, device_identifier), make)
