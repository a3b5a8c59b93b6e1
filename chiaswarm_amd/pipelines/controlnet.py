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
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights
from ..utils import stable_seed


class ControlFeatures:
    """One step's ControlNet output, merged into the UNet skips lazily."""

    def __init__(self, model, feats, mid, scale):
        self.model, self.feats, self.mid, self.scale = model, feats, mid, scale

    def merge_skip(self, i, unet_skip):
        return self.model.merge_skip(i, self.feats[i], unet_skip, self.scale)

    def merge_mid(self, unet_h):
        return self.model.merge_mid(self.mid, unet_h, self.scale)


class ControlContext:
    """Per-request ControlNet state: the embedded conditioning image and the
    ControlNet's cross-attention K/V (both constant over the denoising loop)."""

    def __init__(self, runner, cond_emb, kv, scale):
        self.runner, self.model = runner, runner.model
        self.cond_emb, self.kv, self.scale = cond_emb, kv, scale

    def features(self, x_in, t):
        """Eager per-step evaluation (CPU / reference mode)."""
        dev = self.cond_emb.device
        tt = t if torch.is_tensor(t) else torch.tensor([float(t)], device=dev, dtype=torch.float32)
        with torch.no_grad():
            feats, mid = self.model.features(x_in[..., :self.model.cfg.in_channels], tt, self.cond_emb,
                                             cross_kv=self.kv)
        return ControlFeatures(self.model, feats, mid, self.scale)


class ControlNetRunner:
    def __init__(self, model: ControlNetModel, name: str):
        self.model = model
        self.name = name

    def make_context(self, image, height, width, b, nrep, ctx, scale, dtype) -> ControlContext:
        im = image[0] if isinstance(image, list) else image
        arr = np.asarray(im.convert("RGB").resize((width, height), Image.Resampling.BICUBIC), dtype=np.float32) / 255.0
        dev = self.model.conv_in.weight.device
        cond = torch.from_numpy(arr).to(dev)[None].expand(b * nrep, -1, -1, -1).contiguous()
        with torch.no_grad():
            cond_emb = self.model.embed_cond(cond)
            kv = self.model.encode_context(ctx)
        scale = float(scale if not isinstance(scale, (list, tuple)) else scale[0])
        return ControlContext(self, cond_emb, kv, scale)

    def make_fn(self, image, height, width, b, nrep, ctx, scale, dtype):
        """diffusers-style per-step residuals (down list, mid) — kept for callers
        that want the residual tensors themselves."""
        cc = self.make_context(image, height, width, b, nrep, ctx, scale, dtype)

        def fn(x_in, t):
            tt = torch.tensor([float(t)], device=cc.cond_emb.device, dtype=torch.float32)
            with torch.no_grad():
                downs, mid = self.model(x_in[..., :self.model.cfg.in_channels], tt, cc.cond_emb, cross_kv=cc.kv,
                                        scale=cc.scale)
            return {"down_residuals": downs, "mid_residual": mid}

        return fn


def load_controlnet(name: str, pipe, device_identifier: str, revision: str = "main") -> ControlNetRunner:
    def make():
        w = ensure_weights(name, revision)
        cfg, kw = pipe.unet.cfg, {}
        from ..models.hf_config import component_config, controlnet_config

        raw = component_config(w, "")
        if raw is not None:  # the checkpoint's own config.json (diffusers ControlNetModel.from_pretrained)
            cfg, kw = controlnet_config(raw)
            ux = pipe.unet.cfg.cross_attention_dim
            if (tuple(cfg.block_out_channels) != tuple(pipe.unet.cfg.block_out_channels)
                    or cfg.cross_attention_dim != ux):
                raise ValueError(f"ControlNet {name} (channels {tuple(cfg.block_out_channels)}, cross-attention "
                                 f"{cfg.cross_attention_dim}) does not fit the UNet of this model (channels "
                                 f"{tuple(pipe.unet.cfg.block_out_channels)}, cross-attention {ux})")
        with torch.device(device_identifier):
            m = ControlNetModel(cfg, **kw).to(pipe.dtype).eval().requires_grad_(False)
        init_random_fast_(m, seed=stable_seed(name))
        if w:
            from ..models.weights import load_component

            load_component(m, w, "")
        prepare_model(m)
        return ControlNetRunner(m, name)

    return cache().get(("controlnet", name, revision, device_identifier), make)
