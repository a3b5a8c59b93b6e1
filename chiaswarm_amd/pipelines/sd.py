"""Stable Diffusion family pipeline: txt2img, img2img, inpaint, ControlNet,
instruct-pix2pix and SDXL — one resident bundle of (text encoder(s), UNet, VAE
[, ControlNet]) per model, driven by the hive's pipeline kwargs.

Reference behaviour: the diffusers pipeline object built and called at
swarm/diffusion/diffusion_func.py:41-46 and :96 (kwargs forwarded verbatim from
the job), with ``pipeline_type`` names resolved at
swarm/job_arguments.py:143-145 and the pix2pix ``image_guidance_scale`` rule at
swarm/job_arguments.py:128-131.

MI355X design:
  * weights stay HBM-resident across jobs (ModelCache), no per-job reload;
  * prompt K/V for every cross-attention computed once per request;
  * the UNet step is replayed from a captured hipGraph per (batch, H, W);
  * CFG combine + sampler update + next-input cast = one fused HIP kernel;
  * VAE decode ends in a fused (x/2+0.5).clamp -> uint8 kernel; only uint8
    crosses PCIe.
"""
from __future__ import annotations

import dataclasses
import os
import math
import time
from typing import Any

import numpy as np
import torch
from PIL import Image

from .. import ops
from ..models import clip as clip_mod
from ..models import unet as unet_mod
from ..models import vae as vae_mod
from ..models.layers import init_random_fast_, prepare_model
from ..models.tokenizer import CLIPTokenizer
from ..models.xlmr import TINY_XLMR, XLMR_LARGE, XLMRConfig, XLMRobertaSeries, XLMRTokenizer
from ..schedulers import Scheduler, batch_randn, get_scheduler
from ..utils.trace import trace_range


@dataclasses.dataclass
class Family:
    name: str
    unet: unet_mod.UNetConfig
    vae: vae_mod.VAEConfig
    text: list  # list of CLIPTextConfig
    pad_with_eos: bool = True
    default_size: int = 512
    prediction_type: str = "epsilon"
    pipeline_class: str = "StableDiffusionPipeline"
    # the checkpoint's scheduler_config.json training-schedule fields, applied to
    # whichever sampler a job names (diffusers ``from_config``)
    sched_config: dict = dataclasses.field(default_factory=dict)
    from_config: bool = False  # built from the checkpoint's config files (else a named preset)
    # component directory of each text encoder (the SDXL refiner has text_encoder_2 only)
    text_names: tuple | None = None
    # SDXL refiner: (orig_h, orig_w, crop_top, crop_left, aesthetic_score) time ids
    # (diffusers StableDiffusionXLImg2ImgPipeline, requires_aesthetics_score=True)
    aesthetics: bool = False
    # SDXL: a job without a negative prompt gets ZERO negative embeddings (and
    # pooled), not the encoding of "" (diffusers force_zeros_for_empty_prompt)
    force_zeros: bool = False

    @property
    def text_components(self) -> list:
        if self.text_names:
            return list(self.text_names)
        return ["text_encoder" if i == 0 else f"text_encoder_{i + 1}" for i in range(len(self.text))]

    @property
    def tokenizer_components(self) -> list:
        return [n.replace("text_encoder", "tokenizer") for n in self.text_components]

    @property
    def is_xl(self) -> bool:  # SDXL conditioning: pooled text embeds + size/crop time ids
        return self.unet.addition_embed_type == "text_time"

    @property
    def is_pix2pix(self) -> bool:  # instruct-pix2pix: 8-channel UNet, 3-way CFG
        return self.pipeline_class == "StableDiffusionInstructPix2PixPipeline" or (
            self.unet.in_channels == 8 and self.pipeline_class != "StableDiffusionInpaintPipeline")

    @property
    def is_depth(self) -> bool:  # StableDiffusionDepth2ImgPipeline: latents + 1 depth channel
        return self.unet.in_channels == 5

    @property
    def is_image_variation(self) -> bool:  # CLIP image embedding as the only context token
        return self.pipeline_class == "StableDiffusionImageVariationPipeline"

    @property
    def is_unclip(self) -> bool:  # noised CLIP image embedding as the UNet's class embedding
        return self.pipeline_class == "StableUnCLIPImg2ImgPipeline"

    def scheduler_kwargs(self) -> dict:
        kw = dict(self.sched_config)
        kw["prediction_type"] = self.prediction_type
        return kw

    @classmethod
    def from_spec(cls, name: str, spec) -> "Family":
        """A family from a parsed diffusers directory (models/hf_config.pipeline_spec)."""
        from ..models.hf_config import scheduler_kwargs

        sk = scheduler_kwargs(spec.scheduler)
        pcls = spec.class_name
        if pcls in ("DiffusionPipeline", "StableDiffusionPipeline") and spec.unet.in_channels == 9:
            pcls = "StableDiffusionInpaintPipeline"
        if spec.unet.addition_embed_type == "text_time" and not pcls.startswith("StableDiffusionXL"):
            pcls = "StableDiffusionXLImg2ImgPipeline" if spec.requires_aesthetics_score else \
                "StableDiffusionXLPipeline"
        pad0 = spec.tokenizer_pad[0] if spec.tokenizer_pad else None
        xl = spec.unet.addition_embed_type == "text_time"
        return cls(name=name, unet=spec.unet, vae=spec.vae, text=list(spec.text),
                   pad_with_eos=(pad0 is None or pad0 == "<|endoftext|>") and spec.text_names[:1] == ("text_encoder",),
                   default_size=int(spec.unet.sample_size) * 2 ** (len(spec.vae.block_out_channels) - 1),
                   prediction_type=sk.pop("prediction_type", "epsilon"), pipeline_class=pcls, sched_config=sk,
                   from_config=True, text_names=tuple(spec.text_names),
                   aesthetics=xl and spec.requires_aesthetics_score,
                   force_zeros=xl and spec.force_zeros_for_empty_prompt)


# Named presets: random-init runs (bench, smoke) and directories without config files
FAMILIES = {
    "sd15": Family("sd15", unet_mod.SD15, vae_mod.SD_VAE, [clip_mod.CLIP_L]),
    "sd15-inpaint": Family("sd15-inpaint", unet_mod.INPAINT_SD15, vae_mod.SD_VAE, [clip_mod.CLIP_L],
                           pipeline_class="StableDiffusionInpaintPipeline"),
    "sd21": Family("sd21", unet_mod.SD21, vae_mod.SD_VAE, [clip_mod.OPENCLIP_H], pad_with_eos=False),
    "sd21-v": Family("sd21-v", unet_mod.SD21_V, vae_mod.SD_VAE, [clip_mod.OPENCLIP_H], pad_with_eos=False,
                     default_size=768, prediction_type="v_prediction"),
    "sd2-inpaint": Family("sd2-inpaint", unet_mod.INPAINT_SD2, vae_mod.SD_VAE, [clip_mod.OPENCLIP_H],
                          pad_with_eos=False, pipeline_class="StableDiffusionInpaintPipeline"),
    "pix2pix": Family("pix2pix", unet_mod.PIX2PIX, vae_mod.SD_VAE, [clip_mod.CLIP_L],
                      pipeline_class="StableDiffusionInstructPix2PixPipeline"),
    "sdxl": Family("sdxl", unet_mod.SDXL, vae_mod.SDXL_VAE, [clip_mod.CLIP_L, clip_mod.OPENCLIP_BIGG],
                   default_size=1024, pipeline_class="StableDiffusionXLPipeline", force_zeros=True),
    "sdxl-refiner": Family("sdxl-refiner", unet_mod.SDXL_REFINER, vae_mod.SDXL_VAE, [clip_mod.OPENCLIP_BIGG],
                           pad_with_eos=False, default_size=1024, pipeline_class="StableDiffusionXLImg2ImgPipeline",
                           text_names=("text_encoder_2",), aesthetics=True),
    # StableDiffusionDepth2ImgPipeline (stabilityai/stable-diffusion-2-depth) and
    # StableDiffusionImageVariationPipeline (lambdalabs/sd-image-variations-diffusers:
    # no text encoder, CLIP ViT-L/14 image embedding as the context): pipelines/variants.py
    "sd2-depth": Family("sd2-depth", unet_mod.DEPTH_SD2, vae_mod.SD_VAE, [clip_mod.OPENCLIP_H], pad_with_eos=False,
                        pipeline_class="StableDiffusionDepth2ImgPipeline"),
    "sd15-imagevar": Family("sd15-imagevar", unet_mod.SD15, vae_mod.SD_VAE, [],
                            pipeline_class="StableDiffusionImageVariationPipeline"),
    # StableUnCLIPImg2ImgPipeline (stabilityai/stable-diffusion-2-1-unclip): pipelines/variants.py
    "sd21-unclip": Family("sd21-unclip", unet_mod.SD21_UNCLIP, vae_mod.SD_VAE, [clip_mod.OPENCLIP_H],
                          pad_with_eos=False, default_size=768, prediction_type="v_prediction",
                          pipeline_class="StableUnCLIPImg2ImgPipeline"),
    # AltDiffusion (BAAI): the SD1.x UNet / VAE conditioned on XLM-RoBERTa-large + transformation
    "altdiffusion": Family("altdiffusion", unet_mod.SD15, vae_mod.SD_VAE, [XLMR_LARGE], pad_with_eos=False,
                           pipeline_class="AltDiffusionPipeline"),
    "tiny": Family("tiny", unet_mod.TINY, vae_mod.TINY_VAE, [clip_mod.TINY_TEXT], default_size=64),
    "tiny-alt": Family("tiny-alt", unet_mod.TINY, vae_mod.TINY_VAE, [TINY_XLMR], default_size=64, pad_with_eos=False,
                       pipeline_class="AltDiffusionPipeline"),
    "tiny-unclip": Family("tiny-unclip", unet_mod.TINY_UNCLIP, vae_mod.TINY_VAE, [clip_mod.TINY_TEXT],
                          default_size=64, pipeline_class="StableUnCLIPImg2ImgPipeline"),
    "tiny-depth": Family("tiny-depth", unet_mod.TINY_DEPTH, vae_mod.TINY_VAE, [clip_mod.TINY_TEXT], default_size=64,
                         pipeline_class="StableDiffusionDepth2ImgPipeline"),
    "tiny-imagevar": Family("tiny-imagevar", unet_mod.TINY, vae_mod.TINY_VAE, [], default_size=64,
                            pipeline_class="StableDiffusionImageVariationPipeline"),
    "tiny-xl": Family("tiny-xl", unet_mod.TINY_XL, vae_mod.TINY_VAE, [clip_mod.TINY_TEXT, clip_mod.TINY_TEXT_G],
                      default_size=64, pipeline_class="StableDiffusionXLPipeline", force_zeros=True),
    "tiny-xl-refiner": Family("tiny-xl-refiner", unet_mod.TINY_XL_REFINER, vae_mod.TINY_VAE, [clip_mod.TINY_TEXT_G],
                              pad_with_eos=False, default_size=64, pipeline_class="StableDiffusionXLImg2ImgPipeline",
                              text_names=("text_encoder_2",), aesthetics=True),
}


def family_for_model(model_name: str) -> str:
    """Map a hive model name (HF repo id) to a preset family — ONLY for
    directories without ``model_index.json`` (and random-init runs); a real
    checkpoint is built from its own config files (``resolve_family``)."""
    n = model_name.lower()
    if n.startswith("tiny/") or n == "tiny":
        if "altdiffusion" in n:
            return "tiny-alt"
        if "unclip" in n:
            return "tiny-unclip"
        return "tiny-depth" if "depth" in n else ("tiny-imagevar" if "variation" in n else "tiny")
    if "altdiffusion" in n:
        return "altdiffusion"
    if "unclip" in n:
        return "sd21-unclip"
    if "image-variations" in n:
        return "sd15-imagevar"
    if "stable-diffusion-2-depth" in n:
        return "sd2-depth"
    if "instruct-pix2pix" in n:
        return "pix2pix"
    if "xl" in n and "refiner" in n:
        return "sdxl-refiner"
    if "xl" in n:
        return "sdxl"
    if "inpaint" in n and ("2-" in n or "2." in n):
        return "sd2-inpaint"
    if "inpaint" in n:
        return "sd15-inpaint"
    if "stable-diffusion-2" in n:
        return "sd21" if ("base" in n or "512" in n) else "sd21-v"
    return "sd15"


def resolve_family(model_name: str, weights_dir: str | None) -> Family:
    """The architecture of ``model_name``: parsed from ``weights_dir``'s
    ``model_index.json`` + component configs when present (the reference's
    ``from_pretrained``, swarm/diffusion/diffusion_func.py:41-46), else the
    name-matched preset."""
    if weights_dir:
        from ..models.hf_config import pipeline_spec

        spec = pipeline_spec(weights_dir)
        if spec is not None:
            return Family.from_spec(model_name, spec)
    return FAMILIES[family_for_model(model_name)]


@dataclasses.dataclass
class PipelineOutput:
    images: list
    nsfw_content_detected: list
    latents: torch.Tensor | None = None
    timings: dict | None = None


class StableDiffusion:
    """Resident SD-family bundle.  ``__call__`` accepts the diffusers pipeline
    kwargs the hive forwards (prompt, negative_prompt, guidance_scale,
    num_inference_steps, num_images_per_prompt, height, width, generator,
    image, mask_image, strength, image_guidance_scale, controlnet_conditioning_scale,
    eta, cross_attention_kwargs ...)."""

    def __init__(self, family: "str | Family", device="cpu", dtype=None, seed=0, weights_dir=None,
                 with_encoder=True, controlnet=None):
        self.family = FAMILIES[family] if isinstance(family, str) else family
        self.weights_dir = weights_dir
        self.device = torch.device(device)
        if dtype is None:
            dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        self.dtype = dtype
        fam = self.family
        with torch.device(self.device):
            self.unet = unet_mod.UNet2DConditionModel(fam.unet).to(dtype)
            self.vae = vae_mod.AutoencoderKL(fam.vae, with_encoder=with_encoder).to(dtype)
            self.text_encoders = [(XLMRobertaSeries(c) if isinstance(c, XLMRConfig) else clip_mod.CLIPTextModel(c))
                                  .to(dtype) for c in fam.text]
        for i, m in enumerate([self.unet, self.vae] + self.text_encoders):
            m.eval().requires_grad_(False)
            init_random_fast_(m, seed=seed + i)
        self.weights_source = "random-init"
        self.prepared = set()
        if weights_dir is not None:
            from ..models.weights import load_sd_weights

            if load_sd_weights(self, weights_dir):
                self.weights_source = str(weights_dir)
        names = ["unet", "vae"] + fam.text_components
        for name, m in zip(names, [self.unet, self.vae] + self.text_encoders):
            if name not in self.prepared:  # loaded components were packed (or read packed) already
                prepare_model(m)
        from ..models.weights import CheckpointMismatch, tokenizer_dir

        # tokenizer/ (+ tokenizer_2/ for SDXL, whose OpenCLIP-bigG tokenizer pads with "!")
        tnames = fam.tokenizer_components
        tdirs = [tokenizer_dir(weights_dir, t) for t in tnames]
        if self.weights_source != "random-init" and None in tdirs:
            # real text-encoder weights fed hash-fallback token ids = a random prompt
            raise CheckpointMismatch(f"{weights_dir}: tokenizer files (vocab.json / merges.txt) missing for "
                                     f"{[t for t, d in zip(tnames, tdirs) if d is None]}")
        self.tokenizers = [XLMRTokenizer(tdirs[i], 77, vocab_size=c.vocab_size) if isinstance(c, XLMRConfig) else
                           CLIPTokenizer(tdirs[i], 77, pad_with_eos=fam.pad_with_eos and i == 0,
                                         vocab_size=c.vocab_size)
                           for i, c in enumerate(fam.text)]
        self.controlnet = controlnet
        self.safety_checker = None
        self.config: dict[str, Any] = {
            "_class_name": fam.pipeline_class,
            "_framework": "chiaswarm_amd",
            "unet": ["chiaswarm_amd", "UNet2DConditionModel"],
            "vae": ["chiaswarm_amd", "AutoencoderKL"],
            "text_encoder": ["chiaswarm_amd", "CLIPTextModel"],
            "tokenizer": ["chiaswarm_amd", "CLIPTokenizer"],
            "scheduler": ["chiaswarm_amd", "DPMSolverMultistepScheduler"],
            "family": fam.name,
            "weights": self.weights_source,
        }
        self._graphs: dict = {}
        self.use_graphs = self.device.type == "cuda"

    def invalidate_graphs(self):
        """Drop every captured hipGraph (they hold raw pointers to the weights
        and packed buffers): called whenever an adapter changes the weights."""
        self._graphs = {}
        self.__dict__.pop("_zero_kv", None)
        if hasattr(self, "_text_graphs"):
            del self._text_graphs
        self._kv_static = False
        for m in [self.unet] + self.text_encoders:
            for sub in m.modules():
                sub.__dict__.pop("_ln_folds", None)
                sub.__dict__.pop("_xin", None)

    # ------------------------------------------------------------------
    def _text_fn(self, ids, with_kv=True):
        """Device part of prompt encoding: every text encoder (+ the UNet's
        per-request cross-attention K/V); captured as one hipGraph per batch."""
        hs, pooled = [], None
        for i, te in enumerate(self.text_encoders):
            last, penult, pool, proj = te(ids[i])
            if self.family.is_xl:
                hs.append(penult)
                if proj is not None:
                    pooled = proj
            else:
                hs.append(last)
        ctx = torch.cat(hs, dim=-1) if len(hs) > 1 else hs[0]
        kv = tuple(self.unet.encode_context(ctx)) if with_kv else ()
        return ctx, pooled, kv

    @torch.no_grad()
    def encode(self, prompts: list[str], negatives: list[str], cfg: bool, with_kv=True):
        """(context, added_cond or None, cross-attention K/V tuple)."""
        texts = (negatives + prompts) if cfg else prompts
        ids = tuple(tok(texts).to(self.device) for tok in self.tokenizers)
        # (XLM-RoBERTa cuts each prompt's keys to its real tokens, a host-side
        # length: that encoder runs eagerly, not as a captured graph)
        if self.use_graphs and with_kv and not any(isinstance(c, XLMRConfig) for c in self.family.text):
            if not hasattr(self, "_text_graphs"):
                from .graphs import GraphCache

                self._text_graphs = GraphCache(self._text_fn)
            ctx, pooled, kv = self._text_graphs(self.device, ids=ids)
        else:
            ctx, pooled, kv = self._text_fn(ids, with_kv)
        added = {"text_embeds": pooled} if self.family.is_xl else None
        return ctx, added, kv

    @torch.no_grad()
    def encode_prompt(self, prompts: list[str], negatives: list[str], cfg: bool):
        """Returns (context [2B or B, 77, D], added_cond or None)."""
        ctx, added, _ = self.encode(prompts, negatives, cfg, with_kv=False)
        return ctx, added

    def _zero_rows_kv(self, ctx, n):
        """Every cross-attention K/V of ``n`` all-zero context rows (cached per
        context shape / dtype; dropped with the graphs when weights change)."""
        key = (n, tuple(ctx.shape[1:]), ctx.dtype, ctx.device)
        cache = self.__dict__.setdefault("_zero_kv", {})
        if key not in cache:
            cache.clear()
            z = self.unet.encode_context(ctx.new_zeros((1,) + tuple(ctx.shape[1:])))
            cache[key] = [t.expand((n,) + tuple(t.shape[1:])).contiguous() for t in z]
        return cache[key]

    def _time_ids(self, b, h, w, device, aesthetic=None, n_neg=0):
        """SDXL micro-conditioning rows: (orig_h, orig_w, crop_top, crop_left,
        target_h, target_w); the refiner's (orig_h, orig_w, crop_top, crop_left,
        aesthetic_score), the first ``n_neg`` (CFG negative) rows with the
        negative score (diffusers StableDiffusionXLImg2ImgPipeline._get_add_time_ids)."""
        if aesthetic is not None:
            pos, neg = aesthetic
            rows = [[h, w, 0, 0, neg if i < n_neg else pos] for i in range(b)]
        else:
            rows = [[h, w, 0, 0, h, w]] * b
        return torch.tensor(rows, dtype=torch.float32, device=device)

    def _phase_sync(self):
        """Phase timings are device time: sync at phase boundaries (a ~10 us
        bubble per job; the decode needs the denoised latents anyway)."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------
    def _unet_eval(self, x_in, t, cross_kv, added, cc=None, dup=False, tag=None):
        """One denoiser evaluation.  ``cc``: a ControlNet request context — on
        the graph path the ControlNet encoder copy, its zero convs (fused with
        the skip adds) and the UNet are ONE captured hipGraph.  ``tag``: part of
        the graph key (a CFG-parallel half binds different static K/V rows)."""
        share = bool(getattr(self, "_kv_static", False))
        if (not self.use_graphs or ops.get_mode() != "hip" or not ops._lib.available()
                or self.device.type != "cuda"):
            tt = torch.tensor([t], device=x_in.device, dtype=torch.float32)
            control = cc.features(x_in, tt) if cc is not None else None
            return self.unet(x_in, tt, cross_kv=cross_kv, added_cond=added, control=control,
                             cfg_dup=dup and cc is None)
        key = (x_in.shape, added is not None, len(cross_kv), share, dup,
               None if cc is None else (id(cc.model), cc.scale, tuple(cc.cond_emb.shape)), tag)
        g = self._graphs.get(key)
        if g is None:
            g = (_UNetGraph(self.unet, x_in, cross_kv, added, share_kv=share, cfg_dup=dup) if cc is None else
                 _ControlUNetGraph(self.unet, x_in, cross_kv, added, cc, share_kv=share))
            self._graphs[key] = g
        return g.run(x_in, t, cross_kv, added, cc, req=getattr(self, "_req", None))

    @torch.no_grad()
    def denoise(self, latents, sched: Scheduler, cross_kv, guidance, added=None, generator=None,
                image_latents=None, image_guidance=None, mask=None, masked_latents=None,
                init_latents=None, noise=None, control=None, cfg_split=None):
        """Sampler loop on NHWC fp32 latents.

        * guidance > 1 -> CFG batch [uncond, cond] (pix2pix: [cond, uncond-img, uncond]);
        * ``image_latents`` concatenated on channels (pix2pix / inpaint-9ch);
        * ``mask``/``init_latents`` -> legacy (4-channel) inpaint blending;
        * ``cfg_split`` = {"peer": rank, "half": 0 | 1}: CFG-parallel, this rank
          evaluates one CFG half and swaps predictions with its peer each step.
        """
        ov = self.__dict__.get("_denoise_override")
        if ov is not None:  # a sampling-loop variant class (pipelines/guided.py: Panorama, SAG)
            return ov(self, latents, sched, cross_kv, guidance, added, generator)
        b = latents.shape[0]
        cfg = guidance > 1.0
        three_way = image_guidance is not None
        nrep = 3 if three_way else (2 if cfg else 1)
        x = latents
        if cfg_split is not None:
            from ..parallel import comm

            ok = comm.cfg_handshake(int(cfg_split["peer"]))
            cfg_split["started"] = True
            if not ok:
                raise RuntimeError("CFG-parallel: the peer part failed before its denoise loop")
            if nrep == 2 and image_latents is None and mask is None and control is None:
                return self._denoise_cfg_split(x, sched, cross_kv, guidance, added, generator, cfg_split)
            # (not splittable: both parts run the whole CFG batch, identical results)
        if mask is None and self._loop_ok():
            table = sched.loop_table()
            if table is not None and len(table[0]) > 0:
                return self._denoise_loop(x, sched, table, cross_kv, guidance, added, generator, image_latents,
                                          image_guidance, nrep, control)
        while sched.step_index < sched.n:
            t = sched.current_t()
            s_in = sched.current_scale()
            xi = (x * s_in).to(self.dtype)
            parts = [xi] * nrep
            x_in = torch.cat(parts, 0) if nrep > 1 else xi
            if image_latents is not None:
                x_in = torch.cat([x_in, image_latents.to(self.dtype)], dim=-1)
            e = self._unet_eval(x_in, t, cross_kv, added, control,
                                dup=_cfg_dup(self.unet, nrep, image_latents, added))
            coeffs = sched.fused_coeffs()
            if three_way:
                e_c, e_i, e_u = e.float().chunk(3)
                e_g = e_u + guidance * (e_c - e_i) + image_guidance * (e_i - e_u)
                x = sched.step(e_g, x, generator)
            elif coeffs is not None and ops.use_hip(x) and nrep <= 2:
                need_noise = coeffs.D != 0.0
                nz = batch_randn(x.shape, generator, x.device) if need_noise else None
                x = ops.sched_step(e, x, sched, coeffs, guidance if cfg else None, nz)
            else:
                if cfg:
                    e_u, e_c = e.float().chunk(2)
                    e_g = e_u + guidance * (e_c - e_u)
                else:
                    e_g = e.float()
                x = sched.step(e_g, x, generator)
            if mask is not None and init_latents is not None:
                # legacy inpaint: keep the known region at the current noise level
                i = min(sched.step_index, sched.n - 1)
                known = init_latents if sched.step_index >= sched.n else sched.add_noise(init_latents, noise, i)
                x = known * (1 - mask) + x * mask
        return x

    def _denoise_cfg_split(self, x, sched, cross_kv, guidance, added, generator, split):
        """CFG-parallel sampler loop: rank ``half`` runs the UNet on its rows
        of the CFG batch (0: uncond, 1: cond) at batch b, the two predictions are
        swapped over the process group (comm.exchange_cfg_half), and both parts
        apply the identical guidance + scheduler update, so their latents stay
        bit-identical without further traffic.  SURVEY §2.6 "CFG-parallel"."""
        from ..parallel import comm

        peer, h = int(split["peer"]), int(split["half"])
        b = x.shape[0]
        kv = [t[h * b:(h + 1) * b] for t in cross_kv]
        add_h = {k: v[h * b:(h + 1) * b] for k, v in added.items()} if added is not None else None
        if self._loop_ok():
            table = sched.loop_table()
            if table is not None and len(table[0]) > 0:
                return self._denoise_loop_split(x, sched, table, kv, guidance, add_h, generator, peer, h)
        while sched.step_index < sched.n:
            t = sched.current_t()
            xi = (x * sched.current_scale()).to(self.dtype)
            e = comm.exchange_cfg_half(self._unet_eval(xi, t, kv, add_h, tag=("cfg", h)), peer, h)
            coeffs = sched.fused_coeffs()
            if coeffs is not None and ops.use_hip(x):
                nz = batch_randn(x.shape, generator, x.device) if coeffs.D != 0.0 else None
                x = ops.sched_step(e, x, sched, coeffs, guidance, nz)
            else:
                e_u, e_c = e.float().chunk(2)
                x = sched.step(e_u + guidance * (e_c - e_u), x, generator)
        return x

    def _loop_ok(self) -> bool:
        return (LOOP_GRAPHS and self.use_graphs and self.device.type == "cuda" and ops.get_mode() == "hip"
                and ops._lib.available())

    def _denoise_loop(self, x, sched, table, cross_kv, guidance, added, generator, image_latents,
                      image_guidance, nrep, control):
        """Device-resident sampler loop: ONE hipGraph replay per step and no
        host work in between.  The step graph is [loop_prologue (device step
        counter -> timestep), UNet (+ ControlNet), sched_loop (CFG + update ->
        the next step's bf16 UNet input written in place)]; the per-step
        scalars, the guidance scales and any sampler noise (drawn up front, in
        the order the eager loop draws it) sit in device tables."""
        from ..ops import hip_ops

        ts, rows, s0 = table
        n = len(ts)
        mode = nrep - 1
        g, g2 = (float(guidance), float(image_guidance)) if mode == 2 else (float(guidance), 0.0)
        need_noise = any(r[5] != 0.0 for r in rows)
        x_first = (x * s0).to(self.dtype)
        x_in = torch.cat([x_first] * nrep, 0) if nrep > 1 else x_first
        if image_latents is not None:
            x_in = torch.cat([x_in, image_latents.to(self.dtype)], dim=-1)
        share = bool(getattr(self, "_kv_static", False))
        cap = max(64, -(-n // 64) * 64)
        key = ("loop", x_in.shape, added is not None, len(cross_kv), share, mode, need_noise,
               None if control is None else (id(control.model), control.scale, tuple(control.cond_emb.shape)))
        gph = self._graphs.get(key)
        if gph is not None and gph.loop_cap < n:
            gph = None
        if gph is None:
            spec = _LoopSpec(tuple(x.shape), mode, cap, need_noise, x.device)
            gph = (_UNetGraph(self.unet, x_in, cross_kv, added, share_kv=share, loop=spec,
                              cfg_dup=_cfg_dup(self.unet, nrep, image_latents, added)) if control is None else
                   _ControlUNetGraph(self.unet, x_in, cross_kv, added, control, share_kv=share, loop=spec))
            self._graphs[key] = gph
        L = gph.loop
        coef = torch.zeros((n, hip_ops.LOOP_COEF_STRIDE), dtype=torch.float32)
        coef[:, :7] = torch.tensor(rows, dtype=torch.float64).float()
        coef[:, 7] = g
        coef[:, 8] = g2
        L.coef[:n].copy_(coef.to(self.device, non_blocking=False))
        L.t_tab[:n].copy_(torch.tensor(ts, dtype=torch.float32).to(self.device))
        if need_noise:
            for i, r in enumerate(rows):  # the eager loop's draw order: one draw per noisy step
                if r[5] != 0.0:
                    L.noise[i].copy_(batch_randn(x.shape, generator, x.device))
        L.x.copy_(x)
        if sched.prev_x0 is not None:
            L.x0prev.copy_(sched.prev_x0)
        else:
            L.x0prev.zero_()
        L.counter.zero_()
        if hasattr(gph, "fill_temb"):
            gph.fill_temb(L.t_tab[:n])
        gph.prepare(x_in, cross_kv, added, control, req=getattr(self, "_req", None))
        for _ in range(n):
            gph.graph.replay()
        sched.step_index = sched.n
        sched.prev_x0 = L.x0prev.clone()
        return L.x.clone()

    def _denoise_loop_split(self, x, sched, table, kv, guidance, added, generator, peer, h):
        """Device-resident CFG-parallel loop: per step ONE replay of this half's
        step graph [loop prologue, UNet at batch b, its prediction into its rows
        of the full CFG prediction], the swap with the peer enqueued on the
        stream (RCCL: no host sync), ONE replay of the update graph
        [sched_loop: CFG combine + sampler update + the next bf16 input of this
        half].  Both ranks apply the same update to the same predictions, so
        their latents stay bit-identical with no further traffic."""
        from ..parallel import comm

        ts, rows, s0 = table
        n = len(ts)
        need_noise = any(r[5] != 0.0 for r in rows)
        x_in = (x * s0).to(self.dtype)
        share = False  # this half binds a row slice of the static K/V: own copies
        cap = max(64, -(-n // 64) * 64)
        key = ("loop-split", h, x_in.shape, added is not None, len(kv), need_noise)
        gph = self._graphs.get(key)
        if gph is not None and gph.loop_cap < n:
            gph = None
        if gph is None:
            spec = _LoopSpec(tuple(x.shape), 1, cap, need_noise, x.device)
            gph = _SplitStepGraph(self.unet, x_in, kv, added, h, spec, share_kv=share)
            self._graphs[key] = gph
        L = gph.loop
        from ..ops import hip_ops

        coef = torch.zeros((n, hip_ops.LOOP_COEF_STRIDE), dtype=torch.float32)
        coef[:, :7] = torch.tensor(rows, dtype=torch.float64).float()
        coef[:, 7] = float(guidance)
        L.coef[:n].copy_(coef.to(self.device, non_blocking=False))
        L.t_tab[:n].copy_(torch.tensor(ts, dtype=torch.float32).to(self.device))
        if need_noise:
            for i, r in enumerate(rows):
                if r[5] != 0.0:
                    L.noise[i].copy_(batch_randn(x.shape, generator, x.device))
        L.x.copy_(x)
        if sched.prev_x0 is not None:
            L.x0prev.copy_(sched.prev_x0)
        else:
            L.x0prev.zero_()
        L.counter.zero_()
        gph.fill_temb(L.t_tab[:n])
        gph.prepare(x_in, kv, added, None, req=getattr(self, "_req", None))
        for _ in range(n):
            gph.graph.replay()
            comm.exchange_cfg_half_into(gph.e_full, peer, h)
            gph.update.replay()
        sched.step_index = sched.n
        sched.prev_x0 = L.x0prev.clone()
        return L.x.clone()

    @torch.no_grad()
    def decode(self, latents, to_host=True) -> torch.Tensor:
        """NHWC fp32 latents -> uint8 NHWC images (on the host unless to_host=False)."""
        z = latents / self.vae.cfg.scaling_factor
        img = ops.vae_postprocess(self.vae.decode(z))
        return img.cpu() if to_host else img

    @torch.no_grad()
    def encode_image(self, images: list[Image.Image], h, w, generator=None, sample=True):
        arr = np.stack([np.asarray(im.convert("RGB").resize((w, h), Image.Resampling.LANCZOS))
                        for im in images]).astype(np.float32) / 127.5 - 1.0
        x = torch.from_numpy(arr).to(self.device)
        lat = self.vae.encode(x, generator=generator, sample=sample)
        return lat * self.vae.cfg.scaling_factor

    # ------------------------------------------------------------------
    @torch.no_grad()
    def __call__(self, prompt="", negative_prompt=None, num_inference_steps=30, guidance_scale=7.5,
                 num_images_per_prompt=1, height=None, width=None, generator=None, image=None,
                 mask_image=None, strength=0.8, image_guidance_scale=None, scheduler=None,
                 controlnet_conditioning_scale=1.0, output_type="pil", latents=None, eta=0.0, cfg_split=None,
                 depth_map=None, **unexpected):
        aesthetic = (float(unexpected.pop("aesthetic_score", 6.0)),
                     float(unexpected.pop("negative_aesthetic_score", 2.5))) if self.family.aesthetics else None
        if unexpected:  # the diffusers call raises on unknown kwargs too (a retryable job error)
            raise TypeError(f"{self.family.pipeline_class}.__call__() got unexpected keyword arguments "
                            f"{sorted(unexpected)}")
        t0 = time.perf_counter()
        timings = {}
        prompts = prompt if isinstance(prompt, list) else [prompt]
        prompts = [p for p in prompts for _ in range(num_images_per_prompt)]
        b = len(prompts)
        negs = negative_prompt if isinstance(negative_prompt, list) else [negative_prompt] * b
        if len(negs) != b:
            negs = [negs[0]] * b
        is_pix2pix = self.family.is_pix2pix
        cfg = guidance_scale > 1.0 or is_pix2pix
        # rows without a negative prompt (None): SDXL zeroes their embeddings
        zero_neg = [i for i, n in enumerate(negs) if n is None] if (cfg and self.family.force_zeros) else []
        negs = [n if n is not None else "" for n in negs]
        sched = scheduler or get_scheduler("DPMSolverMultistepScheduler", **self.family.scheduler_kwargs())
        sched.prediction_type = self.family.prediction_type
        if eta and sched.accepts_eta:  # diffusers forwards eta only to samplers whose step takes it (DDIM)
            sched.eta = float(eta)

        if image is not None and not isinstance(image, list):
            image = [image]
        if image is not None and (height is None or width is None):
            width, height = image[0].size
        height = height or self.family.default_size
        width = width or self.family.default_size
        height, width = (height // 8) * 8, (width // 8) * 8
        lh, lw = height // 8, width // 8

        if is_pix2pix:
            ctx, added = self.encode_prompt(prompts, negs, cfg)
            # [cond, cond (image-only guidance), uncond]
            ctx_c, ctx_u = ctx[b:], ctx[:b]
            ctx = torch.cat([ctx_c, ctx_u, ctx_u], 0)
            cross_kv = self.unet.encode_context(ctx)
        else:
            # text encoders + cross-attention K/V in one hipGraph replay on the GPU
            with trace_range("text_encode"):
                ctx, added, cross_kv = self.encode(prompts, negs, cfg)
            cross_kv = list(cross_kv)
            if zero_neg:
                # SDXL force_zeros_for_empty_prompt: zero negative context and
                # pooled embedding; their cross-attention K/V (bias only) are
                # rewritten into the text graph's static outputs
                rows = torch.tensor(zero_neg, device=ctx.device)
                ctx = ctx.index_fill(0, rows, 0)
                if added is not None and added.get("text_embeds") is not None:
                    added["text_embeds"] = added["text_embeds"].index_fill(0, rows, 0)
                # the K/V GEMMs are per token: a zero context row's K/V is the
                # projection bias, the same every request -> cached once, copied
                # in one multi-tensor launch (re-running all ~70 SDXL K/V GEMMs
                # eagerly cost ~2 ms per job)
                zkv = self._zero_rows_kv(ctx, len(zero_neg))
                if zero_neg == list(range(len(zero_neg))):
                    torch._foreach_copy_([dst[:len(zero_neg)] for dst in cross_kv], zkv)
                else:
                    for dst, z in zip(cross_kv, zkv):
                        dst.index_copy_(0, rows, z)
        # K/V are the text graph's static outputs (rewritten in place per request)
        self._kv_static = (not is_pix2pix) and self.use_graphs and hasattr(self, "_text_graphs") and \
            ops.get_mode() == "hip" and ops._lib.available()
        self._req = getattr(self, "_req", 0) + 1
        if added is not None and self.family.is_xl:
            nrep = ctx.shape[0] // b
            added["time_ids"] = self._time_ids(nrep * b, height, width, self.device, aesthetic, b if cfg else 0)
        self._phase_sync()
        timings["text_encode"] = time.perf_counter() - t0

        sched.set_timesteps(num_inference_steps)
        # caller-supplied latents (coalesced batches) already consumed the
        # generators' initial-noise draw: drawing again would shift every
        # later sampler-noise draw away from the job's solo run
        noise = None if (latents is not None and image is None) else batch_randn(
            (b, 4, lh, lw), generator, self.device).permute(0, 2, 3, 1).contiguous()
        image_latents = mask_t = init_latents = None
        start = 0
        img_guid = None
        if is_pix2pix and image is not None:
            il = self.encode_image(image * (b // len(image)) if len(image) < b else image, height, width,
                                   generator, sample=False)
            il = il / self.vae.cfg.scaling_factor  # pix2pix uses unscaled mode latents
            image_latents = torch.cat([il, il, torch.zeros_like(il)], 0)
            img_guid = image_guidance_scale if image_guidance_scale is not None else 1.5
            x = noise * sched.init_noise_sigma
        elif image is not None and self.controlnet is None:
            # img2img / inpaint: start part-way down the ladder
            init_latents = self.encode_image(image[:1] * b if len(image) < b else image, height, width, generator)
            start = min(int(num_inference_steps * (1 - strength)), num_inference_steps - 1)
            sched.step_index = start
            if hasattr(sched, "_i"):
                sched._i = start
            x = sched.add_noise(init_latents, noise, start)
            if self.family.is_depth:
                # Depth2Img: the [-1, 1]-normalised depth of the input at latent
                # size is the UNet's fifth input channel (CFG-duplicated)
                from .variants import depth_latents

                d = depth_latents(self, image[:1] * b if len(image) < b else image, lh, lw, depth_map)
                image_latents = torch.cat([d] * (2 if cfg else 1), 0)
                init_latents = None
            if mask_image is not None:
                m = np.asarray(mask_image.convert("L").resize((lw, lh), Image.Resampling.NEAREST),
                               dtype=np.float32) / 255.0
                mask_t = torch.from_numpy((m > 0.5).astype(np.float32)).to(self.device)[None, :, :, None]
                if self.unet.cfg.in_channels == 9:
                    masked = self.encode_image(
                        [_apply_mask(im, mask_image) for im in (image[:1] * b if len(image) < b else image)],
                        height, width, generator, sample=False)
                    mk = mask_t.expand(b, lh, lw, 1)
                    il = torch.cat([mk, masked], dim=-1)
                    image_latents = torch.cat([il] * (2 if cfg else 1), 0)
                    mask_t = None
                    init_latents = None
        elif noise is not None:
            x = noise * sched.init_noise_sigma
        if latents is not None:
            x = latents.to(self.device).float()

        control = None
        if self.controlnet is not None and image is not None:
            control = self.controlnet.make_context(image, height, width, b, 2 if cfg else 1,
                                                   ctx, controlnet_conditioning_scale, self.dtype)
            control.req = getattr(self, "_req", None)
        timings["prepare"] = time.perf_counter() - t0 - timings["text_encode"]
        t1 = time.perf_counter()
        with trace_range("denoise"):
            x = self.denoise(x, sched, cross_kv, guidance_scale, added, generator,
                             image_latents=image_latents, image_guidance=img_guid,
                             mask=mask_t, init_latents=init_latents, noise=noise, control=control,
                             cfg_split=cfg_split)
            self._phase_sync()
        timings["denoise"] = time.perf_counter() - t1
        if output_type == "latent":
            return PipelineOutput([], [False] * b, x, timings)
        t2 = time.perf_counter()
        with trace_range("vae_decode"):
            imgs = self.decode(x, to_host=False)
        nsfw = [False] * b
        if self.safety_checker is not None:  # on the device, before the D2H copy
            nsfw, imgs = self.safety_checker(imgs)
        if output_type == "uint8_device":  # a split-job part: sent device-to-device to the leader
            timings["decode"] = time.perf_counter() - t2
            return PipelineOutput(imgs, nsfw, x, timings)
        imgs = imgs.cpu()
        timings["decode"] = time.perf_counter() - t2
        pil = [Image.fromarray(a.numpy()) for a in imgs] if output_type == "pil" else imgs
        return PipelineOutput(pil, nsfw, x, timings)


def _apply_mask(image: Image.Image, mask: Image.Image) -> Image.Image:
    arr = np.asarray(image.convert("RGB")).copy()
    m = np.asarray(mask.convert("L").resize(image.size)) > 127
    arr[m] = 0
    return Image.fromarray(arr)


def _cfg_dup(unet, nrep, image_latents, added) -> bool:
    """True when the UNet input's two CFG halves are identical copies with the
    same time embedding (plain 2-way CFG on a conditional UNet: no per-half
    image latents, no per-half added conditioning such as SDXL's pooled text
    embeds), so UNet2DConditionModel.forward may share the prefix up to the
    first cross-attention (``CFG_SHARE_PREFIX``)."""
    return (CFG_SHARE_PREFIX and nrep == 2 and image_latents is None and added is None
            and hasattr(unet, "down_blocks"))


CFG_SHARE_PREFIX = os.environ.get("CSK_CFG_SHARE", "1") != "0"
TEMB_TABLE = os.environ.get("CSK_TEMB_TABLE", "1") != "0"  # per-request time-projection table in the loop graph
ADD_EMB_CACHE = os.environ.get("CSK_ADD_EMB_CACHE", "1") != "0"  # SDXL text_time embedding once per request
LOOP_GRAPHS = True  # device-resident sampler loop (StableDiffusion._denoise_loop); False: per-step host loop


class _LoopSpec:
    """Static device buffers of a device-resident sampler loop (fixed pointers
    captured into the step graph): latents / previous x0 (fp32 NHWC), step
    counter, per-step timestep and coefficient tables sized for ``cap`` steps,
    optional per-step noise table."""

    def __init__(self, shape, mode, cap, need_noise, device):
        from ..ops import hip_ops

        self.mode, self.cap = mode, cap
        self.x = torch.zeros(shape, dtype=torch.float32, device=device)
        self.x0prev = torch.zeros(shape, dtype=torch.float32, device=device)
        self.counter = torch.zeros(1, dtype=torch.int32, device=device)
        self.cur = torch.zeros(1, dtype=torch.int32, device=device)
        self.t_tab = torch.zeros(cap, dtype=torch.float32, device=device)
        self.coef = torch.zeros((cap, hip_ops.LOOP_COEF_STRIDE), dtype=torch.float32, device=device)
        self.noise = torch.zeros((cap,) + tuple(shape), dtype=torch.float32, device=device) if need_noise else None


class _UNetGraph:
    """hipGraph of one UNet forward at a fixed (batch, H, W): static input
    buffers are refreshed by ``copy_`` before each replay.  With ``loop`` the
    graph is a whole sampler step (see StableDiffusion._denoise_loop)."""

    _temb_ok = True  # the step's UNet forward may take precomputed time projections

    def __init__(self, unet, x_in, cross_kv, added, warmup=2, share_kv=False, loop=None, cfg_dup=False):
        self.unet = unet
        self.loop = loop
        self.cfg_dup = cfg_dup  # x_in's two halves are identical CFG copies (UNet forward cfg_dup)
        self.loop_cap = loop.cap if loop is not None else 0
        self.x = x_in.clone()
        self.t = torch.zeros(1, device=x_in.device, dtype=torch.float32)
        # share_kv: the K/V are another graph's static outputs -> capture them directly
        self.kv = list(cross_kv) if share_kv else [k.clone() for k in cross_kv]
        self._kv_req = None
        self.added = {k: v.clone() for k, v in added.items()} if added else None
        # SDXL: the text_time addition embedding is constant over a request, so
        # the graph reads it from a static buffer filled in prepare() (the
        # add_embedding GEMMs and their sinusoidal inputs leave every step)
        self._add_req = None
        if self.added is not None and getattr(unet.cfg, "addition_embed_type", None) == "text_time" and ADD_EMB_CACHE:
            self.added["add_emb"] = unet.add_emb(self.added)
        # device-resident loop: the ResNet time projections of every step come
        # from a per-request table (UNet2DConditionModel.temb_table) gathered by
        # the step's device index, not recomputed (5 small kernels) every step
        self.temb_tab = self.temb_row = None
        if loop is not None and added is None and hasattr(unet, "temb_table") and TEMB_TABLE and self._temb_ok:
            width = sum(unet._resnets()[i].out_channels for i in range(len(unet._resnets())))
            self.temb_tab = torch.zeros((loop.cap, width), dtype=x_in.dtype, device=x_in.device)
            self.temb_row = torch.zeros((x_in.shape[0], width), dtype=x_in.dtype, device=x_in.device)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._fwd()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._fwd()

    def _fwd(self):
        if self.loop is None:
            return self._unet_fwd()
        from ..ops import hip_ops

        L = self.loop
        hip_ops.loop_prologue(L.counter, L.cur, L.t_tab, self.t)
        e = self._unet_fwd().contiguous()
        hip_ops.sched_loop(e, L.x, L.x0prev, L.noise, L.cur, L.coef, self.x, L.mode)
        return e

    def _unet_fwd(self):
        kw = {}
        if self.temb_tab is not None:
            from ..ops import hip_ops

            hip_ops.row_bcast(self.temb_row, self.temb_tab, self.loop.cur)
            kw["temb_proj"] = self.temb_row
        if self.cfg_dup:
            kw["cfg_dup"] = True
        return self.unet(self.x, self.t, cross_kv=self.kv, added_cond=self.added, **kw)

    def fill_temb(self, t_tab):
        """Per-request time-projection table for the step timesteps ``t_tab``."""
        if self.temb_tab is not None:
            self.temb_tab[: t_tab.numel()].copy_(self.unet.temb_table(t_tab))

    def prepare(self, x_in, cross_kv, added, cc=None, req=None):
        self.x.copy_(x_in)
        # per-request cross-attention K/V: copied into the graph's static buffers
        # once per request (a no-op when they ARE the text-encoder graph's static
        # outputs, which that graph rewrites in place for every request)
        if req != self._kv_req:
            for dst, src in zip(self.kv, cross_kv):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src)
            self._kv_req = req
            self._new_request(cc)
        if added:
            for k, v in added.items():
                self.added[k].copy_(v)
            if "add_emb" in self.added and (req is None or req != self._add_req):
                self.added["add_emb"].copy_(self.unet.add_emb(self.added))
                self._add_req = req

    def run(self, x_in, t, cross_kv, added, cc=None, req=None):
        self.prepare(x_in, cross_kv, added, cc, req)
        self.t.fill_(float(t))
        self.graph.replay()
        return self.out

    def _new_request(self, cc):
        pass


class _SplitStepGraph(_UNetGraph):
    """A CFG-parallel half's sampler step as two hipGraphs around the
    prediction swap: ``graph`` = [loop prologue, UNet on this half's b rows, its
    prediction copied into rows [h*b, (h+1)*b) of the static ``e_full``];
    ``update`` = [sched_loop over the full [u; c] prediction, writing this
    half's next bf16 input]."""

    def __init__(self, unet, x_in, cross_kv, added, half, loop, share_kv=False):
        self.half = half
        b = x_in.shape[0]
        self.e_full = torch.zeros((2 * b,) + tuple(x_in.shape[1:3]) + (unet.cfg.out_channels,), dtype=x_in.dtype,
                                  device=x_in.device)
        super().__init__(unet, x_in, cross_kv, added, share_kv=share_kv, loop=loop)
        from ..ops import hip_ops

        L = self.loop
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hip_ops.sched_loop(self.e_full, L.x.clone(), L.x0prev.clone(), L.noise, L.cur, L.coef, self.x.clone(), 1,
                               reps=1)
        torch.cuda.current_stream().wait_stream(s)
        self.update = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.update):
            hip_ops.sched_loop(self.e_full, L.x, L.x0prev, L.noise, L.cur, L.coef, self.x, 1, reps=1)

    def _fwd(self):
        from ..ops import hip_ops

        L = self.loop
        hip_ops.loop_prologue(L.counter, L.cur, L.t_tab, self.t)
        e = self._unet_fwd()
        b = self.x.shape[0]
        self.e_full[self.half * b:(self.half + 1) * b].copy_(e)
        return e


class _ControlUNetGraph(_UNetGraph):
    """ControlNet encoder copy + zero convs fused into the skip merges + UNet,
    all in one hipGraph (the reference ran ControlNet and UNet as separate eager
    modules every step, swarm/diffusion/diffusion_func.py:29-39 -> :96).  The
    conditioning embedding and the ControlNet's prompt K/V are static buffers
    refreshed once per request; the conditioning scale is part of the graph key."""

    _temb_ok = False  # the ControlNet copy embeds the timestep itself

    def __init__(self, unet, x_in, cross_kv, added, cc, warmup=2, share_kv=False, loop=None):
        self.cn, self.scale = cc.model, cc.scale
        self.cond = cc.cond_emb.clone()
        self.ckv = [k.clone() for k in cc.kv]
        super().__init__(unet, x_in, cross_kv, added, warmup=warmup, share_kv=share_kv, loop=loop)

    def _unet_fwd(self):
        from .controlnet import ControlFeatures

        feats, mid = self.cn.features(self.x[..., :self.cn.cfg.in_channels], self.t, self.cond, cross_kv=self.ckv)
        control = ControlFeatures(self.cn, feats, mid, self.scale)
        return self.unet(self.x, self.t, cross_kv=self.kv, added_cond=self.added, control=control)

    def _new_request(self, cc):
        self.cond.copy_(cc.cond_emb)
        for dst, src in zip(self.ckv, cc.kv):
            dst.copy_(src)
