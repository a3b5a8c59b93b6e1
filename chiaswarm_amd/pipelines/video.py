"""Video workflows.

txt2vid (reference swarm/video/tx2vid.py:17-76): ModelScope text-to-video
(UNet3D + SD VAE + OpenCLIP-H text encoder), default 25 frames, DPM-Solver++
Karras, exported at 8 fps; frames stay on the GPU for the whole denoise (the
video is one [B*F, h, w, 4] latent batch) and are VAE-decoded as one batch.
Every UNet3D step replays from a shape-keyed hipGraph (``GraphCache``) and the
CFG combine + DPM-Solver++ update run as the fused ``sched_step`` kernel.

vid2vid (reference swarm/video/pix2pix.py:14-87): instruct-pix2pix applied to
every frame (<= 100 frames, 512 px), Euler-ancestral Karras, default 15 steps,
guidance 7.5 / image guidance 1.5, cost = 512*512*steps*frames.  MI355X change:
frames are processed in BATCHES through one pix2pix pipeline call (3-way CFG
batch of 3*n frames per UNet step) instead of one pipeline call per frame with
a JPEG round trip on disk, and the seeded generator is honoured (the reference
ignored it).
"""
from __future__ import annotations

import io
import os

import numpy as np
import torch

from ..models import clip as clip_mod
from ..models import unet3d, vae as vae_mod
from ..models.layers import init_random_fast_, prepare_model
from ..models.tokenizer import CLIPTokenizer
from ..output.media import frames_to_video, read_video_frames
from ..output.processor import image_to_buffer, make_result
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights
from ..schedulers import batch_randn, get_scheduler
from .graphs import GraphCache


class TextToVideo:
    def __init__(self, model_name, device, dtype=None, tiny=False):
        self.device = torch.device(device)
        self.dtype = dtype or (torch.bfloat16 if self.device.type == "cuda" else torch.float32)
        ucfg = unet3d.TINY_T2V if tiny else unet3d.T2V
        tcfg = clip_mod.TINY_TEXT if tiny else clip_mod.OPENCLIP_H
        vcfg = vae_mod.TINY_VAE if tiny else vae_mod.SD_VAE
        w = ensure_weights(model_name)
        self.sched_config = {}
        if w:  # the checkpoint's own configs (the reference: from_pretrained, swarm/video/tx2vid.py:24-30)
            from ..models import hf_config as hc

            uc, tc, vc = (hc.component_config(w, s) for s in ("unet", "text_encoder", "vae"))
            ucfg = hc.unet3d_config(uc) if uc else ucfg
            tcfg = hc.clip_text_config(tc) if tc else tcfg
            vcfg = hc.vae_config(vc) if vc else vcfg
            self.sched_config = hc.scheduler_kwargs(hc.component_config(w, "scheduler", "scheduler_config.json"))
        with torch.device(self.device):
            self.unet = unet3d.UNet3DConditionModel(ucfg).to(self.dtype)
            self.vae = vae_mod.AutoencoderKL(vcfg, with_encoder=False).to(self.dtype)
            self.text = clip_mod.CLIPTextModel(tcfg).to(self.dtype)
        for i, m in enumerate((self.unet, self.vae, self.text)):
            m.eval().requires_grad_(False)
            init_random_fast_(m, seed=21 + i)
        from ..models.weights import _VAE_RENAMES, CheckpointMismatch, load_component, tokenizer_dir

        loaded = []
        if w:
            for sub, m in (("unet", self.unet), ("vae", self.vae), ("text_encoder", self.text)):
                if load_component(m, w, sub, _VAE_RENAMES if sub == "vae" else None) is not None:
                    loaded.append(sub)
            if loaded and len(loaded) != 3:
                raise CheckpointMismatch(f"{w}: only {loaded} of unet / vae / text_encoder have weights")
            if loaded and tokenizer_dir(w) is None:
                raise CheckpointMismatch(f"{w}: tokenizer files missing beside real text-encoder weights")
        for m in (self.unet, self.vae, self.text):
            prepare_model(m)
        self.tok = CLIPTokenizer(tokenizer_dir(w), 77, pad_with_eos=False, vocab_size=tcfg.vocab_size)
        self._graphs = GraphCache(self._step)
        self.config = {"_class_name": "TextToVideoSDPipeline", "_framework": "chiaswarm_amd",
                       "unet": ["chiaswarm_amd", "UNet3DConditionModel"], "weights": w or "random-init"}

    def _step(self, x, t, kv, frames):
        return self.unet(x, t, frames, list(kv))

    @torch.no_grad()
    def __call__(self, prompt="", negative_prompt="", num_frames=25, num_inference_steps=25, guidance_scale=9.0,
                 height=256, width=256, generator=None, scheduler=None, **_):
        sched = scheduler or get_scheduler("DPMSolverMultistepScheduler", **self.sched_config)
        sched.set_timesteps(num_inference_steps)
        ids = self.tok([negative_prompt or "", prompt]).to(self.device)
        ctx = self.text(ids)[0]
        kv = self.unet.encode_context(ctx, num_frames)
        lh, lw = height // 8, width // 8
        x = torch.randn((1, 4, num_frames, lh, lw), generator=generator, device=self.device,
                        dtype=torch.float32).permute(0, 2, 3, 4, 1).reshape(num_frames, lh, lw, 4).contiguous()
        x = x * sched.init_noise_sigma
        from .. import ops

        t_dev = torch.zeros(1, device=self.device, dtype=torch.float32)
        while sched.step_index < sched.n:
            t_dev.fill_(float(sched.current_t()))
            xi = (x * sched.current_scale()).to(self.dtype)
            e = self._graphs(self.device, x=torch.cat([xi, xi], 0), t=t_dev, kv=tuple(kv), frames=num_frames)
            coeffs = sched.fused_coeffs()
            if coeffs is not None and ops.use_hip(x):
                nz = batch_randn(x.shape, generator, x.device) if coeffs.D != 0.0 else None
                x = ops.sched_step(e, x, sched, coeffs, guidance_scale, nz)
            else:
                e_u, e_c = e.float().chunk(2)
                x = sched.step(e_u + guidance_scale * (e_c - e_u), x, generator)
        img = self.vae.decode(x / self.vae.cfg.scaling_factor)
        return ops.vae_postprocess(img).cpu().numpy()  # [F, H, W, 3] uint8


def load_t2v(model_name, device):
    return cache().get(("t2v", model_name, device),
                       lambda: TextToVideo(model_name, device, tiny=model_name.lower().startswith("tiny")))


def txt2vid_diffusion_callback(device_identifier, model_name, **kwargs):
    scheduler_type = kwargs.pop("scheduler_type", "DPMSolverMultistepScheduler")
    kwargs.pop("pipeline_type", None)
    kwargs["num_frames"] = kwargs.pop("num_frames", 25)
    content_type = kwargs.pop("content_type", "video/mp4")
    kwargs.pop("outputs", None)
    kwargs.pop("revision", None)
    kwargs.pop("variant", None)
    pipe = load_t2v(model_name, device_identifier)
    # the checkpoint's own scheduler config + Karras sigmas (reference:
    # scheduler_type.from_config(pipeline.scheduler.config, use_karras_sigmas=True),
    # swarm/video/tx2vid.py:32-34)
    frames = pipe(scheduler=get_scheduler(scheduler_type, **pipe.sched_config), **kwargs)
    video, ct = frames_to_video(frames, 8, content_type)
    from PIL import Image

    thumb = image_to_buffer(Image.fromarray(frames[0]), "image/jpeg")
    return {"primary": make_result(io.BytesIO(video), thumb, ct)}, dict(pipe.config)


def model_video_callback(device_identifier, model_name, **kwargs):
    from ..jobs.inputs import download_video
    from .diffusion import load_sd

    prompt = kwargs.get("prompt", "")
    negative_prompt = kwargs.pop("negative_prompt", "")
    guidance_scale = kwargs.pop("guidance_scale", 7.5)
    image_guidance_scale = kwargs.pop("image_guidance_scale", 1.5)
    steps = int(kwargs.pop("num_inference_steps", 15))
    generator = kwargs.get("generator")
    path = download_video(kwargs.pop("video_uri"))
    try:
        frames, fps = read_video_frames(path, max_frames=100, max_fps=30, height=512)
    finally:
        os.unlink(path)
    pipe = load_sd(model_name, device_identifier)
    out_frames = []
    nsfw = False
    batch = int(os.environ.get("SDAAS_VID2VID_BATCH", "8"))
    for i in range(0, len(frames), batch):
        chunk = [_fit(f, 512, 512) for f in frames[i:i + batch]]
        r = pipe(prompt=[prompt] * len(chunk), negative_prompt=[negative_prompt] * len(chunk), image=chunk,
                 num_inference_steps=steps, guidance_scale=guidance_scale,
                 image_guidance_scale=image_guidance_scale, generator=generator,
                 height=chunk[0].height, width=chunk[0].width,
                 scheduler=get_scheduler("EulerAncestralDiscreteScheduler", **pipe.family.scheduler_kwargs()))
        out_frames.extend(np.asarray(im.convert("RGB")) for im in r.images)
        nsfw = nsfw or any(r.nsfw_content_detected)
    video, ct = frames_to_video(np.stack(out_frames), max(1, int(round(fps))), "video/mp4")
    from PIL import Image

    thumb = image_to_buffer(Image.fromarray(out_frames[0]), "image/jpeg")
    config = {"nsfw": nsfw, "cost": 512 * 512 * steps * len(out_frames)}
    return {"primary": make_result(io.BytesIO(video), thumb, ct)}, config


def _fit(im, w, h):
    from PIL import Image

    r = min(h / im.height, w / im.width)
    nw, nh = max(8, int(im.width * r) // 8 * 8), max(8, int(im.height * r) // 8 * 8)
    return im.resize((nw, nh), Image.Resampling.LANCZOS)
