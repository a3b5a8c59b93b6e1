"""Text-to-audio workflows (reference: swarm/audio/audioldm.py:12-38 and
swarm/audio/bark.py:11-39).

* ``txt2audio_diffusion_callback`` — AudioLDM: CLAP text embedding -> latent
  diffusion over an 8-channel mel latent [B, T/4, 16, 8] (NHWC; T = 100 mel
  frames per second) -> mel VAE decode -> HiFi-GAN vocoder -> 16 kHz waveform.
  The UNet step is replayed from a hipGraph and the sampler update is the fused
  ``sched_step`` kernel, exactly like the SD path.
* ``bark_diffusion_callback`` — Bark: text -> semantic -> coarse -> fine codec
  tokens (three GPT stages with KV caches) -> EnCodec decoder -> 24 kHz
  waveform (``models.bark``).

Both return one ``primary`` artifact: MP3 when ffmpeg is present (the
reference's pydub export), otherwise 16-bit WAV with ``audio/wav`` content type.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .. import ops
from ..models.clap import CLAP_TEXT, HF_RENAMES, TINY_CLAP, ClapTextEncoder
from ..models.layers import init_random_fast_, prepare_model
from ..models.tokenizer import ByteBPETokenizer
from ..models.unet import AUDIOLDM, TINY_AUDIOLDM, UNet2DConditionModel
from ..models.vae import AUDIOLDM_VAE, TINY_AUDIO_VAE, AutoencoderKL
from ..models.vocoder import AUDIOLDM_HIFIGAN, TINY_HIFIGAN, HifiGan
from ..output.media import encode_audio
from ..output.processor import make_result
from ..runtime.model_cache import cache
from ..runtime.provision import ensure_weights
from ..schedulers import get_scheduler
from .graphs import GraphCache
from ..utils import stable_seed

# AudioLDM's training noise schedule (scheduler/scheduler_config.json of cvssp/audioldm*)
AUDIOLDM_SCHED = dict(beta_start=0.0015, beta_end=0.0195, beta_schedule="scaled_linear",
                      num_train_timesteps=1000, use_karras_sigmas=False)


class AudioLDM:
    def __init__(self, device="cpu", tiny=False, seed=0, weights_dir=None):
        self.device = torch.device(device)
        self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        tcfg, ucfg = (TINY_CLAP, TINY_AUDIOLDM) if tiny else (CLAP_TEXT, AUDIOLDM)
        vcfg, hcfg = (TINY_AUDIO_VAE, TINY_HIFIGAN) if tiny else (AUDIOLDM_VAE, AUDIOLDM_HIFIGAN)
        self.sched_config = dict(AUDIOLDM_SCHED)
        if weights_dir:
            # every size (cvssp/audioldm-s/-m/-l ...) from its own config files
            # (the reference: AudioLDMPipeline.from_pretrained, swarm/audio/audioldm.py:19-20)
            from ..models import hf_config as hc

            c = {s: hc.component_config(weights_dir, s) for s in ("text_encoder", "unet", "vae", "vocoder")}
            tcfg = hc.clap_text_config(c["text_encoder"]) if c["text_encoder"] else tcfg
            ucfg = hc.unet_config(c["unet"]) if c["unet"] else ucfg
            vcfg = hc.vae_config(c["vae"]) if c["vae"] else vcfg
            hcfg = hc.hifigan_config(c["vocoder"]) if c["vocoder"] else hcfg
            sk = hc.scheduler_kwargs(hc.component_config(weights_dir, "scheduler", "scheduler_config.json"))
            if sk:
                self.sched_config = dict(sk, use_karras_sigmas=False)
        with torch.device(self.device):
            self.text_encoder = ClapTextEncoder(tcfg).to(self.dtype)
            self.unet = UNet2DConditionModel(ucfg).to(self.dtype)
            self.vae = AutoencoderKL(vcfg, with_encoder=False).to(self.dtype)
            self.vocoder = HifiGan(hcfg).to(self.dtype)
        mods = [self.text_encoder, self.unet, self.vae, self.vocoder]
        for i, m in enumerate(mods):
            m.eval().requires_grad_(False)
            init_random_fast_(m, seed=seed + i)
        self.weights_source = "random-init"
        if weights_dir:
            if self._load(weights_dir):
                self.weights_source = str(weights_dir)
        for m in mods:
            prepare_model(m)
        self.tokenizer = ByteBPETokenizer(_sub(weights_dir, "tokenizer"), max_length=77,
                                          vocab_size=self.text_encoder.cfg.vocab)
        self._unet_graphs = GraphCache(self._unet_fn)
        self.config = {"_class_name": "AudioLDMPipeline", "_framework": "chiaswarm_amd",
                       "sampling_rate": self.vocoder.cfg.sampling_rate, "weights": self.weights_source}

    def _load(self, d) -> bool:
        from ..models.weights import _VAE_RENAMES, load_component

        from ..models.weights import CheckpointMismatch, tokenizer_dir

        subs = (("text_encoder", self.text_encoder, HF_RENAMES), ("unet", self.unet, None),
                ("vae", self.vae, _VAE_RENAMES), ("vocoder", self.vocoder, None))
        reps = {sub: load_component(mod, d, sub, ren) for sub, mod, ren in subs}
        got = [k for k, r in reps.items() if r is not None]
        if got and len(got) != len(subs):
            raise CheckpointMismatch(f"{d}: only {got} of text_encoder / unet / vae / vocoder have weights")
        if got and tokenizer_dir(d) is None:
            raise CheckpointMismatch(f"{d}: tokenizer files missing beside real text-encoder weights")
        return bool(got)

    # ------------------------------------------------------------------
    def _unet_fn(self, x, t, class_labels):
        return self.unet(x, t, class_labels=class_labels)

    @property
    def vae_scale(self) -> int:
        return 2 ** (len(self.vae.cfg.block_out_channels) - 1)

    @torch.no_grad()
    def __call__(self, prompt="", negative_prompt=None, num_inference_steps=10, guidance_scale=2.5,
                 audio_length_in_s=None, num_waveforms_per_prompt=1, generator=None, scheduler=None,
                 latents=None, **unused):
        t0 = time.perf_counter()
        voc = self.vocoder.cfg
        if audio_length_in_s is None:
            audio_length_in_s = self.unet.cfg.sample_size * self.vae_scale * voc.hop / voc.sampling_rate
        height = int(audio_length_in_s * voc.sampling_rate / voc.hop)  # mel frames
        original_len = int(audio_length_in_s * voc.sampling_rate)
        if height % self.vae_scale:
            height = int(np.ceil(height / self.vae_scale)) * self.vae_scale
        prompts = prompt if isinstance(prompt, list) else [prompt]
        prompts = [p for p in prompts for _ in range(num_waveforms_per_prompt)]
        b = len(prompts)
        cfg = guidance_scale > 1.0
        neg = negative_prompt if negative_prompt is not None else ""
        negs = (neg if isinstance(neg, list) else [neg]) * 1
        negs = [negs[i % len(negs)] for i in range(b)]
        emb = self.text_encoder(self.tokenizer((negs + prompts) if cfg else prompts)).to(self.dtype)

        sched = scheduler or get_scheduler("DPMSolverMultistepScheduler", **self.sched_config)
        sched.set_timesteps(num_inference_steps)
        lh, lw = height // self.vae_scale, voc.model_in_dim // self.vae_scale
        c = self.unet.cfg.in_channels
        if latents is None:
            noise = torch.randn((b, c, lh, lw), generator=generator, device=self.device, dtype=torch.float32)
            x = noise.permute(0, 2, 3, 1).contiguous() * sched.init_noise_sigma
        else:
            x = latents.to(self.device).float()
        t_dev = torch.zeros(1, device=self.device, dtype=torch.float32)
        if self.device.type == "cuda":  # phase timings are GPU-complete, not launch time
            torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        while sched.step_index < sched.n:
            xi = (x * sched.current_scale()).to(self.dtype)
            x_in = torch.cat([xi, xi], 0) if cfg else xi
            t_dev.fill_(float(sched.current_t()))
            e = self._unet_graphs(self.device, x=x_in, t=t_dev, class_labels=emb)
            coeffs = sched.fused_coeffs()
            if coeffs is not None and ops.use_hip(x):
                nz = (torch.randn(x.shape, generator=generator, device=x.device, dtype=torch.float32)
                      if coeffs.D != 0.0 else None)
                x = ops.sched_step(e, x, sched, coeffs, guidance_scale if cfg else None, nz)
            else:
                if cfg:
                    e_u, e_c = e.float().chunk(2)
                    e_g = e_u + guidance_scale * (e_c - e_u)
                else:
                    e_g = e.float()
                x = sched.step(e_g, x, generator)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        t2 = time.perf_counter()
        mel = self.vae.decode((x / self.vae.cfg.scaling_factor).to(self.dtype))  # [B, T, 64, 1]
        wav = self.vocoder(mel[..., 0])  # [B, T * hop]
        audio = wav[:, :original_len].cpu().numpy()
        self.timings = {"text_encode": t1 - t0, "denoise": t2 - t1, "decode_vocode": time.perf_counter() - t2}
        return audio


def _sub(d, name):
    import os

    if d and os.path.isdir(os.path.join(d, name)):
        return os.path.join(d, name)
    return None


def load_audioldm(model_name: str, device: str) -> AudioLDM:
    tiny = model_name.lower().startswith("tiny")
    return cache().get(("audioldm", model_name, device),
                       lambda: AudioLDM(device, tiny=tiny, weights_dir=ensure_weights(model_name),
                                        seed=stable_seed(model_name)))


def _scheduler_for(scheduler_type, pipe):
    if scheduler_type is None:
        return None
    return get_scheduler(scheduler_type, **pipe.sched_config)


def txt2audio_diffusion_callback(device_identifier, model_name, **kwargs):
    scheduler_type = kwargs.pop("scheduler_type", "DPMSolverMultistepScheduler")
    kwargs.pop("pipeline_type", None)
    kwargs["num_inference_steps"] = kwargs.pop("num_inference_steps", 20)
    kwargs["audio_length_in_s"] = kwargs.pop("audio_length_in_s", 10)
    content_type = kwargs.pop("content_type", "audio/mpeg")
    kwargs.pop("outputs", None)
    seed = kwargs.pop("seed", None)
    pipe = load_audioldm(model_name, device_identifier)
    gen = None
    if seed is not None:
        gen = torch.Generator(device=pipe.device).manual_seed(int(seed))
    audio = pipe(scheduler=_scheduler_for(scheduler_type, pipe), generator=kwargs.pop("generator", gen), **kwargs)
    data, ctype = encode_audio(audio[0], pipe.vocoder.cfg.sampling_rate, content_type)
    results = {"primary": make_result(data, None, ctype)}
    return results, dict(pipe.config)


def bark_diffusion_callback(device_identifier, model_name, **kwargs):
    from ..models.bark import load_bark

    content_type = kwargs.pop("content_type", "audio/mpeg")
    kwargs.pop("outputs", None)
    bark = load_bark(model_name, device_identifier)
    audio = bark.generate_audio(kwargs.get("prompt", ""), seed=kwargs.get("seed"))
    data, ctype = encode_audio(audio, bark.sample_rate, content_type)
    return {"primary": make_result(data, None, ctype)}, {}
