"""Stable-Diffusion-family job callback (reference:
swarm/diffusion/diffusion_func.py:14-124).

Same contract: ``diffusion_callback(device_identifier, model_name, **kwargs) ->
(artifacts, pipeline_config)``; kwargs not consumed here are forwarded to the
pipeline call (the hive drives guidance_scale, negative_prompt, strength,
num_images_per_prompt, height, width, ...).  Differences by design: models
come from the resident cache (no per-job reload), no CPU offload / xformers /
VAE slicing heuristics (288 GB HBM), and the optional x2 latent upscale is
applied to every image (the reference returned only images[0],
swarm/diffusion/upscale.py:28-32).
"""
from __future__ import annotations

import os
import time

import torch

from ..jobs.router import GUIDED_PIPELINES
from ..output.processor import OutputProcessor
from ..runtime.model_cache import cache, find_weights
from ..runtime.provision import ensure_weights
from ..schedulers import get_scheduler
from .sd import StableDiffusion, resolve_family
from ..utils import stable_seed

# accepted and ignored: memory / progress / return-format knobs of the diffusers
# call that have no meaning here (the reference's own xformers flag included)
_DROP = ("supports_xformers", "cross_attention_kwargs", "callback", "callback_steps", "output_type",
         "return_dict")

# the diffusers classes the SD-family callback runs as StableDiffusion
SD_CLASSES = {
    "DiffusionPipeline", "StableDiffusionPipeline", "StableDiffusionImg2ImgPipeline",
    "StableDiffusionInpaintPipeline", "StableDiffusionInpaintPipelineLegacy", "StableDiffusionControlNetPipeline",
    "StableDiffusionControlNetImg2ImgPipeline", "StableDiffusionInstructPix2PixPipeline",
    "StableDiffusionXLPipeline", "StableDiffusionXLImg2ImgPipeline", "StableDiffusionXLInpaintPipeline",
    "StableDiffusionDepth2ImgPipeline", "StableDiffusionImageVariationPipeline", "StableUnCLIPImg2ImgPipeline",
    # sampling-loop variants on a plain SD checkpoint (pipelines/guided.py)
    "StableDiffusionPanoramaPipeline", "StableDiffusionSAGPipeline", "StableDiffusionPipelineSafe",
    "SemanticStableDiffusionPipeline", "StableDiffusionModelEditingPipeline", "StableDiffusionAttendAndExcitePipeline",
    # SD1.x UNet + XLM-RoBERTa text encoder (models/xlmr.py)
    "AltDiffusionPipeline", "AltDiffusionImg2ImgPipeline",
}
# checkpoints whose own class must win over a generic requested one (the
# router defaults an image job to StableDiffusionImg2ImgPipeline; these
# architectures cannot run as that class)
_OWN_CLASS = {"StableDiffusionDepth2ImgPipeline", "StableDiffusionImageVariationPipeline", "StableUnCLIPImg2ImgPipeline"}
GUIDED_CLASSES = GUIDED_PIPELINES  # (guided.CLASSES)
UPSCALE_CLASSES = {"StableDiffusionUpscalePipeline", "StableDiffusionLatentUpscalePipeline"}
# job kwargs the SD callback consumes itself (the rest go to the pipeline call)
_CALLBACK_KEYS = {"model_name", "scheduler_type", "pipeline_type", "upscale", "textual_inversion", "lora",
                  "cross_attention_scale", "revision", "variant", "outputs", "content_type", "controlnet_model_name",
                  "controlnet_revision", "save_preprocessed_input", "_image_range", "_return_images", "_split"}


def checkpoint_class(model_name: str, revision: str = "main") -> str | None:
    """The pipeline class a generic ``DiffusionPipeline`` load would build
    (diffusers reads model_index.json's ``_class_name``); name heuristics for
    the two upscalers when no local checkpoint is present."""
    import json

    w = find_weights(model_name, revision)
    if w and os.path.exists(os.path.join(w, "model_index.json")):
        with open(os.path.join(w, "model_index.json")) as f:
            return json.load(f).get("_class_name")
    n = model_name.lower()
    if "image-variations" in n or (n.startswith("tiny/") and "variation" in n):
        return "StableDiffusionImageVariationPipeline"
    if "unclip" in n:
        return "StableUnCLIPImg2ImgPipeline"
    if "stable-diffusion-2-depth" in n or (n.startswith("tiny/") and "depth" in n):
        return "StableDiffusionDepth2ImgPipeline"
    if "x4-upscaler" in n:
        return "StableDiffusionUpscalePipeline"
    if "latent-upscaler" in n:
        return "StableDiffusionLatentUpscalePipeline"
    return None


def pipeline_class_for(pipeline_type: str, model_name: str, revision: str = "main") -> str:
    """The class this job runs as: the hive-named class, or — for the generic
    ``DiffusionPipeline`` — the checkpoint's own (reference:
    swarm/diffusion/diffusion_func.py:41-46 builds ``pipeline_type.from_pretrained``).
    A class with no implementation here is a fatal ``ValueError`` naming it."""
    cls = str(pipeline_type or "DiffusionPipeline")
    if cls == "DiffusionPipeline":
        ck = checkpoint_class(model_name, revision)
        if ck in UPSCALE_CLASSES or (ck is not None and ck not in SD_CLASSES) or ck in _OWN_CLASS:
            cls = ck
    elif cls in ("StableDiffusionPipeline", "StableDiffusionImg2ImgPipeline", "AltDiffusionPipeline",
                 "AltDiffusionImg2ImgPipeline"):
        ck = checkpoint_class(model_name, revision)
        if ck in _OWN_CLASS:
            cls = ck
    if cls in SD_CLASSES or cls in UPSCALE_CLASSES:
        return cls
    raise ValueError(f"pipeline class {cls} is not implemented by the Stable Diffusion callback of this worker")


def safety_checker_dir(weights_dir: str | None) -> str | None:
    """Weights of the NSFW checker this pipeline runs (the reference runs the
    pipeline's own ``safety_checker`` component and aggregates
    ``nsfw_content_detected``, swarm/diffusion/diffusion_func.py:98-111):
    the checkpoint's own ``safety_checker/`` when its model_index.json lists
    one (SD1.x layouts), else a separately provisioned
    CompVis/stable-diffusion-safety-checker; None when neither exists (a
    random tower would be meaningless)."""
    import json

    from ..runtime.provision import has_weights

    if weights_dir and os.path.exists(os.path.join(weights_dir, "model_index.json")):
        with open(os.path.join(weights_dir, "model_index.json")) as f:
            entry = json.load(f).get("safety_checker")
        own = os.path.join(weights_dir, "safety_checker")
        if isinstance(entry, (list, tuple)) and entry and entry[0] and has_weights(own):
            return own
    sw = find_weights("CompVis/stable-diffusion-safety-checker")
    return sw if has_weights(sw) else None


def load_sd(model_name: str, device_identifier: str, revision: str = "main", controlnet_name: str | None = None,
            controlnet_revision: str = "main") -> StableDiffusion:
    def make():
        # fetched on a miss like from_pretrained; no weights -> WeightsMissing
        # (non-fatal job error), random-init only under SDAAS_ALLOW_RANDOM=1
        w = ensure_weights(model_name, revision)
        # architecture from the checkpoint's own model_index.json / config.json
        # files (the reference's from_pretrained); name presets only without them
        fam = resolve_family(model_name, w)
        if fam.is_image_variation:
            from .variants import ImageVariation

            return ImageVariation(fam, device=device_identifier, weights_dir=w, seed=stable_seed(model_name))
        if fam.is_unclip:
            from .variants import UnCLIPImg2Img

            return UnCLIPImg2Img(fam, device=device_identifier, weights_dir=w, seed=stable_seed(model_name))
        return StableDiffusion(fam, device=device_identifier, weights_dir=w, seed=stable_seed(model_name))

    pipe = cache().get(("sd", model_name, revision, device_identifier), make)
    if not hasattr(pipe, "_safety_probed"):
        pipe._safety_probed = True
        sw = safety_checker_dir(find_weights(model_name, revision))
        if sw and os.environ.get("SDAAS_SAFETY", "1") != "0":
            from ..models.safety import load_safety_checker

            pipe.safety_checker = load_safety_checker(device_identifier, sw)
    pipe.controlnet = None
    if controlnet_name:
        from .controlnet import load_controlnet

        pipe.controlnet = load_controlnet(controlnet_name, pipe, device_identifier, controlnet_revision)
    return pipe


def _apply_lora(pipe, lora, scale):
    from ..models.lora import load_lora

    try:
        load_lora(pipe.unet, lora, scale, pipe=pipe)
    except Exception as e:
        raise ValueError(f"Could not load lora \n{lora}\nIt might be incompatible with {pipe.family.name}\n{e}") from e


def _apply_textual_inversion(pipe, ti, model_name):
    from ..models.lora import load_textual_inversion

    try:
        load_textual_inversion(pipe, ti)
    except Exception as e:
        raise ValueError(f"Textual inversion\n{ti}\nis incompatible with\n{model_name}\n\n{e}") from e


def diffusion_callback(device_identifier, model_name, **kwargs):
    # {"role": "leader", "peers": [rank, ...]} | {"role": "helper", "leader": r} (image split) |
    # {"role": "cfg", "peer": r, "half": 0 | 1} (CFG-parallel: half 1 returns only an ack)
    split = kwargs.pop("_split", None)
    state = {"transferred": False}
    try:
        return _diffusion(device_identifier, model_name, split, state, **kwargs)
    except BaseException:
        # ANY failure of a split part (load, adapters, scheduler, arguments, the
        # pipeline) before its transfer started: release the peers blocked on it
        if not state["transferred"] and not state.get("cfg", {}).get("started"):
            _split_failed(split)
        raise


def _diffusion(device_identifier, model_name, split, state, **kwargs):
    t0 = time.perf_counter()
    scheduler_type = kwargs.pop("scheduler_type", "DPMSolverMultistepScheduler")
    pipeline_type = kwargs.pop("pipeline_type", "DiffusionPipeline")
    upscale = kwargs.pop("upscale", False)
    textual_inversion = kwargs.pop("textual_inversion", None)
    lora = kwargs.pop("lora", None)
    cross_attention_scale = kwargs.pop("cross_attention_scale", 1.0)
    revision = kwargs.pop("revision", "main")
    kwargs.pop("variant", None)
    for k in _DROP:
        kwargs.pop(k, None)
    output_processor = OutputProcessor(kwargs.pop("outputs", ["primary"]), kwargs.pop("content_type", "image/jpeg"))

    controlnet_name = kwargs.pop("controlnet_model_name", None)
    controlnet_revision = kwargs.pop("controlnet_revision", "main")
    if kwargs.pop("save_preprocessed_input", False) and kwargs.get("image") is not None:
        output_processor.add_other_outputs("preprocessed_input", [kwargs.get("image")])

    # Multi-image txt2img: image j is seeded with (job seed + j) — its own
    # generator for the initial noise AND every sampler-noise draw — so a job
    # gives the same images whether it runs on one GPU or is split across
    # several (runtime.worker: ``_image_range`` sub-jobs).  The reference drew
    # all images from one generator stream (swarm/gpu/device.py:35-41).
    image_range = kwargs.pop("_image_range", None)
    return_images = bool(kwargs.pop("_return_images", False))
    ensure_weights(model_name, revision)  # provisioned before the class is read from its model_index.json
    pcls = pipeline_class_for(pipeline_type, model_name, revision)
    if pcls in UPSCALE_CLASSES:
        if split is not None or image_range is not None:
            raise ValueError(f"{pcls} jobs are not split across GPUs")
        return _upscale_job(pcls, device_identifier, model_name, scheduler_type, output_processor, **kwargs)
    gen = kwargs.get("generator")
    n_img = int(kwargs.get("num_images_per_prompt", 1) or 1)
    if (isinstance(gen, torch.Generator) and kwargs.get("image") is None
            and (n_img > 1 or image_range is not None)):
        lo = int(image_range[0]) if image_range is not None else 0
        hi = int(image_range[1]) if image_range is not None else n_img
        base = gen.initial_seed()
        kwargs["num_images_per_prompt"] = hi - lo
        kwargs["generator"] = [(torch.Generator(device=gen.device).manual_seed((base + j) % (1 << 63)), 1)
                               for j in range(lo, hi)]

    pipe = load_sd(model_name, device_identifier, revision, controlnet_name, controlnet_revision)
    if textual_inversion is not None:
        _apply_textual_inversion(pipe, textual_inversion, model_name)
    try:
        if lora is not None:
            _apply_lora(pipe, lora, cross_attention_scale)
        # the named sampler built from the checkpoint's scheduler config (diffusers from_config)
        sched = get_scheduler(scheduler_type, **pipe.family.scheduler_kwargs())
        load_s = time.perf_counter() - t0
        helper = split is not None and split.get("role") == "helper"
        cfg_part = split is not None and split.get("role") == "cfg"
        if cfg_part:
            if kwargs.get("image") is not None or int(kwargs.get("num_images_per_prompt", 1) or 1) != 1:
                raise ValueError("CFG-parallel parts are one-image txt2img jobs")
            # the pipeline marks "started" after its handshake: a failure after that
            # must not send a second handshake into the peer's prediction exchange
            kwargs["cfg_split"] = state["cfg"] = {"peer": int(split["peer"]), "half": int(split["half"])}
        out_type = "uint8_device" if helper else ("latent" if cfg_part and int(split["half"]) == 1 else "pil")
        t_pipe = time.perf_counter()
        if pcls in GUIDED_CLASSES:
            if split is not None:
                raise ValueError(f"{pcls} jobs are not split across GPUs")
            from . import guided

            p = guided.run(pcls, pipe, scheduler=sched, **dict(kwargs, output_type=out_type))
        else:
            p = pipe(scheduler=sched, **dict(kwargs, output_type=out_type))
        t_post = time.perf_counter()
    finally:
        from ..models.lora import unload_lora, unload_textual_inversion

        if lora is not None:
            unload_lora(pipe.unet, pipe=pipe)
        if textual_inversion is not None:
            unload_textual_inversion(pipe)

    config = dict(pipe.config)
    config["scheduler"] = ["chiaswarm_amd", sched.name]
    config["_pipeline_type"] = pcls
    if any(bool(x) for x in (p.nsfw_content_detected or [])):
        config["nsfw"] = True

    images = p.images
    if cfg_part and int(split["half"]) == 1:  # the peer (half 0) decodes and answers the job
        return {}, {"_split_ack": 1}
    if cfg_part:
        config["cfg_parallel"] = 2
    if helper:  # a split part: uint8 images straight to the leader's GPU over the process group
        from ..parallel import comm

        state["transferred"] = True  # a failure from here on must not send a second header
        comm.send_images(images, int(split["leader"]), any(bool(x) for x in (p.nsfw_content_detected or [])))
        return {}, {"_split_ack": int(images.shape[0])}
    if split is not None and split.get("role") == "leader":
        state["transferred"] = True  # _gather_split_images drains every helper itself
        images, nsfw_peers = _gather_split_images(images, split)
        if nsfw_peers:
            config["nsfw"] = True
        config["split"] = 1 + len(split.get("peers", []))
    if return_images:  # a split sub-job: the supervisor assembles and encodes the whole job
        import numpy as np

        config["_images"] = [np.asarray(im) for im in images]
        return {}, config
    if upscale:
        from .upscale import upscale_images

        g = kwargs.get("generator")
        images = upscale_images(images, device_identifier, kwargs.get("prompt", ""),
                                g[0][0] if isinstance(g, list) else g)
    output_processor.add_outputs(images)
    results = output_processor.get_results()
    if os.environ.get("SDAAS_TIMINGS"):
        t = dict(p.timings or {})
        t["load"] = load_s
        t["setup"] = t_pipe - t0 - load_s  # scheduler / split arguments
        t["pipe_other"] = t_post - t_pipe - sum(v for k, v in (p.timings or {}).items())
        t["envelope"] = time.perf_counter() - t_post  # images -> encoder pool submission
        config["timings"] = {k: round(v, 4) for k, v in t.items()}
    return results, config


_X4_ARGS = {"prompt", "negative_prompt", "num_inference_steps", "guidance_scale", "noise_level",
            "num_images_per_prompt", "generator", "image", "eta"}
_X2_ARGS = {"prompt", "negative_prompt", "num_inference_steps", "guidance_scale", "num_images_per_prompt",
            "generator", "image"}


def _upscale_job(pcls, device_identifier, model_name, scheduler_type, output_processor, **kwargs):
    """The diffusers upscale pipelines as hive jobs: ``StableDiffusionUpscalePipeline``
    (x4: low-res RGB concatenated to the latents, ``noise_level`` class
    conditioning; diffusers defaults 75 steps / guidance 9 / noise_level 20)
    and ``StableDiffusionLatentUpscalePipeline`` (x2 K-UNet, Euler).  The
    start image is required; unknown call kwargs raise ``TypeError`` like the
    diffusers call would."""
    from .upscale import load_latent_upscaler, load_x4_upscaler

    allowed = _X4_ARGS if pcls == "StableDiffusionUpscalePipeline" else _X2_ARGS
    bad = sorted(k for k in kwargs if k not in allowed)
    if bad:
        raise TypeError(f"{pcls}.__call__() got unexpected keyword arguments {bad}")
    image = kwargs.get("image")
    if image is None:
        raise ValueError(f"{pcls} needs an input image (start_image_uri)")
    n = max(1, int(kwargs.get("num_images_per_prompt", 1) or 1))
    images = [image] * n
    prompt = [kwargs.get("prompt", "")] * n
    neg = kwargs.get("negative_prompt")
    neg = [neg or ""] * n if not isinstance(neg, list) else neg
    g = kwargs.get("generator")
    t0 = time.perf_counter()
    if pcls == "StableDiffusionUpscalePipeline":
        up = load_x4_upscaler(device_identifier, model_name)
        sched = get_scheduler(scheduler_type, **up.scheduler_kwargs())
        if kwargs.get("eta") and sched.accepts_eta:
            sched.eta = float(kwargs["eta"])
        out = up(prompt, images, num_inference_steps=int(kwargs.get("num_inference_steps", 75)),
                 guidance_scale=float(kwargs.get("guidance_scale", 9.0)),
                 noise_level=int(kwargs.get("noise_level", 20)), negative_prompt=neg, generator=g, scheduler=sched)
        sched_name = sched.name
    else:
        up = load_latent_upscaler(device_identifier, model_name)
        out = up(prompt, images, num_inference_steps=int(kwargs.get("num_inference_steps", 75)),
                 guidance_scale=float(kwargs.get("guidance_scale", 9.0)), generator=g, negative_prompt=neg)
        sched_name = "EulerDiscreteScheduler"
    output_processor.add_outputs(out)
    config = {"model_name": model_name, "_pipeline_type": pcls, "scheduler": ["chiaswarm_amd", sched_name],
              "weights": getattr(up, "weights_source", "random-init")}
    if os.environ.get("SDAAS_TIMINGS"):
        config["timings"] = {"total": round(time.perf_counter() - t0, 4)}
    return output_processor.get_results(), config


def _split_failed(split):
    """A split part failed before its transfer: keep the peers from waiting on it
    (a helper sends an error header; the leader drains what its helpers send)."""
    if split is None:
        return
    from ..parallel import comm

    try:
        if split.get("role") == "cfg":
            comm.cfg_handshake(int(split["peer"]), ok=False)
        elif split.get("role") == "helper":
            comm.send_images(None, int(split["leader"]))
        else:
            for r in split.get("peers", []):
                comm.recv_images(int(r))
    except Exception:  # the group itself is gone: the supervisor restarts the parts
        pass


def _gather_split_images(images, split):
    """Leader: its own PIL images + every helper's uint8 images, in image order
    (helpers hold the later image ranges, in ``peers`` order)."""
    from PIL import Image

    from ..parallel import comm

    out, nsfw, failed = list(images), False, []
    for r in split.get("peers", []):
        got, flag = comm.recv_images(int(r))
        if got is None:
            failed.append(r)
            continue
        nsfw = nsfw or flag
        out.extend(Image.fromarray(a) for a in got.cpu().numpy())
    if failed:
        raise RuntimeError(f"split job: the parts on ranks {failed} failed")
    return out, nsfw


def diffusion_batch(device_identifier, jobs: list[dict]) -> list[tuple[dict, dict]]:
    """Several compatible txt2img jobs (``runtime.batcher``) as ONE denoising
    batch.  ``jobs``: routed kwargs, each with its own ``generator``.  Each
    job's initial noise comes from its own generator, so deterministic samplers
    reproduce the job's solo images exactly.  Returns (artifacts, config) per job."""
    import torch

    import inspect

    # the solo path forwards every kwarg it does not consume to the pipeline
    # call, which raises TypeError on unknown ones: same check here, per job,
    # before any GPU work (the batcher then runs the jobs one by one and each
    # gets its own error envelope)
    call_keys = set(inspect.signature(StableDiffusion.__call__).parameters) - {"self", "unexpected"}
    for kw in jobs:
        bad = sorted(k for k in kw if k not in call_keys and k not in _CALLBACK_KEYS and k not in _DROP)
        if bad:
            raise TypeError(f"batched job: unexpected keyword arguments {bad}")
    k0 = jobs[0]
    model_name = k0["model_name"]
    for kw in jobs:  # (runtime.worker._raw_key never batches these: their loop is not the plain one)
        if pipeline_class_for(kw.get("pipeline_type", "DiffusionPipeline"), model_name) in GUIDED_CLASSES:
            raise ValueError("Panorama / SAG / safe-latent-diffusion jobs run alone, not in a denoising batch")
    pipe = load_sd(model_name, device_identifier, k0.get("revision", "main"))
    sched_type = k0.get("scheduler_type", "DPMSolverMultistepScheduler")
    sched = get_scheduler(sched_type, **pipe.family.scheduler_kwargs())
    steps = int(k0.get("num_inference_steps", 30))
    sched.set_timesteps(steps)
    height = int(k0.get("height") or pipe.family.default_size) // 8 * 8
    width = int(k0.get("width") or pipe.family.default_size) // 8 * 8
    prompts, negs, lat, counts, gens = [], [], [], [], []
    for kw in jobs:
        n = max(1, int(kw.get("num_images_per_prompt", 1) or 1))
        counts.append(n)
        prompts += [kw.get("prompt", "")] * n
        negs += [kw.get("negative_prompt")] * n  # None: SDXL zero negative embeddings, else ""
        g = kw["generator"]
        # same per-image seeding as diffusion_callback (image j of a job: seed + j)
        jg = [(g, n)] if n == 1 else [(torch.Generator(device=g.device).manual_seed((g.initial_seed() + j) % (1 << 63)), 1)
                                      for j in range(n)]
        gens += jg
        for gj, nj in jg:
            noise = torch.randn((nj, 4, height // 8, width // 8), generator=gj, device=pipe.device,
                                dtype=torch.float32)
            lat.append(noise.permute(0, 2, 3, 1) * sched.init_noise_sigma)
    p = pipe(prompt=prompts, negative_prompt=negs, num_inference_steps=steps,
             guidance_scale=float(k0.get("guidance_scale", 7.5)), height=height, width=width,
             latents=torch.cat(lat, 0).contiguous(), scheduler=sched,
             eta=float(k0.get("eta") or 0.0),  # batch key: every job of the batch has this eta
             generator=gens)  # per-job / per-image sampler noise
    outs, i = [], 0
    for kw, n in zip(jobs, counts):
        op = OutputProcessor(kw.get("outputs", ["primary"]), kw.get("content_type", "image/jpeg"))
        op.add_outputs(p.images[i:i + n])
        cfg = dict(pipe.config)
        cfg["scheduler"] = ["chiaswarm_amd", sched.name]
        cfg["_pipeline_type"] = pipeline_class_for(kw.get("pipeline_type", "DiffusionPipeline"), model_name)
        if any(bool(x) for x in (p.nsfw_content_detected or [])[i:i + n]):
            cfg["nsfw"] = True
        if os.environ.get("SDAAS_TIMINGS"):
            cfg["timings"] = {k: round(v, 4) for k, v in (p.timings or {}).items()}
        outs.append((op.get_results(), cfg))
        i += n
    return outs
