"""Job normalisation and workflow routing: ``format_args(job) -> (callback, kwargs)``.

Routing table and per-workflow defaults follow the reference exactly
(swarm/job_arguments.py:17-153):

  txt2audio + suno/bark -> bark | txt2audio -> AudioLDM (25 steps) | stitch |
  img2txt -> caption | vid2vid | txt2vid (25 steps, no num_images) |
  DeepFloyd/* -> IF 3-stage | else -> Stable Diffusion family (30 steps).

``parameters.pipeline_type`` / ``scheduler_type`` arrive as diffusers class
*names*; the reference resolved them by reflection (swarm/type_helpers.py:1-3)
so an unknown name raised inside format_args -> fatal result.  We validate the
names against our own registries with the same outcome.  Callbacks are imported
lazily so the supervisor process never imports torch.
"""
from __future__ import annotations

from .inputs import MAX_SIZE, get_image

PIPELINE_TYPES = {
    "DiffusionPipeline", "StableDiffusionPipeline", "StableDiffusionImg2ImgPipeline",
    "StableDiffusionInpaintPipeline", "StableDiffusionInpaintPipelineLegacy", "StableDiffusionControlNetPipeline",
    "StableDiffusionControlNetImg2ImgPipeline", "StableDiffusionInstructPix2PixPipeline",
    "StableDiffusionXLPipeline", "StableDiffusionXLImg2ImgPipeline", "StableDiffusionXLInpaintPipeline",
    "StableDiffusionUpscalePipeline", "StableDiffusionLatentUpscalePipeline", "AudioLDMPipeline",
    "TextToVideoSDPipeline", "VideoToVideoSDPipeline", "IFPipeline", "IFSuperResolutionPipeline",
    "StableDiffusionDepth2ImgPipeline", "StableDiffusionImageVariationPipeline",
    "StableDiffusionPanoramaPipeline", "StableDiffusionSAGPipeline", "StableDiffusionPipelineSafe",
    "StableUnCLIPImg2ImgPipeline", "SemanticStableDiffusionPipeline",
    # its __call__ is StableDiffusionPipeline's (edits happen through edit_model(), which no job reaches)
    "StableDiffusionModelEditingPipeline", "StableDiffusionAttendAndExcitePipeline",
    "AltDiffusionPipeline", "AltDiffusionImg2ImgPipeline",
}
# SD classes with their own sampling loop (pipelines/guided.py): never batched
# with other jobs, never split across GPUs
GUIDED_PIPELINES = frozenset({"StableDiffusionPanoramaPipeline", "StableDiffusionSAGPipeline",
                              "StableDiffusionPipelineSafe", "SemanticStableDiffusionPipeline",
                              "StableDiffusionAttendAndExcitePipeline"})
# real diffusers classes with no implementation here: a fatal error naming the
# class (never silently run as plain SD)
UNIMPLEMENTED_PIPELINES = {"KandinskyPipeline", "KandinskyImg2ImgPipeline", "KandinskyInpaintPipeline",
                           "KandinskyV22Pipeline", "UnCLIPPipeline", "UnCLIPImageVariationPipeline",
                           # diffusers 0.16.1 classes needing an inversion / captioner loop, their own
                           # model families or packages the reference does not install
                           "StableDiffusionPix2PixZeroPipeline",
                           "StableDiffusionKDiffusionPipeline", "PaintByExamplePipeline", "StableUnCLIPPipeline",
                           "VersatileDiffusionPipeline", "VersatileDiffusionTextToImagePipeline",
                           "VersatileDiffusionImageVariationPipeline", "VersatileDiffusionDualGuidedPipeline",
                           "LDMTextToImagePipeline", "LDMSuperResolutionPipeline", "DiTPipeline",
                           "VQDiffusionPipeline", "RePaintPipeline", "DDPMPipeline", "DDIMPipeline",
                           "PNDMPipeline", "ScoreSdeVePipeline", "KarrasVePipeline", "DanceDiffusionPipeline",
                           "AudioDiffusionPipeline", "SpectrogramDiffusionPipeline", "LDMPipeline",
                           "StableDiffusionOnnxPipeline", "OnnxStableDiffusionPipeline"}


class PipelineType(str):
    """A validated diffusers pipeline class name."""


def get_pipeline_type(name: str) -> PipelineType:
    if name in UNIMPLEMENTED_PIPELINES:
        raise ValueError(f"pipeline class {name} is not implemented by this worker")
    if name not in PIPELINE_TYPES:
        raise AttributeError(f"module 'diffusers' has no attribute '{name}'")
    return PipelineType(name)


def get_scheduler_type(name: str) -> str:
    from ..schedulers import scheduler_names

    if name not in scheduler_names():
        raise AttributeError(f"module 'diffusers' has no attribute '{name}'")
    return name


def _cb(module: str, name: str):
    import importlib

    return getattr(importlib.import_module(f"chiaswarm_amd.pipelines.{module}"), name)


def format_args(job: dict):
    args = job.copy()
    workflow = args.pop("workflow", None)
    if workflow == "txt2audio":
        if args["model_name"] == "suno/bark":
            return _cb("audio", "bark_diffusion_callback"), args
        return format_txt2audio_args(args)
    if workflow == "stitch":
        return _cb("stitch", "stitch_callback"), args
    if workflow == "img2txt":
        return format_img2txt_args(args)
    if workflow == "vid2vid":
        return _cb("video", "model_video_callback"), args
    if workflow == "txt2vid":
        return format_txt2vid_args(args)
    if workflow == "upscale" or "esrgan" in args["model_name"].lower():
        # extension: Real-ESRGAN x4 (not in the reference; roadmap README.md:34)
        if "start_image_uri" in args:
            args["image"] = get_image(args.pop("start_image_uri"), None)
        args.pop("parameters", None)
        return _cb("esrgan", "esrgan_callback"), args
    if args["model_name"].startswith("DeepFloyd/"):
        return _cb("deepfloyd", "diffusion_if_callback"), args
    return format_stable_diffusion_args(args)


def format_txt2audio_args(args):
    parameters = dict(args.pop("parameters", None) or {})  # never mutate the caller's job
    args.setdefault("prompt", "")
    args.setdefault("num_inference_steps", 25)
    args["pipeline_type"] = get_pipeline_type(parameters.pop("pipeline_type", "AudioLDMPipeline"))
    args["scheduler_type"] = get_scheduler_type(parameters.pop("scheduler_type", "DPMSolverMultistepScheduler"))
    for arg in parameters.get("unsupported_pipeline_arguments", []):
        args.pop(arg, None)
    return _cb("audio", "txt2audio_diffusion_callback"), args


def format_txt2vid_args(args):
    parameters = dict(args.pop("parameters", None) or {})  # never mutate the caller's job
    args.setdefault("prompt", "")
    args.setdefault("num_inference_steps", 25)
    args.pop("num_images_per_prompt", None)
    args["pipeline_type"] = get_pipeline_type(parameters.pop("pipeline_type", "DiffusionPipeline"))
    args["scheduler_type"] = get_scheduler_type(parameters.pop("scheduler_type", "DPMSolverMultistepScheduler"))
    return _cb("video", "txt2vid_diffusion_callback"), args


def format_img2txt_args(args):
    if "start_image_uri" in args:
        args["image"] = get_image(args.pop("start_image_uri"), None)
    return _cb("caption", "caption_callback"), args


def format_stable_diffusion_args(args):
    size = None
    if "height" in args and "width" in args:
        size = (args["height"], args["width"])
        if size[0] > MAX_SIZE or size[1] > MAX_SIZE:
            raise Exception(f"The max image size is (1024, 1024); got ({size[0]}, {size[1]}).")

    parameters = dict(args.pop("parameters", None) or {})  # never mutate the caller's job
    args.setdefault("prompt", "")
    args["supports_xformers"] = parameters.get("supports_xformers", True)
    args["upscale"] = parameters.get("upscale", False)

    if "start_image_uri" in args:
        args.pop("height", None)
        args.pop("width", None)
        controlnet = parameters.get("controlnet", None)
        args["image"] = get_image(args.pop("start_image_uri"), size, controlnet)
        if controlnet is not None:
            parameters["pipeline_type"] = "StableDiffusionControlNetPipeline"
            args["controlnet_model_name"] = controlnet.get("controlnet_model_name",
                                                           "lllyasviel/control_v11p_sd15_canny")
            args["save_preprocessed_input"] = controlnet.get("preprocess", False)
        elif "pipeline_type" not in parameters:
            parameters["pipeline_type"] = "StableDiffusionImg2ImgPipeline"
        if args["model_name"] == "timbrooks/instruct-pix2pix":
            # pix2pix: strength (0-1) -> image_guidance_scale (0-5)
            args["image_guidance_scale"] = args.pop("strength", 0.6) * 5

    if "mask_image_uri" in args:
        args.pop("height", None)
        args.pop("width", None)
        args["mask_image"] = get_image(args.pop("mask_image_uri"), size)

    args.setdefault("num_inference_steps", 30)
    args["pipeline_type"] = get_pipeline_type(parameters.pop("pipeline_type", "DiffusionPipeline"))
    args["scheduler_type"] = get_scheduler_type(parameters.pop("scheduler_type", "DPMSolverMultistepScheduler"))
    for arg in parameters.get("unsupported_pipeline_arguments", []):
        args.pop(arg, None)
    return _cb("diffusion", "diffusion_callback"), args
