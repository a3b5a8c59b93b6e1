"""Pipeline-class dispatch of the SD-family callback (reference:
swarm/diffusion/diffusion_func.py:41-46 builds ``pipeline_type.from_pretrained``,
:96 forwards every remaining job key into the call; swarm/job_arguments.py:143-145):

* StableDiffusionUpscalePipeline -> the x4 upscaler (low-res concat + noise_level),
  also when a generic ``DiffusionPipeline`` names an x4 checkpoint;
* StableDiffusionLatentUpscalePipeline -> the x2 latent upscaler;
* classes with no implementation are fatal errors naming the class;
* unknown call kwargs raise TypeError like the diffusers call;
* a split part that fails anywhere before its transfer releases its peers."""
import base64
import io

import numpy as np
import pytest
import torch
from PIL import Image

from chiaswarm_amd.jobs import router
from chiaswarm_amd.pipelines import diffusion


def _img(n=16, seed=0):
    return Image.fromarray((np.random.default_rng(seed).random((n, n, 3)) * 255).astype(np.uint8))


def _size(res):
    return Image.open(io.BytesIO(base64.b64decode(res["primary"]["blob"]))).size


@pytest.mark.parametrize("cls", ["KandinskyPipeline", "UnCLIPPipeline", "VersatileDiffusionPipeline",
                                 "StableDiffusionPix2PixZeroPipeline", "PaintByExamplePipeline"])
def test_unimplemented_classes_are_fatal(cls):
    with pytest.raises(ValueError, match=cls):
        router.format_args({"model_name": "m", "parameters": {"pipeline_type": cls}})


def test_model_editing_class_runs_as_plain_sd():
    """StableDiffusionModelEditingPipeline.__call__ is StableDiffusionPipeline's
    (the edits go through edit_model(), which a job cannot call): same image."""
    kw = dict(prompt="a", num_inference_steps=2, scheduler_type="DDIMScheduler", upscale=False, supports_xformers=True)
    a, _ = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type="StableDiffusionPipeline",
                                        generator=torch.Generator().manual_seed(0), **kw)
    b, cfg = diffusion.diffusion_callback("cpu", "tiny/sd", pipeline_type="StableDiffusionModelEditingPipeline",
                                          generator=torch.Generator().manual_seed(0), **kw)
    assert a["primary"]["blob"] == b["primary"]["blob"]


def test_class_resolution():
    assert diffusion.pipeline_class_for("DiffusionPipeline", "stabilityai/stable-diffusion-x4-upscaler") == \
        "StableDiffusionUpscalePipeline"
    assert diffusion.pipeline_class_for("DiffusionPipeline", "stabilityai/sd-x2-latent-upscaler") == \
        "StableDiffusionLatentUpscalePipeline"
    assert diffusion.pipeline_class_for("DiffusionPipeline", "runwayml/stable-diffusion-v1-5") == "DiffusionPipeline"
    assert diffusion.pipeline_class_for("StableDiffusionImg2ImgPipeline", "m") == "StableDiffusionImg2ImgPipeline"
    for cls in ("IFPipeline", "AudioLDMPipeline", "TextToVideoSDPipeline"):
        with pytest.raises(ValueError, match=cls):
            diffusion.pipeline_class_for(cls, "m")


def test_x4_upscale_job():
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/x4-upscaler", pipeline_type="StableDiffusionUpscalePipeline",
                                            prompt="a", image=_img(16), num_inference_steps=2, noise_level=30,
                                            generator=g, scheduler_type="DDIMScheduler", upscale=False,
                                            supports_xformers=True)
    assert _size(res) == (64, 64)
    assert cfg["_pipeline_type"] == "StableDiffusionUpscalePipeline" and cfg["scheduler"][1] == "DDIMScheduler"
    # noise_level is the low-res image's noise AND the class conditioning: it changes the result
    g = torch.Generator().manual_seed(0)
    res2, _ = diffusion.diffusion_callback("cpu", "tiny/x4-upscaler", pipeline_type="StableDiffusionUpscalePipeline",
                                           prompt="a", image=_img(16), num_inference_steps=2, noise_level=250,
                                           generator=g, scheduler_type="DDIMScheduler")
    assert res2["primary"]["sha256_hash"] != res["primary"]["sha256_hash"]


def test_x4_upscale_job_errors():
    with pytest.raises(ValueError, match="input image"):
        diffusion.diffusion_callback("cpu", "tiny/x4-upscaler", pipeline_type="StableDiffusionUpscalePipeline",
                                     prompt="a", num_inference_steps=2)
    with pytest.raises(TypeError, match="strength"):
        diffusion.diffusion_callback("cpu", "tiny/x4-upscaler", pipeline_type="StableDiffusionUpscalePipeline",
                                     prompt="a", image=_img(16), num_inference_steps=2, strength=0.3)


def test_latent_upscale_job():
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/x2-latent-upscaler",
                                            pipeline_type="StableDiffusionLatentUpscalePipeline", prompt="a",
                                            image=_img(32), num_inference_steps=2, generator=g)
    assert _size(res) == (64, 64) and cfg["_pipeline_type"] == "StableDiffusionLatentUpscalePipeline"


def test_sd_unknown_kwarg_is_type_error():
    with pytest.raises(TypeError, match="bogus"):
        diffusion.diffusion_callback("cpu", "tiny/sd", prompt="a", num_inference_steps=1, height=64, width=64,
                                     generator=torch.Generator().manual_seed(0), bogus=1)


@pytest.mark.parametrize("role", ["leader", "helper"])
def test_split_part_failing_in_load_releases_peers(monkeypatch, role):
    calls = []

    def boom(*a, **k):
        raise RuntimeError("load failed")

    monkeypatch.setattr(diffusion, "load_sd", boom)
    monkeypatch.setattr(diffusion, "_split_failed", lambda split: calls.append(split))
    split = {"role": "leader", "peers": [1]} if role == "leader" else {"role": "helper", "leader": 0}
    with pytest.raises(RuntimeError, match="load failed"):
        diffusion.diffusion_callback("cpu", "tiny/sd", prompt="a", num_inference_steps=1, _split=split,
                                     _image_range=[0, 1], generator=torch.Generator().manual_seed(0))
    assert calls == [split]


def test_split_part_failing_in_arguments_releases_peers(monkeypatch):
    calls = []
    monkeypatch.setattr(diffusion, "_split_failed", lambda split: calls.append(split))
    split = {"role": "helper", "leader": 0}
    with pytest.raises(ValueError):
        diffusion.diffusion_callback("cpu", "tiny/sd", scheduler_type="NoSuchScheduler", _split=split,
                                     _image_range=[1, 2], generator=torch.Generator().manual_seed(0))
    assert calls == [split]
