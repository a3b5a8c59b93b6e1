"""Routing table / job normalisation (reference swarm/job_arguments.py)."""
import pytest

from chiaswarm_amd.jobs import router
from tests.fakehive import FakeHive


@pytest.fixture(scope="module")
def hive():
    h = FakeHive().start()
    yield h
    h.stop()


def name(cb):
    return cb.__name__


@pytest.mark.parametrize("job,cb", [
    ({"model_name": "suno/bark", "workflow": "txt2audio"}, "bark_diffusion_callback"),
    ({"model_name": "cvssp/audioldm", "workflow": "txt2audio"}, "txt2audio_diffusion_callback"),
    ({"model_name": "x", "workflow": "stitch", "jobs": []}, "stitch_callback"),
    ({"model_name": "Salesforce/blip", "workflow": "img2txt"}, "caption_callback"),
    ({"model_name": "timbrooks/instruct-pix2pix", "workflow": "vid2vid"}, "model_video_callback"),
    ({"model_name": "damo/t2v", "workflow": "txt2vid"}, "txt2vid_diffusion_callback"),
    ({"model_name": "DeepFloyd/IF-I-XL-v1.0", "workflow": "txt2img"}, "diffusion_if_callback"),
    ({"model_name": "stabilityai/stable-diffusion-2-1"}, "diffusion_callback"),
])
def test_routing(job, cb):
    f, args = router.format_args(job)
    assert name(f) == cb
    assert "workflow" not in args


def test_sd_defaults():
    f, args = router.format_args({"model_name": "runwayml/stable-diffusion-v1-5"})
    assert args["prompt"] == "" and args["num_inference_steps"] == 30
    assert args["pipeline_type"] == "DiffusionPipeline"
    assert args["scheduler_type"] == "DPMSolverMultistepScheduler"
    assert args["supports_xformers"] is True and args["upscale"] is False


def test_audio_video_defaults():
    _, a = router.format_args({"model_name": "cvssp/audioldm", "workflow": "txt2audio"})
    assert a["num_inference_steps"] == 25 and a["pipeline_type"] == "AudioLDMPipeline"
    _, v = router.format_args({"model_name": "m", "workflow": "txt2vid", "num_images_per_prompt": 4})
    assert v["num_inference_steps"] == 25 and "num_images_per_prompt" not in v


def test_size_limit_is_error():
    with pytest.raises(Exception, match="max image size"):
        router.format_args({"model_name": "m", "height": 2048, "width": 512})


def test_unknown_scheduler_is_error():
    with pytest.raises(AttributeError):
        router.format_args({"model_name": "m", "parameters": {"scheduler_type": "NopeScheduler"}})


def test_unsupported_arguments_stripped():
    _, a = router.format_args({"model_name": "m", "negative_prompt": "x", "eta": 0.1,
                               "parameters": {"unsupported_pipeline_arguments": ["negative_prompt", "eta"]}})
    assert "negative_prompt" not in a and "eta" not in a


def test_img2img_and_pix2pix_and_mask(hive):
    uri = hive.add_image("in.png", size=(1500, 700))
    _, a = router.format_args({"model_name": "m", "start_image_uri": uri, "height": 512, "width": 512})
    assert a["pipeline_type"] == "StableDiffusionImg2ImgPipeline"
    assert "height" not in a and a["image"].width <= 512 and a["image"].height <= 512
    _, p = router.format_args({"model_name": "timbrooks/instruct-pix2pix", "start_image_uri": uri, "strength": 0.5})
    assert p["image_guidance_scale"] == pytest.approx(2.5) and "strength" not in p
    m = hive.add_image("mask.png", size=(64, 64), color=(255, 255, 255))
    _, q = router.format_args({"model_name": "m", "start_image_uri": uri, "mask_image_uri": m})
    assert q["mask_image"].size == (64, 64)


def test_thumbnail_uses_width_height_order(hive):
    uri = hive.add_image("wide.png", size=(1000, 400))
    _, a = router.format_args({"model_name": "m", "start_image_uri": uri, "height": 300, "width": 800})
    # bounding box is 800 wide x 300 high -> 750x300 (the reference's transposed call gave 300x120)
    assert a["image"].size == (750, 300)


def test_non_image_and_oversize_inputs(hive):
    t = hive.add_file("x.txt", b"hello", "text/plain")
    with pytest.raises(Exception, match="does not appear to be an image"):
        router.format_args({"model_name": "m", "start_image_uri": t})
    big = hive.add_file("big.png", b"0" * (3 * 1048576 + 10), "image/png")
    with pytest.raises(Exception, match="too large"):
        router.format_args({"model_name": "m", "start_image_uri": big})


def test_controlnet_routing(hive):
    uri = hive.add_image("cn.png", size=(128, 128))
    _, a = router.format_args({"model_name": "runwayml/stable-diffusion-v1-5", "start_image_uri": uri,
                               "parameters": {"controlnet": {"type": "canny", "preprocess": True}}})
    assert a["pipeline_type"] == "StableDiffusionControlNetPipeline"
    assert a["controlnet_model_name"] == "lllyasviel/control_v11p_sd15_canny"
    assert a["save_preprocessed_input"] is True
