"""Reflection-reachable SD variants (reference:
swarm/job_arguments.py:143-145, swarm/type_helpers.py:1-3):
StableDiffusionDepth2ImgPipeline and StableDiffusionImageVariationPipeline.

CPU: the CLIP image encoder against transformers' CLIPVisionModelWithProjection
(state dict loaded through our loader unchanged), the depth map
normalisation, both pipelines end to end at test size through the real
callback / router, and the class resolution (a Depth2Img / ImageVariation
checkpoint wins over the router's Img2Img default; Kandinsky / UnCLIP stay
fatal).  diffusers itself is not importable here: pipeline-level parity is
unpinned.  GPU: both run on the HIP path."""
import base64
import io
import json
import os

import numpy as np
import pytest
import torch
from PIL import Image

from chiaswarm_amd.jobs import router
from chiaswarm_amd.pipelines import diffusion


def _img(n=64, seed=0):
    return Image.fromarray((np.random.default_rng(seed).random((n, n, 3)) * 255).astype(np.uint8))


def _size(res):
    return Image.open(io.BytesIO(base64.b64decode(res["primary"]["blob"]))).size


def test_image_encoder_matches_transformers(tmp_path):
    from safetensors.torch import save_file
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection

    from chiaswarm_amd.pipelines.variants import load_image_encoder

    cfg = CLIPVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=2,
                           image_size=56, patch_size=14, projection_dim=24, hidden_act="quick_gelu")
    torch.manual_seed(0)
    ref = CLIPVisionModelWithProjection(cfg).eval()
    d = tmp_path / "image_encoder"
    d.mkdir()
    save_file({k: v.contiguous() for k, v in ref.state_dict().items()}, str(d / "model.safetensors"))
    with open(d / "config.json", "w") as f:
        json.dump(cfg.to_dict(), f)
    enc = load_image_encoder("cpu", str(tmp_path))
    assert enc.weights_source == str(d)
    imgs = [_img(80, 1), _img(60, 2)]
    x = enc.preprocess(imgs)  # NHWC
    assert x.shape == (2, 56, 56, 3)
    with torch.no_grad():
        want = ref(pixel_values=x.permute(0, 3, 1, 2).contiguous()).image_embeds
        got = enc(x)
    assert torch.allclose(got, want, atol=1e-4, rtol=1e-4), (got - want).abs().max()


def test_depth_latents_normalised_and_given_map():
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.pipelines.variants import depth_latents

    pipe = StableDiffusion("tiny-depth", device="cpu", seed=1)
    assert pipe.family.is_depth and pipe.unet.cfg.in_channels == 5
    dm = torch.linspace(0, 7, 64 * 64).reshape(64, 64)
    d = depth_latents(pipe, [_img()], 8, 8, depth_map=dm)
    assert d.shape == (1, 8, 8, 1)
    assert abs(float(d.min()) + 1) < 1e-5 and abs(float(d.max()) - 1) < 1e-5
    # a monotone map stays monotone along its rows
    assert (d[0, :, 1:, 0] >= d[0, :, :-1, 0] - 1e-5).all()


def test_depth2img_job_end_to_end_cpu():
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd-depth", pipeline_type="StableDiffusionImg2ImgPipeline",
                                            prompt="a red house", image=_img(64), num_inference_steps=3,
                                            strength=0.7, generator=g, scheduler_type="DPMSolverMultistepScheduler",
                                            upscale=False, supports_xformers=True)
    assert _size(res) == (64, 64)
    assert cfg["_pipeline_type"] == "StableDiffusionDepth2ImgPipeline"
    # the depth channel matters: a different depth map changes the image
    pipe = diffusion.load_sd("tiny/sd-depth", "cpu")
    outs = []
    for dm in (torch.zeros(64, 64) + torch.arange(64.0), torch.zeros(64, 64) + torch.arange(64.0)[:, None]):
        g = torch.Generator().manual_seed(0)
        outs.append(pipe(prompt="a", image=_img(64), num_inference_steps=2, strength=0.8, generator=g,
                         depth_map=dm, output_type="latent").latents)
    assert not torch.equal(outs[0], outs[1])


def test_image_variation_job_end_to_end_cpu():
    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd-image-variation", pipeline_type="DiffusionPipeline",
                                            prompt="", image=_img(64), num_inference_steps=3, guidance_scale=3.0,
                                            num_images_per_prompt=2, generator=g,
                                            scheduler_type="DPMSolverMultistepScheduler", upscale=False,
                                            supports_xformers=True)
    assert cfg["_pipeline_type"] == "StableDiffusionImageVariationPipeline"
    assert cfg.get("image_encoder") == ["chiaswarm_amd", "CLIPVisionModelWithProjection"]
    assert _size(res)[0] >= 64
    pipe = diffusion.load_sd("tiny/sd-image-variation", "cpu")
    # context: the image embedding, zeros for the unconditional half
    pipe._img_ctx = pipe.image_embeds([_img(64)])
    ctx, added, kv = pipe.encode([""], [""], True)
    pipe._img_ctx = None
    assert ctx.shape[:2] == (2, 1) and torch.count_nonzero(ctx[0]) == 0 and torch.count_nonzero(ctx[1]) > 0
    # different input images -> different results
    lat = []
    for seed in (1, 2):
        g = torch.Generator().manual_seed(0)
        lat.append(pipe(image=_img(64, seed), num_inference_steps=2, generator=g, output_type="latent").latents)
    assert not torch.equal(lat[0], lat[1])
    with pytest.raises(ValueError, match="input image"):
        pipe(num_inference_steps=2)
    with pytest.raises(TypeError, match="unexpected"):
        pipe(image=_img(64), num_inference_steps=2, mask_image=_img(64))


def test_variant_class_resolution_and_routing():
    assert diffusion.pipeline_class_for("StableDiffusionImg2ImgPipeline", "stabilityai/stable-diffusion-2-depth") == \
        "StableDiffusionDepth2ImgPipeline"
    assert diffusion.pipeline_class_for("DiffusionPipeline", "lambdalabs/sd-image-variations-diffusers") == \
        "StableDiffusionImageVariationPipeline"
    for cls in ("StableDiffusionDepth2ImgPipeline", "StableDiffusionImageVariationPipeline"):
        _, kw = router.format_args({"model_name": "m", "parameters": {"pipeline_type": cls}})
        assert kw["pipeline_type"] == cls
    for cls in ("KandinskyPipeline", "UnCLIPPipeline", "UnCLIPImageVariationPipeline"):
        with pytest.raises(ValueError, match=cls):
            router.format_args({"model_name": "m", "parameters": {"pipeline_type": cls}})


def test_image_variation_checkpoint_without_text_encoder(tmp_path):
    """A diffusers directory with image_encoder/ and no text_encoder/ parses to
    the ImageVariation family (model_index.json class) and loads strictly."""
    from safetensors.torch import save_file
    from transformers import CLIPVisionConfig, CLIPVisionModelWithProjection

    from chiaswarm_amd.models.hf_config import pipeline_spec
    from chiaswarm_amd.pipelines.sd import resolve_family
    from chiaswarm_amd.pipelines.variants import ImageVariation

    from chiaswarm_amd.models import hf_config as hc
    from chiaswarm_amd.models import unet as unet_mod
    from chiaswarm_amd.models import vae as vae_mod
    from chiaswarm_amd.models.layers import init_random_
    from tests.test_hf_config import _j, _save_st, _tiny_unet, _tiny_vae, _write_json

    root = tmp_path / "iv"
    sd15 = "runwayml--stable-diffusion-v1-5"
    uc = _tiny_unet(_j(sd15, "unet", "config.json"), 24)
    _write_json(str(root / "unet" / "config.json"), uc)
    u = unet_mod.UNet2DConditionModel(hc.unet_config(uc))
    init_random_(u, seed=7)
    _save_st(u, str(root / "unet"))
    vc = _tiny_vae(_j(sd15, "vae", "config.json"))
    _write_json(str(root / "vae" / "config.json"), vc)
    v = vae_mod.AutoencoderKL(hc.vae_config(vc))
    init_random_(v, seed=8)
    _save_st(v, str(root / "vae"))
    (root / "scheduler").mkdir()
    _write_json(str(root / "scheduler" / "scheduler_config.json"), _j(sd15, "scheduler", "scheduler_config.json"))
    cfg = CLIPVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=2,
                           image_size=28, patch_size=14, projection_dim=24, hidden_act="quick_gelu")
    enc = CLIPVisionModelWithProjection(cfg).eval()
    (root / "image_encoder").mkdir()
    save_file({k: v.contiguous() for k, v in enc.state_dict().items()}, str(root / "image_encoder" / "model.safetensors"))
    with open(root / "image_encoder" / "config.json", "w") as f:
        json.dump(cfg.to_dict(), f)
    with open(root / "model_index.json", "w") as f:
        json.dump({"_class_name": "StableDiffusionImageVariationPipeline", "unet": ["diffusers", "UNet2DConditionModel"],
                   "vae": ["diffusers", "AutoencoderKL"],
                   "image_encoder": ["transformers", "CLIPVisionModelWithProjection"],
                   "scheduler": ["diffusers", "PNDMScheduler"]}, f)
    spec = pipeline_spec(str(root))
    assert spec.text == [] and spec.class_name == "StableDiffusionImageVariationPipeline"
    f2 = resolve_family("x/iv", str(root))
    assert f2.is_image_variation
    pipe = ImageVariation(f2, device="cpu", weights_dir=str(root))
    assert pipe.weights_source == str(root) and pipe.image_encoder.weights_source.endswith("image_encoder")
    g = torch.Generator().manual_seed(0)
    out = pipe(image=_img(64), num_inference_steps=2, generator=g, output_type="latent")
    assert torch.isfinite(out.latents).all()


def test_unclip_img2img_end_to_end_cpu():
    """StableUnCLIPImg2ImgPipeline: the checkpoint class wins over the router's
    Img2Img default; the class embedding is the noised, level-tagged CLIP image
    embedding (pinned against its formula); image and noise level both steer the
    result; the unconditional CFG half gets zero class labels."""
    import math

    from chiaswarm_amd.models.layers import timestep_embedding
    from chiaswarm_amd.pipelines.variants import UnCLIPImg2Img
    from chiaswarm_amd.schedulers import batch_randn

    g = torch.Generator().manual_seed(0)
    res, cfg = diffusion.diffusion_callback("cpu", "tiny/sd-unclip", pipeline_type="StableDiffusionImg2ImgPipeline",
                                            prompt="a boat", image=_img(64), num_inference_steps=3, generator=g,
                                            scheduler_type="DDIMScheduler", upscale=False, supports_xformers=True)
    assert cfg["_pipeline_type"] == "StableUnCLIPImg2ImgPipeline" and _size(res) == (64, 64)
    assert cfg.get("image_normalizer") == ["chiaswarm_amd", "StableUnCLIPImageNormalizer"]
    pipe = diffusion.load_sd("tiny/sd-unclip", "cpu")
    assert isinstance(pipe, UnCLIPImg2Img) and pipe.unet.cfg.class_embed_type == "projection"
    # noise_image_embeddings against its formula (normaliser mean 0.5 / std 2, level 500)
    m0, s0 = pipe.norm_mean, pipe.norm_std
    pipe.norm_mean, pipe.norm_std = torch.full((1, 32), 0.5), torch.full((1, 32), 2.0)
    try:
        emb = torch.randn(2, 32)
        got = pipe.noise_image_embeds(emb, 500, torch.Generator().manual_seed(3))
        noise = batch_randn((2, 32), torch.Generator().manual_seed(3), torch.device("cpu"))
        a = float(pipe.noise_abar[500])
        want = (math.sqrt(a) * (emb - 0.5) / 2.0 + math.sqrt(1 - a) * noise) * 2.0 + 0.5
        assert torch.allclose(got[:, :32], want, atol=1e-5)
        assert torch.allclose(got[:, 32:], timestep_embedding(torch.full((2,), 500.0), 32), atol=1e-6)
    finally:
        pipe.norm_mean, pipe.norm_std = m0, s0
    assert 0.999 < float(pipe.noise_abar[0]) <= 1.0 and float(pipe.noise_abar[999]) < 1e-3  # squaredcos_cap_v2
    # the unconditional half's class labels are zeros
    pipe._class = torch.ones(1, 64)
    _, added, _ = pipe.encode(["a"], [""], True)
    pipe._class = None
    assert added["class_labels"].shape == (2, 64) and torch.count_nonzero(added["class_labels"][0]) == 0

    def run(**kw):
        g = torch.Generator().manual_seed(0)
        return pipe(prompt="a", num_inference_steps=2, generator=g, output_type="latent", **kw).latents

    base = run(image=_img(64, 1))
    assert not torch.equal(base, run(image=_img(64, 2)))
    assert not torch.equal(base, run(image=_img(64, 1), noise_level=600))
    e = pipe.image_embeds([_img(64, 1)])
    assert torch.equal(base, run(image_embeds=e))
    with pytest.raises(ValueError, match="input image"):
        pipe(prompt="a", num_inference_steps=2)
    with pytest.raises(ValueError, match="noise_level"):
        pipe(image=_img(64), num_inference_steps=2, noise_level=1000)


def test_unet_projection_class_embedding_config():
    from chiaswarm_amd.models import hf_config as hc

    cfg = hc.unet_config({"block_out_channels": [32, 64], "down_block_types": ["CrossAttnDownBlock2D", "DownBlock2D"],
                          "up_block_types": ["UpBlock2D", "CrossAttnUpBlock2D"], "layers_per_block": 1,
                          "attention_head_dim": 2, "cross_attention_dim": 32, "class_embed_type": "projection",
                          "projection_class_embeddings_input_dim": 64, "sample_size": 8, "in_channels": 4,
                          "out_channels": 4})
    assert cfg.class_embed_type == "projection" and cfg.projection_class_embeddings_input_dim == 64
    from chiaswarm_amd.models.unet import UNet2DConditionModel

    u = UNet2DConditionModel(cfg)
    assert {"class_embedding.linear_1.weight", "class_embedding.linear_2.weight"} <= set(u.state_dict())


@pytest.mark.gpu
def test_variants_on_gpu(gpu):
    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.pipelines.variants import ImageVariation

    g = torch.Generator(device=gpu).manual_seed(0)
    d = StableDiffusion("tiny-depth", device=gpu, seed=1)
    out = d(prompt="a", image=_img(64), num_inference_steps=3, strength=0.8, generator=g,
            depth_map=torch.arange(64.0).repeat(64, 1))
    assert len(out.images) == 1 and torch.isfinite(out.latents).all()
    from chiaswarm_amd.pipelines.variants import UnCLIPImg2Img

    un = UnCLIPImg2Img("tiny-unclip", device=gpu, seed=3)
    g = torch.Generator(device=gpu).manual_seed(0)
    out = un(image=_img(64), prompt="a", num_inference_steps=3, generator=g, noise_level=100)
    assert len(out.images) == 1 and torch.isfinite(out.latents).all()
    iv = ImageVariation("tiny-imagevar", device=gpu, seed=2)
    g = torch.Generator(device=gpu).manual_seed(0)
    out = iv(image=_img(64), num_inference_steps=3, generator=g, num_images_per_prompt=2)
    assert len(out.images) == 2 and torch.isfinite(out.latents).all()
