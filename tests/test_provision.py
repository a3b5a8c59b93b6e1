"""Model provisioning at job time (runtime/provision.py; reference: every
callback builds its models with ``from_pretrained`` inside the job, which
downloads on a miss and raises when it cannot — swarm/diffusion/
diffusion_func.py:41-46, swarm/initialize.py:75-89).  No network: a fake
downloader stands in for ``huggingface_hub.snapshot_download``."""
import json
import os
import shutil
import threading
import time

import pytest
import torch

from chiaswarm_amd.runtime import provision
from chiaswarm_amd.runtime.device import Device
from chiaswarm_amd.runtime.generator import synchronous_do_work_function

TINY = {"model_name": "tiny/sd", "prompt": "a red fox", "num_inference_steps": 2, "height": 64, "width": 64}


@pytest.fixture(autouse=True)
def strict_provisioning(tmp_path, monkeypatch):
    """The production contract: no random-init fallback, fetch allowed."""
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path / "root"))
    monkeypatch.setenv("SDAAS_MODEL_DIR", str(tmp_path / "store"))
    monkeypatch.setenv("HF_HOME", str(tmp_path / "hf"))
    monkeypatch.setenv("SDAAS_PACKED_CACHE", "0")
    monkeypatch.delenv("SDAAS_ALLOW_RANDOM", raising=False)
    monkeypatch.delenv("SDAAS_OFFLINE", raising=False)
    from chiaswarm_amd.runtime import model_cache

    monkeypatch.setattr(model_cache, "_CACHE", None)
    monkeypatch.setattr(provision, "DOWNLOADER", None)
    yield


def _failing_downloader(*a, **k):
    raise OSError("no network")


def test_unprovisioned_model_is_a_nonfatal_error_naming_it(monkeypatch):
    monkeypatch.setattr(provision, "DOWNLOADER", _failing_downloader)
    r = synchronous_do_work_function({"id": "j1", **TINY}, Device("cpu"))
    assert "fatal_error" not in r  # retryable: another (provisioned) worker may take it
    err = r["pipeline_config"]["error"]
    assert "tiny/sd" in err and "not provisioned" in err and "no network" in err
    assert "seed" not in r["pipeline_config"]  # no image was generated


def test_offline_skips_the_fetch(monkeypatch):
    calls = []
    monkeypatch.setattr(provision, "DOWNLOADER", lambda *a, **k: calls.append(a))
    monkeypatch.setenv("SDAAS_OFFLINE", "1")
    with pytest.raises(provision.WeightsMissing, match="offline"):
        provision.ensure_weights("org/m")
    assert calls == []


def test_random_init_only_when_allowed(monkeypatch):
    monkeypatch.setattr(provision, "DOWNLOADER", _failing_downloader)
    monkeypatch.setenv("SDAAS_ALLOW_RANDOM", "1")
    assert provision.ensure_weights("org/m") is None
    r = synchronous_do_work_function({"id": "j2", **TINY, "seed": 3}, Device("cpu"))
    assert "error" not in r["pipeline_config"] and r["pipeline_config"]["seed"] == 3


def test_local_copy_needs_no_fetch(tmp_path, monkeypatch):
    d = tmp_path / "store" / "org" / "m"
    d.mkdir(parents=True)
    (d / "model.safetensors").write_bytes(b"x")
    monkeypatch.setattr(provision, "DOWNLOADER", _failing_downloader)
    assert provision.ensure_weights("org/m") == str(d)


def test_fetch_on_miss_once_under_concurrency(tmp_path, monkeypatch):
    """Two jobs of one process miss the same model at once: one download."""
    calls = []

    def fake(repo, revision=None, allow_patterns=None, ignore_patterns=None, token=None):
        calls.append((repo, revision, tuple(allow_patterns)))
        time.sleep(0.2)
        d = tmp_path / "hf" / "hub" / ("models--" + repo.replace("/", "--")) / "snapshots" / "abc"
        d.mkdir(parents=True, exist_ok=True)
        (d / "model.safetensors").write_bytes(b"x")
        return str(d)

    monkeypatch.setattr(provision, "DOWNLOADER", fake)
    out = []
    ts = [threading.Thread(target=lambda: out.append(provision.ensure_weights("org/m", "v2"))) for _ in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(calls) == 1 and calls[0][:2] == ("org/m", "v2") and "*.safetensors" in calls[0][2]
    assert out[0] == out[1] and out[0].endswith("abc")


def test_bin_only_repo_fetches_pickles_second(tmp_path):
    """A repo without safetensors is fetched again with *.bin allowed (what
    from_pretrained reads); safetensors repos never bring pickles."""
    from chiaswarm_amd.initialize import fetch

    calls = []

    def fake(repo, revision=None, allow_patterns=None, ignore_patterns=None, token=None):
        calls.append((tuple(allow_patterns), tuple(ignore_patterns)))
        d = tmp_path / repo
        d.mkdir(parents=True, exist_ok=True)
        if any(p.endswith(".bin") for p in allow_patterns):
            (d / "pytorch_model.bin").write_bytes(b"x")
        return str(d)

    fetch("org/binonly", downloader=fake)
    assert len(calls) == 2
    assert "*.bin" in calls[0][1] and "*.bin" in calls[1][0] and "*.bin" not in calls[1][1]
    assert "*.ckpt" in calls[1][1] and "*.pth" in calls[1][1]


def test_mixed_repo_fetches_bin_for_the_component_without_safetensors(tmp_path):
    """the .bin fallback is decided per component — a safetensors
    unet beside a text_encoder that ships only pytorch_model.bin gets that
    component's .bin fetched (and only that)."""
    from chiaswarm_amd.initialize import fetch

    calls = []

    def fake(repo, revision=None, allow_patterns=None, ignore_patterns=None, token=None):
        calls.append(tuple(allow_patterns))
        d = tmp_path / repo
        for comp in ("unet", "text_encoder"):
            (d / comp).mkdir(parents=True, exist_ok=True)
            (d / comp / "config.json").write_text("{}")
        (d / "unet" / "diffusion_pytorch_model.safetensors").write_bytes(b"x")
        if any(p.endswith(".bin") for p in allow_patterns):
            (d / "text_encoder" / "pytorch_model.bin").write_bytes(b"x")
        return str(d)

    path = fetch("org/mixed", downloader=fake)
    assert len(calls) == 2 and calls[1] == ("text_encoder/*.bin",)
    assert (tmp_path / "org/mixed" / "text_encoder" / "pytorch_model.bin").exists()
    assert path.endswith("org/mixed")


def test_safetensors_win_over_a_stray_pth(tmp_path):
    """a .pth beside safetensors never replaces them."""
    from safetensors.torch import save_file

    from chiaswarm_amd.models.weights import read_weights

    save_file({"w": torch.ones(3)}, str(tmp_path / "model.safetensors"))
    torch.save({"w": torch.zeros(3)}, str(tmp_path / "old.pth"))
    torch.save({"w": torch.zeros(3)}, str(tmp_path / "older.pth"))
    assert torch.equal(read_weights(str(tmp_path))["w"], torch.ones(3))


def test_bin_weights_load_like_safetensors(tmp_path):
    """diffusers / transformers ``*.bin`` component weights go through the
    weights-only unpickler and load strictly, same tensors as safetensors."""
    from safetensors.torch import save_file

    from chiaswarm_amd.models import unet as unet_mod
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.models.weights import load_component

    a = unet_mod.UNet2DConditionModel(unet_mod.TINY)
    init_random_(a, seed=1)
    sd = {k: v.contiguous() for k, v in a.state_dict().items()}
    os.makedirs(tmp_path / "b" / "unet")
    torch.save(sd, tmp_path / "b" / "unet" / "diffusion_pytorch_model.bin")
    (tmp_path / "b" / "unet" / "training_args.bin").write_bytes(b"not weights")
    os.makedirs(tmp_path / "s" / "unet")
    save_file(sd, str(tmp_path / "s" / "unet" / "diffusion_pytorch_model.safetensors"))
    for root in ("b", "s"):
        m = unet_mod.UNet2DConditionModel(unet_mod.TINY)
        init_random_(m, seed=2)
        rep = load_component(m, str(tmp_path / root), "unet")
        assert rep.complete and not rep.unexpected, rep.summary()
        for k, v in m.state_dict().items():
            assert torch.equal(v, sd[k]), (root, k)
    assert provision.has_weights(str(tmp_path / "b"))


def test_bin_loader_executes_nothing(tmp_path):
    """A pickle that would run code is refused by the weights-only loader."""
    from chiaswarm_amd.models.weights import read_weights

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    import pickle

    d = tmp_path / "unet"
    d.mkdir()
    with open(d / "diffusion_pytorch_model.bin", "wb") as f:
        pickle.dump({"w": Evil()}, f)
    with pytest.raises(Exception):
        read_weights(str(d))


def test_sd15_layout_runs_its_own_safety_checker(tmp_path, monkeypatch):
    """The checkpoint's own ``safety_checker/`` (listed in model_index.json) is
    the NSFW checker of the pipeline (reference: diffusion_func.py:98-111)."""
    from safetensors.torch import save_file

    from chiaswarm_amd.models import safety
    from chiaswarm_amd.models.layers import init_random_
    from chiaswarm_amd.pipelines import diffusion
    from tests.test_hf_config import _tiny_sd_dir

    d = _tiny_sd_dir("runwayml--stable-diffusion-v1-5", str(tmp_path / "store"))
    assert d == str(tmp_path / "store" / "runwayml" / "stable-diffusion-v1-5")
    sc = os.path.join(d, "safety_checker")
    os.makedirs(sc)
    t = safety.TINY_SAFETY
    with open(os.path.join(sc, "config.json"), "w") as f:
        json.dump({"projection_dim": t.proj, "vision_config": {
            "image_size": t.image_size, "patch_size": t.patch, "hidden_size": t.dim, "num_hidden_layers": t.depth,
            "num_attention_heads": t.heads, "intermediate_size": t.mlp}}, f)
    m = safety.SafetyChecker(t)
    init_random_(m, seed=5)
    sd = {("vision_model." + k if k.startswith("vision_model.") else k): v.contiguous()
          for k, v in m.state_dict().items()}
    # checkpoint keys follow transformers' CLIPVisionModel naming
    inv = {v: k for k, v in safety._HF_RENAMES.items()}
    out = {}
    for k, v in sd.items():
        kk = k
        for a, b in inv.items():
            kk = kk.replace(a, b)
        out[kk] = v
    save_file(out, os.path.join(sc, "model.safetensors"))
    os.makedirs(os.path.join(d, "feature_extractor"))
    assert diffusion.safety_checker_dir(d) == sc
    pipe = diffusion.load_sd("runwayml/stable-diffusion-v1-5", "cpu")
    assert pipe.safety_checker is not None and pipe.safety_checker.cfg == t
    assert torch.equal(pipe.safety_checker.concept_embeds.float(), m.concept_embeds.float())
    # a layout without one (SD2.x) falls back to a separately provisioned checker, else none
    shutil.rmtree(sc)
    assert diffusion.safety_checker_dir(d) is None


def test_sdxl_refiner_runs_with_aesthetic_time_ids(tmp_path, monkeypatch):
    """stable-diffusion-xl-refiner-1.0 layout (text_encoder_2 only,
    requires_aesthetics_score): img2img through the refiner UNet with
    (h, w, crop, crop, aesthetic score) time ids, negative rows at the negative
    score (diffusers StableDiffusionXLImg2ImgPipeline; parity unpinned: no
    diffusers here)."""
    from PIL import Image

    from chiaswarm_amd.pipelines.sd import StableDiffusion, resolve_family
    from tests.test_hf_config import _tiny_sd_dir

    d = _tiny_sd_dir("stabilityai--stable-diffusion-xl-refiner-1.0", str(tmp_path / "store"))
    fam = resolve_family("stabilityai/stable-diffusion-xl-refiner-1.0", d)
    assert fam.aesthetics and not fam.force_zeros and fam.text_components == ["text_encoder_2"]
    assert fam.pipeline_class == "StableDiffusionXLImg2ImgPipeline"
    pipe = StableDiffusion(fam, device="cpu", weights_dir=d)
    tid = pipe._time_ids(4, 64, 48, "cpu", (7.0, 2.0), 2)
    assert tid.tolist() == [[64, 48, 0, 0, 2.0]] * 2 + [[64, 48, 0, 0, 7.0]] * 2
    img = Image.new("RGB", (64, 64), (120, 30, 200))
    kw = dict(prompt="a fox", image=img, strength=0.5, num_inference_steps=2, guidance_scale=5.0,
              output_type="latent")
    a = pipe(**kw, generator=torch.Generator().manual_seed(0)).latents
    b = pipe(**kw, aesthetic_score=2.0, generator=torch.Generator().manual_seed(0)).latents
    assert torch.isfinite(a).all() and not torch.equal(a, b)  # the score reaches the UNet
    assert pipe.config["_class_name"] == "StableDiffusionXLImg2ImgPipeline"


def test_aesthetic_score_is_refiner_only():
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    pipe = StableDiffusion("tiny-xl", device="cpu")
    with pytest.raises(TypeError, match="aesthetic_score"):
        pipe(prompt="x", num_inference_steps=1, aesthetic_score=6.0, output_type="latent")


def test_sdxl_empty_negative_prompt_is_zero_embeddings():
    """diffusers force_zeros_for_empty_prompt (SDXL base): no negative prompt
    -> zero negative context / pooled, unlike an explicit "" negative."""
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    kw = dict(prompt="x", num_inference_steps=2, guidance_scale=5.0, output_type="latent", height=64, width=64)
    for fam, differs in (("tiny-xl", True), ("tiny", False)):
        pipe = StableDiffusion(fam, device="cpu")
        a = pipe(**kw, generator=torch.Generator().manual_seed(1)).latents
        b = pipe(**kw, negative_prompt="", generator=torch.Generator().manual_seed(1)).latents
        assert torch.equal(a, b) != differs, fam
        # per row: a batch mixing jobs with and without negatives (diffusion_batch)
        c = pipe(**dict(kw, prompt=["x", "x"]), negative_prompt=[None, ""],
                 generator=[(torch.Generator().manual_seed(1), 1), (torch.Generator().manual_seed(1), 1)]).latents
        assert torch.allclose(c[0], a[0], rtol=1e-4, atol=1e-3) and torch.allclose(c[1], b[0], rtol=1e-4, atol=1e-3)


def test_sdxl_zero_negative_kv_cache_matches_full_recompute():
    """The zero-negative K/V rows come from a per-pipeline cache (a zero
    context row's K/V is the projection bias): bitwise what re-running every
    K/V projection on the zeroed context gave, for leading and non-leading
    zero rows."""
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    pipe = StableDiffusion("tiny-xl", device="cpu", seed=3)

    def recompute(ctx, n):
        idx = (ctx.abs().sum((1, 2)) == 0).nonzero().flatten()
        return [t[idx].clone() for t in pipe.unet.encode_context(ctx)]

    for negs in ([None, None], ["blurry", None], [None, "blurry"]):
        kw = dict(prompt=["a fox", "a cat"], negative_prompt=negs, num_inference_steps=2, guidance_scale=6.0,
                  output_type="latent")
        a = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
        cached = pipe._zero_rows_kv
        pipe._zero_rows_kv = recompute
        try:
            b = pipe(generator=torch.Generator().manual_seed(0), **kw).latents
        finally:
            pipe._zero_rows_kv = cached
        assert torch.equal(a, b), negs
    pipe.invalidate_graphs()
    assert "_zero_kv" not in pipe.__dict__


def test_txt2vid_uses_the_checkpoint_scheduler_config(monkeypatch):
    """reference: scheduler_type.from_config(pipeline.scheduler.config,
    use_karras_sigmas=True) (swarm/video/tx2vid.py:32-34)"""
    import numpy as np

    from chiaswarm_amd.pipelines import video

    seen = {}

    class FakePipe:
        sched_config = {"beta_schedule": "scaled_linear", "beta_start": 0.00085, "beta_end": 0.012}
        config = {}

        def __call__(self, scheduler=None, **kw):
            seen["sched"] = scheduler
            return [np.zeros((8, 8, 3), np.uint8)] * 2

    real = video.get_scheduler

    def spy(name, **cfg):
        seen["cfg"] = dict(cfg)
        return real(name, **cfg)

    monkeypatch.setattr(video, "load_t2v", lambda *a, **k: FakePipe())
    monkeypatch.setattr(video, "get_scheduler", spy)
    video.txt2vid_diffusion_callback("cpu", "damo-vilab/text-to-video-ms-1.7b", prompt="x", num_inference_steps=2,
                                     content_type="video/webm")
    assert seen["cfg"] == FakePipe.sched_config and seen["sched"] is not None
