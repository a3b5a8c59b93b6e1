"""Provisioning (reference: swarm/initialize.py:62-116): the hive catalogue is
fetched, every can_preload model is downloaded with revision / variant and only
the file kinds this framework reads; no network in tests (stub downloader).
Plus the packed-weight cache written on first load."""
import json
import os

import torch

from chiaswarm_amd.initialize import IGNORE, allow_patterns, init, prepare_models
from chiaswarm_amd.settings import Settings
from tests.fakehive import FakeHive


def test_prepare_models_fetches_with_revision_variant_and_safe_patterns(tmp_path, monkeypatch):
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    models = {"language_models": [], "models": [
        {"model_name": "org/a", "revision": "fp16", "variant": "fp16", "parameters": {"can_preload": True}},
        {"model_name": "org/b", "revision": "main", "parameters": {"can_preload": False}},
        {"model_name": "org/c", "revision": "main", "parameters": {"can_preload": True}}]}
    hive = FakeHive(models=models).start()
    calls = []

    def fake_download(repo, revision=None, allow_patterns=None, ignore_patterns=None, token=None):
        calls.append((repo, revision, allow_patterns, ignore_patterns, token))
        if repo == "org/c":
            raise OSError("offline")
        d = tmp_path / "cache" / repo
        d.mkdir(parents=True, exist_ok=True)
        (d / "model.fp16.safetensors").write_bytes(b"x")  # a safetensors repo: one fetch, no pickles
        return str(d)

    try:
        s = Settings()
        s.sdaas_uri = hive.base
        s.huggingface_token = "hf_x"
        rep = prepare_models(s, downloader=fake_download)
    finally:
        hive.stop()
    assert [c[0] for c in calls] == ["org/a", "org/c"]  # can_preload only
    assert calls[0][1] == "fp16" and "*.fp16.safetensors" in calls[0][2] and calls[0][4] == "hf_x"
    assert "*.bin" in calls[0][3] and "*.ckpt" in calls[0][3]
    by = {r["model_name"]: r for r in rep}
    assert by["org/a"]["weights"] == str(tmp_path / "cache" / "org" / "a") and by["org/a"]["fetched"]
    assert "fetch_error" in by["org/c"] and by["org/c"]["weights"].startswith("synthetic")
    assert by["org/b"]["weights"].startswith("synthetic")
    assert os.path.exists(os.path.join(str(tmp_path), "models.json"))


def test_patterns_never_allow_pickles():
    for v in (None, "fp16"):
        pats = allow_patterns(v)
        assert not any(p.endswith((".bin", ".ckpt", ".pt", ".pth")) for p in pats)
    assert "*.bin" in IGNORE


def test_init_offline_silent_writes_report(tmp_path, monkeypatch):
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    rep = init(["--silent", "--offline"])
    assert rep == []
    assert json.load(open(os.path.join(str(tmp_path), "prepared_models.json"))) == []


def test_packed_cache_round_trip(tmp_path, monkeypatch):
    """First load packs and writes the cache; the second load reads it and gives
    bitwise-identical parameters and packed buffers without re-packing."""
    from safetensors.torch import save_file

    from chiaswarm_amd.pipelines.sd import StableDiffusion
    from chiaswarm_amd.runtime import packed_cache

    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    src = StableDiffusion("tiny", device="cpu", seed=41)
    d = tmp_path / "model"
    for sub, m in (("unet", src.unet), ("vae", src.vae), ("text_encoder", src.text_encoders[0])):
        os.makedirs(d / sub)
        save_file({k: v.contiguous() for k, v in m.state_dict().items()}, str(d / sub / "m.safetensors"))
    from test_checkpoints import _train_bpe

    _train_bpe(str(d / "tokenizer"))  # real weights need their tokenizer (strict loads)
    a = StableDiffusion("tiny", device="cpu", seed=1, weights_dir=str(d))
    assert all(not isinstance(r, str) for r in a.load_reports.values())
    calls = []
    orig = packed_cache.save
    monkeypatch.setattr(packed_cache, "save", lambda *x: calls.append(1) or orig(*x))
    b = StableDiffusion("tiny", device="cpu", seed=2, weights_dir=str(d))
    assert set(b.load_reports.values()) == {"packed cache"} and not calls
    for ma, mb in ((a.unet, b.unet), (a.vae, b.vae), (a.text_encoders[0], b.text_encoders[0])):
        for k, v in ma.state_dict().items():
            assert torch.equal(v, mb.state_dict()[k]), k
        ta, la = packed_cache._packed_items(ma)
        tb, lb = packed_cache._packed_items(mb)
        assert ta.keys() == tb.keys() and la == lb and len(ta) > 0
        for k in ta:
            assert torch.equal(ta[k], tb[k]), k
    g = torch.Generator().manual_seed(3)
    xa = a(prompt="x", num_inference_steps=2, height=64, width=64, generator=g, output_type="latent").latents
    g = torch.Generator().manual_seed(3)
    xb = b(prompt="x", num_inference_steps=2, height=64, width=64, generator=g, output_type="latent").latents
    assert torch.equal(xa, xb)
    # a changed source file invalidates the cache
    os.utime(d / "unet" / "m.safetensors", ns=(1, 1))
    c = StableDiffusion("tiny", device="cpu", seed=3, weights_dir=str(d))
    assert not isinstance(c.load_reports["unet"], str) and c.load_reports["vae"] == "packed cache"
