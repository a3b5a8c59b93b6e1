"""Per-model tuning context (ops/tuning.py::context): a shape key shared by the
SD2.1 and SDXL steps can carry a separate SDXL entry ("sdxl|<key>") that only
the SDXL UNet's calls see; everything else keeps the plain entry."""
import torch

from chiaswarm_amd.models import unet as unet_mod
from chiaswarm_amd.ops import tuning


def test_context_entry_wins_only_inside_its_context(monkeypatch):
    t = {"g:2048:1280:1280:0": [13, 1, 19.0], "sdxl|g:2048:1280:1280:0": [20, 2, 18.0]}
    monkeypatch.setattr(tuning, "_TABLE", t)
    never = lambda tile, split: (_ for _ in ()).throw(AssertionError("no measuring"))  # noqa: E731
    assert tuning.choose("g:2048:1280:1280:0", 2048, 1280, 1280, never) == (13, 1)
    with tuning.context("sdxl"):
        assert tuning.current_context() == "sdxl"
        assert tuning.choose("g:2048:1280:1280:0", 2048, 1280, 1280, never) == (20, 2)
        # keys without an sdxl entry fall back to the plain one
        t["g:512:640:640:0"] = [14, 1, 5.0]
        assert tuning.choose("g:512:640:640:0", 512, 640, 640, never) == (14, 1)
        with tuning.context(None):
            assert tuning.choose("g:2048:1280:1280:0", 2048, 1280, 1280, never) == (13, 1)
        assert tuning.current_context() == "sdxl"
    assert tuning.current_context() is None


def test_sdxl_unet_forward_runs_in_its_context(monkeypatch):
    seen = []
    m = unet_mod.UNet2DConditionModel(unet_mod.TINY_XL)
    monkeypatch.setattr(m, "_forward", lambda *a, **k: seen.append(tuning.current_context()))
    m(torch.zeros(1))
    assert seen == ["sdxl"]
    m2 = unet_mod.UNet2DConditionModel(unet_mod.TINY)
    monkeypatch.setattr(m2, "_forward", lambda *a, **k: seen.append(tuning.current_context()))
    m2(torch.zeros(1))
    assert seen == ["sdxl", None]
