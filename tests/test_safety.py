"""NSFW safety checker semantics (CompVis checker: concept + special-care cosine
thresholds, flagged images blacked out) and its pipeline / envelope wiring."""
import base64
import io

import numpy as np
import torch
from PIL import Image

from chiaswarm_amd.models.safety import load_safety_checker


def _images(n=3, size=40):
    rng = np.random.default_rng(0)
    return torch.from_numpy((rng.random((n, size, size, 3)) * 255).astype(np.uint8))


def test_random_tower_never_flags():
    sc = load_safety_checker("cpu", tiny=True)
    flags, out = sc(_images())
    assert flags == [False, False, False]
    assert torch.equal(out, _images())


def test_concept_threshold_and_special_care_adjustment():
    sc = load_safety_checker("cpu", tiny=True)
    imgs = _images()
    with torch.no_grad():
        x = sc.preprocess(imgs)
        emb = torch.nn.functional.normalize(sc.visual_projection(sc.vision_model(x)[:, 0]), dim=-1)
        # concept 0 = image 1's embedding; threshold just above image 1's cos sim with itself
        sc.concept_embeds[0] = emb[1]
        cos = emb @ emb[1]
        sc.concept_embeds_weights[0] = float(cos[1]) + 0.005
    flags, _ = sc(imgs)
    assert flags == [False, False, False]  # 1.0 - (1.0 + 0.005) < 0
    with torch.no_grad():  # a special-care hit lowers every concept threshold by 0.01
        sc.special_care_embeds[0] = emb[1]
        sc.special_care_embeds_weights[0] = 0.5
    flags, out = sc(imgs)
    assert flags[1] is True
    assert int(out[1].max()) == 0 and torch.equal(out[0], imgs[0])


def test_pipeline_sets_nsfw_and_blacks_out(monkeypatch, tmp_path):
    monkeypatch.setenv("SDAAS_ROOT", str(tmp_path))
    from chiaswarm_amd.pipelines.sd import StableDiffusion

    pipe = StableDiffusion("tiny", device="cpu")
    sc = load_safety_checker("cpu", tiny=True)
    with torch.no_grad():
        sc.concept_embeds_weights.fill_(-2.0)  # everything flagged
    pipe.safety_checker = sc
    out = pipe(prompt="x", num_inference_steps=2, height=64, width=64, generator=torch.Generator().manual_seed(0))
    assert out.nsfw_content_detected == [True]
    assert np.asarray(out.images[0]).max() == 0
    # the job envelope carries the flag (reference: swarm/diffusion/diffusion_func.py:98-111)
    from chiaswarm_amd.output.processor import OutputProcessor

    op = OutputProcessor(["primary"], "image/png")
    op.add_outputs(out.images)
    blob = op.get_results()["primary"]["blob"]
    assert Image.open(io.BytesIO(base64.b64decode(blob))).size == (64, 64)
