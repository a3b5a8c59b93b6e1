"""Golden result-envelope tests (reference swarm/output_processor.py)."""
import base64
import hashlib
import io
import json

import pytest
from PIL import Image

from chiaswarm_amd.output import processor as op


def img(c=(10, 20, 30), size=(64, 48)):
    return Image.new("RGB", size, c)


@pytest.mark.parametrize("n,grid", [(1, (1, 1)), (2, (1, 2)), (3, (2, 2)), (4, (2, 2)), (5, (2, 3)), (6, (2, 3)),
                                    (7, (3, 3)), (9, (3, 3))])
def test_grid_policy(n, grid):
    out = op.post_process([img((i * 20, 0, 0)) for i in range(n)])
    rows, cols = grid
    assert out.size == (64 * cols, 48 * rows)


def test_too_many_images():
    with pytest.raises(ValueError):
        op.post_process([img()] * 10)


def test_grid_row_major_order():
    ims = [img((255, 0, 0)), img((0, 255, 0)), img((0, 0, 255))]
    g = op.post_process(ims)
    assert g.getpixel((10, 10)) == (255, 0, 0)
    assert g.getpixel((64 + 10, 10)) == (0, 255, 0)
    assert g.getpixel((10, 48 + 10)) == (0, 0, 255)
    assert g.getpixel((64 + 10, 48 + 10)) == (0, 0, 0)


@pytest.mark.parametrize("ct,fmt", [("image/jpeg", "JPEG"), ("image/png", "PNG")])
def test_envelope(ct, fmt):
    p = op.OutputProcessor(["primary"], ct)
    p.add_outputs([img(), img()])
    res = p.get_results()
    a = res["primary"]
    assert set(a) == {"blob", "content_type", "thumbnail", "sha256_hash"}
    blob = base64.b64decode(a["blob"])
    assert a["sha256_hash"] == hashlib.sha256(blob).hexdigest()
    assert Image.open(io.BytesIO(blob)).format == fmt
    th = Image.open(io.BytesIO(base64.b64decode(a["thumbnail"])))
    assert th.format == "JPEG" and max(th.size) <= 100
    assert a["content_type"] == ct


def test_other_outputs_and_unknown_names():
    p = op.OutputProcessor(["primary", "inference_image_strip"], "image/jpeg")
    p.add_outputs([img()])
    p.add_other_outputs("preprocessed_input", [img((1, 2, 3))])
    res = p.get_results()
    assert set(res) == {"primary", "preprocessed_input"}


def test_text_result_hashes_string_not_blob():
    r = op.make_text_result("a caption")
    assert r["content_type"] == "application/json"
    assert json.loads(base64.b64decode(r["blob"])) == {"caption": "a caption"}
    assert r["sha256_hash"] == hashlib.sha256(b"a caption").hexdigest()


def test_audio_thumbnail_is_text_tile():
    r = op.make_result(io.BytesIO(b"ID3fakeaudio"), None, "audio/mpeg")
    th = Image.open(io.BytesIO(base64.b64decode(r["thumbnail"])))
    assert th.size == (100, 100)


def test_bad_content_type():
    with pytest.raises(ValueError):
        op.image_to_buffer(img(), "image/gif")
    with pytest.raises(ValueError):
        op.image_to_buffer(img(), "video/mp4")


def test_deferred_encoding_in_encoder_processes_matches_inline():
    """GPU worker mode: artifacts come back as Futures from spawned encoder
    processes and resolve to exactly the inline envelope."""
    import numpy as np

    from chiaswarm_amd.output.encoder import EncoderPool

    rng = np.random.default_rng(0)
    ims = [Image.fromarray(rng.integers(0, 255, (64, 64, 3), dtype=np.uint8)) for _ in range(3)]
    p = op.OutputProcessor(["primary"], "image/jpeg")
    p.add_outputs(ims)
    inline = p.get_results()
    pool = EncoderPool(1)
    assert pool.kind == "process"
    op.set_encoder_pool(pool)
    try:
        p2 = op.OutputProcessor(["primary"], "image/jpeg")
        p2.add_outputs(ims)
        res = p2.get_results()
        assert hasattr(res["primary"], "result")  # deferred
        out = op.resolve_artifacts({"artifacts": res})["artifacts"]
        assert out == inline
        with pytest.raises(ValueError):  # >9 images: still raised in-line (fatal class)
            p3 = op.OutputProcessor(["primary"], "image/jpeg")
            p3.add_outputs(ims * 4)
            p3.get_results()
    finally:
        op.set_encoder_pool(None)
        pool.shutdown()


def test_thumbnail_from_image_matches_decoded_bytes():
    """make_thumbnail(PIL image) skips the JPEG re-decode; the 100x100 tile must
    match the reference path (thumbnail of the decoded blob) up to JPEG noise."""
    import numpy as np
    from PIL import Image

    from chiaswarm_amd.output.processor import image_to_buffer, make_thumbnail

    rng = np.random.default_rng(0)
    base = rng.integers(0, 255, (8, 8, 3), dtype=np.uint8)
    img = Image.fromarray(base).resize((1024, 1024), Image.Resampling.BILINEAR)
    buf = image_to_buffer(img, "image/jpeg")
    a = np.asarray(Image.open(make_thumbnail(img)), dtype=np.int16)
    b = np.asarray(Image.open(make_thumbnail(buf.getvalue())), dtype=np.int16)
    assert a.shape == b.shape == (100, 100, 3)
    assert np.abs(a - b).mean() < 3.0
    assert img.size == (1024, 1024)  # the caller's image is not resized in place


def test_encoder_pool_survives_a_dead_worker():
    """A killed encoder process: its pending task fails, no replacement is ever
    spawned (the GPU process may not exec), and once no encoder process is left
    the pool degrades to encoder threads; later jobs still encode."""
    import os
    import signal
    import time

    import numpy as np

    from chiaswarm_amd.output.encoder import EncoderPool

    pool = EncoderPool(1)
    assert pool.kind == "process"
    arrs = [np.zeros((32, 32, 3), dtype=np.uint8)]
    try:
        first = pool.submit(arrs, "image/png").result(timeout=60)
        for pid in pool.pids():
            os.kill(pid, signal.SIGKILL)
        time.sleep(1.0)
        try:
            pool.submit(arrs, "image/png").result(timeout=60)  # may be the one that hits the broken pool
        except Exception:
            pass
        again = pool.submit(arrs, "image/png").result(timeout=60)
        assert pool.kind == "thread"
        assert again["primary"]["blob"] == first["primary"]["blob"]
    finally:
        pool.shutdown()
