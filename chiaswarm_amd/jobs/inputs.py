"""Input acquisition for jobs: remote images (HEAD checks + download) and
videos.  Reference: swarm/job_arguments.py:156-190 (image: content type must
start with ``image``, <= 3 MiB, EXIF transpose, RGB, thumbnail) and
swarm/video/pix2pix.py:90-122 (video: ``video/*``, <= 30 MiB).

Quirk fixed: the reference passed (height, width) to
``PIL.Image.thumbnail``, which takes (width, height); we pass (width, height).
"""
from __future__ import annotations

import io
import os
import tempfile

from PIL import Image, ImageOps

MAX_SIZE = 1024
MAX_IMAGE_BYTES = 1048576 * 3
MAX_VIDEO_BYTES = 1048576 * 30

_session = None


def _http():
    global _session
    if _session is None:
        import requests

        _session = requests.Session()
    return _session


def download_image(url: str) -> Image.Image:
    r = _http().get(url, allow_redirects=True, timeout=30)
    r.raise_for_status()
    if len(r.content) > MAX_IMAGE_BYTES:
        raise Exception(f"Input image too large.\nMax size is {MAX_IMAGE_BYTES} bytes.\nImage was {len(r.content)}.")
    image = Image.open(io.BytesIO(r.content))
    image = ImageOps.exif_transpose(image)
    return image.convert("RGB")


def get_image(uri: str, size=None, controlnet=None) -> Image.Image:
    """size: (height, width) like the reference's call sites."""
    head = _http().head(uri, allow_redirects=True, timeout=10)
    content_length = head.headers.get("Content-Length", 0)
    content_type = head.headers.get("Content-Type", "")
    if not content_type.startswith("image"):
        raise Exception(f"Input does not appear to be an image.\nContent type was {content_type}.")
    if int(content_length or 0) > MAX_IMAGE_BYTES:
        raise Exception(
            f"Input image too large.\nMax size is {MAX_IMAGE_BYTES} bytes.\nImage was {content_length}.")
    image = download_image(uri)
    if size is not None and (image.height > size[0] or image.width > size[1]):
        image.thumbnail((size[1], size[0]), Image.Resampling.LANCZOS)
    elif image.height > MAX_SIZE or image.width > MAX_SIZE:
        image.thumbnail((MAX_SIZE, MAX_SIZE), Image.Resampling.LANCZOS)
    if controlnet is not None:
        from ..controlnet.preprocess import preprocess_image

        image = preprocess_image(image, controlnet)
    return image


def download_video(uri: str) -> str:
    head = _http().head(uri, allow_redirects=True, timeout=10)
    content_length = head.headers.get("Content-Length", 0)
    content_type = head.headers.get("Content-Type", "")
    if not content_type.startswith("video"):
        raise Exception(f"Input does not appear to be a video.\nContent type was {content_type}.")
    if int(content_length or 0) > MAX_VIDEO_BYTES:
        raise Exception(
            f"Input video too large.\nMax size is {MAX_VIDEO_BYTES} bytes.\nVideo was {content_length}.")
    fd, path = tempfile.mkstemp(suffix=os.path.splitext(uri.split("?")[0])[1] or ".mp4")
    total = 0
    try:
        with os.fdopen(fd, "wb") as f, _http().get(uri, stream=True, allow_redirects=True, timeout=60) as r:
            r.raise_for_status()
            for chunk in r.iter_content(1 << 16):
                total += len(chunk)
                if total > MAX_VIDEO_BYTES:
                    raise Exception("Input video too large.")
                f.write(chunk)
    except BaseException:
        os.unlink(path)  # never leave a partial download behind
        raise
    return path
