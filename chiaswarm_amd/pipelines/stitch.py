"""``workflow: stitch`` — contact sheet of other jobs' results + HTML image map
(reference: swarm/toolbox/stitch.py:10-110).  CPU only.

Same geometry: 144-px cells, ceil(sqrt(n)) per row, index label drawn at
(10, 10), JPEG web_high output, ``pipeline_config.image_map`` entries
{shape: rect, coords: "x0,y0,x1,y1", href, alt, filename}.
(``Image.ANTIALIAS`` used by the reference no longer exists in Pillow >= 10;
LANCZOS is the same filter.)
"""
from __future__ import annotations

import io
import math

from PIL import Image, ImageDraw

from ..output.processor import image_to_buffer, make_result, make_thumbnail

THUMB = 144


def stitch_callback(device_id, model_name, **kwargs):
    print("Stitching...")
    config = {"model_name": model_name}
    jobs = kwargs["jobs"]
    images = download_images([j["resultUri"] for j in jobs])
    resized = resize_images(images)
    sheet = stitch_images(resized)
    buf = image_to_buffer(sheet, "image/jpeg", "web_high")
    thumb = make_thumbnail(buf)
    results = {"primary": make_result(buf, thumb, "image/jpeg")}
    config["image_map"] = generate_image_map(resized, jobs)
    return results, config


def download_images(urls):
    import requests

    out = []
    for u in urls:
        r = requests.get(u, timeout=30)
        out.append(Image.open(io.BytesIO(r.content)))
    return out


def resize_images(images, size=(THUMB, THUMB)):
    out = []
    for i, im in enumerate(images):
        w, h = im.size
        ar = float(w) / float(h)
        if w > h:
            nw = min(size[0], w)
            nh = int(nw / ar)
        else:
            nh = min(size[1], h)
            nw = int(nh * ar)
        nw, nh = min(nw, size[0]), min(nh, size[1])
        r = im.resize((max(nw, 1), max(nh, 1)), Image.Resampling.LANCZOS)
        ImageDraw.Draw(r).text((10, 10), str(i + 1), fill=(255, 255, 255))
        out.append(r)
    return out


def _per_row(n):
    return math.ceil(math.sqrt(n))


def stitch_images(resized):
    per_row = _per_row(len(resized))
    side = THUMB * per_row
    sheet = Image.new("RGB", (side, side))
    x = y = 0
    for im in resized:
        sheet.paste(im, (x, y))
        x += THUMB
        if x >= side:
            x, y = 0, y + THUMB
    return sheet


def generate_image_map(resized, jobs):
    data = []
    x = y = 0
    side = THUMB * _per_row(len(resized))
    for i, _ in enumerate(resized):
        href = jobs[i]["resultUri"]
        data.append({"shape": "rect", "coords": f"{x},{y},{x + THUMB},{y + THUMB}", "href": href,
                     "alt": jobs[i].get("model_name", f"Image {i + 1}"),
                     "filename": jobs[i].get("fileName", href)})
        x += THUMB
        if x >= side:
            x, y = 0, y + THUMB
    return data
