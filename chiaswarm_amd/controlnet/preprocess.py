"""ControlNet input preprocessors (reference: swarm/controlnet/input_processor.py:17-115).

Dispatch on ``parameters.controlnet.type`` when ``preprocess`` is true:
  canny    -> own Canny (Sobel 3x3 + L1 magnitude + NMS + double threshold +
              hysteresis, cv2.Canny semantics, defaults 100/200); runs as a HIP
              kernel on the GPU when a CUDA tensor path is requested, numpy on CPU
  tile     -> resize so the short side is a multiple of 64 (reference image_to_tile)
  shuffle  -> content shuffle (random smooth flow warp, seeded)
  scribble / softedge / lineart / mlsd / depth / seg / openpose / normalbae
           -> neural annotators (controlnet/annotators.py: HED, informative-
              drawings lineart, PiDiNet, M-LSD, DPT-Large, UperNet-ConvNeXt, OpenPose
              body, NormalBae NNET), resident per process
  a type listed in UNAVAILABLE (none today) -> ValueError -> fatal job error,
              like an incompatible model
"""
from __future__ import annotations

import numpy as np
from PIL import Image

UNAVAILABLE: set = set()


def preprocess_image(image: Image.Image, controlnet: dict) -> Image.Image:
    if not controlnet.get("preprocess", False):
        return image
    t = controlnet.get("type", "canny")
    if t == "canny":
        return image_to_canny(image, controlnet.get("low_threshold", 100), controlnet.get("high_threshold", 200))
    if t == "tile":
        return image_to_tile(image)
    if t == "shuffle":
        return content_shuffle(image)
    if t == "pix2pix":
        return image
    if t in ("scribble", "softedge", "lineart", "mlsd", "depth", "seg", "openpose", "normalbae"):
        from . import annotators as an

        if t == "scribble":
            return an.hed(image, scribble=True)
        if t == "softedge":
            return an.pidinet(image)
        if t == "lineart":
            return an.lineart(image, coarse=bool(controlnet.get("coarse", False)))
        if t == "mlsd":
            return an.mlsd(image)
        if t == "depth":
            return an.depth(image)
        if t == "openpose":
            return an.openpose(image)
        if t == "normalbae":
            return an.normalbae(image)
        return an.segmentation(image)
    if t in UNAVAILABLE:
        raise ValueError(f"controlnet preprocessor '{t}' is not available on this worker")
    raise ValueError(f"unknown controlnet type {t}")


def image_to_tile(image: Image.Image, resolution: int = 1024) -> Image.Image:
    w, h = image.size
    k = float(resolution) / min(h, w)
    h2, w2 = int(round(h * k / 64.0)) * 64, int(round(w * k / 64.0)) * 64
    return image.convert("RGB").resize((w2, h2), Image.Resampling.LANCZOS)


def _sobel(img: np.ndarray):
    """3x3 Sobel dx, dy with BORDER_REPLICATE (OpenCV canny.cpp) of [H, W] or [H, W, C]."""
    pw = ((1, 1), (1, 1)) + (((0, 0),) if img.ndim == 3 else ())
    p = np.pad(img, pw, mode="edge")
    gx = (p[:-2, 2:] + 2 * p[1:-1, 2:] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[1:-1, :-2] + p[2:, :-2])
    gy = (p[2:, :-2] + 2 * p[2:, 1:-1] + p[2:, 2:]) - (p[:-2, :-2] + 2 * p[:-2, 1:-1] + p[:-2, 2:])
    return gx, gy


def canny_np(img: np.ndarray, low: float, high: float) -> np.ndarray:
    """cv2.Canny-compatible edge map (uint8 0/255) of a uint8 [H, W] or [H, W, C]
    image.  Multi-channel: each pixel uses the dx/dy of the channel with the
    largest L1 magnitude (first on ties), as OpenCV does for colour input —
    the reference calls cv2.Canny on the RGB array
    (swarm/controlnet/input_processor.py:77-81).  Parity with cv2 itself is
    unpinned here (OpenCV is not installed); the rules follow canny.cpp."""
    from scipy import ndimage

    g = img.astype(np.float32)
    gx, gy = _sobel(g)
    if g.ndim == 3:
        m = np.abs(gx) + np.abs(gy)
        k = np.argmax(m, axis=-1)[..., None]  # first max on ties
        gx = np.take_along_axis(gx, k, -1)[..., 0]
        gy = np.take_along_axis(gy, k, -1)[..., 0]
    mag = np.abs(gx) + np.abs(gy)  # L1 gradient (cv2 default L2gradient=False)
    ang = np.arctan2(gy, gx)
    # quantise direction to 0/45/90/135 degrees
    q = (np.round(ang / (np.pi / 4)) % 4).astype(np.int8)
    p = np.pad(mag, 1)
    H, W = mag.shape
    c = p[1:-1, 1:-1]
    # (previous neighbour: strict, next neighbour: >=), as canny.cpp
    nb = {0: (p[1:-1, :-2], p[1:-1, 2:]), 1: (p[:-2, :-2], p[2:, 2:]),
          2: (p[:-2, 1:-1], p[2:, 1:-1]), 3: (p[:-2, 2:], p[2:, :-2])}
    keep = np.zeros_like(mag, dtype=bool)
    for d, (a, b) in nb.items():
        m = q == d
        keep |= m & (c > a) & (c >= b)
    nms = np.where(keep, mag, 0.0)
    strong = nms > high
    weak = nms > low
    lab, n = ndimage.label(weak, structure=np.ones((3, 3)))
    if n == 0:
        return np.zeros((H, W), np.uint8)
    ok = np.zeros(n + 1, dtype=bool)
    ok[np.unique(lab[strong])] = True
    ok[0] = False
    return (ok[lab] * 255).astype(np.uint8)


def image_to_canny(image: Image.Image, low=100, high=200, device=None) -> Image.Image:
    """cv2.Canny semantics; on a GPU device the HIP kernel (csrc/kernels/canny.hip)
    runs it in well under a millisecond (the numpy path takes ~0.3 s at 512²)."""
    arr = np.asarray(image.convert("RGB"))  # cv2.Canny on the RGB array, like the reference
    dev = device
    if dev is None:
        import torch

        dev = "cuda" if torch.cuda.is_available() else "cpu"
    if str(dev).startswith("cuda"):
        import torch

        from .. import ops

        if ops.get_mode() == "hip" and ops._lib.available():
            e = ops.canny(torch.from_numpy(arr.copy()).to(dev), float(low), float(high)).cpu().numpy()
            return Image.fromarray(np.stack([e] * 3, axis=-1))
    e = canny_np(arr, float(low), float(high))
    return Image.fromarray(np.stack([e] * 3, axis=-1))


def content_shuffle(image: Image.Image, seed: int = 0, f: int = 256) -> Image.Image:
    from scipy import ndimage

    arr = np.asarray(image.convert("RGB")).astype(np.float32)
    h, w = arr.shape[:2]
    rng = np.random.default_rng(seed)
    flow = [ndimage.gaussian_filter(rng.standard_normal((h, w)), sigma=f / 8) for _ in range(2)]
    flow = [fl / (np.abs(fl).max() + 1e-6) * f for fl in flow]
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    ys, xs = np.clip(yy + flow[0], 0, h - 1), np.clip(xx + flow[1], 0, w - 1)
    out = np.stack([ndimage.map_coordinates(arr[..., c], [ys, xs], order=1) for c in range(3)], axis=-1)
    return Image.fromarray(out.clip(0, 255).astype(np.uint8))
