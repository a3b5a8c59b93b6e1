"""Neural ControlNet annotators (reference: swarm/controlnet/input_processor.py:17-115,
which calls controlnet_aux / transformers detectors):

  scribble  -> HED (ControlNetHED_Apache2) + scribble post-process (nms, blur, threshold)
  softedge  -> PiDiNet (table5_pidinet: pixel-difference convs folded into plain convs)
  lineart   -> "informative drawings" generator (sk_model / sk_model2 coarse)
  mlsd      -> M-LSD large (MobileNetV2 encoder + line-segment decoder)
  depth     -> DPT-Large (ViT-L/16 + reassemble/fusion neck + depth head)
  seg       -> UperNet + ConvNeXt backbone, ADE20K palette
  openpose  -> CMU body-pose model (18 keypoints, PAF grouping), skeleton canvas
  normalbae -> surface normals: EfficientNet-B5 encoder + MLP-refined decoder (NNET)

Module and parameter names follow the public checkpoints (controlnet_aux .pth
files / transformers safetensors) so real weights load unchanged from
``$CSK_ANNOTATOR_DIR`` (default ``<settings dir>/annotators``); loaders never
unpickle (safetensors, or ``torch.load(weights_only=True)``).  Without weights
a detector keeps a seeded random init (like every model in this framework
offline) and says so in the log.

Each detector is built once per process, kept resident on the GPU (bf16 there,
fp32 on CPU) and runs as plain PyTorch modules: these run once per job on one
image, far off the denoising hot path.
"""
from __future__ import annotations

import logging
import math
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from PIL import Image

_CACHE: dict = {}
_FILES = {
    "hed": ["ControlNetHED.pth", "hed.safetensors"],
    "pidinet": ["table5_pidinet.pth", "pidinet.safetensors"],
    "lineart": ["sk_model.pth", "lineart.safetensors"],
    "lineart_coarse": ["sk_model2.pth", "lineart_coarse.safetensors"],
    "mlsd": ["mlsd_large_512_fp32.pth", "mlsd.safetensors"],
    "depth": ["dpt-large.safetensors", "dpt-large/model.safetensors"],
    "seg": ["upernet-convnext-small.safetensors", "upernet-convnext-small/model.safetensors"],
    "openpose": ["body_pose_model.pth", "openpose.safetensors"],
    "normalbae": ["scannet.pt", "normalbae.safetensors"],
}


def annotator_dir() -> str:
    d = os.environ.get("CSK_ANNOTATOR_DIR")
    if d:
        return d
    from ..settings import get_settings_dir

    return os.path.join(get_settings_dir(), "annotators")


def _device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


def load_checkpoint(path: str) -> dict:
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return load_file(path, device="cpu")
    sd = torch.load(path, map_location="cpu", weights_only=True)  # never unpickles code
    for key in ("state_dict", "model"):  # scannet.pt nests its weights under "model"
        if isinstance(sd, dict) and key in sd and isinstance(sd[key], dict):
            sd = sd[key]
    return {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}


def _build(name: str, ctor):
    """Resident detector ``name``: constructed, weights loaded if present, on device."""
    m = _CACHE.get(name)
    if m is not None:
        return m
    torch.manual_seed(1234)
    m = ctor().eval().requires_grad_(False)
    src = "random-init"
    for f in _FILES.get(name, []):
        p = os.path.join(annotator_dir(), f)
        if os.path.exists(p):
            sd = load_checkpoint(p)
            missing, unexpected = m.load_state_dict(sd, strict=False)
            if len(missing) < len(m.state_dict()) // 2:
                src = p
            break
    if src == "random-init":
        logging.warning(f"annotator '{name}': no weights in {annotator_dir()} -> random init")
    dev = _device()
    m = m.to(dev, torch.bfloat16 if dev.type == "cuda" else torch.float32)
    m.weights_source = src
    _CACHE[name] = m
    return m


def _to_tensor(img: np.ndarray, m: nn.Module) -> torch.Tensor:
    p = next(m.parameters())
    return torch.from_numpy(np.ascontiguousarray(img)).to(p.device).permute(2, 0, 1)[None].to(p.dtype)


def _hwc3(a: np.ndarray) -> np.ndarray:
    if a.ndim == 2:
        a = a[:, :, None]
    if a.shape[2] == 1:
        a = np.concatenate([a] * 3, axis=2)
    return a


def _resize_short(img: Image.Image, res: int, mult: int = 64) -> Image.Image:
    """controlnet_aux resize_image: short side -> res, both sides multiples of 64."""
    w, h = img.size
    k = float(res) / min(h, w)
    return img.resize((int(round(w * k / mult)) * mult, int(round(h * k / mult)) * mult), Image.Resampling.LANCZOS)


# ---------------------------------------------------------------------------
# HED (ControlNetHED_Apache2)
# ---------------------------------------------------------------------------
class DoubleConvBlock(nn.Module):
    def __init__(self, cin, cout, n):
        super().__init__()
        self.convs = nn.ModuleList([nn.Conv2d(cin if i == 0 else cout, cout, 3, padding=1) for i in range(n)])
        self.projection = nn.Conv2d(cout, 1, 1)

    def forward(self, x, down_sampling=False):
        h = F.max_pool2d(x, 2, 2) if down_sampling else x
        for c in self.convs:
            h = F.relu(c(h))
        return h, self.projection(h)


class ControlNetHED(nn.Module):
    def __init__(self):
        super().__init__()
        self.norm = nn.Parameter(torch.zeros(1, 3, 1, 1))
        self.block1 = DoubleConvBlock(3, 64, 2)
        self.block2 = DoubleConvBlock(64, 128, 2)
        self.block3 = DoubleConvBlock(128, 256, 3)
        self.block4 = DoubleConvBlock(256, 512, 3)
        self.block5 = DoubleConvBlock(512, 512, 3)

    def forward(self, x):
        h = x - self.norm
        outs = []
        for i, b in enumerate([self.block1, self.block2, self.block3, self.block4, self.block5]):
            h, p = b(h, down_sampling=i > 0)
            outs.append(p)
        return outs


def _nms(x: np.ndarray, t: float, s: float) -> np.ndarray:
    """controlnet_aux nms: directional line maxima of a blurred edge map."""
    from scipy import ndimage

    x = ndimage.gaussian_filter(x.astype(np.float32), sigma=s)
    f1 = np.array([[0, 0, 0], [1, 1, 1], [0, 0, 0]], dtype=bool)
    f2 = np.array([[0, 1, 0], [0, 1, 0], [0, 1, 0]], dtype=bool)
    f3 = np.eye(3, dtype=bool)
    f4 = np.fliplr(np.eye(3, dtype=bool))
    y = np.zeros_like(x)
    for f in (f1, f2, f3, f4):
        np.putmask(y, ndimage.grey_dilation(x, footprint=f) == x, x)
    z = np.zeros_like(y, dtype=np.uint8)
    z[y > t] = 255
    return z


@torch.no_grad()
def hed(image: Image.Image, scribble=False, res=512) -> Image.Image:
    from scipy import ndimage

    m = _build("hed", ControlNetHED)
    img = np.asarray(_resize_short(image.convert("RGB"), res)).astype(np.float32)
    H, W = img.shape[:2]
    edges = m(_to_tensor(img, m))
    edges = [F.interpolate(e.float(), size=(H, W), mode="bilinear", align_corners=False)[0, 0] for e in edges]
    edge = torch.sigmoid(torch.stack(edges, 0).mean(0)).cpu().numpy()
    out = (edge * 255.0).clip(0, 255).astype(np.uint8)
    if scribble:
        out = _nms(out, 127, 3.0)
        out = ndimage.gaussian_filter(out.astype(np.float32), sigma=3.0)
        out = np.where(out > 4, 255, 0).astype(np.uint8)
    return Image.fromarray(_hwc3(out)).resize(image.size, Image.Resampling.BILINEAR)


# ---------------------------------------------------------------------------
# PiDiNet (pixel-difference network, table5_pidinet.pth: inplane 60, carv4, dil 24, sa)
# ---------------------------------------------------------------------------
_AD_PERM = [3, 0, 1, 6, 4, 2, 7, 8, 5]  # clockwise neighbour of each 3x3 tap
_RD_OUTER = [0, 2, 4, 10, 14, 20, 22, 24]  # 5x5 taps two pixels out along the 8 directions
_RD_INNER = [6, 7, 8, 11, 13, 16, 17, 18]  # ... and one pixel out


class PDConv(nn.Module):
    """A pixel-difference convolution stored as its raw 3x3 weight (checkpoint
    layout) and run as the equivalent plain convolution: 'cd' central
    differences fold into the centre tap, 'ad' angular differences into a
    rotated copy, 'rd' radial differences into a 5x5 kernel; 'cv' is vanilla."""

    def __init__(self, kind, cin, cout, groups=1):
        super().__init__()
        self.kind, self.groups = kind, groups
        self.weight = nn.Parameter(torch.empty(cout, cin // groups, 3, 3))
        nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))

    def effective(self):
        w = self.weight
        o, i = w.shape[:2]
        if self.kind == "cd":
            return w - F.pad(w.sum((2, 3), keepdim=True), (1, 1, 1, 1)), 1
        if self.kind == "ad":
            f = w.reshape(o, i, 9)
            return (f - f[:, :, _AD_PERM]).reshape(o, i, 3, 3), 1
        if self.kind == "rd":
            f = w.reshape(o, i, 9)[:, :, 1:]
            b = w.new_zeros(o, i, 25)
            b[:, :, _RD_OUTER] = f
            b[:, :, _RD_INNER] = -f
            return b.reshape(o, i, 5, 5), 2
        return w, 1

    def forward(self, x):
        w, pad = self.effective()
        return F.conv2d(x, w, None, 1, pad, 1, self.groups)


class PDCBlock(nn.Module):
    def __init__(self, kind, cin, cout, stride=1):
        super().__init__()
        self.stride = stride
        if stride > 1:
            self.shortcut = nn.Conv2d(cin, cout, 1)
        self.conv1 = PDConv(kind, cin, cin, groups=cin)
        self.conv2 = nn.Conv2d(cin, cout, 1, bias=False)

    def forward(self, x):
        if self.stride > 1:
            x = F.max_pool2d(x, 2, 2)
        y = self.conv2(F.relu(self.conv1(x)))
        return y + (self.shortcut(x) if self.stride > 1 else x)


class _CDCM(nn.Module):
    """Compact dilation convolution module: 1x1 then four dilated 3x3s, summed."""

    def __init__(self, cin, c):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, c, 1)
        for j, d in enumerate((5, 7, 9, 11)):
            setattr(self, f"conv2_{j + 1}", nn.Conv2d(c, c, 3, padding=d, dilation=d, bias=False))

    def forward(self, x):
        x = self.conv1(F.relu(x))
        return self.conv2_1(x) + self.conv2_2(x) + self.conv2_3(x) + self.conv2_4(x)


class _CSAM(nn.Module):
    """Compact spatial attention: a sigmoid gate from 1x1 (to 4) + 3x3 (to 1)."""

    def __init__(self, c):
        super().__init__()
        self.conv1 = nn.Conv2d(c, 4, 1)
        self.conv2 = nn.Conv2d(4, 1, 3, padding=1, bias=False)

    def forward(self, x):
        return x * torch.sigmoid(self.conv2(self.conv1(F.relu(x))))


class _MapReduce(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, 1, 1)

    def forward(self, x):
        return self.conv(x)


class PiDiNet(nn.Module):
    """Four stages of pixel-difference blocks (C, 2C, 4C, 4C channels), per-stage
    CDCM + CSAM + 1-channel side output upsampled to full size, fused by a
    1x1 classifier; returns the sigmoid side maps and the fused map last."""

    def __init__(self, inplane=60, pdcs=("cd", "ad", "rd", "cv") * 4, dil=24):
        super().__init__()
        self.init_block = PDConv(pdcs[0], 3, inplane)
        planes = [inplane, 2 * inplane, 4 * inplane, 4 * inplane]
        cin, idx = inplane, 1
        for s in range(4):
            for j in range(4 if s else 3):
                stride = 2 if (s and j == 0) else 1
                setattr(self, f"block{s + 1}_{j + 1}", PDCBlock(pdcs[idx], cin, planes[s], stride))
                cin, idx = planes[s], idx + 1
        self.dilations = nn.ModuleList([_CDCM(p, dil) for p in planes])
        self.attentions = nn.ModuleList([_CSAM(dil) for _ in planes])
        self.conv_reduces = nn.ModuleList([_MapReduce(dil) for _ in planes])
        self.classifier = nn.Conv2d(4, 1, 1)

    def stage_blocks(self, s):
        return [getattr(self, f"block{s + 1}_{j + 1}") for j in range(4 if s else 3)]

    def forward(self, x):
        H, W = x.shape[2:]
        h = self.init_block(x)
        side = []
        for s in range(4):
            for b in self.stage_blocks(s):
                h = b(h)
            e = self.conv_reduces[s](self.attentions[s](self.dilations[s](h)))
            side.append(F.interpolate(e, size=(H, W), mode="bilinear", align_corners=False))
        side.append(self.classifier(torch.cat(side, 1)))
        return [torch.sigmoid(e) for e in side]


@torch.no_grad()
def pidinet(image: Image.Image, res=512, apply_filter=False) -> Image.Image:
    """controlnet_aux PidiNetDetector: BGR in [0, 1], fused (last) map x 255."""
    m = _build("pidinet", PiDiNet)
    img = np.asarray(_resize_short(image.convert("RGB"), res))[:, :, ::-1].astype(np.float32) / 255.0
    edge = m(_to_tensor(img, m))[-1][0, 0].float().cpu().numpy()
    if apply_filter:
        edge = (edge > 0.5).astype(np.float32)
    out = (edge * 255.0).clip(0, 255).astype(np.uint8)
    return Image.fromarray(_hwc3(out)).resize(image.size, Image.Resampling.BILINEAR)


# ---------------------------------------------------------------------------
# Lineart ("informative drawings" generator)
# ---------------------------------------------------------------------------
class ResidualBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv_block = nn.Sequential(nn.ReflectionPad2d(1), nn.Conv2d(c, c, 3), nn.InstanceNorm2d(c), nn.ReLU(True),
                                        nn.ReflectionPad2d(1), nn.Conv2d(c, c, 3), nn.InstanceNorm2d(c))

    def forward(self, x):
        return x + self.conv_block(x)


class LineartGenerator(nn.Module):
    def __init__(self, input_nc=3, output_nc=1, n_residual_blocks=3):
        super().__init__()
        self.model0 = nn.Sequential(nn.ReflectionPad2d(3), nn.Conv2d(input_nc, 64, 7), nn.InstanceNorm2d(64),
                                    nn.ReLU(True))
        down, c = [], 64
        for _ in range(2):
            down += [nn.Conv2d(c, c * 2, 3, stride=2, padding=1), nn.InstanceNorm2d(c * 2), nn.ReLU(True)]
            c *= 2
        self.model1 = nn.Sequential(*down)
        self.model2 = nn.Sequential(*[ResidualBlock(c) for _ in range(n_residual_blocks)])
        up = []
        for _ in range(2):
            up += [nn.ConvTranspose2d(c, c // 2, 3, stride=2, padding=1, output_padding=1), nn.InstanceNorm2d(c // 2),
                   nn.ReLU(True)]
            c //= 2
        self.model3 = nn.Sequential(*up)
        self.model4 = nn.Sequential(nn.ReflectionPad2d(3), nn.Conv2d(64, output_nc, 7), nn.Sigmoid())

    def forward(self, x):
        return self.model4(self.model3(self.model2(self.model1(self.model0(x)))))


@torch.no_grad()
def lineart(image: Image.Image, coarse=False, res=512) -> Image.Image:
    m = _build("lineart_coarse" if coarse else "lineart", LineartGenerator)
    img = np.asarray(_resize_short(image.convert("RGB"), res)).astype(np.float32) / 255.0
    line = m(_to_tensor(img, m))[0, 0].float().cpu().numpy()
    line = (line * 255.0).clip(0, 255).astype(np.uint8)
    out = Image.fromarray(_hwc3(line)).resize(image.size, Image.Resampling.BILINEAR)
    return Image.fromarray(255 - np.asarray(out))  # white lines on black, as ControlNet-lineart expects


# ---------------------------------------------------------------------------
# M-LSD (MobileV2_MLSD_Large) line segments
# ---------------------------------------------------------------------------
def _make_divisible(v, divisor=8):
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    return new_v + divisor if new_v < 0.9 * v else new_v


class ConvBNReLU(nn.Sequential):
    """TFLite-style padding: stride-2 convs pad (0, 1, 0, 1) and use padding 0."""

    def __init__(self, cin, cout, kernel_size=3, stride=1, groups=1):
        pad = 0 if stride == 2 else (kernel_size - 1) // 2
        super().__init__(nn.Conv2d(cin, cout, kernel_size, stride, pad, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU6(inplace=True))
        self.stride = stride

    def forward(self, x):
        if self.stride == 2:
            x = F.pad(x, (0, 1, 0, 1))
        for mod in self:
            x = mod(x)
        return x


class InvertedResidual(nn.Module):
    def __init__(self, inp, oup, stride, expand_ratio):
        super().__init__()
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers = [ConvBNReLU(inp, hidden, kernel_size=1)] if expand_ratio != 1 else []
        layers += [ConvBNReLU(hidden, hidden, stride=stride, groups=hidden), nn.Conv2d(hidden, oup, 1, 1, 0, bias=False),
                   nn.BatchNorm2d(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res_connect else self.conv(x)


class MobileNetV2Trunk(nn.Module):
    """MobileNetV2 up to the 96-channel stage; 4 input channels (RGB + ones)."""

    def __init__(self):
        super().__init__()
        cin = _make_divisible(32)
        feats = [ConvBNReLU(4, cin, stride=2)]
        for t, c, n, s in [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1]]:
            cout = _make_divisible(c)
            for i in range(n):
                feats.append(InvertedResidual(cin, cout, s if i == 0 else 1, t))
                cin = cout
        self.features = nn.Sequential(*feats)
        self.fpn_selected = [1, 3, 6, 10, 13]

    def forward(self, x):
        outs = []
        for i, f in enumerate(self.features):
            if i > self.fpn_selected[-1]:
                break
            x = f(x)
            if i in self.fpn_selected:
                outs.append(x)
        return outs


def _cbr(cin, cout, k=1, pad=0, dil=1, relu=True):
    return nn.Sequential(nn.Conv2d(cin, cout, k, padding=pad, dilation=dil), nn.BatchNorm2d(cout),
                         nn.ReLU(inplace=True) if relu else nn.Identity())


class BlockTypeA(nn.Module):
    def __init__(self, in_c1, in_c2, out_c1, out_c2, upscale=True):
        super().__init__()
        self.conv1 = _cbr(in_c2, out_c2)
        self.conv2 = _cbr(in_c1, out_c1)
        self.upscale = upscale

    def forward(self, a, b):
        b = self.conv1(b)
        a = self.conv2(a)
        if self.upscale:
            b = F.interpolate(b, scale_factor=2.0, mode="bilinear", align_corners=True)
        return torch.cat((a, b), dim=1)


class BlockTypeB(nn.Module):
    def __init__(self, in_c, out_c):
        super().__init__()
        self.conv1 = _cbr(in_c, in_c, 3, 1)
        self.conv2 = _cbr(in_c, out_c, 3, 1)

    def forward(self, x):
        return self.conv2(self.conv1(x) + x)


class BlockTypeC(nn.Module):
    def __init__(self, in_c, out_c):
        super().__init__()
        self.conv1 = _cbr(in_c, in_c, 3, 5, 5)
        self.conv2 = _cbr(in_c, in_c, 3, 1)
        self.conv3 = nn.Conv2d(in_c, out_c, 1)

    def forward(self, x):
        return self.conv3(self.conv2(self.conv1(x)))


class MLSDLarge(nn.Module):
    def __init__(self):
        super().__init__()
        self.backbone = MobileNetV2Trunk()
        self.block15 = BlockTypeA(64, 96, 64, 64, upscale=False)
        self.block16 = BlockTypeB(128, 64)
        self.block17 = BlockTypeA(32, 64, 64, 64)
        self.block18 = BlockTypeB(128, 64)
        self.block19 = BlockTypeA(24, 64, 64, 64)
        self.block20 = BlockTypeB(128, 64)
        self.block21 = BlockTypeA(16, 64, 64, 64)
        self.block22 = BlockTypeB(128, 64)
        self.block23 = BlockTypeC(64, 16)

    def forward(self, x):
        c1, c2, c3, c4, c5 = self.backbone(x)
        x = self.block16(self.block15(c4, c5))
        x = self.block18(self.block17(c3, x))
        x = self.block20(self.block19(c2, x))
        x = self.block22(self.block21(c1, x))
        return self.block23(x)[:, 7:]


def _draw_line(img: np.ndarray, p0, p1):
    n = int(max(abs(p1[0] - p0[0]), abs(p1[1] - p0[1]))) + 1
    xs = np.rint(np.linspace(p0[0], p1[0], n)).astype(int)
    ys = np.rint(np.linspace(p0[1], p1[1], n)).astype(int)
    ok = (xs >= 0) & (xs < img.shape[1]) & (ys >= 0) & (ys < img.shape[0])
    img[ys[ok], xs[ok]] = 255


@torch.no_grad()
def mlsd(image: Image.Image, thr_v=0.1, thr_d=0.1, res=512, topk=200, ksize=3) -> Image.Image:
    m = _build("mlsd", MLSDLarge)
    img = np.asarray(_resize_short(image.convert("RGB"), res)).astype(np.float32)
    H, W = img.shape[:2]
    x = np.concatenate([img, np.ones((H, W, 1), np.float32)], -1) / 127.5 - 1.0
    tp = m(_to_tensor(x, m)).float()
    disp = tp[0, 1:5]
    heat = torch.sigmoid(tp[:, 0])
    hmax = F.max_pool2d(heat, ksize, stride=1, padding=(ksize - 1) // 2)
    heat = (heat * (hmax == heat).float()).reshape(-1)
    scores, idx = torch.topk(heat, min(topk, heat.numel()))
    h, w = tp.shape[2], tp.shape[3]
    yy, xx = (idx // w).cpu().numpy(), (idx % w).cpu().numpy()
    scores, disp = scores.cpu().numpy(), disp.permute(1, 2, 0).cpu().numpy()
    dist = np.sqrt(((disp[..., :2] - disp[..., 2:]) ** 2).sum(-1))
    out = np.zeros((H, W), np.uint8)
    for y, x_, sc in zip(yy, xx, scores):
        if sc > thr_v and dist[y, x_] > thr_d:
            dx0, dy0, dx1, dy1 = disp[y, x_]
            # the map is at half resolution: x2 back to the detect resolution
            _draw_line(out, (2 * (x_ + dx0), 2 * (y + dy0)), (2 * (x_ + dx1), 2 * (y + dy1)))
    return Image.fromarray(_hwc3(out)).resize(image.size, Image.Resampling.NEAREST)


# ---------------------------------------------------------------------------
# DPT-Large depth (transformers DPTForDepthEstimation, Intel/dpt-large)
# ---------------------------------------------------------------------------
class _Lin(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.dense = nn.Linear(cin, cout)


class _ViTSelfAttn(nn.Module):
    def __init__(self, c, heads):
        super().__init__()
        self.query, self.key, self.value = nn.Linear(c, c), nn.Linear(c, c), nn.Linear(c, c)
        self.heads = heads

    def forward(self, x):
        b, s, c = x.shape
        q, k, v = (t(x).view(b, s, self.heads, -1).transpose(1, 2) for t in (self.query, self.key, self.value))
        return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, s, c)


class _ViTAttention(nn.Module):
    def __init__(self, c, heads):
        super().__init__()
        self.attention = _ViTSelfAttn(c, heads)
        self.output = _Lin(c, c)


class _ViTLayer(nn.Module):
    def __init__(self, c, heads, mlp):
        super().__init__()
        self.attention = _ViTAttention(c, heads)
        self.intermediate = _Lin(c, mlp)
        self.output = _Lin(mlp, c)
        self.layernorm_before = nn.LayerNorm(c, eps=1e-12)
        self.layernorm_after = nn.LayerNorm(c, eps=1e-12)

    def forward(self, x):
        x = x + self.attention.output.dense(self.attention.attention(self.layernorm_before(x)))
        return x + self.output.dense(F.gelu(self.intermediate.dense(self.layernorm_after(x))))


class _PatchEmb(nn.Module):
    def __init__(self, c, patch):
        super().__init__()
        self.projection = nn.Conv2d(3, c, patch, stride=patch)


class _DPTEmbeddings(nn.Module):
    def __init__(self, c, patch, image):
        super().__init__()
        self.cls_token = nn.Parameter(torch.zeros(1, 1, c))
        self.position_embeddings = nn.Parameter(torch.randn(1, (image // patch) ** 2 + 1, c) * 0.02)
        self.patch_embeddings = _PatchEmb(c, patch)
        self.patch = patch

    def forward(self, x):
        b, _, h, w = x.shape
        t = self.patch_embeddings.projection(x).flatten(2).transpose(1, 2)
        pos = self.position_embeddings
        n0 = int(math.sqrt(pos.shape[1] - 1))
        gh, gw = h // self.patch, w // self.patch
        if (gh, gw) != (n0, n0):  # bilinear resize of the grid (DPT _resize_pos_embed)
            grid = pos[:, 1:].reshape(1, n0, n0, -1).permute(0, 3, 1, 2).float()
            grid = F.interpolate(grid, size=(gh, gw), mode="bilinear").to(pos.dtype)
            pos = torch.cat([pos[:, :1], grid.permute(0, 2, 3, 1).reshape(1, gh * gw, -1)], 1)
        return torch.cat([self.cls_token.expand(b, -1, -1), t], 1) + pos


class _DPTEncoder(nn.Module):
    def __init__(self, c, heads, mlp, n):
        super().__init__()
        self.layer = nn.ModuleList([_ViTLayer(c, heads, mlp) for _ in range(n)])


class _DPTViT(nn.Module):
    def __init__(self, c=1024, heads=16, mlp=4096, n=24, patch=16, image=384):
        super().__init__()
        self.embeddings = _DPTEmbeddings(c, patch, image)
        self.encoder = _DPTEncoder(c, heads, mlp, n)


class _Reassemble(nn.Module):
    def __init__(self, c, out, factor):
        super().__init__()
        self.projection = nn.Conv2d(c, out, 1)
        if factor > 1:
            self.resize = nn.ConvTranspose2d(out, out, factor, stride=factor)
        elif factor == 1:
            self.resize = nn.Identity()
        else:
            self.resize = nn.Conv2d(out, out, 3, stride=int(1 / factor), padding=1)

    def forward(self, x):
        return self.resize(self.projection(x))


class _ReassembleStage(nn.Module):
    def __init__(self, c, sizes, factors):
        super().__init__()
        self.layers = nn.ModuleList([_Reassemble(c, s, f) for s, f in zip(sizes, factors)])
        self.readout_projects = nn.ModuleList([nn.Sequential(nn.Linear(2 * c, c), nn.GELU()) for _ in sizes])

    def forward(self, hs, gh, gw):
        out = []
        for i, h in enumerate(hs):
            cls, tok = h[:, :1], h[:, 1:]
            tok = self.readout_projects[i](torch.cat([tok, cls.expand_as(tok)], -1))
            tok = tok.transpose(1, 2).reshape(h.shape[0], -1, gh, gw)
            out.append(self.layers[i](tok))
        return out


class _PreActRes(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.convolution1 = nn.Conv2d(c, c, 3, padding=1)
        self.convolution2 = nn.Conv2d(c, c, 3, padding=1)

    def forward(self, x):
        return x + self.convolution2(F.relu(self.convolution1(F.relu(x))))


class _Fusion(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.projection = nn.Conv2d(c, c, 1)
        self.residual_layer1 = _PreActRes(c)
        self.residual_layer2 = _PreActRes(c)

    def forward(self, x, residual=None):
        if residual is not None:
            if residual.shape != x.shape:
                residual = F.interpolate(residual, size=x.shape[2:], mode="bilinear", align_corners=False)
            x = x + self.residual_layer1(residual)
        x = self.residual_layer2(x)
        x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=True)
        return self.projection(x)


class _FusionStage(nn.Module):
    def __init__(self, c, n):
        super().__init__()
        self.layers = nn.ModuleList([_Fusion(c) for _ in range(n)])


class _DPTNeck(nn.Module):
    def __init__(self, c, sizes=(256, 512, 1024, 1024), factors=(4, 2, 1, 0.5), fusion=256):
        super().__init__()
        self.reassemble_stage = _ReassembleStage(c, sizes, factors)
        self.convs = nn.ModuleList([nn.Conv2d(s, fusion, 3, padding=1, bias=False) for s in sizes])
        self.fusion_stage = _FusionStage(fusion, len(sizes))

    def forward(self, hs, gh, gw):
        feats = [conv(f) for conv, f in zip(self.convs, self.reassemble_stage(hs, gh, gw))]
        fused = None
        for f, layer in zip(feats[::-1], self.fusion_stage.layers):
            fused = layer(f) if fused is None else layer(fused, f)
        return fused


class _DPTHead(nn.Module):
    def __init__(self, c=256):
        super().__init__()
        self.head = nn.Sequential(nn.Conv2d(c, c // 2, 3, padding=1),
                                  nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True),
                                  nn.Conv2d(c // 2, 32, 3, padding=1), nn.ReLU(), nn.Conv2d(32, 1, 1), nn.ReLU())


class DPTDepth(nn.Module):
    """Defaults are Intel/dpt-large (ViT-L/16 at 384, taps after layers 5/11/17/23)."""

    def __init__(self, c=1024, heads=16, mlp=4096, n=24, patch=16, image=384, out_indices=(5, 11, 17, 23),
                 neck_sizes=(256, 512, 1024, 1024), factors=(4, 2, 1, 0.5), fusion=256):
        super().__init__()
        self.out_indices, self.patch = tuple(out_indices), patch
        self.dpt = _DPTViT(c, heads, mlp, n, patch, image)
        self.neck = _DPTNeck(c, neck_sizes, factors, fusion)
        self.head = _DPTHead(fusion)

    def forward(self, x):
        h = self.dpt.embeddings(x)
        hs = []
        for i, layer in enumerate(self.dpt.encoder.layer):
            h = layer(h)
            if i in self.out_indices:
                hs.append(h)
        gh, gw = x.shape[2] // self.patch, x.shape[3] // self.patch
        return self.head.head(self.neck(hs, gh, gw))[:, 0]


@torch.no_grad()
def depth(image: Image.Image, size=384) -> Image.Image:
    m = _build("depth", DPTDepth)
    img = np.asarray(image.convert("RGB").resize((size, size), Image.Resampling.BICUBIC)).astype(np.float32)
    x = (img / 255.0 - 0.5) / 0.5
    pred = m(_to_tensor(x, m)).float()
    pred = F.interpolate(pred[:, None], size=(image.size[1], image.size[0]), mode="bicubic", align_corners=False)
    d = pred[0, 0].cpu().numpy()
    mx = float(d.max())
    out = (d * 255.0 / mx).clip(0, 255).astype(np.uint8) if mx > 0 else np.zeros_like(d, np.uint8)
    return Image.fromarray(out).convert("RGB")


# ---------------------------------------------------------------------------
# UperNet + ConvNeXt (transformers UperNetForSemanticSegmentation,
# openmmlab/upernet-convnext-small), ADE20K classes
# ---------------------------------------------------------------------------
class _LNcf(nn.Module):
    """LayerNorm over channels of an NCHW map (ConvNeXt "channels_first")."""

    def __init__(self, c, eps=1e-6):
        super().__init__()
        self.weight, self.bias, self.eps = nn.Parameter(torch.ones(c)), nn.Parameter(torch.zeros(c)), eps

    def forward(self, x):
        return F.layer_norm(x.permute(0, 2, 3, 1), x.shape[1:2], self.weight, self.bias, self.eps).permute(0, 3, 1, 2)


class _CNBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dwconv = nn.Conv2d(c, c, 7, padding=3, groups=c)
        self.layernorm = nn.LayerNorm(c, eps=1e-6)
        self.pwconv1 = nn.Linear(c, 4 * c)
        self.pwconv2 = nn.Linear(4 * c, c)
        self.layer_scale_parameter = nn.Parameter(torch.full((c,), 1e-6))

    def forward(self, x):
        h = self.dwconv(x).permute(0, 2, 3, 1)
        h = self.pwconv2(F.gelu(self.pwconv1(self.layernorm(h)))) * self.layer_scale_parameter
        return x + h.permute(0, 3, 1, 2)


class _CNStage(nn.Module):
    def __init__(self, cin, c, depth, down):
        super().__init__()
        self.downsampling_layer = nn.Sequential(_LNcf(cin), nn.Conv2d(cin, c, 2, stride=2)) if down else nn.Identity()
        self.layers = nn.Sequential(*[_CNBlock(c) for _ in range(depth)])

    def forward(self, x):
        return self.layers(self.downsampling_layer(x))


class _CNEmb(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.patch_embeddings = nn.Conv2d(3, c, 4, stride=4)
        self.layernorm = _LNcf(c)


class _CNEncoder(nn.Module):
    def __init__(self, dims, depths):
        super().__init__()
        self.stages = nn.ModuleList([_CNStage(dims[max(i - 1, 0)], dims[i], depths[i], i > 0) for i in range(4)])


class ConvNextBackbone(nn.Module):
    def __init__(self, dims=(96, 192, 384, 768), depths=(3, 3, 27, 3)):
        super().__init__()
        self.embeddings = _CNEmb(dims[0])
        self.encoder = _CNEncoder(dims, depths)
        self.hidden_states_norms = nn.ModuleDict({f"stage{i + 1}": _LNcf(d) for i, d in enumerate(dims)})

    def forward(self, x):
        h = self.embeddings.layernorm(self.embeddings.patch_embeddings(x))
        outs = []
        for i, st in enumerate(self.encoder.stages):
            h = st(h)
            outs.append(self.hidden_states_norms[f"stage{i + 1}"](h))
        return outs


class _ConvModule(nn.Module):
    def __init__(self, cin, cout, k=1, pad=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, padding=pad, bias=False)
        self.batch_norm = nn.BatchNorm2d(cout)

    def forward(self, x):
        return F.relu(self.batch_norm(self.conv(x)))


class _PPMStage(nn.Sequential):
    """Pool + 1x1 ConvModule; children named "0"/"1" (psp_modules.<i>.1.conv.weight)."""

    def __init__(self, scale, cin, c):
        super().__init__(nn.AdaptiveAvgPool2d(scale), _ConvModule(cin, c))


class UperHead(nn.Module):
    def __init__(self, in_channels=(96, 192, 384, 768), c=512, num_classes=150, scales=(1, 2, 3, 6)):
        super().__init__()
        self.psp_modules = nn.ModuleList([_PPMStage(s, in_channels[-1], c) for s in scales])
        self.bottleneck = _ConvModule(in_channels[-1] + len(scales) * c, c, 3, 1)
        self.lateral_convs = nn.ModuleList([_ConvModule(ci, c) for ci in in_channels[:-1]])
        self.fpn_convs = nn.ModuleList([_ConvModule(c, c, 3, 1) for _ in in_channels[:-1]])
        self.fpn_bottleneck = _ConvModule(len(in_channels) * c, c, 3, 1)
        self.classifier = nn.Conv2d(c, num_classes, 1)

    def forward(self, feats):
        x = feats[-1]
        psp = [x] + [F.interpolate(p(x), size=x.shape[2:], mode="bilinear", align_corners=False) for p in self.psp_modules]
        lat = [conv(f) for conv, f in zip(self.lateral_convs, feats)] + [self.bottleneck(torch.cat(psp, 1))]
        for i in range(len(lat) - 1, 0, -1):
            lat[i - 1] = lat[i - 1] + F.interpolate(lat[i], size=lat[i - 1].shape[2:], mode="bilinear",
                                                    align_corners=False)
        outs = [conv(lat[i]) for i, conv in enumerate(self.fpn_convs)] + [lat[-1]]
        outs = [outs[0]] + [F.interpolate(o, size=outs[0].shape[2:], mode="bilinear", align_corners=False)
                            for o in outs[1:]]
        return self.classifier(self.fpn_bottleneck(torch.cat(outs, 1)))


class UperNetConvNext(nn.Module):
    """Defaults are openmmlab/upernet-convnext-small (ADE20K, 150 classes)."""

    def __init__(self, dims=(96, 192, 384, 768), depths=(3, 3, 27, 3), c=512, num_classes=150, scales=(1, 2, 3, 6)):
        super().__init__()
        self.backbone = ConvNextBackbone(dims, depths)
        self.decode_head = UperHead(tuple(dims), c, num_classes, scales)

    def forward(self, x):
        return self.decode_head(self.backbone(x))


# ADE20K colour table used for ControlNet-seg conditioning images (data; the
# reference keeps the same 151 entries at swarm/controlnet/input_processor.py:118-272)
_ADE_HEX = (
    "000000787878b4787806e6e650323204c8037878508c8c8ccc05ffe6e6e604fa07e005ffebff0796053d78784608ff33"
    "ff06528fff8cccff04ff3307cc46030066c83de6faff06330b66ffff0747ff09e00907e6dcdcdcff095c7009ff08ffd6"
    "07ffe0ffb8060aff47ff290a07ffffe0ff086608ffff3d06ffc207ff7a0800ff14ff0829ff05990633ffeb0cffa09614"
    "00a3ff8c8c8cfa0a0f14ff001fff00ff1f00ffe00099ff000000ffff470000ebff00adff1f00ff0bc8c8ff520000fff5"
    "003dff00ff7000ff85ff0000ffa300ff6600c2ff00008fff33ff000052ff00ff2900ffad0a00ffadff0000ff99ff5c00"
    "ff00ffff00f5ff0066ffad00ff0014ffb8b8001fff00ff3d0047ffff00cc00ffc200ff52000aff0070ff3300ff00c2ff"
    "007aff00ffa3ff990000ff0aff70008fff005200ffa3ff00ffeb0008b8aa8500ff00ff5cb800ffff001f00b8ff00d6ff"
    "ff00705cff0000e0ff70e0ff46b8a0a300ff9900ff47ff00ff00a3ffcc00ff008f00ffeb85ff00ff00ebf500ffff007a"
    "fff5000abed4d6ff0000ccff1400ffffff000099ff0029ff00ffcc2900ff29ff00ad00ff00f5ff4700ff7a00ff00ffb8"
    "005cffb8ff000085ffffd60019c2c266ff005c00ff"
)
ADE_PALETTE = np.frombuffer(bytes.fromhex(_ADE_HEX), dtype=np.uint8).reshape(-1, 3)


@torch.no_grad()
def segmentation(image: Image.Image, res=512) -> Image.Image:
    m = _build("seg", UperNetConvNext)
    w, h = image.size
    k = res / min(w, h)
    rw, rh = max(32, int(round(w * k / 32)) * 32), max(32, int(round(h * k / 32)) * 32)
    img = np.asarray(image.convert("RGB").resize((rw, rh), Image.Resampling.BILINEAR)).astype(np.float32) / 255.0
    x = (img - np.array([0.485, 0.456, 0.406], np.float32)) / np.array([0.229, 0.224, 0.225], np.float32)
    logits = m(_to_tensor(x, m)).float()
    logits = F.interpolate(logits, size=(h, w), mode="bilinear", align_corners=False)
    seg = logits.argmax(1)[0].cpu().numpy()
    return Image.fromarray(ADE_PALETTE[np.clip(seg, 0, len(ADE_PALETTE) - 1)].astype(np.uint8))


# ---------------------------------------------------------------------------
# OpenPose body (CMU 18-keypoint model: VGG stem + 6 two-branch stages, PAF
# grouping) — the controlnet_aux OpenposeDetector default (body only)
# ---------------------------------------------------------------------------
def _openpose_stages():
    from collections import OrderedDict

    b0 = OrderedDict([("conv1_1", [3, 64, 3, 1, 1]), ("conv1_2", [64, 64, 3, 1, 1]), ("pool1_stage1", [2, 2, 0]),
                      ("conv2_1", [64, 128, 3, 1, 1]), ("conv2_2", [128, 128, 3, 1, 1]), ("pool2_stage1", [2, 2, 0]),
                      ("conv3_1", [128, 256, 3, 1, 1]), ("conv3_2", [256, 256, 3, 1, 1]),
                      ("conv3_3", [256, 256, 3, 1, 1]), ("conv3_4", [256, 256, 3, 1, 1]), ("pool3_stage1", [2, 2, 0]),
                      ("conv4_1", [256, 512, 3, 1, 1]), ("conv4_2", [512, 512, 3, 1, 1]),
                      ("conv4_3_CPM", [512, 256, 3, 1, 1]), ("conv4_4_CPM", [256, 128, 3, 1, 1])])
    blocks = {"model0": b0}
    for br, cout in ((1, 38), (2, 19)):
        blocks[f"model1_{br}"] = OrderedDict(
            [(f"conv5_{i}_CPM_L{br}", [128, 128, 3, 1, 1]) for i in (1, 2, 3)]
            + [(f"conv5_4_CPM_L{br}", [128, 512, 1, 1, 0]), (f"conv5_5_CPM_L{br}", [512, cout, 1, 1, 0])])
        for st in range(2, 7):
            blocks[f"model{st}_{br}"] = OrderedDict(
                [(f"Mconv1_stage{st}_L{br}", [185, 128, 7, 1, 3])]
                + [(f"Mconv{i}_stage{st}_L{br}", [128, 128, 7, 1, 3]) for i in (2, 3, 4, 5)]
                + [(f"Mconv6_stage{st}_L{br}", [128, 128, 1, 1, 0]), (f"Mconv7_stage{st}_L{br}", [128, cout, 1, 1, 0])])
    return blocks


def _make_layers(block):
    from collections import OrderedDict

    layers = []
    for name, v in block.items():
        if "pool" in name:
            layers.append((name, nn.MaxPool2d(v[0], v[1], v[2])))
        else:
            layers.append((name, nn.Conv2d(v[0], v[1], v[2], v[3], v[4])))
            if not (name.startswith("conv5_5") or name.startswith("Mconv7")):  # the output convs: no ReLU
                layers.append(("relu_" + name, nn.ReLU(inplace=True)))
    return nn.Sequential(OrderedDict(layers))


class BodyPoseModel(nn.Module):
    def __init__(self):
        super().__init__()
        for k, b in _openpose_stages().items():
            setattr(self, k, _make_layers(b))

    def forward(self, x):
        f = self.model0(x)
        paf, heat = self.model1_1(f), self.model1_2(f)
        for st in range(2, 7):
            h = torch.cat([paf, heat, f], 1)
            paf, heat = getattr(self, f"model{st}_1")(h), getattr(self, f"model{st}_2")(h)
        return paf, heat

    def load_state_dict(self, sd, strict=True):  # the published .pth keys lack the "modelX_Y." prefix
        own = self.state_dict()
        flat = {k.split(".", 1)[1]: k for k in own}
        remapped = {flat.get(k, k): v for k, v in sd.items()}
        return super().load_state_dict(remapped, strict=strict)


_LIMBS = [[2, 3], [2, 6], [3, 4], [4, 5], [6, 7], [7, 8], [2, 9], [9, 10], [10, 11], [2, 12], [12, 13], [13, 14],
          [2, 1], [1, 15], [15, 17], [1, 16], [16, 18], [3, 17], [6, 18]]
_PAF_IDX = [[31, 32], [39, 40], [33, 34], [35, 36], [41, 42], [43, 44], [19, 20], [21, 22], [23, 24], [25, 26],
            [27, 28], [29, 30], [47, 48], [49, 50], [53, 54], [51, 52], [55, 56], [37, 38], [45, 46]]
_POSE_COLORS = [[255, 0, 0], [255, 85, 0], [255, 170, 0], [255, 255, 0], [170, 255, 0], [85, 255, 0], [0, 255, 0],
                [0, 255, 85], [0, 255, 170], [0, 255, 255], [0, 170, 255], [0, 85, 255], [0, 0, 255], [85, 0, 255],
                [170, 0, 255], [255, 0, 255], [255, 0, 170], [255, 0, 85]]


def _pose_peaks(heat: np.ndarray, thre1=0.1):
    from scipy import ndimage

    peaks, pid = [], 0
    for part in range(18):
        m = heat[:, :, part]
        s = ndimage.gaussian_filter(m, sigma=3)
        c = s[1:-1, 1:-1]
        ok = ((c >= s[1:-1, :-2]) & (c >= s[1:-1, 2:]) & (c >= s[:-2, 1:-1]) & (c >= s[2:, 1:-1]) & (c > thre1))
        ys, xs = np.nonzero(ok)
        ys, xs = ys + 1, xs + 1
        peaks.append([(int(x), int(y), float(m[y, x]), pid + i) for i, (x, y) in enumerate(zip(xs, ys))])
        pid += len(xs)
    return peaks


def _pose_group(peaks, paf: np.ndarray, img_h: int, thre2=0.05, mid_num=10):
    """Part-affinity-field limb scoring + greedy person assembly (OpenPose)."""
    conns, special = [], []
    for k, (ia, ib) in enumerate(_LIMBS):
        score_mid = paf[:, :, [x - 19 for x in _PAF_IDX[k]]]
        ca, cb = peaks[ia - 1], peaks[ib - 1]
        if not ca or not cb:
            special.append(k)
            conns.append(np.zeros((0, 5)))
            continue
        cand = []
        for i, a in enumerate(ca):
            for j, b in enumerate(cb):
                vec = np.array([b[0] - a[0], b[1] - a[1]], np.float64)
                norm = max(0.001, float(np.hypot(*vec)))
                vec /= norm
                xs = np.rint(np.linspace(a[0], b[0], mid_num)).astype(int)
                ys = np.rint(np.linspace(a[1], b[1], mid_num)).astype(int)
                sc = score_mid[ys, xs, 0] * vec[0] + score_mid[ys, xs, 1] * vec[1]
                prior = sc.mean() + min(0.5 * img_h / norm - 1, 0)
                if (sc > thre2).sum() > 0.8 * len(sc) and prior > 0:
                    cand.append((i, j, prior, prior + a[2] + b[2]))
        cand.sort(key=lambda c: c[2], reverse=True)
        conn = np.zeros((0, 5))
        for i, j, s, _ in cand:
            if i not in conn[:, 3] and j not in conn[:, 4]:
                conn = np.vstack([conn, [ca[i][3], cb[j][3], s, i, j]])
                if len(conn) >= min(len(ca), len(cb)):
                    break
        conns.append(conn)
    cands = np.array([p for part in peaks for p in part], np.float64).reshape(-1, 4)
    subset = -np.ones((0, 20))
    for k, (ia, ib) in enumerate(_LIMBS):
        if k in special:
            continue
        A, B = ia - 1, ib - 1
        for c in conns[k]:
            pa, pb = c[0], c[1]
            found = [j for j in range(len(subset)) if subset[j][A] == pa or subset[j][B] == pb][:2]
            if len(found) == 1:
                j = found[0]
                if subset[j][B] != pb:
                    subset[j][B] = pb
                    subset[j][-1] += 1
                    subset[j][-2] += cands[int(pb), 2] + c[2]
            elif len(found) == 2:
                j1, j2 = found
                member = ((subset[j1] >= 0).astype(int) + (subset[j2] >= 0).astype(int))[:-2]
                if not (member == 2).any():
                    subset[j1][:-2] += subset[j2][:-2] + 1
                    subset[j1][-2:] += subset[j2][-2:]
                    subset[j1][-2] += c[2]
                    subset = np.delete(subset, j2, 0)
                else:
                    subset[j1][B] = pb
                    subset[j1][-1] += 1
                    subset[j1][-2] += cands[int(pb), 2] + c[2]
            elif k < 17:
                row = -np.ones(20)
                row[A], row[B] = pa, pb
                row[-1] = 2
                row[-2] = cands[[int(pa), int(pb)], 2].sum() + c[2]
                subset = np.vstack([subset, row])
    keep = [i for i in range(len(subset)) if subset[i][-1] >= 4 and subset[i][-2] / subset[i][-1] >= 0.4]
    return cands, subset[keep]


def _draw_pose(h, w, cands, subset):
    """Skeleton canvas: limbs as filled 4-px sticks, joints as 4-px discs (OpenPose colours)."""
    canvas = np.zeros((h, w, 3), np.float32)
    yy, xx = np.mgrid[0:h, 0:w]
    for k in range(17):
        for person in subset:
            idx = person[np.array(_LIMBS[k]) - 1]
            if (idx < 0).any():
                continue
            (x0, y0), (x1, y1) = cands[int(idx[0]), :2], cands[int(idx[1]), :2]
            d = np.array([x1 - x0, y1 - y0])
            L2 = max(float(d @ d), 1e-6)
            t = np.clip(((xx - x0) * d[0] + (yy - y0) * d[1]) / L2, 0, 1)
            dist2 = (xx - (x0 + t * d[0])) ** 2 + (yy - (y0 + t * d[1])) ** 2
            m = dist2 <= 16
            canvas[m] = canvas[m] * 0.4 + np.array(_POSE_COLORS[k], np.float32) * 0.6
    for part in range(18):
        for person in subset:
            i = int(person[part])
            if i < 0:
                continue
            x, y = cands[i, :2]
            m = (xx - x) ** 2 + (yy - y) ** 2 <= 16
            canvas[m] = _POSE_COLORS[part]
    return canvas.clip(0, 255).astype(np.uint8)


@torch.no_grad()
def openpose(image: Image.Image, res=512, boxsize=368, stride=8) -> Image.Image:
    m = _build("openpose", BodyPoseModel)
    img = np.asarray(_resize_short(image.convert("RGB"), res)).astype(np.float32)
    H, W = img.shape[:2]
    scale = boxsize / H
    sh, sw = max(stride, int(round(H * scale))), max(stride, int(round(W * scale)))
    test = np.asarray(Image.fromarray(img.astype(np.uint8)).resize((sw, sh), Image.Resampling.BICUBIC), np.float32)
    ph, pw = (-sh) % stride, (-sw) % stride
    test = np.pad(test, ((0, ph), (0, pw), (0, 0)), constant_values=128)
    x = test[:, :, ::-1] / 256.0 - 0.5  # BGR, as the model was trained
    paf, heat = m(_to_tensor(x, m))
    out = []
    for t in (heat, paf):
        t = F.interpolate(t.float(), scale_factor=stride, mode="bicubic", align_corners=False)[:, :, :sh, :sw]
        out.append(F.interpolate(t, size=(H, W), mode="bicubic", align_corners=False)[0].permute(1, 2, 0).cpu().numpy())
    heat_np, paf_np = out
    peaks = _pose_peaks(heat_np)
    cands, subset = _pose_group(peaks, paf_np, H)
    canvas = _draw_pose(H, W, cands, subset)
    return Image.fromarray(canvas).resize(image.size, Image.Resampling.BILINEAR)


# ---------------------------------------------------------------------------
# NormalBae (Bae et al. 2021 surface-normal net "NNET", the controlnet_aux
# NormalBaeDetector, checkpoint scannet.pt): EfficientNet-B5 (TF "same"
# padding, AP weights) encoder + UpSampleBN decoder, coarse-to-fine per-pixel
# MLP refinement at 1/4, 1/2 and 1/1 resolution.  In eval every pixel is
# refined (no uncertainty-guided point sampling, which only trains).
# ---------------------------------------------------------------------------
class _Conv2dSame(nn.Conv2d):
    """TF 'same' padding for strided convs (pad split low/high, extra on the high side)."""

    def forward(self, x):
        ih, iw = x.shape[-2:]
        kh, kw = self.weight.shape[-2:]
        sh, sw = self.stride
        ph = max((math.ceil(ih / sh) - 1) * sh + kh - ih, 0)
        pw = max((math.ceil(iw / sw) - 1) * sw + kw - iw, 0)
        if ph or pw:
            x = F.pad(x, [pw // 2, pw - pw // 2, ph // 2, ph - ph // 2])
        return F.conv2d(x, self.weight, self.bias, self.stride, 0, self.dilation, self.groups)


def _tf_conv(cin, cout, k, stride=1, groups=1, bias=False):
    if stride == 1:
        return nn.Conv2d(cin, cout, k, 1, k // 2, groups=groups, bias=bias)
    return _Conv2dSame(cin, cout, k, stride, 0, groups=groups, bias=bias)


def _bn_tf(c):
    return nn.BatchNorm2d(c, eps=1e-3)


class _SE(nn.Module):
    def __init__(self, c, rd):
        super().__init__()
        self.conv_reduce = nn.Conv2d(c, rd, 1)
        self.conv_expand = nn.Conv2d(rd, c, 1)

    def forward(self, x):
        s = F.silu(self.conv_reduce(x.mean((2, 3), keepdim=True)))
        return x * torch.sigmoid(self.conv_expand(s))


class _DSConv(nn.Module):
    """Depthwise-separable block (EfficientNet stage 0)."""

    def __init__(self, cin, cout, k):
        super().__init__()
        self.conv_dw, self.bn1 = _tf_conv(cin, cin, k, groups=cin), _bn_tf(cin)
        self.se = _SE(cin, max(1, int(cin * 0.25 + 0.5)))
        self.conv_pw, self.bn2 = nn.Conv2d(cin, cout, 1, bias=False), _bn_tf(cout)
        self.skip = cin == cout

    def forward(self, x):
        h = self.bn2(self.conv_pw(self.se(F.silu(self.bn1(self.conv_dw(x))))))
        return x + h if self.skip else h


class _IRBlock(nn.Module):
    """Inverted residual (MBConv) with squeeze-excite sized from the block input."""

    def __init__(self, cin, cout, k, stride, expand=6):
        super().__init__()
        mid = cin * expand
        self.conv_pw, self.bn1 = nn.Conv2d(cin, mid, 1, bias=False), _bn_tf(mid)
        self.conv_dw, self.bn2 = _tf_conv(mid, mid, k, stride, groups=mid), _bn_tf(mid)
        self.se = _SE(mid, max(1, int(cin * 0.25 + 0.5)))
        self.conv_pwl, self.bn3 = nn.Conv2d(mid, cout, 1, bias=False), _bn_tf(cout)
        self.skip = stride == 1 and cin == cout

    def forward(self, x):
        h = F.silu(self.bn1(self.conv_pw(x)))
        h = self.se(F.silu(self.bn2(self.conv_dw(h))))
        h = self.bn3(self.conv_pwl(h))
        return x + h if self.skip else h


class EfficientNetB5(nn.Module):
    """tf_efficientnet_b5_ap trunk (channel x1.6, depth x2.2); classifier removed."""

    # (kernel, stride, expand, channels, repeats) after width/depth scaling
    STAGES = ((3, 1, 1, 24, 3), (3, 2, 6, 40, 5), (5, 2, 6, 64, 5), (3, 2, 6, 128, 7), (5, 1, 6, 176, 7),
              (5, 2, 6, 304, 9), (3, 1, 6, 512, 3))

    def __init__(self, stem=48, head=2048):
        super().__init__()
        self.conv_stem, self.bn1 = _tf_conv(3, stem, 3, 2), _bn_tf(stem)
        stages, cin = [], stem
        for k, s, e, c, r in self.STAGES:
            blocks = []
            for i in range(r):
                blocks.append(_DSConv(cin, c, k) if e == 1 else _IRBlock(cin, c, k, s if i == 0 else 1, e))
                cin = c
            stages.append(nn.Sequential(*blocks))
        self.blocks = nn.Sequential(*stages)
        self.conv_head, self.bn2 = nn.Conv2d(cin, head, 1, bias=False), _bn_tf(head)

    def features(self, x):
        """The decoder's taps: stage 0/1/2/4 outputs and the (pre-BN) conv_head output."""
        h = F.silu(self.bn1(self.conv_stem(x)))
        taps = []
        for i, st in enumerate(self.blocks):
            h = st(h)
            if i in (0, 1, 2, 4):
                taps.append(h)
        taps.append(self.conv_head(h))
        return taps


class _NormalEncoder(nn.Module):
    def __init__(self):
        super().__init__()
        self.original_model = EfficientNetB5()


class _UpSampleBN(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self._net = nn.Sequential(nn.Conv2d(cin, cout, 3, 1, 1), nn.BatchNorm2d(cout), nn.LeakyReLU(),
                                  nn.Conv2d(cout, cout, 3, 1, 1), nn.BatchNorm2d(cout), nn.LeakyReLU())

    def forward(self, x, skip):
        x = F.interpolate(x, size=skip.shape[2:], mode="bilinear", align_corners=True)
        return self._net(torch.cat([x, skip], 1))


def _pixel_mlp(cin):
    return nn.Sequential(nn.Conv1d(cin, 128, 1), nn.ReLU(), nn.Conv1d(128, 128, 1), nn.ReLU(),
                         nn.Conv1d(128, 128, 1), nn.ReLU(), nn.Conv1d(128, 4, 1))


def _norm_normalize(out, min_kappa=0.01):
    n, kappa = out[:, :3], out[:, 3:]
    n = n / (n.float().pow(2).sum(1, keepdim=True).sqrt() + 1e-10).to(n.dtype)
    return torch.cat([n, F.elu(kappa) + 1.0 + min_kappa], 1)


class _NormalDecoder(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv2 = nn.Conv2d(2048, 2048, 1)
        self.up1, self.up2 = _UpSampleBN(2048 + 176, 1024), _UpSampleBN(1024 + 64, 512)
        self.up3, self.up4 = _UpSampleBN(512 + 40, 256), _UpSampleBN(256 + 24, 128)
        self.out_conv_res8 = nn.Conv2d(512, 4, 3, 1, 1)
        self.out_conv_res4, self.out_conv_res2, self.out_conv_res1 = _pixel_mlp(516), _pixel_mlp(260), _pixel_mlp(132)

    @staticmethod
    def _refine(mlp, coarse, feat):
        up = lambda t: F.interpolate(t, scale_factor=2, mode="bilinear", align_corners=True)
        pred, feat = up(coarse), up(feat)
        B, _, H, W = pred.shape
        return _norm_normalize(mlp(torch.cat([pred, feat], 1).view(B, -1, H * W)).view(B, 4, H, W))

    def forward(self, taps):
        b0, b1, b2, b3, b4 = taps
        d1 = self.up1(self.conv2(b4), b3)
        d2 = self.up2(d1, b2)
        d3 = self.up3(d2, b1)
        d4 = self.up4(d3, b0)
        r8 = _norm_normalize(self.out_conv_res8(d2))
        r4 = self._refine(self.out_conv_res4, r8, d2)
        r2 = self._refine(self.out_conv_res2, r4, d3)
        r1 = self._refine(self.out_conv_res1, r2, d4)
        return [r8, r4, r2, r1]


class NormalBaeNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.encoder = _NormalEncoder()
        self.decoder = _NormalDecoder()

    def forward(self, x):
        return self.decoder(self.encoder.original_model.features(x))


@torch.no_grad()
def normalbae(image: Image.Image, res=512) -> Image.Image:
    m = _build("normalbae", NormalBaeNet)
    img = np.asarray(_resize_short(image.convert("RGB"), res)).astype(np.float32) / 255.0
    x = (img - np.array([0.485, 0.456, 0.406], np.float32)) / np.array([0.229, 0.224, 0.225], np.float32)
    normal = m(_to_tensor(x, m))[-1][0, :3].float()
    normal = ((normal + 1) * 0.5).clamp(0, 1).permute(1, 2, 0).cpu().numpy()
    out = (normal * 255.0).clip(0, 255).astype(np.uint8)
    return Image.fromarray(out).resize(image.size, Image.Resampling.BILINEAR)
