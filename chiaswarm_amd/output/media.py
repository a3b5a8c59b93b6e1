"""Host media encoding for audio / video results.

The reference shells out to ffmpeg through moviepy / cv2 / pydub
(swarm/video/tx2vid.py:79-88, swarm/video/pix2pix.py:192-197,
swarm/audio/audioldm.py:28-31) — none of which exist on this image.  We use
an ``ffmpeg`` binary when one is on PATH, and otherwise our own encoders:

  * video/mp4: an H.264 Constrained-Baseline stream made of I_PCM macroblocks
    (every frame an IDR; lossless 4:2:0 samples, no entropy coding needed) in
    an ISO-BMFF container (ftyp / moov[avcC] / mdat, faststart).  Large but
    standard: any H.264 decoder plays it.
  * audio: 16-bit PCM WAV (content type audio/wav) when no MP3 encoder exists.
"""
from __future__ import annotations

import io
import shutil
import struct
import subprocess
import tempfile

import numpy as np


def have_ffmpeg() -> bool:
    return shutil.which("ffmpeg") is not None


# ----------------------------------------------------------------------------
# audio
# ----------------------------------------------------------------------------
def wav_bytes(audio: np.ndarray, rate: int) -> bytes:
    a = np.clip(np.asarray(audio, dtype=np.float32).reshape(-1), -1.0, 1.0)
    pcm = (a * 32767.0).astype("<i2").tobytes()
    hdr = b"RIFF" + struct.pack("<I", 36 + len(pcm)) + b"WAVE"
    hdr += b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, rate, rate * 2, 2, 16)
    hdr += b"data" + struct.pack("<I", len(pcm))
    return hdr + pcm


def encode_audio(audio: np.ndarray, rate: int, content_type: str = "audio/mpeg") -> tuple[bytes, str]:
    wav = wav_bytes(audio, rate)
    if content_type == "audio/mpeg" and have_ffmpeg():
        r = subprocess.run(["ffmpeg", "-hide_banner", "-loglevel", "error", "-f", "wav", "-i", "pipe:0",
                            "-f", "mp3", "pipe:1"], input=wav, capture_output=True)
        if r.returncode == 0 and r.stdout:
            return r.stdout, "audio/mpeg"
    return wav, "audio/wav"


# ----------------------------------------------------------------------------
# H.264 I_PCM + MP4
# ----------------------------------------------------------------------------
class _Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def u(self, val, bits):
        self.v = (self.v << bits) | (val & ((1 << bits) - 1))
        self.n += bits

    def ue(self, val):
        x = val + 1
        ln = x.bit_length()
        self.u(0, ln - 1)
        self.u(x, ln)

    def se(self, val):
        self.ue(2 * val - 1 if val > 0 else -2 * val)

    def align_zero(self):
        if self.n % 8:
            self.u(0, 8 - self.n % 8)

    def trailing(self):
        self.u(1, 1)
        self.align_zero()

    def bytes(self):
        assert self.n % 8 == 0
        return self.v.to_bytes(self.n // 8, "big") if self.n else b""


def _ep(payload: bytes) -> bytes:
    """Insert emulation-prevention bytes (00 00 0x, x<=3 -> 00 00 03 0x)."""
    out = bytearray()
    zeros = 0
    for b in payload:
        if zeros >= 2 and b <= 3:
            out.append(3)
            zeros = 0
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


def _ep_fast(header: bytes, body: bytes) -> bytes:
    # body never contains 00 00 (MB prefix 0D 00 followed by PCM >= 1), only the
    # header and its junction need scanning
    k = min(4, len(body))
    return _ep(header + body[:k]) + body[k:]


def _sps(wmb, hmb, crop_r, crop_b) -> bytes:
    b = _Bits()
    b.u(66, 8)        # profile_idc: Baseline
    b.u(0xC0, 8)      # constraint_set0/1 (Constrained Baseline)
    b.u(51, 8)        # level 5.1 (I_PCM bit rates)
    b.ue(0)           # sps id
    b.ue(0)           # log2_max_frame_num_minus4
    b.ue(2)           # pic_order_cnt_type 2 (output order = decode order)
    b.ue(1)           # max_num_ref_frames
    b.u(0, 1)         # gaps_in_frame_num_value_allowed_flag
    b.ue(wmb - 1)
    b.ue(hmb - 1)
    b.u(1, 1)         # frame_mbs_only_flag
    b.u(1, 1)         # direct_8x8_inference_flag
    crop = crop_r or crop_b
    b.u(1 if crop else 0, 1)
    if crop:
        b.ue(0); b.ue(crop_r); b.ue(0); b.ue(crop_b)  # noqa: E702
    b.u(0, 1)         # vui_parameters_present_flag
    b.trailing()
    return b"\x67" + _ep(b.bytes())


def _pps() -> bytes:
    b = _Bits()
    b.ue(0); b.ue(0)  # noqa: E702  pps id, sps id
    b.u(0, 1)         # entropy_coding_mode_flag (CAVLC)
    b.u(0, 1)         # bottom_field_pic_order_in_frame_present_flag
    b.ue(0)           # num_slice_groups_minus1
    b.ue(0); b.ue(0)  # noqa: E702  num_ref_idx_l0/l1_default_active_minus1
    b.u(0, 1); b.u(0, 2)  # noqa: E702  weighted_pred_flag, weighted_bipred_idc
    b.se(0); b.se(0); b.se(0)  # noqa: E702  pic_init_qp/qs_minus26, chroma_qp_index_offset
    b.u(1, 1)         # deblocking_filter_control_present_flag
    b.u(0, 1)         # constrained_intra_pred_flag
    b.u(0, 1)         # redundant_pic_cnt_present_flag
    b.trailing()
    return b"\x68" + _ep(b.bytes())


def rgb_to_yuv420(frame: np.ndarray, H16: int, W16: int):
    f = frame.astype(np.float32) / 255.0
    h, w = f.shape[:2]
    pad = np.zeros((H16, W16, 3), np.float32)
    pad[:h, :w] = f
    pad[h:, :w] = f[-1:, :, :] if h < H16 else pad[h:, :w]
    pad[:, w:] = pad[:, w - 1:w]
    r, g, b = pad[..., 0], pad[..., 1], pad[..., 2]
    y = 16 + 65.481 * r + 128.553 * g + 24.966 * b
    cb = 128 - 37.797 * r - 74.203 * g + 112.0 * b
    cr = 128 + 112.0 * r - 93.786 * g - 18.214 * b
    sub = lambda c: c.reshape(H16 // 2, 2, W16 // 2, 2).mean(axis=(1, 3))  # noqa: E731
    q = lambda c: np.clip(np.rint(c), 1, 254).astype(np.uint8)  # noqa: E731  (PCM samples must be != 0)
    return q(y), q(sub(cb)), q(sub(cr))


def _idr_slice(frame: np.ndarray, idr_id: int) -> bytes:
    h, w = frame.shape[:2]
    H16, W16 = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    y, cb, cr = rgb_to_yuv420(frame, H16, W16)
    hm, wm = H16 // 16, W16 // 16
    ymb = y.reshape(hm, 16, wm, 16).transpose(0, 2, 1, 3).reshape(hm * wm, 256)
    cbm = cb.reshape(hm, 8, wm, 8).transpose(0, 2, 1, 3).reshape(hm * wm, 64)
    crm = cr.reshape(hm, 8, wm, 8).transpose(0, 2, 1, 3).reshape(hm * wm, 64)
    pcm = np.concatenate([ymb, cbm, crm], axis=1)  # [nmb, 384]
    b = _Bits()
    b.ue(0)            # first_mb_in_slice
    b.ue(7)            # slice_type I (all slices)
    b.ue(0)            # pps id
    b.u(0, 4)          # frame_num
    b.ue(idr_id)       # idr_pic_id
    b.u(0, 1); b.u(0, 1)  # noqa: E702  no_output_of_prior_pics, long_term_reference
    b.se(0)            # slice_qp_delta
    b.ue(1)            # disable_deblocking_filter_idc = 1
    b.ue(25)           # mb_type I_PCM (first MB)
    b.align_zero()     # pcm_alignment_zero_bits
    head = b.bytes()
    prefix = np.frombuffer(b"\x0d\x00", np.uint8)  # ue(25) + 7 alignment bits for MBs 2..N
    rows = [pcm[0]] + [np.concatenate([prefix, pcm[i]]) for i in range(1, pcm.shape[0])]
    body = np.concatenate(rows).tobytes() + b"\x80"  # rbsp_slice_trailing_bits
    return b"\x65" + _ep_fast(head, body)


def _box(tag: bytes, *parts: bytes) -> bytes:
    data = b"".join(parts)
    return struct.pack(">I", 8 + len(data)) + tag + data


def _full(tag: bytes, version: int, flags: int, *parts: bytes) -> bytes:
    return _box(tag, struct.pack(">I", (version << 24) | flags), *parts)


_MATRIX = struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


def frames_to_mp4_ipcm(frames: np.ndarray, fps: int = 8) -> bytes:
    frames = np.asarray(frames, dtype=np.uint8)
    n, h, w = frames.shape[:3]
    wm, hm = (w + 15) // 16, (h + 15) // 16
    sps = _sps(wm, hm, (wm * 16 - w) // 2, (hm * 16 - h) // 2)
    pps = _pps()
    samples = [_idr_slice(frames[i], i & 1) for i in range(n)]
    sizes = [4 + len(s) for s in samples]
    ts, delta = fps * 100, 100
    dur_ms = int(round(1000 * n / fps))
    avcc = _box(b"avcC", bytes([1, 66, 0xC0, 51, 0xFF, 0xE1]) + struct.pack(">H", len(sps)) + sps
                + b"\x01" + struct.pack(">H", len(pps)) + pps)
    avc1 = _box(b"avc1", b"\x00" * 6 + struct.pack(">H", 1) + b"\x00" * 16 + struct.pack(">HH", w, h)
                + struct.pack(">II", 0x480000, 0x480000) + b"\x00" * 4 + struct.pack(">H", 1) + b"\x00" * 32
                + struct.pack(">Hh", 0x18, -1) + avcc)

    def moov(mdat_off):
        stbl = _box(b"stbl",
                    _full(b"stsd", 0, 0, struct.pack(">I", 1), avc1),
                    _full(b"stts", 0, 0, struct.pack(">III", 1, n, delta)),
                    _full(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, n, 1)),
                    _full(b"stsz", 0, 0, struct.pack(">II", 0, n), struct.pack(f">{n}I", *sizes)),
                    _full(b"stco", 0, 0, struct.pack(">II", 1, mdat_off)))
        minf = _box(b"minf", _full(b"vmhd", 0, 1, b"\x00" * 8),
                    _box(b"dinf", _full(b"dref", 0, 0, struct.pack(">I", 1), _full(b"url ", 0, 1))), stbl)
        mdia = _box(b"mdia", _full(b"mdhd", 0, 0, struct.pack(">IIIIHH", 0, 0, ts, n * delta, 0x55C4, 0)),
                    _full(b"hdlr", 0, 0, b"\x00" * 4 + b"vide" + b"\x00" * 12 + b"VideoHandler\x00"), minf)
        tkhd = _full(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, dur_ms), b"\x00" * 8,
                     struct.pack(">hhhH", 0, 0, 0, 0), _MATRIX, struct.pack(">II", w << 16, h << 16))
        mvhd = _full(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, 1000, dur_ms), struct.pack(">IH", 0x10000, 0x100),
                     b"\x00" * 10, _MATRIX, b"\x00" * 24, struct.pack(">I", 2))
        return _box(b"moov", mvhd, _box(b"trak", tkhd, mdia))

    ftyp = _box(b"ftyp", b"isom", struct.pack(">I", 512), b"isomiso2avc1mp41")
    m0 = moov(0)
    off = len(ftyp) + len(m0) + 8
    mdat = b"".join(struct.pack(">I", len(s)) + s for s in samples)
    return ftyp + moov(off) + struct.pack(">I", 8 + len(mdat)) + b"mdat" + mdat


def frames_to_video(frames: np.ndarray, fps: int = 8, content_type: str = "video/mp4") -> tuple[bytes, str]:
    frames = np.asarray(frames, dtype=np.uint8)
    if have_ffmpeg():
        n, h, w = frames.shape[:3]
        codec = ["-c:v", "libvpx-vp9", "-f", "webm"] if content_type == "video/webm" else \
            ["-c:v", "libx264", "-pix_fmt", "yuv420p", "-movflags", "frag_keyframe+empty_moov", "-f", "mp4"]
        r = subprocess.run(["ffmpeg", "-hide_banner", "-loglevel", "error", "-f", "rawvideo", "-pix_fmt", "rgb24",
                            "-s", f"{w}x{h}", "-r", str(fps), "-i", "pipe:0", *codec, "pipe:1"],
                           input=frames.tobytes(), capture_output=True)
        if r.returncode == 0 and r.stdout:
            return r.stdout, content_type
    return frames_to_mp4_ipcm(frames, fps), "video/mp4"


def read_video_frames(path: str, max_frames: int = 100, max_fps: float = 30.0, height: int = 512):
    """Decode a video to RGB frames (ffmpeg if available; animated GIF/WebP/PNG via PIL)."""
    from PIL import Image, ImageSequence

    if have_ffmpeg():
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run(["ffmpeg", "-hide_banner", "-loglevel", "error", "-i", path, "-vf",
                                f"fps={max_fps},scale=-2:{height}", "-frames:v", str(max_frames),
                                f"{d}/f%04d.png"], capture_output=True)
            if r.returncode == 0:
                import glob

                files = sorted(glob.glob(f"{d}/f*.png"))
                return [Image.open(f).convert("RGB") for f in files], max_fps
    try:
        im = Image.open(path)
        frames = []
        for fr in ImageSequence.Iterator(im):
            f = fr.convert("RGB")
            if f.height != height:
                f = f.resize((max(8, round(f.width * height / f.height / 8) * 8), height))
            frames.append(f)
            if len(frames) >= max_frames:
                break
        dur = im.info.get("duration", 100) or 100
        return frames, min(max_fps, 1000.0 / dur)
    except Exception as e:
        raise ValueError(f"cannot decode video input without ffmpeg ({e})") from e


# ----------------------------------------------------------------------------
# decoding our own I_PCM MP4s (no ffmpeg needed) + frame / clip helpers
# ----------------------------------------------------------------------------
def _unescape(nal: bytes) -> bytes:
    return nal.replace(b"\x00\x00\x03", b"\x00\x00")


class _BitReader:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.d[self.p >> 3] >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v

    def ue(self) -> int:
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


def _find_box(data: bytes, tag: bytes, start=0, end=None):
    end = len(data) if end is None else end
    i = start
    while i + 8 <= end:
        size = struct.unpack(">I", data[i:i + 4])[0]
        if data[i + 4:i + 8] == tag:
            return i, size
        if size < 8:
            return None
        i += size
    return None


def decode_ipcm_mp4(data: bytes) -> list[np.ndarray]:
    """Decode an MP4 written by ``frames_to_mp4_ipcm`` (all-I_PCM H.264) back to
    RGB frames.  Raises ValueError for any other stream."""
    k = data.find(b"avc1", max(0, data.find(b"stsd")))  # the sample entry, not the ftyp brand
    md = _find_box(data, b"mdat")
    if k < 0 or md is None:
        raise ValueError("not an avc1 mp4")
    w, h = struct.unpack(">HH", data[k + 4 + 24:k + 4 + 28])
    W16, H16 = (w + 15) // 16 * 16, (h + 15) // 16 * 16
    wm, hm = W16 // 16, H16 // 16
    i, end = md[0] + 8, md[0] + md[1]
    frames = []
    while i + 4 <= end:
        n = struct.unpack(">I", data[i:i + 4])[0]
        nal = data[i + 4:i + 4 + n]
        i += 4 + n
        if not nal or nal[0] & 0x1F != 5:
            continue
        rb = _unescape(nal[1:])
        br = _BitReader(rb)
        br.ue(); br.ue(); br.ue(); br.u(4); br.ue(); br.u(1); br.u(1); br.se()  # noqa: E702
        if br.ue() != 1:
            raise ValueError("unsupported slice header")
        if br.ue() != 25:
            raise ValueError("not an I_PCM stream")
        pos = (br.p + 7) >> 3
        nmb = wm * hm
        buf = np.frombuffer(rb, np.uint8)
        mbs = np.empty((nmb, 384), np.uint8)
        for m in range(nmb):
            if m:
                pos += 2  # ue(25) + alignment of the next I_PCM macroblock
            mbs[m] = buf[pos:pos + 384]
            pos += 384
        y = mbs[:, :256].reshape(hm, wm, 16, 16).transpose(0, 2, 1, 3).reshape(H16, W16).astype(np.float32)
        cb = mbs[:, 256:320].reshape(hm, wm, 8, 8).transpose(0, 2, 1, 3).reshape(H16 // 2, W16 // 2)
        cr = mbs[:, 320:].reshape(hm, wm, 8, 8).transpose(0, 2, 1, 3).reshape(H16 // 2, W16 // 2)
        cb = cb.astype(np.float32).repeat(2, 0).repeat(2, 1) - 128.0
        cr = cr.astype(np.float32).repeat(2, 0).repeat(2, 1) - 128.0
        yy = (y - 16.0) * (255.0 / 219.0)
        r = yy + 1.402 * cr * (255.0 / 224.0)
        g = yy - (0.344136 * cb + 0.714136 * cr) * (255.0 / 224.0)
        b = yy + 1.772 * cb * (255.0 / 224.0)
        rgb = np.clip(np.rint(np.stack([r, g, b], -1)), 0, 255).astype(np.uint8)
        frames.append(rgb[:h, :w])
    return frames


def get_frame(video_path: str, frame_index: int = 0):
    """JPEG ``BytesIO`` of one frame of a video, or None (reference:
    swarm/toolbox/video_helpers.py:6-25, used for video thumbnails)."""
    import io

    from PIL import Image

    try:
        frame = None
        if have_ffmpeg():
            r = subprocess.run(["ffmpeg", "-hide_banner", "-loglevel", "error", "-i", video_path, "-vf",
                                f"select=eq(n\\,{int(frame_index)})", "-vframes", "1", "-f", "image2pipe",
                                "-vcodec", "png", "pipe:1"], capture_output=True)
            if r.returncode == 0 and r.stdout:
                frame = Image.open(io.BytesIO(r.stdout)).convert("RGB")
        if frame is None:
            with open(video_path, "rb") as f:
                data = f.read()
            try:
                frames = decode_ipcm_mp4(data)
                frame = Image.fromarray(frames[min(int(frame_index), len(frames) - 1)])
            except ValueError:
                frames, _ = read_video_frames(video_path, max_frames=int(frame_index) + 1)
                frame = frames[min(int(frame_index), len(frames) - 1)]
        buf = io.BytesIO()
        frame.save(buf, format="JPEG")
        buf.seek(0)
        return buf
    except Exception as e:  # the reference prints and returns None
        print(e)
        return None


def make_video(images, duration_seconds: float, content_type: str = "video/webm") -> tuple[bytes, str]:
    """Clip of PIL images / HWC arrays spread over ``duration_seconds``
    (reference: swarm/diffusion/video_maker.py:7-21, dead code there)."""
    frames = np.stack([np.asarray(im.convert("RGB") if hasattr(im, "convert") else im, dtype=np.uint8)
                       for im in images])
    fps = max(1, int(round(len(frames) / max(duration_seconds, 1e-3))))
    return frames_to_video(frames, fps, content_type)
