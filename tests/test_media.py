"""Own media encoders: WAV, H.264 I_PCM-in-MP4 (structure + sample round trip)."""
import struct

import numpy as np

from chiaswarm_amd.output import media


def boxes(buf, off=0, end=None):
    end = len(buf) if end is None else end
    out = {}
    while off < end:
        size, tag = struct.unpack(">I4s", buf[off:off + 8])
        out.setdefault(tag.decode(), []).append((off + 8, off + size))
        off += size
    return out


def test_wav_roundtrip():
    a = np.sin(np.linspace(0, 100, 16000)).astype(np.float32) * 0.5
    w = media.wav_bytes(a, 16000)
    assert w[:4] == b"RIFF" and w[8:12] == b"WAVE"
    import io
    import wave

    with wave.open(io.BytesIO(w)) as f:
        assert f.getframerate() == 16000 and f.getnframes() == 16000 and f.getsampwidth() == 2


def test_ipcm_mp4_structure_and_samples():
    rng = np.random.default_rng(0)
    frames = rng.integers(0, 256, (3, 40, 56, 3), dtype=np.uint8)  # not multiples of 16 -> cropping
    mp4 = media.frames_to_mp4_ipcm(frames, fps=8)
    top = boxes(mp4)
    assert list(top)[:3] == ["ftyp", "moov", "mdat"]
    ms, me = top["moov"][0]
    moov = boxes(mp4, ms, me)
    ts, te = moov["trak"][0]
    assert "mdia" in boxes(mp4, ts, te)
    # stco points at the first sample inside mdat
    i = mp4.find(b"stco")
    off = struct.unpack(">I", mp4[i + 12:i + 16])[0]
    ds, de = top["mdat"][0]
    assert off == ds
    # sample 0: 4-byte length + IDR NAL (0x65)
    n0 = struct.unpack(">I", mp4[off:off + 4])[0]
    nal = mp4[off + 4: off + 4 + n0]
    assert nal[0] == 0x65
    # strip emulation prevention and check the first macroblock's PCM luma
    raw = bytearray()
    z = 0
    for b in nal[1:]:
        if z >= 2 and b == 3:
            z = 0
            continue
        raw.append(b)
        z = z + 1 if b == 0 else 0
    hm, wm = 3, 4
    y, cb, cr = media.rgb_to_yuv420(frames[0], hm * 16, wm * 16)
    first = y[:16, :16].reshape(-1).tobytes()
    assert first in bytes(raw)
    # every MB is present: prefix 0D 00 before MBs 2..N
    assert bytes(raw).count(b"\x0d\x00") >= hm * wm - 1
    # avcC carries SPS (0x67) and PPS (0x68)
    j = mp4.find(b"avcC")
    assert mp4[j + 4] == 1 and mp4[j + 5] == 66
    assert b"\x67" in mp4[j:j + 64] and b"\x68" in mp4[j:j + 80]


def test_frames_to_video_fallback():
    frames = np.zeros((2, 32, 32, 3), np.uint8)
    data, ct = media.frames_to_video(frames, 8, "video/mp4")
    assert ct == "video/mp4" and data[4:8] == b"ftyp"


def test_ipcm_decoder_roundtrip_and_get_frame(tmp_path):
    import numpy as np

    from chiaswarm_amd.output import media

    fr = np.zeros((3, 40, 56, 3), np.uint8)
    fr[0] = (200, 30, 30)
    fr[1] = (30, 200, 30)
    fr[2, :, :28] = (30, 30, 200)
    data = media.frames_to_mp4_ipcm(fr, 8)
    dec = media.decode_ipcm_mp4(data)
    assert len(dec) == 3 and dec[0].shape == (40, 56, 3)
    # flat colours survive the BT.601 limited-range round trip within rounding
    assert np.abs(dec[0].astype(int) - fr[0].astype(int)).max() <= 3
    assert np.abs(dec[1].astype(int) - fr[1].astype(int)).max() <= 3
    p = tmp_path / "clip.mp4"
    p.write_bytes(data)
    from PIL import Image

    jpg = media.get_frame(str(p), 1)
    im = Image.open(jpg)
    assert im.size == (56, 40)
    assert media.get_frame(str(tmp_path / "missing.mp4")) is None
    blob, ct = media.make_video([fr[0], fr[1]], 0.25)
    assert ct in ("video/webm", "video/mp4") and len(blob) > 100


def test_type_helpers():
    from chiaswarm_amd.utils import get_type, has_method

    assert get_type("chiaswarm_amd.schedulers", "EulerDiscreteScheduler").__name__ == "EulerDiscreteScheduler"
    assert has_method([], "append") and not has_method([], "nope")


def test_roctx_ranges_are_safe_without_a_profiler():
    from chiaswarm_amd.utils import trace

    old = trace.enabled()
    try:
        trace.set_enabled(True)
        with trace.trace_range("unit-test"):
            trace.mark("inside")
        trace.set_enabled(False)
        with trace.trace_range("disabled"):
            pass
    finally:
        trace.set_enabled(old)


def test_download_video_removes_partial_file_over_cap(monkeypatch, tmp_path):
    """The reference leaves nothing behind when a video exceeds its 30 MiB cap
    (swarm/video/pix2pix.py:95-104); a streamed body larger than its HEAD claims
    must not leak the temp file either."""
    import tempfile

    import pytest

    from chiaswarm_amd.jobs import inputs

    class Resp:
        headers = {"Content-Length": "10", "Content-Type": "video/mp4"}

        def raise_for_status(self):
            pass

        def iter_content(self, n):
            for _ in range(8):
                yield b"x" * 1000

        def __enter__(self):
            return self

        def __exit__(self, *a):
            return False

    class Sess:
        def head(self, *a, **k):
            return Resp()

        def get(self, *a, **k):
            return Resp()

    monkeypatch.setattr(inputs, "_http", lambda: Sess())
    monkeypatch.setattr(inputs, "MAX_VIDEO_BYTES", 2500)
    monkeypatch.setattr(tempfile, "tempdir", str(tmp_path))
    with pytest.raises(Exception, match="too large"):
        inputs.download_video("http://x/v.mp4")
    assert list(tmp_path.iterdir()) == []
