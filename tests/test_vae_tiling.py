"""VAE slicing / tiled decode (models/vae.py::AutoencoderKL.decode,
tiled_decode) — the reference's enable_vae_slicing / enable_vae_tiling
(swarm/diffusion/diffusion_func.py:89-92) for outputs too large to decode at
once.  Checked on a tiny random VAE on the CPU against the full decode and the
cross-fade rule."""
import torch

from chiaswarm_amd.models import vae as vae_mod
from chiaswarm_amd.models.layers import init_random_


def _tiny():
    torch.manual_seed(0)
    m = vae_mod.AutoencoderKL(vae_mod.TINY_VAE, with_encoder=False).eval()
    init_random_(m, seed=1)
    return m


@torch.no_grad()
def test_single_tile_equals_full_decode():
    m = _tiny()
    z = torch.randn(1, 6, 6, 4)
    full = m._decode_full(z)
    assert torch.equal(m.tiled_decode(z, tile=8), full)  # the latent fits in one stride: one tile


@torch.no_grad()
def test_tiled_decode_shape_and_cross_fade():
    m = _tiny()
    f = m.upscale
    z = torch.randn(1, 20, 12, 4)
    tile, overlap = 8, 0.25
    out = m.tiled_decode(z, tile=tile, overlap=overlap)
    assert out.shape == (1, 20 * f, 12 * f, 3)
    # first tile row, second tile column: its leading columns are the linear mix
    # of the left tile's trailing columns and its own (left tile untouched there)
    stride, blend = int(tile * (1 - overlap)), int(tile * f * overlap)
    left = m._decode_full(z[:, 0:tile, 0:tile])
    right = m._decode_full(z[:, 0:tile, stride:stride + tile])
    keep = tile * f - blend
    w = torch.arange(blend, dtype=torch.float32).view(1, 1, blend, 1) / blend
    expect = left[:, :, -blend:] * (1 - w) + right[:, :, :blend] * w
    got = out[:, :keep, keep:keep + blend]
    assert torch.allclose(got, expect[:, :keep], atol=1e-5)
    # away from the seams the tiled decode is the tile's own decode
    assert torch.allclose(out[:, :keep, :keep - blend], left[:, :keep, :keep - blend])


@torch.no_grad()
def test_decode_switches_to_slices_and_tiles(monkeypatch):
    m = _tiny()
    z = torch.randn(3, 8, 8, 4)
    full = m._decode_full(z)
    monkeypatch.setattr(vae_mod.AutoencoderKL, "SLICE_PIXELS", 1)
    sliced = m.decode(z)
    assert torch.allclose(sliced, full, atol=1e-5)
    monkeypatch.setattr(vae_mod.AutoencoderKL, "TILE_PIXELS", 1)
    calls = []
    orig = vae_mod.AutoencoderKL.tiled_decode
    monkeypatch.setattr(vae_mod.AutoencoderKL, "tiled_decode",
                        lambda self, zz, **kw: calls.append(zz.shape) or orig(self, zz, **kw))
    out = m.decode(z)
    assert len(calls) == 3 and out.shape == full.shape
