"""Sliced-K GEMM tile 44 (csrc/kernels/gemm_slk.hip) against the fp32 PyTorch
reference: small-M projection shapes of the CFG-2 UNet step, ragged M / N,
K-step counts below / at / above the 8-wave split, bias + residual + per-sample
bias + activations, and the epilogues it refuses (GEGLU, fused LN, row / GN
statistics) falling back to the one-tile kernel."""
import ctypes

import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.ops import _lib, hip_ops, tuning

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / (ref.norm() + 1e-12)).item()


def _launches():
    n = ctypes.c_ulonglong(0)
    assert _lib.load().csk_gemm_slk_launches(ctypes.byref(n)) == 0
    return n.value


class _Force:
    def __init__(self, keys):
        self.keys = keys

    def __enter__(self):
        t = tuning.table()
        self.old = {k: t.get(k) for k in self.keys}
        for k in self.keys:
            t[k] = [44, 1, 0.0]

    def __exit__(self, *exc):
        t = tuning.table()
        for k, v in self.old.items():
            if v is None:
                t.pop(k, None)
            else:
                t[k] = v


@pytest.mark.parametrize("M,N,K", [(128, 1280, 1280), (512, 1280, 1280), (1000, 640, 640), (2048, 320, 320),
                                   (130, 200, 64), (77, 1024, 448), (512, 1280, 5120), (64, 64, 1024)])
@pytest.mark.parametrize("act", [None, "silu", "gelu"])
def test_gemm_slk_matches_fp32(gpu, M, N, K, act):
    torch.manual_seed(M + N + K)
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    r = rnd(M, N, dev=gpu)
    code = hip_ops.ACT[act]
    n0 = _launches()
    with _Force([f"g:{M}:{N}:{K}:{code}"]):
        y = hip_ops.gemm(a, w, b, r, act)
    torch.cuda.synchronize()
    assert _launches() == n0 + 1
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), act)
    assert rel_err(y.cpu(), ref) < 1e-2


def test_gemm_slk_per_sample_bias_and_scale(gpu):
    """Time-embedding bias per sample (bias2d) + out_scale, called on tile 44 directly."""
    B, P, N, K = 2, 64, 1280, 1280
    a, w = rnd(B * P, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5)
    b2 = rnd(B, N, dev=gpu)
    y = torch.empty(B * P, N, dtype=torch.bfloat16, device=gpu)
    n0 = _launches()
    _lib.call("csk_gemm", y.data_ptr(), a.data_ptr(), w.data_ptr(), None, b2.data_ptr(), None,
              B * P, N, K, K, K, N, N, P, 2, 0.5, None, 44, 1, None, _lib.stream_ptr())
    torch.cuda.synchronize()
    assert _launches() == n0 + 1
    ref = (a.float() @ w.float().t()).view(B, P, N) + b2.float()[:, None, :]
    ref = torch.nn.functional.silu(ref) * 0.5
    assert rel_err(y.view(B, P, N).cpu(), ref.cpu()) < 1e-2


def test_gemm_slk_refused_epilogues_fall_back(gpu):
    M, N, K = 512, 2560, 640
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    n0 = _launches()
    with _Force([f"g:{M}:{N}:{K}:3", f"g:{M}:{N}:{K}:0"]):
        y = hip_ops.gemm(a, w, b, None, "geglu")
        h = hip_ops.gemm(a, w, None, None, None, row_stats=True)
    torch.cuda.synchronize()
    assert _launches() == n0  # neither ran on tile 44
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), None, "geglu")
    assert rel_err(y.cpu(), ref) < 1e-2
    assert rel_err(h.cpu(), a.float().cpu() @ w.float().cpu().t()) < 1e-2


def test_gemm_slk_deterministic(gpu):
    M, N, K = 512, 1280, 5120
    a, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5)
    with _Force([f"g:{M}:{N}:{K}:0"]):
        y1 = hip_ops.gemm(a, w)
        y2 = hip_ops.gemm(a, w)
    assert torch.equal(y1, y2)
