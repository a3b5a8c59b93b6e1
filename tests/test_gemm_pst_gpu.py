"""Persistent cross-tile-ring GEMM tiles 50-53 (csrc/kernels/gemm_pst.hip)
against the fp32 PyTorch reference: UNet short-K shapes, ragged M / N, fewer
tiles than workgroup slots, bias + residual + activation, GEGLU, per-sample
bias, graph replay; the epilogues it declines (GroupNorm / LayerNorm / row
statistics) fall back to the one-tile kernel."""
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
    assert _lib.load().csk_gemm_pst_launches(ctypes.byref(n)) == 0
    return n.value


class _Force:
    def __init__(self, keys, tile):
        self.keys, self.tile = keys, tile

    def __enter__(self):
        t = tuning.table()
        self.old = {k: t.get(k) for k in self.keys}
        for k in self.keys:
            t[k] = [self.tile, 1, 0.0]

    def __exit__(self, *exc):
        t = tuning.table()
        for k, v in self.old.items():
            if v is None:
                t.pop(k, None)
            else:
                t[k] = v


@pytest.mark.parametrize("tile", [50, 51, 52, 53])
@pytest.mark.parametrize("M,N,K", [(32768, 320, 320), (8192, 640, 640), (130, 200, 64), (2048, 1280, 1280),
                                   (1000, 968, 2560)])
@pytest.mark.parametrize("act", [None, "silu"])
def test_pst_matches_fp32(gpu, tile, M, N, K, act):
    torch.manual_seed(M + N + K + tile)
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    r = rnd(M, N, dev=gpu)
    n0 = _launches()
    with _Force([f"g:{M}:{N}:{K}:{hip_ops.ACT[act]}"], tile):
        y = hip_ops.gemm(a, w, b, r, act)
        y2 = hip_ops.gemm(a, w, b, r, act)
    torch.cuda.synchronize()
    assert _launches() == n0 + 2
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), act)
    assert rel_err(y.cpu(), ref) < 1e-2
    assert torch.equal(y, y2)


@pytest.mark.parametrize("tile,runs", [(50, True), (52, True), (53, True), (51, False)])
def test_pst_geglu(gpu, tile, runs):
    """GEGLU needs 4 fragments per wave (the 64x64 tile declines: fallback)."""
    M, N, K = 4096, 2560, 320
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    n0 = _launches()
    with _Force([f"g:{M}:{N}:{K}:3"], tile):
        y = hip_ops.gemm(a, w, b, None, "geglu")
    torch.cuda.synchronize()
    assert _launches() == n0 + (1 if runs else 0)
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), None, "geglu")
    assert rel_err(y.cpu(), ref) < 1e-2


def test_pst_per_sample_bias(gpu):
    B, P, N, K = 4, 1024, 640, 640
    a, w = rnd(B * P, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5)
    b2 = rnd(B, N, dev=gpu)
    y = torch.empty(B * P, N, dtype=torch.bfloat16, device=gpu)
    n0 = _launches()
    _lib.call("csk_gemm", y.data_ptr(), a.data_ptr(), w.data_ptr(), None, b2.data_ptr(), None,
              B * P, N, K, K, K, N, N, P, 2, 0.5, None, 50, 1, None, _lib.stream_ptr())
    torch.cuda.synchronize()
    assert _launches() == n0 + 1
    ref = torch.nn.functional.silu((a.float() @ w.float().t()).view(B, P, N) + b2.float()[:, None, :]) * 0.5
    assert rel_err(y.view(B, P, N).cpu(), ref.cpu()) < 1e-2


def test_pst_declined_epilogues_fall_back(gpu):
    B, P, C, N = 2, 1024, 640, 1280
    x, w0 = rnd(B * P, C, dev=gpu), rnd(C, C, dev=gpu, scale=C ** -0.5)
    w1, b1 = rnd(N, C, dev=gpu, scale=C ** -0.5), rnd(N, dev=gpu)
    gam, bet = rnd(C, dev=gpu) + 1.0, rnd(C, dev=gpu)
    wf, colsum, bf = ops.fold_layer_norm(w1, b1, gam, bet)
    n0 = _launches()
    with _Force([f"g:{B * P}:{C}:{C}:0", f"g:{B * P}:{N}:{C}:0"], 50):
        h = hip_ops.gemm(x, w0, None, None, None, row_stats=True)
        y = hip_ops.gemm(h, wf, bf, None, None, ln=(h._csk_rows, colsum, 1e-5))
        g = hip_ops.gemm(x, w0, None, None, None, gn_rows=P)
    torch.cuda.synchronize()
    assert _launches() == n0  # all three took the one-tile fallback
    hf = h.float().cpu()
    ln = torch.nn.functional.layer_norm(hf, (C,), gam.float().cpu(), bet.float().cpu(), 1e-5)
    assert rel_err(y.cpu(), ln @ w1.float().cpu().t() + b1.float().cpu()) < 1.5e-2
    assert getattr(g, "_csk_gn", None) is not None
    g3 = g.view(B, P, 1, C)
    gg, gb = rnd(C, dev=gpu), rnd(C, dev=gpu)
    fused = hip_ops.group_norm(g3, gg, gb, 32, 1e-5, True)
    ref = ops._ref_group_norm(g3.float().cpu(), gg.float().cpu(), gb.float().cpu(), 32, 1e-5, True)
    assert rel_err(fused.cpu(), ref) < 1e-2


def test_pst_graph_replay(gpu):
    M, N, K = 32768, 320, 320
    a, w, r = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(M, N, dev=gpu)
    with _Force([f"g:{M}:{N}:{K}:0"], 50):
        ref = hip_ops.gemm(a, w, None, r)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hip_ops.gemm(a, w, None, r)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = hip_ops.gemm(a, w, None, r)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)
