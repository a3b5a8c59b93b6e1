"""Stream-K GEMM tiles 40-43 (csrc/kernels/gemm_sk.hip) against the fp32
PyTorch reference: every fixup shape the worker split can produce (forced with
small worker counts: tiles cut into 2..many pieces, pieces of one K-step),
ragged M / N, bias + residual, GEGLU, fused GroupNorm statistics and the fused
LayerNorm consumer / row-statistics producer epilogues."""
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


def _errors():
    import ctypes

    e = ctypes.c_uint(0)
    assert _lib.load().csk_gemm_sk_errors(ctypes.byref(e)) == 0
    return e.value


class _Force:
    """Pin tuning-table entries to (tile, 1) and cap the stream-K workers."""

    def __init__(self, keys, tile, workers=0):
        self.keys, self.tile, self.workers = keys, tile, workers

    def __enter__(self):
        t = tuning.table()
        self.old = {k: t.get(k) for k in self.keys}
        for k in self.keys:
            t[k] = [self.tile, 1, 0.0]
        _lib.load().csk_set_gemm_sk_workers(self.workers)

    def __exit__(self, *exc):
        t = tuning.table()
        for k, v in self.old.items():
            if v is None:
                t.pop(k, None)
            else:
                t[k] = v
        _lib.load().csk_set_gemm_sk_workers(0)


@pytest.mark.parametrize("tile", [40, 41, 42, 43])
@pytest.mark.parametrize("M,N,K", [(2048, 1280, 1280), (1000, 320, 320), (130, 200, 64), (512, 640, 2560)])
@pytest.mark.parametrize("workers", [0, 7, 61])
def test_gemm_sk_matches_fp32(gpu, tile, M, N, K, workers):
    torch.manual_seed(M + N + K + tile + workers)
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    r = rnd(M, N, dev=gpu)
    with _Force([f"g:{M}:{N}:{K}:0"], tile, workers):
        y = hip_ops.gemm(a, w, b, r, None)
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), None)
    assert rel_err(y.cpu(), ref) < 1e-2
    assert _errors() == 0


@pytest.mark.parametrize("tile", [40, 42])
def test_gemm_sk_geglu_and_repeat_bits(gpu, tile):
    M, N, K = 2048, 2560, 640
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    with _Force([f"g:{M}:{N}:{K}:3"], tile, 37):
        y1 = hip_ops.gemm(a, w, b, None, "geglu")
        y2 = hip_ops.gemm(a, w, b, None, "geglu")
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), None, "geglu")
    assert rel_err(y1.cpu(), ref) < 1e-2
    assert torch.equal(y1, y2)  # fixed merge order: deterministic
    assert _errors() == 0


@pytest.mark.parametrize("tile", [40, 41])
def test_gemm_sk_gn_stats(gpu, tile):
    """GroupNorm statistics from the stream-K epilogue feed the fused GN."""
    B, P, N, K = 2, 1024, 640, 640
    a, w = rnd(B * P, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5)
    g, bb = rnd(N, dev=gpu), rnd(N, dev=gpu)
    with _Force([f"g:{B * P}:{N}:{K}:0"], tile, 29):
        y = hip_ops.gemm(a, w, None, None, None, gn_rows=P)
    assert getattr(y, "_csk_gn", None) is not None
    y3 = y.view(B, P, 1, N)
    fused = hip_ops.group_norm(y3, g, bb, 32, 1e-5, True)
    ref = ops._ref_group_norm(y3.float().cpu(), g.float().cpu(), bb.float().cpu(), 32, 1e-5, True)
    assert rel_err(fused.cpu(), ref) < 1e-2
    assert _errors() == 0


@pytest.mark.parametrize("tile", [40, 41, 43])
def test_gemm_sk_fused_layernorm_chain(gpu, tile):
    """Row-statistics producer -> fused-LN consumer, both on stream-K tiles."""
    M, C, N = 2048, 640, 1280
    x, w0 = rnd(M, C, dev=gpu), rnd(C, C, dev=gpu, scale=C ** -0.5)
    w1, b1 = rnd(N, C, dev=gpu, scale=C ** -0.5), rnd(N, dev=gpu)
    gam, bet = rnd(C, dev=gpu) + 1.0, rnd(C, dev=gpu)
    wf, colsum, bf = ops.fold_layer_norm(w1, b1, gam, bet)
    with _Force([f"g:{M}:{C}:{C}:0", f"g:{M}:{N}:{C}:0"], tile, 53):
        h = hip_ops.gemm(x, w0, None, None, None, row_stats=True)
        y = hip_ops.gemm(h, wf, bf, None, None, ln=(h._csk_rows, colsum, 1e-5))
    hf = h.float().cpu()
    ln = torch.nn.functional.layer_norm(hf, (C,), gam.float().cpu(), bet.float().cpu(), 1e-5)
    ref = ln @ w1.float().cpu().t() + b1.float().cpu()
    assert rel_err(h.cpu(), x.float().cpu() @ w0.float().cpu().t()) < 1e-2
    assert rel_err(y.cpu(), ref) < 1.5e-2
    assert _errors() == 0


def test_gemm_sk_graph_replay(gpu):
    M, N, K = 2048, 1280, 1280
    a, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5)
    with _Force([f"g:{M}:{N}:{K}:0"], 40):
        ref = hip_ops.gemm(a, w)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            hip_ops.gemm(a, w)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = hip_ops.gemm(a, w)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert _errors() == 0
