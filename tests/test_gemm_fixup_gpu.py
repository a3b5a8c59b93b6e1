"""In-kernel split-K fixup (tuning split < 0: gemm_common.h splitk_fixup on the
LDS-DMA tiles of gemm_glds.hip) against the fp32 PyTorch reference: every
split count, ragged M / N, bias + residual + activation, GEGLU, the fused
LayerNorm consumer / row-statistics producer, GroupNorm statistics of a conv,
bit-identical repeats (fixed summation order), counters left clean for the next
launch, and hipGraph capture / replay."""
import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.ops import hip_ops, tuning

pytestmark = pytest.mark.gpu


def rnd(*shape, dev, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def rel_err(y, ref):
    y, ref = y.float(), ref.float()
    return ((y - ref).norm() / (ref.norm() + 1e-12)).item()


class _Force:
    def __init__(self, keys, tile, split):
        self.keys, self.tile, self.split = keys, tile, split

    def __enter__(self):
        t = tuning.table()
        self.old = {k: t.get(k) for k in self.keys}
        for k in self.keys:
            t[k] = [self.tile, self.split, 0.0]

    def __exit__(self, *exc):
        t = tuning.table()
        for k, v in self.old.items():
            if v is None:
                t.pop(k, None)
            else:
                t[k] = v


@pytest.mark.parametrize("tile", [14, 18, 11, 12, 26, 36])
@pytest.mark.parametrize("split", [1, -2, -4, -8])
@pytest.mark.parametrize("M,N,K", [(128, 1280, 1280), (512, 640, 5120), (130, 200, 1024)])
def test_fixup_matches_fp32(gpu, tile, split, M, N, K):
    torch.manual_seed(M + N + K + tile - split)
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    r = rnd(M, N, dev=gpu)
    with _Force([f"g:{M}:{N}:{K}:2"], tile, split):
        y = hip_ops.gemm(a, w, b, r, "silu")
        y2 = hip_ops.gemm(a, w, b, r, "silu")
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), r.float().cpu(), "silu")
    assert rel_err(y.cpu(), ref) < 1e-2
    assert torch.equal(y, y2)  # split-order sum; counters re-zeroed by the previous launch


@pytest.mark.parametrize("tile", [11, 14])
def test_fixup_geglu(gpu, tile):
    M, N, K = 512, 2560, 1280
    a, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5), rnd(N, dev=gpu)
    with _Force([f"g:{M}:{N}:{K}:3"], tile, -4):
        y = hip_ops.gemm(a, w, b, None, "geglu")
    ref = ops._ref_gemm(a.float().cpu(), w.float().cpu(), b.float().cpu(), None, "geglu")
    assert rel_err(y.cpu(), ref) < 1e-2


@pytest.mark.parametrize("tile", [14, 12])
def test_fixup_fused_layernorm_chain(gpu, tile):
    """Row-statistics producer -> fused-LN consumer, both split with the fixup."""
    M, C, N = 512, 1280, 1280
    x, w0 = rnd(M, C, dev=gpu), rnd(C, C, dev=gpu, scale=C ** -0.5)
    w1, b1 = rnd(N, C, dev=gpu, scale=C ** -0.5), rnd(N, dev=gpu)
    gam, bet = rnd(C, dev=gpu) + 1.0, rnd(C, dev=gpu)
    wf, colsum, bf = ops.fold_layer_norm(w1, b1, gam, bet)
    with _Force([f"g:{M}:{C}:{C}:0", f"g:{M}:{N}:{C}:0"], tile, -4):
        h = hip_ops.gemm(x, w0, None, None, None, row_stats=True)
        y = hip_ops.gemm(h, wf, bf, None, None, ln=(h._csk_rows, colsum, 1e-5))
    hf = h.float().cpu()
    ln = torch.nn.functional.layer_norm(hf, (C,), gam.float().cpu(), bet.float().cpu(), 1e-5)
    ref = ln @ w1.float().cpu().t() + b1.float().cpu()
    assert rel_err(h.cpu(), x.float().cpu() @ w0.float().cpu().t()) < 1e-2
    assert rel_err(y.cpu(), ref) < 1.5e-2


@pytest.mark.parametrize("tile,split", [(14, -4), (26, -2), (12, -8)])
def test_fixup_conv_gn_stats(gpu, tile, split):
    """A split 3x3 conv (the 8x8 / 16x16 UNet levels) with GroupNorm statistics
    from the last split's epilogue feeding the fused GN."""
    B, H, W, Cin, Cout = 2, 16, 16, 640, 640
    x = rnd(B, H, W, Cin, dev=gpu)
    wt = rnd(Cout, Cin, 3, 3, dev=gpu, scale=(9 * Cin) ** -0.5)
    wp = ops.pack_conv_weight(wt)
    bias = rnd(Cout, dev=gpu)
    g, bb = rnd(Cout, dev=gpu) + 1.0, rnd(Cout, dev=gpu)
    with _Force([f"c:{B}:{H}:{W}:{Cin}:{Cout}:3:1:0"], tile, split):
        y = hip_ops.conv2d(x, wp, bias, 1, 1, None, False, None, gn_stats=True)
    assert getattr(y, "_csk_gn", None) is not None
    ref = ops._ref_conv2d(x.float().cpu(), wp.float().cpu(), bias.float().cpu(), 1, 1, None, False, None)
    assert rel_err(y.cpu(), ref) < 1e-2
    fused = hip_ops.group_norm(y, g, bb, 32, 1e-5, True)
    gref = ops._ref_group_norm(y.float().cpu(), g.float().cpu(), bb.float().cpu(), 32, 1e-5, True)
    assert rel_err(fused.cpu(), gref) < 1e-2


def test_fixup_graph_replay(gpu):
    M, N, K = 128, 1280, 5120
    a, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=K ** -0.5)
    with _Force([f"g:{M}:{N}:{K}:0"], 14, -8):
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
        eager = hip_ops.gemm(a, w)  # eager launch after the replays: the stream's counters are clean
    assert torch.equal(out, ref)
    assert torch.equal(eager, ref)
