"""Cross-attention query projection with the attention in its epilogue
(csrc/kernels/gemm_common.h gemm_attn_epilogue, csk_gemm_ln_attn; SURVEY K8 +
K9 + K11) for the C = 640 / 1280 transformer blocks (SD2.1 32x32 / 16x16
levels, SDXL): O = softmax((LN(x) Wq^T + bq) * scale) K^T) V, one head per
128x64 tile.  CPU: the composed reference equals LN -> to_q -> attention.
GPU: the HIP kernel against that fp32 composition with the LayerNorm folded
(producer row statistics) and unfolded, and whole transformer blocks with the
fused path on and off."""
import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.models.layers import BasicTransformerBlock, init_random_


def _ref_o(x, blk, kv):
    """fp32: LayerNorm2 -> to_q -> softmax attention over the context K/V."""
    a2 = blk.attn2
    h = torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), blk.norm2.weight.float(), blk.norm2.bias.float(),
                                       blk.norm2.eps)
    q = h @ a2.to_q.weight.float().t()
    if a2.to_q.bias is not None:
        q = q + a2.to_q.bias.float()
    b, s, c = x.shape
    H, D = kv.shape[3], kv.shape[4]
    k, v = kv[:, :, 0].float(), kv[:, :, 1].float()
    att = torch.softmax(q.view(b, s, H, D).transpose(1, 2) @ k.permute(0, 2, 3, 1) * a2.scale, -1)
    return (att @ v.transpose(1, 2)).transpose(1, 2).reshape(b, s, c)


def _setup(dev, dtype, B=2, S=256, C=640, Skv=77, ctx_dim=1024, seed=0):
    torch.manual_seed(seed)
    blk = BasicTransformerBlock(C, C // 64, 64, ctx_dim).to(dev)
    init_random_(blk, seed=seed)
    with torch.no_grad():  # non-trivial LayerNorm affine and query bias
        blk.norm2.weight.uniform_(0.5, 1.5)
        blk.norm2.bias.normal_(0, 0.2)
    blk = blk.to(dtype)
    x = (torch.randn(B, S, C, device=dev) * 2 + 0.5).to(dtype)
    ctx = torch.randn(B, Skv, ctx_dim, device=dev).to(dtype)
    kv = blk.attn2.context_kv(ctx)
    return blk, x, kv


@pytest.fixture
def any_grid(monkeypatch):
    """Numerics tests run the fused path on small grids too (the product gates
    it on >= 256 tiles, hip_ops.QATTN_MIN_TILES)."""
    from chiaswarm_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "QATTN_MIN_TILES", 0)


def test_qattn_grid_gate_cpu():
    """The fused path is taken for the CFG-batch-8 SD2.1 blocks and the SDXL
    blocks (>= 256 tiles) and not for the CFG-batch-2 SD2.1 ones."""
    from chiaswarm_amd.ops import hip_ops

    def ok(B, S, C):
        x = torch.empty(B, S, C, dtype=torch.bfloat16)
        kv = torch.empty(B, 77, 2, C // 64, 64, dtype=torch.bfloat16)
        return hip_ops.qattn_ok(x, kv, S)

    assert ok(8, 1024, 640) and ok(8, 256, 1280)  # SD2.1 batch 4 (CFG 8): 32x32 / 16x16 levels
    assert ok(2, 1024, 1280) and ok(2, 4096, 640)  # SDXL batch 1 (CFG 2)
    assert not ok(2, 1024, 640) and not ok(2, 256, 1280)  # SD2.1 batch 1: 160 / 80 tiles
    assert not ok(8, 64, 1280)  # 8x8 level: 64 rows per sample, no whole 128-row tiles


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_composed_reference_matches_unfused_cpu():
    blk, x, kv = _setup("cpu", torch.float32)
    a2 = blk.attn2
    with ops.ops_mode("reference"):
        o = ops.layer_norm_gemm_attn(x, blk.norm2, a2.to_q.weight, a2.to_q.bias, None, kv, a2.scale, x.shape[1])
    assert rel(o, _ref_o(x, blk, kv)) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [19, 12])
@pytest.mark.parametrize("B,S,C,Skv", [(2, 1024, 640, 77), (2, 256, 1280, 77), (1, 128, 1280, 1), (3, 384, 640, 80),
                                       (2, 512, 1280, 40)])
def test_gemm_attn_kernel_vs_fp32(gpu, any_grid, B, S, C, Skv, tile):
    """Unfolded (plain query projection of LayerNorm'd rows) and folded
    (LayerNorm from the producer's row statistics inside the GEMM)."""
    from chiaswarm_amd.ops import hip_ops

    blk, x, kv = _setup(gpu, torch.bfloat16, B=B, S=S, C=C, Skv=Skv)
    a2 = blk.attn2
    assert hip_ops.qattn_ok(x, kv, S)
    import copy

    twin = copy.deepcopy(blk).cpu().float()  # Module.float() is in place: keep blk bf16 on the GPU
    ref = _ref_o(x.cpu().float(), twin, kv.cpu().float())
    M = B * S
    xn = ops.layer_norm(x, blk.norm2.weight, blk.norm2.bias, blk.norm2.eps)
    o = hip_ops.gemm_attn(xn.reshape(M, C), a2.to_q.weight, a2.to_q.bias, kv, a2.scale, S, tile=tile)
    assert rel(o.view(B, S, C).cpu(), ref) < 2e-2
    # LayerNorm folded: x produced by a GEMM that emits row statistics
    x1 = ops.gemm(x, blk.attn1.to_out[0].weight, None, row_stats=True)
    w2, colsum, b2 = ops.fold_layer_norm(a2.to_q.weight, a2.to_q.bias, blk.norm2.weight, blk.norm2.bias)
    o2 = hip_ops.gemm_attn(x1.reshape(M, C), w2, b2, kv, a2.scale, S,
                           ln=(x1._csk_rows, colsum, float(blk.norm2.eps)), tile=tile)
    ref2 = _ref_o(x1.cpu().float(), twin, kv.cpu().float())
    assert rel(o2.view(B, S, C).cpu(), ref2) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("C,S", [(640, 1024), (1280, 256)])
def test_transformer_block_qattn_vs_unfused(gpu, any_grid, C, S):
    """The BasicTransformerBlock takes the attention-epilogue path for the
    C = 640 / 1280 blocks and matches its own unfused HIP path and the fp32
    twin."""
    import copy

    from chiaswarm_amd.models.layers import prepare_model
    from chiaswarm_amd.ops import hip_ops

    blk, x, kv = _setup(gpu, torch.bfloat16, B=2, S=S, C=C)
    prepare_model(blk)
    x = ops.gemm(x, blk.attn1.to_out[0].weight, None, row_stats=True)  # carries row statistics
    n0 = hip_ops.QATTN_STATS[0]
    y_fused = blk(x, kv=kv)
    assert hip_ops.QATTN_STATS[0] - n0 == 1
    hip_ops.QATTN = False
    try:
        y_plain = blk(x, kv=kv)
    finally:
        hip_ops.QATTN = True
    assert rel(y_fused, y_plain) < 2e-2
    twin = copy.deepcopy(blk).float()
    with ops.ops_mode("reference"):
        ref = twin(x.float(), kv=kv.float())
    assert rel(y_fused, ref) < 2e-2
