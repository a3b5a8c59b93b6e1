"""Fused cross-attention sub-block (csrc/kernels/xattn.hip; SURVEY K8+K9+K11):
x + Attn2(LayerNorm2(x)) of an SD transformer block in one kernel.  CPU: the
folded-LayerNorm reference equals the unfused composition (LayerNorm ->
to_q -> softmax attention over the context K/V -> to_out + residual).  GPU:
the HIP kernel against that fp32 composition, its row statistics against the
output's, and the transformer block with and without the fused path."""
import pytest
import torch

from chiaswarm_amd import ops
from chiaswarm_amd.models.layers import BasicTransformerBlock, init_random_


@pytest.fixture(autouse=True)
def _any_grid(monkeypatch):
    """Numerics run the fused kernel on small grids too (the product gates it
    on >= XATTN_MIN_WG workgroups)."""
    from chiaswarm_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "XATTN_MIN_WG", 0)


def test_xattn_grid_gate_cpu(monkeypatch):
    """The fused block runs for the CFG-batch-8 64x64 level (256 workgroups),
    the unfused chain for CFG batch 2 (64)."""
    from chiaswarm_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "XATTN_MIN_WG", 256)
    kv = torch.empty(8, 77, 2, 5, 64, dtype=torch.bfloat16)
    assert hip_ops.xattn_ok(torch.empty(8, 4096, 320, dtype=torch.bfloat16), kv, 4096)
    assert not hip_ops.xattn_ok(torch.empty(2, 4096, 320, dtype=torch.bfloat16), kv, 4096)


def _unfused(x, blk, kv):
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
    o = (att @ v.transpose(1, 2)).transpose(1, 2).reshape(b, s, c)
    return o @ a2.to_out[0].weight.float().t() + a2.to_out[0].bias.float() + x.float()


def _setup(dev, dtype, B=2, S=256, C=320, Skv=77, ctx_dim=1024, seed=0):
    torch.manual_seed(seed)
    blk = BasicTransformerBlock(C, C // 64, 64, ctx_dim).to(dev)
    init_random_(blk, seed=seed)
    with torch.no_grad():  # non-trivial LayerNorm affine
        blk.norm2.weight.uniform_(0.5, 1.5)
        blk.norm2.bias.normal_(0, 0.2)
    blk = blk.to(dtype)
    x = (torch.randn(B, S, C, device=dev) * 2 + 0.5).to(dtype)
    ctx = torch.randn(B, Skv, ctx_dim, device=dev).to(dtype)
    kv = blk.attn2.context_kv(ctx)
    return blk, x, kv


def test_folded_reference_matches_unfused_cpu():
    blk, x, kv = _setup("cpu", torch.float32)
    a2 = blk.attn2
    w2, colsum, b2 = ops.fold_layer_norm(a2.to_q.weight, a2.to_q.bias, blk.norm2.weight, blk.norm2.bias)
    with ops.ops_mode("reference"):
        y = ops.xattn_block(x, w2, colsum, b2, kv, a2.to_out[0].weight, a2.to_out[0].bias, blk.norm2.eps, a2.scale,
                            x.shape[1])
    ref = _unfused(x, blk, kv)
    assert ((y - ref).norm() / ref.norm()).item() < 1e-5


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("B,S,Skv", [(2, 256, 77), (8, 4096, 77), (1, 128, 1), (3, 384, 80), (2, 512, 40)])
def test_xattn_block_kernel_vs_fp32(gpu, B, S, Skv, waves):
    from chiaswarm_amd.ops import _lib, hip_ops

    blk, x, kv = _setup(gpu, torch.bfloat16, B=B, S=S, Skv=Skv)
    a2 = blk.attn2
    w2, colsum, b2 = ops.fold_layer_norm(a2.to_q.weight, a2.to_q.bias, blk.norm2.weight, blk.norm2.bias)
    assert hip_ops.xattn_ok(x, kv, S)
    _lib.call("csk_set_xattn_waves", waves)
    hip_ops._xattn_waves_applied[0] = waves
    try:
        y = hip_ops.xattn_block(x, w2, colsum, b2, kv, a2.to_out[0].weight, a2.to_out[0].bias, blk.norm2.eps,
                                a2.scale, S)
        torch.cuda.synchronize()
    finally:
        _lib.call("csk_set_xattn_waves", hip_ops.XATTN_WAVES)
        hip_ops._xattn_waves_applied[0] = hip_ops.XATTN_WAVES
    ref = _unfused(x.cpu().float(), blk.cpu().float(), kv.cpu().float())
    blk.to(gpu)
    # the residual dominates y: bound the attention branch on its own too
    assert rel(y.cpu(), ref) < 1e-2
    assert rel(y.cpu().float() - x.cpu().float(), ref - x.cpu().float()) < 2e-2
    rp, nparts, pcols = y._csk_rows
    assert nparts == 1 and pcols == 320
    st = rp.view(-1, 2).cpu()
    yf = y.float().view(-1, 320).cpu()
    assert torch.allclose(st[:, 0], yf.mean(1), atol=2e-3, rtol=1e-3)
    assert torch.allclose(st[:, 1], ((yf - yf.mean(1, keepdim=True)) ** 2).sum(1), rtol=2e-3, atol=1e-2)


@pytest.mark.gpu
def test_transformer_block_fused_vs_unfused(gpu):
    """The BasicTransformerBlock takes the fused path for C = 320 with per-request
    K/V and matches its own unfused HIP path and the fp32 twin."""
    from chiaswarm_amd.ops import hip_ops

    blk, x, kv = _setup(gpu, torch.bfloat16, B=2, S=1024)
    ctx = None
    y_fused = blk(x, ctx=ctx, kv=kv)
    hip_ops.XATTN_FUSED = False
    try:
        y_plain = blk(x, ctx=ctx, kv=kv)
    finally:
        hip_ops.XATTN_FUSED = True
    assert rel(y_fused, y_plain) < 2e-2
