"""ctypes bindings of the gfx950 kernels in libcsk.so.

Every function allocates its output with the torch caching allocator and
launches on torch's current stream (graph-capture safe: no host syncs, no
hipMalloc).  Shape/stride preconditions are checked on the host BEFORE launch
so a bad call raises here instead of faulting the GPU.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib, tuning
from ._lib import c_float, c_int, c_int64, c_void_p, sig

ACT = {None: 0, "none": 0, "gelu": 1, "silu": 2, "geglu": 3, "quick_gelu": 4}

sig("csk_gemm", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
    c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_int, c_int, c_void_p, c_void_p)
sig("csk_conv2d", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
    c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
    c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p)
sig("csk_gemm_ln", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
    c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p,
    c_void_p, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p)
sig("csk_conv2d_ex", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
    c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
    c_int, c_int, c_int, c_int, c_float, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p)
sig("csk_group_norm_part", c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
    c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_void_p)
sig("csk_group_norm_part2", c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
    c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_void_p)


# ---------------------------------------------------------------------------
# GroupNorm statistics fused into producer epilogues
# ---------------------------------------------------------------------------
GN_FINE = 0  # mirrors the library's g_gn_fine (set_gn_fine)


def set_gn_fine(v: int):
    global GN_FINE
    GN_FINE = int(v)
    _lib.call("csk_set_gn_fine", GN_FINE)


GN_TARGET_WG = 512  # GroupNorm apply/stats workgroups per call (rows per chunk follow); 512: -0.05 ms/step vs 1024 (tools/abstep.py gnwgN, profiles/unet_step_ab_gnwg_r3e.txt)
SPLITK_GN_SEG = 64  # gemm_common.h SPLITK_GN_SEG: segment rows of the split-K reduce's GN statistics
SPLITK_GN = True  # split-K producers emit GN statistics from their reduce (tools/abstep.py arms skgn0 / skgn1)


def _gn_seg(tile, split, rows_per_b, M, code, N=8):
    """Rows per fused-GN statistics segment (fine: the epilogue's column pass
    splits each BM-row tile into 256/BN segments of BM*BN/256 rows; else one
    segment per tile; split-K: the reduce kernel's SPLITK_GN_SEG rows), or 0."""
    bm, bn = tuning.TILES.get(tile, (0, 0))
    if code == 3 or bm == 0 or rows_per_b <= 0:
        return 0
    if split > 1:  # (split < 0, the in-kernel fixup, writes the tile's own segments)
        if not SPLITK_GN:
            return 0
        s = SPLITK_GN_SEG
        return s if rows_per_b % s == 0 and M % s == 0 and N % 8 == 0 else 0
    if rows_per_b % bm or M % bm:
        return 0
    seg = bm * bn // 256 if GN_FINE else bm
    band = bm // tuning.EPI_WM.get(tile, 2) if (bm > 128 or bn == 160) else bm  # epilogue row band (epi_passes)
    return min(seg, band)


def _ws(split, M, N, device):
    """fp32 split-K workspace: [split][M][N] for the reduce kernel; split < 0
    (in-kernel fixup, gemm_common.h splitk_fixup) stores whole padded tiles, at
    most (M + 255) x (N + 255) outputs per split for every tile geometry"""
    if split > 1:
        return torch.empty(split * M * N, dtype=torch.float32, device=device)
    if split < 0:
        return torch.empty(-split * (M + 255) * (N + 255), dtype=torch.float32, device=device)
    return None


def _gn_part(M, N, seg, device):
    return torch.empty((M // seg) * N * 2, dtype=torch.float32, device=device)
sig("csk_axpby", c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_void_p)
ACT.update({"lrelu": 5, "lrelu0.1": 6, "tanh": 7, "relu": 8, "lrelu0.01": 9, "elu": 10, "gelu_tanh": 11})
sig("csk_group_norm", c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
    c_int, c_int, c_float, c_int, c_int, c_void_p)
sig("csk_layer_norm", c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p)
ATTN_VARIANT = int(os.environ.get("CSK_ATTN", "0"))  # 0 auto, 1 plain, 2 pipelined (D <= 64)
sig("csk_attention", c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_int64), c_int, c_int, c_int, c_int,
    c_int, c_float, c_int, c_int, c_void_p, c_void_p)
sig("csk_silu", c_void_p, c_void_p, c_int64, c_void_p)
sig("csk_canny", c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_float, c_void_p, c_void_p)
sig("csk_add", c_void_p, c_void_p, c_void_p, c_int64, c_void_p)
sig("csk_sched_step", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
    c_float, c_float, c_float, c_float, c_float, c_float, c_float, c_int, c_void_p)
sig("csk_vae_post", c_void_p, c_void_p, c_int64, c_void_p)
sig("csk_loop_prologue", c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p)
sig("csk_sched_loop", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int64,
    c_int, c_void_p)
LOOP_COEF_STRIDE = 12  # elementwise.hip: {p, q, A, B, C, D, s_next, g, g2, -, -, -} per step
sig("csk_pad_channels", c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p)
sig("csk_set_gn_prologue_max", c_int)
sig("csk_debug_selftest", c_int, c_void_p)  # CSK_DEBUG builds: one deliberate record (tests)
sig("csk_set_gn_lds", c_int)
sig("csk_set_sw_odd", c_int)
sig("csk_set_epi_band", c_int)
sig("csk_set_epi_nt", c_int)
sig("csk_set_skr_unroll", c_int)
sig("csk_set_short_kv_variant", c_int)
sig("csk_set_short_kv_rows", c_int)
sig("csk_set_attn32", c_int)
sig("csk_xattn_block", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
    c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_void_p)
sig("csk_attention_fa", c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_int64), c_int, c_int, c_int, c_int,
    c_int, c_float, c_int, c_void_p)
sig("csk_set_attn_fa", c_int)
sig("csk_attn_fa_ok", c_int, c_int, c_int, c_int, c_int, c_int, c_int)
sig("csk_attention_split", c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_int64), c_int, c_int, c_int, c_int,
    c_int, c_float, c_int, c_void_p, c_void_p, c_void_p)
sig("csk_dup2", c_void_p, c_void_p, c_int64, c_void_p)
sig("csk_row_bcast", c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p)
sig("csk_set_ln_in_kernel", c_int)
sig("csk_set_gn_finalize_wg", c_int)
sig("csk_set_gn_cb", c_int)
sig("csk_set_gn_cb_mult", c_int)
sig("csk_set_gn_cb_small", c_int)
sig("csk_set_gn_fine", c_int)
sig("csk_timestep_embedding", c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float, c_void_p)


def timestep_embedding(t, batch, dim, flip_sin_to_cos=True, shift=0.0, max_period=10000.0):
    """bf16 [batch, dim] sinusoidal embedding of fp32 timesteps t ([1] broadcast or [batch])."""
    t = t.reshape(-1)
    if t.dtype != torch.float32 or not t.is_contiguous():
        t = t.float().contiguous()
    if t.numel() not in (1, batch):
        raise ValueError(f"timestep_embedding: {t.numel()} timesteps for batch {batch}")
    y = torch.empty((batch, dim), dtype=torch.bfloat16, device=t.device)
    _lib.call("csk_timestep_embedding", _p(y), _p(t), 0 if t.numel() == 1 else 1, batch, dim,
              int(bool(flip_sin_to_cos)), float(shift), float(max_period), _s())
    return y


def _bf16(t, name):
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name}: HIP kernels take bfloat16, got {t.dtype}")


def _p(t):
    return None if t is None else t.data_ptr()


def _s():
    return _lib.stream_ptr()


def _round8(n):
    return (n + 7) // 8 * 8


def pad_last(x: torch.Tensor, n: int) -> torch.Tensor:
    """Zero-pad the last (contiguous) dim of a bf16 tensor to n."""
    c = x.shape[-1]
    if c == n:
        return x
    x = x.contiguous()
    y = torch.empty(x.shape[:-1] + (n,), dtype=x.dtype, device=x.device)
    rows = x.numel() // c
    _lib.call("csk_pad_channels", _p(y), _p(x), rows, c, n, _s())
    return y


# ---------------------------------------------------------------------------
def gemm(a2, w, bias=None, residual=None, act=None, out=None, gn_rows=0, ln=None, row_stats=False):
    """``gn_rows`` > 0: also produce GroupNorm statistics of the output for a
    consumer GN (rows per sample = gn_rows), attached as ``out._csk_gn``.

    ``row_stats``: also produce per-row (mean, M2) partials of the output for a
    consumer's fused LayerNorm, attached as ``out._csk_rows = (part, nparts, pcols)``.
    ``ln = (rows, colsum, eps)``: this GEMM's input rows are LayerNorm'd on the
    fly — ``w``/``bias`` are the gamma/beta-folded weights (``fold_layer_norm``)
    and ``rows`` the producer's ``_csk_rows``."""
    _bf16(a2, "gemm.a")
    _bf16(w, "gemm.w")
    M, K = a2.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError(f"gemm: K mismatch {a2.shape} x {w.shape}")
    if a2.stride(1) != 1 or a2.stride(0) % 8 != 0 or (a2.data_ptr() % 16):
        a2 = a2.contiguous()
    if w.stride(1) != 1 or w.stride(0) % 8 != 0:
        w = w.contiguous()
    if K % 8 != 0:
        kp = _round8(K)
        a2 = pad_last(a2, kp)
        w = pad_last(w, kp)
        K = kp
    code = ACT[act]
    n_out = N // 2 if code == 3 else N
    if out is None:
        out = torch.empty((M, n_out), dtype=torch.bfloat16, device=a2.device)
    if residual is not None:
        residual = residual.reshape(M, n_out)
        _bf16(residual, "gemm.residual")
        if not residual.is_contiguous():
            residual = residual.contiguous()
    if bias is not None:
        _bf16(bias, "gemm.bias")
    lda, ldb = a2.stride(0), w.stride(0)

    def run(tile, split, part=None):
        ws = _ws(split, M, N, a2.device)
        _lib.call("csk_gemm", _p(out), _p(a2), _p(w), _p(bias), None, _p(residual),
                  M, N, K, lda, ldb, n_out, n_out, 1, code, 1.0, _p(part), tile, split, _p(ws), _s())

    tile, split = tuning.choose(f"g:{M}:{N}:{K}:{code}", M, N, K, run)
    if split < 0 and tile not in tuning.GLDS:
        split = 1  # the in-kernel fixup exists in the LDS-DMA tiles only
    if ln is not None or row_stats:
        if split > 1:  # the split-K reduce has no LN / row-statistics epilogue
            tile, split = (19 if N <= 1280 else 20), 1
        # mirror the library's own tile substitutions: the row-statistics slabs
        # (and the buffer sized for them below) follow the tile that actually runs
        if tile in (25, 26, 31, 32, 33, 34):  # 160-column and 8-wave tiles: no LN / row statistics -> tile 11
            tile = 11
        elif tile == 36:  # 64x160 -> 64x128 (gemm_glds.hip csk_gemm_glds_launch)
            tile = 13
        if ln is None and code == 3:
            row_stats = False
    seg = _gn_seg(tile, split, gn_rows, M, code, N) if gn_rows and out.is_contiguous() else 0
    part = _gn_part(M, N, seg, a2.device) if seg else None
    if ln is None and not row_stats:
        run(tile, split, part)
    else:
        bn = tuning.TILES[tile][1]
        rp = torch.empty(-(-N // bn) * M * 2, dtype=torch.float32, device=a2.device) if row_stats else None
        lp = lc = rowbuf = None
        nparts = pcols = 0
        eps = 0.0
        if ln is not None:
            (lp, nparts, pcols), lc, eps = ln
            if K % 8 or nparts * pcols < K or lp.numel() < nparts * M * 2:
                raise ValueError("gemm: fused LayerNorm statistics do not match the input")
            rowbuf = torch.empty(M * 2, dtype=torch.float32, device=a2.device)
        _lib.call("csk_gemm_ln", _p(out), _p(a2), _p(w), _p(bias), None, _p(residual),
                  M, N, K, lda, ldb, n_out, n_out, 1, code, 1.0, _p(part), _p(lp), _p(lc), nparts, pcols,
                  float(eps), _p(rowbuf), _p(rp), tile, 1, None, _s())
        if rp is not None:
            out._csk_rows = (rp, -(-N // bn), bn)
    if part is not None:
        out._csk_gn = (part, seg)
    return out


# Cross-attention query projection with the attention in the GEMM epilogue
# (gemm_common.h gemm_attn_epilogue): O = softmax(q K^T * scale) V straight from
# the Q-projection accumulators, one head per 128x64 tile.
sig("csk_gemm_ln_attn", c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
    c_void_p, c_void_p, c_int, c_int, c_float, c_void_p, c_void_p, c_int, c_int, c_float, c_int, c_void_p)
QATTN = os.environ.get("CSK_QATTN", "1") == "1"
# below this many 128x64 tiles the one-head-per-tile grid under-fills the chip
# and the unfused query GEMM + short-KV attention win (CFG batch 2 of SD2.1:
# 80 / 160 tiles, +0.01 ms/step; batch 8: 320 / 640 tiles, -0.09 ms/step,
# profiles/unet_step_ab_qattn_r6s.txt)
QATTN_MIN_TILES = int(os.environ.get("CSK_QATTN_MIN_TILES", "256"))
QATTN_STATS = [0]  # calls (tests assert the fused path ran)


def qattn_ok(x, kv, rows_per_b) -> bool:
    """Shapes the attention-epilogue GEMM takes: head dim 64 (heads = C / 64),
    <= 80 context tokens, 128-row tiles inside one sample."""
    C = x.shape[-1]
    M = x.numel() // C
    return (QATTN and kv is not None and kv.dim() == 5 and kv.shape[2] == 2 and kv.shape[4] == 64
            and kv.shape[3] * 64 == C and 1 <= kv.shape[1] <= 80 and C % 64 == 0 and rows_per_b % 128 == 0
            and M % rows_per_b == 0 and kv.shape[0] >= M // rows_per_b
            and (M // 128) * (C // 64) >= QATTN_MIN_TILES)


def gemm_attn(a2, w, bias, kv, scale, rows_per_b, ln=None, tile=None):
    """Attention output O [M, C] of the cross-attention whose query projection
    is ``a2 @ w^T + bias`` (``ln = (rows, colsum, eps)``: LayerNorm folded as in
    ``gemm``), over the per-request ``kv`` [Bc, Skv, 2, H, 64]."""
    _bf16(a2, "gemm_attn.a")
    _bf16(w, "gemm_attn.w")
    _bf16(kv, "gemm_attn.kv")
    M, K = a2.shape
    N = w.shape[0]
    if w.shape[1] != K or K % 8:
        raise ValueError(f"gemm_attn: K mismatch {a2.shape} x {w.shape}")
    if a2.stride(1) != 1 or a2.stride(0) % 8 != 0 or (a2.data_ptr() % 16):
        a2 = a2.contiguous()
    w = w.contiguous()
    kv = kv.contiguous()
    if bias is not None:
        _bf16(bias, "gemm_attn.bias")
        bias = bias.contiguous()
    # 128x64 row-layout tile: 3-stage (12) for the long-K C = 1280 projections,
    # 2-stage (19) otherwise (18.3 vs 19.1 us at K = 1280, 21.7 vs 18.9 at K = 640;
    # profiles/qattnbench_r7a.txt)
    if tile is None:
        tile = 12 if K >= 1280 else 19
    elif tile not in (12, 19):
        raise ValueError("gemm_attn: tile 12 or 19")
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a2.device)
    lp = lc = rowbuf = None
    nparts = pcols = 0
    eps = 0.0
    if ln is not None:
        (lp, nparts, pcols), lc, eps = ln
        if nparts * pcols < K or lp.numel() < nparts * M * 2:
            raise ValueError("gemm_attn: fused LayerNorm statistics do not match the input")
        rowbuf = torch.empty(M * 2, dtype=torch.float32, device=a2.device)
    QATTN_STATS[0] += 1
    _lib.call("csk_gemm_ln_attn", _p(out), _p(a2), _p(w), _p(bias), M, N, K, a2.stride(0), w.stride(0), N,
              int(rows_per_b), _p(lp), _p(lc), nparts, pcols, float(eps), _p(rowbuf), _p(kv), int(kv.shape[0]),
              int(kv.shape[1]), float(scale), tile, _s())
    return out


def _pix_stride(t):
    """Pixel stride of an NHWC tensor / channel-slice view (None if not NHWC-strided)."""
    B, H, W, C = t.shape
    s = t.stride()
    if s[3] != 1:
        return None
    ps = s[2]
    if (W > 1 and s[2] != ps) or (H > 1 and s[1] != W * ps) or (B > 1 and s[0] != H * W * ps):
        return None
    return ps


# Persistent halo-tile conv for 3x3 / stride-1 / Cout = 16 / 32 / 64 and < 16
# (csrc/kernels/conv_tile.hip: the Real-ESRGAN dense-block convs, its x2
# up-convs and RGB conv_last); CSK_CONV_TILE=0 keeps the implicit GEMM
sig("csk_conv_tile_ok2", c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int)
sig("csk_conv_tile2", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
    c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_int, c_int, c_void_p)
CONV_TILE = os.environ.get("CSK_CONV_TILE", "1") == "1"
CONV_TILE64 = os.environ.get("CSK_CONV_TILE64", "1") == "1"  # the Cout = 64 instance: 1.2x faster than the GEMM (profiles/conv_tile64_r5.txt)
# Cout <= 16 (16-wide instance; e.g. the x4 upscaler's 64 -> 3 conv_last at 2048^2) on
# maps of at least this many output pixels (below it the grid is a fraction of the chip)
CONV_TILE_NARROW_MIN_PX = int(os.environ.get("CSK_CONV_TILE_NARROW_MIN_PX", str(1 << 18)))
CONV_TILE_STATS = [0]  # calls (tests assert the kernel ran)


def conv2d(x, wp, bias, stride, padding, residual, up2x, bias2d, act=None, out_scale=1.0, out=None, dilation=1,
           gn_stats=False, residual2=None, res_scale=1.0, out_u8=False):
    """NHWC conv.  ``x``, ``residual`` and ``out`` may be channel-slice views of
    wider NHWC buffers (last dim contiguous): the kernel takes their pixel
    strides, so dense/concat blocks need no copies.  ``residual2`` /
    ``res_scale`` (y = ... * out_scale + res_scale * residual + residual2, ``out``
    may alias ``residual2``) run in the halo-tile kernel's epilogue, elsewhere as
    one extra pass.  ``out_u8``: uint8 image output round(clamp(y, 0, 1) * 255)
    (the halo-tile kernel stores it directly for Cout < 16)."""
    from . import conv_out_size, norm_padding

    _bf16(x, "conv.x")
    _bf16(wp, "conv.w")
    B, H, W, Cin = x.shape
    xs = _pix_stride(x)
    if xs is None or xs % 8 != 0 or Cin % 8 != 0 or x.data_ptr() % 16:
        x = x.contiguous()
        xs = Cin
    Cout, kh, kw, Cw = wp.shape
    if Cw != Cin:
        raise ValueError(f"conv2d: Cin mismatch {tuple(x.shape)} vs {tuple(wp.shape)}")
    if Cin % 8 != 0:
        cp = _round8(Cin)
        x = pad_last(x, cp)
        wp = pad_last(wp.contiguous(), cp)
        Cin = xs = cp
    wp = wp.contiguous()
    pt, pl, pb, pr = norm_padding(padding)
    Ho, Wo = conv_out_size(H, W, kh, kw, stride, padding, up2x, dilation)
    if out_u8:
        return _conv2d_u8(x, wp, bias, stride, padding, residual, up2x, bias2d, act, out_scale, out, dilation,
                          residual2, res_scale, Ho, Wo)
    if out is None:
        out = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=x.device)
    ys = _pix_stride(out)
    if out.shape != (B, Ho, Wo, Cout) or ys is None:
        raise ValueError(f"conv2d out {tuple(out.shape)} / strides unsupported")
    rs = 0
    if residual is not None:
        if residual.shape != out.shape:
            raise ValueError(f"conv2d residual {tuple(residual.shape)} != {tuple(out.shape)}")
        rs = _pix_stride(residual)
        if rs is None:
            residual = residual.contiguous()
            rs = Cout
    b2s = 0
    if bias2d is not None:
        # a column slice of the UNet's one batched time-embedding GEMM: pass its
        # row stride instead of copying it out (one copy kernel per ResNet)
        if bias2d.shape != (B, Cout):
            raise ValueError("conv2d bias2d shape")
        _bf16(bias2d, "conv.bias2d")
        if bias2d.stride(1) != 1 or bias2d.data_ptr() % 16 or bias2d.stride(0) % 8:
            bias2d = bias2d.contiguous()
        b2s = bias2d.stride(0) if B > 1 else Cout
    M, K = B * Ho * Wo, kh * kw * Cin
    code = ACT[act]

    def run(tile, split, part=None):
        ws = _ws(split, M, Cout, x.device)
        _lib.call("csk_conv2d_ex", _p(out), _p(x), _p(wp), _p(bias), _p(bias2d), b2s, _p(residual),
                  B, H, W, Cin, Cout, kh, kw, stride, pt, pl, Ho, Wo, int(bool(up2x)), xs, ys, rs, code,
                  float(out_scale), int(dilation), _p(part), tile, split, _p(ws), _s())

    rs2 = 0
    if residual2 is not None:
        if residual2.shape != out.shape:
            raise ValueError(f"conv2d residual2 {tuple(residual2.shape)} != {tuple(out.shape)}")
        rs2 = _pix_stride(residual2)
        if rs2 is None:
            residual2 = residual2.contiguous()
            rs2 = Cout
    key = f"c:{B}:{H}:{W}:{Cin}:{Cout}:{kh}:{stride}:{int(bool(up2x))}"
    if kh != kw or dilation != 1:
        key += f":{kw}:{dilation}"
    narrow = Cout < 16
    if (CONV_TILE and kh == 3 and kw == 3 and stride == 1 and (pt, pl, pb, pr) == (1, 1, 1, 1) and dilation == 1
            and bias2d is None and not gn_stats
            and code in (0, 2, 5, 6, 8, 9)
            and (Cout == 32 or (Cout == 64 and CONV_TILE64) or (Cout <= 16 and M >= CONV_TILE_NARROW_MIN_PX))
            and (residual is None or (not narrow and rs % 4 == 0 and residual.data_ptr() % 8 == 0))
            and (residual2 is None or (not narrow and rs2 % 4 == 0 and residual2.data_ptr() % 8 == 0))
            and _lib.call_int("csk_conv_tile_ok2", B, Ho, Wo, Cin, Cout, xs, ys, int(bool(up2x))) > 0
            and x.data_ptr() % 16 == 0 and (narrow or out.data_ptr() % 8 == 0) and wp.data_ptr() % 16 == 0):
        # narrow-output 3x3 (the Real-ESRGAN convs): persistent halo-tile kernel
        _lib.call("csk_conv_tile2", _p(out), _p(x), _p(wp), _p(bias), _p(residual), _p(residual2), B, Ho, Wo, Cin,
                  Cout, xs, ys, rs, rs2, code, float(out_scale), float(res_scale), int(bool(up2x)), 0, _s())
        CONV_TILE_STATS[0] += 1
        return out
    if residual2 is not None or res_scale != 1.0:
        # the implicit GEMM's epilogue has one unscaled residual: conv into a
        # temporary, then one combining pass (residual2 is read before out is written)
        y = conv2d(x, wp, bias, stride, padding, None, up2x, bias2d, act, out_scale, None, dilation)
        if residual is not None:
            y = torch.add(y, residual, alpha=res_scale) if res_scale != 1.0 else y + residual
        if residual2 is not None:
            y = y + residual2
        out.copy_(y)
        return out
    tile, split = tuning.choose(key, M, Cout, K, run)
    seg = _gn_seg(tile, split, Ho * Wo, M, code, Cout) if gn_stats and ys == Cout else 0
    part = _gn_part(M, Cout, seg, x.device) if seg else None
    run(tile, split, part)
    if part is not None:
        out._csk_gn = (part, seg)
    return out


def _conv2d_u8(x, wp, bias, stride, padding, residual, up2x, bias2d, act, out_scale, out, dilation, residual2,
               res_scale, Ho, Wo):
    """conv2d with a uint8 image output (``out``: None or a contiguous uint8 [B, Ho, Wo, Cout])."""
    from . import norm_padding

    B, H, W, Cin = x.shape
    Cout = wp.shape[0]
    if out is None:
        out = torch.empty((B, Ho, Wo, Cout), dtype=torch.uint8, device=x.device)
    if out.dtype != torch.uint8 or out.shape != (B, Ho, Wo, Cout) or not out.is_contiguous():
        raise ValueError("conv2d out_u8: out must be a contiguous uint8 [B, Ho, Wo, Cout]")
    xs = _pix_stride(x)
    if (CONV_TILE and Cout < 16 and residual is None and residual2 is None and bias2d is None and stride == 1
            and wp.shape[1:3] == (3, 3) and norm_padding(padding) == (1, 1, 1, 1) and dilation == 1
            and code_ok(act) and B * Ho * Wo >= CONV_TILE_NARROW_MIN_PX and xs is not None
            and x.data_ptr() % 16 == 0 and wp.is_contiguous() and wp.data_ptr() % 16 == 0
            and _lib.call_int("csk_conv_tile_ok2", B, Ho, Wo, Cin, Cout, xs, Cout, int(bool(up2x))) > 0):
        _lib.call("csk_conv_tile2", _p(out), _p(x), _p(wp), _p(bias), None, None, B, Ho, Wo, Cin, Cout, xs, Cout,
                  0, 0, ACT[act], float(out_scale), 1.0, int(bool(up2x)), 1, _s())
        CONV_TILE_STATS[0] += 1
        return out
    y = conv2d(x, wp, bias, stride, padding, residual, up2x, bias2d, act, out_scale, None, dilation,
               residual2=residual2, res_scale=res_scale)
    out.copy_((y.float().clamp(0, 1) * 255).round().to(torch.uint8))
    return out


def code_ok(act):
    """activations the halo-tile kernel's epilogue applies"""
    return ACT[act] in (0, 2, 5, 6, 8, 9)


sig("csk_axpby_nhwc", c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int64, c_int, c_float, c_float, c_int,
    c_void_p)


def axpby_nhwc(x, z, a, b, out, act=None):
    """out = act(a*x + b*z) on NHWC channel-slice views (in place allowed; z may be None)."""
    xs, ys = _pix_stride(x), _pix_stride(out)
    zs = _pix_stride(z) if z is not None else 0
    if None in (xs, zs, ys) or (z is not None and x.shape != z.shape) or x.shape != out.shape:
        raise ValueError("axpby_nhwc: operands must be same-shape NHWC views")
    C = x.shape[-1]
    P = x.numel() // C
    if C % 8 or xs % 8 or ys % 8 or zs % 8:
        raise ValueError("axpby_nhwc: channels / pixel strides must be multiples of 8")
    _lib.call("csk_axpby_nhwc", _p(out), ys, _p(x), xs, _p(z), zs, P, C, float(a), float(b), ACT[act], _s())
    return out


def axpby(x, y, a, b, out=None):
    """out = a*x + b*y (bf16, contiguous)."""
    x, y = x.contiguous(), y.contiguous()
    out = torch.empty_like(x) if out is None else out
    _lib.call("csk_axpby", _p(out), _p(x), _p(y), x.numel(), float(a), float(b), _s())
    return out


def group_norm(x, gamma, beta, groups, eps, silu):
    _bf16(x, "group_norm.x")
    x = x.contiguous()
    B, C = x.shape[0], x.shape[-1]
    P = x.numel() // (B * C)
    # a chunk gives every thread >= 4 independent row loads (the kernels' unroll;
    # R = 256 threads / (C/8 vector columns) rows per pass), with <= ~1024
    # workgroups over the whole tensor (each apply workgroup re-merges the
    # statistics partials in its prologue: fewer, longer workgroups amortise it)
    rows = max(1, 256 // max(1, -(-(C // 8) // (2 if C > 2048 else 1))))
    chunk = max(4 * rows, -(-P * B // GN_TARGET_WG))
    nchunk = -(-P // chunk)
    chunk = -(-P // nchunk)
    bstride = 0
    if gamma.dim() == 2:
        if gamma.shape != (B, C) or beta.shape != (B, C):
            raise ValueError("group_norm: per-sample affine must be [B, C]")
        # rows of a wider matrix (e.g. slices of one batched projection) are
        # read in place when both share the row stride
        if gamma.stride(1) != 1 or beta.stride(1) != 1 or gamma.stride(0) != beta.stride(0):
            gamma, beta = gamma.contiguous(), beta.contiguous()
        bstride = gamma.stride(0)
    act = 2 if silu == "gelu" else int(bool(silu))
    y = torch.empty_like(x)
    fused = getattr(x, "_csk_gn", None)
    if fused is not None:
        fpart, seg = fused
        if P % seg == 0 and fpart.numel() == (B * P // seg) * C * 2:
            stat = torch.empty(B * groups * 2, dtype=torch.float32, device=x.device)
            _lib.call("csk_group_norm_part", _p(y), _p(x), None, 0, _p(fpart), seg, _p(stat), _p(gamma), _p(beta),
                      B, P, C, groups, chunk, nchunk, float(eps), act, bstride, _s())
            return y
    part = torch.empty(B * nchunk * groups * 3 + B * groups * 2, dtype=torch.float32, device=x.device)
    _lib.call("csk_group_norm", _p(y), _p(x), None, 0, _p(part), _p(gamma), _p(beta), B, P, C, groups, chunk, nchunk,
              float(eps), act, bstride, _s())
    return y


def group_norm_cat(a, b, gamma, beta, groups, eps, silu):
    """GroupNorm(+SiLU) of the channel concat [a | b] without materialising it
    (UNet skip connections): the apply kernel reads both tensors in place.
    Needs the fused epilogue statistics of both (same segment height);
    returns None otherwise (the caller concatenates)."""
    sa, sb = getattr(a, "_csk_gn", None), getattr(b, "_csk_gn", None)
    GN_CAT_STATS[1] += 1
    if a.shape[:-1] != b.shape[:-1] or not (a.is_contiguous() and b.is_contiguous()):
        return None
    B, Ca, Cb = a.shape[0], a.shape[-1], b.shape[-1]
    C = Ca + Cb
    P = a.numel() // (B * Ca)
    if Ca % 8 or Cb % 8 or gamma.dim() != 1 or C % groups or C > 4096:
        return None
    rows = max(1, 256 // max(1, -(-(C // 8) // (2 if C > 2048 else 1))))
    chunk = max(4 * rows, -(-P * B // GN_TARGET_WG))
    nchunk = -(-P // chunk)
    chunk = -(-P // nchunk)
    y = torch.empty(a.shape[:-1] + (C,), dtype=torch.bfloat16, device=a.device)
    fused = sa is not None and sb is not None and sa[1] == sb[1] and P % sa[1] == 0
    if fused:
        seg = sa[1]
        nseg = sa[0].numel() // (2 * Ca)
        fused = nseg * 2 * Cb == sb[0].numel()
    if fused:  # both producers emitted epilogue statistics: merged from both buffers in place
        stat = torch.empty(B * groups * 2, dtype=torch.float32, device=a.device)
        _lib.call("csk_group_norm_part2", _p(y), _p(a), _p(b), Ca, _p(sa[0]), _p(sb[0]), seg, _p(stat), _p(gamma),
                  _p(beta), B, P, C, groups, chunk, nchunk, float(eps), int(bool(silu)), 0, _s())
    else:  # statistics pass over both tensors in place (e.g. a split-K producer)
        part = torch.empty(B * nchunk * groups * 3 + B * groups * 2, dtype=torch.float32, device=a.device)
        _lib.call("csk_group_norm", _p(y), _p(a), _p(b), Ca, _p(part), _p(gamma), _p(beta), B, P, C, groups, chunk,
                  nchunk, float(eps), int(bool(silu)), 0, _s())
    GN_CAT_STATS[0] += 1
    return y


GN_CAT_STATS = [0, 0]  # (concats normalised in place, attempts)


def layer_norm(x, gamma, beta, eps):
    _bf16(x, "layer_norm.x")
    x = x.contiguous()
    C = x.shape[-1]
    y = torch.empty_like(x)
    _lib.call("csk_layer_norm", _p(y), _p(x), _p(gamma), _p(beta), x.numel() // C, C, float(eps), _s())
    return y


def attention(q, k, v, scale, causal=False, kv_len=None):
    """``kv_len``: optional int32 device tensor [1] = number of valid keys
    (<= k.shape[1]), read by the kernel (graph-capturable KV-cache decode)."""
    for t, n in ((q, "q"), (k, "k"), (v, "v")):
        _bf16(t, "attention." + n)
        if t.stride(-1) != 1:
            raise ValueError("attention: last dim must be contiguous")
    B, Sq, H, D = q.shape
    Skv = k.shape[1]
    if D > 512 or (D > 256 and (causal or kv_len is not None or D % 16)):
        raise ValueError(f"attention: head dim {D} unsupported (<= 256, or <= 512 non-causal, multiple of 16)")
    o = torch.empty((B, Sq, H, D), dtype=torch.bfloat16, device=q.device)
    st = (c_int64 * 12)(*q.stride()[:3], *k.stride()[:3], *v.stride()[:3], *o.stride()[:3])
    if kv_len is not None and (kv_len.dtype != torch.int32 or not kv_len.is_cuda):
        raise TypeError("attention: kv_len must be an int32 device tensor")
    plain = not causal and kv_len is None and ATTN_VARIANT == 0
    if plain and attn_fa_ok(B, H, Sq, Skv, D):  # persistent stream-K kernel (no split path needed)
        _lib.call("csk_attention_fa", _p(o), _p(q), _p(k), _p(v), st, B, H, Sq, Skv, D, float(scale), ATTN_FA_WORKERS,
                  _s())
        return o
    split = attn_kv_split(B, H, Sq, Skv, D) if plain else 1
    if split > 1:
        return attention_split(q, k, v, scale, split, o)
    _lib.call("csk_attention", _p(o), _p(q), _p(k), _p(v), st, B, H, Sq, Skv, D, float(scale), int(bool(causal)),
              ATTN_VARIANT, _p(kv_len), _s())
    return o


def attention_split(q, k, v, scale, split, o=None):
    """d = 64 non-causal attention with the keys split over ``split`` workgroups
    per query block (fp32 partials in a torch workspace, then a combine pass)."""
    B, Sq, H, D = q.shape
    Skv = k.shape[1]
    if D != 64 or not 2 <= split <= 16:
        raise ValueError("attention_split: head dim 64, 2..16 splits")
    if o is None:
        o = torch.empty((B, Sq, H, D), dtype=torch.bfloat16, device=q.device)
    st = (c_int64 * 12)(*q.stride()[:3], *k.stride()[:3], *v.stride()[:3], *o.stride()[:3])
    rows = B * H * Sq
    part_o = torch.empty((split, rows, 64), dtype=torch.float32, device=q.device)
    part_ml = torch.empty((split, rows, 2), dtype=torch.float32, device=q.device)
    _lib.call("csk_attention_split", _p(o), _p(q), _p(k), _p(v), st, B, H, Sq, Skv, D, float(scale), split,
              _p(part_o), _p(part_ml), _s())
    return o


ATTN_FA = os.environ.get("CSK_ATTN_FA", "1") == "1"  # mirrors csk_set_attn_fa (set_attn_fa)
ATTN_FA_WORKERS = 0  # 0: one persistent workgroup per CU; tests pass fewer to force more stream-K cuts


def attn_fa_ok(B, H, Sq, Skv, D) -> bool:
    """Shapes the persistent stream-K d = 64 attention (csrc/kernels/attn_fa.hip) takes."""
    return ATTN_FA and _lib.call_int("csk_attn_fa_ok", B, H, Sq, Skv, D, 0, 0) == 1


def set_attn_fa(on: bool):
    global ATTN_FA
    ATTN_FA = bool(on)
    _lib.call("csk_set_attn_fa", int(ATTN_FA))


def attn_fa_errors() -> int:
    """Merge-protocol spins that gave up since the library loaded (must stay 0)."""
    out = ctypes.c_uint(0)
    fn = _lib.load().csk_attn_fa_errors
    fn.restype = ctypes.c_int
    err = fn(ctypes.byref(out))
    if err:
        raise RuntimeError(f"csk_attn_fa_errors: hipError {err}")
    return int(out.value)


sig("csk_attn_fa_reset")


def attn_fa_health() -> bool:
    """Per-job check of the stream-K attention's merge protocol (called by
    runtime/device.py after every GPU job).  A spin that gave up means a late
    contributor may publish into a slot after its owner released it, so the
    partials of every later launch are suspect: the kernel is switched off for
    this process, its flags are zeroed, and False is returned (the caller fails
    the job and drops the captured graphs, which still launch the kernel)."""
    if attn_fa_errors() == 0:
        return True
    set_attn_fa(False)
    _lib.call("csk_attn_fa_reset")
    return False


ATTN32 = True  # mirrors the library's csk_set_attn32 (set_attn32): the split-KV path runs attn32_kernel only


def set_attn32(on: bool):
    """Turn the 32x32x16 self-attention kernel on / off (A/B and fallback
    switch) in the library AND here: with it off, the key-split path (which
    always runs attn32_kernel) is skipped too."""
    global ATTN32
    ATTN32 = bool(on)
    _lib.call("csk_set_attn32", int(ATTN32))


ATTN_SPLIT_WG = int(os.environ.get("CSK_ATTN_SPLIT_WG", "1024"))  # split the keys below this many workgroups (0: off); 1024 vs 512: -0.045 ms/step at CFG batch 2 (profiles/unet_step_ab_attn_split_wg_b2_r5p.txt)


def attn_kv_split(B, H, Sq, Skv, D) -> int:
    """Key splits for the d = 64 self-attention when its 128-query workgroups
    cannot fill the chip (batch-1 jobs): up to 4."""
    if D != 64 or Skv <= 128 or ATTN_SPLIT_WG <= 0 or not ATTN32:
        return 1
    wg = B * H * -(-Sq // 128)
    split = 1
    # each split keeps >= 16 key blocks: at S = 1024 (16 blocks) the combine and
    # the shorter pipelines cost more than the extra workgroups gain (30.6 vs
    # 22.5 us, profiles/attn_split_r4t.txt); S = 4096 at batch 1-2: 58 vs 75 us
    while wg * split < ATTN_SPLIT_WG and split < 4 and -(-Skv // 64) >= 32 * split:
        split *= 2
    return split


def silu(x):
    """Any length: the kernel does 8-element vectors plus a scalar tail."""
    _bf16(x, "silu")
    x = x.contiguous()
    y = torch.empty_like(x)
    _lib.call("csk_silu", _p(y), _p(x), x.numel(), _s())
    return y


def row_bcast(dst, tab, cur):
    """dst[r] = tab[cur[0]] for every row r (bf16 [rows, W] <- [n, W], int32 device index)."""
    _bf16(dst, "row_bcast.dst")
    _bf16(tab, "row_bcast.tab")
    if dst.dim() != 2 or tab.dim() != 2 or dst.shape[1] != tab.shape[1] or not dst.is_contiguous() \
            or not tab.is_contiguous() or cur.dtype != torch.int32:
        raise ValueError("row_bcast: contiguous bf16 [rows, W] / [n, W], int32 cur")
    _lib.call("csk_row_bcast", _p(dst), _p(tab), _p(cur), dst.shape[0], dst.shape[1], tab.shape[0], _s())


def dup2(x):
    """[x; x] along dim 0 (CFG-shared prefix -> both guidance halves) in one pass."""
    x = x.contiguous()
    y = torch.empty((2 * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if x.dtype != torch.bfloat16 or x.numel() % 8 or x.data_ptr() % 16:
        y[: x.shape[0]].copy_(x)
        y[x.shape[0]:].copy_(x)
        return y
    _lib.call("csk_dup2", _p(y), _p(x), x.numel(), _s())
    return y


def add(x, y):
    _bf16(x, "add")
    if x.shape != y.shape:
        raise ValueError(f"hip add: shapes {tuple(x.shape)} and {tuple(y.shape)} differ (no broadcasting)")
    x, y = x.contiguous(), y.contiguous().to(x.dtype)
    out = torch.empty_like(x)
    _lib.call("csk_add", _p(out), _p(x), _p(y), x.numel(), _s())
    return out


def sched_step(e, x, prev_x0, c, guidance, noise):
    _bf16(e, "sched_step.e")
    x = x.contiguous()
    n = x.numel()
    cfg = guidance is not None
    if e.numel() != n * (2 if cfg else 1):
        raise ValueError("sched_step: model output / latent size mismatch")
    xn = torch.empty_like(x)
    x0 = torch.empty_like(x)
    _lib.call("csk_sched_step", _p(xn), _p(x0), _p(e.contiguous()), _p(x),
              _p(prev_x0) if (prev_x0 is not None and c.C != 0.0) else None,
              _p(noise) if (noise is not None and c.D != 0.0) else None, n,
              float(c.p), float(c.q), float(c.A), float(c.B), float(c.C), float(c.D),
              float(guidance or 0.0), int(cfg), _s())
    return xn, x0


def loop_prologue(counter, cur, t_tab, t_out):
    """Head of a device-resident sampler step: cur = counter++, t_out = t_tab[cur]
    (int32 [1] counter / cur, fp32 table, fp32 [1] output; 1-thread kernel)."""
    if counter.dtype != torch.int32 or cur.dtype != torch.int32 or t_tab.dtype != torch.float32 \
            or t_out.dtype != torch.float32 or t_tab.numel() < 1:
        raise TypeError("loop_prologue: int32 counter/cur, fp32 t_tab/t_out")
    _lib.call("csk_loop_prologue", _p(counter), _p(cur), _p(t_tab), _p(t_out), t_tab.numel(), _s())


def sched_loop(e, x, x0prev, noise_tab, cur, coef, x_in, mode, reps=None):
    """Tail of a device-resident sampler step (elementwise.hip sched_loop_kernel):
    CFG combine (mode 0 none, 1 [u, c], 2 pix2pix [c, i, u]) + the linear update
    with the coefficients of step ``cur`` from the device table ``coef``
    [n, LOOP_COEF_STRIDE] (guidance scales in the row),
    x / x0prev updated in place, the next UNet input written into ``x_in``
    ([reps * B, H, W, Cin] bf16, channels 0..3 of every replica; reps defaults
    to the CFG replica count, 1 for a CFG-parallel half)."""
    _bf16(e, "sched_loop.e")
    _bf16(x_in, "sched_loop.x_in")
    nrep = mode + 1
    reps = nrep if reps is None else int(reps)
    B, H, W, C = x.shape
    if C != 4 or x.dtype != torch.float32 or not x.is_contiguous() or not x0prev.is_contiguous() \
            or x0prev.shape != x.shape or x0prev.dtype != torch.float32:
        raise ValueError("sched_loop: x / x0prev must be contiguous fp32 [B, H, W, 4]")
    if e.numel() != nrep * x.numel() or not e.is_contiguous():
        raise ValueError(f"sched_loop: model output {tuple(e.shape)} vs {nrep} x {tuple(x.shape)}")
    if x_in.dim() != 4 or x_in.shape[0] != reps * B or x_in.shape[1:3] != (H, W) or x_in.shape[3] < 4 \
            or not x_in.is_contiguous():
        raise ValueError(f"sched_loop: x_in {tuple(x_in.shape)} for {reps} x {tuple(x.shape)}")
    if coef.dtype != torch.float32 or coef.dim() != 2 or coef.shape[1] != LOOP_COEF_STRIDE \
            or cur.dtype != torch.int32:
        raise ValueError("sched_loop: coef must be fp32 [n, LOOP_COEF_STRIDE], cur int32")
    if noise_tab is not None and (noise_tab.dtype != torch.float32 or
                                  noise_tab.numel() != coef.shape[0] * x.numel()):
        raise ValueError("sched_loop: noise table must be fp32 [n, B, H, W, 4]")
    _lib.call("csk_sched_loop", _p(e), _p(x), _p(x0prev), _p(noise_tab), _p(cur), _p(coef), _p(x_in),
              x_in.shape[3], reps, B * H * W, mode, _s())


def vae_postprocess(img):
    _bf16(img, "vae_post")
    img = img.contiguous()
    y = torch.empty(img.shape, dtype=torch.uint8, device=img.device)
    _lib.call("csk_vae_post", _p(y), _p(img), img.numel(), _s())
    return y


def canny(img, low, high):
    """uint8 [H, W] or [H, W, C] device image -> uint8 0/255 edge map [H, W]
    (csrc/kernels/canny.hip; multi-channel: cv2's per-pixel max-gradient channel)."""
    if img.dtype != torch.uint8 or img.dim() not in (2, 3):
        raise TypeError("canny: uint8 [H, W] or [H, W, C] expected")
    img = img.contiguous()
    H, W = img.shape[:2]
    C = 1 if img.dim() == 2 else img.shape[2]
    out = torch.empty((H, W), dtype=torch.uint8, device=img.device)
    a4, a1 = -(-(H * W * 4) // 256) * 256, -(-(H * W) // 256) * 256
    ws = torch.empty(256 + a4 + 2 * a1, dtype=torch.uint8, device=img.device)  # torch: 256 B-aligned
    _lib.call("csk_canny", _p(out), _p(img), H, W, C, float(low), float(high), _p(ws), _s())
    return out


XATTN_FUSED = os.environ.get("CSK_XATTN", "1") == "1"  # fused cross-attention sub-block (csrc/kernels/xattn.hip)
XATTN_CHANNELS = (320,)
# workgroup shape of the fused kernel: 4 waves x 32 rows or 8 waves x 16 rows (csk_set_xattn_waves)
XATTN_WAVES = int(os.environ.get("CSK_XATTN_WAVES", "8"))  # 8: 40 vs 50 us, profiles/xattnbench_waves_r6h.txt
_xattn_waves_applied = [None]


# below this many 128-row workgroups the fused kernel (one workgroup per CU)
# leaves CUs idle and the unfused Q GEMM + short-KV attention + out GEMM chain
# wins: CFG batch 2 (64 workgroups) 5.632 vs 5.679 ms per step unfused / fused,
# CFG batch 8 (256) 11.765 vs 11.799 fused / unfused (profiles/unet_step_ab_xattn_gate_r7j.txt)
XATTN_MIN_WG = int(os.environ.get("CSK_XATTN_MIN_WG", "256"))


def xattn_ok(x, kv, rows_per_b) -> bool:
    """Shapes the fused cross-attention sub-block kernel takes: C = 320 (5 heads
    of 64), <= 80 context tokens, whole 128-row tiles of one sample, and a grid
    of at least XATTN_MIN_WG workgroups."""
    C = x.shape[-1]
    if x.numel() // max(C, 1) // 128 < XATTN_MIN_WG:
        return False
    return (XATTN_FUSED and C in XATTN_CHANNELS and kv is not None and kv.dim() == 5 and kv.shape[2] == 2
            and kv.shape[3] * kv.shape[4] == C and kv.shape[4] == 64 and 1 <= kv.shape[1] <= 80
            and rows_per_b % 128 == 0 and x.numel() // C % rows_per_b == 0
            and kv.shape[0] >= x.numel() // C // rows_per_b)


def xattn_block(x, wq, colsum, bq, kv, wo, bo, eps, scale, rows_per_b, row_stats=True):
    """y = x + softmax((LN(x) Wq^T) scale K^T) V Wo^T + bo in ONE kernel
    (LayerNorm folded into ``wq`` / ``colsum`` / ``bq``: ops.fold_layer_norm).
    x: [B, S, C] bf16; kv: [Bc, Skv, 2, H, 64] (Attention.context_kv).  With
    ``row_stats`` the output carries ``_csk_rows`` = (part, 1, C) for the next
    fused LayerNorm."""
    for t, n in ((x, "x"), (wq, "wq"), (bq, "bq"), (kv, "kv"), (wo, "wo")):
        _bf16(t, "xattn_block." + n)
    if bo is not None:
        _bf16(bo, "xattn_block.bo")
    C = x.shape[-1]
    M = x.numel() // C
    x2 = x.reshape(M, C)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    kv = kv.contiguous()
    if colsum.dtype != torch.float32 or colsum.numel() != C:
        raise ValueError("xattn_block: colsum must be fp32 [C]")
    y = torch.empty((M, C), dtype=torch.bfloat16, device=x.device)
    rp = torch.empty(M * 2, dtype=torch.float32, device=x.device) if row_stats else None
    if _xattn_waves_applied[0] != XATTN_WAVES:
        _lib.call("csk_set_xattn_waves", int(XATTN_WAVES))
        _xattn_waves_applied[0] = XATTN_WAVES
    _lib.call("csk_xattn_block", _p(y), _p(x2), _p(wq.contiguous()), _p(colsum.contiguous()), _p(bq.contiguous()),
              _p(kv), _p(wo.contiguous()), _p(None if bo is None else bo.contiguous()), _p(rp), M, C, int(rows_per_b),
              int(kv.shape[0]), int(kv.shape[1]), float(eps), float(scale), _s())
    out = y.view(x.shape)
    if rp is not None:
        out._csk_rows = (rp, 1, C)
    return out


# Fused feed-forward (csrc/kernels/ff.hip): LN3 + GEGLU + down-projection +
# residual in one kernel at C = 320; the [M, 4C] intermediate stays on chip.
sig("csk_ff_geglu_ok", c_int, c_int, c_int)
sig("csk_ff_geglu", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
    c_int, c_float, c_void_p)
sig("csk_set_ff_probe", c_int)
# below this many rows (CFG batch 2 at 64x64: 8192) the 128-row workgroups
# leave most CUs idle and the two tuned GEMMs win (tools/ffbench.py)
FF_MIN_ROWS = int(os.environ.get("CSK_FF_MIN_ROWS", "16384"))
FF_FUSED = os.environ.get("CSK_FF_FUSED", "1") == "1"


def ff_fused_ok(x, inner: int) -> bool:
    C = x.shape[-1]
    M = x.numel() // C
    return (FF_FUSED and x.dtype == torch.bfloat16 and M >= FF_MIN_ROWS
            and _lib.call_int("csk_ff_geglu_ok", M, C, inner) == 1)


def ff_geglu(x, gamma, beta, w1p, b1p, w2p, b2, eps):
    """y = x + W2 GEGLU(W1 LayerNorm(x) + b1) + b2 in ONE kernel (C = 320).
    Weights packed by ``ops.pack_ff_fused`` (the kernel's LDS images, swizzle
    included): w1p [I/16, C/64, 32, 64] bf16, b1p [I/16, 32] fp32,
    w2p [I/32, C/32, 32, 32] bf16."""
    for t, n in ((x, "x"), (gamma, "gamma"), (w1p, "w1p"), (w2p, "w2p")):
        _bf16(t, "ff_geglu." + n)
    C = x.shape[-1]
    M = x.numel() // C
    inner = 32 * w2p.shape[0]
    x2 = x.reshape(M, C)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    y = torch.empty((M, C), dtype=torch.bfloat16, device=x.device)
    if beta is not None:
        _bf16(beta, "ff_geglu.beta")
    if b2 is not None:
        _bf16(b2, "ff_geglu.b2")
    if b1p is not None and b1p.dtype != torch.float32:
        raise ValueError("ff_geglu: b1p must be fp32")
    _lib.call("csk_ff_geglu", _p(y), _p(x2), _p(gamma.contiguous()), _p(None if beta is None else beta.contiguous()),
              _p(w1p.contiguous()), _p(None if b1p is None else b1p.contiguous()), _p(w2p.contiguous()),
              _p(None if b2 is None else b2.contiguous()), M, C, inner, float(eps), _s())
    return y.view(x.shape)


sig("csk_set_xattn_probe", c_int)
sig("csk_set_xattn_waves", c_int)


# Fused transformer input (csrc/kernels/xin.hip): GroupNorm apply + proj_in +
# LN1 + QKV projection in one kernel at C = 320; the normalised input stays in
# registers, h is stored once (the out-projection's residual).
sig("csk_xin_qkv_ok", c_int, c_int, c_int, c_int)
sig("csk_xin_qkv", c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
    c_void_p, c_int, c_int, c_float, c_void_p)
sig("csk_set_xin_probe", c_int)
sig("csk_set_conv_tile_no_rw", c_int)
sig("csk_gn_finalize", c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p)
XIN_FUSED = os.environ.get("CSK_XIN_FUSED", "1") == "1"
XIN_MIN_ROWS = int(os.environ.get("CSK_XIN_MIN_ROWS", "16384"))  # CFG-2 grids (8192 rows: 64 workgroups) keep the GEMMs (tools/xinbench.py)


def gn_stats(x, groups, eps):
    """(mean, rstd) [B, G, 2] fp32 of a [B, ..., C] bf16 tensor from its
    producer's fused epilogue statistics (``x._csk_gn``), or None without them."""
    fused = getattr(x, "_csk_gn", None)
    if fused is None:
        return None
    B, C = x.shape[0], x.shape[-1]
    P = x.numel() // (B * C)
    part, seg = fused
    if P % seg or part.numel() != (B * P // seg) * C * 2 or C % groups:
        return None
    stat = torch.empty((B, groups, 2), dtype=torch.float32, device=x.device)
    _lib.call("csk_gn_finalize", _p(stat), _p(part), None, 0, seg, B, P, C, groups, float(eps), _s())
    return stat


def xin_ok(x, groups) -> bool:
    """x: [B, P, C] (or NHWC) block input with fused GN statistics attached."""
    if not XIN_FUSED or x.dtype != torch.bfloat16 or getattr(x, "_csk_gn", None) is None:
        return False
    B, C = x.shape[0], x.shape[-1]
    M = x.numel() // C
    return M >= XIN_MIN_ROWS and _lib.call_int("csk_xin_qkv_ok", M, C, M // B, groups) == 1


def xin_qkv(x, stat, gamma, beta, w, bi, colsum, bq, eps):
    """(h, qkv) = (proj_in(GroupNorm(x)), LayerNorm1(h) Wqkv^T + b) in ONE
    kernel; weights / tables from ``ops.pack_xin_qkv``, ``stat`` from
    ``gn_stats``.  Returns h [M, C] and qkv [M, 3C] (bf16)."""
    _bf16(x, "xin.x")
    _bf16(w, "xin.w")
    _bf16(gamma, "xin.gamma")
    B, C = x.shape[0], x.shape[-1]
    M = x.numel() // C
    x2 = x.reshape(M, C)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    for t, n in ((bi, "bi"), (colsum, "colsum"), (bq, "bq"), (stat, "stat")):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous()):
            raise ValueError(f"xin_qkv: {n} must be contiguous fp32")
    if beta is not None:
        _bf16(beta, "xin.beta")
    h = torch.empty((M, C), dtype=torch.bfloat16, device=x.device)
    qkv = torch.empty((M, 3 * C), dtype=torch.bfloat16, device=x.device)
    _lib.call("csk_xin_qkv", _p(h), _p(qkv), _p(x2), _p(stat), _p(gamma.contiguous()),
              _p(None if beta is None else beta.contiguous()), stat.shape[1], _p(w.contiguous()), _p(bi), _p(colsum),
              _p(bq), M, M // B, float(eps), _s())
    return h, qkv
