// Flash attention for wide heads, 256 < D <= 512 (the VAE mid-block's single
// head, d = 512).  Replaces the GEMM -> row-softmax -> GEMM path
// that materialised the S x S score matrix (512 MB per image at 1024^2): here
// nothing of size S x S exists, O(S) memory.
//
// Same swapped-operand MFMA structure as attention.hip (S^T = K Q^T puts one
// query column and 4 keys on each lane; P^T feeds the PV MFMA straight from the
// accumulators; V^T via ds_read_b64_tr_b16), with the wide-head specifics:
//   * Q (16 x 512 per wave and QT) lives in registers for the whole key loop,
//     the O^T accumulator (512 x 16 per QT) too: 64 + 128 VGPRs per QT, one
//     wave per SIMD (launch_bounds(256, 1): up to 512 registers);
//   * key blocks of 32 rows (a 32 x 512 bf16 tile is 32 KB): K and V double
//     buffered = 128 KB of LDS, filled by LDS-DMA (global_load_lds, 16 B per
//     lane, one 1 KB row per wave-instruction) with the XOR swizzle applied to
//     the per-lane SOURCE address (the DMA destination is lane-linear);
//     out-of-range keys read the zero page;
//   * at d = 512 the softmax is ~2 % of the work (8 scores per lane per block),
//     so the loop is MFMA + LDS-read bound, not VALU bound as at d = 64.
#include "gemm_common.h"

typedef __attribute__((address_space(3))) v4s lds_v4s_w;

struct AttnWideArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  long long sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh;
  int B, H, Sq, Skv, D;
  float scale_log2;
  const bf16_t* zero;
  const bf16_t* k_end;  // one past the last K / V element (CSK_DEBUG checks)
  const bf16_t* v_end;
};

template <int CPR>
__device__ __forceinline__ int wkv_off(int row, int chunk) {
  return row * (CPR * 8) + ((chunk ^ (row & 15)) << 3);
}

template <int QT>
__global__ __launch_bounds__(256, 1) void attn_wide_kernel(const AttnWideArgs a) {
  constexpr int DP = 512, CPR = DP / 8, KB = 32;
  constexpr int DS = DP / 32, DT = DP / 16;
  constexpr int TILE = KB * DP;
  constexpr int QROWS = QT * 16 * 4;
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE];  // K0 V0 K1 V1 (128 KB)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int nqb = (a.Sq + QROWS - 1) / QROWS;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = wg / nqb, qb = wg % nqb;
  const int b = bh / a.H, h = bh % a.H;
  const int q0 = qb * QROWS + wid * QT * 16;
  const bf16_t* qp = a.q + b * a.sqb + h * a.sqh;
  const bf16_t* kp = a.k + b * a.skb + h * a.skh;
  const bf16_t* vp = a.v + b * a.svb + h * a.svh;
  const int Skv = a.Skv;
  const int nkb = (Skv + KB - 1) / KB;

  v8s qf[QT][DS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      const int qi = q0 + qt * 16 + fr, d = ds * 32 + 8 * fg;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qi < a.Sq && d < a.D) v = *reinterpret_cast<const uint4*>(qp + qi * a.sqs + d);
      qf[qt][ds] = __builtin_bit_cast(v8s, v);
    }
  v4f oacc[QT][DT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int i = 0; i < DT; ++i) oacc[qt][i] = v4f{0.f, 0.f, 0.f, 0.f};
  float mrow[QT], lrow[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) { mrow[qt] = -1e30f; lrow[qt] = 0.f; }

  // DMA: wave w stages rows w*8 .. w*8+7 of the K and V tiles (one 1 KB row per
  // instruction); lane L lands in LDS chunk L and fetches source chunk L ^ (row & 15)
  const bool dfull = a.D == DP;
  auto issue = [&](int kb, int buf) {
    bf16_t* ks = smem + buf * 2 * TILE;
    bf16_t* vs = ks + TILE;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = wid * 8 + i, key = kb * KB + row;
      const int c = lane ^ (row & 15), d = c * 8;
      const bool ok = key < Skv && (dfull || d < a.D);
      const bf16_t* sk = ok ? kp + (size_t)key * a.sks + d : a.zero + lane * 8;
      const bf16_t* sv = ok ? vp + (size_t)key * a.svs + d : a.zero + lane * 8;
      CSK_DCHECK((sk >= a.k && sk + 8 <= a.k_end) || (sk >= a.zero && sk + 8 <= a.zero + ZERO_BYTES / 2), SITE_WIDE_KV,
                 key, Skv);
      CSK_DCHECK((sv >= a.v && sv + 8 <= a.v_end) || (sv >= a.zero && sv + 8 <= a.zero + ZERO_BYTES / 2), SITE_WIDE_KV,
                 key, Skv);
      CSK_DCHECK(buf * 2 * TILE + TILE + row * DP + 512 <= 4 * TILE, SITE_WIDE_KV + 100, row, buf);
      __builtin_amdgcn_global_load_lds((csk_gptr_t)sk, (csk_lptr_t)(ks + row * DP), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((csk_gptr_t)sv, (csk_lptr_t)(vs + row * DP), 16, 0, 0);
    }
  };

  if (nkb > 0) issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float sl2 = a.scale_log2;
  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nkb) issue(kb + 1, cur ^ 1);
    const bf16_t* ks = smem + cur * 2 * TILE;
    const bf16_t* vs = ks + TILE;
    // ---- S^T = K Q^T over 2 key tiles ----
    v4f s[2][QT];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[kt][qt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < DS; ++ds)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        const v8s kf = *reinterpret_cast<const v8s*>(ks + wkv_off<CPR>(kt * 16 + fr, ds * 4 + fg));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][ds], s[kt][qt], 0, 0, 0);
      }
    // ---- online softmax ----
    const int kbase = kb * KB;
    v8s pf[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if (kbase + KB > Skv) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (kbase + kt * 16 + 4 * fg + r >= Skv) s[kt][qt][r] = -INFINITY;
      }
      float mx = vmax3(s[0][qt][0], s[0][qt][1], s[0][qt][2]);
      mx = vmax3(mx, s[0][qt][3], s[1][qt][0]);
      mx = vmax3(mx, s[1][qt][1], s[1][qt][2]);
      mx = max_rowgroups(fmaxf(mx, s[1][qt][3]));
      const float mnew = fmaxf(mrow[qt], mx * sl2);
      const float alpha = __builtin_amdgcn_exp2f(mrow[qt] - mnew);
      mrow[qt] = mnew;
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[kt][qt][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][qt][r], sl2, -mnew));
          l += s[kt][qt][r];
        }
      lrow[qt] = lrow[qt] * alpha + l;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[qt][dt] *= alpha;
      const u32 w0 = pack2(s[0][qt][0], s[0][qt][1]), w1 = pack2(s[0][qt][2], s[0][qt][3]);
      const u32 w2 = pack2(s[1][qt][0], s[1][qt][1]), w3 = pack2(s[1][qt][2], s[1][qt][3]);
      pf[qt] = __builtin_bit_cast(v8s, make_uint4(w0, w1, w2, w3));
    }
    // ---- O^T += V^T P^T (one 32-key k-step); V^T by transpose reads ----
    const int qq = fr >> 2, pp = fr & 3;
    const int r0 = 4 * fg + qq, r1 = r0 + 16;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int col = dt * 16 + 4 * pp;
      const bf16_t* a0 = vs + wkv_off<CPR>(r0, col >> 3) + (col & 7);
      const bf16_t* a1 = vs + wkv_off<CPR>(r1, col >> 3) + (col & 7);
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_w*)(a0));
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_w*)(a1));
      const v8s vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
        oacc[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[qt], oacc[qt][dt], 0, 0, 0);
    }
    // next block's DMA landed (every wave waited for its own) and every wave is
    // done reading this buffer before the barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  bf16_t* op = a.o + b * a.sob + h * a.soh;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l = lrow[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    const int qi = q0 + qt * 16 + fr;
    if (qi >= a.Sq) continue;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = dt * 16 + 4 * fg;
      if (d >= a.D) continue;
      uint2 w;
      w.x = pack2(oacc[qt][dt][0] * inv, oacc[qt][dt][1] * inv);
      w.y = pack2(oacc[qt][dt][2] * inv, oacc[qt][dt][3] * inv);
      *reinterpret_cast<uint2*>(op + qi * a.sos + d) = w;
    }
  }
}

// 256 < D <= 512, D % 16 == 0, no causal mask (the VAE's attention is bidirectional)
CSK_API int csk_attention_wide(void* o, const void* q, const void* k, const void* v, const long long* strides, int B,
                               int H, int Sq, int Skv, int D, float scale, hipStream_t stream) {
  if (D <= 256 || D > 512 || D % 16 != 0) return (int)hipErrorInvalidValue;
  const bf16_t* zero = csk_zero_ptr();
  if (!zero) return (int)hipErrorNotInitialized;
  AttnWideArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.sqb = strides[0]; a.sqs = strides[1]; a.sqh = strides[2];
  a.skb = strides[3]; a.sks = strides[4]; a.skh = strides[5];
  a.svb = strides[6]; a.svs = strides[7]; a.svh = strides[8];
  a.sob = strides[9]; a.sos = strides[10]; a.soh = strides[11];
  a.B = B; a.H = H; a.Sq = Sq; a.Skv = Skv; a.D = D;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.zero = zero;
  a.k_end = a.k + (B - 1) * a.skb + (long long)(Skv - 1) * a.sks + (H - 1) * a.skh + D;
  a.v_end = a.v + (B - 1) * a.svb + (long long)(Skv - 1) * a.svs + (H - 1) * a.svh + D;
  if (Sq <= 0 || B * H == 0) return 0;
  // QT = 1: 16 query rows per wave (QT = 2 needs ~640 registers: spills)
  attn_wide_kernel<1><<<(unsigned)((long long)B * H * ((Sq + 63) / 64)), 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}

CSK_DEBUG_EXPORT(attention_wide)
