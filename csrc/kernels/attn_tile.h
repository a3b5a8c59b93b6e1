// Short-context attention of one 16-query row tile against K / V images staged
// in LDS, shared by the fused cross-attention block (xattn.hip) and the
// Q-projection GEMM's attention epilogue (gemm_common.h, gemm_attn_epilogue).
//
// Layouts (head dim 64, Skv <= 80 keys, images of 96 rows, rows past Skv
// repeat a valid key and are masked):
//   * K / V images: [96][64] bf16, 16-byte chunk c of row r at slot c ^ at_key(r);
//   * the queries arrive as the B fragments of S^T = K Q^T: lane (fr, g) holds
//     query row fr, head-dims {4g + r, 16 + 4g + r} (k-step 0) and
//     {32 + 4g + r, 48 + 4g + r} (k-step 1) — exactly the row-layout
//     accumulators of an MFMA whose rows are the queries (16 dt + 4 g + r), so a
//     projection's accumulators feed it with one pack each;
//   * S^T leaves keys 16 kt + 4 g + r of query fr on the lane: the softmax is
//     in-lane + two cross-row-group reductions; P^T and the transposed V
//     fragments (ds_read_tr16_b64 of the row-major V image) give O^T with
//     head-dims 16 dt + 4 g + r of query fr on the lane.
#pragma once
#include "common.h"

typedef __attribute__((address_space(3))) v4s at_lds_v4s;

// chunk swizzle key of row r: (r & 7) ^ ((r >> 3) & 1).  The 8-byte fragment
// reads (at_perm_frag) take 16 consecutive rows per 32-lane bank group; with the
// plain (r & 7) key rows r and r + 8 (128-byte rows: same bank half) hit the same
// banks, a 2-way conflict on every K / Wo read (PMC: 1.5 conflict cycles per LDS
// instruction in the fused block, profiles/pmc_unet_step_r6r_1.txt); flipping the
// low bit for the second 8 rows spreads the 16 rows over all 64 banks
__device__ __forceinline__ int at_key(int r) { return (r & 7) ^ ((r >> 3) & 1); }

// element offset of 16-byte chunk c of row r in a [rows][64] image
__device__ __forceinline__ int at_off64(int r, int c) { return r * 64 + ((c ^ at_key(r)) << 3); }

__device__ __forceinline__ v8s at_cat(v4s a, v4s b) { return v8s{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]}; }

// two 8-byte halves (head-dims d0..d0+3 and d0+16..d0+19) of row r of a [rows][64] image
__device__ __forceinline__ v8s at_perm_frag(const bf16_t* img, int r, int d0) {
  const int c0 = d0 >> 3, h = d0 & 7;
  const v4s a = *reinterpret_cast<const v4s*>(img + at_off64(r, c0) + h);
  const v4s b = *reinterpret_cast<const v4s*>(img + at_off64(r, c0 + 2) + h);
  return at_cat(a, b);
}

__device__ __forceinline__ v8s at_pack8(const v4f& lo, const v4f& hi, float s) {
  const uint4 u = make_uint4(pack2(lo[0] * s, lo[1] * s), pack2(lo[2] * s, lo[3] * s), pack2(hi[0] * s, hi[1] * s),
                             pack2(hi[2] * s, hi[3] * s));
  return __builtin_bit_cast(v8s, u);
}

// o[dt][r] * inv = (softmax_keys(q K^T) V)[fr][16 dt + 4 g + r] for the query
// row tile whose S^T B fragments are qf[0..1] (already scaled by
// scale * log2(e)); the caller applies inv (1 / row sum) where it converts.
__device__ __forceinline__ void at_attend_rowtile(const bf16_t* ks, const bf16_t* vs, const v8s (&qf)[2], int Skv,
                                                  v4f (&o)[4], float& inv) {
  const int lane = threadIdx.x & 63, fr = lane & 15, g = lane >> 4;
  const int qq = fr >> 2, pp = fr & 3;
  v4f s[5];
#pragma unroll
  for (int kt = 0; kt < 5; ++kt) {
    s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < 2; ++ds)
      s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at_perm_frag(ks, 16 * kt + fr, 32 * ds + 4 * g), qf[ds], s[kt],
                                                      0, 0, 0);
  }
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < 5; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (16 * kt + 4 * g + r >= Skv) s[kt][r] = -INFINITY;
      mx = fmaxf(mx, s[kt][r]);
    }
  mx = max_rowgroups(mx);
  float l = 0.f;
#pragma unroll
  for (int kt = 0; kt < 5; ++kt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = __builtin_amdgcn_exp2f(s[kt][r] - mx);
      s[kt][r] = p;
      l += p;
    }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k2 = 0; k2 < 3; ++k2) {
    const v4f z = v4f{0.f, 0.f, 0.f, 0.f};
    const v8s pf = at_pack8(s[2 * k2], k2 < 2 ? s[2 * k2 + 1] : z, 1.0f);
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int col = dt * 16 + 4 * pp;
      const int r0 = k2 * 32 + 4 * g + qq, r1 = r0 + 16;
      const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((at_lds_v4s*)(vs + at_off64(r0, col >> 3) + (col & 7)));
      const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((at_lds_v4s*)(vs + at_off64(r1, col >> 3) + (col & 7)));
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at_cat(lo, hi), pf, o[dt], 0, 0, 0);
    }
  }
  inv = l > 0.f ? 1.0f / l : 0.f;
}
