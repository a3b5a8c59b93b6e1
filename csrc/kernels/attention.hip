// Flash-style fused attention forward, bf16 in/out, fp32 softmax (SURVEY K7/K8,
// K14 causal for CLIP).  O = softmax(Q K^T * scale) V for [B, S, H, D] strided
// views (D contiguous), so fused QKV projection outputs are consumed in place.
//
// CDNA4 structure ("swapped" QK^T, everything lane-local):
//   * workgroup = 4 waves; each wave owns QT x 16 query rows; KV blocks of 64 keys
//     are register-staged into double-buffered, XOR-swizzled LDS tiles (one
//     barrier per block).
//   * S^T = K Q^T with v_mfma_f32_16x16x32_bf16 (A = K rows from LDS via
//     ds_read_b128, B = Q fragments held in registers for the whole loop): the
//     accumulator puts ONE query column on each lane and 4 consecutive keys in
//     its registers, so the online-softmax row max / sum are in-lane plus two
//     cross-group shuffles, and the rescale factor is a per-lane scalar.
//   * O^T = V^T P^T: P^T comes straight from the S^T accumulators (converted to
//     bf16, no lane movement) by permuting the k order of the PV MFMA; the
//     matching V^T operand is fetched with ds_read_b64_tr_b16 (gfx950 hardware
//     transpose read) from the same row-major V tile.
//   * exp2 with log2(e)*scale folded in; masked keys (tail, causal) -> -inf.
#include "common.h"

typedef __attribute__((address_space(3))) v4s lds_v4s;

template <int CPR>
__device__ __forceinline__ int kv_off(int row, int chunk) {
  // element offset of 16-byte chunk `chunk` of row `row` in a [64][CPR*8] tile
  constexpr int MASK = CPR >= 16 ? 15 : CPR - 1;
  return row * (CPR * 8) + ((chunk ^ (row & MASK)) << 3);
}

struct AttnArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  long long sqb, sqs, sqh;  // element strides of q (b, s, h)
  long long skb, sks, skh;
  long long svb, svs, svh;
  long long sob, sos, soh;
  int B, H, Sq, Skv, D;
  float scale_log2;
  int causal;
  const int* kv_len;  // optional device-side key count (<= Skv): lets a fixed-shape
                      // KV-cache decode step be captured once in a hipGraph
  // split-KV (attn32_kernel): kv_split workgroups share a query block, each
  // over 1/kv_split of the key blocks, and write unnormalised fp32 partials
  // part_o [split][B*H][Sq][64] and (max, sum) part_ml [split][B*H][Sq][2]
  int kv_split;
  float* part_o;
  float* part_ml;
};

// DV: the head dim rounded up to 16 (SD1.5's 40 / 80 / 160 live in 64 / 128 / 256
// wide tiles): the QK^T k-steps and O d-tiles past DV only multiply zeros and
// are not instantiated (compile-time bounds — MFMAs ignore EXEC, so a runtime
// skip would have to be a scalar branch the compiler keeps)
template <int DP, int QT, int DV = DP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const AttnArgs a) {
  constexpr int CPR = DP / 8;          // 16B chunks per K/V row
  constexpr int KB = 64;               // keys per block
  constexpr int DS = DP / 32;          // k-steps of S = K Q^T over d
  constexpr int DT = DP / 16;          // O^T d-tiles
  constexpr int DSV = (DV + 31) / 32;  // k-steps / d-tiles that touch a real column
  constexpr int DTV = (DV + 15) / 16;
  static_assert(DV <= DP && DV % 16 == 0, "DV: head dim rounded up to 16");
  constexpr int QROWS = QT * 16 * 4;   // query rows per workgroup
  constexpr int TILE = KB * DP;        // elements per K or V tile
  constexpr int LPT = KB * CPR / 256;  // 16B chunks per thread per tile
  __shared__ __attribute__((aligned(16))) bf16_t smem[4 * TILE];  // K0 V0 K1 V1

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR address math
  const int fr = lane & 15, fg = lane >> 4;
  const int Skv = a.kv_len ? min(a.Skv, *a.kv_len) : a.Skv;
  const int nqb = (a.Sq + QROWS - 1) / QROWS;
  // XCD-aware: the query blocks of one (batch, head) run on one XCD, so its
  // K/V (re-read by every query block) is fetched into one L2, not eight
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = wg / nqb, qb = wg % nqb;
  const int b = bh / a.H, h = bh % a.H;
  const int q0 = qb * QROWS + wid * QT * 16;

  const bf16_t* qp = a.q + b * a.sqb + h * a.sqh;
  const bf16_t* kp = a.k + b * a.skb + h * a.skh;
  const bf16_t* vp = a.v + b * a.svb + h * a.svh;

  // Q fragments (B operand): lane holds Q[q0 + qt*16 + fr][ds*32 + 8*fg .. +7]
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

  v4f oacc[DT][QT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int j = 0; j < QT; ++j) oacc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float mrow[QT], lrow[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) { mrow[qt] = -1e30f; lrow[qt] = 0.f; }

  int kv_end = Skv;
  if (a.causal) {  // keys beyond the last query row of this workgroup are never visible
    const int qlast = min(a.Sq, (qb + 1) * QROWS) - 1 + (Skv - a.Sq);
    kv_end = min(Skv, qlast + 1);
  }
  const int nkb = (kv_end + KB - 1) / KB;

  uint4 rk[LPT], rv[LPT];
  auto load_kv = [&](int kb) {
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
      const int key = kb * KB + row, d = c * 8;
      uint4 vk = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (key < Skv && d < a.D) {
        vk = *reinterpret_cast<const uint4*>(kp + key * a.sks + d);
        vv = *reinterpret_cast<const uint4*>(vp + key * a.svs + d);
      }
      rk[i] = vk;
      rv[i] = vv;
    }
  };
  auto store_kv = [&](int buf) {
    bf16_t* ks = smem + buf * 2 * TILE;
    bf16_t* vs = ks + TILE;
    CSK_DCHECK(buf >= 0 && buf < 2, 20, buf, 2);  // the 2-buffer K/V ring
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
      CSK_DCHECK(kv_off<CPR>(row, c) + 8 <= TILE, 21, kv_off<CPR>(row, c), TILE);
      *reinterpret_cast<uint4*>(ks + kv_off<CPR>(row, c)) = rk[i];
      *reinterpret_cast<uint4*>(vs + kv_off<CPR>(row, c)) = rv[i];
    }
  };

  if (nkb > 0) {
    load_kv(0);
    store_kv(0);
  }
  __syncthreads();
  const float sl2 = a.scale_log2;
  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nkb) load_kv(kb + 1);
    const bf16_t* ks = smem + cur * 2 * TILE;
    const bf16_t* vs = ks + TILE;

    // ---- S^T = K Q^T : 4 key tiles x QT query tiles ----
    // key tiles wholly past kv_end (the tail block: Skv = 77 cross-attention
    // keeps 1 of its 4) skip their QK^T and PV MFMAs (wave-uniform branches)
    const int ktn = DP == 64 ? min(4, (kv_end - kb * KB + 15) >> 4) : 4;
    v4f s[4][QT];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[kt][qt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ds = 0; ds < DSV; ++ds) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        if (kt >= ktn) continue;
        const v8s kf = *reinterpret_cast<const v8s*>(ks + kv_off<CPR>(kt * 16 + fr, ds * 4 + fg));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][ds], s[kt][qt], 0, 0, 0);
      }
    }
    // ---- online softmax (per lane: one query column, 16 keys) ----
    // max on raw scores (scale > 0), then p = exp2(s * scale*log2e - m): one
    // v_fma + one v_exp per score; masking only on the tail / causal blocks.
    const int kbase = kb * KB;
    const bool masked = a.causal || (kbase + KB > kv_end);
    v8s pf[2][QT];  // P^T fragments for the two 32-key PV k-steps
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if (masked) {
        const int qi = q0 + qt * 16 + fr + (Skv - a.Sq);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kbase + kt * 16 + 4 * fg + r;
            if (key >= kv_end || (a.causal && key > qi)) s[kt][qt][r] = -INFINITY;
          }
      }
      mfma_fence4(s[0][qt], s[1][qt], s[2][qt], s[3][qt]);
      float mx = vmax3(s[0][qt][0], s[0][qt][1], s[0][qt][2]);
      mx = vmax3(mx, s[0][qt][3], s[1][qt][0]);
      mx = vmax3(mx, s[1][qt][1], s[1][qt][2]);
      mx = vmax3(mx, s[1][qt][3], s[2][qt][0]);
      mx = vmax3(mx, s[2][qt][1], s[2][qt][2]);
      mx = vmax3(mx, s[2][qt][3], s[3][qt][0]);
      mx = vmax3(mx, s[3][qt][1], s[3][qt][2]);
      mx = max_rowgroups(vmax3(mx, s[3][qt][3], s[3][qt][3]));
      const float mnew = fmaxf(mrow[qt], mx * sl2);
      const float alpha = __builtin_amdgcn_exp2f(mrow[qt] - mnew);
      mrow[qt] = mnew;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[kt][qt][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[kt][qt][r], sl2, -mnew));
      float l4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) l4[r] = vadd(vadd_t(s[0][qt][r], s[1][qt][r]), vadd_t(s[2][qt][r], s[3][qt][r]));
      lrow[qt] = lrow[qt] * alpha + vadd(vadd(l4[0], l4[1]), vadd(l4[2], l4[3]));
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) oacc[dt][qt] *= alpha;
#pragma unroll
      for (int kp2 = 0; kp2 < 2; ++kp2) {
        u32 w0 = pack2(s[2 * kp2][qt][0], s[2 * kp2][qt][1]);
        u32 w1 = pack2(s[2 * kp2][qt][2], s[2 * kp2][qt][3]);
        u32 w2 = pack2(s[2 * kp2 + 1][qt][0], s[2 * kp2 + 1][qt][1]);
        u32 w3 = pack2(s[2 * kp2 + 1][qt][2], s[2 * kp2 + 1][qt][3]);
        pf[kp2][qt] = __builtin_bit_cast(v8s, make_uint4(w0, w1, w2, w3));
      }
    }
    // ---- O^T += V^T P^T ; V^T fragments via ds_read_b64_tr_b16 ----
#pragma unroll
    for (int kp2 = 0; kp2 < 2; ++kp2) {
      if (2 * kp2 >= ktn) continue;  // keys kp2*32 .. +31 all masked: P^T is zero there
#pragma unroll
      for (int dt = 0; dt < DTV; ++dt) {
        // group fg reads rows (keys) kp2*32 + 4*fg + {0..3} and kp2*32 + 16 + 4*fg + {0..3},
        // lane 4q+p of the group addresses row q, columns dt*16 + 4p .. +3
        const int qq = fr >> 2, pp = fr & 3;
        const int col = dt * 16 + 4 * pp;
        const int r0 = kp2 * 32 + 4 * fg + qq, r1 = r0 + 16;
        const bf16_t* a0 = vs + kv_off<CPR>(r0, col >> 3) + (col & 7);
        const bf16_t* a1 = vs + kv_off<CPR>(r1, col >> 3) + (col & 7);
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a1));
        v8s vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          oacc[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[kp2][qt], oacc[dt][qt], 0, 0, 0);
      }
    }
    if (kb + 1 < nkb) store_kv(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: reduce l over the 4 lane groups, normalise, store ----
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
      w.x = pack2(oacc[dt][qt][0] * inv, oacc[dt][qt][1] * inv);
      w.y = pack2(oacc[dt][qt][2] * inv, oacc[dt][qt][3] * inv);
      *reinterpret_cast<uint2*>(op + qi * a.sos + d) = w;
    }
  }
}

// Software-pipelined variant (D <= 64, 3 LDS K/V buffers, one barrier per
// block): S for block kb+1 is issued on the matrix cores BEFORE the online
// softmax of block kb, so the exp/max/sum VALU work of one block overlaps the
// QK^T MFMAs of the next inside a single wave (cdna_hip_programming.md T15
// "compute[cur] || finish[prev]"); block kb+2 is register-staged meanwhile and
// written to the buffer freed two blocks ago, so no second barrier is needed.
//
// The softmax is VALU-issue bound at D = 64 (one exp per 64 MACs), so two
// options move per-score work elsewhere:
//   PRE  : Q is pre-scaled by scale*log2(e) and the QK^T chain starts from the
//          accumulator value -m (the running max when the block was issued,
//          one shared C operand per query tile): p = exp2(s) directly, no
//          per-score FMA.  A rescale between issue and use (rare: lazy max,
//          T13) is corrected by one wave-uniform subtract pass.
//   ONES : the row sum l rides on the PV MFMAs as an extra all-ones V^T tile
//          (4 MFMAs per block instead of 32 adds + 2 shuffles per query tile).
//
// PROBE (profiling builds of the same loop, variants 11/12/14/18; results are
// wrong by design): 1 = no exp (P = S), 2 = no K/V global loads (LDS keeps its
// first blocks), 4 = no PV MFMAs (P kept alive), 8 = no QK^T MFMAs.
template <int QT, bool PRE, bool ONES, int PROBE = 0, int MINB = 2>
__global__ __launch_bounds__(256, MINB) void attn_fwd_pipe_kernel(const AttnArgs a) {
  constexpr int DP = 64;
  constexpr int CPR = DP / 8;
  constexpr int KB = 64;
  constexpr int DS = DP / 32;
  constexpr int DT = DP / 16;
  constexpr int DTO = DT + (ONES ? 1 : 0);
  constexpr int QROWS = QT * 16 * 4;
  constexpr int TILE = KB * DP;
  constexpr int LPT = KB * CPR / 256;
  __shared__ __attribute__((aligned(16))) bf16_t smem[3 * 2 * TILE];  // (K, V) x 3

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int Skv = a.kv_len ? min(a.Skv, *a.kv_len) : a.Skv;
  const int nqb = (a.Sq + QROWS - 1) / QROWS;
  // XCD-aware: the query blocks of one (batch, head) run on one XCD, so its
  // K/V (re-read by every query block) is fetched into one L2, not eight
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = wg / nqb, qb = wg % nqb;
  const int b = bh / a.H, h = bh % a.H;
  const int q0 = qb * QROWS + wid * QT * 16;
  const bf16_t* qp = a.q + b * a.sqb + h * a.sqh;
  const bf16_t* kp = a.k + b * a.skb + h * a.skh;
  const bf16_t* vp = a.v + b * a.svb + h * a.svh;
  const float sl2 = a.scale_log2;

  v8s qf[QT][DS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      const int qi = q0 + qt * 16 + fr, d = ds * 32 + 8 * fg;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qi < a.Sq && d < a.D) v = *reinterpret_cast<const uint4*>(qp + qi * a.sqs + d);
      if constexpr (PRE) {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= sl2;
        v = pack8(f);
      }
      qf[qt][ds] = __builtin_bit_cast(v8s, v);
    }
  v4f oacc[DTO][QT];
#pragma unroll
  for (int i = 0; i < DTO; ++i)
#pragma unroll
    for (int j = 0; j < QT; ++j) oacc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float mrow[QT], lrow[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) { mrow[qt] = -1e30f; lrow[qt] = 0.f; }
  const short one_bf = 0x3f80;
  const v8s ones = {one_bf, one_bf, one_bf, one_bf, one_bf, one_bf, one_bf, one_bf};

  int kv_end = Skv;
  if (a.causal) {
    const int qlast = min(a.Sq, (qb + 1) * QROWS) - 1 + (Skv - a.Sq);
    kv_end = min(Skv, qlast + 1);
  }
  const int nkb = (kv_end + KB - 1) / KB;

  uint4 rk[LPT], rv[LPT];
  auto load_kv = [&](int kb) {
    if constexpr ((PROBE & 2) != 0) {
      if (kb >= 2) return;
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
      const int key = min(kb * KB + row, Skv - 1), d = c * 8;  // clamped rows are masked later
      CSK_DCHECK(key >= 0, 22, key, Skv);  // Skv >= 1 whenever a block is loaded
      uint4 vk = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (d < a.D) {
        vk = *reinterpret_cast<const uint4*>(kp + key * a.sks + d);
        vv = *reinterpret_cast<const uint4*>(vp + key * a.svs + d);
      }
      rk[i] = vk;
      rv[i] = vv;
    }
  };
  auto store_kv = [&](int buf) {
    bf16_t* ks = smem + buf * 2 * TILE;
    bf16_t* vs = ks + TILE;
    CSK_DCHECK(buf >= 0 && buf < 3, 20, buf, 3);  // the 3-buffer K/V ring
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
      CSK_DCHECK(kv_off<CPR>(row, c) + 8 <= TILE, 21, kv_off<CPR>(row, c), TILE);
      *reinterpret_cast<uint4*>(ks + kv_off<CPR>(row, c)) = rk[i];
      *reinterpret_cast<uint4*>(vs + kv_off<CPR>(row, c)) = rv[i];
    }
  };
  // mu[qt]: the offset the block's scores were issued with (PRE), else 0
  auto qk = [&](int buf, v4f (&s)[4][QT], float (&mu)[QT]) {
    const bf16_t* ks = smem + buf * 2 * TILE;
    v4f cinit[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      mu[qt] = (PRE && mrow[qt] > -1e29f) ? mrow[qt] : 0.f;
      cinit[qt] = v4f{-mu[qt], -mu[qt], -mu[qt], -mu[qt]};
    }
    if constexpr ((PROBE & 8) != 0) {
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[kt][qt] = cinit[qt] + (float)kt;
      return;
    }
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      const v8s kf = *reinterpret_cast<const v8s*>(ks + kv_off<CPR>(kt * 16 + fr, fg));
#pragma unroll
      for (int qt = 0; qt < QT; ++qt)
        s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][0], cinit[qt], 0, 0, 0);
    }
#pragma unroll
    for (int ds = 1; ds < DS; ++ds)
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const v8s kf = *reinterpret_cast<const v8s*>(ks + kv_off<CPR>(kt * 16 + fr, ds * 4 + fg));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[qt][ds], s[kt][qt], 0, 0, 0);
      }
  };

  if (nkb > 0) { load_kv(0); store_kv(0); }
  if (nkb > 1) { load_kv(1); store_kv(1); }
  __syncthreads();
  v4f s_a[4][QT], s_b[4][QT];
  float mu_a[QT], mu_b[QT];
  // one pipelined block: softmax + PV of block kb (scores in sc) while the QK^T
  // of block kb+1 fills sn.  Called alternately with (s_a, s_b) / (s_b, s_a) so
  // the score registers are never copied.
  auto block = [&](int kb, v4f (&sc)[4][QT], float (&muc)[QT], v4f (&sn)[4][QT], float (&mun)[QT]) {
    const int cur = kb % 3;
    if (kb + 2 < nkb) load_kv(kb + 2);
    if (kb + 1 < nkb) qk((kb + 1) % 3, sn, mun);  // matrix cores busy while the softmax below runs

    const int kbase = kb * KB;
    const bool masked = a.causal || (kbase + KB > kv_end);
    v8s pf[2][QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      if (masked) {
        const int qi = q0 + qt * 16 + fr + (Skv - a.Sq);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kbase + kt * 16 + 4 * fg + r;
            if (key >= kv_end || (a.causal && key > qi)) sc[kt][qt][r] = -INFINITY;
          }
      }
      // 16 scores -> 8 v_max3, then the 4 row groups via permlane swaps
      mfma_fence4(sc[0][qt], sc[1][qt], sc[2][qt], sc[3][qt]);
      float mx = vmax3(sc[0][qt][0], sc[0][qt][1], sc[0][qt][2]);
      mx = vmax3(mx, sc[0][qt][3], sc[1][qt][0]);
      mx = vmax3(mx, sc[1][qt][1], sc[1][qt][2]);
      mx = vmax3(mx, sc[1][qt][3], sc[2][qt][0]);
      mx = vmax3(mx, sc[2][qt][1], sc[2][qt][2]);
      mx = vmax3(mx, sc[2][qt][3], sc[3][qt][0]);
      mx = vmax3(mx, sc[3][qt][1], sc[3][qt][2]);
      mx = max_rowgroups(vmax3(mx, sc[3][qt][3], sc[3][qt][3]));
      // lazy rescale (cdna_hip_programming.md T13): keep the reference max unless
      // the block max exceeds it by > 2^8; p stays <= 256, exact after the final 1/l
      const float mb = PRE ? mx + muc[qt] : mx * sl2;  // block max in log2 units
      if (mb > mrow[qt] + 8.f) {
        const float mnew = fmaxf(mrow[qt], mb);
        const float alpha = __builtin_amdgcn_exp2f(mrow[qt] - mnew);
        mrow[qt] = mnew;
        lrow[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < DTO; ++dt) oacc[dt][qt] *= alpha;
      }
      if constexpr (PRE) {
        const float shift = mrow[qt] - muc[qt];  // 0 unless the max moved since issue
        if (__any(shift != 0.f)) {
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[kt][qt][r] -= shift;
        }
        if constexpr ((PROBE & 1) == 0) {
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[kt][qt][r] = __builtin_amdgcn_exp2f(sc[kt][qt][r]);
        }
      } else {
        const float mref = mrow[qt];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            sc[kt][qt][r] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kt][qt][r], sl2, -mref));
      }
      if constexpr (!ONES) {
        // 4 independent single-instruction chains (no v_pk_add_f32 beside MFMAs)
        float l4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) l4[r] = vadd_t(sc[0][qt][r], sc[1][qt][r]);
#pragma unroll
        for (int r = 0; r < 4; ++r) l4[r] = vadd(l4[r], vadd_t(sc[2][qt][r], sc[3][qt][r]));
        lrow[qt] = vadd(lrow[qt], vadd(vadd(l4[0], l4[1]), vadd(l4[2], l4[3])));
      }
#pragma unroll
      for (int kp2 = 0; kp2 < 2; ++kp2) {
        u32 w0 = pack2(sc[2 * kp2][qt][0], sc[2 * kp2][qt][1]);
        u32 w1 = pack2(sc[2 * kp2][qt][2], sc[2 * kp2][qt][3]);
        u32 w2 = pack2(sc[2 * kp2 + 1][qt][0], sc[2 * kp2 + 1][qt][1]);
        u32 w3 = pack2(sc[2 * kp2 + 1][qt][2], sc[2 * kp2 + 1][qt][3]);
        pf[kp2][qt] = __builtin_bit_cast(v8s, make_uint4(w0, w1, w2, w3));
      }
    }
    const bf16_t* vs = smem + cur * 2 * TILE + TILE;
    if constexpr ((PROBE & 4) != 0) {
#pragma unroll
      for (int kp2 = 0; kp2 < 2; ++kp2)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) asm volatile("" ::"v"(pf[kp2][qt]));
    }
#pragma unroll
    for (int kp2 = 0; kp2 < ((PROBE & 4) ? 0 : 2); ++kp2) {
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int qq = fr >> 2, pp = fr & 3;
        const int col = dt * 16 + 4 * pp;
        const int r0 = kp2 * 32 + 4 * fg + qq, r1 = r0 + 16;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vs + kv_off<CPR>(r0, col >> 3) + (col & 7)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vs + kv_off<CPR>(r1, col >> 3) + (col & 7)));
        v8s vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          oacc[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[kp2][qt], oacc[dt][qt], 0, 0, 0);
      }
      if constexpr (ONES) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
          oacc[DT][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[kp2][qt], oacc[DT][qt], 0, 0, 0);
      }
    }
    // block kb+2 -> the buffer that held block kb-1 (last read before the previous barrier)
    if (kb + 2 < nkb) store_kv((kb + 2) % 3);
    __syncthreads();
  };
  if (nkb > 0) qk(0, s_a, mu_a);
  for (int kb = 0; kb < nkb; kb += 2) {
    block(kb, s_a, mu_a, s_b, mu_b);
    if (kb + 1 < nkb) block(kb + 1, s_b, mu_b, s_a, mu_a);
  }

  bf16_t* op = a.o + b * a.sob + h * a.soh;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l;
    if constexpr (ONES) {
      l = oacc[DT][qt][0];  // every row of the ones tile holds this query's sum over all keys
    } else {
      l = lrow[qt];
      l += __shfl_xor(l, 16, 64);
      l += __shfl_xor(l, 32, 64);
    }
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    const int qi = q0 + qt * 16 + fr;
    if (qi >= a.Sq) continue;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d = dt * 16 + 4 * fg;
      if (d >= a.D) continue;
      uint2 w;
      w.x = pack2(oacc[dt][qt][0] * inv, oacc[dt][qt][1] * inv);
      w.y = pack2(oacc[dt][qt][2] * inv, oacc[dt][qt][3] * inv);
      *reinterpret_cast<uint2*>(op + qi * a.sos + d) = w;
    }
  }
}

// [64][64] bf16 K / V tile image of attn32_kernel: 16-byte chunk c of row r at
// slot c ^ f(r), f(r) = bits (r1, r2, r3) -> (4, 2, 1).  Conflict-free for the
// kernel's three access patterns (tools/attn32_swizzle.py checks them against
// the gfx950 lane groups): the K-fragment ds_read_b128 (lanes 0-31 = 32
// consecutive rows, one chunk: rows r and r + 8 share a lane group), the V^T
// ds_read_b64_tr_b16 (4 rows x 4 chunks per 32-lane half) and the row-wise
// ds_write_b128 staging.  The plain (r & 7) swizzle of kv_off is 2-way on the
// first two (SQ_LDS_BANK_CONFLICT 2.3 cycles per LDS instruction).
__device__ __forceinline__ int kv_off32(int row, int chunk) {
  const int f = ((row & 2) << 1) | ((row & 4) >> 1) | ((row & 8) >> 3);
  return row * 64 + ((chunk ^ f) << 3);
}

// 32x32x16 variant of the pipelined kernel (D <= 64): S^T = K Q^T and
// O^T = V^T P^T on v_mfma_f32_32x32x16_bf16.  At D = 64 the softmax is
// VALU-issue bound: a 16x16x32 MFMA (16 cycles) blocks vector issue for 8 of
// its cycles and leaves room for ~2 VALU instructions, a 32x32x16 one (32
// cycles) for ~5 (MI355X_MICROARCH.md 'vector-instruction ISSUE cost'), so the
// same exp / max / convert / sum work per score hides under the MFMAs with
// 1.5x the slack.  Layout (cdna_hip_programming.md §3 'An accumulator tile as
// the next MFMA's operand'): the S^T accumulator puts query r = lane & 31 on
// the lane and keys (i & 3) + 8 (i >> 2) + 4 (lane >> 5) of the 32-key tile in
// register i, so registers 8s..8s+7 (bf16 pairs) ARE the P^T fragment of PV
// k-step s, and the matching V^T fragment (keys 16s + 4h + 0..3 and +8) is two
// ds_read_b64_tr_b16 of the row-major V tile.  Row max: in-lane over 32 scores
// + one permlane32 swap; row sum: in-lane partials, the two lane halves added
// at the end.  Q pre-scaled, the QK^T chain starts from -max (PRE), lazy
// rescale (T13, threshold 2^8), same 3-buffer register-staged K/V ring and
// one-barrier-per-block software pipeline (QK^T of block kb+1 issued before
// the softmax of block kb) as attn_fwd_pipe_kernel.
// QB: 32-query tiles per wave (QB = 2, 256 rows per workgroup at one wave per
// SIMD, was 1.6x slower and spills; only QB = 1 is instantiated).
// PROBE (profiling builds, wrong results by design; variants 31/32/34/38):
// 1 = no exp, 2 = no K/V global loads past the first two blocks, 4 = no PV
// MFMAs, 8 = no QK^T MFMAs
// Measured and removed (round 4): the -mu offset as one MFMA from a zero
// accumulator, and the row sum on an all-ones O^T tile of the PV chain — both
// slower than the register moves / VALU adds they replaced.
template <int QB, int PROBE = 0>
__global__ __launch_bounds__(256, (QB == 1 ? 2 : 1)) void attn32_kernel(const AttnArgs a) {
  constexpr int DP = 64, CPR = DP / 8, KB = 64;
  constexpr int QROWS = QB * 32 * 4;
  constexpr int TILE = KB * DP;
  constexpr int LPT = KB * CPR / 256;
  constexpr int NBUF = 3;
  __shared__ __attribute__((aligned(16))) bf16_t smem[NBUF * 2 * TILE];  // (K, V) x 3

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int fr = lane & 15, fg = lane >> 4;
  const int Skv = a.kv_len ? min(a.Skv, *a.kv_len) : a.Skv;
  const int nqb = (a.Sq + QROWS - 1) / QROWS;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int nsp = a.kv_split > 1 ? a.kv_split : 1;
  const int ks = wg % nsp;  // key split of this workgroup (the splits of a query block share an XCD)
  const int bh = (wg / nsp) / nqb, qb = (wg / nsp) % nqb;
  const int b = bh / a.H, h = bh % a.H;
  const int q0 = qb * QROWS + wid * QB * 32;
  const bf16_t* qp = a.q + b * a.sqb + h * a.sqh;
  const bf16_t* kp = a.k + b * a.skb + h * a.skh;
  const bf16_t* vp = a.v + b * a.svb + h * a.svh;
  const float sl2 = a.scale_log2;

  // Q^T fragments (B operand): lane holds Q[q0 + qt*32 + r][ds*16 + 8*hh .. +7] * scale*log2(e)
  v8s qf[QB][4];
#pragma unroll
  for (int qt = 0; qt < QB; ++qt)
#pragma unroll
    for (int ds = 0; ds < 4; ++ds) {
      const int qi = q0 + qt * 32 + r, d = ds * 16 + 8 * hh;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (qi < a.Sq && d < a.D) v = *reinterpret_cast<const uint4*>(qp + qi * a.sqs + d);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[qt][ds] = __builtin_bit_cast(v8s, pack8(f));
    }
  v16f oacc[2][QB];  // O^T d-tile dt: query r, d = dt*32 + (i & 3) + 8 (i >> 2) + 4 hh
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int qt = 0; qt < QB; ++qt)
#pragma unroll
      for (int i = 0; i < 16; ++i) oacc[dt][qt][i] = 0.f;
  float mrow[QB], lrow[QB];  // running max (log2 units); this lane's partial row sum
#pragma unroll
  for (int qt = 0; qt < QB; ++qt) {
    mrow[qt] = -1e30f;
    lrow[qt] = 0.f;
  }

  int kv_end = Skv;
  if (a.causal) {
    const int qlast = min(a.Sq, (qb + 1) * QROWS) - 1 + (Skv - a.Sq);
    kv_end = min(Skv, qlast + 1);
  }
  const int nkb_all = (kv_end + KB - 1) / KB;
  const int per = (nkb_all + nsp - 1) / nsp;
  const int kb0 = ks * per;  // this workgroup's first key block; kb below counts from it
  const int nkb = max(0, min(nkb_all, kb0 + per) - kb0);

  uint4 rk[LPT], rv[LPT];
  auto load_kv = [&](int kb) {
    if constexpr ((PROBE & 2) != 0) {
      if (kb >= 2) return;
    }
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
      const int key = min((kb0 + kb) * KB + row, Skv - 1), d = c * 8;  // clamped rows are masked later
      CSK_DCHECK(key >= 0, 24, key, Skv);
      uint4 vk = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (d < a.D) {
        vk = *reinterpret_cast<const uint4*>(kp + key * a.sks + d);
        vv = *reinterpret_cast<const uint4*>(vp + key * a.svs + d);
      }
      rk[i] = vk;
      rv[i] = vv;
    }
  };
  auto store_kv = [&](int buf) {
    bf16_t* ks = smem + buf * 2 * TILE;
    bf16_t* vs = ks + TILE;
    CSK_DCHECK(buf >= 0 && buf < 3, 25, buf, 3);
#pragma unroll
    for (int i = 0; i < LPT; ++i) {
      const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
      *reinterpret_cast<uint4*>(ks + kv_off32(row, c)) = rk[i];
      *reinterpret_cast<uint4*>(vs + kv_off32(row, c)) = rv[i];
    }
  };
  // scores of one 64-key block: s[kt][qt] = S^T of keys kt*32.. (issued with offset -mu)
  auto qk = [&](int buf, v16f (&s)[2][QB], float (&mu)[QB]) {
    const bf16_t* ks = smem + buf * 2 * TILE;
#pragma unroll
    for (int qt = 0; qt < QB; ++qt) mu[qt] = mrow[qt] > -1e29f ? mrow[qt] : 0.f;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int qt = 0; qt < QB; ++qt)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[kt][qt][i] = -mu[qt];
#pragma unroll
      for (int ds = 0; ds < ((PROBE & 8) ? 0 : 4); ++ds) {
        const v8s kf = *reinterpret_cast<const v8s*>(ks + kv_off32(kt * 32 + r, 2 * ds + hh));
#pragma unroll
        for (int qt = 0; qt < QB; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[qt][ds], s[kt][qt], 0, 0, 0);
      }
    }
  };

  if (nkb > 0) { load_kv(0); store_kv(0); }
  if (nkb > 1) { load_kv(1); store_kv(1); }
  __syncthreads();
  v16f s_a[2][QB], s_b[2][QB];
  float mu_a[QB], mu_b[QB];
  auto block = [&](int kb, v16f (&sc)[2][QB], float (&muc)[QB], v16f (&sn)[2][QB], float (&mun)[QB]) {
    const int cur = kb % NBUF;
    if (kb + 2 < nkb) load_kv(kb + 2);
    if (kb + 1 < nkb) qk((kb + 1) % NBUF, sn, mun);  // matrix cores busy while the softmax below runs

    const int kbase = (kb0 + kb) * KB;
    const bool masked = a.causal || (kbase + KB > kv_end);
    v8s pf[2][2][QB];  // [key tile][PV k-step][query tile]
#pragma unroll
    for (int qt = 0; qt < QB; ++qt) {
      if (masked) {
        const int qi = q0 + qt * 32 + r + (Skv - a.Sq);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kbase + kt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
            if (key >= kv_end || (a.causal && key > qi)) sc[kt][qt][i] = -INFINITY;
          }
      }
      mfma_fence16(sc[0][qt], sc[1][qt]);
      // row max as a depth-3 tree of max3 (11 independent, then 4 + 2) instead of
      // a 17-deep dependent chain: -0.018 ms per CFG-8 step, neutral at CFG 2
      // (profiles/unet_step_ab_attn32_tree_r7g.txt)
      float mx;
      {
        const v16f& x0 = sc[0][qt];
        const v16f& x1 = sc[1][qt];
        const float t0 = vmax3(x0[0], x0[1], x0[2]), t1 = vmax3(x0[3], x0[4], x0[5]);
        const float t2 = vmax3(x0[6], x0[7], x0[8]), t3 = vmax3(x0[9], x0[10], x0[11]);
        const float t4 = vmax3(x0[12], x0[13], x0[14]), t5 = vmax3(x0[15], x1[0], x1[1]);
        const float t6 = vmax3(x1[2], x1[3], x1[4]), t7 = vmax3(x1[5], x1[6], x1[7]);
        const float t8 = vmax3(x1[8], x1[9], x1[10]), t9 = vmax3(x1[11], x1[12], x1[13]);
        const float t10 = vmax3(x1[14], x1[15], x1[15]);
        const float u0 = vmax3(t0, t1, t2), u1 = vmax3(t3, t4, t5), u2 = vmax3(t6, t7, t8);
        const float u3 = vmax3(t9, t10, t10);
        mx = vmax3(vmax3(u0, u1, u2), u3, u3);
      }
      {  // the other 32 keys of this query live in lane ^ 32
        const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(mx), __float_as_uint(mx), false, false);
        mx = vmax3(__uint_as_float(x[0]), __uint_as_float(x[1]), __uint_as_float(x[1]));
      }
      const float mb = mx + muc[qt];  // block max, log2 units
      if (mb > mrow[qt] + 8.f) {
        const float mnew = fmaxf(mrow[qt], mb);
        const float alpha = __builtin_amdgcn_exp2f(mrow[qt] - mnew);
        mrow[qt] = mnew;
        lrow[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) oacc[dt][qt] *= alpha;
      }
      const float shift = mrow[qt] - muc[qt];  // 0 unless the max moved since the block was issued
      if (__any(shift != 0.f)) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) sc[kt][qt][i] -= shift;
      }
      if constexpr ((PROBE & 1) == 0) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) sc[kt][qt][i] = __builtin_amdgcn_exp2f(sc[kt][qt][i]);
      }
      {
        // 4 independent single-instruction add chains (no v_pk_add_f32 beside MFMAs)
        float l4[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          l4[c] = vadd_t(sc[0][qt][c], sc[0][qt][c + 4]);  // (exp results: trans-hazard-safe adds)
          l4[c] = vadd(l4[c], vadd_t(sc[0][qt][c + 8], sc[0][qt][c + 12]));
          l4[c] = vadd(l4[c], vadd_t(sc[1][qt][c], sc[1][qt][c + 4]));
          l4[c] = vadd(l4[c], vadd_t(sc[1][qt][c + 8], sc[1][qt][c + 12]));
        }
        lrow[qt] = vadd(lrow[qt], vadd(vadd(l4[0], l4[1]), vadd(l4[2], l4[3])));
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int o = 8 * st;
          const u32 w0 = pack2(sc[kt][qt][o + 0], sc[kt][qt][o + 1]);
          const u32 w1 = pack2(sc[kt][qt][o + 2], sc[kt][qt][o + 3]);
          const u32 w2 = pack2(sc[kt][qt][o + 4], sc[kt][qt][o + 5]);
          const u32 w3 = pack2(sc[kt][qt][o + 6], sc[kt][qt][o + 7]);
          pf[kt][st][qt] = __builtin_bit_cast(v8s, make_uint4(w0, w1, w2, w3));
        }
    }
    const bf16_t* vs = smem + cur * 2 * TILE + TILE;
    // V^T fragment of PV k-step (kt, st), d-tile dt: lane 4q+p of 16-lane group g
    // addresses key row kt*32 + 16 st + 4 (g >> 1) + q (+8 for elements 4..7),
    // columns dt*32 + 16 (g & 1) + 4p .. +3; lane i of the group receives column i
    const int qq = fr >> 2, pp = fr & 3;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const int col = dt * 32 + 16 * (fg & 1) + 4 * pp;
          const int r0 = kt * 32 + 16 * st + 4 * (fg >> 1) + qq, r1 = r0 + 8;
          const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vs + kv_off32(r0, col >> 3) + (col & 7)));
          const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vs + kv_off32(r1, col >> 3) + (col & 7)));
          const v8s vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int qt = 0; qt < QB; ++qt) {
            if constexpr ((PROBE & 4) != 0) {
              asm volatile("" ::"v"(vf), "v"(pf[kt][st][qt]));
            } else {
              oacc[dt][qt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt][st][qt], oacc[dt][qt], 0, 0, 0);
            }
          }
        }
    if (kb + 2 < nkb) store_kv((kb + 2) % 3);
    __syncthreads();
  };
  if (nkb > 0) qk(0, s_a, mu_a);
  for (int kb = 0; kb < nkb; kb += 2) {
    block(kb, s_a, mu_a, s_b, mu_b);
    if (kb + 1 < nkb) block(kb + 1, s_b, mu_b, s_a, mu_a);
  }

  if (nsp > 1) {  // unnormalised partials; attn_split_combine_kernel merges the splits
    const size_t rows = (size_t)a.B * a.H * a.Sq;
#pragma unroll
    for (int qt = 0; qt < QB; ++qt) {
      const float l = lrow[qt] + __shfl_xor(lrow[qt], 32, 64);
      const int qi = q0 + qt * 32 + r;
      if (qi >= a.Sq) continue;
      const size_t row = (size_t)ks * rows + (size_t)bh * a.Sq + qi;
      if (hh == 0) *reinterpret_cast<float2*>(a.part_ml + row * 2) = make_float2(mrow[qt], l);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hh;
          *reinterpret_cast<float4*>(a.part_o + row * 64 + d) =
              make_float4(oacc[dt][qt][4 * g], oacc[dt][qt][4 * g + 1], oacc[dt][qt][4 * g + 2], oacc[dt][qt][4 * g + 3]);
        }
    }
    return;
  }
  bf16_t* op = a.o + b * a.sob + h * a.soh;
#pragma unroll
  for (int qt = 0; qt < QB; ++qt) {
    const float l = lrow[qt] + __shfl_xor(lrow[qt], 32, 64);
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    const int qi = q0 + qt * 32 + r;
    if (qi >= a.Sq) continue;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        if (d >= a.D) continue;
        uint2 w;
        w.x = pack2(oacc[dt][qt][4 * g] * inv, oacc[dt][qt][4 * g + 1] * inv);
        w.y = pack2(oacc[dt][qt][4 * g + 2] * inv, oacc[dt][qt][4 * g + 3] * inv);
        *reinterpret_cast<uint2*>(op + qi * a.sos + d) = w;
      }
  }
}

// Split-KV combine: O = sum_s 2^(m_s - M) O_s / sum_s 2^(m_s - M) l_s with
// M = max_s m_s, one thread per (b, h, query, 8 head-dim columns)
__global__ void attn_split_combine_kernel(const AttnArgs a) {
  const size_t rows = (size_t)a.B * a.H * a.Sq;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= rows * 8) return;
  const size_t row = i / 8;
  const int d = (int)(i % 8) * 8;
  const int nsp = a.kv_split;
  float mmax = -1e30f;
  for (int s = 0; s < nsp; ++s) mmax = fmaxf(mmax, a.part_ml[((size_t)s * rows + row) * 2]);
  float l = 0.f, o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = 0.f;
  for (int s = 0; s < nsp; ++s) {
    const float2 ml = *reinterpret_cast<const float2*>(a.part_ml + ((size_t)s * rows + row) * 2);
    const float w = __builtin_amdgcn_exp2f(ml.x - mmax);
    l = __builtin_fmaf(w, ml.y, l);
    const float4 lo = *reinterpret_cast<const float4*>(a.part_o + ((size_t)s * rows + row) * 64 + d);
    const float4 hi = *reinterpret_cast<const float4*>(a.part_o + ((size_t)s * rows + row) * 64 + d + 4);
    o[0] += w * lo.x; o[1] += w * lo.y; o[2] += w * lo.z; o[3] += w * lo.w;
    o[4] += w * hi.x; o[5] += w * hi.y; o[6] += w * hi.z; o[7] += w * hi.w;
  }
  const float inv = l > 0.f ? 1.0f / l : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] *= inv;
  const int bh = (int)(row / a.Sq), qi = (int)(row % a.Sq);
  const int b = bh / a.H, h = bh % a.H;
  if (d < a.D) *reinterpret_cast<uint4*>(a.o + b * a.sob + h * a.soh + (size_t)qi * a.sos + d) = pack8(o);
}

// Short-KV attention (Skv <= 128, D <= 64, no mask: the UNet's cross-attention
// over 77 text tokens): the whole K and V (<= 128 x 64 each, 32 KB) are staged
// into LDS ONCE per workgroup, then each wave walks ROWS / 64 query tiles of 16
// rows with no further barrier.  Every key is present, so the softmax is exact
// in one pass (row max, exp2, sum) — no online rescale.  The pipelined kernel
// spent most of its time here in per-block prologue / epilogue for a 2-block
// key loop, and re-loaded K / V for every 64 query rows.
template <int ROWS>
__global__ __launch_bounds__(256) void attn_shortkv_kernel(const AttnArgs a) {
  constexpr int DP = 64, CPR = 8, KMAX = 128, DT = 4;
  constexpr int TILE = KMAX * DP;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * TILE];  // K, V: [128][64] each
  bf16_t* ks = smem;
  bf16_t* vs = smem + TILE;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int Skv = a.Skv;
  const int nkt = (Skv + 15) / 16;  // 16-key tiles holding a real key
  const int nqb = (a.Sq + ROWS - 1) / ROWS;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int bh = wg / nqb, qb = wg % nqb;
  const int b = bh / a.H, h = bh % a.H;
  const bf16_t* qp = a.q + b * a.sqb + h * a.sqh;
  const bf16_t* kp = a.k + b * a.skb + h * a.skh;
  const bf16_t* vp = a.v + b * a.svb + h * a.svh;
  const float sl2 = a.scale_log2;

  // Q rows of tile t (lane: query q0 + fr, d chunk ds * 32 + 8 * fg), loaded one
  // tile ahead so the next tile's global loads overlap this tile's MFMAs
  auto load_q = [&](int t, uint4 (&v)[2]) {
    const int qi = qb * ROWS + t * 16 + fr;
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      const int d = ds * 32 + 8 * fg;
      v[ds] = (t < ROWS / 16 && qi < a.Sq && d < a.D) ? *reinterpret_cast<const uint4*>(qp + qi * a.sqs + d)
                                                     : make_uint4(0, 0, 0, 0);
    }
  };
  uint4 qnext[2];
  load_q(wid, qnext);  // issued before the K / V staging so the two global latencies overlap

  // K / V -> LDS (rows >= Skv and columns >= D zero: their P and V^T entries
  // vanish); all 8 loads of a thread issued before its first LDS store
  constexpr int KVI = KMAX * CPR / 256;
  uint4 vk[KVI], vv[KVI];
#pragma unroll
  for (int i = 0; i < KVI; ++i) {
    const int id = tid + 256 * i, row = id / CPR, d = (id % CPR) * 8;
    vk[i] = vv[i] = make_uint4(0, 0, 0, 0);
    if (row < Skv && d < a.D) {
      vk[i] = *reinterpret_cast<const uint4*>(kp + row * a.sks + d);
      vv[i] = *reinterpret_cast<const uint4*>(vp + row * a.svs + d);
    }
  }
#pragma unroll
  for (int i = 0; i < KVI; ++i) {
    const int id = tid + 256 * i, row = id / CPR, c = id % CPR;
    CSK_DCHECK(kv_off<CPR>(row, c) + 8 <= TILE, 23, row, TILE);
    *reinterpret_cast<uint4*>(ks + kv_off<CPR>(row, c)) = vk[i];
    *reinterpret_cast<uint4*>(vs + kv_off<CPR>(row, c)) = vv[i];
  }
  __syncthreads();
  for (int t = wid; t < ROWS / 16; t += 4) {
    const int q0 = qb * ROWS + t * 16;
    if (q0 >= a.Sq) break;
    // Q fragments (B operand), pre-scaled into log2 units
    uint4 qraw[2] = {qnext[0], qnext[1]};
    if (ROWS > 64) load_q(t + 4, qnext);
    v8s qf[2];
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) {
      float f[8];
      unpack8(qraw[ds], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[ds] = __builtin_bit_cast(v8s, pack8(f));
    }
    // S^T = K Q^T: lane (fr, fg) holds keys kt*16 + 4fg + r of query q0 + fr
    v4f s[8];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      s[kt] = v4f{0.f, 0.f, 0.f, 0.f};
      if (kt < nkt) {
#pragma unroll
        for (int ds = 0; ds < 2; ++ds) {
          const v8s kf = *reinterpret_cast<const v8s*>(ks + kv_off<CPR>(kt * 16 + fr, ds * 4 + fg));
          s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ds], s[kt], 0, 0, 0);
        }
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (kt * 16 + 4 * fg + r >= Skv) s[kt][r] = -INFINITY;
          mx = fmaxf(mx, s[kt][r]);
        }
      }
    }
    mx = max_rowgroups(mx);
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = kt < nkt ? __builtin_amdgcn_exp2f(s[kt][r] - mx) : 0.f;
        s[kt][r] = p;
        l += p;
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    // O^T = V^T P^T over 32-key groups (P^T straight from the S^T registers)
    v4f o[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kp2 = 0; kp2 < 4; ++kp2) {
      if (2 * kp2 < nkt) {
        const u32 w0 = pack2(s[2 * kp2][0], s[2 * kp2][1]);
        const u32 w1 = pack2(s[2 * kp2][2], s[2 * kp2][3]);
        const u32 w2 = pack2(s[2 * kp2 + 1][0], s[2 * kp2 + 1][1]);
        const u32 w3 = pack2(s[2 * kp2 + 1][2], s[2 * kp2 + 1][3]);
        const v8s pf = __builtin_bit_cast(v8s, make_uint4(w0, w1, w2, w3));
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int qq = fr >> 2, pp = fr & 3;
          const int col = dt * 16 + 4 * pp;
          const int r0 = kp2 * 32 + 4 * fg + qq, r1 = r0 + 16;
          v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vs + kv_off<CPR>(r0, col >> 3) + (col & 7)));
          v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(vs + kv_off<CPR>(r1, col >> 3) + (col & 7)));
          v8s vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
        }
      }
    }
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    const int qi = q0 + fr;
    if (qi < a.Sq) {
      bf16_t* op = a.o + b * a.sob + h * a.soh + qi * a.sos;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int d = dt * 16 + 4 * fg;
        if (d >= a.D) continue;
        uint2 w;
        w.x = pack2(o[dt][0] * inv, o[dt][1] * inv);
        w.y = pack2(o[dt][2] * inv, o[dt][3] * inv);
        *reinterpret_cast<uint2*>(op + d) = w;
      }
    }
  }
}

template <int DP, int QT, int DV = DP>
static int launch_attn(const AttnArgs& a, hipStream_t s) {
  constexpr int QROWS = QT * 64;
  const int nqb = (a.Sq + QROWS - 1) / QROWS;
  attn_fwd_kernel<DP, QT, DV><<<a.B * a.H * nqb, 256, 0, s>>>(a);
  return (int)hipGetLastError();
}

// Short-KV (Skv <= 128, D <= 64: UNet cross-attention over 77 text tokens)
// kernel choice for variant 0: 1 = plain, 64-row workgroups; 2 = pipelined
// QT=1; 3 = K/V-resident one-pass kernel (attn_shortkv_kernel, no mask / no
// device-side length: otherwise 2).
static int g_short_kv_variant = 3;
static int g_short_kv_rows = 0;  // attn_shortkv_kernel query rows per workgroup: 0 = auto, 64 / 128 / 256
CSK_API int csk_set_short_kv_rows(int r) {
  g_short_kv_rows = r;
  return 0;
}
CSK_API int csk_set_short_kv_variant(int v) {
  g_short_kv_variant = v;
  return 0;
}

// Default for D = 64, Skv > 128 (the UNet self-attention): the 32x32x16 kernel
// (attn32_kernel, 1) or the 16x16x32 pipelined one (0; A/B knob)
static int g_attn32 = 1;
CSK_API int csk_set_attn32(int on) {
  g_attn32 = on;
  return 0;
}

// variant: 0 = default choice, 1 = plain double-buffered loop, 2 = pipelined (D <= 64),
// 3 = pipelined + PRE, 4 = pipelined + ONES, 5 = pipelined + PRE + ONES
extern "C" int csk_attention_wide(void* o, const void* q, const void* k, const void* v, const long long* strides,
                                  int B, int H, int Sq, int Skv, int D, float scale, hipStream_t stream);
// attn_fa.hip: persistent stream-K d = 64 kernel (default for the shapes it takes)
extern "C" int csk_attn_fa_ok(int B, int H, int Sq, int Skv, int D, int causal, int has_kv_len);
extern "C" int csk_attention_fa(void* o, const void* q, const void* k, const void* v, const long long* strides, int B,
                                int H, int Sq, int Skv, int D, float scale, int workers, hipStream_t stream);

CSK_API int csk_attention(void* o, const void* q, const void* k, const void* v, const long long* strides, int B, int H,
                          int Sq, int Skv, int D, float scale, int causal, int variant, const void* kv_len,
                          hipStream_t stream) {
  // strides: q(b,s,h), k(b,s,h), v(b,s,h), o(b,s,h) in elements
  if (D > 256 && D <= 512 && !causal && !kv_len)  // VAE mid-block: single head, d = 512
    return csk_attention_wide(o, q, k, v, strides, B, H, Sq, Skv, D, scale, stream);
  if (D % 8 != 0 || D > 256) return (int)hipErrorInvalidValue;
  if (variant == 0 && csk_attn_fa_ok(B, H, Sq, Skv, D, causal, kv_len != nullptr))
    return csk_attention_fa(o, q, k, v, strides, B, H, Sq, Skv, D, scale, 0, stream);
  AttnArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.sqb = strides[0]; a.sqs = strides[1]; a.sqh = strides[2];
  a.skb = strides[3]; a.sks = strides[4]; a.skh = strides[5];
  a.svb = strides[6]; a.svs = strides[7]; a.svh = strides[8];
  a.sob = strides[9]; a.sos = strides[10]; a.soh = strides[11];
  a.B = B; a.H = H; a.Sq = Sq; a.Skv = Skv; a.D = D;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.causal = causal;
  a.kv_len = (const int*)kv_len;
  a.kv_split = 1;
  a.part_o = a.part_ml = nullptr;
  const long long wg4 = (long long)B * H * ((Sq + 255) / 256);
  (void)wg4;  // QT=4 (64 rows/wave) measured slower on MI355X (1 wave/SIMD at 364 regs)
  if (D <= 64) {
    if (variant == 0 && g_attn32 && D == 64 && Skv > 128) variant = 20;
    if (variant >= 31 && variant <= 38) {  // attn32 profiling probes (wrong results by design)
      const dim3 g1(B * H * ((Sq + 127) / 128));
      switch (variant) {
        case 31: attn32_kernel<1, 1><<<g1, 256, 0, stream>>>(a); break;
        case 32: attn32_kernel<1, 2><<<g1, 256, 0, stream>>>(a); break;
        case 34: attn32_kernel<1, 4><<<g1, 256, 0, stream>>>(a); break;
        case 38: attn32_kernel<1, 8><<<g1, 256, 0, stream>>>(a); break;
        default: return (int)hipErrorInvalidValue;
      }
      return (int)hipGetLastError();
    }
    if (variant == 20) {  // 32x32x16 MFMA kernel, 128 query rows per workgroup
      const dim3 g32(B * H * ((Sq + 127) / 128));
      attn32_kernel<1><<<g32, 256, 0, stream>>>(a);
      return (int)hipGetLastError();
    }
    if (variant >= 2 || (variant == 0 && Skv > 128)) {
      // PRE+ONES: 279 vs 283 (PRE) vs 306 us (plain) at B8 S4096 H5, same box; for
      // short grids (< 1024 workgroups of 128 rows: S1024 H10) 64-row workgroups
      // fill the chip better (55 vs 58 us)
      if (variant == 0) variant = ((long long)B * H * ((Sq + 127) / 128) < 1024) ? 7 : 5;
      if (variant == 6) {  // 48 query rows per wave (QT = 3): more MFMA work per K/V block and barrier
        const dim3 grid3(B * H * ((Sq + 191) / 192));
        attn_fwd_pipe_kernel<3, true, true><<<grid3, 256, 0, stream>>>(a);
        return (int)hipGetLastError();
      }
      if (variant == 9) {  // 3 workgroups per CU (12 waves): registers capped at 168
        attn_fwd_pipe_kernel<2, true, true, 0, 3><<<dim3(B * H * ((Sq + 127) / 128)), 256, 0, stream>>>(a);
        return (int)hipGetLastError();
      }
      if (variant >= 11 && variant <= 18) {  // profiling probes (wrong results by design)
        const dim3 gp(B * H * ((Sq + 127) / 128));
        switch (variant) {
          case 11: attn_fwd_pipe_kernel<2, true, true, 1><<<gp, 256, 0, stream>>>(a); break;
          case 12: attn_fwd_pipe_kernel<2, true, true, 2><<<gp, 256, 0, stream>>>(a); break;
          case 14: attn_fwd_pipe_kernel<2, true, true, 4><<<gp, 256, 0, stream>>>(a); break;
          case 18: attn_fwd_pipe_kernel<2, true, true, 8><<<gp, 256, 0, stream>>>(a); break;
          default: return (int)hipErrorInvalidValue;
        }
        return (int)hipGetLastError();
      }
      if (variant == 7) {  // 16 query rows per wave (QT = 1): twice the workgroups for short sequences
        const dim3 grid1(B * H * ((Sq + 63) / 64));
        attn_fwd_pipe_kernel<1, true, true><<<grid1, 256, 0, stream>>>(a);
        return (int)hipGetLastError();
      }
      const int nqb = (Sq + 127) / 128;
      const dim3 grid(B * H * nqb);
      switch (variant) {
        case 2: attn_fwd_pipe_kernel<2, false, false><<<grid, 256, 0, stream>>>(a); break;
        case 3: attn_fwd_pipe_kernel<2, true, false><<<grid, 256, 0, stream>>>(a); break;
        case 4: attn_fwd_pipe_kernel<2, false, true><<<grid, 256, 0, stream>>>(a); break;
        default: attn_fwd_pipe_kernel<2, true, true><<<grid, 256, 0, stream>>>(a); break;
      }
      return (int)hipGetLastError();
    }
    if (variant == 0 && Skv <= 128) {
      if (g_short_kv_variant == 3 && !causal && !kv_len && Skv >= 1) {
        // auto: 128 query rows per workgroup (2 tiles per wave) when that still
        // gives >= 512 workgroups, else 64 (one tile per wave); 128 measured best
        // at S = 4096 / 1024 (20.6 / 12.8 us vs 24.0 / 16.8 for the pipelined
        // kernel, 22.1 / 16.7 at 256 rows: profiles/attn_shortkv_r3j.txt)
        int rows = g_short_kv_rows;
        if (rows == 0) rows = (long long)B * H * ((Sq + 127) / 128) >= 512 ? 128 : 64;
        if (rows == 256) {
          attn_shortkv_kernel<256><<<dim3(B * H * ((Sq + 255) / 256)), 256, 0, stream>>>(a);
        } else if (rows == 128) {
          attn_shortkv_kernel<128><<<dim3(B * H * ((Sq + 127) / 128)), 256, 0, stream>>>(a);
        } else {
          attn_shortkv_kernel<64><<<dim3(B * H * ((Sq + 63) / 64)), 256, 0, stream>>>(a);
        }
        return (int)hipGetLastError();
      }
      if (g_short_kv_variant == 1) return launch_attn<64, 1>(a, stream);
      if (g_short_kv_variant >= 2) {  // (3 with a mask or device-side length)
        attn_fwd_pipe_kernel<1, true, true><<<dim3(B * H * ((Sq + 63) / 64)), 256, 0, stream>>>(a);
        return (int)hipGetLastError();
      }
    }
    if (D <= 48) return launch_attn<64, 2, 48>(a, stream);  // SD1.5 64x64 level, d = 40
    return launch_attn<64, 2>(a, stream);
  }
  if (D <= 80) return launch_attn<128, 2, 80>(a, stream);  // SD1.5 32x32 level
  if (D <= 128) return launch_attn<128, 2>(a, stream);
  if (D <= 160) return launch_attn<256, 1, 160>(a, stream);  // SD1.5 16x16 / 8x8 levels
  return launch_attn<256, 1>(a, stream);
}

CSK_DEBUG_EXPORT(attention)

// Split-KV self-attention for grids that cannot fill the chip (batch-1 jobs:
// CFG batch 2, the CFG-shared prefix at batch 1): kv_split workgroups per
// 128-query block, fp32 partials in the caller's workspace (graph-capturable),
// then one combine pass.  D == 64, no mask, no device-side key count.
// part_o: kv_split * B*H*Sq * 64 floats, part_ml: kv_split * B*H*Sq * 2 floats.
CSK_API int csk_attention_split(void* o, const void* q, const void* k, const void* v, const long long* strides,
                                int B, int H, int Sq, int Skv, int D, float scale, int kv_split, void* part_o,
                                void* part_ml, hipStream_t stream) {
  if (D != 64 || kv_split < 2 || kv_split > 16 || !part_o || !part_ml) return (int)hipErrorInvalidValue;
  AttnArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.sqb = strides[0]; a.sqs = strides[1]; a.sqh = strides[2];
  a.skb = strides[3]; a.sks = strides[4]; a.skh = strides[5];
  a.svb = strides[6]; a.svs = strides[7]; a.svh = strides[8];
  a.sob = strides[9]; a.sos = strides[10]; a.soh = strides[11];
  a.B = B; a.H = H; a.Sq = Sq; a.Skv = Skv; a.D = D;
  a.scale_log2 = scale * 1.4426950408889634f;
  a.causal = 0;
  a.kv_len = nullptr;
  a.kv_split = kv_split;
  a.part_o = (float*)part_o;
  a.part_ml = (float*)part_ml;
  const dim3 gs(B * H * ((Sq + 127) / 128) * kv_split);
  attn32_kernel<1><<<gs, 256, 0, stream>>>(a);
  const size_t n = (size_t)B * H * Sq * 8;
  attn_split_combine_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(a);
  return (int)hipGetLastError();
}
