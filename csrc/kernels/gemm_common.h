// Shared pieces of the MFMA GEMM / implicit-GEMM conv kernels (gemm.hip:
// register-staged pipeline; gemm_glds.hip: LDS-DMA multi-stage pipeline).
#pragma once
#include "common.h"
#include "attn_tile.h"

enum {
  ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_GEGLU = 3, ACT_QGELU = 4,
  ACT_LRELU = 5,       // leaky relu 0.2 (ESRGAN)
  ACT_LRELU_01 = 6,    // leaky relu 0.1 (HiFi-GAN)
  ACT_TANH = 7,
  ACT_RELU = 8,
  ACT_LRELU_001 = 9,   // leaky relu 0.01 (torch default)
  ACT_ELU = 10,        // EnCodec
  ACT_GELU_TANH = 11,  // T5 "gelu_new"
  ACT_PROBE_NO_EPILOGUE = 99,  // profiling only: skip the epilogue (tilebench --probe)
  ACT_PROBE_NO_STORE = 97,     // profiling only: LDS-staged epilogue without its global stores
  ACT_PROBE_NO_A = 98,         // profiling only (2-stage conv tiles): skip the A DMA of kx != 0 taps
                               // (wrong results; times a kx-halo A reuse, tilebench --probe-halo)
};

// The libm-heavy activations (tanh, ELU's expm1, tanh-GELU: vocoder / EnCodec /
// T5 paths only) live in ONE out-of-line function per code object.  Inlined
// into every epilogue site they made the epilogue of each GEMM / conv
// instantiation ~22 K instructions long (10 activations x 8 unrolled values x
// every store path); the executed path then ran from a cold instruction cache
// on every workgroup's single epilogue.  The UNet's activations (none / SiLU /
// GELU / quick-GELU / ReLU / leaky ReLU) stay inline.
struct Act8 {
  float v[8];
};
static __device__ __attribute__((noinline)) Act8 act8_exotic(int act, Act8 x) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float v = x.v[j];
    float r = v;
    if (act == ACT_TANH) r = tanhf(v);
    else if (act == ACT_ELU) r = v > 0.f ? v : expm1f(v);
    else if (act == ACT_GELU_TANH) r = 0.5f * v * (1.f + tanhf(0.7978845608028654f * (v + 0.044715f * v * v * v)));
    x.v[j] = r;
  }
  return x;
}

__device__ __forceinline__ bool act_exotic(int act) {
  return act == ACT_TANH || act == ACT_ELU || act == ACT_GELU_TANH;
}

// pointwise epilogue activation (every act except GEGLU, which pairs columns)
__device__ __forceinline__ float apply_act(int act, float v) {
  switch (act) {
    case ACT_GELU: return gelu_f(v);
    case ACT_SILU: return silu_f(v);
    case ACT_QGELU: return qgelu_f(v);
    case ACT_LRELU: return v > 0.f ? v : 0.2f * v;
    case ACT_LRELU_01: return v > 0.f ? v : 0.1f * v;
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_LRELU_001: return v > 0.f ? v : 0.01f * v;
    default: break;
  }
  if (act_exotic(act)) {
    Act8 x{};
    x.v[0] = v;
    return act8_exotic(act, x).v[0];
  }
  return v;
}

struct GemmArgs {
  const bf16_t* A;  // GEMM: [M][lda];  CONV: NHWC input [B][H][W][Cin]
  const bf16_t* W;  // [N][ldb] (K-contiguous rows)
  bf16_t* C;        // [M][ldc]
  const bf16_t* bias;    // [N] or null
  const bf16_t* bias2d;  // [B][ldb2] or null (row m uses b = m / rows_per_b)
  const bf16_t* res;     // [M][ldc] or null
  const bf16_t* zero;    // >= 16 zero bytes in global memory (LDS-DMA source for padding)
  int M, N, K, lda, ldb, ldc, rows_per_b, act;  // CONV: lda = input pixel stride (>= Cin)
  int ldr;          // residual row stride
  int ldb2;         // bias2d row stride (a column slice of one batched time-embedding GEMM)
  float out_scale;  // y = act(acc + bias + bias2d) * out_scale + residual
  float* ws;   // split-K fp32 partials [ksplit][M][N] (null: no split)
  int kchunk;  // K elements per split (multiple of BK)
  // conv geometry
  int H, Wd, Cin, Ho, Wo, kh, kw, stride, pt, pl, up2x;
  int dil;  // dilation (both spatial dims)
  // fused GroupNorm statistics of the OUTPUT (null: off): per (row tile, column)
  // (mean, M2) over the tile's BM rows; requires rows_per_batch % BM == 0, no
  // split-K, no GEGLU.  gn_part[((m0 / BM) * N + n) * 2 + {0, 1}]
  float* gn_part;
  int gn_seg;  // rows per gn_part segment (divides BM; 0 -> BM)
  int gn_lds;  // 1: GroupNorm statistics through the LDS epilogue even where the direct one can (A/B knob)
  int sw_odd;  // 1: row-layout tiles with an odd fragment count (160 wide) use the direct epilogue (A/B knob)
  int epi_band;  // 1: LDS-staged epilogue stores through the compile-time band path (A/B knob, default 1)
  int epi_nt;    // 1: the direct epilogue's C stores (2: and residual loads) are non-temporal (A/B knob)
  // fused LayerNorm of the INPUT rows (SURVEY K11 folded into K9/K10): the
  // weight was pre-multiplied by gamma (W' = W diag(gamma)), the bias holds
  // b + W beta, and the epilogue applies
  //   y = rstd_m * (acc - mean_m * ln_colsum[n]) + bias'
  // with (mean_m, rstd_m) merged from the PRODUCER's row partials
  // ln_part[(p * M + m) * 2 + {mean, M2}], p < ln_nparts, ln_pcols columns each
  // (the last part may be short; K columns in all).  No split-K.
  const float* ln_part;
  const float* ln_colsum;
  int ln_nparts, ln_pcols;
  float ln_eps;
  const float* ln_row;  // [M][2] (mean, rstd) merged from ln_part (ln_rowstats_kernel)
  // row statistics of the OUTPUT for a consumer's fused LayerNorm:
  // row_part[((n0 / BN) * M + m) * 2 + {mean, M2}] over the tile's columns.
  // No split-K, no GEGLU.
  float* row_part;
  // one past the last element an LDS-DMA may read from A / W (CSK_DEBUG checks)
  const bf16_t* a_end;
  const bf16_t* w_end;
  // attention epilogue (csk_gemm_ln_attn, 128x64 row-layout tiles): the tile's
  // 64 output columns are ONE head's queries; they attend over that head's
  // per-request K / V (attn_kv [Bc][attn_skv][2][N/64][64], sample m / rows_per_b)
  // and the tile stores the attention output instead of the projection
  const bf16_t* attn_kv;
  const bf16_t* attn_kv_end;
  int attn_skv;
  float attn_sl2;  // softmax scale * log2(e)
  // in-kernel split-K fixup (gemm_glds.hip, tuning split < 0): the fx_split
  // workgroups of an output tile each publish their fp32 partial to
  // fx_ws[tile][split] and bump fx_cnt[tile]; the last one sums the partials in
  // split order and runs the normal epilogue (every fusion of the unsplit tile)
  float* fx_ws;
  unsigned* fx_cnt;
  int fx_split;
};

#define ZERO_BYTES (128 * 1024)  // the LDS-DMA zero page (gemm_glds.hip: csk_init)

// Debug-check sites (CSK_DEBUG record field 1); +100: the LDS destination
enum DmaSite { SITE_GLDS_A = 1, SITE_GLDS_B, SITE_PERSIST_A, SITE_PERSIST_B,
               SITE_8P_A, SITE_8P_B, SITE_8R_A, SITE_8R_B, SITE_WIDE_KV };

typedef __attribute__((address_space(1))) const void* csk_gptr_t;
typedef __attribute__((address_space(3))) void* csk_lptr_t;

// One 16-byte-per-lane LDS-DMA (a wave writes 1 KB at dst).  CSK_DEBUG builds
// check each lane's source against the operand extents (A, W or the zero page)
// and the wave's destination against the workgroup's LDS array.
template <int SITE>
__device__ __forceinline__ void dma16(const GemmArgs& args, const bf16_t* src, bf16_t* dst, const bf16_t* lds,
                                      int lds_elems) {
#ifdef CSK_DEBUG
  const bool ok = (src >= args.A && src + 8 <= args.a_end) || (src >= args.W && src + 8 <= args.w_end) ||
                  (src >= args.zero && src + 8 <= args.zero + ZERO_BYTES / 2);
  CSK_DCHECK(ok, SITE, src - args.A, args.a_end - args.A);
  const long long off = dst - lds;
  CSK_DCHECK(off >= 0 && off + 512 <= lds_elems, SITE + 100, off, lds_elems);
#endif
  __builtin_amdgcn_global_load_lds((csk_gptr_t)src, (csk_lptr_t)dst, 16, 0, 0);
}

// Epilogue passes: tiles taller than 128 rows, and the 160-column tiles, stage
// their fp32 accumulators one wave-row band at a time (a 256x160 tile would need
// 168 KB of LDS at once; a 128x160 one 84 KB, more than its 74 KB 2-stage ring,
// which would cost it its second workgroup per CU)
template <int BM, int BN, int WM>
constexpr int epi_passes() {
  return (BM > 128 || BN == 160) ? WM : 1;
}

// epilogue LDS (bf16-element units): fp32 [BM / EP][BN + 4] band + [BM][2] row LN
// stats + [BM / EP / 16][BN][2] GroupNorm row-slice moments (gn_column_pass)
template <int BM, int BN, int EP = 1>
constexpr int epi_smem_elems() {
  return BM / EP * (BN + 4) * 2 + 4 * BM + (BM / EP / 16) * BN * 4;
}

#define BK 64

// zero page owned by gemm_glds.hip (allocated by csk_init): LDS-DMA padding
// source and the FAST staging paths' pointer target for invalid rows / taps
const bf16_t* csk_zero_ptr();
int csk_zero_bytes();

// element offset of 16-byte chunk `chunk` (0..7) of row `row` in a [rows][64] bf16
// tile; chunk XOR (row & 7) makes the ds_read_b128 fragment reads conflict-free.
__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

// Epilogue: accumulators -> fp32 LDS tile -> coalesced row pass applying bias,
// bias2d, activation / GEGLU gating and residual; or raw split-K partials.
// RAW: raw s_barrier + lgkmcnt(0) instead of __syncthreads (whose vmcnt(0) would
// drain LDS-DMA loads a persistent kernel keeps in flight across the epilogue)
template <bool RAW>
__device__ __forceinline__ void epi_barrier() {
  if constexpr (RAW) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  } else {
    __syncthreads();
  }
}

__device__ __forceinline__ void add8(float (&f)[8], const bf16_t* p, bool vec, int valid) {
  if (vec) {
    float g[8];
    unpack8(*reinterpret_cast<const uint4*>(p), g);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] += g[j];
  } else {
    for (int j = 0; j < 8 && j < valid; ++j) f[j] += bf2f(p[j]);
  }
}

__device__ __forceinline__ void act8(int act, float (&f)[8]) {
#define CSK_ACT8(CODE)                                     \
  case CODE:                                               \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) f[j] = apply_act(CODE, f[j]); \
    break;
  switch (act) {
    CSK_ACT8(ACT_GELU)
    CSK_ACT8(ACT_SILU)
    CSK_ACT8(ACT_QGELU)
    CSK_ACT8(ACT_LRELU)
    CSK_ACT8(ACT_LRELU_01)
    CSK_ACT8(ACT_RELU)
    CSK_ACT8(ACT_LRELU_001)
    case ACT_TANH:
    case ACT_ELU:
    case ACT_GELU_TANH: {
      Act8 x;
#pragma unroll
      for (int j = 0; j < 8; ++j) x.v[j] = f[j];
      x = act8_exotic(act, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = x.v[j];
      break;
    }
    default: break;
  }
#undef CSK_ACT8
}

// Fused-LayerNorm statistics (mean, rstd) of input row m0 + threadIdx.x
// (threads < BM), precomputed per row by ln_rowstats_kernel (gemm.hip) from
// the producer's column-slab partials.  Loaded BEFORE the K loop so the
// L2/HBM round trip overlaps the operand staging; one float2 in registers
// (merging the partials here raised every tile's VGPR peak and cost the
// small tiles a workgroup per CU; merging them in the epilogue serialised
// ln_nparts dependent loads per row and cost the UNet step 0.8 ms).
template <int BM>
__device__ __forceinline__ float2 ln_row_stats(const GemmArgs& args, int m0) {
  const int r = threadIdx.x;
  if (!args.ln_row || r >= BM) return make_float2(0.f, 0.f);
  return *reinterpret_cast<const float2*>(args.ln_row + (size_t)min(m0 + r, args.M - 1) * 2);
}

// Fused-LN row statistics merged INSIDE the consumer GEMM (no ln_rowstats
// launch in front of it): the 256 threads load the producer's column-slab
// partials of the tile's BM rows (NPH = 256 / BM threads per row, each merging
// every NPH-th slab, <= 8 in one round trip), combine them (Chan) through a
// [NPH][BM][3] + [BM][2] float scratch, and every lane keeps the (mean, rstd)
// of its MT epilogue rows in registers (threads < BM also their own row, for
// the LDS epilogue).  Called right after the prologue DMA issue with the LAST
// ring stage as scratch: the DMA first writes that stage after the main loop's
// first barrier, which every wave reaches only after its scratch reads retired
// (lgkmcnt(0) below).  Raw barriers: __syncthreads' vmcnt(0) would also wait for
// the ring prologue.
template <int BM, int MT, int WTM>
__device__ __forceinline__ void ln_merge_tile(const GemmArgs& args, int m0, int wm, float* scratch,
                                              float2 (&lane_rows)[MT], float2& own) {
  constexpr int NPH = 256 / BM, CAP = 8;
  const int t = threadIdx.x, r = t % BM, ph = t / BM;
  const int M = args.M, K = args.K, np = args.ln_nparts, pc = args.ln_pcols;
  const int m = min(m0 + r, M - 1);
  float n = 0.f, mean = 0.f, m2 = 0.f;
  float2 st[CAP];
#pragma unroll
  for (int j = 0; j < CAP; ++j) {
    const int p = ph + j * NPH;
    st[j] = p < np ? *reinterpret_cast<const float2*>(args.ln_part + ((size_t)p * M + m) * 2) : make_float2(0.f, 0.f);
  }
#pragma unroll
  for (int j = 0; j < CAP; ++j) {
    const int p = ph + j * NPH;
    if (p < np) chan_combine(n, mean, m2, (float)min(pc, K - p * pc), st[j].x, st[j].y);
  }
  for (int p = ph + CAP * NPH; p < np; p += NPH) {
    const float2 s2 = *reinterpret_cast<const float2*>(args.ln_part + ((size_t)p * M + m) * 2);
    chan_combine(n, mean, m2, (float)min(pc, K - p * pc), s2.x, s2.y);
  }
  float* part = scratch;              // [NPH][BM][3]
  float* rows = scratch + NPH * BM * 3;  // [BM][2] (mean, rstd)
  part[(ph * BM + r) * 3 + 0] = n;
  part[(ph * BM + r) * 3 + 1] = mean;
  part[(ph * BM + r) * 3 + 2] = m2;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (t < BM) {
    float nn = part[t * 3], mm = part[t * 3 + 1], qq = part[t * 3 + 2];
#pragma unroll
    for (int q = 1; q < NPH; ++q) chan_combine(nn, mm, qq, part[(q * BM + t) * 3], part[(q * BM + t) * 3 + 1],
                                                part[(q * BM + t) * 3 + 2]);
    rows[t * 2] = mm;
    rows[t * 2 + 1] = rsqrtf(qq / fmaxf(nn, 1.f) + args.ln_eps);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  own = t < BM ? make_float2(rows[t * 2], rows[t * 2 + 1]) : make_float2(0.f, 0.f);
  const int fr = t & 15;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int lr = wm * WTM + i * 16 + fr;
    lane_rows[i] = make_float2(rows[lr * 2], rows[lr * 2 + 1]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// The 8-column output vector a lane owns after the v_permlane16_swap of a pair of
// row-layout fragments (SW epilogues): fragments f and f+1 hold columns
// f*16 + fq*4 + r and (f+1)*16 + fq*4 + r of one row; after the swap an even-row
// lane (fq even) holds columns (f+1)*16 + fq*4 .. +7 and an odd-row lane
// f*16 + (fq-1)*4 .. +7, in register order [Y, X].  Returns that first column.
__device__ __forceinline__ int sw_pair(v4f& x, v4f& y, int f, int fq, float (&o)[8]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(y[r]), __float_as_uint(x[r]), false, false);
    o[r] = __uint_as_float(p[0]);
    o[4 + r] = __uint_as_float(p[1]);
  }
  return (fq & 1) ? f * 16 + (fq - 1) * 4 : (f + 1) * 16 + fq * 4;
}

// Attention epilogue of the cross-attention query projection (SURVEY K8 + K9;
// reference call site swarm/diffusion/diffusion_func.py:96): the 128x64 tile's
// accumulators are the queries of one head for 128 rows of one sample, in row
// layout — lane (row fr, head-dims 16 j + 4 g + r) — which is exactly the
// B-fragment layout of S^T = K Q^T (attn_tile.h), so each wave attends its own
// 32 rows over the head's K / V staged once per workgroup in LDS and stores
// O = softmax(q K^T) V: the [M, C] query tensor never reaches memory and the
// separate short-KV attention launch disappears.
template <int BM, int WM, int NTHR, bool RAW>
__device__ __forceinline__ void gemm_attn_epilogue(const GemmArgs& args, v4f (&acc)[BM / WM / 16][4], bf16_t* smem,
                                                   int m0, int n0, const float2 (&ln_lane)[BM / WM / 16],
                                                   bool ln_in) {
  constexpr int WTM = BM / WM, MT = WTM / 16, KVR = 96, KVI = KVR * 64;
  constexpr int CH = 2 * KVR * 8, CPT = (CH + NTHR - 1) / NTHR;  // 16-byte chunks of the two images
  const int tid = threadIdx.x, lane = tid & 63;
  const int wm = __builtin_amdgcn_readfirstlane(tid >> 6);  // WN == 1: the wave's row band
  const int fr = lane & 15, g = lane >> 4;
  const int M = args.M, H = args.N / 64, Skv = args.attn_skv;
  const int h = n0 / 64, b = m0 / args.rows_per_b;
  // K / V rows of (b, h), issued before the barrier that frees the main loop's LDS
  uint4 kvv[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int q = tid + i * NTHR;
    kvv[i] = make_uint4(0, 0, 0, 0);
    if (q < CH) {
      const int which = q / (KVR * 8), rem = q - which * (KVR * 8), row = rem >> 3, c = rem & 7;
      const int rr = min(row, Skv - 1);  // rows past Skv repeat the last key: finite, masked below
      const bf16_t* src = args.attn_kv + ((size_t)(b * Skv + rr) * 2 + which) * (H * 64) + h * 64 + c * 8;
      CSK_DCHECK(src + 8 <= args.attn_kv_end, 60, rr, Skv);
      kvv[i] = *reinterpret_cast<const uint4*>(src);
    }
  }
  // queries: the fused LayerNorm correction and bias, scaled by scale * log2(e)
  const bool lnf = args.ln_part != nullptr;
  v8s qf[MT][2];
  {
    float4 cs[4], bq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + 16 * j + 4 * g;
      cs[j] = lnf ? *reinterpret_cast<const float4*>(args.ln_colsum + col) : make_float4(0.f, 0.f, 0.f, 0.f);
      bq[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (args.bias) {
        const uint2 u = *reinterpret_cast<const uint2*>(args.bias + col);
        bq[j] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                            __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float mu = 0.f, rs = 1.f;
      if (lnf && ln_in) {
        mu = ln_lane[i].x;
        rs = ln_lane[i].y;
      } else if (lnf) {
        const float2 st = *reinterpret_cast<const float2*>(args.ln_row + (size_t)min(m0 + wm * WTM + i * 16 + fr, M - 1) * 2);
        mu = st.x;
        rs = st.y;
      }
      v4f qv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c4[4] = {cs[j].x, cs[j].y, cs[j].z, cs[j].w};
        const float b4[4] = {bq[j].x, bq[j].y, bq[j].z, bq[j].w};
#pragma unroll
        for (int r = 0; r < 4; ++r) qv[j][r] = __builtin_fmaf(rs, acc[i][j][r] - mu * c4[r], b4[r]);
      }
      qf[i][0] = at_pack8(qv[0], qv[1], args.attn_sl2);
      qf[i][1] = at_pack8(qv[2], qv[3], args.attn_sl2);
    }
  }
  bf16_t* ks = smem;
  bf16_t* vs = smem + KVI;
  epi_barrier<RAW>();  // the main loop's LDS reads are done
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    const int q = tid + i * NTHR;
    if (q < CH) {
      const int which = q / (KVR * 8), rem = q - which * (KVR * 8), row = rem >> 3, c = rem & 7;
      *reinterpret_cast<uint4*>((which ? vs : ks) + at_off64(row, c)) = kvv[i];
    }
  }
  epi_barrier<RAW>();
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    v4f o[4];
    float inv;
    at_attend_rowtile(ks, vs, qf[i], Skv, o, inv);
    const int m = m0 + wm * WTM + i * 16 + fr;
    if (m < M) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const uint2 w = make_uint2(pack2(o[dt][0] * inv, o[dt][1] * inv), pack2(o[dt][2] * inv, o[dt][3] * inv));
        *reinterpret_cast<uint2*>(args.C + (size_t)m * args.ldc + n0 + 16 * dt + 4 * g) = w;
      }
    }
  }
}

// SW: the accumulators are row-layout (the MFMA ran as B * A, C^T in registers):
// lane = output row i*16 + fr, registers = 4 consecutive output columns
// j*16 + fq*4 + r.  Lets the common short-K epilogue (bias / per-sample bias /
// activation incl. GEGLU / scale / residual) store 16-byte row vectors straight
// from registers — no fp32 LDS round trip, no barrier (the probe measured the
// LDS epilogue at about half of a K = 320 GEMM's time, tools/tilebench.py --probe).
// ln_lane / ln_in: per-lane (mean, rstd) of the MT epilogue rows merged in the
// kernel prologue (ln_merge_tile); a reference to a fixed-size array so the
// values stay in registers (a pointer that may be null made hipcc keep the
// array in scratch)
typedef unsigned int fx_u4 __attribute__((ext_vector_type(4)));

// In-kernel split-K fixup: true in the ONE workgroup of the tile that arrives
// last, with acc = sum of every split's partial in split order (deterministic
// whichever workgroup is last); false in the others, which are done.
// Fence-free hand-off (cdna_hip_programming.md Guideline 16 R1): partials stored write-through (sc1) and drained before the
// counter's atomic; the last arriver reads them all back sc1.  Each thread stores
// and reloads its own accumulator registers (16 B per lane per fragment: no
// layout math, fully coalesced).  The last arriver re-zeroes the counter for
// the next launch that uses it (gemm_glds.hip fixup_counters).
template <int MT, int NT, int NTHR>
__device__ __forceinline__ bool splitk_fixup(const GemmArgs& args, v4f (&acc)[MT][NT], int tile, int split,
                                             int* flag) {
  constexpr int SLOT = MT * NT * NTHR * 16;  // bytes per split partial
  const int tid = threadIdx.x, ns = args.fx_split;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(args.fx_ws + (size_t)tile * ns * (SLOT / 4)), 0, ns * SLOT, 0x00020000);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fx_u4, acc[i][j]), rs, ((i * NT + j) * NTHR + tid) * 16,
                                             split * SLOT, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned old = __hip_atomic_fetch_add(args.fx_cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(ns - 1);
    if (last) __hip_atomic_store(args.fx_cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __syncthreads();  // every wave has read the flag before the epilogue reuses its LDS word
  if (!last) return false;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only: the loads below are sc1)
  // every partial (this workgroup's own too) re-read in split order: a
  // deterministic sum with no second accumulator array live (the 128x160 and
  // 256-row tiles are at their register limit)
  // split 0 straight into acc (all fragments in flight), then the others in
  // groups of 4 fragments (16 temporaries), adding in split order
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
      acc[i][j] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, ((i * NT + j) * NTHR + tid) * 16, 0, 16));
  constexpr int NF = MT * NT, G = 4;
  for (int z = 1; z < ns; ++z) {
#pragma unroll
    for (int f0 = 0; f0 < NF; f0 += G) {
      v4f t[G];
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (f0 + g < NF)
          t[g] = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rs, ((f0 + g) * NTHR + tid) * 16, z * SLOT, 16));
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (f0 + g < NF) acc[(f0 + g) / NT][(f0 + g) % NT] += t[g];
    }
  }
  return true;
}

template <int BM, int BN, int WM, int WN, bool RAW = false, int EP = 1, int NTHR = 256, bool SW = false,
          bool ATTN = false>
__device__ __forceinline__ void gemm_epilogue_ln(const GemmArgs& args, v4f (&acc)[BM / WM / 16][BN / WN / 16],
                                                 bf16_t* smem, int m0, int n0, int split, float2 lnrow,
                                                 const float2 (&ln_lane)[BM / WM / 16], bool ln_in) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int LDC_S = BN + 4;
  // the 128x160 and 256-row tiles' main loops already hold 256 VGPRs: the
  // epilogue operand prefetch and the band store path below spilled there
  // (scratch 32-112 B per lane, tiles 26 / 33 / 31 slower: profiles/lib_ab_epilogue_prefetch_r6l.txt),
  // so those tiles keep the loads at their use and the generic store loop
  constexpr bool ROOMY = !((BM == 128 && BN == 160) || BM >= 256);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR address math
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int M = args.M, N = args.N;
  if (args.ws) {  // split-K: raw fp32 partials, epilogue applied by the reduce kernel
    float* wp = args.ws + (size_t)split * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (SW) {
          const int m = m0 + wm * WTM + i * 16 + fr, n = n0 + wn * WTN + j * 16 + fq * 4;
          if (m < M) {
            if (n + 3 < N && (N & 3) == 0) {
              *reinterpret_cast<float4*>(wp + (size_t)m * N + n) =
                  make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (n + r < N) wp[(size_t)m * N + n + r] = acc[i][j][r];
            }
          }
        } else {
          const int n = n0 + wn * WTN + j * 16 + fr;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
            if (m < M && n < N) wp[(size_t)m * N + n] = acc[i][j][r];
          }
        }
      }
    return;
  }
  if constexpr (ATTN && SW && BN == 64 && WN == 1) {  // a separate instance: the others keep their registers
    {
      gemm_attn_epilogue<BM, WM, NTHR, RAW>(args, acc, smem, m0, n0, ln_lane, ln_in);
      return;
    }
  }
  if constexpr (SW) {
    // ---- direct row-vector stores (no fp32 LDS staging) ----
    // Also covers the fused-LayerNorm consumer (ln_part: rstd * (acc - mean *
    // colsum) from the merged per-row statistics ln_row) and the row-statistics
    // producer (row_part: per-row (mean, M2) over this tile's BN columns, the
    // WN waves' sums combined through a few bytes of LDS).
    const bool geglu = args.act == ACT_GEGLU;
    constexpr bool geglu_ok = NT % 4 == 0;
    const bool lnf = args.ln_part != nullptr;
    const bool rst = args.row_part != nullptr;
    const bool gnp = args.gn_part != nullptr;
    const int gseg = args.gn_seg > 0 ? args.gn_seg : BM;
    const bool direct = (NT % 2 == 0 || args.sw_odd) && (!gnp || (!args.gn_lds && !geglu && !rst && gseg % WTM == 0 && BM % gseg == 0)) && (!lnf || args.ln_row || ln_in) &&
                        (!rst || !geglu) && (geglu_ok || !geglu) &&
                        (N % (geglu ? 16 : 8)) == 0 && (args.ldc % 8) == 0 && ((((size_t)args.C) & 15) == 0) &&
                        (!args.bias || ((((size_t)args.bias) & 15) == 0)) &&
                        (!args.bias2d || ((args.ldb2 % 8) == 0 && ((((size_t)args.bias2d) & 15) == 0))) &&
                        (!args.res || ((args.ldr % 8) == 0 && ((((size_t)args.res) & 15) == 0)));
    if (direct) {
      // Output-fragment pairs outer, row blocks inner: the bias of a pair is read
      // once into registers (reloading it per row block is forced otherwise, as
      // the C stores may alias it).
      const int outN = geglu ? N / 2 : N;
      const int ob = geglu ? (n0 + wn * WTN) / 2 : n0 + wn * WTN;  // this wave's first output column
      const float osc = args.out_scale;
      const int act = args.act;
      float lnm[MT], lnr[MT];  // fused LN: (mean, rstd) of each row block's row
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        lnm[i] = 0.f;
        lnr[i] = 1.f;
      }
      if (lnf && ln_in) {  // merged in the kernel prologue (ln_merge_tile)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          lnm[i] = ln_lane[i].x;
          lnr[i] = ln_lane[i].y;
        }
      } else if (lnf) {  // independent loads, issued together before the fragment loop
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const float2 st =
              *reinterpret_cast<const float2*>(args.ln_row + (size_t)min(m0 + wm * WTM + i * 16 + fr, M - 1) * 2);
          lnm[i] = st.x;
          lnr[i] = st.y;
        }
      }
      if (geglu) {
        if constexpr (NT % 4 == 0) {
#pragma unroll
          for (int f = 0; f < NT / 2; f += 2) {
            // packed columns: fragments 2f, 2f+1 = hidden, gate of output fragment f
            float bq[4][4], cq[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int nh = n0 + wn * WTN + (2 * f + q) * 16 + fq * 4;
              const bool in = nh < N;
#pragma unroll
              for (int r = 0; r < 4; ++r) cq[q][r] = (lnf && in) ? args.ln_colsum[nh + r] : 0.f;
              if (args.bias && in) {
                const uint2 u = *reinterpret_cast<const uint2*>(args.bias + nh);
                bq[q][0] = __uint_as_float(u.x << 16);
                bq[q][1] = __uint_as_float(u.x & 0xffff0000u);
                bq[q][2] = __uint_as_float(u.y << 16);
                bq[q][3] = __uint_as_float(u.y & 0xffff0000u);
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) bq[q][r] = 0.f;
              }
            }
#pragma unroll
            for (int i = 0; i < MT; ++i) {
              const int m = m0 + wm * WTM + i * 16 + fr;
              v4f x, y;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float h0 = lnr[i] * (acc[i][2 * f][r] - lnm[i] * cq[0][r]) + bq[0][r];
                const float g0 = lnr[i] * (acc[i][2 * f + 1][r] - lnm[i] * cq[1][r]) + bq[1][r];
                const float h1 = lnr[i] * (acc[i][2 * f + 2][r] - lnm[i] * cq[2][r]) + bq[2][r];
                const float g1 = lnr[i] * (acc[i][2 * f + 3][r] - lnm[i] * cq[3][r]) + bq[3][r];
                x[r] = h0 * gelu_geglu(g0);
                y[r] = h1 * gelu_geglu(g1);
              }
              float o[8];
              const int col = ob + sw_pair(x, y, f, fq, o);
              if (m >= M || col >= outN) continue;
              if (osc != 1.0f) {
#pragma unroll
                for (int r = 0; r < 8; ++r) o[r] *= osc;
              }
              if (args.res) add8(o, args.res + (size_t)m * args.ldr + col, true, 8);
              *reinterpret_cast<uint4*>(args.C + (size_t)m * args.ldc + col) = pack8(o);
            }
          }
        }
      } else {
        float rs[MT], rq[MT];  // row statistics: sum, sum of squares over this lane's columns
#pragma unroll
        for (int i = 0; i < MT; ++i) rs[i] = rq[i] = 0.f;
        // GroupNorm statistics of the output: per column, (sum, sum^2) over the
        // wave's WTM rows -> LDS [WM][BN][2] -> (mean, M2) per gn_seg-row segment
        float* gred = reinterpret_cast<float*>(smem);
        if (gnp) epi_barrier<RAW>();  // main-loop LDS reads are done
        // The epilogue operands of a fragment pair (bias, LN colsum, the residual
        // rows of every row block, the per-sample bias row) are issued together
        // before the pair's first store: C may alias them, so the compiler will
        // not move a load over a store, and loaded at their use every residual
        // row cost one exposed memory latency (global_load; s_waitcnt vmcnt(0);
        // global_store, per row block).  Now one latency per pair.
        const bool b2u = args.bias2d && (args.rows_per_b % BM) == 0 && (m0 % args.rows_per_b) + BM <= args.rows_per_b;
#pragma unroll
        for (int f = 0; f + 1 < NT; f += 2) {
          // the 8 columns this lane stores for fragment pair f (same for every row block)
          const int col = ob + ((fq & 1) ? f * 16 + (fq - 1) * 4 : (f + 1) * 16 + fq * 4);
          float bb[8], cs[8], gs[8], gq[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) bb[r] = cs[r] = gs[r] = gq[r] = 0.f;
          uint4 rpre[MT];
          uint4 b2pre = make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int m = m0 + wm * WTM + i * 16 + fr;
            rpre[i] = make_uint4(0, 0, 0, 0);
            if (ROOMY && args.res && col < outN && m < M) {
              const uint4* rp = reinterpret_cast<const uint4*>(args.res + (size_t)m * args.ldr + col);
              if (args.epi_nt >= 2) {
                const fx_u4 v = __builtin_nontemporal_load(reinterpret_cast<const fx_u4*>(rp));
                rpre[i] = make_uint4(v[0], v[1], v[2], v[3]);
              } else {
                rpre[i] = *rp;
              }
            }
          }
          if (b2u && col < outN) b2pre = *reinterpret_cast<const uint4*>(args.bias2d + (size_t)(m0 / args.rows_per_b) * args.ldb2 + col);
          if (col < outN) {
            if (args.bias) add8(bb, args.bias + col, true, 8);
            if (lnf) {
              const float4 c0 = *reinterpret_cast<const float4*>(args.ln_colsum + col);
              const float4 c1 = *reinterpret_cast<const float4*>(args.ln_colsum + col + 4);
              cs[0] = c0.x; cs[1] = c0.y; cs[2] = c0.z; cs[3] = c0.w;
              cs[4] = c1.x; cs[5] = c1.y; cs[6] = c1.z; cs[7] = c1.w;
            }
          }
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int m = m0 + wm * WTM + i * 16 + fr;
            float o[8];
            sw_pair(acc[i][f], acc[i][f + 1], f, fq, o);
            if (m >= M || col >= outN) continue;
#pragma unroll
            for (int r = 0; r < 8; ++r) o[r] = lnr[i] * (o[r] - lnm[i] * cs[r]) + bb[r];
            if (b2u) {
              float g[8];
              unpack8(b2pre, g);
#pragma unroll
              for (int r = 0; r < 8; ++r) o[r] += g[r];
            } else if (args.bias2d) {
              add8(o, args.bias2d + (size_t)(m / args.rows_per_b) * args.ldb2 + col, true, 8);
            }
            act8(act, o);
            if (osc != 1.0f) {
#pragma unroll
              for (int r = 0; r < 8; ++r) o[r] *= osc;
            }
            if (args.res) {
              if constexpr (ROOMY) {
                float g[8];
                unpack8(rpre[i], g);
#pragma unroll
                for (int r = 0; r < 8; ++r) o[r] += g[r];
              } else {
                add8(o, args.res + (size_t)m * args.ldr + col, true, 8);
              }
            }
            if (rst) {
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                rs[i] += o[r];
                rq[i] = __builtin_fmaf(o[r], o[r], rq[i]);
              }
            }
            if (gnp) {
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                gs[r] += o[r];
                gq[r] = __builtin_fmaf(o[r], o[r], gq[r]);
              }
            }
            if (args.epi_nt) {
              const uint4 pv = pack8(o);
              __builtin_nontemporal_store(fx_u4{pv.x, pv.y, pv.z, pv.w},
                                          reinterpret_cast<fx_u4*>(args.C + (size_t)m * args.ldc + col));
            } else {
              *reinterpret_cast<uint4*>(args.C + (size_t)m * args.ldc + col) = pack8(o);
            }
          }
          if (gnp) {
            // the 16 lanes of a 16-row group (fr) hold the same 8 columns
#pragma unroll
            for (int r = 0; r < 8; ++r) {
#pragma unroll
              for (int x = 1; x < 16; x <<= 1) {
                gs[r] += __shfl_xor(gs[r], x);
                gq[r] += __shfl_xor(gq[r], x);
              }
            }
            if (fr == 0 && col < outN) {
              const int c = col - n0;
#pragma unroll
              for (int r = 0; r < 8; ++r) {
                gred[(wm * BN + c + r) * 2] = gs[r];
                gred[(wm * BN + c + r) * 2 + 1] = gq[r];
              }
            }
          }
        }
        if constexpr (NT % 2 == 1) {
          // odd fragment count (80 columns per wave: the 160-wide tiles): the last
          // fragment unpaired, 4 consecutive columns per lane, 8-byte stores
          constexpr int f = NT - 1;
          const int col = ob + f * 16 + fq * 4;
          float bb[4], cs[4], gs[4], gq[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) bb[r] = cs[r] = gs[r] = gq[r] = 0.f;
          if (col < outN) {
            if (args.bias) {
              const uint2 u = *reinterpret_cast<const uint2*>(args.bias + col);
              bb[0] = __uint_as_float(u.x << 16); bb[1] = __uint_as_float(u.x & 0xffff0000u);
              bb[2] = __uint_as_float(u.y << 16); bb[3] = __uint_as_float(u.y & 0xffff0000u);
            }
            if (lnf) {
              const float4 c0 = *reinterpret_cast<const float4*>(args.ln_colsum + col);
              cs[0] = c0.x; cs[1] = c0.y; cs[2] = c0.z; cs[3] = c0.w;
            }
          }
          uint2 r4[MT], b4[MT];  // residual / per-sample bias rows, issued before the stores (see above)
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int m = m0 + wm * WTM + i * 16 + fr;
            r4[i] = b4[i] = make_uint2(0, 0);
            if (ROOMY && m < M && col < outN) {
              if (args.res) r4[i] = *reinterpret_cast<const uint2*>(args.res + (size_t)m * args.ldr + col);
              if (args.bias2d)
                b4[i] = *reinterpret_cast<const uint2*>(args.bias2d + (size_t)(m / args.rows_per_b) * args.ldb2 + col);
            }
          }
          auto add4u = [](float (&o)[4], uint2 u) {
            o[0] += __uint_as_float(u.x << 16); o[1] += __uint_as_float(u.x & 0xffff0000u);
            o[2] += __uint_as_float(u.y << 16); o[3] += __uint_as_float(u.y & 0xffff0000u);
          };
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            const int m = m0 + wm * WTM + i * 16 + fr;
            if (m >= M || col >= outN) continue;
            float o[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = lnr[i] * (acc[i][f][r] - lnm[i] * cs[r]) + bb[r];
            if (args.bias2d) {
              if constexpr (!ROOMY)
                b4[i] = *reinterpret_cast<const uint2*>(args.bias2d + (size_t)(m / args.rows_per_b) * args.ldb2 + col);
              add4u(o, b4[i]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = apply_act(act, o[r]);
            if (osc != 1.0f) {
#pragma unroll
              for (int r = 0; r < 4; ++r) o[r] *= osc;
            }
            if (args.res) {
              if constexpr (!ROOMY) r4[i] = *reinterpret_cast<const uint2*>(args.res + (size_t)m * args.ldr + col);
              add4u(o, r4[i]);
            }
            if (rst) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                rs[i] += o[r];
                rq[i] = __builtin_fmaf(o[r], o[r], rq[i]);
              }
            }
            if (gnp) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                gs[r] += o[r];
                gq[r] = __builtin_fmaf(o[r], o[r], gq[r]);
              }
            }
            const unsigned lo = (unsigned)f2bf(o[0]) | ((unsigned)f2bf(o[1]) << 16);
            const unsigned hi = (unsigned)f2bf(o[2]) | ((unsigned)f2bf(o[3]) << 16);
            *reinterpret_cast<uint2*>(args.C + (size_t)m * args.ldc + col) = make_uint2(lo, hi);
          }
          if (gnp) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
              for (int x = 1; x < 16; x <<= 1) {
                gs[r] += __shfl_xor(gs[r], x);
                gq[r] += __shfl_xor(gq[r], x);
              }
            }
            if (fr == 0 && col < outN) {
              const int c = col - n0;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                gred[(wm * BN + c + r) * 2] = gs[r];
                gred[(wm * BN + c + r) * 2 + 1] = gq[r];
              }
            }
          }
        }
        if (gnp) {
          epi_barrier<RAW>();
          const int nseg = BM / gseg, wps = gseg / WTM;  // segments per tile, waves per segment
          for (int t = tid; t < BN * nseg; t += NTHR) {
            const int c = t % BN, sq = t / BN;
            if (n0 + c >= N) continue;
            float sv = 0.f, qv = 0.f;
            for (int w = sq * wps; w < (sq + 1) * wps; ++w) {
              sv += gred[(w * BN + c) * 2];
              qv += gred[(w * BN + c) * 2 + 1];
            }
            const float mean = sv / (float)gseg;
            *reinterpret_cast<float2*>(args.gn_part + ((size_t)((m0 + sq * gseg) / gseg) * N + n0 + c) * 2) =
                make_float2(mean, fmaxf(qv - sv * mean, 0.f));
          }
          epi_barrier<RAW>();  // persistent kernels reuse this LDS for the next tile
        }
        if (rst) {
          // the 4 lanes of a row (fq) -> the wave's WTN columns -> the WN waves (LDS)
          float* red = reinterpret_cast<float*>(smem);  // [WN][BM][2]
          epi_barrier<RAW>();                            // main-loop LDS reads are done
#pragma unroll
          for (int i = 0; i < MT; ++i) {
            float sv = rs[i], qv = rq[i];
            sv += __shfl_xor(sv, 16);
            qv += __shfl_xor(qv, 16);
            sv += __shfl_xor(sv, 32);
            qv += __shfl_xor(qv, 32);
            if (fq == 0) {
              const int row = wm * WTM + i * 16 + fr;
              red[(wn * BM + row) * 2] = sv;
              red[(wn * BM + row) * 2 + 1] = qv;
            }
          }
          epi_barrier<RAW>();
          const int ncols = min(BN, N - n0);
          for (int row = tid; row < BM; row += NTHR) {
            const int m = m0 + row;
            if (m >= M) continue;
            float sv = 0.f, qv = 0.f;
#pragma unroll
            for (int w = 0; w < WN; ++w) {
              sv += red[(w * BM + row) * 2];
              qv += red[(w * BM + row) * 2 + 1];
            }
            const float mean = sv / (float)ncols;
            *reinterpret_cast<float2*>(args.row_part + ((size_t)(n0 / BN) * M + m) * 2) =
                make_float2(mean, fmaxf(qv - sv * mean, 0.f));
          }
          epi_barrier<RAW>();  // persistent kernels reuse this LDS for the next tile
        }
      }
      return;
    }
  }
  static_assert(WM % EP == 0, "epilogue passes split the wave rows");
  constexpr int PR = BM / EP;                  // tile rows staged per pass
  float* cs = reinterpret_cast<float*>(smem);  // [PR][LDC_S]
  float* lnst = cs + PR * LDC_S;               // [BM][2]: (mean, rstd) of the input rows (fused LN)
  const int act = args.act;
  const bool ln = args.ln_part != nullptr;
  if (ln) {
    if (tid < BM) *reinterpret_cast<float2*>(lnst + 2 * tid) = lnrow;
    epi_barrier<RAW>();
  }
  // this lane's column sums of the folded weight, loaded once (fused LN; the
  // row layout loads them per fragment below)
  float lncs[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) lncs[j] = (ln && !SW) ? args.ln_colsum[min(n0 + wn * WTN + j * 16 + fr, N - 1)] : 0.f;
  // acc -> LayerNorm-corrected value (identity without a fused LN)
  auto lnfix = [&](float v, int row, int j) {
    if (!ln) return v;
    return lnst[2 * row + 1] * (v - lnst[2 * row] * lncs[j]);
  };
  for (int pass = 0; pass < EP; ++pass) {
  const int pr0 = pass * PR;  // first tile row of this pass
  if (pass) epi_barrier<RAW>();  // the previous band's readers are done with cs
  const bool mine = EP == 1 || (wm * WTM) / PR == pass;
  if (!mine) {
  } else if (SW && act == ACT_GEGLU) {
    // row layout: fragment columns outer so each lane's 8 folded-weight column
    // sums (fused LN) are loaded once per fragment pair and die with it
#pragma unroll
    for (int j = 0; j < NT; j += 2) {
      const int ch = wn * WTN + j * 16 + fq * 4;  // packed hidden column (tile-relative)
      const int oc = (wn * WTN + j * 16) / 2 + fq * 4;
      float bh[4], bg[4], ch_s[4], cg_s[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int nh = n0 + ch + r;
        bh[r] = (args.bias && nh < N) ? bf2f(args.bias[nh]) : 0.f;
        bg[r] = (args.bias && nh + 16 < N) ? bf2f(args.bias[nh + 16]) : 0.f;
        ch_s[r] = ln ? args.ln_colsum[min(nh, N - 1)] : 0.f;
        cg_s[r] = ln ? args.ln_colsum[min(nh + 16, N - 1)] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int row = wm * WTM + i * 16 + fr;
        const float mu = ln ? lnst[2 * row] : 0.f, rs = ln ? lnst[2 * row + 1] : 1.f;
        float g[4];
#pragma unroll
        for (int r = 0; r < 4; ++r)
          g[r] = (rs * (acc[i][j][r] - mu * ch_s[r]) + bh[r]) * gelu_geglu(rs * (acc[i][j + 1][r] - mu * cg_s[r]) + bg[r]);
        *reinterpret_cast<float4*>(cs + (row - pr0) * LDC_S + oc) = make_float4(g[0], g[1], g[2], g[3]);
      }
    }
  } else if (SW) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = wn * WTN + j * 16 + fq * 4;
      float c_s[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) c_s[r] = ln ? args.ln_colsum[min(n0 + col + r, N - 1)] : 0.f;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int row = wm * WTM + i * 16 + fr;
        const float mu = ln ? lnst[2 * row] : 0.f, rs = ln ? lnst[2 * row + 1] : 1.f;
        *reinterpret_cast<float4*>(cs + (row - pr0) * LDC_S + col) =
            make_float4(rs * (acc[i][j][0] - mu * c_s[0]), rs * (acc[i][j][1] - mu * c_s[1]),
                        rs * (acc[i][j][2] - mu * c_s[2]), rs * (acc[i][j][3] - mu * c_s[3]));
      }
    }
  } else if (act == ACT_GEGLU) {
    // packed columns: even 16-tiles = hidden, odd = gate (same output column in the same lane)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; j += 2) {
        const int nh = n0 + wn * WTN + j * 16 + fr;
        const float bh = (args.bias && nh < N) ? bf2f(args.bias[nh]) : 0.f;
        const float bg = (args.bias && nh + 16 < N) ? bf2f(args.bias[nh + 16]) : 0.f;
        const int oc = (wn * WTN + j * 16) / 2 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fq * 4 + r;
          cs[(row - pr0) * LDC_S + oc] =
              (lnfix(acc[i][j][r], row, j) + bh) * gelu_geglu(lnfix(acc[i][j + 1][r], row, j + 1) + bg);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fq * 4 + r, col = wn * WTN + j * 16 + fr;
          cs[(row - pr0) * LDC_S + col] = lnfix(acc[i][j][r], row, j);
        }
  }
  epi_barrier<RAW>();
  // Band store path with compile-time geometry: VPR = BN / 8 column vectors per
  // row, NTHR / VPR rows per iteration (the threads past that idle when VPR does
  // not divide NTHR: the 160-wide tiles), so no runtime division per 8 outputs;
  // each thread keeps ONE column vector, its bias (+ a band-uniform per-sample
  // bias row) loaded once, and the residual rows of all its iterations are
  // issued before the first store (C may alias them, so loaded at the use every
  // row waited one memory latency).  Covers the GroupNorm statistics (final
  // values back into LDS for the column pass below) and the fused-LN consumer
  // (applied while staging).  At K = 320 the epilogue is most of a tile's
  // instruction stream (the SIMDs were issue-saturated, PMC r1i).
  bool banded = false;
  {
    constexpr int VPR = BN / 8, RPI = NTHR / VPR, NIT = (PR + RPI - 1) / RPI;
    const int mb0 = m0 + pr0, mb1 = min(mb0 + PR, M) - 1;
    const bool b2 = args.bias2d != nullptr;
    banded = ROOMY && args.epi_band && !args.row_part && act != ACT_GEGLU && act != ACT_PROBE_NO_STORE && (N % 8) == 0 &&
             (args.ldc % 8) == 0 && ((((size_t)args.C) & 15) == 0) &&
             (!args.bias || ((((size_t)args.bias) & 15) == 0)) &&
             (!args.res || ((args.ldr % 8) == 0 && ((((size_t)args.res) & 15) == 0))) &&
             (!b2 || ((args.ldb2 % 8) == 0 && ((((size_t)args.bias2d) & 15) == 0) &&
                      mb0 / args.rows_per_b == mb1 / args.rows_per_b));
    if (banded) {
      const int cv = tid % VPR, r0 = tid / VPR;
      const int n = n0 + cv * 8;
      if (r0 < RPI && n < N) {
        float bb[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = 0.f;
        const float osc = args.out_scale;
        auto ld_res = [&](int k) {
          const int row = r0 + k * RPI, m = mb0 + row;
          uint4 u = make_uint4(0, 0, 0, 0);
          // uniform base + 32-bit element offset (saddr + voffset: no 64-bit
          // per-thread pointers kept live, which spilled the 256-VGPR tiles)
          if (args.res && row < PR && m < M) u = *reinterpret_cast<const uint4*>(args.res + (unsigned)(m * args.ldr + n));
          return u;
        };
        auto store_row = [&](int k, uint4 rres) {
          const int row = r0 + k * RPI, m = mb0 + row;
          const float4 lo = *reinterpret_cast<const float4*>(cs + row * LDC_S + cv * 8);
          const float4 hi = *reinterpret_cast<const float4*>(cs + row * LDC_S + cv * 8 + 4);
          float f[8] = {lo.x + bb[0], lo.y + bb[1], lo.z + bb[2], lo.w + bb[3],
                        hi.x + bb[4], hi.y + bb[5], hi.z + bb[6], hi.w + bb[7]};
          act8(act, f);
          if (osc != 1.0f) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] *= osc;
          }
          if (args.res) {
            float rf[8];
            unpack8(rres, rf);
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += rf[j];
          }
          *reinterpret_cast<uint4*>(args.C + (unsigned)(m * args.ldc + n)) = pack8(f);
          if (args.gn_part) {
            float* crow = cs + row * LDC_S + cv * 8;
            *reinterpret_cast<float4*>(crow) = make_float4(f[0], f[1], f[2], f[3]);
            *reinterpret_cast<float4*>(crow + 4) = make_float4(f[4], f[5], f[6], f[7]);
          }
        };
        uint4 rv[NIT];
#pragma unroll
        for (int k = 0; k < NIT; ++k) rv[k] = ld_res(k);
        if (args.bias) add8(bb, args.bias + n, true, 8);
        if (b2) add8(bb, args.bias2d + (size_t)(mb0 / args.rows_per_b) * args.ldb2 + n, true, 8);
#pragma unroll
        for (int k = 0; k < NIT; ++k) {
          if (r0 + k * RPI >= PR || mb0 + r0 + k * RPI >= M) break;
          store_row(k, rv[k]);
        }
      }
      if (!args.gn_part) continue;  // next band: nothing else to do without GN statistics
    }
  }
  const int outN = act == ACT_GEGLU ? N / 2 : N;
  const int BNo = act == ACT_GEGLU ? BN / 2 : BN;
  const int on0 = act == ACT_GEGLU ? n0 / 2 : n0;
  const int vpr = BNo / 8;
  // PR * vpr is a multiple of NTHR for every tile, so each wave runs the same
  // number of iterations and the row-statistics shuffles below see all lanes
  for (int v = banded ? PR * vpr : tid; v < PR * vpr; v += NTHR) {
    const int row = v / vpr, cv = v - row * vpr;  // row within the band
    const int m = m0 + pr0 + row, n = on0 + cv * 8;
    const bool live = m < M && n < outN;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.f;
    if (live) {
      const float4 lo = *reinterpret_cast<const float4*>(cs + row * LDC_S + cv * 8);
      const float4 hi = *reinterpret_cast<const float4*>(cs + row * LDC_S + cv * 8 + 4);
      f[0] = lo.x; f[1] = lo.y; f[2] = lo.z; f[3] = lo.w; f[4] = hi.x; f[5] = hi.y; f[6] = hi.z; f[7] = hi.w;
      const bool full = n + 8 <= outN;
      if (act != ACT_GEGLU) {
        // bias / bias2d: one 16-byte load for a full, aligned group of 8 columns
        // (per-element guarded loads otherwise) — keeps the epilogue branch-free
        // in the common case, which matters for short-K GEMMs (K = 320)
        if (args.bias) add8(f, args.bias + n, full && (N % 8 == 0), outN - n);
        if (args.bias2d) add8(f, args.bias2d + (size_t)(m / args.rows_per_b) * args.ldb2 + n,
                                   full && (N % 8 == 0) && (args.ldb2 % 8 == 0), outN - n);
        act8(act, f);  // one uniform switch per 8 values, not per value
      }
      if (args.out_scale != 1.0f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] *= args.out_scale;
      }
      bf16_t* cp = args.C + (size_t)m * args.ldc + n;
      float* crow = cs + row * LDC_S + cv * 8;  // final values back into LDS for the GN statistics
      if (full && ((((size_t)cp) & 15) == 0)) {
        if (args.res) {
          float rf[8];
          unpack8(*reinterpret_cast<const uint4*>(args.res + (size_t)m * args.ldr + n), rf);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] += rf[j];
        }
        if (args.act != ACT_PROBE_NO_STORE) *reinterpret_cast<uint4*>(cp) = pack8(f);
        if (args.gn_part) {
          *reinterpret_cast<float4*>(crow) = make_float4(f[0], f[1], f[2], f[3]);
          *reinterpret_cast<float4*>(crow + 4) = make_float4(f[4], f[5], f[6], f[7]);
        }
      } else {
        for (int j = 0; j < 8 && n + j < outN; ++j) {
          float o = f[j];
          if (args.res) o += bf2f(args.res[(size_t)m * args.ldr + n + j]);
          cp[j] = f2bf(o);
          crow[j] = o;
          f[j] = o;
        }
      }
    }
    if (args.row_part) {
      // (mean, M2) of this output row over the tile's columns for a consumer
      // GEMM's fused LayerNorm: the row's vpr chunks sit in vpr consecutive
      // lanes, so two xor-butterflies (sum, then squared deviations) finish it
      // in registers
      const int nv = live ? min(8, outN - n) : 0;
      float sm = 0.f, cnt = (float)nv;
#pragma unroll
      for (int j = 0; j < 8; ++j) sm += j < nv ? f[j] : 0.f;
      for (int o = 1; o < vpr; o <<= 1) {
        sm += __shfl_xor(sm, o, 64);
        cnt += __shfl_xor(cnt, o, 64);
      }
      const float mean = cnt > 0.f ? sm / cnt : 0.f;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = j < nv ? f[j] - mean : 0.f;
        q += d * d;
      }
      for (int o = 1; o < vpr; o <<= 1) q += __shfl_xor(q, o, 64);
      if (cv == 0 && m < M)
        *reinterpret_cast<float2*>(args.row_part + ((size_t)(n0 / BN) * M + m) * 2) = make_float2(mean, q);
    }
  }
  if (args.gn_part) {
    // column pass: (mean, M2) of each output channel over row segments of
    // gn_seg rows (a divisor of BM chosen by the host, _gn_seg).  Each segment
    // is cut into slices of <= 16 rows: thread = (segment, slice, channel), with
    // consecutive channels in consecutive lanes (conflict-free LDS reads), loads
    // its slice into registers at once (16 independent LDS reads in flight, not
    // 2 x seg dependent ones: that chain was 3-10 us per conv) and takes the
    // two-pass moments in registers (exact, no E[x^2]-E[x]^2 cancellation); the
    // slices are then Chan-merged.  The consumer GroupNorm merges the segments.
    const int seg = args.gn_seg > 0 ? args.gn_seg : PR;
    const int qrows = seg < 16 ? seg : 16, qs = seg / qrows, nsq = PR / seg;
    float* qpart = lnst + 2 * BM;  // [nsq * qs][BN][2]
    epi_barrier<RAW>();
    for (int t = tid; t < BN * nsq * qs; t += NTHR) {
      const int c = t % BN, sl = t / BN;  // slice sl = sq * qs + qq
      const int r0 = sl * qrows;
      float v[16], sm = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        v[r] = r < qrows ? cs[(r0 + r) * LDC_S + c] : 0.f;
        sm += v[r];
      }
      const float mean = sm / (float)qrows;
      float m2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = r < qrows ? v[r] - mean : 0.f;
        m2 = __builtin_fmaf(d, d, m2);
      }
      *reinterpret_cast<float2*>(qpart + ((size_t)sl * BN + c) * 2) = make_float2(mean, m2);
    }
    epi_barrier<RAW>();
    for (int t = tid; t < BN * nsq; t += NTHR) {
      const int c = t % BN, sq = t / BN;
      const int n = n0 + c, r0 = sq * seg;
      if (n >= N || m0 + pr0 + r0 >= M) continue;
      float cnt = 0.f, mean = 0.f, m2 = 0.f;
      for (int qq = 0; qq < qs; ++qq) {
        const float2 p = *reinterpret_cast<const float2*>(qpart + ((size_t)(sq * qs + qq) * BN + c) * 2);
        chan_combine(cnt, mean, m2, (float)qrows, p.x, p.y);
      }
      *reinterpret_cast<float2*>(args.gn_part + ((size_t)((m0 + pr0 + r0) / seg) * N + n) * 2) =
          make_float2(mean, m2);
    }
  }
  }  // passes
}

template <int BM, int BN, int WM, int WN, bool RAW = false, int EP = 1, int NTHR = 256, bool SW = false>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& args, v4f (&acc)[BM / WM / 16][BN / WN / 16],
                                              bf16_t* smem, int m0, int n0, int split,
                                              float2 lnrow = make_float2(0.f, 0.f)) {
  float2 none[BM / WM / 16];
#pragma unroll
  for (int i = 0; i < BM / WM / 16; ++i) none[i] = make_float2(0.f, 1.f);
  gemm_epilogue_ln<BM, BN, WM, WN, RAW, EP, NTHR, SW>(args, acc, smem, m0, n0, split, lnrow, none, false);
}

// GN statistics granularity: 1 = fine segments (BM*BN/256 rows, every thread of
// the column pass busy), 0 = one segment per BM-row tile.  The host mirrors it
// (hip_ops._gn_seg).
extern int g_gn_fine;
// rows per GroupNorm-statistics segment written by the split-K reduce
// (splitk_reduce8_gn_kernel); the host requires it to divide the rows per sample
constexpr int SPLITK_GN_SEG = 64;
template <int BM, int BN, int WM>
__host__ __forceinline__ int gn_seg_for() {
  constexpr int PR = BM / epi_passes<BM, BN, WM>();  // the epilogue's row band
  const int seg = g_gn_fine ? BM * BN / 256 : BM;
  return seg > PR ? PR : seg;
}

int csk_gemm_glds_launch(const GemmArgs& a, int tile, int ksplit, bool conv, hipStream_t s);
int csk_gemm8p_launch(const GemmArgs& a, int tile, int ksplit, bool conv, hipStream_t s);
