// Shared pieces of the MFMA GEMM / implicit-GEMM conv kernels (gemm.hip:
// register-staged pipeline; gemm_glds.hip: LDS-DMA multi-stage pipeline).
#pragma once
#include "common.h"

enum {
  ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_GEGLU = 3, ACT_QGELU = 4,
  ACT_LRELU = 5,       // leaky relu 0.2 (ESRGAN)
  ACT_LRELU_01 = 6,    // leaky relu 0.1 (HiFi-GAN)
  ACT_TANH = 7,
  ACT_RELU = 8,
  ACT_LRELU_001 = 9,   // leaky relu 0.01 (torch default)
  ACT_ELU = 10,        // EnCodec
  ACT_GELU_TANH = 11,  // T5 "gelu_new"
};

// pointwise epilogue activation (every act except GEGLU, which pairs columns)
__device__ __forceinline__ float apply_act(int act, float v) {
  switch (act) {
    case ACT_GELU: return gelu_f(v);
    case ACT_SILU: return silu_f(v);
    case ACT_QGELU: return qgelu_f(v);
    case ACT_LRELU: return v > 0.f ? v : 0.2f * v;
    case ACT_LRELU_01: return v > 0.f ? v : 0.1f * v;
    case ACT_TANH: return tanhf(v);
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_LRELU_001: return v > 0.f ? v : 0.01f * v;
    case ACT_ELU: return v > 0.f ? v : expm1f(v);
    case ACT_GELU_TANH: return 0.5f * v * (1.f + tanhf(0.7978845608028654f * (v + 0.044715f * v * v * v)));
    default: return v;
  }
}

struct GemmArgs {
  const bf16_t* A;  // GEMM: [M][lda];  CONV: NHWC input [B][H][W][Cin]
  const bf16_t* W;  // [N][ldb] (K-contiguous rows)
  bf16_t* C;        // [M][ldc]
  const bf16_t* bias;    // [N] or null
  const bf16_t* bias2d;  // [B][N] or null (row m uses b = m / rows_per_b)
  const bf16_t* res;     // [M][ldc] or null
  const bf16_t* zero;    // >= 16 zero bytes in global memory (LDS-DMA source for padding)
  int M, N, K, lda, ldb, ldc, rows_per_b, act;  // CONV: lda = input pixel stride (>= Cin)
  int ldr;          // residual row stride
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
};

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
    CSK_ACT8(ACT_TANH)
    CSK_ACT8(ACT_RELU)
    CSK_ACT8(ACT_LRELU_001)
    CSK_ACT8(ACT_ELU)
    CSK_ACT8(ACT_GELU_TANH)
    default: break;
  }
#undef CSK_ACT8
}

template <int BM, int BN, int WM, int WN, bool RAW = false>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs& args, v4f (&acc)[BM / WM / 16][BN / WN / 16],
                                              bf16_t* smem, int m0, int n0, int split) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int LDC_S = BN + 4;
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
        const int n = n0 + wn * WTN + j * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + i * 16 + fq * 4 + r;
          if (m < M && n < N) wp[(size_t)m * N + n] = acc[i][j][r];
        }
      }
    return;
  }
  float* cs = reinterpret_cast<float*>(smem);  // [BM][LDC_S]
  const int act = args.act;
  if (act == ACT_GEGLU) {
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
          cs[row * LDC_S + oc] = (acc[i][j][r] + bh) * gelu_f(acc[i][j + 1][r] + bg);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(wm * WTM + i * 16 + fq * 4 + r) * LDC_S + wn * WTN + j * 16 + fr] = acc[i][j][r];
  }
  epi_barrier<RAW>();
  const int outN = act == ACT_GEGLU ? N / 2 : N;
  const int BNo = act == ACT_GEGLU ? BN / 2 : BN;
  const int on0 = act == ACT_GEGLU ? n0 / 2 : n0;
  const int vpr = BNo / 8;
  for (int v = tid; v < BM * vpr; v += 256) {
    const int row = v / vpr, cv = v - row * vpr;
    const int m = m0 + row, n = on0 + cv * 8;
    if (m >= M || n >= outN) continue;
    float f[8];
    const float4 lo = *reinterpret_cast<const float4*>(cs + row * LDC_S + cv * 8);
    const float4 hi = *reinterpret_cast<const float4*>(cs + row * LDC_S + cv * 8 + 4);
    f[0] = lo.x; f[1] = lo.y; f[2] = lo.z; f[3] = lo.w; f[4] = hi.x; f[5] = hi.y; f[6] = hi.z; f[7] = hi.w;
    const bool full = n + 8 <= outN;
    if (act != ACT_GEGLU) {
      // bias / bias2d: one 16-byte load for a full, aligned group of 8 columns
      // (per-element guarded loads otherwise) — keeps the epilogue branch-free
      // in the common case, which matters for short-K GEMMs (K = 320)
      if (args.bias) add8(f, args.bias + n, full && (N % 8 == 0), outN - n);
      if (args.bias2d) add8(f, args.bias2d + (size_t)(m / args.rows_per_b) * N + n, full && (N % 8 == 0), outN - n);
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
      *reinterpret_cast<uint4*>(cp) = pack8(f);
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
      }
    }
  }
  if (args.gn_part) {
    // column pass: (mean, M2) of each output channel over this tile's rows
    // (two-pass in LDS: exact, no E[x^2]-E[x]^2 cancellation)
    epi_barrier<RAW>();
    const int rows = min(BM, M - m0);
    for (int c = tid; c < BN; c += 256) {
      const int n = n0 + c;
      if (n >= N || rows <= 0) continue;
      float sm = 0.f;
      for (int r = 0; r < rows; ++r) sm += cs[r * LDC_S + c];
      const float mean = sm / (float)rows;
      float m2 = 0.f;
      for (int r = 0; r < rows; ++r) { const float d = cs[r * LDC_S + c] - mean; m2 += d * d; }
      float* o = args.gn_part + ((size_t)(m0 / BM) * N + n) * 2;
      o[0] = mean;
      o[1] = m2;
    }
  }
}

int csk_gemm_glds_launch(const GemmArgs& a, int tile, int ksplit, bool conv, hipStream_t s);
