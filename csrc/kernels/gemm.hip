// MFMA bf16 GEMM and NHWC implicit-GEMM convolution for gfx950.
//
//   C[M, N] = epilogue( A[M, K] . W[N, K]^T )
//
// A is either a row-major activation matrix (Linear / 1x1 conv) or the implicit
// im2col of an NHWC image (3x3 / strided / nearest-x2-upsampled conv, computed
// on the fly by the loader: no im2col buffer).  W rows are K-contiguous
// ([N][K] linear weights, [Cout][kh][kw][Cin] packed conv weights), so both
// MFMA operands are read from identical K-contiguous LDS tiles.
//
// Tiling (CDNA4 wave64): 256 threads = 4 waves arranged WM x WN; each wave owns
// a (BM/WM) x (BN/WN) sub-tile made of 16x16 accumulators fed by
// v_mfma_f32_16x16x32_bf16 (lane l holds A[l&15][8(l>>4)..+7] -> one 16-byte
// ds_read_b128 per fragment).  BK = 64.  LDS tiles are [rows][64] bf16 with the
// 16-byte chunk index XOR-swizzled by (row & 7): the b128 fragment reads of a
// 16-lane group then hit 16 distinct bank slots (conflict-free, verified on
// paper against the ds_read_b128 lane groups in MI355X_MICROARCH.md §LDS).
// Global->LDS is register-staged and double-buffered with one barrier per
// K-step (loads for k+1 are in flight while MFMAs consume k).
//
// Epilogue: accumulators -> fp32 LDS tile (padded rows) -> coalesced 16-byte
// row-contiguous pass that applies bias, per-sample bias2d (ResNet time
// embedding), activation (GELU/SiLU/quick-GELU), GEGLU gating (done in
// registers: packed weights put (hidden, gate) for the same column in the same
// lane), and the residual add, then stores bf16.
//
// Workgroup -> tile mapping is XCD-aware (common.h xcd_remap): consecutive
// tiles of one A row-panel land on one XCD's L2.
#include "common.h"

enum { ACT_NONE = 0, ACT_GELU = 1, ACT_SILU = 2, ACT_GEGLU = 3, ACT_QGELU = 4 };

struct GemmArgs {
  const bf16_t* A;  // GEMM: [M][lda];  CONV: NHWC input [B][H][W][Cin]
  const bf16_t* W;  // [N][K]
  bf16_t* C;        // [M][ldc]
  const bf16_t* bias;    // [N] or null
  const bf16_t* bias2d;  // [B][N] or null (row m uses b = m / rows_per_b)
  const bf16_t* res;     // [M][ldc] or null
  int M, N, K, lda, ldb, ldc, rows_per_b, act;
  float* ws;   // split-K fp32 partials [ksplit][M][N] (null: no split)
  int kchunk;  // K elements per split (multiple of BK)
  // conv geometry
  int H, Wd, Cin, Ho, Wo, kh, kw, stride, pt, pl, up2x;
};

#define BK 64

__device__ __forceinline__ int swz(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

template <int BM, int BN, int WM, int WN, bool CONV>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const GemmArgs args) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int CA = BM * 8 / 256, CB = BN * 8 / 256;  // 16B chunks per thread per K-step
  constexpr int SMEM_MAIN = 2 * (BM + BN) * BK;          // bf16 elements
  constexpr int LDC_S = BN + 4;                          // fp32 staging row stride (floats)
  constexpr int SMEM_EPI = BM * LDC_S * 2;               // in bf16-element units
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];
  bf16_t* As = smem;                 // [2][BM*BK]
  bf16_t* Bs = smem + 2 * BM * BK;   // [2][BN*BK]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int M = args.M, N = args.N, K = args.K;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int split = blockIdx.y;
  const int kbeg = split * args.kchunk;
  const int kend = args.ws ? min(K, kbeg + args.kchunk) : K;
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;

  // ---- per-thread load bookkeeping (each thread's 16B chunk column is fixed) ----
  const int lc = tid & 7;  // chunk within the 64-wide K slice
  const bf16_t* a_ptr[CA];
  bool a_ok[CA];
  int a_ihb[CA], a_iwb[CA];
  size_t a_bbase[CA];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int row = (tid >> 3) + 32 * i;
    const int m = m0 + row;
    a_ok[i] = m < M;
    if constexpr (CONV) {
      const int mm = a_ok[i] ? m : 0;
      const int hw = args.Ho * args.Wo;
      const int b = mm / hw, r = mm - b * hw;
      const int oh = r / args.Wo, ow = r - oh * args.Wo;
      a_ihb[i] = oh * args.stride - args.pt;
      a_iwb[i] = ow * args.stride - args.pl;
      a_bbase[i] = (size_t)b * args.H * args.Wd;
      a_ptr[i] = nullptr;
    } else {
      a_ptr[i] = args.A + (size_t)(a_ok[i] ? m : 0) * args.lda + lc * 8;
      a_ihb[i] = a_iwb[i] = 0;
      a_bbase[i] = 0;
    }
  }
  const bf16_t* b_ptr[CB];
  bool b_ok[CB];
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int n = n0 + (tid >> 3) + 32 * i;
    b_ok[i] = n < N;
    b_ptr[i] = args.W + (size_t)(b_ok[i] ? n : 0) * args.ldb + lc * 8;
  }
  // conv K-position state for this thread's chunk: k = kbeg + kt*64 + lc*8 -> (tap, ci)
  int c_ci = 0, c_ky = 0, c_kx = 0;
  if constexpr (CONV) {
    const int k0 = kbeg + lc * 8;
    const int tap = k0 / args.Cin;
    c_ci = k0 - tap * args.Cin;
    c_ky = tap / args.kw;
    c_kx = tap - c_ky * args.kw;
  }
  const int Hin = args.up2x ? 2 * args.H : args.H;
  const int Win = args.up2x ? 2 * args.Wd : args.Wd;

  uint4 ra[CA], rb[CB];
  auto load_tiles = [&](int kt) {
    const int k = kbeg + kt * BK + lc * 8;
    const bool kin = k < kend;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if constexpr (CONV) {
        const int ih = a_ihb[i] + c_ky, iw = a_iwb[i] + c_kx;
        if (kin && a_ok[i] && ih >= 0 && ih < Hin && iw >= 0 && iw < Win) {
          const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
          v = *reinterpret_cast<const uint4*>(args.A + (a_bbase[i] + (size_t)sh * args.Wd + sw) * args.Cin + c_ci);
        }
      } else {
        if (kin && a_ok[i]) v = *reinterpret_cast<const uint4*>(a_ptr[i] + (size_t)kbeg + (size_t)kt * BK);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < CB; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (kin && b_ok[i]) v = *reinterpret_cast<const uint4*>(b_ptr[i] + (size_t)kbeg + (size_t)kt * BK);
      rb[i] = v;
    }
    if constexpr (CONV) {  // advance (tap, ci) by 64 channels
      c_ci += BK;
      while (c_ci >= args.Cin) { c_ci -= args.Cin; if (++c_kx == args.kw) { c_kx = 0; ++c_ky; } }
    }
  };
  auto store_tiles = [&](int buf) {
    bf16_t* as = As + buf * BM * BK;
    bf16_t* bs = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < CA; ++i) *reinterpret_cast<uint4*>(as + swz((tid >> 3) + 32 * i, lc)) = ra[i];
#pragma unroll
    for (int i = 0; i < CB; ++i) *reinterpret_cast<uint4*>(bs + swz((tid >> 3) + 32 * i, lc)) = rb[i];
  };

  v4f acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nk = (kend - kbeg + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);
    const bf16_t* as = As + cur * BM * BK;
    const bf16_t* bs = Bs + cur * BN * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8s af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *reinterpret_cast<const v8s*>(as + swz(wm * WTM + i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < NT; ++j)
        bfr[j] = *reinterpret_cast<const v8s*>(bs + swz(wn * WTN + j * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
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
        const int oc = (wn * WTN + j * 16) / 2 + fr;  // column within the half-width output tile
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = wm * WTM + i * 16 + fq * 4 + r;
          const float h = acc[i][j][r] + bh, g = acc[i][j + 1][r] + bg;
          cs[row * LDC_S + oc] = h * gelu_f(g);
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
  __syncthreads();
  const int outN = act == ACT_GEGLU ? N / 2 : N;
  const int BNo = act == ACT_GEGLU ? BN / 2 : BN;
  const int on0 = act == ACT_GEGLU ? n0 / 2 : n0;
  const int vpr = BNo / 8;  // 16-byte vectors per tile row
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
      if (args.bias) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += (n + j < outN) ? bf2f(args.bias[n + j]) : 0.f;
      }
      if (args.bias2d) {
        const bf16_t* b2 = args.bias2d + (size_t)(m / args.rows_per_b) * N;
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += (n + j < outN) ? bf2f(b2[n + j]) : 0.f;
      }
      if (act == ACT_GELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = gelu_f(f[j]);
      } else if (act == ACT_SILU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = silu_f(f[j]);
      } else if (act == ACT_QGELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = qgelu_f(f[j]);
      }
    }
    bf16_t* cp = args.C + (size_t)m * args.ldc + n;
    if (full && ((((size_t)cp) & 15) == 0)) {
      if (args.res) {
        float rf[8];
        unpack8(*reinterpret_cast<const uint4*>(args.res + (size_t)m * args.ldc + n), rf);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += rf[j];
      }
      *reinterpret_cast<uint4*>(cp) = pack8(f);
    } else {
      for (int j = 0; j < 8 && n + j < outN; ++j) {
        float o = f[j];
        if (args.res) o += bf2f(args.res[(size_t)m * args.ldc + n + j]);
        cp[j] = f2bf(o);
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, bool CONV>
static int launch(const GemmArgs& a, int ksplit, hipStream_t s) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  gemm_kernel<BM, BN, WM, WN, CONV><<<dim3(tiles, ksplit), 256, 0, s>>>(a);
  return (int)hipGetLastError();
}

// split-K reduce: out = epilogue(sum_s ws[s]) (bias, bias2d, act, residual)
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, bf16_t* __restrict__ C, const bf16_t* __restrict__ bias,
                                     const bf16_t* __restrict__ bias2d, const bf16_t* __restrict__ res, int M, int N,
                                     int ldc, int rows_per_b, int act, int ksplit) {
  const size_t total = (size_t)M * N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / N), n = (int)(i - (size_t)m * N);
    float v = 0.f;
    for (int sidx = 0; sidx < ksplit; ++sidx) v += ws[(size_t)sidx * total + i];
    if (bias) v += bf2f(bias[n]);
    if (bias2d) v += bf2f(bias2d[(size_t)(m / rows_per_b) * N + n]);
    if (act == ACT_GELU) v = gelu_f(v);
    else if (act == ACT_SILU) v = silu_f(v);
    else if (act == ACT_QGELU) v = qgelu_f(v);
    if (res) v += bf2f(res[(size_t)m * ldc + n]);
    C[(size_t)m * ldc + n] = f2bf(v);
  }
}

template <bool CONV>
static int dispatch(GemmArgs a, int tile, int ksplit, hipStream_t s) {
  if (ksplit > 1 && a.act == ACT_GEGLU) ksplit = 1;
  if (ksplit > 1) {
    if (!a.ws) return (int)hipErrorInvalidValue;
    const int nk = (a.K + BK - 1) / BK;
    a.kchunk = ((nk + ksplit - 1) / ksplit) * BK;
    ksplit = (a.K + a.kchunk - 1) / a.kchunk;
  } else {
    a.ws = nullptr;
    a.kchunk = a.K;
    ksplit = 1;
  }
  if (tile == 0) {  // heuristic: wide tiles for big problems, narrow-N tiles for Cout <= 64
    const long long t128 = (long long)((a.M + 127) / 128) * ((a.N + 127) / 128);
    if (a.N <= 32) tile = 5;
    else if (a.N <= 64) tile = 6;
    else if (t128 >= 512 || a.act == ACT_GEGLU) tile = 1;
    else tile = 4;
  }
  if (a.act == ACT_GEGLU && tile != 1 && tile != 3) tile = 1;  // needs >= 32 cols per wave
  int err;
  switch (tile) {
    case 1: err = launch<128, 128, 2, 2, CONV>(a, ksplit, s); break;
    case 2: err = launch<128, 64, 2, 2, CONV>(a, ksplit, s); break;
    case 3: err = launch<64, 128, 2, 2, CONV>(a, ksplit, s); break;
    case 4: err = launch<64, 64, 2, 2, CONV>(a, ksplit, s); break;
    case 5: err = launch<128, 32, 4, 1, CONV>(a, ksplit, s); break;
    case 6: err = launch<128, 64, 4, 1, CONV>(a, ksplit, s); break;
    default: return (int)hipErrorInvalidValue;
  }
  if (err || ksplit == 1) return err;
  const size_t total = (size_t)a.M * a.N;
  int grid = (int)((total + 255) / 256);
  if (grid > 8192) grid = 8192;
  splitk_reduce_kernel<<<grid, 256, 0, s>>>(a.ws, a.C, a.bias, a.bias2d, a.res, a.M, a.N, a.ldc, a.rows_per_b, a.act,
                                             ksplit);
  return (int)hipGetLastError();
}

CSK_API int csk_gemm(void* C, const void* A, const void* W, const void* bias, const void* bias2d, const void* res,
                     int M, int N, int K, int lda, int ldb, int ldc, int rows_per_b, int act, int tile, int ksplit,
                     void* ws, hipStream_t stream) {
  if (K % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || (act == ACT_GEGLU && N % 32 != 0)) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias; a.bias2d = (const bf16_t*)bias2d; a.res = (const bf16_t*)res;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.rows_per_b = rows_per_b > 0 ? rows_per_b : 1; a.act = act;
  a.ws = (float*)ws;
  if (M == 0 || N == 0) return 0;
  return dispatch<false>(a, tile, ksplit, stream);
}

CSK_API int csk_conv2d(void* Y, const void* X, const void* Wp, const void* bias, const void* bias2d, const void* res,
                       int B, int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pt, int pl, int Ho, int Wo,
                       int up2x, int tile, int ksplit, void* ws, hipStream_t stream) {
  if (Cin % 8 != 0) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)X; a.W = (const bf16_t*)Wp; a.C = (bf16_t*)Y;
  a.bias = (const bf16_t*)bias; a.bias2d = (const bf16_t*)bias2d; a.res = (const bf16_t*)res;
  a.M = B * Ho * Wo; a.N = Cout; a.K = kh * kw * Cin; a.lda = 0; a.ldb = kh * kw * Cin; a.ldc = Cout; a.rows_per_b = Ho * Wo;
  a.act = ACT_NONE;
  a.H = H; a.Wd = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.kh = kh; a.kw = kw; a.stride = stride; a.pt = pt; a.pl = pl;
  a.up2x = up2x;
  a.ws = (float*)ws;
  if (a.M == 0) return 0;
  return dispatch<true>(a, tile, ksplit, stream);
}
