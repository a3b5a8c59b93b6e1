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
#include "gemm_common.h"

template <int BM, int BN, int WM, int WN, bool CONV, bool FAST>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const GemmArgs args) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int CA = BM * 8 / 256, CB = BN * 8 / 256;  // 16B chunks per thread per K-step
  constexpr int SMEM_MAIN = 2 * (BM + BN) * BK;          // bf16 elements
  constexpr int LDC_S = BN + 4;                          // fp32 staging row stride (floats)
  constexpr int SMEM_EPI = epi_smem_elems<BM, BN>();    // in bf16-element units
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];
  bf16_t* As = smem;                 // [2][BM*BK]
  bf16_t* Bs = smem + 2 * BM * BK;   // [2][BN*BK]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR address math
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

  // FAST staging (see gemm_glds.hip): uniform tap, running per-row pointers,
  // invalid rows / padding read the zero page -> no per-step address math.
  const bf16_t* fa[CA];
  const bf16_t* fb[CB];
  int f_ky = 0, f_kx = 0, f_c = 0;
  auto set_rows = [&]() {
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int ih = a_ihb[i] + f_ky * args.dil, iw = a_iwb[i] + f_kx * args.dil;
      const bool v = a_ok[i] && ih >= 0 && ih < Hin && iw >= 0 && iw < Win;
      const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
      fa[i] = v ? args.A + (a_bbase[i] + (size_t)sh * args.Wd + sw) * args.lda + lc * 8 : args.zero + lc * 8;
    }
  };
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < CB; ++i) fb[i] = b_ok[i] ? b_ptr[i] + kbeg : args.zero + lc * 8;
    if constexpr (CONV) {
      const int tap = kbeg / args.Cin;
      f_c = kbeg - tap * args.Cin;
      f_ky = tap / args.kw;
      f_kx = tap - f_ky * args.kw;
      set_rows();
    } else {
#pragma unroll
      for (int i = 0; i < CA; ++i) fa[i] = a_ok[i] ? a_ptr[i] + kbeg : args.zero + lc * 8;
    }
  }

  uint4 ra[CA], rb[CB];
  auto load_tiles = [&](int kt) {
    if constexpr (FAST) {
#pragma unroll
      for (int i = 0; i < CA; ++i) ra[i] = *reinterpret_cast<const uint4*>(CONV ? fa[i] + f_c : fa[i]);
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        rb[i] = *reinterpret_cast<const uint4*>(fb[i]);
        fb[i] += BK;
      }
      if constexpr (CONV) {
        f_c += BK;
        if (f_c == args.Cin) {
          f_c = 0;
          if (++f_kx == args.kw) { f_kx = 0; ++f_ky; }
          set_rows();
        }
      } else {
#pragma unroll
        for (int i = 0; i < CA; ++i) fa[i] += BK;
      }
      return;
    }
    const int k = kbeg + kt * BK + lc * 8;
    const bool kin = k < kend;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if constexpr (CONV) {
        const int ih = a_ihb[i] + c_ky * args.dil, iw = a_iwb[i] + c_kx * args.dil;
        if (kin && a_ok[i] && ih >= 0 && ih < Hin && iw >= 0 && iw < Win) {
          const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
          v = *reinterpret_cast<const uint4*>(args.A + (a_bbase[i] + (size_t)sh * args.Wd + sw) * args.lda + c_ci);
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
  const float2 lnrow = ln_row_stats<BM>(args, m0);
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

  gemm_epilogue<BM, BN, WM, WN>(args, acc, smem, m0, n0, split, lnrow);
}

template <int BM, int BN, int WM, int WN, bool CONV>
static int launch(const GemmArgs& a0, int ksplit, hipStream_t s) {
  GemmArgs a = a0;
  a.gn_seg = gn_seg_for<BM, BN, WM>();
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int span = ksplit > 1 ? a.kchunk : a.K;
  // FAST staging measured SLOWER on this register-staged pipeline (127 -> 309 us on
  // the 64x64x320 conv: the running-pointer loads lose their overlap with the
  // MFMAs); it stays on for the LDS-DMA kernels only (gemm_glds.hip, 512 -> 732 TF/s).
  constexpr bool kFastRegStaged = false;
  const bool fast = kFastRegStaged && a.zero && (CONV ? (a.Cin % BK == 0) : true) && a.K % BK == 0 &&
                    (size_t)(span + 2 * BK) * sizeof(bf16_t) <= (size_t)csk_zero_bytes() &&
                    (!CONV || (size_t)(a.Cin + BK) * sizeof(bf16_t) <= (size_t)csk_zero_bytes());
  if (fast)
    gemm_kernel<BM, BN, WM, WN, CONV, true><<<dim3(tiles, ksplit), 256, 0, s>>>(a);
  else
    gemm_kernel<BM, BN, WM, WN, CONV, false><<<dim3(tiles, ksplit), 256, 0, s>>>(a);
  return (int)hipGetLastError();
}

// f[q][0..7] += partials of splits [s0, s0 + U) at rows w[q] (split stride
// `total` floats): all U * R * 2 loads issued before the first add
template <int U, int R>
__device__ __forceinline__ void add_splits(float (&f)[R][8], const float* const (&w)[R], size_t total, int s0) {
  float4 lo[U][R], hi[U][R];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const float* p = w[q] + (size_t)(s0 + u) * total;
      lo[u][q] = *reinterpret_cast<const float4*>(p);
      hi[u][q] = *reinterpret_cast<const float4*>(p + 4);
    }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int q = 0; q < R; ++q) {
      f[q][0] += lo[u][q].x; f[q][1] += lo[u][q].y; f[q][2] += lo[u][q].z; f[q][3] += lo[u][q].w;
      f[q][4] += hi[u][q].x; f[q][5] += hi[u][q].y; f[q][6] += hi[u][q].z; f[q][7] += hi[u][q].w;
    }
  // keep the loads together: under register pressure (the GN reduce) the
  // scheduler otherwise interleaves each load pair with its adds and waits
  __builtin_amdgcn_sched_group_barrier(0x020, 2 * U * R, 0);  // VMEM reads
  __builtin_amdgcn_sched_group_barrier(0x002, 8 * U * R, 0);  // VALU adds
}

// sum of all ksplit partials, SU (1 / 4 / 8) splits per memory round trip
template <int SU, int R>
__device__ __forceinline__ void sum_splits(float (&f)[R][8], const float* const (&w)[R], size_t total, int ksplit) {
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int j = 0; j < 8; ++j) f[q][j] = 0.f;
  int s = 0;
  if constexpr (SU >= 8)
    for (; s + 8 <= ksplit; s += 8) add_splits<8, R>(f, w, total, s);
  if constexpr (SU >= 4)
    for (; s + 4 <= ksplit; s += 4) add_splits<4, R>(f, w, total, s);
  for (; s < ksplit; ++s) add_splits<1, R>(f, w, total, s);
}

// split-K reduce: out = epilogue(sum_s ws[s]) (bias, bias2d, act, residual)
__global__ void splitk_reduce_kernel(const GemmArgs a, int ksplit) {
  const int M = a.M, N = a.N;
  const size_t total = (size_t)M * N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / N), n = (int)(i - (size_t)m * N);
    float v = 0.f;
    for (int sidx = 0; sidx < ksplit; ++sidx) v += a.ws[(size_t)sidx * total + i];
    if (a.bias) v += bf2f(a.bias[n]);
    if (a.bias2d) v += bf2f(a.bias2d[(size_t)(m / a.rows_per_b) * a.ldb2 + n]);
    v = apply_act(a.act, v);
    v *= a.out_scale;
    if (a.res) v += bf2f(a.res[(size_t)m * a.ldr + n]);
    a.C[(size_t)m * a.ldc + n] = f2bf(v);
  }
}

// 8 columns per thread: 2x float4 per split, 16-byte bias / residual / output
// accesses (the scalar kernel above issues one 4-byte load per split per value)
template <int SU>
__global__ void splitk_reduce8_kernel(const GemmArgs a, int ksplit) {
  const int M = a.M, N = a.N, NV = N / 8;
  const size_t total = (size_t)M * N, nvec = (size_t)M * NV;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / NV), n = (int)(i - (size_t)m * NV) * 8;
    const float* const w[1] = {a.ws + (size_t)m * N + n};
    float ff[1][8];
    sum_splits<SU, 1>(ff, w, total, ksplit);
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = ff[0][j];
    if (a.bias) add8(f, a.bias + n, true, 8);
    if (a.bias2d) add8(f, a.bias2d + (size_t)(m / a.rows_per_b) * a.ldb2 + n, true, 8);
    act8(a.act, f);
    if (a.out_scale != 1.0f) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= a.out_scale;
    }
    if (a.res) add8(f, a.res + (size_t)m * a.ldr + n, true, 8);
    *reinterpret_cast<uint4*>(a.C + (size_t)m * a.ldc + n) = pack8(f);
  }
}

// Split-K reduce that also emits the consumer GroupNorm's statistics (the
// partial layout of the GEMM epilogue: gn_part[((m / gn_seg) * N + n) * 2] =
// (mean, M2) of the final fp32 outputs of a gn_seg-row segment), so a split-K
// producer no longer forces the separate statistics pass over its output.
// Workgroup = (segment, 8*VC-column block); thread (cv, r0) finishes rows
// r0, r0 + RPI, ... of its 8 columns and keeps their running (mean, M2)
// (Welford); the RPI row groups are merged in LDS (Chan).  The first version
// walked its rows one dependent load at a time and cost the step 0.36 ms
// (tools/abstep.py skgn0 / skgn1); the rows' loads now go out together.
// SU: splits whose partials are loaded together (one memory round trip per SU
// splits; the plain loop waited on every split's loads before issuing the next)
template <int VC, int SU>
__global__ __launch_bounds__(256) void splitk_reduce8_gn_kernel(const GemmArgs a, int ksplit) {
  constexpr int RPI = 256 / VC, RPT = SPLITK_GN_SEG / RPI;  // row groups, rows per thread
  static_assert(SPLITK_GN_SEG % RPI == 0, "segment rows split evenly over the row groups");
  __shared__ float smean[RPI * (8 * VC + 1)], sm2[RPI * (8 * VC + 1)];
  const int N = a.N;
  const size_t total = (size_t)a.M * N;
  const int cv = threadIdx.x % VC, r0 = threadIdx.x / VC;
  const int n = (blockIdx.y * VC + cv) * 8;
  const bool live = n < N;
  float mean[8], m2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) mean[j] = m2[j] = 0.f;
  if (live) {
    // all of this thread's rows' partial sums first (independent loads in flight
    // together), then the epilogue and the Welford update row by row
    float f[RPT][8];
    const float* w[RPT];
#pragma unroll
    for (int q = 0; q < RPT; ++q) w[q] = a.ws + (size_t)(blockIdx.x * SPLITK_GN_SEG + r0 + q * RPI) * N + n;
    sum_splits<SU, RPT>(f, w, total, ksplit);
    float bb[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bb[j] = 0.f;
    if (a.bias) add8(bb, a.bias + n, true, 8);
#pragma unroll
    for (int q = 0; q < RPT; ++q) {
      const int m = blockIdx.x * SPLITK_GN_SEG + r0 + q * RPI;
#pragma unroll
      for (int j = 0; j < 8; ++j) f[q][j] += bb[j];
      if (a.bias2d) add8(f[q], a.bias2d + (size_t)(m / a.rows_per_b) * a.ldb2 + n, true, 8);
      act8(a.act, f[q]);
      if (a.out_scale != 1.0f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[q][j] *= a.out_scale;
      }
      if (a.res) add8(f[q], a.res + (size_t)m * a.ldr + n, true, 8);
      *reinterpret_cast<uint4*>(a.C + (size_t)m * a.ldc + n) = pack8(f[q]);
      const float inv = 1.0f / (float)(q + 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[q][j] - mean[j];
        mean[j] += d * inv;
        m2[j] += d * (f[q][j] - mean[j]);
      }
    }
  }
  // merge the RPI row groups of each of the WG's 8*VC columns: 4 lanes per
  // column (consecutive lanes, shuffle-reduced), RPI/4 groups each; equal counts
  // (RPT rows per group): mean = average of the group means, M2 = sum of the
  // group M2 + RPT * sum (mean_g - mean)^2 (exact Chan merge)
  constexpr int CW = 8 * VC, LS = CW + 1;  // padded row-group stride: the 4 lanes of a column hit 4 banks
  static_assert(CW * 4 == 256 && RPI % 4 == 0, "4 merge lanes per column");
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    smean[r0 * LS + cv * 8 + j] = mean[j];
    sm2[r0 * LS + cv * 8 + j] = m2[j];
  }
  __syncthreads();
  const int c = threadIdx.x >> 2, part = threadIdx.x & 3;
  float sm = 0.f;
#pragma unroll
  for (int g = part; g < RPI; g += 4) sm += smean[g * LS + c];
  sm += __shfl_xor(sm, 1);
  sm += __shfl_xor(sm, 2);
  const float mu = sm / (float)RPI;
  float q = 0.f;
#pragma unroll
  for (int g = part; g < RPI; g += 4) {
    const float d = smean[g * LS + c] - mu;
    q += sm2[g * LS + c] + (float)RPT * d * d;
  }
  q += __shfl_xor(q, 1);
  q += __shfl_xor(q, 2);
  const int nc = blockIdx.y * CW + c;
  if (part == 0 && nc < N)
    *reinterpret_cast<float2*>(a.gn_part + ((size_t)blockIdx.x * N + nc) * 2) = make_float2(mu, q);
}

// splits loaded per memory round trip in the split-K reduces (1: the old
// one-split-at-a-time loop; A/B knob for tools/abstep.py skr1 / skr4 / skr8)
static int g_skr_unroll = 4;  // 4: -0.022 ms (CFG 8) / -0.023 ms (CFG 2) per step vs 1; 8 no better (profiles/unet_step_ab_skr_r7d.txt)
CSK_API int csk_set_skr_unroll(int v) {
  g_skr_unroll = v;
  return 0;
}

static int splitk_reduce(const GemmArgs& a, int ksplit, hipStream_t s) {
  const size_t total = (size_t)a.M * a.N;
  const bool vec = a.N % 8 == 0 && a.ldc % 8 == 0 && (!a.res || a.ldr % 8 == 0) && (!a.bias2d || a.ldb2 % 8 == 0) &&
                   ((size_t)a.C % 16 == 0) && (!a.res || (size_t)a.res % 16 == 0) && (!a.bias || (size_t)a.bias % 16 == 0) &&
                   (!a.bias2d || (size_t)a.bias2d % 16 == 0) && ((size_t)a.ws % 16 == 0);
  if (a.gn_part) {  // host guarantees the vector layout and gn_seg | M (hip_ops._gn_seg)
    constexpr int VC = 8;
    if (!vec || a.gn_seg != SPLITK_GN_SEG || a.M % SPLITK_GN_SEG != 0) return (int)hipErrorInvalidValue;
    const dim3 g(a.M / SPLITK_GN_SEG, (a.N / 8 + VC - 1) / VC);
    if (g_skr_unroll >= 8) splitk_reduce8_gn_kernel<VC, 8><<<g, 256, 0, s>>>(a, ksplit);
    else if (g_skr_unroll >= 4) splitk_reduce8_gn_kernel<VC, 4><<<g, 256, 0, s>>>(a, ksplit);
    else splitk_reduce8_gn_kernel<VC, 1><<<g, 256, 0, s>>>(a, ksplit);
    return (int)hipGetLastError();
  }
  if (vec) {
    int grid = (int)((total / 8 + 255) / 256);
    if (grid > 8192) grid = 8192;
    if (g_skr_unroll >= 8) splitk_reduce8_kernel<8><<<grid, 256, 0, s>>>(a, ksplit);
    else if (g_skr_unroll >= 4) splitk_reduce8_kernel<4><<<grid, 256, 0, s>>>(a, ksplit);
    else splitk_reduce8_kernel<1><<<grid, 256, 0, s>>>(a, ksplit);
    return (int)hipGetLastError();
  }
  int grid = (int)((total + 255) / 256);
  if (grid > 8192) grid = 8192;
  splitk_reduce_kernel<<<grid, 256, 0, s>>>(a, ksplit);
  return (int)hipGetLastError();
}

int g_gn_lds = 0;  // tools/abstep.py arms gnd0 / gnd1: GN statistics in the direct (0) or LDS (1) epilogue
int g_sw_odd = 0;  // tools/abstep.py arms swodd0 / swodd1: 160-wide tiles on the direct (1) or LDS (0) epilogue; direct measured 0.11 ms/step slower
CSK_API int csk_set_sw_odd(int v) {
  g_sw_odd = v;
  return 0;
}
int g_epi_nt = 0;  // tools/abstep.py arms nt0 / nt1 / nt2: non-temporal direct-epilogue stores (/ residual loads)
CSK_API int csk_set_epi_nt(int v) {
  g_epi_nt = v;
  return 0;
}
int g_epi_band = 1;  // tools/abstep.py arms band0 / band1: LDS-staged epilogue band path off / on
CSK_API int csk_set_epi_band(int v) {
  g_epi_band = v;
  return 0;
}
CSK_API int csk_set_gn_lds(int v) {
  g_gn_lds = v;
  return 0;
}

// the LDS-DMA tiles of gemm_glds.hip (csk_gemm_glds_launch)
static inline bool glds_tile(int t) { return (t >= 11 && t <= 29) || t == 36; }

template <bool CONV>
static int dispatch(GemmArgs a, int tile, int ksplit, hipStream_t s) {
  a.zero = csk_zero_ptr();
  a.gn_lds = g_gn_lds;
  a.sw_odd = g_sw_odd;
  a.epi_band = g_epi_band;
  a.epi_nt = g_epi_nt;
  // profiling probes (act 97-99) exist only in the LDS-DMA tiles (gemm_glds.hip);
  // any other kernel would run them as a plain full-width epilogue — into a
  // caller's GEGLU-sized (N/2) output that is an out-of-bounds write
  if ((a.act == ACT_PROBE_NO_EPILOGUE || a.act == ACT_PROBE_NO_STORE || a.act == ACT_PROBE_NO_A) &&
      !glds_tile(tile))
    return (int)hipErrorInvalidValue;
  // ksplit < 0: split -ksplit ways with the in-kernel fixup (LDS-DMA tiles only:
  // the last split of each tile runs the full epilogue, so GEGLU / LN / row and
  // GN statistics work as unsplit; the host sizes GN segments for the tile)
  const bool fixup = ksplit < 0;
  if (fixup) {
    if (!glds_tile(tile) || !a.ws || a.attn_kv) return (int)hipErrorInvalidValue;
    ksplit = -ksplit;
  }
  if (ksplit > 1 && a.act == ACT_GEGLU && !fixup) ksplit = 1;
  if (a.gn_part && (a.act == ACT_GEGLU || tile == 0)) return (int)hipErrorInvalidValue;
  if ((a.ln_part || a.row_part) && ((ksplit > 1 && !fixup) || tile == 0)) return (int)hipErrorInvalidValue;
  if (a.row_part && a.act == ACT_GEGLU) return (int)hipErrorInvalidValue;
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
  if (fixup && ksplit > 1) {  // gemm_glds.hip launch_glds: per-tile counters, no reduce kernel
    a.fx_ws = a.ws;
    const int err = csk_gemm_glds_launch(a, tile, ksplit, CONV, s);
    return err;
  }
  if (tile == 0) {  // heuristic: wide tiles for big problems, narrow-N tiles for Cout <= 64
    const long long t128 = (long long)((a.M + 127) / 128) * ((a.N + 127) / 128);
    if (a.N <= 32) tile = 5;
    else if (a.N <= 64) tile = 6;
    else if (t128 >= 512 || a.act == ACT_GEGLU) tile = 1;
    else tile = 4;
  }
  int err;
  // (stream-K, sliced-K and persistent cross-tile tiles 40-44 / 50-53 were built,
  // measured slower in round 5 and removed: README "Measured and removed")
  if (tile >= 31 && tile <= 34) {  // 8-wave phased / ring tiles (gemm8p.hip)
    err = csk_gemm8p_launch(a, tile, ksplit, CONV, s);
    if (err == (int)hipErrorNotSupported) {
      // the fallback must write the GN-statistics segments the host sized gn_part
      // for (hip_ops._gn_seg of the REQUESTED tile): 33 / 34 (64-row band) ->
      // tile 26 (128x160, two bands); 31 / 32 -> tile 11 only when its segment
      // matches (fine segments: 31 / 32 write 128 rows, tile 11 64 -> an
      // out-of-bounds gn_part write).  A mismatch fails loudly instead.
      const int fb = tile >= 33 ? 26 : 11;
      if (a.gn_part && ksplit == 1) {
        const int want = tile >= 33 ? (tile == 33 ? gn_seg_for<256, 160, 4>() : gn_seg_for<256, 128, 4>())
                                    : 128;  // launch8p: min(BN or 256, one 128-row band)
        const int got = fb == 26 ? gn_seg_for<128, 160, 2>() : gn_seg_for<128, 128, 2>();
        if (want != got) return (int)hipErrorInvalidValue;
      }
      err = csk_gemm_glds_launch(a, fb, ksplit, CONV, s);
    }
  } else if (tile >= 11) {
    err = csk_gemm_glds_launch(a, tile, ksplit, CONV, s);
  } else {
    if (a.act == ACT_GEGLU && tile != 1 && tile != 3) tile = 1;  // needs >= 32 cols per wave
    switch (tile) {
      case 1: err = launch<128, 128, 2, 2, CONV>(a, ksplit, s); break;
      case 2: err = launch<128, 64, 2, 2, CONV>(a, ksplit, s); break;
      case 3: err = launch<64, 128, 2, 2, CONV>(a, ksplit, s); break;
      case 4: err = launch<64, 64, 2, 2, CONV>(a, ksplit, s); break;
      case 5: err = launch<128, 32, 4, 1, CONV>(a, ksplit, s); break;
      case 6: err = launch<128, 64, 4, 1, CONV>(a, ksplit, s); break;
      default: return (int)hipErrorInvalidValue;
    }
  }
  if (err || ksplit == 1) return err;
  if (a.gn_part) a.gn_seg = SPLITK_GN_SEG;  // mirrored by hip_ops._gn_seg
  return splitk_reduce(a, ksplit, s);
}

// y[M, ldc] = act(A[M, lda] . W[N, ldb]^T + bias + bias2d) * out_scale + res[M, ldr]
// (+ fused input LayerNorm / output row statistics: GemmArgs::ln_part / row_part)
// Per-row LayerNorm statistics for a fused-LN consumer GEMM: row m merges the
// producer's column-slab partials part[(p * M + m) * 2 + {mean, M2}] (Chan,
// exact) into out[m] = (mean, rstd).  One thread per row.
__global__ void ln_rowstats_kernel(const float* __restrict__ part, float* __restrict__ out, int M, int K, int nparts,
                                   int pcols, float eps) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float n = 0.f, mean = 0.f, m2 = 0.f;
  // up to 16 slabs (K / producer BN: 2-10 in the UNet) loaded in one round trip,
  // then merged; a load-combine loop serialised one memory latency per slab
  constexpr int CAP = 16;
  float2 st[CAP];
#pragma unroll
  for (int p = 0; p < CAP; ++p)
    st[p] = p < nparts ? *reinterpret_cast<const float2*>(part + ((size_t)p * M + m) * 2) : make_float2(0.f, 0.f);
#pragma unroll
  for (int p = 0; p < CAP; ++p)
    if (p < nparts) chan_combine(n, mean, m2, (float)min(pcols, K - p * pcols), st[p].x, st[p].y);
  for (int p = CAP; p < nparts; ++p) {
    const float2 s2 = *reinterpret_cast<const float2*>(part + ((size_t)p * M + m) * 2);
    chan_combine(n, mean, m2, (float)min(pcols, K - p * pcols), s2.x, s2.y);
  }
  *reinterpret_cast<float2*>(out + (size_t)m * 2) = make_float2(mean, rsqrtf(m2 / fmaxf(n, 1.f) + eps));
}

int g_gn_fine = 0;  // tile segments: same step time as fine ones (tools/abstep.py), 4x fewer partials
CSK_API int csk_set_gn_fine(int v) {
  g_gn_fine = v;
  return 0;
}

static int g_ln_in_kernel = 1;  // A/B knob: 0 = ln_rowstats_kernel in front of every fused-LN consumer
CSK_API int csk_set_ln_in_kernel(int v) {
  g_ln_in_kernel = v;
  return 0;
}

CSK_API int csk_gemm_ln(void* C, const void* A, const void* W, const void* bias, const void* bias2d, const void* res,
                        int M, int N, int K, int lda, int ldb, int ldc, int ldr, int rows_per_b, int act,
                        float out_scale, void* gn_part, const void* ln_part, const void* ln_colsum, int ln_nparts,
                        int ln_pcols, float ln_eps, void* ln_rowbuf, void* row_part, int tile, int ksplit, void* ws,
                        hipStream_t stream) {
  if (K % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0 || (act == ACT_GEGLU && N % 32 != 0)) return (int)hipErrorInvalidValue;
  if (ln_part && (!ln_colsum || ln_nparts <= 0 || ln_pcols <= 0 ||
                  (long long)ln_nparts * ln_pcols < K))
    return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias; a.bias2d = (const bf16_t*)bias2d; a.res = (const bf16_t*)res;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldr = ldr > 0 ? ldr : ldc;
  a.rows_per_b = rows_per_b > 0 ? rows_per_b : 1; a.act = act; a.out_scale = out_scale;
  a.ldb2 = N;
  a.ws = (float*)ws;
  a.gn_part = (float*)gn_part;
  a.ln_part = (const float*)ln_part; a.ln_colsum = (const float*)ln_colsum;
  a.ln_nparts = ln_nparts; a.ln_pcols = ln_pcols; a.ln_eps = ln_eps;
  a.row_part = (float*)row_part;
  a.a_end = a.A + (size_t)(M > 0 ? M - 1 : 0) * lda + K;
  a.w_end = a.W + (size_t)(N > 0 ? N - 1 : 0) * ldb + K;
  if (M == 0 || N == 0) return 0;
  // the LDS-DMA tiles merge the row statistics themselves (gemm_common.h
  // ln_merge_tile); the others read them from a merge kernel launched first
  const bool in_kernel = glds_tile(tile) && g_ln_in_kernel;  // 21-26 remap to LDS-DMA tiles
  if (ln_part && !in_kernel) {  // (mean, rstd) per input row into the tail of the partials workspace' sibling
    float* rows = (float*)ln_rowbuf;
    if (!rows) return (int)hipErrorInvalidValue;
    ln_rowstats_kernel<<<(M + 255) / 256, 256, 0, stream>>>((const float*)ln_part, rows, M, K, ln_nparts, ln_pcols,
                                                           ln_eps);
    a.ln_row = rows;
  }
  return dispatch<false>(a, tile, ksplit, stream);
}

// Cross-attention query projection with the attention in its epilogue:
// O = softmax(((LN(A) W^T + bias) * scale) K^T) V per head (heads = N / 64,
// head dim 64), K / V from kv [Bc][Skv][2][N/64][64] (Attention.context_kv),
// sample m / rows_per_b.  Tiles 12 / 19 only (128 x 64, one head per tile, one
// sample per tile: rows_per_b % 128 == 0); no residual / activation / split-K.
CSK_API int csk_gemm_ln_attn(void* C, const void* A, const void* W, const void* bias, int M, int N, int K, int lda,
                             int ldb, int ldc, int rows_per_b, const void* ln_part, const void* ln_colsum,
                             int ln_nparts, int ln_pcols, float ln_eps, void* ln_rowbuf, const void* kv, int Bc,
                             int Skv, float scale, int tile, hipStream_t stream) {
  if ((tile != 12 && tile != 19) || N % 64 != 0 || Skv < 1 || Skv > 80 || rows_per_b <= 0 || rows_per_b % 128 != 0 ||
      M % rows_per_b != 0 || M / rows_per_b > Bc || ldc % 4 != 0 || !kv)
    return (int)hipErrorInvalidValue;
  if (K % 8 != 0 || lda % 8 != 0 || ldb % 8 != 0) return (int)hipErrorInvalidValue;
  if (ln_part && (!ln_colsum || ln_nparts <= 0 || ln_pcols <= 0 || (long long)ln_nparts * ln_pcols < K))
    return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A; a.W = (const bf16_t*)W; a.C = (bf16_t*)C;
  a.bias = (const bf16_t*)bias;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.ldr = ldc;
  a.rows_per_b = rows_per_b; a.act = ACT_NONE; a.out_scale = 1.0f;
  a.ldb2 = N;
  a.ln_part = (const float*)ln_part; a.ln_colsum = (const float*)ln_colsum;
  a.ln_nparts = ln_nparts; a.ln_pcols = ln_pcols; a.ln_eps = ln_eps;
  a.a_end = a.A + (size_t)(M > 0 ? M - 1 : 0) * lda + K;
  a.w_end = a.W + (size_t)(N > 0 ? N - 1 : 0) * ldb + K;
  a.attn_kv = (const bf16_t*)kv;
  a.attn_kv_end = a.attn_kv + (size_t)Bc * Skv * 2 * N;
  a.attn_skv = Skv;
  a.attn_sl2 = scale * 1.4426950408889634f;
  if (M == 0) return 0;
  if (ln_part && !g_ln_in_kernel) {
    float* rows = (float*)ln_rowbuf;
    if (!rows) return (int)hipErrorInvalidValue;
    ln_rowstats_kernel<<<(M + 255) / 256, 256, 0, stream>>>((const float*)ln_part, rows, M, K, ln_nparts, ln_pcols,
                                                           ln_eps);
    a.ln_row = rows;
  }
  return dispatch<false>(a, tile, 1, stream);
}

CSK_API int csk_gemm(void* C, const void* A, const void* W, const void* bias, const void* bias2d, const void* res,
                     int M, int N, int K, int lda, int ldb, int ldc, int ldr, int rows_per_b, int act, float out_scale,
                     void* gn_part, int tile, int ksplit, void* ws, hipStream_t stream) {
  return csk_gemm_ln(C, A, W, bias, bias2d, res, M, N, K, lda, ldb, ldc, ldr, rows_per_b, act, out_scale, gn_part,
                     nullptr, nullptr, 0, 0, 0.f, nullptr, nullptr, tile, ksplit, ws, stream);
}

// NHWC conv; xs / ys / rs: pixel strides (elements) of input / output / residual
// buffers (>= channel counts: lets dense blocks read and write channel slices of
// one concat buffer without copies).
// b2s: row stride of bias2d ([B][b2s], 0 -> Cout)
CSK_API int csk_conv2d_ex(void* Y, const void* X, const void* Wp, const void* bias, const void* bias2d, int b2s,
                          const void* res, int B, int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pt,
                          int pl, int Ho, int Wo, int up2x, int xs, int ys, int rs, int act, float out_scale, int dil,
                          void* gn_part, int tile, int ksplit, void* ws, hipStream_t stream) {
  if (Cin % 8 != 0 || xs % 8 != 0 || xs < Cin || (b2s != 0 && b2s < Cout)) return (int)hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)X; a.W = (const bf16_t*)Wp; a.C = (bf16_t*)Y;
  a.bias = (const bf16_t*)bias; a.bias2d = (const bf16_t*)bias2d; a.res = (const bf16_t*)res;
  a.M = B * Ho * Wo; a.N = Cout; a.K = kh * kw * Cin; a.lda = xs; a.ldb = kh * kw * Cin; a.ldc = ys;
  a.ldr = rs > 0 ? rs : ys; a.rows_per_b = Ho * Wo;
  a.act = act; a.out_scale = out_scale;
  a.H = H; a.Wd = W; a.Cin = Cin; a.Ho = Ho; a.Wo = Wo; a.kh = kh; a.kw = kw; a.stride = stride; a.pt = pt; a.pl = pl;
  a.up2x = up2x;
  a.dil = dil > 0 ? dil : 1;
  a.ldb2 = b2s > 0 ? b2s : Cout;
  a.ws = (float*)ws;
  a.gn_part = (float*)gn_part;
  a.a_end = a.A + ((size_t)B * H * W - 1) * xs + Cin;
  a.w_end = a.W + (size_t)(Cout - 1) * a.ldb + a.K;
  if (a.M == 0) return 0;
  return dispatch<true>(a, tile, ksplit, stream);
}

CSK_API int csk_conv2d(void* Y, const void* X, const void* Wp, const void* bias, const void* bias2d, const void* res,
                       int B, int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pt, int pl, int Ho, int Wo,
                       int up2x, int xs, int ys, int rs, int act, float out_scale, int dil, void* gn_part, int tile,
                       int ksplit, void* ws, hipStream_t stream) {
  return csk_conv2d_ex(Y, X, Wp, bias, bias2d, 0, res, B, H, W, Cin, Cout, kh, kw, stride, pt, pl, Ho, Wo, up2x, xs, ys,
                       rs, act, out_scale, dil, gn_part, tile, ksplit, ws, stream);
}

CSK_DEBUG_EXPORT(gemm)
