// Sliced-K GEMM for small M (tile 44: 64 x 64 outputs per 512-thread
// workgroup): the UNet projections at CFG batch 2 and the 8x8 level
// (M = 128 .. 2048 rows, K = 640 .. 5120; SURVEY K4 / K9, the batch-1 job the
// hive sends most).
//
// Why: at M <= 512 a 64 x 64 tile grid has 40-160 workgroups and each runs its
// K-steps one after another: the step time is the length of that dependent
// chain (LDS-DMA latency per K-step), not bandwidth or MFMA rate — M128 N1280
// K1280 took 11.2 us, M512 N1280 K1280 11.8 us in the CFG-2 step
// (profiles/callprof_unet_step_b2_r5c.txt), 2-4x their HBM / MFMA floors.
// Split-K cuts the chain but pays an fp32 partial round trip and a second
// launch (the tuner rejects it at these shapes).
//
// Structure: the 8 waves of a workgroup split the K-steps of ONE output tile
// (wave w takes steps w, w + 8, ...), each loading its A / W fragments straight
// from global memory into registers (16-byte loads in the MFMA operand layout,
// two K-steps in flight per wave) and accumulating the full 64 x 64 tile on
// v_mfma_f32_16x16x32_bf16; the eight partial tiles are summed through LDS
// (row stride padded to 68 floats: conflict-free float4 writes) and every
// thread finishes 8 consecutive outputs of one row: bias, activation, scale,
// residual, one 16-byte store.  The K chain per workgroup is nk / 8 steps and
// nothing leaves the chip but the result.
//
// MEASURED STANDING (profiles/tilebench_slk_fixup_r5.txt): slower than the
// 64x64 LDS-DMA tile everywhere (M128 N1280 K1280 13.0 vs 9.2 us, M512 N1280
// K5120 39.0 vs 24.4 us).  Splitting K inside one CU does not help: these
// grids are bound by the per-CU L2 -> CU read rate (~20-70 GB/s per CU,
// MI355X_MICROARCH.md "Indexed rows"), not by the K-step chain, so the
// winning move is spreading K over MORE CUs -- the in-kernel split-K fixup of
// the LDS-DMA tiles (gemm_common.h splitk_fixup, tuning split < 0).  Kept for
// A/B; the tuner does not propose tile 44.
#include "gemm_common.h"

namespace {
constexpr int SLK_BM = 64, SLK_BN = 64, SLK_WAVES = 8;
constexpr int SLK_LDC = 68;  // padded LDS row stride (floats)
unsigned long long g_slk_launches = 0;  // host-side count (tests check the kernel ran)
}  // namespace

__global__ __launch_bounds__(512, 1) void gemm_slk_kernel(const GemmArgs args) {
  __shared__ __attribute__((aligned(16))) float red[SLK_WAVES * SLK_BM * SLK_LDC];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = args.M, N = args.N, K = args.K;
  const int tiles_n = (N + SLK_BN - 1) / SLK_BN, tiles_m = (M + SLK_BM - 1) / SLK_BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * SLK_BM, n0 = (t % tiles_n) * SLK_BN;
  const int nk = K / BK;
  const int fr = lane & 15, fq = lane >> 4;

  // per-lane operand row pointers (rows past the end re-read the last row: never stored)
  const bf16_t* ap[4];
  const bf16_t* bp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ap[i] = args.A + (size_t)min(m0 + i * 16 + fr, M - 1) * args.lda + fq * 8;
    bp[i] = args.W + (size_t)min(n0 + i * 16 + fr, N - 1) * args.ldb + fq * 8;
  }

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  auto mma_step = [&](const v8s (&af)[4][2], const v8s (&bf)[4][2]) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][h], af[i][h], acc[i][j], 0, 0, 0);
  };
  // two K-steps (this wave's s and s + 8) in flight per round
  for (int s = wv; s < nk; s += 2 * SLK_WAVES) {
    const int k0 = s * BK;
    v8s a0[4][2], b0[4][2], a1[4][2], b1[4][2];
    const bool two = s + SLK_WAVES < nk;
    const int k1 = k0 + SLK_WAVES * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        a0[i][h] = *reinterpret_cast<const v8s*>(ap[i] + k0 + h * 32);
        b0[i][h] = *reinterpret_cast<const v8s*>(bp[i] + k0 + h * 32);
      }
    if (two) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          a1[i][h] = *reinterpret_cast<const v8s*>(ap[i] + k1 + h * 32);
          b1[i][h] = *reinterpret_cast<const v8s*>(bp[i] + k1 + h * 32);
        }
    }
    mma_step(a0, b0);
    if (two) mma_step(a1, b1);
  }

  // ---- sum the eight wave partials through LDS ----
  float* mine = red + wv * SLK_BM * SLK_LDC;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<float4*>(mine + (i * 16 + fr) * SLK_LDC + j * 16 + fq * 4) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
  __syncthreads();
  const int row = tid >> 3, c8 = (tid & 7) * 8;  // this thread's 8 outputs
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = 0.f;
#pragma unroll
  for (int w = 0; w < SLK_WAVES; ++w) {
    const float4 x = *reinterpret_cast<const float4*>(red + (w * SLK_BM + row) * SLK_LDC + c8);
    const float4 y = *reinterpret_cast<const float4*>(red + (w * SLK_BM + row) * SLK_LDC + c8 + 4);
    v[0] += x.x; v[1] += x.y; v[2] += x.z; v[3] += x.w;
    v[4] += y.x; v[5] += y.y; v[6] += y.z; v[7] += y.w;
  }
  const int m = m0 + row, n = n0 + c8;
  if (m >= M || n >= N) return;
  if (args.bias) {
    float b[8];
    unpack8(*reinterpret_cast<const uint4*>(args.bias + n), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += b[e];
  }
  if (args.bias2d) {
    float b[8];
    unpack8(*reinterpret_cast<const uint4*>(args.bias2d + (size_t)(m / args.rows_per_b) * args.ldb2 + n), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += b[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = apply_act(args.act, v[e]) * args.out_scale;
  if (args.res) {
    float r[8];
    unpack8(*reinterpret_cast<const uint4*>(args.res + (size_t)m * args.ldr + n), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
  *reinterpret_cast<uint4*>(args.C + (size_t)m * args.ldc + n) = pack8(v);
}

// tile 44: GEMMs with K % 64 == 0, N % 8 == 0, 16-byte aligned rows, and an
// epilogue of bias / per-sample bias / pointwise activation / scale / residual
// (no GEGLU, fused LN / GN / row statistics or split-K: hipErrorNotSupported
// lets the caller fall back)
int csk_gemm_slk_launch(const GemmArgs& a, bool conv, hipStream_t s) {
  if (conv || a.attn_kv || a.ws || a.act == ACT_GEGLU || a.act == ACT_TANH || a.act == ACT_ELU ||
      a.act == ACT_GELU_TANH || a.ln_part || a.ln_row ||
      a.row_part || a.gn_part || a.act >= 97)
    return (int)hipErrorNotSupported;
  if (a.K % BK != 0 || a.N % 8 != 0 || a.lda % 8 != 0 || a.ldb % 8 != 0 || a.ldc % 8 != 0 ||
      (a.res && a.ldr % 8 != 0) || (a.bias2d && a.ldb2 % 8 != 0) || (((size_t)a.A | (size_t)a.W | (size_t)a.C) & 15) ||
      (a.bias && (((size_t)a.bias) & 15)) || (a.res && (((size_t)a.res) & 15)) ||
      (a.bias2d && (((size_t)a.bias2d) & 15)))
    return (int)hipErrorNotSupported;
  const int tiles = ((a.M + SLK_BM - 1) / SLK_BM) * ((a.N + SLK_BN - 1) / SLK_BN);
  gemm_slk_kernel<<<tiles, 512, 0, s>>>(a);
  ++g_slk_launches;
  return (int)hipGetLastError();
}

CSK_API int csk_gemm_slk_launches(unsigned long long* out) {
  *out = g_slk_launches;
  return 0;
}
