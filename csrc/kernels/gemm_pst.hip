// Persistent LDS-DMA GEMM with a ring that runs across output tiles (tiles 50-53).
//
// Why: in the short-K GEMMs of the UNet's 64x64 / 32x32 levels (K = 320 / 640,
// 5-10 K-steps per tile) the epilogue is half the kernel: M32768 N320 K320 on
// the 128x64 tile takes 18.3 us with its epilogue and 10.2 us without it
// (graph-timed, profiles/cache_policy_ab_r5.txt), while writing the 21 MB
// output alone takes ~5.5 us (tools/store_pattern_bench.hip).  A one-tile
// workgroup ends with its stores and the next workgroup starts with an empty
// ring, so each tile pays the store drain and the first loads' latency back to
// back.  Here one workgroup per slot walks the tiles t = b, b + G, ... (G a
// multiple of 8: every tile of a workgroup stays on its XCD, then xcd_remap
// for L2 locality) and the ring never drains: the DMA of the next tile's first
// S-1 K-steps is issued during the current tile's last K-steps, so it is in
// flight while the epilogue computes and stores.
//
// Counted waits stay correct with the epilogue's loads / stores between the
// DMA groups: loads retire in issue order, so "at most (S-2) * LPG ops
// outstanding" still implies the needed stage has landed (younger epilogue
// ops only make the wait longer).  The epilogue is the direct row-vector one
// of gemm_common.h and must not touch LDS (the ring is live): the launcher
// admits only shapes whose epilogue takes that path (no GN / LN / row
// statistics, aligned vectors), others get hipErrorNotSupported.
//
// MEASURED STANDING (profiles/tilebench_graph_pst_r5.txt, graph-timed): slower
// than the one-tile kernels everywhere — M32768 N320 K320 22.1 us (128x64,
// 3 workgroups per CU) / 25.9 us (3-stage, 2 per CU) vs 19.2 us for tile 19;
// M8192 N640 K640 20.1 vs 15.3 us.  The one-tile grid already overlaps one
// workgroup's epilogue with the others' main loops (3-5 resident per CU) and
// its dynamic dispatch balances better than the static tile walk, which also
// drains the epilogue's stores at the next counted wait.  Kept for A/B; the
// tuner does not propose tiles 50-53.
#include "gemm_common.h"

namespace {
int g_pst_cus = 0;
unsigned long long g_pst_launches = 0;
}  // namespace

template <int BM, int BN, int WM, int WN, int S>
__global__ __launch_bounds__(256, 3) void gemm_pst_kernel(const GemmArgs args, int tiles) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int IA = BM / 32, IB = BN / 32;  // LDS-DMA instructions per wave per stage
  constexpr int LPG = IA + IB;
  constexpr int STAGE = (BM + BN) * BK;
  __shared__ __attribute__((aligned(16))) bf16_t smem[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int M = args.M, N = args.N;
  const int tiles_n = (N + BN - 1) / BN;
  const int nk = args.K / BK;
  const int G = gridDim.x, b = blockIdx.x;
  const int mine = b < tiles ? (tiles - 1 - b) / G + 1 : 0;  // tiles of this workgroup
  const int T = mine * nk;                                   // its K-steps over all of them
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  const bf16_t* zero = args.zero + lchunk * 8;

  auto tile_of = [&](int j) { return xcd_remap(b + j * G, tiles); };
  // stage g = (tile j, K-step k) into ring slot g % S
  auto issue = [&](int g) {
    const int j = g / nk, k = g - j * nk;
    const int t = tile_of(j);
    const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
    bf16_t* as = smem + (g % S) * STAGE;
    bf16_t* bs = as + BM * BK;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int m = m0 + (wid * IA + i) * 8 + lrow;
      const bf16_t* src = m < M ? args.A + (size_t)m * args.lda + k * BK + lchunk * 8 : zero;
      dma16<SITE_GLDS_A>(args, src, as + (wid * IA + i) * 8 * BK, smem, S * STAGE);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int n = n0 + (wid * IB + i) * 8 + lrow;
      const bf16_t* src = n < N ? args.W + (size_t)n * args.ldb + k * BK + lchunk * 8 : zero;
      dma16<SITE_GLDS_B>(args, src, bs + (wid * IB + i) * 8 * BK, smem, S * STAGE);
    }
  };

  v4f acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  float2 lnlane[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) lnlane[i] = make_float2(0.f, 1.f);

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < T) issue(s);
  const int fr = lane & 15, fq = lane >> 4;
  for (int g = 0; g < T; ++g) {
    const int younger = min(S - 2, T - 1 - g);
    if constexpr (S >= 4) {
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPG) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPG) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if constexpr (S == 3) {
      if (younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPG) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    if (g + S - 1 < T) issue(g + S - 1);
    const bf16_t* as = smem + (g % S) * STAGE;
    const bf16_t* bs = as + BM * BK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8s af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i) af[i] = *reinterpret_cast<const v8s*>(as + swz(wm * WTM + i * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int j = 0; j < NT; ++j) bfr[j] = *reinterpret_cast<const v8s*>(bs + swz(wn * WTN + j * 16 + fr, ks * 4 + fq));
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    const int jt = g / nk;
    if (g - jt * nk == nk - 1) {  // last K-step of tile jt: epilogue (direct path: registers -> global only)
      const int t = tile_of(jt);
      const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
      gemm_epilogue_ln<BM, BN, WM, WN, false, 1, 256, true>(args, acc, smem, m0, n0, 0, make_float2(0.f, 0.f),
                                                              lnlane, false);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    }
  }
}

template <int BM, int BN, int WM, int WN, int S>
static int launch_pst(const GemmArgs& a0, hipStream_t s) {
  constexpr int NT = BN / WN / 16;
  GemmArgs a = a0;
  const bool geglu = a.act == ACT_GEGLU;
  // the direct epilogue's conditions (gemm_common.h gemm_epilogue_ln `direct`), so it never stages through LDS
  const bool ok = a.K % BK == 0 && a.K > 0 && !a.ws && !a.gn_part && !a.ln_part && !a.ln_row && !a.row_part &&
                  !a.attn_kv && a.act < 97 && (!geglu || (NT % 4 == 0 && a.N % 16 == 0)) && a.N % 8 == 0 &&
                  a.ldc % 8 == 0 && a.lda % 8 == 0 && a.ldb % 8 == 0 && ((size_t)a.C & 15) == 0 &&
                  ((size_t)a.A & 15) == 0 && ((size_t)a.W & 15) == 0 && (!a.bias || ((size_t)a.bias & 15) == 0) &&
                  (!a.bias2d || (a.ldb2 % 8 == 0 && ((size_t)a.bias2d & 15) == 0)) &&
                  (!a.res || (a.ldr % 8 == 0 && ((size_t)a.res & 15) == 0)) && NT % 2 == 0;
  if (!ok) return (int)hipErrorNotSupported;
  a.kchunk = a.K;
  a.gn_seg = 0;
  const long long tiles = (long long)((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  if (tiles >= (1ll << 30) || (long long)a.K / BK * tiles >= (1ll << 31)) return (int)hipErrorNotSupported;
  constexpr int LDS = S * (BM + BN) * BK * 2;
  const int occ = LDS * 4 <= 160 * 1024 ? 4 : LDS * 3 <= 160 * 1024 ? 3 : LDS * 2 <= 160 * 1024 ? 2 : 1;
  int G = (g_pst_cus > 0 ? g_pst_cus : 256) * occ;  // a multiple of 8: a workgroup's tiles share its XCD
  if (G > tiles) G = (int)((tiles + 7) / 8 * 8);
  gemm_pst_kernel<BM, BN, WM, WN, S><<<G, 256, 0, s>>>(a, (int)tiles);
  ++g_pst_launches;
  return (int)hipGetLastError();
}

// tiles 50-53 (ops/tuning.py TILES); the caller falls back to the same-geometry
// one-tile LDS-DMA tile on hipErrorNotSupported
int csk_gemm_pst_launch(const GemmArgs& a, int tile, bool conv, hipStream_t s) {
  if (conv) return (int)hipErrorNotSupported;
  if (g_pst_cus == 0) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      g_pst_cus = cus;
  }
  switch (tile) {
    case 50: return launch_pst<128, 64, 4, 1, 2>(a, s);  // 48 KB: 3 per CU
    case 51: return launch_pst<64, 64, 2, 2, 2>(a, s);   // 32 KB: 4 per CU
    case 52: return launch_pst<128, 128, 2, 2, 2>(a, s);
    case 53: return launch_pst<64, 128, 2, 2, 3>(a, s);
    default: return (int)hipErrorInvalidValue;
  }
}

CSK_API int csk_gemm_pst_launches(unsigned long long* out) {
  *out = g_pst_launches;
  return 0;
}
