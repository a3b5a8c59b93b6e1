// Stream-K LDS-DMA GEMM with an in-kernel fixup (the UNet's
// mid-size projections, e.g. M2048 N1280 K1280 — 25 calls per SD2.1 step and
// 137 per SDXL step — and M8192 N640 K640).
//
// Why: at these shapes a tile grid is 1.25-2.5 rounds of 256 CUs, and the
// tuned one-tile-per-workgroup kernels (gemm_glds.hip) ran 350-370 TF/s in the
// step (profiles/callprof_unet_step_r5a.txt) against ~570 TF/s for their main
// loops alone (tools/tilebench.py --probe: 11.2-12 us of 14.3-16.5): the
// quantised last round and a per-tile epilogue that nothing overlaps.
//
// Structure (MI355X-first):
//   * OCC 256-thread workgroups per CU, persistent (grid = OCC x #CUs).  The work is
//     the flat list of (output tile, 64-deep K-step) units; worker w owns the
//     contiguous range [U w / G, U (w+1) / G): every CU gets the same number of
//     K-steps whatever the tile count (stream-K).
//   * The LDS-DMA ring (global_load_lds, the operand images and swizzle of
//     gemm_glds.hip) runs CONTINUOUSLY over the worker's units: the next tile's
//     first K-steps are in flight while this tile's epilogue runs.  The
//     epilogue stages through its own LDS region (not the ring) and uses raw
//     barriers (gemm_epilogue_ln<RAW>: __syncthreads' vmcnt(0) would drain the
//     ring).  Waits are counted (`s_waitcnt vmcnt`), barriers raw.
//   * A tile cut between workers is fixed up in-kernel (the persistent
//     attention's protocol, attn_fa.hip): a worker whose range STARTS inside a
//     tile (it runs that piece first) writes its fp32 accumulators to its
//     workspace slot and publishes a flag (agent-scope release); the worker
//     holding the tile's K-step 0 (it reaches the tile last) acquires, adds the
//     pieces in worker order (deterministic), runs the one epilogue (bias,
//     activation / GEGLU, residual, fused LN / GN / row statistics) and resets
//     the flags.  Bounded spins: a give-up counts into an error word.
//   * Residency: contributors never wait and run their piece first, owners
//     wait only for higher-numbered workers; G = OCC x #CUs with OCC
//     workgroups' LDS and registers per CU keeps every worker resident.
//
// MEASURED STANDING (profiles/tilebench_streamk_r5.txt): correct (tests/
// test_gemm_sk_gpu.py) but 1.8-3.4x SLOWER than the tuned gemm_glds tiles on
// every UNet shape (M2048 N1280 K1280: 30.7 us at two workgroups per CU vs
// 14.3 us for the 64x64 tile at four).  Each worker's K-step takes ~1 us: the
// steps are bound by the LDS-DMA latency under load, which the one-tile
// kernels hide with 3-5 resident workgroups per CU and this kernel (ring +
// separate epilogue region: 1-3 per CU) cannot; balancing K-steps does not
// buy that back.  No tuning-table entry selects tiles 40-43; they stay for
// A/B runs (tools/tilebench.py --tiles 40,41,42,43).
#include "gemm_common.h"

namespace {

constexpr int SK_MAX_ELEMS = 128 * 64;  // fp32 accumulators per worker slot (largest tile)
typedef unsigned int sk_u4 __attribute__((ext_vector_type(4)));

struct SkArgs {
  float* part;      // [G][BM * BN] partial accumulators
  unsigned* flags;  // [G] published partials (the owner resets them)
  unsigned* err;    // [1] spins that gave up
  int U;            // units = tiles * nk
  int nk;           // K-steps per tile
  int tiles_n;
};

template <int N>
__device__ __forceinline__ void sk_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void sk_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

}  // namespace

template <int BM, int BN, int WM, int WN, int S, int OCC>
__global__ __launch_bounds__(256, OCC) void gemm_sk_kernel(const GemmArgs args, const SkArgs sk) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int IA = BM / 32, IB = BN / 32;  // LDS-DMA instructions per wave per K-step (8 rows each)
  constexpr int LPG = IA + IB;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int SMEM_MAIN = S * STAGE;
  constexpr int EP = epi_passes<BM, BN, WM>();
  constexpr int SMEM_EPI = epi_smem_elems<BM, BN, EP>();
  static_assert(BM * BN <= SK_MAX_ELEMS, "workspace slot");
  static_assert(S >= 2 && S <= 4, "ring depth");
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM_MAIN + SMEM_EPI];
  bf16_t* const epi = smem + SMEM_MAIN;  // the epilogue's own region: the ring stays live across it

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int G = gridDim.x;
  const int w = xcd_remap(blockIdx.x, G);  // adjacent ranges (same / neighbouring tiles) share an XCD's L2
  const int U = sk.U, nk = sk.nk, tiles_n = sk.tiles_n;
  const int u0 = (int)((long long)U * w / G), u1 = (int)((long long)U * (w + 1) / G);
  if (u0 >= u1) return;
  const int M = args.M, N = args.N;

  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const bf16_t* zero = args.zero + lchunk * 8;

  // ---- DMA stream: unit d (tile d_t, K-step d_k) into ring slot d_s ----
  const bf16_t* fa[IA];
  const bf16_t* fb[IB];
  int d_t = u0 / nk, d_k = u0 - (u0 / nk) * nk, d_s = 0;
  auto set_ptrs = [&]() {  // row sources of tile d_t from K-step d_k
    const int m0 = (d_t / tiles_n) * BM, n0 = (d_t % tiles_n) * BN;
    const int ko = d_k * BK + lchunk * 8;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int m = m0 + (wid * IA + i) * 8 + lrow;
      fa[i] = m < M ? args.A + (size_t)m * args.lda + ko : zero + d_k * BK;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int n = n0 + (wid * IB + i) * 8 + lrow;
      fb[i] = n < N ? args.W + (size_t)n * args.ldb + ko : zero + d_k * BK;
    }
  };
  set_ptrs();
  auto issue = [&]() {
    bf16_t* as = smem + d_s * STAGE;
    bf16_t* bs = as + BM * BK;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      dma16<SITE_PERSIST_A>(args, fa[i], as + (wid * IA + i) * 8 * BK, smem, SMEM_MAIN);
      fa[i] += BK;
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      dma16<SITE_PERSIST_B>(args, fb[i], bs + (wid * IB + i) * 8 * BK, smem, SMEM_MAIN);
      fb[i] += BK;
    }
    d_s = d_s + 1 == S ? 0 : d_s + 1;
    if (++d_k == nk) {
      d_k = 0;
      ++d_t;
      set_ptrs();
    }
  };

  v4f acc[MT][NT];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();

  // ---- fixup ----
  // fence-free hand-off (cdna_hip_programming.md Guideline 16 R1; an agent
  // fence costs ~1.7 us): partials stored write-through (sc1) and drained
  // before the flag's atomic store; the owner polls relaxed, reads them sc1
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void*)sk.part, 0, G * SK_MAX_ELEMS * (int)sizeof(float), 0x00020000);
  auto publish = [&]() {  // contributor: this worker's first (partial) tile piece
    const int so = w * SK_MAX_ELEMS * (int)sizeof(float);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(sk_u4, make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3])), prs,
            ((i * NT + j) * 256 + tid) * 16, so, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave (also drains the ring: once per worker)
    sk_barrier();
    if (tid == 0) __hip_atomic_store(sk.flags + w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto merge = [&](int tile_end) {  // owner: every worker whose range starts inside the tile
    if (tid == 0) {
      for (int j = w + 1; j < G && (int)((long long)U * j / G) < tile_end; ++j) {
        unsigned spins = 0;
        while (__hip_atomic_load(sk.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 22)) {
            atomicAdd(sk.err, 1u);
            break;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only: the loads below are sc1)
    sk_barrier();
    for (int j = w + 1; j < G && (int)((long long)U * j / G) < tile_end; ++j) {
      const int so = j * SK_MAX_ELEMS * (int)sizeof(float);
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int jj = 0; jj < NT; ++jj) {
          const float4 x = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(prs, ((i * NT + jj) * 256 + tid) * 16, so, 16));
          acc[i][jj][0] += x.x;
          acc[i][jj][1] += x.y;
          acc[i][jj][2] += x.z;
          acc[i][jj][3] += x.w;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sk_barrier();  // every wave has read the slots before they are released
    if (tid == 0)
      for (int j = w + 1; j < G && (int)((long long)U * j / G) < tile_end; ++j)
        __hip_atomic_store(sk.flags + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto epilogue = [&](int tile) {
    const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
    float2 lnrow = make_float2(0.f, 0.f);
    float2 lnlane[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) lnlane[i] = make_float2(0.f, 1.f);
    bool lnl = false;
    if (args.ln_part && !args.ln_row) {
      ln_merge_tile<BM, MT, WTM>(args, m0, wm, reinterpret_cast<float*>(epi), lnlane, lnrow);
      lnl = true;
      sk_barrier();  // the merge scratch is the epilogue's staging region
    }
    if (!lnl) lnrow = ln_row_stats<BM>(args, m0);
    gemm_epilogue_ln<BM, BN, WM, WN, true, EP, 256, true>(args, acc, epi, m0, n0, 0, lnrow, lnlane, lnl);
    sk_barrier();  // the staging region is free for the next tile
  };

  // ---- prologue: S-1 units of operands in flight ----
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (u0 + s < u1) issue();

  const int fr = lane & 15, fq = lane >> 4;
  int seg = u0;            // first unit of the current tile piece
  int c_t = u0 / nk;       // its tile
  int c_k = u0 - c_t * nk; // K-step of unit u
  int c_s = 0;             // ring slot of unit u
  for (int u = u0; u < u1; ++u) {
    // unit u has landed once at most min(S-2, u1-1-u) younger units are in flight
    const int younger = min(S - 2, u1 - 1 - u);
    if constexpr (S >= 4) {
      if (younger >= 2) sk_vmcnt<2 * LPG>();
      else if (younger == 1) sk_vmcnt<LPG>();
      else sk_vmcnt<0>();
    } else if constexpr (S == 3) {
      if (younger >= 1) sk_vmcnt<LPG>();
      else sk_vmcnt<0>();
    } else {
      sk_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (u + S - 1 < u1) issue();
    const bf16_t* as = smem + c_s * STAGE;
    const bf16_t* bs = as + BM * BK;
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
        for (int j = 0; j < NT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    c_s = c_s + 1 == S ? 0 : c_s + 1;
    const bool tile_end = ++c_k == nk;
    if (!tile_end && u + 1 < u1) continue;
    // ---- the piece [seg, u] of tile c_t ends here ----
    if (seg != c_t * nk) {
      publish();  // (only ever this worker's first piece)
    } else {
      if (!tile_end) merge((c_t + 1) * nk);  // the tile's remaining K-steps are in later workers' slots
      epilogue(c_t);
    }
    zero_acc();
    seg = u + 1;
    c_t += 1;
    c_k = 0;
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static float* g_sk_part = nullptr;
static unsigned* g_sk_flags = nullptr;  // [workers] flags + [1] error counter
static int g_sk_workers = 0;  // slots: 3 workers per CU (the densest tile's residency)
static int g_sk_cus = 0;

// workspace of the fixup: allocated once per process from the library init
// (never inside a graph capture); flags are reset by their consumers
CSK_API int csk_gemm_sk_init() {
  if (g_sk_part) return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  g_sk_cus = cus > 0 ? cus : 256;
  g_sk_workers = 3 * g_sk_cus;
  hipError_t e = hipMalloc(&g_sk_part, (size_t)g_sk_workers * SK_MAX_ELEMS * sizeof(float));
  if (e != hipSuccess) return (int)e;
  e = hipMalloc(&g_sk_flags, (size_t)(g_sk_workers + 1) * sizeof(unsigned));
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(g_sk_flags, 0, (size_t)(g_sk_workers + 1) * sizeof(unsigned));
}

CSK_API int csk_gemm_sk_errors(unsigned* out) {
  if (!g_sk_flags) return (int)hipErrorNotInitialized;
  return (int)hipMemcpy(out, g_sk_flags + g_sk_workers, sizeof(unsigned), hipMemcpyDeviceToHost);
}

static int g_sk_max_workers = 0;  // tests: fewer workers (more cuts)
CSK_API int csk_set_gemm_sk_workers(int n) {
  g_sk_max_workers = n;
  return 0;
}

template <int BM, int BN, int WM, int WN, int S, int OCC>
static int launch_sk(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  a.gn_seg = gn_seg_for<BM, BN, WM>();
  a.ws = nullptr;
  a.kchunk = a.K;
  // the running K offset of an invalid row stays inside the zero page
  if (a.K % BK != 0 || (size_t)(a.K + 2 * BK) * sizeof(bf16_t) > ZERO_BYTES) return (int)hipErrorNotSupported;
  SkArgs sk;
  sk.tiles_n = (a.N + BN - 1) / BN;
  const long long tiles = (long long)((a.M + BM - 1) / BM) * sk.tiles_n;
  sk.nk = a.K / BK;
  const long long U = tiles * sk.nk;
  if (U >= (1ll << 30) || sk.nk < 1) return (int)hipErrorNotSupported;
  sk.U = (int)U;
  sk.part = g_sk_part;
  sk.flags = g_sk_flags;
  sk.err = g_sk_flags + g_sk_workers;
  // OCC workgroups per CU fit by LDS and registers: every worker is resident
  int G = OCC * g_sk_cus;
  if (g_sk_max_workers > 0 && g_sk_max_workers < G) G = g_sk_max_workers;
  if (G > U) G = (int)U;
  gemm_sk_kernel<BM, BN, WM, WN, S, OCC><<<G, 256, 0, s>>>(a, sk);
  return (int)hipGetLastError();
}

// tiles 40-43 (ops/tuning.py TILES): GEMMs only (K % 64 == 0), no split-K, no
// attention epilogue; hipErrorNotSupported lets the caller fall back
int csk_gemm_sk_launch(const GemmArgs& a, int tile, bool conv, hipStream_t s) {
  if (!g_sk_part) return (int)hipErrorNotInitialized;
  if (conv || a.attn_kv) return (int)hipErrorNotSupported;
  switch (tile) {
    case 40: return launch_sk<64, 128, 2, 2, 4, 1>(a, s);
    case 41: return launch_sk<128, 64, 4, 1, 4, 1>(a, s);
    case 42: return launch_sk<64, 64, 2, 2, 3, 2>(a, s);   // 67.5 KB: two workgroups per CU
    case 43: return launch_sk<64, 64, 2, 2, 2, 3>(a, s);   // 51.5 KB: three per CU
    default: return (int)hipErrorInvalidValue;
  }
}
