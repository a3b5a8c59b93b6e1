// LDS-DMA (global_load_lds, 16 B/lane) multi-stage MFMA GEMM / implicit-GEMM conv.
//
// Same math, operand layouts, swizzled LDS image and epilogue as gemm.hip, but
// the global->LDS staging is done by the LDS-DMA engine:
//   * no staging VGPRs and no ds_write instructions; the per-lane SOURCE
//     address carries the XOR swizzle (LDS destination is lane-linear: lane L
//     of a wave-instruction lands at base + 16 L, i.e. row L/8, slot L%8, so
//     it fetches chunk (L%8) ^ (L/8) of its row -> the same image as swz());
//   * conv padding / out-of-range rows read a 16-byte zero block in global
//     memory (DMA cannot zero-fill);
//   * S-stage ring (S = 2..4): stage kt+S-1 is issued right after the barrier
//     of step kt, so S-2 K-steps of loads stay in flight across every barrier;
//     the wait is a COUNTED `s_waitcnt vmcnt((S-2) * loads_per_stage)` and the
//     barrier is a raw s_barrier (never __syncthreads, whose vmcnt(0) would
//     drain the ring) — cdna_hip_programming.md §5 "Pipelining across barriers".
//   * FAST staging (Cin % 64 == 0 for convs, K % 64 == 0 for GEMMs — every UNet /
//     VAE layer): a K-step never straddles a conv tap, so the tap is wave-uniform
//     (SGPRs) and each lane keeps one source pointer per DMA row, recomputed only
//     when the tap changes (every Cin/64 K-steps).  A K-step then costs one 64-bit
//     pointer add per DMA instruction instead of the full im2col address + bounds
//     logic (the PMC run measured ~6 VALU per MFMA on the generic path).  Invalid
//     rows / padding taps point into a 128 KB zero page, large enough that the
//     running channel offset never leaves it, so no per-step select is needed.
#include "gemm_common.h"

#include <mutex>
#include <unordered_map>

static bf16_t* g_zero = nullptr;

template <int N>
__device__ __forceinline__ void vmcnt_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}


// waves per SIMD the register budget must allow: the 128x160 tile runs two
// workgroups per CU (its 74 KB ring), so <= 256 registers per lane; 64x160 too
// (unconstrained it took 271 and one workgroup per CU)
template <int BM, int BN>
constexpr int glds_min_waves() {
  return (BN == 160 && BM <= 128) ? 2 : 1;
}

template <int BM, int BN, int WM, int WN, int S, bool CONV, bool FAST, bool ATTN = false, bool FX = false>
__global__ __launch_bounds__(256, (glds_min_waves<BM, BN>())) void gemm_glds_kernel(const GemmArgs args) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int IA = BM / 32, IB = BN / 32;  // LDS-DMA instructions per wave per stage (8 rows each)
  constexpr int LPG = IA + IB;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int SMEM_MAIN = S * STAGE;
  constexpr int EP = epi_passes<BM, BN, WM>();
  constexpr int SMEM_EPI = epi_smem_elems<BM, BN, EP>();
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform -> SGPR address math
  const int wm = wid / WN, wn = wid % WN;
  const int M = args.M, N = args.N, K = args.K;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int split = blockIdx.y;
  const int kbeg = split * args.kchunk;
  const int kend = (args.ws || FX) ? min(K, kbeg + args.kchunk) : K;
  const int nk = (kend - kbeg + BK - 1) / BK;

  const int lrow = lane >> 3;                 // row within the 8-row DMA group
  const int lchunk = (lane & 7) ^ lrow;       // source chunk for this lane's LDS slot
  const bf16_t* zero = args.zero;

  // ---- per-lane source bookkeeping ----
  const bf16_t* a_ptr[IA];
  bool a_ok[IA];
  int a_ihb[IA], a_iwb[IA];
  size_t a_bbase[IA];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int m = m0 + (wid * IA + i) * 8 + lrow;
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
      a_ptr[i] = args.A + (size_t)(a_ok[i] ? m : 0) * args.lda + kbeg + lchunk * 8;
      a_ihb[i] = a_iwb[i] = 0;
      a_bbase[i] = 0;
    }
  }
  const bf16_t* b_ptr[IB];
  bool b_ok[IB];
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int n = n0 + (wid * IB + i) * 8 + lrow;
    b_ok[i] = n < N;
    b_ptr[i] = args.W + (size_t)(b_ok[i] ? n : 0) * args.ldb + kbeg + lchunk * 8;
  }
  int c_ci = 0, c_ky = 0, c_kx = 0;
  if constexpr (CONV) {
    const int k0 = kbeg + lchunk * 8;
    const int tap = k0 / args.Cin;
    c_ci = k0 - tap * args.Cin;
    c_ky = tap / args.kw;
    c_kx = tap - c_ky * args.kw;
  }
  const int Hin = args.up2x ? 2 * args.H : args.H;
  const int Win = args.up2x ? 2 * args.Wd : args.Wd;


  // ---- FAST path state: per-row running source pointers, uniform tap / channel offset ----
  const bf16_t* fa[IA];
  const bf16_t* fb[IB];
  int f_ky = 0, f_kx = 0, f_c = 0;
  auto set_rows = [&]() {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int ih = a_ihb[i] + f_ky * args.dil, iw = a_iwb[i] + f_kx * args.dil;
      const bool v = a_ok[i] && ih >= 0 && ih < Hin && iw >= 0 && iw < Win;
      const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
      fa[i] = v ? args.A + (a_bbase[i] + (size_t)sh * args.Wd + sw) * args.lda + lchunk * 8 : zero + lchunk * 8;
    }
  };
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < IB; ++i) fb[i] = b_ok[i] ? b_ptr[i] : zero + lchunk * 8;
    if constexpr (CONV) {
      const int tap = kbeg / args.Cin;
      f_c = kbeg - tap * args.Cin;
      f_ky = tap / args.kw;
      f_kx = tap - f_ky * args.kw;
      set_rows();
    } else {
#pragma unroll
      for (int i = 0; i < IA; ++i) fa[i] = a_ok[i] ? a_ptr[i] : zero + lchunk * 8;
    }
  }

  auto issue = [&](int kt, int buf) {
    bf16_t* as = smem + buf * STAGE;
    bf16_t* bs = as + BM * BK;
    if constexpr (FAST) {
      if (!(CONV && S == 2 && args.act == ACT_PROBE_NO_A && f_kx != 0)) {
#pragma unroll
        for (int i = 0; i < IA; ++i) {
          const bf16_t* src = CONV ? fa[i] + f_c : fa[i];
          dma16<SITE_GLDS_A>(args, src, as + (wid * IA + i) * 8 * BK, smem, SMEM);
        }
      }
#pragma unroll
      for (int i = 0; i < IB; ++i) {
        dma16<SITE_GLDS_B>(args, fb[i], bs + (wid * IB + i) * 8 * BK, smem, SMEM);
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
        for (int i = 0; i < IA; ++i) fa[i] += BK;
      }
      return;
    }
    const int k = kbeg + kt * BK + lchunk * 8;
    const bool kin = k < kend;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const bf16_t* src = zero;
      if constexpr (CONV) {
        const int ih = a_ihb[i] + c_ky * args.dil, iw = a_iwb[i] + c_kx * args.dil;
        if (kin && a_ok[i] && ih >= 0 && ih < Hin && iw >= 0 && iw < Win) {
          const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
          src = args.A + (a_bbase[i] + (size_t)sh * args.Wd + sw) * args.lda + c_ci;
        }
      } else {
        if (kin && a_ok[i]) src = a_ptr[i] + (size_t)kt * BK;
      }
      dma16<SITE_GLDS_A>(args, src, as + (wid * IA + i) * 8 * BK, smem, SMEM);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const bf16_t* src = (kin && b_ok[i]) ? b_ptr[i] + (size_t)kt * BK : zero;
      dma16<SITE_GLDS_B>(args, src, bs + (wid * IB + i) * 8 * BK, smem, SMEM);
    }
    if constexpr (CONV) {
      c_ci += BK;
      while (c_ci >= args.Cin) { c_ci -= args.Cin; if (++c_kx == args.kw) { c_kx = 0; ++c_ky; } }
    }
  };

  v4f acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s, s);
  // fused-LN row stats while the first stages land: merged here from the
  // producer's partials (no ln_rowstats launch), or precomputed per row
  float2 lnrow = make_float2(0.f, 0.f);
  float2 lnlane[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) lnlane[i] = make_float2(0.f, 1.f);
  bool lnl = false;
  if constexpr (!CONV) {
    if (args.ln_part && !args.ln_row) {
      ln_merge_tile<BM, MT, WTM>(args, m0, wm, reinterpret_cast<float*>(smem + (S - 1) * STAGE), lnlane, lnrow);
      lnl = true;
    }
  }
  if (!lnl) lnrow = ln_row_stats<BM>(args, m0);

  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once at most min(S-2, nk-1-kt) younger stages are in flight
    const int younger = min(S - 2, nk - 1 - kt);
    if constexpr (S >= 4) {
      if (younger >= 2) vmcnt_wait<2 * LPG>();
      else if (younger == 1) vmcnt_wait<LPG>();
      else vmcnt_wait<0>();
    } else if constexpr (S == 3) {
      if (younger >= 1) vmcnt_wait<LPG>();
      else vmcnt_wait<0>();
    } else {
      vmcnt_wait<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) issue(kt + S - 1, (kt + S - 1) % S);
    const bf16_t* as = smem + (kt % S) * STAGE;
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
  }
  __syncthreads();
  if constexpr (FX) {  // in-kernel split-K: only the tile's last-arriving split continues, with the full sum
    // (the flag borrows the drained ring's first word: no extra LDS, which would
    // cost the 32 KB / 80 KB tiles a workgroup slot per CU)
    if (!splitk_fixup<MT, NT, 256>(args, acc, t, split, reinterpret_cast<int*>(smem))) return;
  }
  if (args.act == ACT_PROBE_NO_EPILOGUE || args.act == ACT_PROBE_NO_A) {  // profiling probes: main loop only
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) sum += acc[i][j][0];
    if (sum == 1234.5f) args.C[threadIdx.x] = f2bf(sum);  // keeps the MFMAs alive
    return;
  }
  gemm_epilogue_ln<BM, BN, WM, WN, false, EP, 256, true, ATTN>(args, acc, smem, m0, n0, split, lnrow, lnlane, lnl);
}

// Counters of the in-kernel split-K fixup (one per output tile, zero between
// launches: the tile's last workgroup re-zeroes its own).  Launches on one
// stream never overlap, so every eager launch on a stream shares that stream's
// block; a launch captured into a hipGraph may replay beside other streams'
// work, so each captured launch gets counters of its own, bump-allocated from a
// ring that wraps only after 2^24 tiles (~2,000 UNet-step captures: two graph
// replays would have to run concurrently across that distance to collide).
static constexpr int FX_STREAM_CNT = 1 << 16;     // tiles per launch (M x N <= 2^28 outputs at 64x64)
static constexpr int FX_GRAPH_CNT = 1 << 24;      // 64 MB of counters for captured launches
static unsigned* g_fx_graph = nullptr;
static long long g_fx_graph_used = 0;
static std::mutex g_fx_mu;
static std::unordered_map<hipStream_t, unsigned*> g_fx_stream;

static unsigned* fixup_counters(hipStream_t s, int tiles) {
  if (tiles > FX_STREAM_CNT) return nullptr;
  std::lock_guard<std::mutex> lk(g_fx_mu);
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess) return nullptr;
  if (st != hipStreamCaptureStatusNone) {
    if (!g_fx_graph) return nullptr;
    if (g_fx_graph_used + tiles > FX_GRAPH_CNT) g_fx_graph_used = 0;
    unsigned* p = g_fx_graph + g_fx_graph_used;
    g_fx_graph_used += (tiles + 63) / 64 * 64;
    return p;
  }
  auto it = g_fx_stream.find(s);
  if (it != g_fx_stream.end()) return it->second;
  unsigned* p = nullptr;
  if (hipMalloc(&p, FX_STREAM_CNT * sizeof(unsigned)) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, FX_STREAM_CNT * sizeof(unsigned)) != hipSuccess) return nullptr;
  g_fx_stream[s] = p;
  return p;
}

template <int BM, int BN, int WM, int WN, int S>
static int launch_glds(const GemmArgs& a0, int ksplit, bool conv, hipStream_t s) {
  GemmArgs a = a0;
  a.gn_seg = gn_seg_for<BM, BN, WM>();
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  // FAST staging: K-steps never straddle a tap / the K tail, and every running
  // offset stays inside the zero page
  const int span = ksplit > 1 ? a.kchunk : a.K;
  if (a.fx_ws) {  // in-kernel split-K fixup: a zeroed counter per output tile
    a.fx_cnt = fixup_counters(s, tiles);
    if (!a.fx_cnt) return (int)hipErrorOutOfMemory;
    a.fx_split = ksplit;
    a.ws = nullptr;
  }
  const bool fast = (conv ? (a.Cin % BK == 0) : (a.K % BK == 0)) && a.K % BK == 0 &&
                    (size_t)(span + 2 * BK) * sizeof(bf16_t) <= ZERO_BYTES &&
                    (!conv || (size_t)(a.Cin + BK) * sizeof(bf16_t) <= ZERO_BYTES);
  dim3 grid(tiles, ksplit);
  if (a.attn_kv) {  // the query projection with the attention epilogue (csk_gemm_ln_attn)
    if constexpr (BM == 128 && BN == 64 && WM == 4 && WN == 1) {
      if (conv || !fast || ksplit != 1) return (int)hipErrorInvalidValue;
      gemm_glds_kernel<BM, BN, WM, WN, S, false, true, true><<<grid, 256, 0, s>>>(a);
      return (int)hipGetLastError();
    } else {
      return (int)hipErrorInvalidValue;
    }
  }
  if (a.fx_cnt) {  // a separate instance: the unsplit kernels keep their code (measured 1 % of the step)
    if (!fast) return (int)hipErrorInvalidValue;
    if (conv) gemm_glds_kernel<BM, BN, WM, WN, S, true, true, false, true><<<grid, 256, 0, s>>>(a);
    else gemm_glds_kernel<BM, BN, WM, WN, S, false, true, false, true><<<grid, 256, 0, s>>>(a);
    return (int)hipGetLastError();
  }
  if (conv) {
    if (fast) gemm_glds_kernel<BM, BN, WM, WN, S, true, true><<<grid, 256, 0, s>>>(a);
    else gemm_glds_kernel<BM, BN, WM, WN, S, true, false><<<grid, 256, 0, s>>>(a);
  } else {
    if (fast) gemm_glds_kernel<BM, BN, WM, WN, S, false, true><<<grid, 256, 0, s>>>(a);
    else gemm_glds_kernel<BM, BN, WM, WN, S, false, false><<<grid, 256, 0, s>>>(a);
  }
  return (int)hipGetLastError();
}

const bf16_t* csk_zero_ptr() { return g_zero; }
int csk_zero_bytes() { return ZERO_BYTES; }

extern "C" int csk_attn_fa_init();  // attn_fa.hip: the stream-K attention's merge workspace

CSK_API int csk_init() {
  if (g_zero) return 0;
  hipError_t e = hipMalloc(&g_zero, ZERO_BYTES);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(g_zero, 0, ZERO_BYTES);
  if (e != hipSuccess) return (int)e;
  e = hipMalloc(&g_fx_graph, (size_t)FX_GRAPH_CNT * sizeof(unsigned));
  if (e != hipSuccess) return (int)e;
  e = hipMemset(g_fx_graph, 0, (size_t)FX_GRAPH_CNT * sizeof(unsigned));
  if (e != hipSuccess) return (int)e;
  return csk_attn_fa_init();
}

int csk_gemm_glds_launch(const GemmArgs& a0, int tile, int ksplit, bool conv, hipStream_t s) {
  if (!g_zero) return (int)hipErrorNotInitialized;
  GemmArgs a = a0;
  a.zero = g_zero;
  // GEGLU pairs 16-column (hidden, gate) tiles inside one wave's columns: every
  // tile below has a per-wave width (BN / WN) that is a multiple of 32
  // 256x160: 80 columns per wave (odd 16-column tile count: no GEGLU pairing),
  // 20 vectors per output row (no power-of-two row-statistics butterfly)
  if ((tile == 25 || tile == 26) && (a.act == ACT_GEGLU || a.ln_part || a.row_part)) tile = 11;
  if (tile == 36 && (a.act == ACT_GEGLU || a.ln_part || a.row_part)) tile = 13;
  switch (tile) {
    case 11: return launch_glds<128, 128, 2, 2, 2>(a, ksplit, conv, s);
    case 12: return launch_glds<128, 64, 4, 1, 3>(a, ksplit, conv, s);
    case 13: return launch_glds<64, 128, 2, 2, 3>(a, ksplit, conv, s);
    case 14: return launch_glds<64, 64, 2, 2, 4>(a, ksplit, conv, s);
    case 15: return launch_glds<128, 128, 2, 2, 3>(a, ksplit, conv, s);
    case 16: return launch_glds<128, 32, 4, 1, 4>(a, ksplit, conv, s);
    case 17: return launch_glds<128, 64, 2, 2, 3>(a, ksplit, conv, s);
    // small-LDS 2-stage variants: 3-5 workgroups per CU, for short-K (K = 320..640)
    // GEMMs that are bound by memory latency rather than by the MFMA pipe
    case 18: return launch_glds<64, 64, 2, 2, 2>(a, ksplit, conv, s);
    case 19: return launch_glds<128, 64, 4, 1, 2>(a, ksplit, conv, s);
    case 20: return launch_glds<64, 128, 2, 2, 2>(a, ksplit, conv, s);
    // one 256x160 workgroup per CU, 3-stage ring (156 KB): 2.3x fewer L2->LDS
    // bytes per output than 128x64 for the N = 320 / 1280 layers of the 64x64
    // level, whose convs are bound by the LDS-DMA fill rate (~80 GB/s per CU)
    case 25: return launch_glds<256, 160, 2, 2, 3>(a, ksplit, conv, s);
    // 128x160, 2-stage (74 KB): two workgroups per CU, 1.66x fewer L2->LDS bytes
    // per output than 128x64 and no padded columns at N = 320 (2 x 160)
    case 26: return launch_glds<128, 160, 2, 2, 2>(a, ksplit, conv, s);
    // deep rings for the latency-bound low-M / long-K shapes (8x8 and 16x16
    // levels: M = 512 / 2048 rows, K up to 23040): three K-steps of loads in
    // flight per workgroup instead of one
    case 27: return launch_glds<128, 128, 2, 2, 4>(a, ksplit, conv, s);
    case 28: return launch_glds<64, 128, 2, 2, 4>(a, ksplit, conv, s);
    case 29: return launch_glds<128, 64, 2, 2, 4>(a, ksplit, conv, s);
    // 64x160, 2-stage, two workgroups per CU: fewest L2->LDS bytes per output
    // among the 64-row tiles; wins M8192 N640 K2560 in isolation (36.5 vs 39.9 us).
    // Its 3-stage sibling (one workgroup per CU: exactly 256 tiles at M2048 N1280)
    // was slower than 64x64 there (19.7 vs 14.8 us, profiles/tilebench_64x160_r6m.txt)
    case 36: return launch_glds<64, 160, 2, 2, 2>(a, ksplit, conv, s);
    // (deep rings, S = 5..8 at 64x64 / 128x64 / 64x128, were measured and dropped:
    // never faster in the step or in graph-timed isolation, profiles/tilebench_graph_deep_r5.txt)
    default: return (int)hipErrorInvalidValue;
  }
}

// CSK_DEBUG positive control: one wave records a deliberate violation (site 99,
// value v, limit 3) so a test can prove the record path works end to end
#ifdef CSK_DEBUG
__global__ void csk_debug_selftest_kernel(int v) { CSK_DCHECK(v < 0, 99, v, 3); }
#endif
CSK_API int csk_debug_selftest(int v, hipStream_t s) {
#ifdef CSK_DEBUG
  csk_debug_selftest_kernel<<<1, 64, 0, s>>>(v);
  return (int)hipGetLastError();
#else
  (void)v;
  (void)s;
  return (int)hipErrorNotSupported;
#endif
}

CSK_DEBUG_EXPORT(gemm_glds)
