// 256-row, 8-wave phased MFMA GEMM / implicit-GEMM conv (LDS-DMA staging).
//
// Why a second main loop: the 128-row tiles of gemm_glds.hip move
// (BM + BN) * 64 * 2 bytes through L2 -> LDS per K-step for BM * BN * 128 FLOP,
// i.e. 1 byte per 64 FLOP at 128x128.  The per-CU LDS-DMA fill rate from L2
// (~70-80 GB/s, MI355X_MICROARCH.md "Indexed rows: gather into LDS") then caps
// a CU at ~5 TFLOP/s — about half its MFMA rate — which is what the PMC of the
// UNet step showed (profiles/pmc_unet_step_r1z.txt: MFMA busy 0.05-0.19, convs
// L2->LDS bound).  A 256x256 tile needs half the bytes per FLOP.  It only pays
// with a schedule that keeps the DMA in flight across barriers while every SIMD
// issues MFMAs back to back (cdna_hip_programming.md §5 "The 256² 8-phase
// template", T3/T4/T5): here each K-tile (BK = 64) is 4 phases of
//     ds_read the phase's fragments -> [issue next tile's A or B DMA] ->
//     s_barrier -> lgkmcnt(0) -> setprio(1) 16 MFMAs setprio(0) -> s_barrier
// with two LDS buffers: tile t+1's A is issued in phase 1 and its B in phase 2
// of tile t and retired by ONE vmcnt(0) at the end of phase 4 (>= 2 phases of
// MFMAs later), before the barrier after which phase 1 of t+1 reads it.
//
// Wave layout 2 (M) x 4 (N): a wave owns 128 x BN/4 outputs = 8 x NT 16x16
// accumulators.  Phase p multiplies A m-frags {0-3 | 4-7} with B n-frag halves:
//   p1: A0-3 x Bh0   p2: A0-3 x Bh1   p3: A4-7 x Bh1   p4: A4-7 x Bh0
// so each fragment is read from LDS once per K-tile (A0-3 and Bh0 in p1, Bh1 in
// p2, A4-7 in p3; p4 reads nothing).
//
// Staging is the FAST path of gemm_glds.hip only (K % 64 == 0; convs Cin % 64
// == 0): wave-uniform conv tap, one running source pointer per DMA row, invalid
// rows / padding taps pointed into the zero page.  Split-K writes fp32 partials
// reduced by splitk_reduce (gemm.hip).
#include "gemm_common.h"

template <int N>
__device__ __forceinline__ void p8_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void p8_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int BN, bool CONV>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(const GemmArgs args) {
  constexpr int BM = 256, WM = 2, WN = 4;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16, NH = NT / 2;
  static_assert(MT == 8 && NT % 2 == 0, "phase split needs 8 m-frags and an even n-frag count");
  constexpr int IA = BM / 64, IB = BN / 64;  // DMA instructions per thread per K-tile (8 waves x 8 rows each)
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int SMEM_MAIN = 2 * STAGE;
  constexpr int EP = 2;  // epilogue in two 128-row bands
  constexpr int SMEM_EPI = epi_smem_elems<BM, BN, EP>();
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int M = args.M, N = args.N;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int split = blockIdx.y;
  const int kbeg = split * args.kchunk;
  const int kend = args.ws ? min(args.K, kbeg + args.kchunk) : args.K;
  const int nk = (kend - kbeg) / BK;

  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;  // swizzled source chunk for this lane's lane-linear LDS slot
  const bf16_t* zero = args.zero + lchunk * 8;

  // ---- per-lane DMA source state: DMA instruction i of wave w stages rows (i*8 + w)*8 .. +8 ----
  // B (and GEMM A) rows of one lane are 64 rows apart: ONE running pointer plus a
  // wave-uniform stride (rows past the end are clamped to the last row — their
  // outputs are never stored), which keeps the 256-register budget spill-free.
  const int Hin = args.up2x ? 2 * args.H : args.H;
  const int Win = args.up2x ? 2 * args.Wd : args.Wd;
  // Ragged last tiles: a lane's rows r0 + 64 i past the end re-read its last valid
  // row (clamped count; that row's outputs are never stored).  Interior tiles —
  // all but the last row / column of tiles — skip the clamp (wave-uniform branch).
  const size_t bstride = (size_t)64 * args.ldb;
  const int rb0 = n0 + wid * 8 + lrow;
  const bool b_full = n0 + BN <= N;
  const int b_cnt = max(1, min(IB, (N - rb0 + 63) / 64));
  const bf16_t* fb = args.W + (size_t)min(rb0, N - 1) * args.ldb + kbeg + lchunk * 8;
  const bf16_t* fa0 = nullptr;
  size_t astride = 0;
  const bool a_full = m0 + BM <= M;
  int a_cnt = IA;
  // conv rows: sample base pixel + packed (oh*stride - pt, ow*stride - pl); an
  // out-of-range row gets an impossible ih so every tap reads the zero page
  int a_pix[CONV ? IA : 1], a_hw[CONV ? IA : 1];
  const bf16_t* fa[CONV ? IA : 1];
  if constexpr (CONV) {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int m = m0 + (i * 8 + wid) * 8 + lrow;
      const int mm = m < M ? m : 0;
      const int hw = args.Ho * args.Wo;
      const int b = mm / hw, r = mm - b * hw;
      const int oh = r / args.Wo, ow = r - oh * args.Wo;
      const int ihb = m < M ? oh * args.stride - args.pt : -30000;
      a_hw[i] = (ihb << 16) | ((ow * args.stride - args.pl) & 0xffff);
      a_pix[i] = b * args.H * args.Wd;
      fa[i] = zero;
    }
  } else {
    astride = (size_t)64 * args.lda;
    const int ra0 = m0 + wid * 8 + lrow;
    a_cnt = max(1, min(IA, (M - ra0 + 63) / 64));
    fa0 = args.A + (size_t)min(ra0, M - 1) * args.lda + kbeg + lchunk * 8;
  }
  int f_ky = 0, f_kx = 0, f_c = 0;
  auto set_rows = [&]() {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int ih = (a_hw[i] >> 16) + f_ky * args.dil, iw = (int)(short)(a_hw[i] & 0xffff) + f_kx * args.dil;
      const bool v = ih >= 0 && ih < Hin && iw >= 0 && iw < Win;
      const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
      fa[i] = v ? args.A + ((size_t)a_pix[i] + (size_t)sh * args.Wd + sw) * args.lda + lchunk * 8 : zero;
    }
  };
  if constexpr (CONV) {
    const int tap = kbeg / args.Cin;
    f_c = kbeg - tap * args.Cin;
    f_ky = tap / args.kw;
    f_kx = tap - f_ky * args.kw;
    set_rows();
  }

  auto issue_a = [&](int buf) {
    bf16_t* as = smem + buf * STAGE;
    if (CONV || a_full) {
#pragma unroll
      for (int i = 0; i < IA; ++i) {
        const bf16_t* src = CONV ? fa[CONV ? i : 0] + f_c : fa0 + i * astride;
        dma16<SITE_8P_A>(args, src, as + (i * 8 + wid) * 8 * BK, smem, SMEM_MAIN);
      }
    } else {
#pragma unroll
      for (int i = 0; i < IA; ++i)
        dma16<SITE_8P_A>(args, fa0 + min(i, a_cnt - 1) * astride, as + (i * 8 + wid) * 8 * BK, smem, SMEM_MAIN);
    }
    if constexpr (CONV) {
      f_c += BK;
      if (f_c == args.Cin) {
        f_c = 0;
        if (++f_kx == args.kw) { f_kx = 0; ++f_ky; }
        set_rows();
      }
    } else {
      fa0 += BK;
    }
  };
  auto issue_b = [&](int buf) {
    bf16_t* bs = smem + buf * STAGE + BM * BK;
    if (b_full) {
#pragma unroll
      for (int i = 0; i < IB; ++i)
        dma16<SITE_8P_B>(args, fb + i * bstride, bs + (i * 8 + wid) * 8 * BK, smem, SMEM_MAIN);
    } else {
#pragma unroll
      for (int i = 0; i < IB; ++i)
        dma16<SITE_8P_B>(args, fb + min(i, b_cnt - 1) * bstride, bs + (i * 8 + wid) * 8 * BK, smem, SMEM_MAIN);
    }
    fb += BK;
  };

  v4f acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  const int arow = wm * WTM + fr, brow = wn * WTN + fr;

  if (nk > 0) {
    issue_a(0);
    issue_b(0);
  }
  p8_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  v8s af[4][2], bf0[NH][2], bf1[NH][2];
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    const bf16_t* as = smem + cur * STAGE;
    const bf16_t* bs = as + BM * BK;
    // ---- phase 1: A m-frags 0-3, B half 0; stage next tile's A ----
#pragma unroll
    for (int j = 0; j < NH; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) bf0[j][ks] = *reinterpret_cast<const v8s*>(bs + swz(brow + j * 16, ks * 4 + fq));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) af[i][ks] = *reinterpret_cast<const v8s*>(as + swz(arow + i * 16, ks * 4 + fq));
    if (more) issue_a(cur ^ 1);
    __builtin_amdgcn_s_barrier();
    p8_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NH; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf0[j][ks], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 2: B half 1; stage next tile's B ----
#pragma unroll
    for (int j = 0; j < NH; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        bf1[j][ks] = *reinterpret_cast<const v8s*>(bs + swz(brow + (NH + j) * 16, ks * 4 + fq));
    if (more) issue_b(cur ^ 1);
    __builtin_amdgcn_s_barrier();
    p8_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NH; ++j)
          acc[i][NH + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf1[j][ks], acc[i][NH + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 3: A m-frags 4-7 x B half 1 ----
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        af[i][ks] = *reinterpret_cast<const v8s*>(as + swz(arow + (4 + i) * 16, ks * 4 + fq));
    __builtin_amdgcn_s_barrier();
    p8_lgkm0();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NH; ++j)
          acc[4 + i][NH + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf1[j][ks], acc[4 + i][NH + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_s_barrier();
    // ---- phase 4: A m-frags 4-7 x B half 0 (no LDS reads); retire the next tile ----
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NH; ++j)
          acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf0[j][ks], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    // the next tile's DMA (issued >= 2 phases ago) has landed for every wave once
    // each waited for its own and all passed this barrier
    p8_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
  }
  __syncthreads();
  gemm_epilogue<BM, BN, WM, WN, false, EP, 512>(args, acc, smem, m0, n0, split);
}

// ---------------------------------------------------------------------------
// 8-wave LDS-DMA RING kernel, 256 x BN tiles with BN = 160 (tile 33) / 128 (34).
//
// Why: the UNet's 64x64 level (M = 32768 rows, N = 320 output channels) is
// bound by the per-CU L2 -> LDS fill rate (~70 GB/s per CU at ~72 KB in
// flight, MI355X_MICROARCH.md "Indexed rows: gather into LDS").  Its best tile
// so far, 128x160 at two workgroups per CU, moves (128 + 160) / (128 * 160) =
// 0.0141 B per FLOP; 256x160 moves 0.0102 (-28 %) and keeps 256 tiles (one
// per CU, no padded columns at N = 320).  The 4-wave 256x160 tile 25 ran ONE
// wave per SIMD, so LDS fragment reads, DMA issue and MFMAs of that wave
// serialised; here 8 waves (2 per SIMD) share the ring: waves 4 (M) x 2 (N),
// 64 x 80 outputs per wave (4 x 5 fragments, row-layout accumulators for the
// SW epilogue), a 3-stage ring (3 x 52 KB = 156 KB: two stages, ~104 KB, in
// flight per CU while the third is consumed) with one raw barrier per K-step
// and a counted vmcnt, as gemm_glds.hip.
//
// DMA split: A = 32 eight-row groups -> 4 per wave; B = 20 groups -> 3 for
// waves 0-3 and 2 for waves 4-7, so the per-wave vmcnt is wave-dependent (a
// scalar branch on the SGPR wave id).  FAST staging only (K % 64 == 0, conv
// Cin % 64 == 0); no fused LN / row statistics / GEGLU (host falls back).
// ---------------------------------------------------------------------------
template <int BN, int S, bool CONV>
__global__ __launch_bounds__(512, 1) void gemm8r_kernel(const GemmArgs args) {
  constexpr int BM = 256, WM = 4, WN = 2, NW = 8;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int GA = BM / 8, GB = BN / 8;  // eight-row DMA groups
  static_assert(GA % NW == 0 && WTN % 16 == 0, "tile shape");
  constexpr int IA = GA / NW;
  constexpr int IBL = GB / NW, IBX = GB % NW;  // waves < IBX stage one group more
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int SMEM_MAIN = S * STAGE;
  constexpr int EP = epi_passes<BM, BN, WM>();
  constexpr int SMEM_EPI = epi_smem_elems<BM, BN, EP>();
  constexpr int SMEM = SMEM_MAIN > SMEM_EPI ? SMEM_MAIN : SMEM_EPI;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int M = args.M, N = args.N;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int split = blockIdx.y;
  const int kbeg = split * args.kchunk;
  const int kend = args.ws ? min(args.K, kbeg + args.kchunk) : args.K;
  const int nk = (kend - kbeg) / BK;
  const bool xb = wid < IBX;  // this wave stages IBL + 1 B groups

  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;
  const bf16_t* zero = args.zero + lchunk * 8;
  const int Hin = args.up2x ? 2 * args.H : args.H;
  const int Win = args.up2x ? 2 * args.Wd : args.Wd;

  // A: DMA instruction i of wave w stages group i * NW + w (rows 8 g .. 8 g + 7)
  const bf16_t* fa[IA];
  int a_ihb[CONV ? IA : 1], a_iwb[CONV ? IA : 1];
  size_t a_bbase[CONV ? IA : 1];
#pragma unroll
  for (int i = 0; i < IA; ++i) {
    const int m = m0 + (i * NW + wid) * 8 + lrow;
    const bool ok = m < M;
    if constexpr (CONV) {
      const int mm = ok ? m : 0;
      const int hw = args.Ho * args.Wo;
      const int b = mm / hw, r = mm - b * hw;
      const int oh = r / args.Wo, ow = r - oh * args.Wo;
      a_ihb[i] = ok ? oh * args.stride - args.pt : -30000;  // invalid row: every tap reads the zero page
      a_iwb[i] = ow * args.stride - args.pl;
      a_bbase[i] = (size_t)b * args.H * args.Wd;
      fa[i] = zero;
    } else {
      fa[i] = ok ? args.A + (size_t)m * args.lda + kbeg + lchunk * 8 : zero;
    }
  }
  const bf16_t* fb[IBL + 1];
#pragma unroll
  for (int i = 0; i <= IBL; ++i) {
    const int n = n0 + (i * NW + wid) * 8 + lrow;
    fb[i] = (n < N && (i < IBL || xb)) ? args.W + (size_t)n * args.ldb + kbeg + lchunk * 8 : zero;
  }
  int f_ky = 0, f_kx = 0, f_c = 0;
  auto set_rows = [&]() {
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const int ih = a_ihb[i] + f_ky * args.dil, iw = a_iwb[i] + f_kx * args.dil;
      const bool v = ih >= 0 && ih < Hin && iw >= 0 && iw < Win;
      const int sh = args.up2x ? (ih >> 1) : ih, sw = args.up2x ? (iw >> 1) : iw;
      fa[i] = v ? args.A + (a_bbase[i] + (size_t)sh * args.Wd + sw) * args.lda + lchunk * 8 : zero;
    }
  };
  if constexpr (CONV) {
    const int tap = kbeg / args.Cin;
    f_c = kbeg - tap * args.Cin;
    f_ky = tap / args.kw;
    f_kx = tap - f_ky * args.kw;
    set_rows();
  }

  auto issue = [&](int buf) {
    bf16_t* as = smem + buf * STAGE;
    bf16_t* bs = as + BM * BK;
#pragma unroll
    for (int i = 0; i < IA; ++i) {
      const bf16_t* src = CONV ? fa[i] + f_c : fa[i];
      dma16<SITE_8R_A>(args, src, as + (i * NW + wid) * 8 * BK, smem, SMEM_MAIN);
    }
#pragma unroll
    for (int i = 0; i < IBL; ++i) dma16<SITE_8R_B>(args, fb[i], bs + (i * NW + wid) * 8 * BK, smem, SMEM_MAIN);
    if (IBX > 0 && xb) dma16<SITE_8R_B>(args, fb[IBL], bs + (IBL * NW + wid) * 8 * BK, smem, SMEM_MAIN);
#pragma unroll
    for (int i = 0; i <= IBL; ++i) fb[i] += BK;  // the zero page is large enough for the running offset
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
  };

  v4f acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nk) issue(s);

  const int fr = lane & 15, fq = lane >> 4;
  constexpr int LA = IA + IBL;  // loads per stage of a wave without the extra B group
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt has landed once at most min(S-2, nk-1-kt) younger stages are in flight
    const int younger = min(S - 2, nk - 1 - kt);
    if constexpr (S == 3) {
      if (younger >= 1) {
        if (xb) p8_vmcnt<LA + 1>();
        else p8_vmcnt<LA>();
      } else {
        p8_vmcnt<0>();
      }
    } else {
      static_assert(S == 2, "ring depth");
      p8_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) issue((kt + S - 1) % S);
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
  gemm_epilogue<BM, BN, WM, WN, false, EP, 512, true>(args, acc, smem, m0, n0, split);
}

template <int BN, int S>
static int launch8r(const GemmArgs& a0, int ksplit, bool conv, hipStream_t s) {
  GemmArgs a = a0;
  a.gn_seg = gn_seg_for<256, BN, 4>();
  const int tiles = ((a.M + 255) / 256) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, ksplit);
  if (conv)
    gemm8r_kernel<BN, S, true><<<grid, 512, 0, s>>>(a);
  else
    gemm8r_kernel<BN, S, false><<<grid, 512, 0, s>>>(a);
  return (int)hipGetLastError();
}

template <int BN>
static int launch8p(const GemmArgs& a0, int ksplit, bool conv, hipStream_t s) {
  GemmArgs a = a0;
  {
    // GN segments: one per 128-row epilogue band (gemm_common.h gn_seg_for mirrors)
    const int seg = g_gn_fine ? 256 * BN / 256 : 256;
    a.gn_seg = seg > 128 ? 128 : seg;
  }
  const int tiles = ((a.M + 255) / 256) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles, ksplit);
  if (conv)
    gemm8p_kernel<BN, true><<<grid, 512, 0, s>>>(a);
  else
    gemm8p_kernel<BN, false><<<grid, 512, 0, s>>>(a);
  return (int)hipGetLastError();
}

// tile 31: 256x256, tile 32: 256x128 (phased), tiles 33 / 34: 256x160 / 256x128
// (8-wave 3-stage ring).  Returns hipErrorNotSupported when the shape needs a feature this
// kernel lacks (the caller falls back).
int csk_gemm8p_launch(const GemmArgs& a, int tile, int ksplit, bool conv, hipStream_t s) {
  const int span = ksplit > 1 ? a.kchunk : a.K;
  const bool fast = (conv ? (a.Cin % BK == 0) : true) && a.K % BK == 0 && span % BK == 0 &&
                    (size_t)(span + 2 * BK) * sizeof(bf16_t) <= (size_t)csk_zero_bytes() &&
                    (!conv || (size_t)(a.Cin + BK) * sizeof(bf16_t) <= (size_t)csk_zero_bytes());
  if (!fast || a.ln_part || a.row_part) return (int)hipErrorNotSupported;
  if (tile == 33 && a.act == ACT_GEGLU) return (int)hipErrorNotSupported;  // 80 columns per wave: no GEGLU pairing
  switch (tile) {
    case 33: return launch8r<160, 3>(a, ksplit, conv, s);
    case 34: return launch8r<128, 3>(a, ksplit, conv, s);  // 64 x 64 per wave: direct row-layout epilogue
    case 31: return launch8p<256>(a, ksplit, conv, s);
    case 32: return launch8p<128>(a, ksplit, conv, s);
    default: return (int)hipErrorInvalidValue;
  }
}

CSK_DEBUG_EXPORT(gemm8p)
