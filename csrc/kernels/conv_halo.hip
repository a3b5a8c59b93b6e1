// Halo-tiled 3x3 stride-1 convolution with an optional GroupNorm(+SiLU)
// prologue on its input (SURVEY K1 + K6; the ResNet norm1 -> conv1 and
// norm2 -> conv2 pairs of every UNet block, reference call site
// swarm/diffusion/diffusion_func.py:96).
//
// The implicit-GEMM conv (gemm_glds.hip) stages an A tile per K-step per tap:
// each input pixel crosses L2 -> LDS nine times, and the UNet's long-K convs
// are bound by that fill (~33 B/clk/CU measured, README).  Here a workgroup
// owns R whole image rows (BM = R * W output pixels of one sample) and keeps
// the (R + 2) x (W + 2) input halo of one 64-channel chunk in LDS: the nine
// taps read it at a pixel offset (ky (W + 2) + kx), so A crosses L2 -> LDS
// ~(R+2)(W+2)/(R W) times instead of 9 and only the weights stream per tap.
//
// GroupNorm fusion: the producer's epilogue emitted GN statistics partials, a
// tiny finalize turned them into (mean, rstd) per (sample, group); here each
// chunk's halo is normalised (+ SiLU) IN LDS once, after it lands — once per
// input element per column tile instead of nine times per element in an A
// operand path — and the separate GroupNorm apply pass (a full read + write of
// the activation) disappears.  Padding pixels stay zero (the conv pads the
// normalised tensor).
//
// Pipeline (one workgroup per CU, 4 waves, wave tile BM/2 x BN/2 on
// v_mfma_f32_16x16x32_bf16, B·A order so the row-layout epilogue of
// gemm_common.h applies): the A halo is double-buffered (chunk c + 1 lands
// during chunk c's nine taps), the weights run through a 4-stage LDS-DMA ring
// over the (chunk, tap) steps (three steps in flight: one workgroup per CU has
// no second workgroup to cover a load wait) with one raw barrier per step and
// exact counted vmcnt waits.  The input may be
// the channel concat [a | a2] of two tensors read in place (UNet skip
// connections), split at a multiple of 64 channels.
#include "gemm_common.h"

struct HaloArgs {
  GemmArgs g;             // B operand (packed [Cout][3][3][Cin] weights) + epilogue; M, N, K = 9 Cin
  const bf16_t* a2;       // channels [Ca, Cin) of the input, or null
  int Ca, lda2;           // channels read from g.A; pixel stride of a2
  const float* gn_stat;   // [B][G][2] (mean, rstd) of the conv INPUT, or null (no GroupNorm)
  const bf16_t* gamma;    // [Cin]
  const bf16_t* beta;     // [Cin]
  int G, silu;
  const bf16_t* a2_end;   // CSK_DEBUG bounds
};

// s_waitcnt vmcnt(N) as the builtin (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14,
// expcnt / lgkmcnt at their no-wait maxima): unlike inline asm the compiler's
// wait insertion sees it and knows which LDS-DMAs it retired
template <int N>
__device__ __forceinline__ void halo_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

__device__ __forceinline__ void halo_dma(const bf16_t* src, bf16_t* dst) {
  __builtin_amdgcn_global_load_lds((csk_gptr_t)src, (csk_lptr_t)dst, 16, 0, 0);
}

// element offset of 16-byte chunk c of halo pixel hp in a [pixels][64] image
__device__ __forceinline__ int halo_off(int hp, int c) { return hp * 64 + ((c ^ (hp & 7)) << 3); }

template <int BM, int BN, int IW>
struct HaloGeom {
  static constexpr int R = BM / IW;                   // image rows per tile
  static constexpr int HW = IW + 2;                   // halo row width
  static constexpr int HP = (R + 2) * HW;             // halo pixels
  static constexpr int HPP = (HP + 31) / 32 * 32;     // padded: 4 waves x 8-pixel DMA pieces
  static constexpr int A_ELEMS = HPP * 64;
  static constexpr int B_ELEMS = BN * 64;
  static constexpr int PIECES_A = HPP / 8 / 4;        // DMA pieces per wave per chunk
  static constexpr int PIECES_B = BN / 8 / 4;
  static constexpr int NB = 4;                        // weight ring stages (NB - 1 steps in flight)
  static constexpr int CMAX = IW == 64 ? 960 : (IW == 32 ? 1920 : 2560);  // largest Cin (UNet up blocks)
  static constexpr int EPI = epi_smem_elems<BM, BN, epi_passes<BM, BN, 2>()>();
  static_assert(EPI <= 2 * A_ELEMS, "the epilogue stages through the halo buffers");
  static_assert(BM % IW == 0 && BN % 32 == 0, "tile");
};

template <int BM, int BN, int IW>
__global__ __launch_bounds__(256, 1) void conv_halo_kernel(const HaloArgs ha) {
  using Gm = HaloGeom<BM, BN, IW>;
  constexpr int WM = 2, WN = 2, WTM = BM / WM, WTN = BN / WN, MT = WTM / 16, NT = WTN / 16;
  constexpr int EP = epi_passes<BM, BN, WM>();
  constexpr int NB = Gm::NB;
  static_assert(NB == 4, "wait counts below assume two younger weight steps");
  // separate LDS objects for the halo buffers and the weight ring: the
  // compiler's wait insertion then tells a weight DMA in flight from the
  // transform's halo writes (one array made it drain every DMA there)
  __shared__ __attribute__((aligned(16))) bf16_t s_ah[2 * Gm::A_ELEMS];
  __shared__ __attribute__((aligned(16))) bf16_t s_bw[NB * Gm::B_ELEMS];
  // GroupNorm operands staged once in the prologue (no global loads inside the
  // main loop: any would make the compiler drain the DMAs in flight before it)
  __shared__ float s_stat[2 * 64];                                      // (mean, rstd) per group, G <= 64
  __shared__ __attribute__((aligned(16))) bf16_t s_gb[2 * Gm::CMAX];    // gamma | beta
  const GemmArgs& a = ha.g;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  const int H = a.H;
  const int tiles_n = a.N / BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;
  const int hw = H * IW;
  const int b = m0 / hw, y0 = (m0 - b * hw) / IW;  // sample, first output row
  const int Cin = a.Cin, nch = Cin / 64, steps = 9 * nch;
  const int lrow = lane >> 3, lslot = lane & 7;
  const bool gn = ha.gn_stat != nullptr;

  // opaque per call: keeps the compiler from hoisting every DMA piece's address
  // math out of the chunk / step loops (13 live 64-bit pointers spilled)
  auto fresh = [](int v) {
    asm volatile("" : "+v"(v));
    return v;
  };

  // ---- A halo of chunk c -> abuf[c & 1] (padding / out-of-image pixels: zero page) ----
  auto issue_a = [&](int c) {
    const bool second = ha.a2 && 64 * c >= ha.Ca;
    const bf16_t* src_t = second ? ha.a2 : a.A;
    const int ld = second ? ha.lda2 : a.lda;
    const int ch = second ? 64 * c - ha.Ca : 64 * c;
    const int lr = fresh(lrow);
    bf16_t* dst = s_ah + (c & 1) * Gm::A_ELEMS;
#pragma unroll
    for (int i = 0; i < Gm::PIECES_A; ++i) {
      const int p = wid * Gm::PIECES_A + i;
      const int hp = 8 * p + lr;
      const int hr = hp / Gm::HW, hc = hp - hr * Gm::HW;
      const int y = y0 - 1 + hr, x = hc - 1;
      const bool ok = hp < Gm::HP && y >= 0 && y < H && x >= 0 && x < IW;
      const bf16_t* src = a.zero + 8 * lslot;
      if (ok) {
        src = src_t + ((size_t)(b * H + y) * IW + x) * ld + ch + 8 * (lslot ^ (hp & 7));
        CSK_DCHECK(second ? (src + 8 <= ha.a2_end) : (src + 8 <= a.a_end), 81, hp, Gm::HP);
      }
      halo_dma(src, dst + 512 * p);
    }
  };
  // ---- weights of step s = 9 c + tap -> bbuf[s & 1] ----
  auto issue_b = [&](int s) {
    const int c = s / 9, tap = s - 9 * c;
    const int koff = tap * Cin + 64 * c;
    const int lr = fresh(lrow);
    bf16_t* dst = s_bw + (s % Gm::NB) * Gm::B_ELEMS;
#pragma unroll
    for (int i = 0; i < Gm::PIECES_B; ++i) {
      const int n = n0 + (wid * Gm::PIECES_B + i) * 8 + lr;
      const bf16_t* src = a.W + ((unsigned)(n * a.ldb + koff + 8 * (lslot ^ lr)));
      CSK_DCHECK(src + 8 <= a.w_end, 82, n, a.N);
      halo_dma(src, dst + 512 * (wid * Gm::PIECES_B + i));
    }
  };
  // ---- normalise (+ SiLU) the landed halo of chunk c in place ----
  auto transform = [&](int c) {
    bf16_t* as = s_ah + (c & 1) * Gm::A_ELEMS;
    const int cg = Cin / ha.G;
    for (int e = tid; e < Gm::HP * 8; e += 256) {
      const int hp = e >> 3, phys = e & 7;
      const int hr = hp / Gm::HW, hc = hp - hr * Gm::HW;
      const int y = y0 - 1 + hr, x = hc - 1;
      if (y < 0 || y >= H || x < 0 || x >= IW) continue;  // padding stays zero
      const int ch0 = 64 * c + 8 * (phys ^ (hp & 7));
      float gm[8], bt[8];
      unpack8(*reinterpret_cast<const uint4*>(s_gb + ch0), gm);
      unpack8(*reinterpret_cast<const uint4*>(s_gb + Gm::CMAX + ch0), bt);
      uint4* q = reinterpret_cast<uint4*>(as + hp * 64 + phys * 8);
      float f[8];
      unpack8(*q, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int g = (ch0 + j) / cg;
        const float sc = gm[j] * s_stat[2 * g + 1];
        const float v = __builtin_fmaf(f[j] - s_stat[2 * g], sc, bt[j]);
        f[j] = ha.silu ? silu_f(v) : v;
      }
      *q = pack8(f);
    }
  };

  // per-lane halo pixel of each MFMA row (tap (0, 0)): output pixel (r, w) -> r (W + 2) + w
  int hbase[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int pl = wm * WTM + i * 16 + fr;
    hbase[i] = (pl / IW) * Gm::HW + (pl % IW);
  }

  v4f acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // prologue: chunk 0's halo, the first NB - 1 steps' weights, chunk 0's affine
  issue_a(0);
#pragma unroll
  for (int s = 0; s < NB - 1; ++s)
    if (s < steps) issue_b(s);
  if (gn) {
    for (int i = tid; i < 2 * ha.G; i += 256) s_stat[i] = ha.gn_stat[(size_t)b * ha.G * 2 + i];
    for (int i = tid; i < Cin; i += 256) {
      s_gb[i] = ha.gamma[i];
      s_gb[Gm::CMAX + i] = ha.beta[i];
    }
  }

  for (int s = 0; s < steps; ++s) {
    const int c = s / 9, tap = s - 9 * c;
    // B(s) (and at a chunk's first tap its halo A(c)) landed.  Loads retire in
    // issue order, so the count of younger ones is exact: B(s+1), B(s+2) and,
    // for the three steps after a chunk start, A(c+1) (issued after B(9c+3))
    const int y2 = min(NB - 2, steps - 1 - s);
    const bool ya = tap >= 1 && tap <= NB - 1 && c + 1 < nch;
    if (tap == 0) {
      // a chunk's first step: at least 8 more steps follow, so exactly
      // B(s+1), B(s+2) are younger; this branch's own wait tells the compiler
      // the halo DMA retired before the transform touches that buffer
      halo_vmcnt<2 * Gm::PIECES_B>();
      __builtin_amdgcn_s_barrier();
      if (gn) {
        transform(c);
        __syncthreads();
      }
    } else {
      if (ya) {
        if (y2 == 2) halo_vmcnt<2 * Gm::PIECES_B + Gm::PIECES_A>();
        else if (y2 == 1) halo_vmcnt<Gm::PIECES_B + Gm::PIECES_A>();
        else halo_vmcnt<Gm::PIECES_A>();
      } else {
        if (y2 == 2) halo_vmcnt<2 * Gm::PIECES_B>();
        else if (y2 == 1) halo_vmcnt<Gm::PIECES_B>();
        else halo_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
    }
    // B(s + NB - 1) into the stage step s - 1 used; at a chunk start the next
    // chunk's halo into the buffer chunk c - 1 used (both free past the barrier)
    if (s + NB - 1 < steps) issue_b(s + NB - 1);
    if (tap == 0 && c + 1 < nch) issue_a(c + 1);
    const bf16_t* as = s_ah + (c & 1) * Gm::A_ELEMS;
    const bf16_t* bs = s_bw + (s % NB) * Gm::B_ELEMS;
    const int ky = tap / 3, kx = tap - 3 * ky;
    const int toff = ky * Gm::HW + kx;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8s af[MT], bfr[NT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        af[i] = *reinterpret_cast<const v8s*>(as + halo_off(hbase[i] + toff, ks * 4 + fq));
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
  const float2 lnrow = make_float2(0.f, 0.f);
  float2 lnlane[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) lnlane[i] = make_float2(0.f, 1.f);
  gemm_epilogue_ln<BM, BN, WM, WN, false, EP, 256, true>(a, acc, s_ah, m0, n0, 0, lnrow, lnlane, false);
}

CSK_DEBUG_EXPORT(conv_halo)

const bf16_t* csk_zero_ptr();

template <int BM, int BN, int IW>
static int launch_halo(HaloArgs ha, hipStream_t s) {
  ha.g.gn_seg = gn_seg_for<BM, BN, 2>();
  const dim3 grid((ha.g.M / BM) * (ha.g.N / BN));
  conv_halo_kernel<BM, BN, IW><<<grid, 256, 0, s>>>(ha);
  return (int)hipGetLastError();
}

// Which halo tile serves (W, Cout), or 0: 128x160 for W = 64 / 32 / 16 (a 256-row
// tile at W = 64 spills: 160 accumulators + 8 A fragments per lane).
static int halo_bm(int W) { return (W == 64 || W == 32 || W == 16) ? 128 : 0; }

static int halo_cmax(int W) { return W == 64 ? 960 : (W == 32 ? 1920 : 2560); }

CSK_API int csk_conv_halo_supported(int B, int H, int W, int Cin, int Cout) {
  const int bm = halo_bm(W);
  return bm && Cin % 64 == 0 && Cin <= halo_cmax(W) && Cout % 160 == 0 && (H * W) % bm == 0 && B > 0 ? bm : 0;
}

// y = conv3x3(act(GN(x)))  [+ bias + bias2d, act, * out_scale, + residual], NHWC.
// x: [B][H][W][Ca] (pixel stride lda); x2: [B][H][W][Cin - Ca] (pixel stride lda2) or null;
// wp: packed [Cout][3][3][Cin]; gn_stat: [B][G][2] (mean, rstd) of the input or null.
// gn_part: GN statistics of the OUTPUT for the next GroupNorm (segment height returned
// by csk_conv_halo_gn_seg).
CSK_API int csk_conv_halo(void* y, const void* x, int lda, const void* x2, int lda2, int Ca, const void* wp,
                          const void* bias, const void* bias2d, int ldb2, const void* res, int B, int H, int W,
                          int Cin, int Cout, int act, float out_scale, void* gn_part, const void* gn_stat,
                          const void* gamma, const void* beta, int G, int silu, hipStream_t stream) {
  const int bm = csk_conv_halo_supported(B, H, W, Cin, Cout);
  if (!bm || !csk_zero_ptr() || (x2 && (Ca % 64 || Ca >= Cin)) ||
      (gn_stat && (!gamma || !beta || Cin % G || G > 64 || Cin > halo_cmax(W))))
    return (int)hipErrorInvalidValue;
  HaloArgs ha{};
  GemmArgs& a = ha.g;
  a.A = (const bf16_t*)x;
  a.W = (const bf16_t*)wp;
  a.C = (bf16_t*)y;
  a.bias = (const bf16_t*)bias;
  a.bias2d = (const bf16_t*)bias2d;
  a.res = (const bf16_t*)res;
  a.zero = csk_zero_ptr();
  a.M = B * H * W;
  a.N = Cout;
  a.K = 9 * Cin;
  a.lda = lda;
  a.ldb = 9 * Cin;
  a.ldc = Cout;
  a.ldr = Cout;
  a.ldb2 = ldb2;
  a.rows_per_b = H * W;
  a.act = act;
  a.out_scale = out_scale;
  a.H = H;
  a.Wd = W;
  a.Cin = Cin;
  a.Ho = H;
  a.Wo = W;
  a.kh = a.kw = 3;
  a.stride = 1;
  a.pt = a.pl = 1;
  a.dil = 1;
  a.gn_part = (float*)gn_part;
  a.a_end = a.A + ((size_t)B * H * W - 1) * lda + (x2 ? Ca : Cin);
  a.w_end = a.W + (size_t)Cout * 9 * Cin;
  ha.a2 = (const bf16_t*)x2;
  ha.Ca = x2 ? Ca : Cin;
  ha.lda2 = lda2;
  ha.a2_end = x2 ? ha.a2 + ((size_t)B * H * W - 1) * lda2 + (Cin - Ca) : nullptr;
  ha.gn_stat = (const float*)gn_stat;
  ha.gamma = (const bf16_t*)gamma;
  ha.beta = (const bf16_t*)beta;
  ha.G = G > 0 ? G : 1;
  ha.silu = silu;
  switch (W) {
    case 64: return launch_halo<128, 160, 64>(ha, stream);
    case 32: return launch_halo<128, 160, 32>(ha, stream);
    case 16: return launch_halo<128, 160, 16>(ha, stream);
    default: return (int)hipErrorInvalidValue;
  }
}

CSK_API int csk_conv_halo_gn_seg(int W) {
  switch (W) {
    case 64:
    case 32:
    case 16: return gn_seg_for<128, 160, 2>();
    default: return 0;
  }
}
