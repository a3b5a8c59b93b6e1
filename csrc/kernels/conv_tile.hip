// Persistent halo-tile 3x3 convolution for narrow outputs (Cout = 32 / 64): the
// Real-ESRGAN dense-block convs (north-star config #5; RRDBNet
// conv1..conv4 of every residual dense block, 276 of the 345 convs of an x4
// upscale).
//
// Why: the implicit-GEMM conv (gemm_glds.hip / gemm.hip) stages an A tile per
// K-step per tap — each input pixel crosses L2 -> LDS nine times — and with
// N = 32 output channels every staged A byte feeds only 32 FLOP.  The four
// Cout = 32 convs ran at 290-420 TF/s bound by the LDS-DMA fill
// (profiles/esrgan_kernels_r5a.txt).  Here a workgroup owns an 8 x 32 pixel
// output tile and stages its (8+2) x (32+2) input halo ONCE per 32-channel
// chunk; the nine taps read it at a pixel offset, so A crosses L2 -> LDS
// ~1.33x instead of 9x and per chunk a workgroup issues 48 LDS-DMA
// instructions for 4.7 MFLOP (the 128x32 implicit GEMM: ~190).
//
// Structure (MI355X-first):
//   * persistent: one 512-thread workgroup per CU walks tiles w, w + G, ...;
//     the (tile, chunk) units form ONE LDS-DMA stream through a 3-stage ring
//     (two chunks in flight), so the next tile's first chunks land during this
//     tile's last chunk and its register-direct epilogue (no LDS in the
//     epilogue: the ring stays live).  Counted `vmcnt` waits, raw barriers.
//   * LDS images are row-major, 64 B (one 32-channel chunk) per halo pixel or
//     (tap, cout) weight row, the four 16-byte channel groups XOR-swizzled by
//     row (ct_slot: conflict-free on the b128 lane groups); one
//     LDS-DMA instruction fills 16 rows (16 x 64 contiguous source bytes; a
//     first version that filled 64 pixels of one group per instruction touched
//     64 cache lines per 1 KB: 33.6-58.4 us against 26.7-43.9 us now);
//     out-of-image halo pixels read the zero page.
//
// Measured (tools/convtilebench.py, 512^2, profiles/conv_tile_r5.txt): 64 /
// 96 / 128 / 160 -> 32 in 26.7 / 33.4 / 38.0 / 43.9 us (362-551 TF/s) against
// 38.7 / 54.7 / 62.5 / 87.7 us for the tuned implicit GEMM; Real-ESRGAN x4
// 512 -> 2048 29.3 -> 24.2 ms.  The Cout = 64 instance (2-stage ring: 64 KB
// stages) with the fused "* 0.2 + x" epilogue of conv5: 192 -> 64 77.9 vs 96.6
// us, 64 -> 64 at 1024^2 / 2048^2 133 / 522 vs 158 / 622 us
// (profiles/conv_tile64_r5.txt).
//   * resident weights (RWC > 0 instances, Cout <= 32, Cin <= 160): the packed
//     weight (<= 90 KB) is DMA'd once per workgroup and the ring carries halos
//     only (per-unit LDS fill halved; Cin = 160 with a 2-stage ring): 64 / 96 /
//     128 / 160 -> 32 in 25.2 / 29.6 / 32.6 / 36.7 us against 28.2 / 31.6 /
//     37.0 / 41.9 us with per-unit weight DMA, same process
//     (profiles/conv_tile_r6.txt); csk_set_conv_tile_no_rw is the A/B switch.
//   * Cout = 64 runs 16 x 32 tiles (TR = 2: wave w computes rows w and w + 8;
//     80 KB stages): 192 -> 64 77.1 vs 80.6 us, 64 -> 64 at 2048^2 525.8 vs
//     579.0 us against 8-row tiles, same process (profiles/conv_tile_r6.txt).
//   * wave w computes tile row w (32 px = 2 MFMA row fragments) x 32 outputs
//     with v_mfma_f32_16x16x32_bf16 (B . A order: row-layout accumulators, a
//     lane holds one pixel's 4 consecutive outputs -> 8-byte stores).
//   * input / output are channel slices of wider NHWC buffers (pixel strides
//     lda / ldc): the dense block's concat is never materialised.
#include "gemm_common.h"

namespace {

constexpr int CT_TW = 32, CT_HW = CT_TW + 2;  // output tile width, halo width

// per output width NOUT (16, 32 or 64): weight rows 9 x NOUT padded to whole
// 8-wave x 16-row DMA rounds, ring depth (3 stages at 16 / 32: 120 / 144 KB; 2 at 64: 128 KB)
//
// RW (resident weights, NOUT <= 32 and Cin <= 128): the whole packed weight,
// nc chunks x 9 NOUT rows, is DMA'd once per workgroup ahead of a halo-only
// ring (the per-unit weight DMA was half of every unit's LDS fill)
constexpr int CT_RW_MAXC = 5;  // chunks (Cin <= 160) a resident image holds (5: 2-stage ring)
//
// TR = tile rows per wave (TALL tiles, TR = 2: 16 x 32 pixels; NOUT = 64 only,
// where a 37 KB weight chunk per 8 x 32 tile was 62 % of every unit's fill):
// halo 18 x 34 = 612 pixels in 640 slots, stage 80 KB, 2 stages = 160 KB.
template <int NOUT, int RWC, int TR = 1>
struct CtGeo {
  static constexpr bool RW = RWC > 0;
  static constexpr int TH = 8 * TR;                           // output tile height
  static constexpr int HPX = (TH + 2) * CT_HW;                // 340 / 612 halo pixels
  static constexpr int HSLOT = (HPX + 127) / 128 * 128;       // 384 / 640 slots: whole 8-wave x 16-pixel DMA rounds
  static constexpr int HALO = HSLOT * 64;                     // halo bytes per stage ([pixel][4 x 16 B])
  static constexpr int HI = HSLOT / 16 / 8;                   // halo DMA instructions per wave per chunk (3 / 5)
  static constexpr int WROWS = (9 * NOUT + 127) / 128 * 128;  // 384 / 640
  static constexpr int WGT = RW ? 0 : WROWS * 64;             // weight bytes per ring stage ([tap x cout][4 x 16 B])
  static constexpr int WCH = 9 * NOUT * 64;                   // RW: bytes per resident chunk (unpadded rows)
  static constexpr int WRES = RWC * WCH;                      // RW: resident image (72 / 90 KB at NOUT = 32)
  static constexpr int STAGE = HALO + WGT;
  static constexpr int S = NOUT == 64 || RWC > 4 ? 2 : 3;
  static constexpr int WI = RW ? 0 : WROWS / 16 / 8;          // weight DMA instructions per wave per chunk (3 / 5)
  static constexpr int NF = NOUT / 16;                        // output fragments per pixel row
};

// 16-byte slot of channel group g (of 4) in LDS row r (a pixel or a (tap, cout)
// row of 64 B).  A ds_read_b128 serves lanes {0-3,12-15,20-27} (and the three
// other groups of MICROARCH §LDS) in one cycle: rows base+0..3 and base+12..15
// of group g with rows base+4..11 of group g^1, for ANY base (the A reads sit
// at a kx pixel offset).  Per row residue mod 4 the four rows r, r+4, r+8,
// r+12 then need four distinct slots: g ^ 2·((r >> 2) & 1) gives them
// (g, g^1^2, g^1, g^2); the former g ^ ((r >> 2) & 3) was 2-way on 120 of the
// 144 A reads and on every B read
__device__ __forceinline__ int ct_slot(int r, int g) { return g ^ (((r >> 2) & 1) << 1); }

struct ConvTileArgs {
  const bf16_t* x;     // [B][H][W] pixels, pixel stride lda, channels [0, Cin)
  const bf16_t* w;     // packed [NOUT][3][3][Cin]
  const bf16_t* bias;  // [NOUT] or null
  bf16_t* y;           // [B][H][W] pixels, pixel stride ldc, channels [0, NOUT)
  const bf16_t* zero;  // zero page (LDS-DMA source for padding)
  const bf16_t* res;   // [B][H][W] pixels, pixel stride ldr, or null
  const bf16_t* res2;  // [B][H][W] pixels, pixel stride ldr2, or null:
                       // y = act(conv + bias) * out_scale + res_scale * res + res2
  int B, H, W, Cin, lda, ldc, act, ldr, ldr2;
  int Cout;            // <= NOUT: weight rows / bias / stores of channels >= Cout are skipped
  int u8;              // narrow outputs only: store round(clamp(y, 0, 1) * 255) as uint8 (y: unsigned char*, stride ldc bytes)
  int up;              // 1: nearest-x2 upsampled input (x is [B][H/2][W/2]); the halo reads input pixel (iy/2, ix/2)
  int Wi;              // input row width in pixels (W, or W/2 with up)
  float out_scale, res_scale;
  int tiles_x, tiles_y, ntiles;
};

typedef __attribute__((address_space(1))) const void* ct_gptr_t;
typedef __attribute__((address_space(3))) void* ct_lptr_t;

__device__ __forceinline__ void ct_dma(const bf16_t* src, unsigned char* dst) {
  __builtin_amdgcn_global_load_lds((ct_gptr_t)src, (ct_lptr_t)dst, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void ct_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void ct_ld(v8s& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
// wait until at most N LDS reads issued after the fragments f[0..R) are
// outstanding (LDS reads return in order); names every fragment it waits for
template <int N, int R>
__device__ __forceinline__ void ct_wait(v8s (&f)[R]) {
  if constexpr (R == 3) {
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]) : "n"(N));
  } else if constexpr (R == 4) {
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]) : "n"(N));
  } else if constexpr (R == 8) {
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7])
                 : "n"(N));
  } else {
    static_assert(R == 6, "2 TR + NF fragments");
    asm volatile("s_waitcnt lgkmcnt(%6)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5])
                 : "n"(N));
  }
}

}  // namespace

template <int NOUT, int RWC, int TR>
__global__ __launch_bounds__(512, 1) void conv_tile_kernel(const ConvTileArgs a) {
  using Geo = CtGeo<NOUT, RWC, TR>;
  constexpr bool RW = Geo::RW;
  constexpr int CT_S = Geo::S, CT_STAGE = Geo::STAGE, CT_WI = Geo::WI, NF = Geo::NF, CT_R = 2 * TR + NF;
  constexpr int CT_TH = Geo::TH, CT_HPX = Geo::HPX, CT_HALO = Geo::HALO, CT_HI = Geo::HI;
  __shared__ __attribute__((aligned(16))) unsigned char smem_all[Geo::WRES + CT_S * CT_STAGE];
  unsigned char* const smem = smem_all + Geo::WRES;  // the ring (after the resident weights)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int w = xcd_remap(blockIdx.x, G);
  const int my_tiles = w < a.ntiles ? (a.ntiles - 1 - w) / G + 1 : 0;
  const int nc = a.Cin / 32;  // 32-channel chunks per tile
  const int U = my_tiles * nc;
  if (U == 0) return;
  const int H = a.H, W = a.W;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- weight DMA (tile-independent): instruction k = wv * 3 + i writes rows
  // 16 k .. 16 k + 15 (lane L: row 16 k + L / 4, LDS slot L % 4) ----
  const bf16_t* wsrc[CT_WI > 0 ? CT_WI : 1];
#pragma unroll
  for (int i = 0; i < CT_WI; ++i) {
    const int row = (wv * CT_WI + i) * 16 + (lane >> 2);  // tap * NOUT + output channel
    const int tap = row / NOUT, co = row % NOUT;
    const int g = (lane & 3) ^ (((row >> 2) & 1) << 1);  // source channel group landing in this lane's slot
    wsrc[i] = row < 9 * NOUT && co < a.Cout ? a.w + ((size_t)co * 9 + tap) * a.Cin + g * 8 : a.zero;
  }
  // ---- RW: the resident weight image, DMA instruction k (k = wv, wv + 8, ...)
  // writes flattened rows 16 k .. 16 k + 15 of [chunk][tap x cout] ----
  if constexpr (RW) {
    const int nrow = nc * 9 * NOUT;
    for (int k = wv; k * 16 < nrow; k += 8) {
      const int r = k * 16 + (lane >> 2);
      const int c = r / (9 * NOUT), rr = r - c * (9 * NOUT);
      const int tap = rr / NOUT, co = rr % NOUT;
      const int g = (lane & 3) ^ (((r >> 2) & 1) << 1);
      ct_dma(co < a.Cout ? a.w + ((size_t)co * 9 + tap) * a.Cin + c * 32 + g * 8 : a.zero, smem_all + k * 1024);
    }
  }
  // ---- halo DMA: instruction k = wv * 3 + i writes halo pixels 16 k .. 16 k + 15 ----
  const bf16_t* hsrc[CT_HI];
  int d_tile = w, d_c = 0, d_s = 0;  // next unit to issue: tile, chunk, ring stage
  auto set_halo = [&]() {
    const int b = d_tile / (a.tiles_x * a.tiles_y);
    const int rem = d_tile - b * (a.tiles_x * a.tiles_y);
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
#pragma unroll
    for (int i = 0; i < CT_HI; ++i) {
      const int hp = (wv * CT_HI + i) * 16 + (lane >> 2);
      const int hy = hp / CT_HW, hx = hp - hy * CT_HW;
      const int iy = ty * CT_TH - 1 + hy, ix = tx * CT_TW - 1 + hx;
      const bool ok = hp < CT_HPX && iy >= 0 && iy < H && ix >= 0 && ix < W;
      const int g = (lane & 3) ^ (((hp >> 2) & 1) << 1);
      const int sy = iy >> a.up, sx = ix >> a.up;  // (the input grid of an upsampled conv)
      hsrc[i] = ok ? a.x + ((size_t)(b * (H >> a.up) + sy) * a.Wi + sx) * a.lda + g * 8 : a.zero;
    }
  };
  set_halo();
  auto issue = [&]() {
    unsigned char* st = smem + d_s * CT_STAGE;
    const int co = d_c * 32;  // channel offset of this chunk
#pragma unroll
    for (int i = 0; i < CT_HI; ++i) ct_dma(hsrc[i] + co, st + (wv * CT_HI + i) * 1024);
    if constexpr (!RW) {
#pragma unroll
      for (int i = 0; i < CT_WI; ++i) ct_dma(wsrc[i] + co, st + CT_HALO + (wv * CT_WI + i) * 1024);
    }
    d_s = d_s + 1 == CT_S ? 0 : d_s + 1;
    if (++d_c == nc) {
      d_c = 0;
      d_tile += G;
      if (d_tile < a.ntiles) set_halo();
    }
  };

  v4f acc[TR][2][NF];  // [tile row wv + 8 t][pixel half][output fragment]
  auto zero_acc = [&]() {
#pragma unroll
    for (int t = 0; t < TR; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[t][i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();
  float bias[NF][4];
#pragma unroll
  for (int j = 0; j < NF; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = j * 16 + fq * 4 + r;
      bias[j][r] = a.bias && co < a.Cout ? bf2f(a.bias[co]) : 0.f;
    }

  auto epilogue = [&](int tile) {
    const int b = tile / (a.tiles_x * a.tiles_y);
    const int rem = tile - b * (a.tiles_x * a.tiles_y);
    const int ty = rem / a.tiles_x, tx = rem - ty * a.tiles_x;
#pragma unroll
    for (int t = 0; t < TR; ++t) {
    const int y = ty * CT_TH + wv + 8 * t;
    if (y >= H) return;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int x = tx * CT_TW + i * 16 + fr;
      if (x >= W) continue;
      bf16_t* op = a.y + ((size_t)(b * H + y) * W + x) * a.ldc;
      const bf16_t* rp = a.res ? a.res + ((size_t)(b * H + y) * W + x) * a.ldr : nullptr;
      const bf16_t* rp2 = a.res2 ? a.res2 + ((size_t)(b * H + y) * W + x) * a.ldr2 : nullptr;
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int c0 = j * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_act(a.act, acc[t][i][j][r] + bias[j][r]) * a.out_scale;
        if (c0 + 4 > a.Cout) {  // narrow output (Cout < 16, e.g. RGB): element stores, no residuals
          if (a.u8) {  // image output: the upscaler's uint8 pixels straight from the accumulators
            unsigned char* ob = reinterpret_cast<unsigned char*>(a.y) + ((size_t)(b * H + y) * W + x) * a.ldc;
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (c0 + r < a.Cout) ob[c0 + r] = (unsigned char)__float2int_rn(fminf(fmaxf(v[r], 0.f), 1.f) * 255.f);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (c0 + r < a.Cout) op[c0 + r] = f2bf(v[r]);
          }
          continue;
        }
        if (rp) {
          const uint2 rr = *reinterpret_cast<const uint2*>(rp + c0);
          const float rs = a.res_scale;
          v[0] += rs * __uint_as_float(rr.x << 16);
          v[1] += rs * __uint_as_float(rr.x & 0xffff0000u);
          v[2] += rs * __uint_as_float(rr.y << 16);
          v[3] += rs * __uint_as_float(rr.y & 0xffff0000u);
        }
        if (rp2) {
          const uint2 rr = *reinterpret_cast<const uint2*>(rp2 + c0);
          v[0] += __uint_as_float(rr.x << 16);
          v[1] += __uint_as_float(rr.x & 0xffff0000u);
          v[2] += __uint_as_float(rr.y << 16);
          v[3] += __uint_as_float(rr.y & 0xffff0000u);
        }
        uint2 wd;
        wd.x = pack2(v[0], v[1]);
        wd.y = pack2(v[2], v[3]);
        *reinterpret_cast<uint2*>(op + c0) = wd;
      }
    }
    }
  };

  // per-lane LDS byte offsets of the fragment reads inside a stage (the same
  // for every unit).  The swizzle depends on bit 2 of the row only, which
  // whole 8-row / 16-pixel / 16-row steps keep: A (halo pixel of tile row
  // wv + 8 t + ky, shifted by kx) = aoff[tap] + compile-time offset of (t,
  // half); B (weight row tap x NOUT + 16 j + fr) = boff + compile-time offset.
  const unsigned sbase = (unsigned)(size_t)(ct_lptr_t)(void*)smem;
  unsigned aoff[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int hp = (wv + tap / 3) * CT_HW + fr + tap % 3;
    aoff[tap] = (unsigned)(hp * 64 + ct_slot(hp, fq) * 16);
  }
  const unsigned boff = (unsigned)(fr * 64 + ct_slot(fr, fq) * 16);

  // ---- prologue: S - 1 units in flight ----
#pragma unroll
  for (int k = 0; k < CT_S - 1; ++k)
    if (k < U) issue();
  int c = 0, s = 0, tile = w;
  for (int u = 0; u < U; ++u) {
    // unit u landed once at most S - 2 younger units (CT_HI + CT_WI instructions each) are in flight
    if (CT_S == 3 && u + 1 < U) ct_vmcnt<CT_HI + CT_WI>();
    else ct_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (u + CT_S - 1 < U) issue();
    // nine taps, fragment reads one tap ahead of the MFMAs that consume them
    // (inline asm, counted lgkmcnt: the compiler's own waits drained every read
    // in front of each tap's MFMAs)
    const unsigned hb = sbase + (unsigned)(s * CT_STAGE);
    const unsigned wb = RW ? sbase - (unsigned)Geo::WRES + (unsigned)(c * Geo::WCH) : hb + CT_HALO;
    v8s fr2[2][CT_R];
    auto rd = [&](v8s (&f)[CT_R], int tap) {
#pragma unroll
      for (int i = 0; i < 2 * TR; ++i) ct_ld(f[i], hb + aoff[tap] + (unsigned)(((i >> 1) * 8 * CT_HW + (i & 1) * 16) * 64));
#pragma unroll
      for (int j = 0; j < NF; ++j) ct_ld(f[2 * TR + j], wb + boff + (unsigned)((tap * NOUT + j * 16) * 64));
    };
    rd(fr2[0], 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      v8s (&f)[CT_R] = fr2[tap & 1];
      if (tap + 1 < 9) {
        rd(fr2[(tap + 1) & 1], tap + 1);
        ct_wait<CT_R>(f);
      } else {
        ct_wait<0>(f);
      }
#pragma unroll
      for (int i = 0; i < 2 * TR; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j)
          acc[i >> 1][i & 1][j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(f[2 * TR + j], f[i], acc[i >> 1][i & 1][j], 0, 0, 0);
    }
    s = s + 1 == CT_S ? 0 : s + 1;
    if (++c == nc) {
      epilogue(tile);
      zero_acc();
      c = 0;
      tile += G;
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static int g_ct_cus = 0;
static int g_ct_no_rw = 0;

// A/B switch (tools/convtilebench.py --rw): bit 0 = per-unit weight DMA everywhere, bit 1 = 8-row tiles at Cout = 64
CSK_API int csk_set_conv_tile_no_rw(int v) {
  g_ct_no_rw = v;
  return 0;
}

// 1 when csk_conv_tile takes this conv: 3x3 / stride 1 / pad 1, Cout = 32 or
// 64 (or <= 16: the 16-wide instance, element stores below 16, e.g. Real-ESRGAN's RGB conv_last),
// Cin % 32 == 0 (<= 64 chunks), 16-byte aligned input pixel strides; H, W are
// the OUTPUT size (even with up: the input is H/2 x W/2)
CSK_API int csk_conv_tile_ok2(int B, int H, int W, int Cin, int Cout, int lda, int ldc, int up) {
  const bool narrow = Cout > 0 && Cout < 16;
  return B > 0 && H > 0 && W > 0 && (Cout == 16 || Cout == 32 || Cout == 64 || narrow) && Cin % 32 == 0 && Cin >= 32 &&
         Cin <= 2048 && lda >= Cin && lda % 8 == 0 && ldc >= Cout && (narrow || ldc % 4 == 0) &&
         (!up || (H % 2 == 0 && W % 2 == 0)) && (long long)B * H * W * lda < (1ll << 31) &&
         (long long)B * H * W * ldc < (1ll << 31);
}

CSK_API int csk_conv_tile_ok(int B, int H, int W, int Cin, int Cout, int lda, int ldc) {
  return csk_conv_tile_ok2(B, H, W, Cin, Cout, lda, ldc, 0);
}

// y[..., :Cout] = act(conv3x3(up?(x)[..., :Cin]) + bias) * out_scale (+ res_scale * res[..., :Cout])
// (+ res2[..., :Cout]), NHWC with pixel strides lda / ldc / ldr / ldr2 (res, res2 may be null;
// residuals need Cout >= 16; u8: Cout < 16 only, y is uint8 with pixel stride ldc bytes).  H, W: output size.
CSK_API int csk_conv_tile2(void* y, const void* x, const void* wp, const void* bias, const void* res, const void* res2,
                           int B, int H, int W, int Cin, int Cout, int lda, int ldc, int ldr, int ldr2, int act,
                           float out_scale, float res_scale, int up, int u8, hipStream_t stream) {
  if (!csk_conv_tile_ok2(B, H, W, Cin, Cout, lda, ldc, up) || !csk_zero_ptr()) return (int)hipErrorInvalidValue;
  const bool narrow = Cout < 16;
  if ((((size_t)x) & 15) || (!narrow && (((size_t)y) & 7)) || (((size_t)wp) & 15)) return (int)hipErrorInvalidValue;
  if (u8 && !narrow) return (int)hipErrorInvalidValue;  // uint8 images: the Cout < 16 instance only
  if ((res || res2) && narrow) return (int)hipErrorInvalidValue;
  if (res && ((((size_t)res) & 7) || ldr < Cout || ldr % 4 || (long long)B * H * W * ldr >= (1ll << 31)))
    return (int)hipErrorInvalidValue;
  if (res2 && ((((size_t)res2) & 7) || ldr2 < Cout || ldr2 % 4 || (long long)B * H * W * ldr2 >= (1ll << 31)))
    return (int)hipErrorInvalidValue;
  if ((size_t)(Cin + 64) * sizeof(bf16_t) > (size_t)csk_zero_bytes()) return (int)hipErrorInvalidValue;
  if (!g_ct_cus) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    g_ct_cus = cus > 0 ? cus : 256;
  }
  ConvTileArgs a;
  a.x = (const bf16_t*)x;
  a.w = (const bf16_t*)wp;
  a.bias = (const bf16_t*)bias;
  a.y = (bf16_t*)y;
  a.zero = csk_zero_ptr();
  a.res = (const bf16_t*)res;
  a.res2 = (const bf16_t*)res2;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.lda = lda; a.ldc = ldc; a.act = act;
  a.ldr = ldr; a.ldr2 = ldr2; a.Cout = Cout; a.up = up ? 1 : 0; a.Wi = up ? W / 2 : W; a.u8 = u8 ? 1 : 0;
  a.out_scale = out_scale; a.res_scale = res_scale;
  const bool tall = Cout == 64 && !(g_ct_no_rw & 2);  // 16 x 32 tiles (TR = 2)
  a.tiles_x = (W + CT_TW - 1) / CT_TW;
  a.tiles_y = (H + (tall ? 16 : 8) - 1) / (tall ? 16 : 8);
  a.ntiles = B * a.tiles_x * a.tiles_y;
  const int G = a.ntiles < g_ct_cus ? a.ntiles : g_ct_cus;
  // resident weights (Cout <= 32): Cin <= 128 with the 3-stage halo ring, 160 with 2 stages
  const int rwc = (g_ct_no_rw & 1) ? 0 : Cin <= 128 ? 4 : Cin <= 32 * CT_RW_MAXC ? 5 : 0;
  if (Cout == 64 && tall) conv_tile_kernel<64, 0, 2><<<G, 512, 0, stream>>>(a);
  else if (Cout == 64) conv_tile_kernel<64, 0, 1><<<G, 512, 0, stream>>>(a);
  else if (Cout == 32 && rwc == 4) conv_tile_kernel<32, 4, 1><<<G, 512, 0, stream>>>(a);
  else if (Cout == 32 && rwc == 5) conv_tile_kernel<32, 5, 1><<<G, 512, 0, stream>>>(a);
  else if (Cout == 32) conv_tile_kernel<32, 0, 1><<<G, 512, 0, stream>>>(a);
  else if (rwc == 4) conv_tile_kernel<16, 4, 1><<<G, 512, 0, stream>>>(a);
  else conv_tile_kernel<16, 0, 1><<<G, 512, 0, stream>>>(a);
  return (int)hipGetLastError();
}

CSK_API int csk_conv_tile(void* y, const void* x, const void* wp, const void* bias, const void* res, int B, int H,
                          int W, int Cin, int Cout, int lda, int ldc, int ldr, int act, float out_scale,
                          hipStream_t stream) {
  return csk_conv_tile2(y, x, wp, bias, res, nullptr, B, H, W, Cin, Cout, lda, ldc, ldr, 0, act, out_scale, 1.f, 0,
                        0, stream);
}
