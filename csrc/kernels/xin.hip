// Fused transformer INPUT chain of an SD UNet block at C = 320 (SURVEY K6 + K9 +
// K11; reference call site swarm/diffusion/diffusion_func.py:96, the diffusers
// Transformer2DModel: norm -> proj_in -> BasicTransformerBlock.norm1 ->
// attn1.to_q / to_k / to_v):
//
//   xg  = GroupNorm(x)          statistics merged from the producer's epilogue
//                               partials (csk_gn_finalize): per-sample affine
//   h   = Wi xg + bi            -> stored: the residual of attn1's out-projection
//   qkv = LN1(h) Wqkv^T + bqkv  -> stored [M, 960]
//
// ONE kernel instead of the GroupNorm apply pass, the proj_in GEMM and the
// LN-folded QKV GEMM: the normalised input never reaches HBM, h is read back
// by nobody but the residual, and the 960-wide QKV projection (424 TF/s as a
// K = 320 GEMM, profiles/callprof_r6_sd21_b8.txt) runs on operands that are
// already in registers.
//
// Wave layout (the fused FF's, ff.hip): 4 waves x 32 rows, one 128-row
// workgroup per CU, 32x32x16 MFMAs whose B operand is the wave's 32 rows:
//   * GN(x) of its rows lives in registers as 20 B fragments (lane: row l % 32,
//     channels 16 ks + 8 h .. +7, h = l / 32);
//   * proj_in: h^T = Wi xg^T, ten 32-channel output tiles of 20 MFMAs; each
//     tile's accumulators (channels 8 q + 4 h + r of the lane's row) ARE two B
//     fragments of the next GEMM in the k-slot order {4h + j, 8 + 4h + j}, so
//     h never leaves the registers (bf16-rounded exactly as stored); Wqkv's
//     columns are permuted the same way on the host (ops.pack_xin_qkv);
//   * LN1 folds into the QKV epilogue (ops.fold_layer_norm):
//     y = rstd (acc - mean colsum) + b', with the row's (mean, rstd) from the
//     fp32 h values of the ten proj_in tiles (sum / sum of squares per lane,
//     the two half-rows combined by one lane swap);
//   * the 40 weight tiles (10 Wi + 30 Wqkv, 20 KB each, packed as the LDS
//     images) stream through a 6-slot LDS-DMA ring, one barrier per tile;
//   * wave roles: 4 compute waves (no global memory traffic in the loop), 2
//     loader waves issuing ONLY the weight DMAs, so their counted `vmcnt`
//     waits are exact (a wave that also stores waits for its stores too:
//     that first version spent ~14 us of a 54 us kernel there), and 2 store
//     waves copying each finished 128 x 32 output tile from an LDS staging
//     buffer (double-buffered, 80-byte rows) to h / qkv with 16-byte stores.
// Measured (tools/xinbench.py, profiles/xin_fused_input_r6.txt): 47 us
// against 85 us for the GN apply + proj_in + QKV chain at 64x64 x CFG batch 8;
// the SD2.1 CFG-8 step 10.54 -> 10.42 ms same-box.  At 8192 rows (CFG-2) the
// 64 workgroups lose to the GEMMs (38 vs 35 us): ops take it from 16384 rows.
// MFMA floor: 800 32x32x16 MFMAs x 32 cycles per wave per 128 rows.
#include "common.h"

#include "attn_tile.h"

#include <type_traits>

typedef __attribute__((address_space(1))) const void* xin_gptr_t;
typedef __attribute__((address_space(3))) void* xin_lptr_t;

namespace {

constexpr int XC = 320;             // channels
constexpr int XQ = 3 * XC;          // QKV width
constexpr int XW = 4;               // waves
constexpr int XROWS = 32 * XW;      // rows per workgroup
constexpr int XSLOT = 32 * XC;      // elements per weight tile (20 KB)
constexpr int XNSLOT = 6;           // ring depth
constexpr int XLEAD = XNSLOT - 1;   // tiles issued before the loop (4 stay in flight)
constexpr int XDW = 2;              // loader waves (LDS-DMA only: their counted vmcnt waits are exact)
constexpr int XSW = 2;              // store waves (staging -> global)
constexpr int XTHREADS = 64 * (XW + XDW + XSW);
constexpr int XSTG = 80;            // staging row stride in bytes (64 + 16: 2-way LDS conflicts at most)
constexpr int XTI = XC / 32;        // proj_in tiles (10)
constexpr int XT = XTI + XQ / 32;   // all tiles (40)
constexpr int XKS = XC / 16;        // 16-deep k-steps (20)
constexpr int XDPW = XSLOT / 512 / XDW;  // 1 KB DMA pieces per loader wave per tile (10)
constexpr int XSPL = XROWS * 4 / 64 / XSW;  // 16-byte staging chunks per store-wave lane per tile (4)

struct XinArgs {
  const bf16_t* x;      // [M][320] block input (pre-GroupNorm)
  const float* stat;    // [B][G][2] GroupNorm (mean, rstd)
  const bf16_t* gamma;  // [320] GroupNorm affine
  const bf16_t* beta;
  const bf16_t* w;      // [40][5][32][64]: 10 Wi tiles then 30 LN1-folded Wqkv tiles (ops.pack_xin_qkv)
  const float* bi;      // [320] proj_in bias (fp32)
  const float* colsum;  // [960] row sums of the folded Wqkv (fp32)
  const float* bq;      // [960] folded QKV bias (fp32)
  bf16_t* h;            // [M][320]
  bf16_t* qkv;          // [M][960]
  const bf16_t* x_end;  // CSK_DEBUG bounds
  const bf16_t* w_end;
  int M, rows_per_b, G;
  float eps;            // LN1 epsilon
};

template <int N>
__device__ __forceinline__ void xin_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void xin_ld(v8s& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
__device__ __forceinline__ void xin_ldf(v4f& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
__device__ __forceinline__ void xin_wait(int n, v8s& d) {
  switch (n) {
    case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(d)); break;
    case 1: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(d)); break;
    case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(d)); break;
    case 3: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(d)); break;
    case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(d)); break;
    case 5: asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(d)); break;
    case 6: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(d)); break;
    case 7: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(d)); break;
    case 8: asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(d)); break;
    case 9: asm volatile("s_waitcnt lgkmcnt(9)" : "+v"(d)); break;
    case 10: asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(d)); break;
    default: asm volatile("s_waitcnt lgkmcnt(11)" : "+v"(d)); break;
  }
}
typedef unsigned int xu2_t __attribute__((ext_vector_type(2)));
typedef unsigned int xu4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ xu2_t make_xu2(unsigned x, unsigned y) { return xu2_t{x, y}; }

__device__ __forceinline__ void xin_waitf(v4f (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]));
}

}  // namespace

// PROBE (profiling builds, wrong results by design; csk_set_xin_probe): 1 = no
// global stores, 2 = no MFMAs, 4 = no weight DMA after the prologue (slots reused),
// 8 = no barriers in the tile loop (every role runs free), 16 = the proj_in phase's
// tiles do nothing but their barriers (h fragments left zero)
template <int PROBE>
__global__ __launch_bounds__(XTHREADS, 1) void xin_qkv_kernel(const XinArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t ring[XNSLOT * XSLOT];
  // output staging: two [128 rows][XSTG bytes] bf16 tiles (compute -> store waves)
  __shared__ __attribute__((aligned(16))) unsigned char stg[2 * XROWS * XSTG];
  // per-channel tables (plain stores in the prologue, asm reads after):
  // GroupNorm scale / shift of this workgroup's sample, proj_in bias, folded
  // QKV colsum / bias
  __shared__ __attribute__((aligned(16))) float s_ga[XC];
  __shared__ __attribute__((aligned(16))) float s_gb[XC];
  __shared__ __attribute__((aligned(16))) float s_bi[XC];
  __shared__ __attribute__((aligned(16))) float s_cs[XQ];
  __shared__ __attribute__((aligned(16))) float s_bq[XQ];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * XROWS;
  const int b = m0 / a.rows_per_b;  // every row of the workgroup is in this sample (host check)

  const unsigned ring0 = (unsigned)(size_t)(xin_lptr_t)(void*)ring;
  const unsigned stg0 = (unsigned)(size_t)(xin_lptr_t)(void*)stg;

  // ======================= loader waves (XW .. XW + XDW - 1) =======================
  if (wid >= XW && wid < XW + XDW) {
    const int dw = wid - XW;
    auto dma_tile = [&](int t) {
      bf16_t* base = ring + (t % XNSLOT) * XSLOT;
#pragma unroll
      for (int i = 0; i < XDPW; ++i) {
        const int p = dw + XDW * i;
        const bf16_t* src = a.w + (size_t)t * XSLOT + 512 * p + 8 * lane;
        CSK_DCHECK(src + 8 <= a.w_end, 95, t, XT);
        __builtin_amdgcn_global_load_lds((xin_gptr_t)src, (xin_lptr_t)(base + 512 * p), 16, 0, 0);
      }
    };
    for (int t = 0; t < XLEAD; ++t) dma_tile(t);
    __builtin_amdgcn_s_barrier();  // tables written
#pragma unroll 1
    for (int t = 0; t <= XT + 1; ++t) {
      if (t < XT) {
        // tile t landed once at most min(XLEAD - 1, XT - 1 - t) younger tiles' pieces are in flight
        switch ((PROBE & 4) ? 0 : min(XLEAD - 1, XT - 1 - t)) {
          case 4: xin_vmcnt<4 * XDPW>(); break;
          case 3: xin_vmcnt<3 * XDPW>(); break;
          case 2: xin_vmcnt<2 * XDPW>(); break;
          case 1: xin_vmcnt<1 * XDPW>(); break;
          default: xin_vmcnt<0>(); break;
        }
      }
      if constexpr ((PROBE & 8) == 0) __builtin_amdgcn_s_barrier();
      // every compute wave is done with tile t - 1: its ring slot takes tile t + XLEAD
      if (!(PROBE & 4) && t + XLEAD < XT) dma_tile(t + XLEAD);
    }
    return;
  }

  // ============================ store waves ============================
  if (wid >= XW + XDW) {
    const int sw = wid - XW - XDW;
    __builtin_amdgcn_s_barrier();  // tables written
#pragma unroll 1
    for (int t = 0; t <= XT + 1; ++t) {
      if constexpr ((PROBE & 8) == 0) __builtin_amdgcn_s_barrier();
      if (t < 2) continue;
      // tile t - 2 sits in staging buffer (t - 2) & 1 (written between barriers t - 1 and t):
      // 128 rows x 4 16-byte chunks
      const int u = t - 2;
      const unsigned sb = stg0 + (unsigned)((u & 1) * XROWS * XSTG);
      xu4_t v[XSPL];
#pragma unroll
      for (int i = 0; i < XSPL; ++i) {
        const int id = (sw * XSPL + i) * 64 + lane, r = id >> 2, c = id & 3;
        asm volatile("ds_read_b128 %0, %1" : "=v"(v[i]) : "v"(sb + (unsigned)(r * XSTG + c * 16)));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
      if (!(PROBE & 1)) {
        bf16_t* dst;
        int ld;
        if (u < XTI) {
          dst = a.h + 32 * u;
          ld = XC;
        } else {
          dst = a.qkv + 32 * (u - XTI);
          ld = XQ;
        }
#pragma unroll
        for (int i = 0; i < XSPL; ++i) {
          const int id = (sw * XSPL + i) * 64 + lane, r = id >> 2, c = id & 3;
          if (m0 + r < a.M) *reinterpret_cast<xu4_t*>(dst + (size_t)(m0 + r) * ld + 8 * c) = v[i];
        }
      }
    }
    return;
  }

  // ============================ compute waves ============================
  const int r32 = lane & 31, h = lane >> 5;
  const int row = m0 + wid * 32 + r32;
  const bool row_ok = row < a.M;
  uint4 xu[XKS];
#pragma unroll
  for (int ks = 0; ks < XKS; ++ks) {
    xu[ks] = make_uint4(0, 0, 0, 0);
    if (row_ok) {
      CSK_DCHECK(a.x + (size_t)row * XC + 16 * ks + 8 * h + 8 <= a.x_end, 96, row, a.M);
      xu[ks] = *reinterpret_cast<const uint4*>(a.x + (size_t)row * XC + 16 * ks + 8 * h);
    }
  }
  {
    const int Cg = XC / a.G;
    for (int c = tid; c < XC; c += XW * 64) {
      const float2 st = *reinterpret_cast<const float2*>(a.stat + ((size_t)b * a.G + c / Cg) * 2);
      const float sc = bf2f(a.gamma[c]) * st.y;
      s_ga[c] = sc;
      s_gb[c] = (a.beta ? bf2f(a.beta[c]) : 0.f) - st.x * sc;
      s_bi[c] = a.bi ? a.bi[c] : 0.f;
    }
    for (int c = tid; c < XQ; c += XW * 64) {
      s_cs[c] = a.colsum[c];
      s_bq[c] = a.bq ? a.bq[c] : 0.f;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // tables written

  const unsigned ga0 = (unsigned)(size_t)(xin_lptr_t)(void*)s_ga;
  const unsigned gb0 = (unsigned)(size_t)(xin_lptr_t)(void*)s_gb;
  const unsigned bi0 = (unsigned)(size_t)(xin_lptr_t)(void*)s_bi;
  const unsigned cs0 = (unsigned)(size_t)(xin_lptr_t)(void*)s_cs;
  const unsigned bq0 = (unsigned)(size_t)(xin_lptr_t)(void*)s_bq;

  // GN(x) -> B fragments
  v8s xf[XKS];
#pragma unroll
  for (int ks = 0; ks < XKS; ++ks) {
    v4f sa[4];
    const unsigned off = (unsigned)((16 * ks + 8 * h) * 4);
    xin_ldf(sa[0], ga0 + off);
    xin_ldf(sa[1], ga0 + off + 16);
    xin_ldf(sa[2], gb0 + off);
    xin_ldf(sa[3], gb0 + off + 16);
    xin_waitf(sa);
    float f[8], v[8];
    unpack8(xu[ks], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = __builtin_fmaf(f[j], sa[j >> 2][j & 3], sa[2 + (j >> 2)][j & 3]);
    xf[ks] = __builtin_bit_cast(v8s, pack8(v));
  }

  unsigned wo[4];  // byte offset of k-step (4 si + j)'s A fragment inside sub-image si
#pragma unroll
  for (int j = 0; j < 4; ++j) wo[j] = 2u * (unsigned)at_off64(r32, 2 * j + h);
  // this lane's staging row (8-byte pieces at channel 8 q + 4 h)
  const unsigned srow = (unsigned)((wid * 32 + r32) * XSTG + 8 * h);

  v8s hf[XKS];  // h^T as the QKV projection's B fragments
  float rsum = 0.f, rsq = 0.f, mean = 0.f, rstd = 0.f;

  // Software pipeline per tile t: barrier t (tile t landed, every wave done with
  // tile t - 1) -> issue tile t's first D fragment reads -> the EPILOGUE of tile
  // t - 1 (its accumulators kept in acc_prev) while they are in flight -> the
  // MFMA chain of tile t.  The staging buffer of tile t - 1 is written between
  // barriers t and t + 1; the store waves copy it out after barrier t + 1.
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr ((PROBE & 8) == 0) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto slot = [&](int t) -> unsigned {
    return ring0 + (unsigned)(((PROBE & 4) ? t % XLEAD : t % XNSLOT) * XSLOT * 2);
  };
  // 16 outputs (channels 8 q + 4 h + r of the lane's row) -> staging buffer t & 1
  auto stage = [&](int t, const uint4& lo, const uint4& hi) {
    const unsigned d = stg0 + (unsigned)((t & 1) * XROWS * XSTG) + srow;
    asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %2 offset:16\n\tds_write_b64 %0, %3 offset:32\n\t"
                 "ds_write_b64 %0, %4 offset:48"
                 :: "v"(d), "v"(make_xu2(lo.x, lo.y)), "v"(make_xu2(lo.z, lo.w)), "v"(make_xu2(hi.x, hi.y)),
                    "v"(make_xu2(hi.z, hi.w))
                 : "memory");
  };
  // proj_in epilogue of tile o: + bias -> h (staged, kept as B fragments hf[2o], hf[2o + 1], LN1 sums)
  auto epi_in = [&](int o, v16f& acc, const v4f (&bb)[4]) {
    mfma_fence16(acc, acc);
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      v[i] = acc[i] + bb[i >> 2][i & 3];
      rsum += v[i];
      rsq = __builtin_fmaf(v[i], v[i], rsq);
    }
    const uint4 lo = pack8(v), hi = pack8(v + 8);
    hf[2 * o] = __builtin_bit_cast(v8s, lo);
    hf[2 * o + 1] = __builtin_bit_cast(v8s, hi);
    stage(o, lo, hi);
  };
  // QKV epilogue of tile t: y = rstd (acc - mean colsum) + b'
  auto epi_qkv = [&](int t, v16f& acc, const v4f (&cs)[4], const v4f (&bq)[4]) {
    mfma_fence16(acc, acc);
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __builtin_fmaf(rstd, acc[i] - mean * cs[i >> 2][i & 3], bq[i >> 2][i & 3]);
    stage(t, pack8(v), pack8(v + 8));
  };
  // MFMA chain of the tile in `sb` whose first D fragment reads are in wf[0..D-1]
  auto chain = [&](unsigned sb, v8s (&wf)[XKS], const v8s (&bf)[XKS], v16f& acc, auto dconst) {
    constexpr int D = decltype(dconst)::value;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < XKS; ++ks) {
      xin_wait(ks + D - 1 < XKS ? D - 1 : XKS - 1 - ks, wf[ks]);
      if constexpr ((PROBE & 2) != 0) asm volatile("" ::"v"(wf[ks]), "v"(bf[ks]));
      else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], bf[ks], acc, 0, 0, 0);
      if (ks + D < XKS) {
        const int k1 = ks + D;
        xin_ld(wf[k1], sb + wo[k1 & 3] + (unsigned)((k1 >> 2) * 4096));
      }
    }
  };
  auto first_reads = [&](unsigned sb, v8s (&wf)[XKS], auto dconst) {
    constexpr int D = decltype(dconst)::value;
#pragma unroll
    for (int ks = 0; ks < D; ++ks) xin_ld(wf[ks], sb + wo[ks & 3] + (unsigned)((ks >> 2) * 4096));
  };
  auto read_bias = [&](int o, v4f (&bb)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) xin_ldf(bb[q], bi0 + (unsigned)((32 * o + 8 * q + 4 * h) * 4));
  };
  auto read_qkv_tables = [&](int p, v4f (&cs)[4], v4f (&bq)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) xin_ldf(cs[q], cs0 + (unsigned)((32 * p + 8 * q + 4 * h) * 4));
#pragma unroll
    for (int q = 0; q < 4; ++q) xin_ldf(bq[q], bq0 + (unsigned)((32 * p + 8 * q + 4 * h) * 4));
  };
  using DIN = std::integral_constant<int, 8>;    // proj_in: x and h fragments both live
  using DQKV = std::integral_constant<int, 12>;  // QKV: x fragments dead, deeper read-ahead

  // table reads of the tile whose epilogue runs now are issued BEFORE this
  // tile's first fragment reads, so a counted lgkmcnt(D) retires just them
  auto wait_tables = [&](v4f (&x)[4], v4f (&y)[4], auto dconst) {
    constexpr int D = decltype(dconst)::value;
    asm volatile("s_waitcnt lgkmcnt(%8)"
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3])
                 : "n"(D));
  };
  auto wait_table = [&](v4f (&x)[4], auto dconst) {  // one array: naming it twice in one asm would copy it
    constexpr int D = decltype(dconst)::value;
    asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]) : "n"(D));
  };
  v16f acc_prev;
  // ---- proj_in: ten tiles, unrolled (tile o's epilogue runs in tile o + 1) ----
#pragma unroll
  for (int o = 0; o < XTI; ++o) {
    barrier();
    if constexpr ((PROBE & 16) != 0) {
      hf[2 * o] = v8s{0, 0, 0, 0, 0, 0, 0, 0};
      hf[2 * o + 1] = v8s{0, 0, 0, 0, 0, 0, 0, 0};
      acc_prev = v16f{};
      continue;
    }
    v8s wf[XKS];
    const unsigned sb = slot(o);
    v4f bb[4];
    if (o > 0) read_bias(o - 1, bb);
    first_reads(sb, wf, DIN{});
    if (o > 0) {
      wait_table(bb, DIN{});
      epi_in(o - 1, acc_prev, bb);
    }
    v16f acc;
    chain(sb, wf, xf, acc, DIN{});
    acc_prev = acc;
  }

  // ---- QKV: thirty tiles (tile t's epilogue runs in tile t + 1) ----
#pragma unroll 1
  for (int p = 0; p < XQ / 32; ++p) {
    const int t = XTI + p;
    barrier();
    v8s wf[XKS];
    const unsigned sb = slot(t);
    v4f cs[4], bq[4];
    if (p == 0) read_bias(XTI - 1, cs);
    else read_qkv_tables(p - 1, cs, bq);
    first_reads(sb, wf, DQKV{});
    if (p == 0) {  // the last proj_in tile, then the rows' LN1 statistics (the other half-row sits in lane l ^ 32)
      wait_table(cs, DQKV{});
      epi_in(XTI - 1, acc_prev, cs);
      rsum += __shfl_xor(rsum, 32, 64);
      rsq += __shfl_xor(rsq, 32, 64);
      mean = rsum * (1.0f / XC);
      rstd = rsqrtf(fmaxf(rsq * (1.0f / XC) - mean * mean, 0.f) + a.eps);
    } else {
      wait_tables(cs, bq, DQKV{});
      epi_qkv(t - 1, acc_prev, cs, bq);
    }
    v16f acc;
    chain(sb, wf, hf, acc, DQKV{});
    acc_prev = acc;
  }
  barrier();  // barrier XT: the last tile's epilogue, then one more round for the store waves
  {
    v4f cs[4], bq[4];
    read_qkv_tables(XQ / 32 - 1, cs, bq);
    xin_waitf(cs);
    xin_waitf(bq);
    epi_qkv(XT - 1, acc_prev, cs, bq);
  }
  barrier();
}

CSK_DEBUG_EXPORT(xin)

static int g_xin_probe = 0;
CSK_API int csk_set_xin_probe(int p) {
  g_xin_probe = p;
  return 0;
}

// 1 when csk_xin_qkv takes this shape: C = 320 (QKV 960), whole 128-row
// workgroups inside one sample
CSK_API int csk_xin_qkv_ok(int M, int C, int rows_per_b, int G) {
  return (C == XC && M > 0 && rows_per_b > 0 && rows_per_b % XROWS == 0 && M % rows_per_b == 0 && G > 0 &&
          XC % G == 0)
             ? 1
             : 0;
}

// h = proj_in(GroupNorm(x)), qkv = LN1(h) Wqkv^T (weights packed by ops.pack_xin_qkv; stat from csk_gn_finalize)
CSK_API int csk_xin_qkv(void* hout, void* qkv, const void* x, const void* stat, const void* gamma, const void* beta,
                        int G, const void* w, const void* bi, const void* colsum, const void* bq, int M, int rows_per_b,
                        float eps, hipStream_t stream) {
  if (!csk_xin_qkv_ok(M, XC, rows_per_b, G) || !hout || !qkv || !x || !stat || !gamma || !w || !colsum)
    return (int)hipErrorInvalidValue;
  XinArgs a;
  a.x = (const bf16_t*)x;
  a.stat = (const float*)stat;
  a.gamma = (const bf16_t*)gamma;
  a.beta = (const bf16_t*)beta;
  a.w = (const bf16_t*)w;
  a.bi = (const float*)bi;
  a.colsum = (const float*)colsum;
  a.bq = (const float*)bq;
  a.h = (bf16_t*)hout;
  a.qkv = (bf16_t*)qkv;
  a.x_end = a.x + (size_t)M * XC;
  a.w_end = a.w + (size_t)XT * XSLOT;
  a.M = M;
  a.rows_per_b = rows_per_b;
  a.G = G;
  a.eps = eps;
  const dim3 grid((M + XROWS - 1) / XROWS);
  switch (g_xin_probe) {
    case 1: xin_qkv_kernel<1><<<grid, XTHREADS, 0, stream>>>(a); break;
    case 2: xin_qkv_kernel<2><<<grid, XTHREADS, 0, stream>>>(a); break;
    case 4: xin_qkv_kernel<4><<<grid, XTHREADS, 0, stream>>>(a); break;
    case 7: xin_qkv_kernel<7><<<grid, XTHREADS, 0, stream>>>(a); break;
    case 8: xin_qkv_kernel<8><<<grid, XTHREADS, 0, stream>>>(a); break;
    case 15: xin_qkv_kernel<15><<<grid, XTHREADS, 0, stream>>>(a); break;
    case 16: xin_qkv_kernel<16><<<grid, XTHREADS, 0, stream>>>(a); break;
    default: xin_qkv_kernel<0><<<grid, XTHREADS, 0, stream>>>(a); break;
  }
  return (int)hipGetLastError();
}
