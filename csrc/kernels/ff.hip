// Fused transformer feed-forward of an SD UNet block at C = 320 (SURVEY K10 +
// K11; reference call site swarm/diffusion/diffusion_func.py:96, the diffusers
// BasicTransformerBlock ff path):
//
//   y = x + W2 (GEGLU(W1 LN3(x) + b1)) + b2,   GEGLU(v | g) = v * gelu(g)
//
// ONE kernel instead of the LN-fused GEGLU GEMM [M, 2560] -> the [M, 1280]
// intermediate in HBM -> the down-projection GEMM with the residual: the
// intermediate never leaves the registers, and every weight byte streamed into
// LDS is used by 128 rows (4 waves x 32 rows).
//
// Wave layout: each of the 4 waves (one per SIMD) owns 32 rows end to end and
// runs the matrix cores on 32x32x16 MFMAs whose B operand (the N side) is its
// 32 rows:
//   * LN3(x) of its rows lives in registers as 20 B fragments (lane: row l%32,
//     channels 16 ks + 8 h .. +7, h = l / 32), normalised in the prologue;
//   * H^T = W1 x^T for one W1 tile of 32 rows — 16 GEGLU value rows followed by
//     the 16 gate rows of the same 16 intermediates (packed that way on the
//     host) — leaves value and gate of intermediates {4h + r, 8 + 4h + r} in the
//     SAME lane (accumulator rows 8q + 4h + r, q = 0, 1 values, 2, 3 gates), so
//     GEGLU is in-lane and its 8 results are exactly the B fragment of the
//     down-projection's 16-intermediate k-step (k-slot order {4h + j, 8 + 4h + j};
//     W2's columns are permuted the same way on the host, so its A fragments are
//     plain 16-byte reads);
//   * out^T = W2 H^T accumulates the 32 x 320 output in 10 32x32 tiles
//     (160 accumulator registers) over all 1280 intermediates.
// Weights stream through an LDS ring of 7 slots x 20 KB by LDS-DMA
// (global_load_lds, 16 B per lane, XOR-swizzled images, per-lane source
// address): per 32 intermediates the slots are [W1 tile a][W1 tile b][W2 slice
// 320 x 32], each 20 MFMAs per wave; six slots stay in flight, one barrier per
// slot frees the slot just consumed for the next DMA (counted vmcnt waits).
// The MFMA floor is 32 us per 128 rows (2400 MFMAs x 32 cycles per wave).
#include "common.h"

#include "attn_tile.h"

typedef __attribute__((address_space(1))) const void* ff_gptr_t;
typedef __attribute__((address_space(3))) void* ff_lptr_t;

struct FfArgs {
  const bf16_t* x;      // [M][C]: LayerNorm input and residual
  const bf16_t* gamma;  // [C] LN3 weight
  const bf16_t* beta;   // [C] LN3 bias (or null)
  const bf16_t* w1;     // [I/16][C/64][32][64]: per 16 intermediates 16 value rows, then their 16 gate
                        // rows, as swizzled [32][64] sub-images (ops.pack_ff_fused)
  const float* b1;      // [I/16][32] fp32, same row order (or null)
  const bf16_t* w2;     // [I/32][C/32][32][32]: swizzled [32 out rows][32 intermediates] images, every
                        // 16-column block ordered 0-3, 8-11, 4-7, 12-15
  const bf16_t* b2;     // [C] (or null)
  bf16_t* y;            // [M][C]
  const bf16_t* x_end;  // CSK_DEBUG bounds
  const bf16_t* w1_end;
  const bf16_t* w2_end;
  int M, I;
  float eps;
};

#define FF_WAVES 4
#define FF_ROWS (32 * FF_WAVES)
#define FF_SLOT 10240  // elements (20 KB) per ring slot
#define FF_NSLOT 7
#define FF_PIECES (FF_SLOT / 512)       // 1 KB DMA pieces per slot
#define FF_PPW (FF_PIECES / FF_WAVES)   // pieces per wave per slot
#define FF_IMAX 1280                    // b1 staged in LDS: 2 * I floats

template <int N>
__device__ __forceinline__ void ff_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void ff_ld(v8s& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
__device__ __forceinline__ void ff_ldf(v4f& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
// wait until at most n LDS reads issued after the one that fills d are outstanding
__device__ __forceinline__ void ff_wait(int n, v8s& d) {
  switch (n) {
    case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(d)); break;
    case 1: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(d)); break;
    case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(d)); break;
    case 3: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(d)); break;
    case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(d)); break;
    case 5: asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(d)); break;
    case 6: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(d)); break;
    default: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(d)); break;
  }
}
template <int N>
__device__ __forceinline__ void ff_waitf(v4f (&b)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]) : "n"(N));
}

// PROBE (profiling builds, wrong results by design; csk_set_ff_probe): 1 = no
// MFMAs, 2 = no GEGLU math, 4 = no weight DMA after the prologue (slots reused)
template <int C, int PROBE = 0>
__global__ __launch_bounds__(FF_WAVES * 64, 1) void ff_geglu_kernel(const FfArgs a) {
  constexpr int KS = C / 16;   // 16-deep k-steps of the GEGLU projection
  constexpr int NOT = C / 32;  // 32-wide output tiles
  constexpr int SI = C / 64;   // [32][64] sub-images of a W1 tile
  static_assert(32 * C == FF_SLOT && 32 * C == NOT * 1024, "one W1 tile / one W2 slice per slot");
  static_assert(FF_PIECES % FF_WAVES == 0, "pieces per wave");
  __shared__ __attribute__((aligned(16))) bf16_t ring[FF_NSLOT * FF_SLOT];
  // b1 in LDS: no global load inside the main loop (its compiler-inserted wait
  // would be a vmcnt that drains every LDS-DMA issued before it)
  __shared__ __attribute__((aligned(16))) float s_b1[2 * FF_IMAX];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.x * FF_ROWS;
  const int row = m0 + wid * 32 + r32;
  const bool row_ok = row < a.M;
  const int I = a.I;
  const int nchunk = I / 32;
  const int nslots = 3 * nchunk;

  // ---- LDS-DMA: this wave's piece i (of FF_PPW) of ring slot t ----
  auto dma_piece = [&](int t, int i) {
    bf16_t* base = ring + (t % FF_NSLOT) * FF_SLOT;
    const int c = t / 3, kind = t - 3 * c;
    const int p = wid + FF_WAVES * i;
    // the packed weights ARE the slot images (ops.pack_ff_fused): a slot is
    // one contiguous 20 KB run, piece p its p-th KB
    const bf16_t* src = (kind < 2 ? a.w1 + (size_t)(2 * c + kind) * FF_SLOT : a.w2 + (size_t)c * FF_SLOT) +
                        512 * p + 8 * lane;
    CSK_DCHECK(src + 8 <= (kind < 2 ? a.w1_end : a.w2_end), 91, t, I);
    __builtin_amdgcn_global_load_lds((ff_gptr_t)src, (ff_lptr_t)(base + 512 * p), 16, 0, 0);
  };
  auto dma_slot = [&](int t) {
#pragma unroll
    for (int i = 0; i < FF_PPW; ++i) dma_piece(t, i);
  };

  // ---- prologue: the rows, b1, then six slots in flight while the rows normalise ----
  constexpr int LEAD = FF_NSLOT - 2;  // slots issued before the first barrier
  uint4 xu[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    xu[ks] = make_uint4(0, 0, 0, 0);
    if (row_ok) {
      CSK_DCHECK(a.x + (size_t)row * C + 16 * ks + 8 * h + 8 <= a.x_end, 93, row, a.M);
      xu[ks] = *reinterpret_cast<const uint4*>(a.x + (size_t)row * C + 16 * ks + 8 * h);
    }
  }
  uint4 gmu[KS], btu[KS];  // (loaded before the DMAs: a wait for them then leaves the DMAs in flight)
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    gmu[ks] = *reinterpret_cast<const uint4*>(a.gamma + 16 * ks + 8 * h);
    btu[ks] = a.beta ? *reinterpret_cast<const uint4*>(a.beta + 16 * ks + 8 * h) : make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < 2 * I; i += FF_WAVES * 64) s_b1[i] = a.b1 ? a.b1[i] : 0.f;
  for (int t = 0; t < LEAD && t < nslots; ++t) dma_slot(t);

  v8s xf[KS];
  float mean = 0.f, rstd = 0.f;
  {
    float f[KS][8];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) unpack8(xu[ks], f[ks]);
    float s = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[ks][j];
    s += __shfl_xor(s, 32, 64);
    mean = s * (1.0f / C);
    float q = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[ks][j] - mean;
        q = __builtin_fmaf(d, d, q);
      }
    q += __shfl_xor(q, 32, 64);
    rstd = rsqrtf(q * (1.0f / C) + a.eps);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      float gm[8], bt[8];
      unpack8(gmu[ks], gm);
      unpack8(btu[ks], bt);
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = __builtin_fmaf((f[ks][j] - mean) * rstd, gm[j], bt[j]);
      xf[ks] = __builtin_bit_cast(v8s, pack8(v));
    }
  }

  v16f out[NOT];
#pragma unroll
  for (int o = 0; o < NOT; ++o)
#pragma unroll
    for (int i = 0; i < 16; ++i) out[o][i] = 0.f;

  // Ring protocol (7 slots, one barrier per PAIR of slots): the barrier in
  // front of an even slot s waits for this wave's pieces of s and s + 1
  // (slots s + 2 .. s + 4 stay in flight: vmcnt(15)) and retires its LDS
  // reads; after it every wave is done with s - 2 and s - 1, so slot u issues
  // the DMA of slot u + 5 into ring position (u - 2) % 7, one piece after every
  // fourth MFMA (the issue cost hides under the matrix pipe).
  auto enter_pair = [&](int t) {
    if constexpr ((PROBE & 4) == 0) {
      if (t + 4 < nslots) ff_vmcnt<FF_PPW * 3>();
      else ff_vmcnt<0>();
    } else {
      ff_vmcnt<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  auto dma_hook = [&](int t, int k) {  // after MFMA k of slot t: piece k / 4 of slot t + 5
    if constexpr ((PROBE & 4) == 0) {
      if ((k & 3) == 3 && t + 5 < nslots) dma_piece(t + 5, k >> 2);
    }
  };

  // Fragment reads are inline asm: hipcc would otherwise see LDS reads of the
  // array the DMAs write and put an s_waitcnt vmcnt(0) — every slot in flight —
  // in front of the first one after each DMA issue.  The waits are counted by
  // hand (LDS reads return in order) and name the fragment they wait for.
  const unsigned ring0 = (unsigned)(size_t)(ff_lptr_t)(void*)ring;
  const unsigned b1base = (unsigned)(size_t)(ff_lptr_t)(void*)s_b1 + (unsigned)(16 * h);
  unsigned w1o[4];  // byte offset of k-step (4 si + j)'s A fragment inside sub-image si
#pragma unroll
  for (int j = 0; j < 4; ++j) w1o[j] = 2u * (unsigned)at_off64(r32, 2 * j + h);
  unsigned w2o[2];  // ... of W2 k-step s inside an output tile's [32][32] image
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) w2o[s2] = 2u * (unsigned)(r32 * 32 + (((2 * s2 + h) ^ ((r32 >> 2) & 3)) << 3));
  auto slot_base = [&](int t) -> unsigned {
    return ring0 + (unsigned)(((PROBE & 4) ? (t % 3) : (t % FF_NSLOT)) * FF_SLOT * 2);
  };
  constexpr int D = 6;  // fragment reads in flight ahead of the MFMA that consumes them
  constexpr int GAT = 2;  // the previous tile's GEGLU runs after this MFMA of the next slot

  // GEGLU in-lane: H of intermediates {4h + j, 8 + 4h + j} as one B fragment.
  // Accumulator slot j = 4q + r: value rows q = 0, 1; their gates sit 16 rows
  // (two q) further.  bq (b1 of the tile) was read in the tile's own slot and
  // has arrived (every read of that slot was waited for): the empty asm only
  // keeps its uses behind that wait.
  auto geglu = [&](v16f& acc, v4f (&bq)[4]) -> v8s {
    asm volatile("" : "+v"(bq[0]), "+v"(bq[1]), "+v"(bq[2]), "+v"(bq[3]));
    mfma_fence16(acc, acc);
    float hv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = acc[j] + bq[j >> 2][j & 3];
      const float g = acc[j + 8] + bq[2 + (j >> 2)][j & 3];
      if constexpr ((PROBE & 2) != 0) hv[j] = v + g;
      else hv[j] = v * gelu_geglu(g);
    }
    return __builtin_bit_cast(v8s, pack8(hv));
  };

  // acc = W1 tile tt (slot t) x^T: 20 MFMAs; bq <- b1 of the tile.  `pend`
  // (if set): the previous tile's GEGLU, run after MFMA GAT of this slot.
  auto w1_tile = [&](int t, int tt, v16f& acc, v4f (&bq)[4], v16f* pacc, v4f (*pbq)[4], v8s* pout) {
    const unsigned sb = slot_base(t);
#pragma unroll
    for (int q = 0; q < 4; ++q) ff_ldf(bq[q], b1base + (unsigned)((tt * 32 + 8 * q) * 4));
    v8s wf[KS];
#pragma unroll
    for (int ks = 0; ks < D; ++ks) ff_ld(wf[ks], sb + w1o[ks & 3] + (unsigned)((ks >> 2) * 4096));
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      ff_wait(ks + D - 1 < KS ? D - 1 : KS - 1 - ks, wf[ks]);
      if constexpr ((PROBE & 1) != 0) asm volatile("" ::"v"(wf[ks]), "v"(xf[ks]));
      else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks], xf[ks], acc, 0, 0, 0);
      if (ks + D < KS) {
        const int k1 = ks + D;
        ff_ld(wf[k1], sb + w1o[k1 & 3] + (unsigned)((k1 >> 2) * 4096));
      }
      dma_hook(t, ks);
      if (ks == GAT && pacc) *pout = geglu(*pacc, *pbq);
    }
  };

  // out^T += W2 slice (slot t) [H_a; H_b]^T: 2 k-steps x 10 output tiles;
  // H_b = GEGLU(acc_b) is formed after MFMA GAT (the first 10 need only H_a)
  auto w2_slice = [&](int t, const v8s& ha, v16f& acc_b, v4f (&bqb)[4]) {
    const unsigned sb = slot_base(t);
    constexpr int NR = 2 * NOT;
    v8s wf[NR];
    v8s hb;
#pragma unroll
    for (int i = 0; i < D; ++i) ff_ld(wf[i], sb + w2o[i / NOT] + (unsigned)((i % NOT) * 2048));
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      ff_wait(i + D - 1 < NR ? D - 1 : NR - 1 - i, wf[i]);
      const int o = i % NOT;
      if constexpr ((PROBE & 1) != 0) asm volatile("" ::"v"(wf[i]), "v"(ha), "v"(hb));
      else out[o] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[i], i < NOT ? ha : hb, out[o], 0, 0, 0);
      if (i + D < NR) {
        const int i1 = i + D;
        ff_ld(wf[i1], sb + w2o[i1 / NOT] + (unsigned)((i1 % NOT) * 2048));
      }
      dma_hook(t, i);
      if (i == GAT) hb = geglu(acc_b, bqb);
    }
  };

  // two chunks (6 slots, 3 pairs) per trip: barriers in front of t, t + 2, t + 4
  for (int c = 0; c < nchunk; c += 2) {
    const int t = 3 * c;
    v16f acc_a, acc_b;
    v4f bqa[4], bqb[4];
    v8s ha;
    enter_pair(t);
    w1_tile(t, 2 * c, acc_a, bqa, nullptr, nullptr, nullptr);
    w1_tile(t + 1, 2 * c + 1, acc_b, bqb, &acc_a, &bqa, &ha);
    enter_pair(t + 2);
    w2_slice(t + 2, ha, acc_b, bqb);
    w1_tile(t + 3, 2 * c + 2, acc_a, bqa, nullptr, nullptr, nullptr);
    enter_pair(t + 4);
    w1_tile(t + 4, 2 * c + 3, acc_b, bqb, &acc_a, &bqa, &ha);
    w2_slice(t + 5, ha, acc_b, bqb);
  }

  // ---- epilogue: + b2 + residual x; accumulator rows 32 o + 8 q + 4 h + r of row `row` ----
  if (!row_ok) return;
  uint2 xr[NOT][4], br[NOT][4];
#pragma unroll
  for (int o = 0; o < NOT; ++o)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 32 * o + 8 * q + 4 * h;
      xr[o][q] = *reinterpret_cast<const uint2*>(a.x + (size_t)row * C + n);
      br[o][q] = a.b2 ? *reinterpret_cast<const uint2*>(a.b2 + n) : make_uint2(0, 0);
    }
#pragma unroll
  for (int o = 0; o < NOT; ++o)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 32 * o + 8 * q + 4 * h;
      const uint2 u = xr[o][q], ub = br[o][q];
      const float rv[4] = {bf2f((bf16_t)(u.x & 0xffff)), bf2f((bf16_t)(u.x >> 16)), bf2f((bf16_t)(u.y & 0xffff)),
                           bf2f((bf16_t)(u.y >> 16))};
      const float bb[4] = {bf2f((bf16_t)(ub.x & 0xffff)), bf2f((bf16_t)(ub.x >> 16)), bf2f((bf16_t)(ub.y & 0xffff)),
                           bf2f((bf16_t)(ub.y >> 16))};
      uint2 w;
      w.x = pack2(out[o][4 * q] + bb[0] + rv[0], out[o][4 * q + 1] + bb[1] + rv[1]);
      w.y = pack2(out[o][4 * q + 2] + bb[2] + rv[2], out[o][4 * q + 3] + bb[3] + rv[3]);
      *reinterpret_cast<uint2*>(a.y + (size_t)row * C + n) = w;
    }
}

CSK_DEBUG_EXPORT(ff)

static int g_ff_probe = 0;
CSK_API int csk_set_ff_probe(int p) {
  g_ff_probe = p;
  return 0;
}

// 1 when csk_ff_geglu takes this shape
CSK_API int csk_ff_geglu_ok(int M, int C, int I) {
  return (C == 320 && I > 0 && I % 64 == 0 && I <= FF_IMAX && M > 0) ? 1 : 0;  // chunk pairs
}

// y[M][C] = x + W2 GEGLU(W1 LN(x) + b1) + b2 (weights packed by ops.pack_ff_fused).
// y must not alias x.
CSK_API int csk_ff_geglu(void* y, const void* x, const void* gamma, const void* beta, const void* w1, const void* b1,
                         const void* w2, const void* b2, int M, int C, int I, float eps, hipStream_t stream) {
  if (!csk_ff_geglu_ok(M, C, I) || !x || !y || !gamma || !w1 || !w2 || x == y) return (int)hipErrorInvalidValue;
  FfArgs a;
  a.x = (const bf16_t*)x;
  a.gamma = (const bf16_t*)gamma;
  a.beta = (const bf16_t*)beta;
  a.w1 = (const bf16_t*)w1;
  a.b1 = (const float*)b1;
  a.w2 = (const bf16_t*)w2;
  a.b2 = (const bf16_t*)b2;
  a.y = (bf16_t*)y;
  a.x_end = a.x + (size_t)M * C;
  a.w1_end = a.w1 + (size_t)2 * I * C;
  a.w2_end = a.w2 + (size_t)C * I;
  a.M = M;
  a.I = I;
  a.eps = eps;
  const dim3 grid((M + FF_ROWS - 1) / FF_ROWS);
  switch (g_ff_probe) {
    case 1: ff_geglu_kernel<320, 1><<<grid, FF_WAVES * 64, 0, stream>>>(a); break;
    case 2: ff_geglu_kernel<320, 2><<<grid, FF_WAVES * 64, 0, stream>>>(a); break;
    case 4: ff_geglu_kernel<320, 4><<<grid, FF_WAVES * 64, 0, stream>>>(a); break;
    default: ff_geglu_kernel<320><<<grid, FF_WAVES * 64, 0, stream>>>(a); break;
  }
  return (int)hipGetLastError();
}
