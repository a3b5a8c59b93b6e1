// Persistent stream-K flash attention, d = 64 or 40, bf16 in / out (SURVEY K7:
// the UNet self-attention at S = 256 .. 16384, SD2.1 / SDXL heads of 64, the
// SD1.5 / ControlNet 64x64-level heads of 40).
//
// d = 40 runs the same kernel on the d = 64 LDS images with the head zero-padded
// in LDS: the K / V / Q DMA lanes whose 16-byte source chunk lies past the head
// (chunks 5-7 of a row) are masked off, their LDS slots are zeroed once at kernel
// entry and never written again (a chunk's slot depends only on the row within
// the tile), Q's padded k-step half is zeroed in registers.  QK^T then runs 3
// k-steps instead of 4 and only d < 40 is stored; softmax / PV / merge are the
// d = 64 code (profiles/attn_fa_d40_r6.txt).
//
// Why a new kernel (attn32_kernel in attention.hip is the design it replaces
// for these shapes): the PMC of the UNet step measured 12.5 VALU instructions
// per MFMA in attn32 (profiles/pmc_unet_step_r7i_1.txt) — register staging of
// K / V (global -> VGPR -> ds_write), per-block LDS address math, a
// 32-register -max accumulator init per block — and its grid of 128-row
// workgroups leaves the chip 17 % idle in the last round at B8 H5 S4096 (1280
// workgroups on 512 slots), more at CFG batch 2.
//
// Structure (MI355X / CDNA4 first):
//   * ONE 8-wave workgroup per CU (2 waves per SIMD), persistent: grid = #CUs.
//     The work is the flat list of (256-row query block, 64-key tile) units;
//     worker w owns the contiguous range [U w / G, U (w+1) / G) — stream-K, so
//     every CU gets the same number of key tiles whatever B, H, S are (no tail
//     round; the batch-1 grids need no separate split-KV path).
//   * A query block cut between workers is merged in-kernel: a worker whose
//     range STARTS inside a block (it processes that piece first) writes its
//     unnormalised (O, m, l) to its own workspace slot and publishes a flag
//     (agent-scope release); the worker holding the block's first tile (it
//     reaches it last) acquires, merges and stores (cdna_hip_programming.md
//     §6 Guideline 16; the owner resets the flag; bounded spins).
//   * K / V tiles arrive by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave
//     instruction: each wave moves 8 K rows + 8 V rows per tile) into an 8-slot
//     ring, five units ahead and across query-block seams; the XOR swizzle of
//     the LDS image (kv_off32 of attention.hip: conflict-free for the K
//     ds_read_b128 and the V ds_read_b64_tr_b16 patterns) is carried by the
//     per-lane SOURCE address.  Q arrives the same way into a per-wave region.
//     Waits are counted (`s_waitcnt vmcnt(n)` from a scalar issue counter),
//     barriers raw: one barrier per TWO key tiles (the waves drift apart by up
//     to a tile between barriers, which spreads their DMA issue and MFMA
//     phases; 4-slot ring with a barrier per tile: 243-248 us, this: 234 us at
//     B8 H5 S4096).
//   * Inline-asm adds of exp results use vadd_t (one wait state: the trans
//     forwarding hazard hipcc does not pad before inline asm); _build.py lints
//     the assembly for any trans result read by the next instruction.
//   * Every LDS address is a per-lane base fixed at kernel entry plus a
//     compile-time offset (the ring slot is one scalar add).
//   * Per wave: 32 query rows.  S^T = K Q^T and O^T = V^T P^T on
//     v_mfma_f32_32x32x16_bf16 (query on the lane, keys in the accumulator
//     registers; P^T is the S^T accumulator converted in place).  Software
//     pipeline: QK^T of tile t+1 is issued beside the exp / convert of tile t,
//     PV of tile t beside the row sum of t and the row max of t+1.
//   * Softmax without a per-score subtract: Q is pre-scaled by scale*log2(e)
//     and p = exp2(s - m_ref) with a LAZY reference m_ref that starts at 0 and
//     moves only when a tile's row max exceeds it by 64 (T13-style deferral:
//     bf16 P keeps its relative precision at any magnitude, fp32 O / l stay far
//     from overflow below 2^64 * 2^14).  While every row of a wave has
//     m_ref == 0 (the usual case) the exponent is s itself: one v_exp per
//     score.  A first-tile row max below -40 also moves m_ref (no underflow).
#include <type_traits>

#include "common.h"

namespace {

constexpr int FA_WAVES = 8;
constexpr int FA_ROWS = FA_WAVES * 32;  // query rows per block
constexpr int FA_SLOT = 16384;          // one 64-key tile: K (8 KiB) + V (8 KiB)
constexpr int FA_NSLOT = 8;             // K/V ring slots (unit v -> slot v & 7)
constexpr int FA_LEAD = 5;              // units of K/V DMA in flight ahead of the compute
constexpr int FA_BE = 2;                // one workgroup barrier every FA_BE units
// WAR: DMA(v) (issued at unit v - LEAD, after that unit's barrier or the one
// before it) overwrites unit v - NSLOT's slot, whose last reader (its PV) ran
// before that barrier
static_assert(FA_NSLOT >= FA_LEAD + FA_BE, "ring too short for the barrier spacing");
static_assert(FA_LEAD > FA_BE, "a barrier must find the next FA_BE units' DMA issued");
static_assert((FA_NSLOT & (FA_NSLOT - 1)) == 0, "slot index is a mask");
constexpr int FA_PART = FA_WAVES * 9 * 64 * 4;      // floats per worker slot: 8 waves x 9 float4 x 64 lanes
constexpr float FA_THR_HI = 64.f;  // move m_ref when a tile's row max exceeds it by this (log2 units)
constexpr float FA_THR_LO = -40.f; // first-tile row max below m_ref + this: m_ref = that max

typedef __attribute__((address_space(3))) v4s fa_lds_v4s;
typedef unsigned int fa_u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const void* fa_gptr_t;
typedef __attribute__((address_space(3))) void* fa_lptr_t;

// swizzle of a 64-column (128-byte) bf16 row: 16-byte chunk c of row r at slot c ^ f(r)
__device__ __forceinline__ int fa_f(int row) { return ((row & 2) << 1) | ((row & 4) >> 1) | ((row & 8) >> 3); }

// n is wave-uniform (a scalar branch chain); a larger n than needed only waits longer
__device__ __forceinline__ void fa_vmcnt(int n) {
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (n == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
  else if (n == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
}

__device__ __forceinline__ void fa_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// ds_read_b64_tr_b16 as inline asm: hipcc treats the builtin's LDS access as
// unknown and waits vmcnt(0) (every LDS-DMA in flight) before it — which would
// drain the K / V ring each tile.  The caller waits lgkmcnt itself.
template <int OFF>
__device__ __forceinline__ void fa_tr(v4s& d, unsigned addr) {
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}

// x(lane) + x(lane ^ 32): the two lane halves of a query hold disjoint key halves
// (permlane32_swap returns {x[l], x[l^32]} in some order in every lane)
__device__ __forceinline__ float fa_pair_sum(float x) {
  const auto s = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

}  // namespace

struct FaArgs {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  bf16_t* o;
  int sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh;  // element strides (host checks < 2^31)
  int B, H, Sq, Skv;
  float sl2;        // softmax scale * log2(e)
  int nq;           // query blocks per (batch, head)
  int T;            // key tiles per block (Skv / 64)
  int U;            // units = B * H * nq * T
  float* part;      // [G][FA_PART] partial slots
  unsigned* flags;  // [G] published partials (the owner resets them)
  unsigned* err;    // [1] spins that gave up (never expected)
  unsigned long long* dbg;  // PROBE & 128: per-wave phase cycle sums [G][8 waves][8]
};

// in-kernel stamp (diagnostic builds only: its lgkmcnt(0) and fences forbid overlaps)
__device__ __forceinline__ unsigned long long fa_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int D, int PROBE = 0>
__global__ __launch_bounds__(512) void attn_fa_kernel(const FaArgs a) {
  static_assert(D == 64 || D == 40, "head dims 64 and 40");
  constexpr int NCH = D / 8;         // 16-byte chunks per row that carry data (8 / 5)
  constexpr int KS = (D + 15) / 16;  // QK^T k-steps (4 / 3)
  // (probe 256: the 4-slot ring of the first version, a barrier every unit)
  constexpr int NSLOT = (PROBE & 256) ? 4 : FA_NSLOT;
  constexpr int LEAD = (PROBE & 256) ? 3 : FA_LEAD;
  constexpr int QOFF = NSLOT * FA_SLOT;
  __shared__ __attribute__((aligned(16))) unsigned char smem[QOFF + FA_WAVES * 4096];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int fr = lane & 15, fg = lane >> 4;
  const int G = gridDim.x;
  const int w = xcd_remap(blockIdx.x, G);  // consecutive workers (adjacent unit ranges) share an XCD's L2
  const int U = a.U, T = a.T, nq = a.nq;
  const int u0 = (int)((long long)U * w / G), u1 = (int)((long long)U * (w + 1) / G);
  if (u0 >= u1) return;  // whole workgroup: no barrier is shared with anyone
  const float sl2 = a.sl2;

  // ---- per-lane constants ----
  const int lr = lane >> 3;                        // row of the 8-row DMA piece
  const int kvrow = 8 * wv + lr;                   // tile row this lane's DMA piece fetches
  const int kvch = (lane & 7) ^ fa_f(kvrow);       // source chunk that lands in this lane's slot
  const bool kv_on = D == 64 || kvch < NCH;         // (d = 40: chunks past the head stay zero)
  const unsigned k_lane = (unsigned)(kvrow * a.sks + kvch * 8) * 2u;  // byte offsets (32-bit: saddr + voffset)
  const unsigned v_lane = (unsigned)(kvrow * a.svs + kvch * 8) * 2u;
  int q_lane[4];                                   // Q piece i: local row 8 i + lr
#pragma unroll
  for (int i = 0; i < 4; ++i) q_lane[i] = ((lane & 7) ^ fa_f(8 * i + lr)) * 8;
  if constexpr (D != 64) {
    // zero the whole LDS once: the pad slots (source chunk >= NCH) are never
    // written by the masked DMA below; the barrier orders these stores before it
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (int i = tid; i < (int)(sizeof(smem) / 16); i += 512) reinterpret_cast<uint4*>(smem)[i] = z;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  const unsigned kv_dst = (unsigned)wv * 1024u;    // this wave's 1 KiB of a K or V tile
  const unsigned lds0 = (unsigned)(size_t)(fa_lptr_t)(void*)smem;  // LDS byte address of the array
  const unsigned q_base = QOFF + (unsigned)wv * 4096u;
  unsigned koff[4];  // K / Q fragment (row r, chunk 2 ds + hh) byte offsets
#pragma unroll
  for (int ds = 0; ds < 4; ++ds) koff[ds] = (unsigned)(r * 128 + (((2 * ds + hh) ^ fa_f(r)) << 4));
  unsigned voff[2][2];  // V^T fragment (ds_read_b64_tr_b16) byte offsets, [+8 rows][d-tile]
  {
    const int qq = fr >> 2, pp = fr & 3;
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int row0 = 8 * e + 4 * (fg >> 1) + qq;
        const int ch = 4 * dt + 2 * (fg & 1) + (pp >> 1);
        voff[e][dt] = (unsigned)(8192 + row0 * 128 + ((ch ^ fa_f(row0)) << 4) + (pp & 1) * 8);
      }
  }

  // ---- DMA stream (scalar bookkeeping, every wave identical) ----
  int issued = 0;             // LDS-DMA instructions this wave has issued
  int dma_u0 = 0;             // issue count right after DMA(u0) (prologue wait)
  int q_end = 0;              // issue count right after the latest Q DMA
  // position of the next unit to DMA, advanced incrementally (no divisions per tile)
  int d_tile, d_qb, d_h, d_b;
  {
    const int blk = u0 / T;
    d_tile = u0 - blk * T;
    const int bh = blk / nq;
    d_qb = blk - bh * nq;
    d_b = bh / a.H;
    d_h = bh - d_b * a.H;
  }
  auto dma_unit = [&](int v) {  // v == the next unit in order
    const char* kb = (const char*)(a.k + (size_t)(d_b * a.skb + d_h * a.skh) + (size_t)(d_tile * 64 * a.sks));
    const char* vb = (const char*)(a.v + (size_t)(d_b * a.svb + d_h * a.svh) + (size_t)(d_tile * 64 * a.svs));
    unsigned char* dst = smem + (v & (NSLOT - 1)) * FA_SLOT + kv_dst;
    if ((!(PROBE & 64) || v < u0 + 2) && kv_on) {
      __builtin_amdgcn_global_load_lds((fa_gptr_t)(kb + k_lane), (fa_lptr_t)dst, 16, 0, 0);
      __builtin_amdgcn_global_load_lds((fa_gptr_t)(vb + v_lane), (fa_lptr_t)(dst + 8192), 16, 0, 0);
    }
    issued += 2;
    if (v == u0) dma_u0 = issued;
    if (++d_tile == T) {
      d_tile = 0;
      if (++d_qb == nq) {
        d_qb = 0;
        if (++d_h == a.H) {
          d_h = 0;
          ++d_b;
        }
      }
    }
  };
  auto dma_q = [&](int blk) {
    const int bh = blk / nq, qb = blk - bh * nq;
    const int b = bh / a.H, h = bh - b * a.H;
    const bf16_t* qp = a.q + (size_t)(b * a.sqb + h * a.sqh);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = min(qb * FA_ROWS + wv * 32 + 8 * i + lr, a.Sq - 1);
      if (D == 64 || q_lane[i] < 8 * NCH)
        __builtin_amdgcn_global_load_lds((fa_gptr_t)(qp + (unsigned)(row * a.sqs + q_lane[i])),
                                         (fa_lptr_t)(smem + q_base + i * 1024), 16, 0, 0);
    }
    issued += 4;
    q_end = issued;
  };
  auto wait_issue = [&](int end) { fa_vmcnt(issued - end); };

  // ---- registers ----
  v8s qf[KS];
  v16f o[2];
  float mref = 0.f, lsum = 0.f;
  const v16f zero16 = {0.f};
  v16f cneg = zero16;  // -m_ref in every register: the QK^T chain's initial accumulator
                       // (scores come out relative to the reference: no per-score subtract)
  unsigned long long ph0 = 0, ph1 = 0, ph2 = 0, ph3 = 0, ph4 = 0, ph5 = 0, ph6 = 0, tl = 0;

  auto load_q = [&]() {  // this wave's 32 query rows -> B fragments, pre-scaled into log2 units
#pragma unroll
    for (int ds = 0; ds < KS; ++ds) {
      const uint4 raw = *reinterpret_cast<const uint4*>(smem + q_base + koff[ds]);
      float f[8];
      unpack8(raw, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= sl2;
      qf[ds] = __builtin_bit_cast(v8s, pack8(f));
      // (d = 40: the last k-step's upper half, chunk 5, is head padding; the Q
      // region's pad slots hold stale data of no row, so zero it here)
      if (D != 64 && 2 * ds + hh >= NCH) qf[ds] = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto qk = [&](int v, v16f (&s)[2]) {  // S^T of unit v's keys (its K tile is in LDS)
    const unsigned char* kb = smem + (v & (NSLOT - 1)) * FA_SLOT;
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int ds = 0; ds < KS; ++ds) {
        const v8s kf = *reinterpret_cast<const v8s*>(kb + kt * 4096 + koff[ds]);
        if constexpr ((PROBE & 8) != 0) {
          asm volatile("" ::"v"(kf), "v"(qf[ds]));
          if (ds == 0) s[kt] = zero16 + (float)kt;
        } else {
          s[kt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[ds], ds == 0 ? cneg : s[kt], 0, 0, 0);
        }
      }
    }
  };
  auto rowmax = [&](v16f (&s)[2]) {  // max over the query's 64 keys (both lane halves)
    mfma_fence16(s[0], s[1]);
    const v16f& x0 = s[0];
    const v16f& x1 = s[1];
    const float t0 = vmax3(x0[0], x0[1], x0[2]), t1 = vmax3(x0[3], x0[4], x0[5]);
    const float t2 = vmax3(x0[6], x0[7], x0[8]), t3 = vmax3(x0[9], x0[10], x0[11]);
    const float t4 = vmax3(x0[12], x0[13], x0[14]), t5 = vmax3(x0[15], x1[0], x1[1]);
    const float t6 = vmax3(x1[2], x1[3], x1[4]), t7 = vmax3(x1[5], x1[6], x1[7]);
    const float t8 = vmax3(x1[8], x1[9], x1[10]), t9 = vmax3(x1[11], x1[12], x1[13]);
    const float t10 = vmax3(x1[14], x1[15], x1[15]);
    const float m = vmax3(vmax3(t0, t1, t2), vmax3(t3, t4, t5), vmax3(vmax3(t6, t7, t8), t9, t10));
    const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
    return vmax3(__uint_as_float(x[0]), __uint_as_float(x[1]), m);
  };
  // new segment: reference for its first tile's scores (row max mb)
  // (the segment's first scores s were computed with cneg = 0)
  auto seg_init = [&](float mb, v16f (&s)[2]) {
    mref = (mb > FA_THR_HI || mb < FA_THR_LO) ? mb : 0.f;
    lsum = 0.f;
    o[0] = zero16;
    o[1] = zero16;
    if (__any(mref != 0.f)) {
      s[0] -= mref;
      s[1] -= mref;
      cneg = zero16 - mref;
    }
  };
  // the NEXT tile's row max mb (of s - m_ref) arrives while this tile's P is
  // in O: deferred rescale of O and l, and the next tile's scores re-referenced
  auto rescale = [&](float mb, v16f (&s)[2]) {
    const bool up = mb > FA_THR_HI;
    if (__any(up)) {
      const float d = up ? mb : 0.f;  // new reference - old
      const float alpha = __builtin_amdgcn_exp2f(-d);
      o[0] *= alpha;
      o[1] *= alpha;
      lsum *= alpha;
      s[0] -= d;
      s[1] -= d;
      mref += d;
      cneg = zero16 - mref;
    }
  };

  // ---- one unit: softmax + PV of unit u (scores in Sc, already relative to
  // m_ref), QK^T of unit u+1 into Sn ----
  // NEXT: u + 1 is in the same segment (its QK^T overlaps this unit's softmax)
  auto body = [&](int u, bool nxt, v16f (&Sc)[2], v16f (&Sn)[2]) {
    // QK^T of unit u+1 always (branch-free body: at a segment end or the range
    // end it multiplies the wrong Q or a stale slot and Sn is recomputed / unused)
    qk(u + 1, Sn);
    if constexpr ((PROBE & 512) != 0) {  // (A/B: the K / V DMA issued behind the QK^T MFMAs:
      if (u + LEAD < u1) dma_unit(u + LEAD);  //  248-252 vs 230-233 us at B8 H5 S4096, profiles/attn_fa_r5b.txt)
    }
    // V^T fragments of this unit (after the K reads of the QK^T above) (16 asm tr-reads: lo keys +0..3, hi
    // +8..11 of each 16-key step, [kt][st][dt]); their latency hides under the
    // QK^T / exp work below and one lgkmcnt wait naming them precedes the PV
    const unsigned vs = lds0 + (unsigned)((u & (NSLOT - 1)) * FA_SLOT);
    const unsigned va00 = vs + voff[0][0], va01 = vs + voff[0][1], va10 = vs + voff[1][0], va11 = vs + voff[1][1];
    v4s vl[2][2][2], vh[2][2][2];
    fa_tr<0 * 2048>(vl[0][0][0], va00); fa_tr<0 * 2048>(vh[0][0][0], va10);
    fa_tr<0 * 2048>(vl[0][0][1], va01); fa_tr<0 * 2048>(vh[0][0][1], va11);
    fa_tr<1 * 2048>(vl[0][1][0], va00); fa_tr<1 * 2048>(vh[0][1][0], va10);
    fa_tr<1 * 2048>(vl[0][1][1], va01); fa_tr<1 * 2048>(vh[0][1][1], va11);
    fa_tr<2 * 2048>(vl[1][0][0], va00); fa_tr<2 * 2048>(vh[1][0][0], va10);
    fa_tr<2 * 2048>(vl[1][0][1], va01); fa_tr<2 * 2048>(vh[1][0][1], va11);
    fa_tr<3 * 2048>(vl[1][1][0], va00); fa_tr<3 * 2048>(vh[1][1][0], va10);
    fa_tr<3 * 2048>(vl[1][1][1], va01); fa_tr<3 * 2048>(vh[1][1][1], va11);
    // exp (scores -> P), in place
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        Sc[kt][i] = (PROBE & 1) ? Sc[kt][i] : __builtin_amdgcn_exp2f(Sc[kt][i]);
    // row sum of P (this lane's half of the keys): 4 single-instruction chains
    float l4[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      l4[c] = vadd_t(Sc[0][c], Sc[0][c + 4]);  // (exp results: trans-hazard-safe adds)
      l4[c] = vadd(l4[c], vadd_t(Sc[0][c + 8], Sc[0][c + 12]));
      l4[c] = vadd(l4[c], vadd_t(Sc[1][c], Sc[1][c + 4]));
      l4[c] = vadd(l4[c], vadd_t(Sc[1][c + 8], Sc[1][c + 12]));
    }
    lsum = vadd(lsum, vadd(vadd(l4[0], l4[1]), vadd(l4[2], l4[3])));
    v8s pf[2][2];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        const int o8 = 8 * st;
        pf[kt][st] = __builtin_bit_cast(
            v8s, make_uint4(pack2(Sc[kt][o8 + 0], Sc[kt][o8 + 1]), pack2(Sc[kt][o8 + 2], Sc[kt][o8 + 3]),
                            pack2(Sc[kt][o8 + 4], Sc[kt][o8 + 5]), pack2(Sc[kt][o8 + 6], Sc[kt][o8 + 7])));
      }
    // PV: O^T += V^T P^T
    if constexpr ((PROBE & 128) != 0) { const auto t = fa_stamp(); ph3 += t - tl; tl = t; }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(vl[0][0][0]), "+v"(vh[0][0][0]), "+v"(vl[0][0][1]), "+v"(vh[0][0][1]),
                   "+v"(vl[0][1][0]), "+v"(vh[0][1][0]), "+v"(vl[0][1][1]), "+v"(vh[0][1][1]),
                   "+v"(vl[1][0][0]), "+v"(vh[1][0][0]), "+v"(vl[1][0][1]), "+v"(vh[1][0][1]),
                   "+v"(vl[1][1][0]), "+v"(vh[1][1][0]), "+v"(vl[1][1][1]), "+v"(vh[1][1][1]));
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          const v4s lo = vl[kt][st][dt], hi = vh[kt][st][dt];
          const v8s vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if constexpr ((PROBE & 4) != 0) {
            asm volatile("" ::"v"(vf), "v"(pf[kt][st]));
          } else {
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf[kt][st], o[dt], 0, 0, 0);
          }
        }
    if constexpr ((PROBE & 128) != 0) { const auto t = fa_stamp(); ph4 += t - tl; tl = t; }
    const float mb = rowmax(Sn);
    if (nxt) rescale(mb, Sn);
    if constexpr ((PROBE & 128) != 0) { const auto t = fa_stamp(); ph5 += t - tl; tl = t; }
  };

  // ---- epilogues ----
  auto store_o = [&](int blk) {  // normalise and store this wave's 32 rows
    const float l = fa_pair_sum(lsum);
    const float inv = l > 0.f ? __builtin_amdgcn_rcpf(l) : 0.f;
    const int bh = blk / nq, qb = blk - bh * nq;
    const int b = bh / a.H, h = bh - b * a.H;
    const int qi = qb * FA_ROWS + wv * 32 + r;
    if (qi < a.Sq) {
      bf16_t* op = a.o + (size_t)(b * a.sob + h * a.soh) + (unsigned)(qi * a.sos);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = dt * 32 + 8 * g + 4 * hh;
          if (D != 64 && d >= D) continue;  // (compile-time per lane half: g, dt unrolled)
          uint2 wd;
          wd.x = pack2(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
          wd.y = pack2(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
          *reinterpret_cast<uint2*>(op + d) = wd;
        }
    }
  };
  // Hand-off without fences (cdna_hip_programming.md Guideline 16 R1; an
  // agent-scope fence costs ~1.7 us): the partial is stored write-through
  // (sc1) and drained before the flag's atomic store; the owner polls relaxed
  // and reads the partial with sc1 loads.
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.part, 0, G * FA_PART * (int)sizeof(float), 0x00020000);
  auto slot_off = [&](int worker) { return (worker * FA_PART + wv * 9 * 64 * 4) * (int)sizeof(float); };
  auto publish = [&]() {  // contributor: partial (O, m_ref, l) of this worker's first block piece
    const int so = slot_off(w);
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(fa_u4, make_float4(o[dt][4 * g], o[dt][4 * g + 1], o[dt][4 * g + 2], o[dt][4 * g + 3])),
            prs, ((dt * 4 + g) * 64 + lane) * 16, so, 16);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fa_u4, make_float4(mref, lsum, 0.f, 0.f)), prs,
                                           (8 * 64 + lane) * 16, so, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    fa_barrier();
    if (tid == 0) __hip_atomic_store(a.flags + w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto merge = [&](int blk_end) {  // owner: every worker whose range starts inside this block
    if (tid == 0) {
      for (int j = w + 1; j < G && (int)((long long)U * j / G) < blk_end; ++j) {
        unsigned spins = 0;
        while (__hip_atomic_load(a.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins > (1u << 22)) {
            atomicAdd(a.err, 1u);
            break;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler order only: the loads below are sc1)
    fa_barrier();
    for (int j = w + 1; j < G && (int)((long long)U * j / G) < blk_end; ++j) {
      const int so = slot_off(j);
      const float4 ml =
          __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prs, (8 * 64 + lane) * 16, so, 16));
      const float mn = fmaxf(mref, ml.x);
      const float ca = __builtin_amdgcn_exp2f(mref - mn), cb = __builtin_amdgcn_exp2f(ml.x - mn);
#pragma unroll
      for (int dt = 0; dt < 2; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 x = __builtin_bit_cast(
              float4, __builtin_amdgcn_raw_buffer_load_b128(prs, ((dt * 4 + g) * 64 + lane) * 16, so, 16));
          o[dt][4 * g] = o[dt][4 * g] * ca + x.x * cb;
          o[dt][4 * g + 1] = o[dt][4 * g + 1] * ca + x.y * cb;
          o[dt][4 * g + 2] = o[dt][4 * g + 2] * ca + x.z * cb;
          o[dt][4 * g + 3] = o[dt][4 * g + 3] * ca + x.w * cb;
        }
      lsum = lsum * ca + ml.y * cb;
      mref = mn;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fa_barrier();  // every wave has read the slots before they are released
    if (tid == 0)
      for (int j = w + 1; j < G && (int)((long long)U * j / G) < blk_end; ++j)
        __hip_atomic_store(a.flags + j, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  // ---- prologue: Q of the first segment, then three units of K / V ----
  int seg_lo = u0;                                   // first unit of the current segment
  int seg_hi = min(u1, (u0 / T + 1) * T);            // one past its last
  int q_for = u0;                                    // segment start whose Q DMA was issued last
  dma_q(u0 / T);
  for (int v = u0; v < min(u1, u0 + LEAD); ++v) dma_unit(v);
  wait_issue(max(q_end, dma_u0));
  fa_barrier();
  v16f sA[2], sB[2];
  load_q();
  qk(u0, sA);
  seg_init(rowmax(sA), sA);

  // ---- main loop over units, two per trip (the score registers swap roles) ----
  // BAR: a barrier unit (every FA_BE-th from u0).  Its barrier publishes units
  // u+1 .. u+FA_BE (K for the QK^Ts, V for the PVs up to the next barrier):
  // each wave first waits for its own share of them; the DMA units issued after
  // u+FA_BE (2 instructions each, any Q DMA issued among them only makes the
  // wait stricter) may stay in flight
  auto unit = [&](auto bar_c, int u, v16f (&Sc)[2], v16f (&Sn)[2]) {
    constexpr bool BAR = decltype(bar_c)::value;
    if constexpr ((PROBE & 128) != 0) tl = fa_stamp();
    if constexpr (BAR) {
      if constexpr ((PROBE & 2) == 0) {
        if (u + LEAD <= u1) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * (LEAD - FA_BE - 1)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      if constexpr ((PROBE & 128) != 0) { const auto t = fa_stamp(); ph0 += t - tl; tl = t; }
      if constexpr ((PROBE & 16) == 0) fa_barrier();
      if constexpr ((PROBE & 128) != 0) { const auto t = fa_stamp(); ph1 += t - tl; tl = t; }
    }
    // next segment's Q: its DMA goes out once this segment's Q has been read
    if (seg_hi < u1 && q_for != seg_hi && seg_hi <= u + LEAD) {
      dma_q(seg_hi / T);
      q_for = seg_hi;
    }
    if constexpr ((PROBE & 512) == 0) {
      if (u + LEAD < u1) dma_unit(u + LEAD);
    }
    if constexpr ((PROBE & 128) != 0) { const auto t = fa_stamp(); ph2 += t - tl; tl = t; }
    body(u, u + 1 < seg_hi, Sc, Sn);
    if (u + 1 < seg_hi) return;
    if constexpr ((PROBE & 128) != 0) ph6 += 1;  // segment ends
    // ---- segment [seg_lo, seg_hi) of block blk ends here ----
    const int blk = u / T;
    const bool owns_first = seg_lo == blk * T;
    if (!owns_first) {
      publish();  // (only ever this worker's first segment)
    } else {
      if (seg_hi < (blk + 1) * T) merge((blk + 1) * T);  // the rest of the block is in later workers' slots
      store_o(blk);
    }
    if (u + 1 >= u1) return;
    seg_lo = u + 1;
    seg_hi = min(u1, (seg_lo / T + 1) * T);
    if (q_for != seg_lo) {  // (short first segment: issued late)
      dma_q(seg_lo / T);
      q_for = seg_lo;
    }
    wait_issue(q_end);  // own wave's Q region (K of unit u+1 was waited for above)
    load_q();
    cneg = zero16;
    qk(u + 1, Sn);
    seg_init(rowmax(Sn), Sn);
  };
  static_assert(FA_BE == 2, "the unrolled loop below pairs one barrier unit with one plain unit");
  for (int u = u0; u < u1; u += 2) {
    unit(std::true_type{}, u, sA, sB);
    if (u + 1 < u1) {
      if constexpr ((PROBE & (32 | 256)) != 0) unit(std::true_type{}, u + 1, sB, sA);  // (probe: a barrier every unit)
      else unit(std::false_type{}, u + 1, sB, sA);
    }
  }
  if constexpr ((PROBE & 128) != 0) {
    if (lane == 0) {
      unsigned long long* d = a.dbg + ((size_t)w * FA_WAVES + wv) * 8;
      d[0] = ph0; d[1] = ph1; d[2] = ph2; d[3] = ph3; d[4] = ph4; d[5] = ph5; d[6] = ph6;
      d[7] = (unsigned long long)(u1 - u0);
    }
  }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
static float* g_fa_part = nullptr;
static unsigned* g_fa_flags = nullptr;  // [G] flags + [1] error counter
static unsigned long long* g_fa_dbg = nullptr;  // [G][8][8] phase stamps (probe 128)
static int g_fa_workers = 0;
static int g_fa_min_skv = 512;  // csk_set_attn_fa_min_skv (tests: 128)

CSK_API int csk_set_attn_fa_min_skv(int n) {
  g_fa_min_skv = n;
  return 0;
}
static int g_fa_enabled = 1;
static int g_fa_probe = 0;  // profiling builds (wrong results by design): 1 no exp, 2 no K/V waits,
                            // 4 no PV MFMAs, 8 no QK^T MFMAs, 16 no per-tile barrier

CSK_API int csk_set_attn_fa_probe(int p) {
  g_fa_probe = p;
  return 0;
}

CSK_API int csk_set_attn_fa(int on) {
  g_fa_enabled = on;
  return 0;
}

// workspace of the stream-K merge: allocated once per process (outside any graph
// capture: call it from the library init), flags zeroed once and reset by their
// consumers inside every launch
CSK_API int csk_attn_fa_init() {
  if (g_fa_part) return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  g_fa_workers = cus > 0 ? cus : 256;
  hipError_t e = hipMalloc(&g_fa_part, (size_t)g_fa_workers * FA_PART * sizeof(float));
  if (e != hipSuccess) return (int)e;
  e = hipMalloc(&g_fa_flags, (size_t)(g_fa_workers + 1) * sizeof(unsigned));
  if (e != hipSuccess) return (int)e;
  e = hipMalloc(&g_fa_dbg, (size_t)g_fa_workers * FA_WAVES * 8 * sizeof(unsigned long long));
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(g_fa_flags, 0, (size_t)(g_fa_workers + 1) * sizeof(unsigned));
}

// probe 128: copy the per-wave phase cycle sums of the last launch ([G][8][8])
CSK_API int csk_attn_fa_dbg(unsigned long long* out, int n) {
  if (!g_fa_dbg) return (int)hipErrorNotInitialized;
  return (int)hipMemcpy(out, g_fa_dbg, (size_t)n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
}

CSK_API int csk_attn_fa_errors(unsigned* out) {
  if (!g_fa_flags) return (int)hipErrorNotInitialized;
  return (int)hipMemcpy(out, g_fa_flags + g_fa_workers, sizeof(unsigned), hipMemcpyDeviceToHost);
}

// After a merge spin gave up (csk_attn_fa_errors > 0) a late contributor may
// still set its flag after the owner cleared it, and the next launch that uses
// that slot would read a stale partial.  The host therefore disables the
// kernel for the process (csk_set_attn_fa(0), hip_ops.attn_fa_health) and
// zeroes every flag and the counter here — outside any graph capture, with the
// device idle (synchronous memset).
CSK_API int csk_attn_fa_reset() {
  if (!g_fa_flags) return (int)hipErrorNotInitialized;
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(g_fa_flags, 0, (size_t)(g_fa_workers + 1) * sizeof(unsigned));
}

// test hook: pretend n merge spins gave up (tests/test_attn_fa_gpu.py)
CSK_API int csk_attn_fa_inject_errors(unsigned n) {
  if (!g_fa_flags) return (int)hipErrorNotInitialized;
  return (int)hipMemcpy(g_fa_flags + g_fa_workers, &n, sizeof(unsigned), hipMemcpyHostToDevice);
}

// 1 when csk_attention_fa takes this shape
CSK_API int csk_attn_fa_ok(int B, int H, int Sq, int Skv, int D, int causal, int has_kv_len) {
  if (!g_fa_enabled || (D != 64 && D != 40) || causal || has_kv_len || !g_fa_part) return 0;
  // short key ranges (S = 256: 4 tiles per block) spend more on stream-K
  // merges than they gain (profiles/attn_fa_r8a.txt: 23.4 vs 12.6 us at B8 H20)
  if (Skv % 64 != 0 || Skv < g_fa_min_skv || Sq < 128) return 0;
  const long long units = (long long)B * H * ((Sq + FA_ROWS - 1) / FA_ROWS) * (Skv / 64);
  return units < (1ll << 30) ? 1 : 0;
}

// workers: 0 = one per CU (the only residency the merge protocol is built for:
// every worker must be resident at once); tests pass fewer to force more cuts
CSK_API int csk_attention_fa(void* o, const void* q, const void* k, const void* v, const long long* strides, int B,
                             int H, int Sq, int Skv, int D, float scale, int workers, hipStream_t stream) {
  if (!g_fa_part) return (int)hipErrorNotInitialized;  // csk_init allocates it (never inside a capture)
  if (!csk_attn_fa_ok(B, H, Sq, Skv, D, 0, 0)) return (int)hipErrorInvalidValue;
  // every element offset the kernel forms fits 32 bits
  const long long ext[4] = {(B - 1) * strides[0] + (Sq - 1) * strides[1] + (H - 1) * strides[2] + D,
                            (B - 1) * strides[3] + (Skv - 1) * strides[4] + (H - 1) * strides[5] + D,
                            (B - 1) * strides[6] + (Skv - 1) * strides[7] + (H - 1) * strides[8] + D,
                            (B - 1) * strides[9] + (Sq - 1) * strides[10] + (H - 1) * strides[11] + D};
  for (int i = 0; i < 4; ++i)
    if (ext[i] >= (1ll << 31)) return (int)hipErrorInvalidValue;
  for (int i = 0; i < 12; ++i)
    if (strides[i] < 0) return (int)hipErrorInvalidValue;
  FaArgs a;
  a.q = (const bf16_t*)q; a.k = (const bf16_t*)k; a.v = (const bf16_t*)v; a.o = (bf16_t*)o;
  a.sqb = (int)strides[0]; a.sqs = (int)strides[1]; a.sqh = (int)strides[2];
  a.skb = (int)strides[3]; a.sks = (int)strides[4]; a.skh = (int)strides[5];
  a.svb = (int)strides[6]; a.svs = (int)strides[7]; a.svh = (int)strides[8];
  a.sob = (int)strides[9]; a.sos = (int)strides[10]; a.soh = (int)strides[11];
  a.B = B; a.H = H; a.Sq = Sq; a.Skv = Skv;
  a.sl2 = scale * 1.4426950408889634f;
  a.nq = (Sq + FA_ROWS - 1) / FA_ROWS;
  a.T = Skv / 64;
  a.U = B * H * a.nq * a.T;
  a.part = g_fa_part;
  a.flags = g_fa_flags;
  a.err = g_fa_flags + g_fa_workers;
  a.dbg = g_fa_dbg;
  int G = g_fa_workers;
  if (workers > 0 && workers < G) G = workers;
  if (G > a.U) G = a.U;
  if (D == 40) {  // (no probe variants)
    attn_fa_kernel<40><<<G, 512, 0, stream>>>(a);
    return (int)hipGetLastError();
  }
  switch (g_fa_probe) {
    case 1: attn_fa_kernel<64, 1><<<G, 512, 0, stream>>>(a); break;
    case 2: attn_fa_kernel<64, 2><<<G, 512, 0, stream>>>(a); break;
    case 4: attn_fa_kernel<64, 4><<<G, 512, 0, stream>>>(a); break;
    case 8: attn_fa_kernel<64, 8><<<G, 512, 0, stream>>>(a); break;
    case 16: attn_fa_kernel<64, 16><<<G, 512, 0, stream>>>(a); break;
    case 32: attn_fa_kernel<64, 32><<<G, 512, 0, stream>>>(a); break;
    case 256: attn_fa_kernel<64, 256><<<G, 512, 0, stream>>>(a); break;
    case 512: attn_fa_kernel<64, 512><<<G, 512, 0, stream>>>(a); break;
    case 64: attn_fa_kernel<64, 66><<<G, 512, 0, stream>>>(a); break;      // no K/V DMA (and no waits)
    case 76: attn_fa_kernel<64, 66 + 12><<<G, 512, 0, stream>>>(a); break; // ... and no MFMAs
    case 77: attn_fa_kernel<64, 66 + 13><<<G, 512, 0, stream>>>(a); break; // ... and no exp
    case 128: attn_fa_kernel<64, 128><<<G, 512, 0, stream>>>(a); break;    // phase stamps
    default: attn_fa_kernel<64, 0><<<G, 512, 0, stream>>>(a); break;
  }
  return (int)hipGetLastError();
}
