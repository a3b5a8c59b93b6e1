// Fused cross-attention sub-block of an SD transformer block (SURVEY K8 + K9 +
// K11; reference call site swarm/diffusion/diffusion_func.py:96, the diffusers
// BasicTransformerBlock attn2 path):
//
//   y = x + softmax(((LN(x) Wq^T) * scale) K^T) V Wo^T + bo
//
// ONE kernel instead of the LN-fused Q-projection GEMM -> attn_shortkv -> the
// out-projection GEMM: the [M, C] query and attention-output tensors never
// leave the chip (two HBM round trips of the activation and two launches per
// block gone).  Also emits the per-row (mean, M2) of y over all C columns for
// the next LayerNorm's consumer GEMM (ln_nparts = 1).
//
// Shape: C = 64 H (head dim 64), Skv <= 80 context tokens (77 CLIP tokens).
// Workgroup = 128 rows of one sample: 4 waves x 32 rows (two 16-row tiles) or
// 8 waves x 16 rows (csk_set_xattn_waves); every wave owns its rows end to end,
// so no intermediate crosses a lane or a wave:
//   * x rows live in registers as MFMA B fragments (lane: row fr, channels
//     32 cs + 8 g ..+7); the LayerNorm statistics are reduced from them;
//   * Q^T = Wq' x^T (A = Wq' rows from LDS) puts row fr and head-dims
//     16 dt + 4 g + r on the lane: with the (4 g + r, 16 + 4 g + r) k-slot order
//     the accumulators ARE the B fragments of S^T = K Q^T (K read in the same
//     permuted order, two 8-byte LDS reads);
//   * S^T leaves keys 16 kt + 4 g + r of query fr on the lane: the softmax is
//     in-lane + two permlane swaps; P^T and the V^T fragments (transpose reads
//     of the row-major V tile) follow attn_shortkv_kernel;
//   * O^T has head-dims 16 dt + 4 g + r of row fr on the lane: again the B
//     fragment of out^T = Wo_h O^T (Wo_h read in the permuted order);
//   * out accumulates over the heads in registers (2 x C/16 tiles per wave).
// Operands shared by the waves (the head's Wq' rows, Wo columns, K and V) are
// staged by LDS-DMA (global_load_lds, 16 B per lane, XOR-swizzled images; rows
// past Skv repeat the last key, masked) on a per-head schedule with one buffer per
// weight and two K/V buffers:
//   head h:  [DMA Wo_h, K/V_{h+1}]  Q-proj h  |B1| [DMA Wq_{h+1}]  attention h
//            |B2: Wo_h landed|  out-proj h  |B3: Wq_{h+1}, K/V_{h+1} landed|
// so every transfer has at least one compute phase to land in, and the waits
// are counted (vmcnt) — the prefetches stay in flight across B1 / B2.
#include "attn_tile.h"

typedef __attribute__((address_space(1))) const void* xa_gptr_t;
typedef __attribute__((address_space(3))) void* xa_lptr_t;

struct XattnArgs {
  const bf16_t* x;      // [M][C]: LayerNorm input and residual
  const bf16_t* wq;     // [C][C] gamma-folded query weight (ops.fold_layer_norm)
  const float* colsum;  // [C] row sums of wq
  const bf16_t* bq;     // [C] folded query bias (b + Wq beta)
  const bf16_t* kv;     // [Bc][Skv][2][H][64]: the per-request K / V (context_kv)
  const bf16_t* wo;     // [C][C] out-projection weight
  const bf16_t* bo;     // [C] out-projection bias or null
  bf16_t* y;            // [M][C]
  float* row_part;      // [M][2] (mean, M2) of y over C, or null
  const bf16_t* zero;   // zero page (DMA source of K / V padding rows)
  const bf16_t* x_end;  // CSK_DEBUG bounds
  const bf16_t* kv_end;
  int M, rows_per_b, Skv;
  float eps, scale_log2;
};

#define XA_BM 128
#define XA_KVR 96  // K / V image rows (keys), zero past Skv: three 32-key PV steps

template <int N>
__device__ __forceinline__ void xa_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void xa_dma(const bf16_t* src, bf16_t* dst) {
  __builtin_amdgcn_global_load_lds((xa_gptr_t)src, (xa_lptr_t)dst, 16, 0, 0);
}
// uniform base + 32-bit per-lane element offset: one VGPR per address (the
// saddr + voffset form), so the per-head DMA issue keeps no 64-bit pointers live
__device__ __forceinline__ void xa_dma_off(const bf16_t* base, unsigned off, bf16_t* dst) {
  xa_dma(base + off, dst);
}

__device__ __forceinline__ int xa_off64(int r, int c) { return at_off64(r, c); }
__device__ __forceinline__ v8s xa_pack8(const v4f& lo, const v4f& hi, float s) { return at_pack8(lo, hi, s); }

// PROBE (profiling builds, wrong results by design; csk_set_xattn_probe): 1 = no
// Q-projection MFMAs, 2 = no attention (S / softmax / PV), 4 = no out-projection
// MFMAs, 8 = no per-head DMA (operands of head 0 reused)
template <int C, int NW, int RT, int PROBE = 0>
__global__ __launch_bounds__(NW * 64, 1) void xattn_block_kernel(const XattnArgs a) {
  constexpr int H = C / 64, NCS = C / 32, NNT = C / 16, CPR = C / 8;
  constexpr int WQ = 64 * C, WO = C * 64, KVI = XA_KVR * 64;
  constexpr int WQ_PIECES = WQ / 512, WO_PIECES = WO / 512, KV_PIECES = 2 * KVI / 512;
  static_assert(WQ_PIECES % NW == 0 && WO_PIECES % NW == 0 && KV_PIECES % NW == 0, "pieces per wave");
  static_assert(NW * RT * 16 == XA_BM, "workgroup rows");
  constexpr int NWQ = WQ_PIECES / NW, NWO = WO_PIECES / NW, NKV = KV_PIECES / NW;
  // separate LDS objects: the compiler's wait insertion can then tell an
  // LDS-DMA into one buffer from reads of another (one array made it drain
  // every DMA in flight before the first LDS read after an issue)
  __shared__ __attribute__((aligned(16))) bf16_t s_wq[WQ];
  __shared__ __attribute__((aligned(16))) bf16_t s_wo[WO];
  __shared__ __attribute__((aligned(16))) bf16_t s_kv0[2 * KVI];  // K | V, [96][64] each
  __shared__ __attribute__((aligned(16))) bf16_t s_kv1[2 * KVI];
  __shared__ __attribute__((aligned(16))) float s_cb[2 * C];  // LN-fold colsum | bq (fp32)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, g = lane >> 4;
  const int m0 = xcd_remap(blockIdx.x, gridDim.x) * XA_BM;
  const int b = m0 / a.rows_per_b;
  const int Skv = a.Skv;
  const int row_w = m0 + wid * (RT * 16);  // this wave's first row

  // ---- LDS-DMA issue helpers (every wave issues the same counts) ----
  auto dma_wq = [&](int h) {
#pragma unroll
    for (int i = 0; i < NWQ; ++i) {
      const int p = wid + NW * i;
      const int f = 64 * p + lane, row = f / CPR, slot = f % CPR;
      CSK_DCHECK(h * 64 + row < C, 71, row, C);
      xa_dma_off(a.wq, (unsigned)((h * 64 + row) * C + 8 * (slot ^ (row & 7))), s_wq + 512 * p);
    }
  };
  auto dma_wo = [&](int h) {
#pragma unroll
    for (int i = 0; i < NWO; ++i) {
      const int p = wid + NW * i;
      const int row = 8 * p + (lane >> 3), slot = lane & 7;
      CSK_DCHECK(row < C, 72, row, C);
      xa_dma_off(a.wo, (unsigned)(row * C + h * 64 + 8 * (slot ^ at_key(row))), s_wo + 512 * p);
    }
  };
  auto dma_kv = [&](int h, bf16_t* dst) {
#pragma unroll
    for (int i = 0; i < NKV; ++i) {
      const int p = wid + NW * i;  // pieces 0..11: K rows, 12..23: V rows
      const int which = p >= KV_PIECES / 2;
      const int row = 8 * (p - which * (KV_PIECES / 2)) + (lane >> 3), slot = lane & 7;
      // rows past Skv repeat the last key: finite values whose scores are
      // masked to -inf and whose P is 0 (no per-lane pointer select)
      const int rr = min(row, Skv - 1);
      const unsigned off = (unsigned)(((b * Skv + rr) * 2 + which) * (H * 64) + h * 64 + 8 * (slot ^ at_key(row)));
      CSK_DCHECK(a.kv + off + 8 <= a.kv_end, 73, row, Skv);
      xa_dma_off(a.kv, off, dst + 512 * p);
    }
  };

  // ---- prologue: head 0 operands in flight while the x rows load ----
  for (int i = tid; i < C; i += NW * 64) {
    s_cb[i] = a.colsum[i];
    s_cb[C + i] = bf2f(a.bq[i]);
  }
  dma_wq(0);
  dma_wo(0);
  dma_kv(0, s_kv0);
  v8s xf[RT][NCS];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int m = row_w + rt * 16 + fr;
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      uint4 u = make_uint4(0, 0, 0, 0);
      if (m < a.M) {
        CSK_DCHECK(a.x + (size_t)m * C + 32 * cs + 8 * g + 8 <= a.x_end, 74, m, a.M);
        u = *reinterpret_cast<const uint4*>(a.x + (size_t)m * C + 32 * cs + 8 * g);
      }
      xf[rt][cs] = __builtin_bit_cast(v8s, u);
    }
  }
  // LayerNorm statistics of the two rows this lane holds (four lane groups x NCS x 8)
  float mean[RT], rstd[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    float s = 0.f;
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      float f[8];
      unpack8(__builtin_bit_cast(uint4, xf[rt][cs]), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[j];
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    mean[rt] = s * (1.0f / C);
    float q = 0.f;
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      float f[8];
      unpack8(__builtin_bit_cast(uint4, xf[rt][cs]), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = f[j] - mean[rt];
        q = __builtin_fmaf(d, d, q);
      }
    }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    rstd[rt] = rsqrtf(q * (1.0f / C) + a.eps);
  }

  v4f out[RT][NNT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int nt = 0; nt < NNT; ++nt) out[rt][nt] = v4f{0.f, 0.f, 0.f, 0.f};

  xa_vmcnt<0>();
  __syncthreads();

  const float sl2 = a.scale_log2;
  for (int h = 0; h < H; ++h) {
    const int cur = h & 1;
    const bool more = h + 1 < H;
    // K / V of the next head into the other buffer (its last reader, the
    // attention of head h - 1, finished before barrier B2 of that head)
    if (more && (PROBE & 8) == 0) {
      if (cur) dma_kv(h + 1, s_kv0);
      else dma_kv(h + 1, s_kv1);
    }

    // ---------------- Q projection (LayerNorm folded) ----------------
    v4f qa[RT][4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) qa[rt][dt] = v4f{0.f, 0.f, 0.f, 0.f};
    // one k-step of Wq' fragments in flight ahead of the MFMAs (the fences keep
    // the compiler from hoisting every step's reads at once: 160 registers)
    auto ld_wq = [&](int cs, v8s (&wf)[4]) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int r = 16 * dt + fr;
        wf[dt] = *reinterpret_cast<const v8s*>(s_wq + r * C + 8 * ((4 * cs + g) ^ (r & 7)));
      }
    };
    v8s wf[2][4];
    ld_wq(0, wf[0]);
#pragma unroll
    for (int cs = 0; cs < NCS; ++cs) {
      if (cs + 1 < NCS) ld_wq(cs + 1, wf[(cs + 1) & 1]);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          if constexpr ((PROBE & 1) != 0) asm volatile("" ::"v"(wf[cs & 1][dt]), "v"(xf[rt][cs]));
          else qa[rt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cs & 1][dt], xf[rt][cs], qa[rt][dt], 0, 0, 0);
        }
      asm volatile("" ::: "memory");
    }
    // B1: every wave is done with Wq_h -> the next head's rows may land there
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (more && (PROBE & 8) == 0) dma_wq(h + 1);

    // q = (rstd (acc - mean colsum) + bq) * scale * log2(e), as S^T B fragments
    v8s qf[RT][2];
    {
      v4f cw[4], bw[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int d = h * 64 + 16 * dt + 4 * g;
        cw[dt] = *reinterpret_cast<const v4f*>(s_cb + d);
        bw[dt] = *reinterpret_cast<const v4f*>(s_cb + C + d);
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        v4f qv[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            qv[dt][r] = __builtin_fmaf(rstd[rt], qa[rt][dt][r] - mean[rt] * cw[dt][r], bw[dt][r]);
        qf[rt][0] = xa_pack8(qv[0], qv[1], sl2);
        qf[rt][1] = xa_pack8(qv[2], qv[3], sl2);
      }
    }

    // ---------------- attention over the Skv context tokens ----------------
    v8s of[RT][2];
    auto attend = [&](const bf16_t* ks) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        v4f o[4];
        float inv;
        at_attend_rowtile(ks, ks + KVI, qf[rt], Skv, o, inv);
        of[rt][0] = xa_pack8(o[0], o[1], inv);
        of[rt][1] = xa_pack8(o[2], o[3], inv);
      }
    };
    if constexpr ((PROBE & 2) != 0) {
      for (int rt = 0; rt < RT; ++rt) {
        of[rt][0] = qf[rt][0];
        of[rt][1] = qf[rt][1];
      }
    } else {
      if (cur) attend(s_kv1);
      else attend(s_kv0);
    }
    // B2: Wo_h has landed (newer in flight: K/V_{h+1}, Wq_{h+1})
    if (more && (PROBE & 8) == 0) xa_vmcnt<NKV + NWQ>();
    else xa_vmcnt<0>();
    __builtin_amdgcn_s_barrier();

    // ---------------- out-projection of this head, accumulated ----------------
    v8s wof[2][2];
    wof[0][0] = at_perm_frag(s_wo, fr, 4 * g);
    wof[0][1] = at_perm_frag(s_wo, fr, 32 + 4 * g);
#pragma unroll
    for (int nt = 0; nt < NNT; ++nt) {
      if (nt + 1 < NNT) {
        wof[(nt + 1) & 1][0] = at_perm_frag(s_wo, 16 * (nt + 1) + fr, 4 * g);
        wof[(nt + 1) & 1][1] = at_perm_frag(s_wo, 16 * (nt + 1) + fr, 32 + 4 * g);
      }
#pragma unroll
      for (int ds = 0; ds < 2; ++ds)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          if constexpr ((PROBE & 4) != 0) asm volatile("" ::"v"(wof[nt & 1][ds]), "v"(of[rt][ds]));
          else out[rt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wof[nt & 1][ds], of[rt][ds], out[rt][nt], 0, 0, 0);
        }
      asm volatile("" ::: "memory");
    }
    // B3: everyone is done with Wo_h and K/V_h; Wq_{h+1} and K/V_{h+1} landed
    xa_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (more && (PROBE & 8) == 0) dma_wo(h + 1);
  }

  // ---------------- epilogue: + bias + residual, row statistics ----------------
  // Every residual / bias fragment is loaded before the first store: y may alias
  // x as far as the compiler knows, so loads left at their use each waited one
  // memory latency behind the previous store (20 per row tile).
  uint2 xres[RT][NNT], bres[NNT];
#pragma unroll
  for (int nt = 0; nt < NNT; ++nt) {
    bres[nt] = make_uint2(0, 0);
    if (a.bo) bres[nt] = *reinterpret_cast<const uint2*>(a.bo + 16 * nt + 4 * g);
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int m = row_w + rt * 16 + fr;
#pragma unroll
    for (int nt = 0; nt < NNT; ++nt) {
      xres[rt][nt] = make_uint2(0, 0);
      if (m < a.M) xres[rt][nt] = *reinterpret_cast<const uint2*>(a.x + (size_t)m * C + 16 * nt + 4 * g);
    }
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int m = row_w + rt * 16 + fr;
    const bool ok = m < a.M;
    float s = 0.f;
#pragma unroll
    for (int nt = 0; nt < NNT; ++nt) {
      const int n = 16 * nt + 4 * g;
      const uint2 u = xres[rt][nt];
      const uint2 ub = bres[nt];
      float rv[4] = {bf2f((bf16_t)(u.x & 0xffff)), bf2f((bf16_t)(u.x >> 16)), bf2f((bf16_t)(u.y & 0xffff)),
                     bf2f((bf16_t)(u.y >> 16))};
      const float bov[4] = {bf2f((bf16_t)(ub.x & 0xffff)), bf2f((bf16_t)(ub.x >> 16)), bf2f((bf16_t)(ub.y & 0xffff)),
                            bf2f((bf16_t)(ub.y >> 16))};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // round to the stored bf16 first: the statistics describe the tensor the consumer reads
        const float v = bf2f(f2bf(out[rt][nt][r] + bov[r] + rv[r]));
        out[rt][nt][r] = v;
        s += v;
      }
      if (ok) {
        uint2 w;
        w.x = pack2(out[rt][nt][0], out[rt][nt][1]);
        w.y = pack2(out[rt][nt][2], out[rt][nt][3]);
        *reinterpret_cast<uint2*>(a.y + (size_t)m * C + n) = w;
      }
    }
    if (a.row_part) {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float mu = s * (1.0f / C);
      float q = 0.f;
#pragma unroll
      for (int nt = 0; nt < NNT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float d = out[rt][nt][r] - mu;
          q = __builtin_fmaf(d, d, q);
        }
      q += __shfl_xor(q, 16, 64);
      q += __shfl_xor(q, 32, 64);
      if (ok && g == 0) *reinterpret_cast<float2*>(a.row_part + (size_t)m * 2) = make_float2(mu, q);
    }
  }
}

CSK_DEBUG_EXPORT(xattn)

static int g_xattn_probe = 0;
static int g_xattn_waves = 8;  // profiles/xattnbench_waves_r6h.txt: 40.1 vs 49.8 us (4 waves)
CSK_API int csk_set_xattn_probe(int p) {
  g_xattn_probe = p;
  return 0;
}
// 8 waves x 16 rows (default) or 4 waves x 32 rows per 128-row workgroup
CSK_API int csk_set_xattn_waves(int w) {
  if (w != 4 && w != 8) return (int)hipErrorInvalidValue;
  g_xattn_waves = w;
  return 0;
}

template <int C, int NW, int RT>
static void xattn_launch(const XattnArgs& a, dim3 grid, hipStream_t stream) {
  switch (g_xattn_probe) {
    case 1: xattn_block_kernel<C, NW, RT, 1><<<grid, NW * 64, 0, stream>>>(a); break;
    case 2: xattn_block_kernel<C, NW, RT, 2><<<grid, NW * 64, 0, stream>>>(a); break;
    case 4: xattn_block_kernel<C, NW, RT, 4><<<grid, NW * 64, 0, stream>>>(a); break;
    case 8: xattn_block_kernel<C, NW, RT, 8><<<grid, NW * 64, 0, stream>>>(a); break;
    case 15: xattn_block_kernel<C, NW, RT, 15><<<grid, NW * 64, 0, stream>>>(a); break;
    default: xattn_block_kernel<C, NW, RT><<<grid, NW * 64, 0, stream>>>(a); break;
  }
}

const bf16_t* csk_zero_ptr();

// x, wq, wo: [M][C] / [C][C] bf16; colsum fp32 [C]; bq / bo bf16 [C];
// kv: [Bc][Skv][2][H][64] bf16 contiguous; row_part: [M][2] fp32 or null.
// Requires C = 320, Skv <= 80, rows_per_b % 128 == 0 (one sample per workgroup).
CSK_API int csk_xattn_block(void* y, const void* x, const void* wq, const void* colsum, const void* bq,
                            const void* kv, const void* wo, const void* bo, void* row_part, int M, int C,
                            int rows_per_b, int Bc, int Skv, float eps, float scale, hipStream_t stream) {
  if (!csk_zero_ptr()) return (int)hipErrorNotInitialized;
  if (Skv < 1 || Skv > 80 || rows_per_b % XA_BM != 0 || M % rows_per_b != 0 || M / rows_per_b > Bc)
    return (int)hipErrorInvalidValue;
  XattnArgs a;
  a.x = (const bf16_t*)x;
  a.wq = (const bf16_t*)wq;
  a.colsum = (const float*)colsum;
  a.bq = (const bf16_t*)bq;
  a.kv = (const bf16_t*)kv;
  a.wo = (const bf16_t*)wo;
  a.bo = (const bf16_t*)bo;
  a.y = (bf16_t*)y;
  a.row_part = (float*)row_part;
  a.zero = csk_zero_ptr();
  a.x_end = a.x + (size_t)M * C;
  a.kv_end = a.kv + (size_t)Bc * Skv * 2 * C;
  a.M = M;
  a.rows_per_b = rows_per_b;
  a.Skv = Skv;
  a.eps = eps;
  a.scale_log2 = scale * 1.4426950408889634f;
  const dim3 grid((M + XA_BM - 1) / XA_BM);
  switch (C) {
    case 320:
      if (g_xattn_waves == 8) xattn_launch<320, 8, 1>(a, grid, stream);
      else xattn_launch<320, 4, 2>(a, grid, stream);
      break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
