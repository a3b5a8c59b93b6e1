// GroupNorm(+SiLU) on channels-last [B, P, C] bf16 and LayerNorm on rows.
//
// GroupNorm is two streaming passes:
//   gn_stats : grid (chunks, B). Each workgroup reads a chunk of pixels with
//              16-byte vector loads (C contiguous -> fully coalesced), reduces
//              per-channel sums in LDS, and writes per-(b, chunk, group)
//              partial moments (n, mean, M2).
//   gn_apply : grid (chunks, B). Prologue: one wave per group merges the chunk
//              partials with Chan's parallel formula (numerically robust even
//              for the 1 Mi-element VAE groups), folds gamma/beta into a
//              per-channel scale/shift in LDS; body: y = x*a + b (+SiLU),
//              16-byte loads/stores.
#include "common.h"

#define GN_THREADS 256
#define GN_MAXC 4096

// Largest number of statistics partials per sample that every apply workgroup
// merges itself in a prologue; above it a finalize kernel merges them once.
static int g_gn_prologue_max = 1024;
CSK_API int csk_set_gn_prologue_max(int n) {
  g_gn_prologue_max = n;
  return 0;
}

// Thread layout shared by the stats and apply kernels: thread = (cv, r); cv is
// the 8-channel vector column the thread owns for the whole chunk (so its
// per-channel constants live in registers), r its pixel row; R = 256 / NVT rows
// advance together.  C > 2048 (NV > 256) gives each thread two columns
// (cv, cv + NVT).
struct GnLayout {
  int NV, NVT, TPV, R, cv, r;
  __device__ GnLayout(int C, int tid) {
    NV = C >> 3;
    TPV = NV > GN_THREADS ? 2 : 1;
    NVT = (NV + TPV - 1) / TPV;
    R = GN_THREADS / NVT;
    cv = tid % NVT;
    r = tid / NVT;
  }
};

// part[((b * nchunk + chunk) * G + g) * 3 + {n, mean, M2}]
// The pixel loop issues GN_UNROLL independent 16-byte loads before accumulating
// (a chunk is only a few rows per thread, so a dependent load->add chain would
// leave the kernel latency-bound at ~1 TB/s); LDS is sized to C (dynamic), not
// GN_MAXC, so more workgroups fit per CU.
#define GN_UNROLL 4
// dynamic LDS of gn_stats_kernel: R rows x 2 x C floats (<= 32 KB)
static inline size_t gn_stats_lds(int C) {
  const int NV = C >> 3, TPV = NV > GN_THREADS ? 2 : 1, NVT = (NV + TPV - 1) / TPV;
  return (size_t)(GN_THREADS / NVT) * 2 * C * sizeof(float);
}
__global__ __launch_bounds__(GN_THREADS) void gn_stats_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                              int P, int C, int G, int chunk, int nchunk,
                                                              const bf16_t* __restrict__ x2 = nullptr, int C1 = 0) {
  // x2 != null: statistics of the channel concat [x (C1) | x2 (C - C1)] read in place
  extern __shared__ float red[];  // [R][2][C]: per-row partials, reduced in a fixed order (deterministic)
  const int b = blockIdx.y, ck = blockIdx.x, tid = threadIdx.x;
  const GnLayout L(C, tid);
  const int p0 = ck * chunk, p1 = min(P, p0 + chunk);
  if (!x2) C1 = C;
  float s[2][8], ss[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[u][j] = ss[u][j] = 0.f;
  if (L.r < L.R) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int v = L.cv + u * L.NVT;
      if (u < L.TPV && v < L.NV) {
        const bool second = v * 8 >= C1;
        const int xst = second ? C - C1 : C1;
        const bf16_t* xsrc = (second ? x2 : x) + (size_t)b * P * xst + (second ? v * 8 - C1 : v * 8);
        for (int p = p0 + L.r; p < p1; p += GN_UNROLL * L.R) {
          // unconditional loads from clamped rows (a select around each load would
          // make hipcc wait vmcnt(0) per element); out-of-chunk rows are masked
          uint4 q[GN_UNROLL];
#pragma unroll
          for (int w = 0; w < GN_UNROLL; ++w)
            q[w] = *reinterpret_cast<const uint4*>(xsrc + (size_t)min(p + w * L.R, p1 - 1) * xst);
#pragma unroll
          for (int w = 0; w < GN_UNROLL; ++w) {
            const float mk = (p + w * L.R < p1) ? 1.f : 0.f;
            float f[8];
            unpack8(q[w], f);
#pragma unroll
            for (int j = 0; j < 8; ++j) { const float t = f[j] * mk; s[u][j] += t; ss[u][j] += t * t; }
          }
        }
      }
    }
  }
  // every (row r, vector column v) slot has exactly one owner thread: plain
  // stores, then a fixed-order sum over rows (LDS float atomics made the
  // statistics, and so whole denoising runs, vary run to run)
  if (L.r < L.R) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int v = L.cv + u * L.NVT;
      if (u < L.TPV && v < L.NV) {
        float* rs = red + (size_t)L.r * 2 * C + v * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          rs[j] = s[u][j];
          rs[C + j] = ss[u][j];
        }
      }
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += GN_THREADS) {
    float a = red[c], q = red[C + c];
    for (int rr = 1; rr < L.R; ++rr) {
      a += red[(size_t)rr * 2 * C + c];
      q += red[(size_t)rr * 2 * C + C + c];
    }
    red[c] = a;
    red[C + c] = q;
  }
  __syncthreads();
  const int Cg = C / G;
  for (int g = tid; g < G; g += GN_THREADS) {
    float sm = 0.f, sq = 0.f;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) { sm += red[c]; sq += red[C + c]; }
    const float n = (float)(p1 - p0) * (float)Cg;
    const float mean = n > 0.f ? sm / n : 0.f;
    float* o = part + (((size_t)b * nchunk + ck) * G + g) * 3;
    o[0] = n;
    o[1] = mean;
    o[2] = fmaxf(sq - sm * mean, 0.f);
  }
}

// Group moments from per-entry partials (count n_i, mean m_i, M2_i), merged by
// `tpg` consecutive lanes (a power of two <= 64):
//   mean = sum(n_i m_i) / N,   M2 = sum(M2_i) + sum(n_i (m_i - mean)^2)
// Two passes of independent loads + FMAs and a butterfly per pass: the
// sequential Chan chain (a division per entry, each step waiting on the last)
// made the merge the slowest part of a GroupNorm over a few hundred partials.
template <class Get>
__device__ __forceinline__ void group_moments(const Get& get, int ne, int sub, int tpg, float& mean, float& rstd,
                                              float eps) {
  float sn = 0.f, sm = 0.f;
#pragma unroll 4
  for (int e = sub; e < ne; e += tpg) {
    float n, m, q;
    get(e, n, m, q);
    sn += n;
    sm = __builtin_fmaf(n, m, sm);
  }
  for (int o = 1; o < tpg; o <<= 1) {
    sn += __shfl_xor(sn, o, 64);
    sm += __shfl_xor(sm, o, 64);
  }
  mean = sn > 0.f ? sm / sn : 0.f;
  float sq = 0.f;
#pragma unroll 4
  for (int e = sub; e < ne; e += tpg) {
    float n, m, q;
    get(e, n, m, q);
    const float d = m - mean;
    sq += __builtin_fmaf(n * d, d, q);
  }
  for (int o = 1; o < tpg; o <<= 1) sq += __shfl_xor(sq, o, 64);
  rstd = rsqrtf(sq / fmaxf(sn, 1.f) + eps);
}

// One wave per group: up to 16 entries per lane are loaded ONCE (all in flight
// together) and kept in registers for both passes, so a finalize over <= 1024
// partials costs one memory round trip instead of two dependent loops.
template <class Get>
__device__ __forceinline__ void group_moments_wave(const Get& get, int ne, int lane, float& mean, float& rstd,
                                                   float eps) {
  constexpr int CAP = 16;  // 1024 entries in one round trip (64x64x320 fused stats: 640 per group)
  float en[CAP], em[CAP], eq[CAP];
#pragma unroll
  for (int j = 0; j < CAP; ++j) {
    const int e = lane + 64 * j;
    en[j] = em[j] = eq[j] = 0.f;
    if (e < ne) get(e, en[j], em[j], eq[j]);
  }
  float sn = 0.f, sm = 0.f;
#pragma unroll
  for (int j = 0; j < CAP; ++j) {
    sn += en[j];
    sm = __builtin_fmaf(en[j], em[j], sm);
  }
  for (int e = lane + 64 * CAP; e < ne; e += 64) {  // > 1024 partials (large VAE maps)
    float n, m, q;
    get(e, n, m, q);
    sn += n;
    sm = __builtin_fmaf(n, m, sm);
  }
  sn = wave_sum(sn);
  sm = wave_sum(sm);
  mean = sn > 0.f ? sm / sn : 0.f;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < CAP; ++j) {
    const float d = em[j] - mean;
    sq += __builtin_fmaf(en[j] * d, d, eq[j]);
  }
  for (int e = lane + 64 * CAP; e < ne; e += 64) {
    float n, m, q;
    get(e, n, m, q);
    const float d = m - mean;
    sq += __builtin_fmaf(n * d, d, q);
  }
  rstd = rsqrtf(wave_sum(sq) / fmaxf(sn, 1.f) + eps);
}

// stat[(b * G + g) * 2 + {mean, rstd}]: merge chunk partials (Chan); one wave
// per (b, g) so the merge is spread over B*G/4 workgroups instead of B.
__global__ __launch_bounds__(GN_THREADS) void gn_finalize_kernel(const float* __restrict__ part, float* __restrict__ stat,
                                                                 int B, int G, int nchunk, float eps) {
  const int lane = threadIdx.x & 63;
  const int bg = blockIdx.x * (GN_THREADS / 64) + (threadIdx.x >> 6);
  if (bg >= B * G) return;  // whole waves leave together (one (b, g) per wave)
  const int b = bg / G, g = bg - b * G;
  float mean, rstd;
  group_moments_wave(
      [&](int c, float& n, float& m, float& q) {
        const float* pp = part + (((size_t)b * nchunk + c) * G + g) * 3;
        n = pp[0]; m = pp[1]; q = pp[2];
      },
      nchunk, lane, mean, rstd, eps);
  if (lane == 0) {
    stat[bg * 2] = mean;
    stat[bg * 2 + 1] = rstd;
  }
}

// Epilogue partial (mean, M2) of channel c in segment sg: [seg][C][2] in `part`,
// or, for a channel concat whose producers each wrote their own partials,
// channels < C1 in part ([seg][C1][2]) and the rest in part2 ([seg][C - C1][2])
__device__ __forceinline__ float2 load_part(const float* part, const float* part2, int sg, int c, int C, int C1) {
  if (part2 == nullptr) return *reinterpret_cast<const float2*>(part + ((size_t)sg * C + c) * 2);
  if (c < C1) return *reinterpret_cast<const float2*>(part + ((size_t)sg * C1 + c) * 2);
  return *reinterpret_cast<const float2*>(part2 + ((size_t)sg * (C - C1) + c - C1) * 2);
}

// MODE 0: `stat` holds final (mean, rstd) per (b, g) (a finalize kernel ran).
// MODE 1: `stat` is the stats kernel's chunk partials [b][nent][g][3];
// MODE 2: `stat` is epilogue partials [seg][c][2] (nent = segments per sample,
//         seg_rows rows each).  MODES 1/2 merge them in the prologue (Chan),
// which removes the finalize launch when there are few entries per group.
template <int MODE>
__global__ __launch_bounds__(GN_THREADS) void gn_apply_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                              const float* __restrict__ stat,
                                                              const bf16_t* __restrict__ gamma,
                                                              const bf16_t* __restrict__ beta, int P, int C, int G,
                                                              int chunk, int silu, int affine_bstride, int nent,
                                                              int seg_rows, float eps,
                                                              const bf16_t* __restrict__ x2 = nullptr, int C1 = 0,
                                                              const float* __restrict__ part2 = nullptr) {
  // x2 != null: the input is the channel concat [x (C1 channels) | x2 (C - C1)]
  // of two separate tensors (UNet skip connections), read in place
  __shared__ float gst[2 * 64];
  if (!x2) C1 = C;
  const int b = blockIdx.y, ck = blockIdx.x, tid = threadIdx.x;
  gamma += (size_t)b * affine_bstride;  // per-sample affine ([B, C]) when affine_bstride == C
  beta += (size_t)b * affine_bstride;
  const int Cg = C / G;
  if constexpr (MODE != 0) {
    // tpg threads (a power of two) merge one group's entries, then shuffle-merge
    int tpg = 1;
    while (tpg * 2 * G <= GN_THREADS && tpg < 64) tpg *= 2;
    const int g = tid / tpg, sub = tid % tpg;
    float mean, rstd;
    if constexpr (MODE == 1) {
      group_moments(
          [&](int e, float& n, float& m, float& q) {
            const float* pp = stat + (((size_t)b * nent + e) * G + g) * 3;
            n = pp[0]; m = pp[1]; q = pp[2];
          },
          g < G ? nent : 0, sub, tpg, mean, rstd, eps);
    } else {
      const float fn = (float)seg_rows;
      group_moments(
          [&](int e, float& n, float& m, float& q) {
            const int sg = b * nent + e / Cg, c = g * Cg + e % Cg;
            const float2 mq = load_part(stat, part2, sg, c, C, C1);
            n = fn; m = mq.x; q = mq.y;
          },
          g < G ? nent * Cg : 0, sub, tpg, mean, rstd, eps);
    }
    if (g < G && sub == 0) {
      gst[2 * g] = mean;
      gst[2 * g + 1] = rstd;
    }
    __syncthreads();
  }
  const GnLayout L(C, tid);
  if (L.r >= L.R) return;
  // per-channel scale / shift of this thread's (up to two) 8-channel columns:
  // gamma / beta as one 16-byte load each, the (mean, rstd) of the <= 2 groups
  // an 8-channel vector touches when Cg == 4 or Cg >= 6 (24 scalar loads per
  // thread before the first pixel otherwise).  Cg = 5 is excluded: an aligned
  // 8-channel vector can span THREE 5-channel groups (channels 8..15 = groups
  // 1, 2, 3), so it takes the per-channel path.
  float sa[2][8], sb[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int v = min(L.cv + u * L.NVT, L.NV - 1);
    const int c0 = v * 8;
    float gf[8], bfv[8];
    if (((((size_t)(gamma + c0)) | ((size_t)(beta + c0))) & 15) == 0) {
      unpack8(*reinterpret_cast<const uint4*>(gamma + c0), gf);
      unpack8(*reinterpret_cast<const uint4*>(beta + c0), bfv);
    } else {  // a strided per-sample affine view
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        gf[j] = bf2f(gamma[c0 + j]);
        bfv[j] = bf2f(beta[c0 + j]);
      }
    }
    const int g0 = c0 / Cg;
    const bool two = Cg == 4 || Cg >= 6;  // <= 2 groups per aligned 8-channel vector
    float2 s0, s1;
    if (two) {
      const int g1 = min(g0 + 1, G - 1);
      if constexpr (MODE == 0) {
        s0 = *reinterpret_cast<const float2*>(stat + (b * G + g0) * 2);
        s1 = *reinterpret_cast<const float2*>(stat + (b * G + g1) * 2);
      } else {
        s0 = make_float2(gst[2 * g0], gst[2 * g0 + 1]);
        s1 = make_float2(gst[2 * g1], gst[2 * g1 + 1]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const int g = c / Cg;
      float2 st;
      if (two) {
        st = g == g0 ? s0 : s1;
      } else if constexpr (MODE == 0) {
        st = *reinterpret_cast<const float2*>(stat + (b * G + g) * 2);
      } else {
        st = make_float2(gst[2 * g], gst[2 * g + 1]);
      }
      const float a = gf[j] * st.y;
      sa[u][j] = a;
      sb[u][j] = bfv[j] - st.x * a;
    }
  }
  const int p0 = ck * chunk, p1 = min(P, p0 + chunk);
  const size_t boff = (size_t)b * P * C;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int v = L.cv + u * L.NVT;
    if (u < L.TPV && v < L.NV) {
      const bool second = v * 8 >= C1;  // this column vector lives in x2
      const int xst = second ? C - C1 : C1;
      const bf16_t* xsrc = (second ? x2 : x) + (size_t)b * P * xst + (second ? v * 8 - C1 : v * 8);
      for (int p = p0 + L.r; p < p1; p += GN_UNROLL * L.R) {
        uint4 q[GN_UNROLL];
#pragma unroll
        for (int w = 0; w < GN_UNROLL; ++w)
          q[w] = *reinterpret_cast<const uint4*>(xsrc + (size_t)min(p + w * L.R, p1 - 1) * xst);
#pragma unroll
        for (int w = 0; w < GN_UNROLL; ++w) {
          const int pp = p + w * L.R;
          if (pp < p1) {
            float f[8];
            unpack8(q[w], f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float t = f[j] * sa[u][j] + sb[u][j];
              f[j] = silu == 1 ? silu_f(t) : (silu == 2 ? gelu_f(t) : t);  // act: 0 none, 1 SiLU, 2 GELU
            }
            *reinterpret_cast<uint4*>(y + boff + (size_t)pp * C + v * 8) = pack8(f);
          }
        }
      }
    }
  }
}

// GroupNorm from statistics fused into the producing GEMM/conv epilogue
// (GemmArgs::gn_part: per (row tile of seg_rows rows, channel) (mean, M2)):
// merge them per (b, g) — one wave each — then the usual apply pass.  The
// stats pass over the tensor disappears.
__global__ __launch_bounds__(GN_THREADS) void gn_finalize_part_kernel(const float* __restrict__ part,
                                                                      float* __restrict__ stat, int B, int C, int G,
                                                                      int nseg, int seg_rows, float eps,
                                                                      const float* __restrict__ part2, int C1) {
  const int lane = threadIdx.x & 63;
  const int bg = blockIdx.x * (GN_THREADS / 64) + (threadIdx.x >> 6);
  if (bg >= B * G) return;
  const int b = bg / G, g = bg - b * G, Cg = C / G;
  const float fn = (float)seg_rows;
  float mean, rstd;
  group_moments_wave(
      [&](int e, float& n, float& m, float& q) {
        const int sg = b * nseg + e / Cg, c = g * Cg + e % Cg;
        const float2 mq = load_part(part, part2, sg, c, C, C1);
        n = fn; m = mq.x; q = mq.y;
      },
      nseg * Cg, lane, mean, rstd, eps);
  if (lane == 0) {
    stat[bg * 2] = mean;
    stat[bg * 2 + 1] = rstd;
  }
}

// The same merge with one WORKGROUP per (b, g), for the large partial counts of
// VAE maps (512^2 and 1024^2 images: 8K-64K entries per group, where the
// one-wave kernel's tail loop serialised a memory round trip per 64 entries):
// 256 threads, 8 loads in flight each, block-reduced sums.
static int g_gn_wg_min = 1024;  // partials per group above which the finalize runs a workgroup per group
CSK_API int csk_set_gn_finalize_wg(int n) {
  g_gn_wg_min = n;
  return 0;
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // red is reused by the next call
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void gn_finalize_part_wg_kernel(const float* __restrict__ part,
                                                                  float* __restrict__ stat, int B, int C, int G,
                                                                  int nseg, int seg_rows, float eps,
                                                                  const float* __restrict__ part2, int C1) {
  __shared__ float red[4];
  const int bg = blockIdx.x;
  const int b = bg / G, g = bg - b * G, Cg = C / G;
  const int ne = nseg * Cg;
  const float fn = (float)seg_rows;
  float sm = 0.f;
#pragma unroll 8
  for (int e = threadIdx.x; e < ne; e += 256) {
    const float2 mq = load_part(part, part2, b * nseg + e / Cg, g * Cg + e % Cg, C, C1);
    sm += mq.x;
  }
  const float mean = block_sum256(sm, red) / (float)ne;  // every entry holds seg_rows rows
  float sq = 0.f;
#pragma unroll 8
  for (int e = threadIdx.x; e < ne; e += 256) {
    const float2 mq = load_part(part, part2, b * nseg + e / Cg, g * Cg + e % Cg, C, C1);
    const float d = mq.x - mean;
    sq += __builtin_fmaf(fn * d, d, mq.y);
  }
  const float m2 = block_sum256(sq, red);
  if (threadIdx.x == 0) {
    stat[bg * 2] = mean;
    stat[bg * 2 + 1] = rsqrtf(m2 / fmaxf(fn * (float)ne, 1.f) + eps);
  }
}

// Channel-blocked apply that merges its OWN groups' epilogue partials: grid
// (C / CB, chunks, B) with CB = lcm(8, C/G) channels (<= 4 whole groups) per
// workgroup.  The finalize launch between the producer and the apply
// disappears: every workgroup merges only the nseg*CB partials of its <= 4
// groups (one wave per group, one memory round trip) instead of all C channels
// (which made the full-row MODE-2 prologue cost more than a finalize launch at
// 64x64x320).  The channel block is the fastest grid dimension, so the
// workgroups sharing a pixel row's cache lines are dispatched together.
static int g_gn_cb_wg = 512;  // target workgroups of the channel-blocked apply; 0 = off
static int g_gn_cb_mult = 2;  // channel block = this many lcm(8, C/G) units (<= 16 groups); 2: -0.03 ms/step vs 1 (profiles/unet_step_ab_gn_cb_mult_r5f.txt, _r5g)
CSK_API int csk_set_gn_cb(int wg) {
  g_gn_cb_wg = wg;
  return 0;
}
CSK_API int csk_set_gn_cb_mult(int m) {
  g_gn_cb_mult = m;
  return 0;
}
// grids below a quarter of the workgroup target (batch-1 jobs) switch to
// single-unit blocks and one row per thread minimum, for more workgroups
static int g_gn_cb_small = 1;
CSK_API int csk_set_gn_cb_small(int v) {
  g_gn_cb_small = v;
  return 0;
}

__global__ __launch_bounds__(GN_THREADS) void gn_apply_cb_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                 const float* __restrict__ part,
                                                                 const float* __restrict__ part2,
                                                                 const bf16_t* __restrict__ gamma,
                                                                 const bf16_t* __restrict__ beta, int P, int C, int G,
                                                                 int CB, int chunk, int silu, int affine_bstride,
                                                                 int nseg, int seg_rows, float eps,
                                                                 const bf16_t* __restrict__ x2, int C1) {
  __shared__ float gst[2 * 16];
  if (!x2) C1 = C;
  const int cb = blockIdx.x, ck = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
  gamma += (size_t)b * affine_bstride;
  beta += (size_t)b * affine_bstride;
  const int Cg = C / G, ng = CB / Cg, gbase = cb * ng;
  const int NVC = CB >> 3, R = GN_THREADS / NVC;
  const int cv = tid % NVC, r = tid / NVC;
  const bool rows = r < R;
  const int c0 = cb * CB + cv * 8;
  const int p0 = ck * chunk, p1 = min(P, p0 + chunk);
  const bool second = c0 >= C1;  // this column vector lives in x2
  const int xst = second ? C - C1 : C1;
  const bf16_t* xsrc = (second ? x2 : x) + (size_t)b * P * xst + (second ? c0 - C1 : c0);
  bf16_t* ydst = y + (size_t)b * P * C + c0;
  // The first unrolled batch of x rows and the affine parameters do not depend
  // on the statistics: issued before the partials merge so the two memory round
  // trips overlap (at batch-1 grids that batch is a thread's whole chunk).
  uint4 q[GN_UNROLL];
  uint4 gq = make_uint4(0, 0, 0, 0), bq = make_uint4(0, 0, 0, 0);
  const bool avec = ((((size_t)(gamma + c0)) | ((size_t)(beta + c0))) & 15) == 0;
  if (rows) {
#pragma unroll
    for (int u = 0; u < GN_UNROLL; ++u) q[u] = *reinterpret_cast<const uint4*>(xsrc + (size_t)min(p0 + r + u * R, p1 - 1) * xst);
    if (avec) {
      gq = *reinterpret_cast<const uint4*>(gamma + c0);
      bq = *reinterpret_cast<const uint4*>(beta + c0);
    }
  }
  for (int w = tid >> 6; w < ng; w += GN_THREADS / 64) {  // whole waves: wave w merges group gbase + w
    const int g = gbase + w;
    const float fn = (float)seg_rows;
    float mean, rstd;
    group_moments_wave(
        [&](int e, float& n, float& m, float& qq) {
          const int sg = b * nseg + e / Cg, c = g * Cg + e % Cg;
          const float2 mq = load_part(part, part2, sg, c, C, C1);
          n = fn; m = mq.x; qq = mq.y;
        },
        nseg * Cg, tid & 63, mean, rstd, eps);
    if ((tid & 63) == 0) {
      gst[2 * w] = mean;
      gst[2 * w + 1] = rstd;
    }
  }
  __syncthreads();
  if (!rows) return;
  float gf[8], bfv[8], sa[8], sb[8];
  if (avec) {
    unpack8(gq, gf);
    unpack8(bq, bfv);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gf[j] = bf2f(gamma[c0 + j]);
      bfv[j] = bf2f(beta[c0 + j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int lg = (c0 + j) / Cg - gbase;
    const float a = gf[j] * gst[2 * lg + 1];
    sa[j] = a;
    sb[j] = bfv[j] - gst[2 * lg] * a;
  }
  for (int p = p0 + r; p < p1; p += GN_UNROLL * R) {
    if (p != p0 + r) {
#pragma unroll
      for (int u = 0; u < GN_UNROLL; ++u) q[u] = *reinterpret_cast<const uint4*>(xsrc + (size_t)min(p + u * R, p1 - 1) * xst);
    }
#pragma unroll
    for (int u = 0; u < GN_UNROLL; ++u) {
      const int pp = p + u * R;
      if (pp < p1) {
        float f[8];
        unpack8(q[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = f[j] * sa[j] + sb[j];
          f[j] = silu == 1 ? silu_f(t) : (silu == 2 ? gelu_f(t) : t);
        }
        *reinterpret_cast<uint4*>(ydst + (size_t)pp * C) = pack8(f);
      }
    }
  }
}

// stat: B*G*2 floats of workspace
// x2 / C1: optional second input (channel concat [x | x2], x has C1 channels)
// part2: optional partials of x2's channels (then `part` holds only x's), so a
// skip concat's two producers' statistics are merged without concatenating them
CSK_API int csk_group_norm_part2(void* y, const void* x, const void* x2, int C1, const void* part, const void* part2,
                                 int seg_rows, void* stat, const void* gamma, const void* beta, int B, int P, int C,
                                 int G, int chunk, int nchunk, float eps, int silu, int affine_bstride,
                                 hipStream_t stream) {
  if (C % 8 != 0 || C > GN_MAXC || C % G != 0 || seg_rows <= 0 || P % seg_rows != 0) return (int)hipErrorInvalidValue;
  if (x2 && (C1 <= 0 || C1 >= C || C1 % 8 != 0)) return (int)hipErrorInvalidValue;
  if (part2 && !x2) return (int)hipErrorInvalidValue;
  float* st = (float*)stat;
  const int nseg = P / seg_rows;
  if (g_gn_cb_wg > 0) {
    const int Cg = C / G;
    int CB0 = 8;
    while (CB0 % Cg) CB0 += 8;  // lcm(8, Cg)
    int CB = CB0;
    for (int m = g_gn_cb_mult; m > 1; --m)  // wider blocks (fewer, longer row segments) when they divide C
      if (C % (CB0 * m) == 0 && CB0 * m / Cg <= 16 && CB0 * m <= 1024) {
        CB = CB0 * m;
        break;
      }
    if (CB0 / Cg <= 16 && CB0 <= 1024 && C % CB0 == 0 && nseg * Cg <= 1024) {
      // ~g_gn_cb_wg workgroups in all, >= minr rows per thread (4: the unroll)
      int nblk = 0, ch = 0, nch = 0;
      auto plan = [&](int cbw, int minr) {
        nblk = C / cbw;
        const int R = GN_THREADS / (cbw / 8);
        ch = max(minr * R, (int)(((long)P * B * nblk + g_gn_cb_wg - 1) / g_gn_cb_wg));
        nch = (P + ch - 1) / ch;
        ch = (P + nch - 1) / nch;
        return (long)nblk * nch * B;
      };
      if (plan(CB, 4) * 4 < g_gn_cb_wg && g_gn_cb_small) {
        CB = CB0;
        plan(CB, 1);
      }
      gn_apply_cb_kernel<<<dim3(nblk, nch, B), GN_THREADS, 0, stream>>>(
          (const bf16_t*)x, (bf16_t*)y, (const float*)part, (const float*)part2, (const bf16_t*)gamma,
          (const bf16_t*)beta, P, C, G, CB, ch, silu, affine_bstride, nseg, seg_rows, eps, (const bf16_t*)x2, C1);
      CSK_CHECK_LAUNCH();
    }
  }
  // every apply workgroup re-reads ALL of its sample's partials in a prologue
  // merge; past ~1K entries that L2 traffic (1024 workgroups x nseg*C*8 bytes)
  // costs more than a finalize launch (measured: 24 vs ~12 us at 64x64x320 B8)
  if (G <= 64 && nseg * C <= g_gn_prologue_max) {
    gn_apply_kernel<2><<<dim3(nchunk, B), GN_THREADS, 0, stream>>>(
        (const bf16_t*)x, (bf16_t*)y, (const float*)part, (const bf16_t*)gamma, (const bf16_t*)beta, P, C, G, chunk,
        silu, affine_bstride, nseg, seg_rows, eps, (const bf16_t*)x2, C1, (const float*)part2);
    CSK_CHECK_LAUNCH();
  }
  if (nseg * (C / G) > g_gn_wg_min)  // large VAE maps (> one round trip of the wave kernel): a workgroup per group
    gn_finalize_part_wg_kernel<<<B * G, 256, 0, stream>>>((const float*)part, st, B, C, G, nseg, seg_rows, eps,
                                                          (const float*)part2, C1);
  else
    gn_finalize_part_kernel<<<(B * G + GN_THREADS / 64 - 1) / (GN_THREADS / 64), GN_THREADS, 0, stream>>>(
        (const float*)part, st, B, C, G, nseg, seg_rows, eps, (const float*)part2, C1);
  gn_apply_kernel<0><<<dim3(nchunk, B), GN_THREADS, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, st,
                                                                 (const bf16_t*)gamma, (const bf16_t*)beta, P, C, G,
                                                                 chunk, silu, affine_bstride, 0, 0, eps,
                                                                 (const bf16_t*)x2, C1);
  CSK_CHECK_LAUNCH();
}

// Statistics only: (mean, rstd) per (sample, group) merged from the producer's
// epilogue partials, for a consumer that applies the GroupNorm itself (the
// fused transformer-input kernel, xin.hip).  stat: B*G*2 floats.
CSK_API int csk_gn_finalize(void* stat, const void* part, const void* part2, int C1, int seg_rows, int B, int P, int C,
                            int G, float eps, hipStream_t stream) {
  if (C % G != 0 || seg_rows <= 0 || P % seg_rows != 0 || !stat || !part) return (int)hipErrorInvalidValue;
  const int nseg = P / seg_rows;
  if (nseg * (C / G) > g_gn_wg_min)
    gn_finalize_part_wg_kernel<<<B * G, 256, 0, stream>>>((const float*)part, (float*)stat, B, C, G, nseg, seg_rows,
                                                          eps, (const float*)part2, C1);
  else
    gn_finalize_part_kernel<<<(B * G + GN_THREADS / 64 - 1) / (GN_THREADS / 64), GN_THREADS, 0, stream>>>(
        (const float*)part, (float*)stat, B, C, G, nseg, seg_rows, eps, (const float*)part2, C1);
  return (int)hipGetLastError();
}

CSK_API int csk_group_norm_part(void* y, const void* x, const void* x2, int C1, const void* part, int seg_rows,
                                void* stat, const void* gamma, const void* beta, int B, int P, int C, int G, int chunk,
                                int nchunk, float eps, int silu, int affine_bstride, hipStream_t stream) {
  return csk_group_norm_part2(y, x, x2, C1, part, nullptr, seg_rows, stat, gamma, beta, B, P, C, G, chunk, nchunk,
                              eps, silu, affine_bstride, stream);
}

// part: B*nchunk*G*3 floats followed by B*G*2 floats of final stats
// x2 / C1: optional second input (channel concat [x | x2] read in place, x has C1 channels)
CSK_API int csk_group_norm(void* y, const void* x, const void* x2, int C1, void* part, const void* gamma,
                           const void* beta, int B, int P, int C, int G, int chunk, int nchunk, float eps, int silu,
                           int affine_bstride, hipStream_t stream) {
  if (C % 8 != 0 || C > GN_MAXC || C % G != 0) return (int)hipErrorInvalidValue;
  if (x2 && (C1 <= 0 || C1 >= C || C1 % 8 != 0)) return (int)hipErrorInvalidValue;
  float* pt = (float*)part;
  float* st = pt + (size_t)B * nchunk * G * 3;
  dim3 grid(nchunk, B);
  gn_stats_kernel<<<grid, GN_THREADS, gn_stats_lds(C), stream>>>((const bf16_t*)x, pt, P, C, G, chunk, nchunk,
                                                                 (const bf16_t*)x2, C1);
  if (G <= 64 && nchunk * G <= g_gn_prologue_max) {  // few partials: merge them in the apply prologue (no finalize launch)
    gn_apply_kernel<1><<<grid, GN_THREADS, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, pt, (const bf16_t*)gamma,
                                                        (const bf16_t*)beta, P, C, G, chunk, silu, affine_bstride,
                                                        nchunk, 0, eps, (const bf16_t*)x2, C1);
    CSK_CHECK_LAUNCH();
  }
  gn_finalize_kernel<<<(B * G + GN_THREADS / 64 - 1) / (GN_THREADS / 64), GN_THREADS, 0, stream>>>(pt, st, B, G,
                                                                                                  nchunk, eps);
  gn_apply_kernel<0><<<grid, GN_THREADS, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, st, (const bf16_t*)gamma,
                                                      (const bf16_t*)beta, P, C, G, chunk, silu, affine_bstride, 0,
                                                      0, eps, (const bf16_t*)x2, C1);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// LayerNorm: a row is owned by LPR lanes (a power of two dividing 64), each
// holding VPL 16-byte vectors in registers, so one wave normalises 64/LPR rows
// and issues VPL loads per lane up front.  One wave per row (the earlier form)
// left 24 of 64 lanes idle at C = 320 and kept only 640 B in flight per wave:
// the UNet's LayerNorms ran at 2.3-3.5 TB/s, latency-bound.  Reductions are
// xor-shuffles inside the lane group.
// --------------------------------------------------------------------------
template <int VPL>
__global__ __launch_bounds__(256) void layer_norm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         const bf16_t* __restrict__ gamma,
                                                         const bf16_t* __restrict__ beta, int rows, int C, float eps,
                                                         int lpr_log2) {
  const int lane = threadIdx.x & 63;
  const int LPR = 1 << lpr_log2;
  const int rpw = 64 >> lpr_log2;  // rows per wave
  const int sub = lane & (LPR - 1);
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * rpw + (lane >> lpr_log2);
  const bool live = row < rows;
  const int NV = C >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)(live ? row : 0) * C);
  uint4 raw[VPL];
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int cv = sub + LPR * u;
    raw[u] = (live && cv < NV) ? xr[cv] : make_uint4(0, 0, 0, 0);
  }
  float f[VPL][8];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    unpack8(raw[u], f[u]);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += f[u][j];
  }
  for (int o = LPR >> 1; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    if (sub + LPR * u < NV) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = f[u][j] - mean; q += d * d; }
    }
  }
  for (int o = LPR >> 1; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rstd = rsqrtf(q / (float)C + eps);
  if (!live) return;
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * C);
#pragma unroll
  for (int u = 0; u < VPL; ++u) {
    const int cv = sub + LPR * u;
    if (cv < NV) {
      float gg[8], bb[8], o[8];
      unpack8(reinterpret_cast<const uint4*>(gamma)[cv], gg);
      if (beta) {
        unpack8(reinterpret_cast<const uint4*>(beta)[cv], bb);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bb[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (f[u][j] - mean) * rstd * gg[j] + bb[j];
      yr[cv] = pack8(o);
    }
  }
}

CSK_API int csk_layer_norm(void* y, const void* x, const void* gamma, const void* beta, int rows, int C, float eps,
                           hipStream_t stream) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  const int nv = C / 8;
  if (nv > 64 * 8) return (int)hipErrorInvalidValue;
  // smallest lane group with <= 8 vectors per lane: C = 320 -> 8 lanes x 5,
  // 640 -> 16 x 5, 1280 -> 32 x 5, 768 -> 16 x 6, 1024 -> 16 x 8
  int l2 = 0;
  while ((1 << l2) * 8 < nv) ++l2;
  const int vpl = (nv + (1 << l2) - 1) >> l2;
  const int rows_per_block = 4 * (64 >> l2);
  const dim3 grid((rows + rows_per_block - 1) / rows_per_block);
#define CSK_LN(V)                                                                                                  \
  layer_norm_kernel<V><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,               \
                                                 (const bf16_t*)beta, rows, C, eps, l2)
  switch (vpl) {
    case 1: CSK_LN(1); break;
    case 2: CSK_LN(2); break;
    case 3: CSK_LN(3); break;
    case 4: CSK_LN(4); break;
    case 5: CSK_LN(5); break;
    case 6: CSK_LN(6); break;
    default: CSK_LN(8); break;
  }
#undef CSK_LN
  CSK_CHECK_LAUNCH();
}
