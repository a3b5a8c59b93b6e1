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

// partial layout: part[((b * nchunk + chunk) * G + g) * 3 + {0:n, 1:mean, 2:M2}]
__global__ __launch_bounds__(GN_THREADS) void gn_stats_kernel(const bf16_t* __restrict__ x, float* __restrict__ part,
                                                              int P, int C, int G, int chunk, int nchunk) {
  __shared__ float red[2][GN_MAXC];
  const int b = blockIdx.y, ck = blockIdx.x;
  const int NV = C >> 3;
  const int tid = threadIdx.x;
  const int p0 = ck * chunk;
  const int p1 = min(P, p0 + chunk);
  const bf16_t* xb = x + (size_t)b * P * C;
  // vector slots handled by this thread: cv = tid, tid+256 (C <= 4096 -> NV <= 512)
  const int R = NV >= GN_THREADS ? 1 : GN_THREADS / NV;  // pixel rows per pass
  float s[2][8], ss[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[u][j] = ss[u][j] = 0.f;
  if (NV < GN_THREADS) {
    const int cv = tid % NV, r = tid / NV;
    if (r < R) {
      for (int p = p0 + r; p < p1; p += R) {
        uint4 v = *reinterpret_cast<const uint4*>(xb + (size_t)p * C + cv * 8);
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) { s[0][j] += f[j]; ss[0][j] += f[j] * f[j]; }
      }
    }
  } else {
    for (int p = p0; p < p1; ++p) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        int cv = tid + u * GN_THREADS;
        if (cv < NV) {
          uint4 v = *reinterpret_cast<const uint4*>(xb + (size_t)p * C + cv * 8);
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) { s[u][j] += f[j]; ss[u][j] += f[j] * f[j]; }
        }
      }
    }
  }
  // reduce over rows -> per-channel sums in LDS
  const int Cg = C / G;
  for (int i = tid; i < C; i += GN_THREADS) { red[0][i] = 0.f; red[1][i] = 0.f; }
  __syncthreads();
  if (NV < GN_THREADS) {
    const int cv = tid % NV, r = tid / NV;
    if (r < R) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { atomicAdd(&red[0][cv * 8 + j], s[0][j]); atomicAdd(&red[1][cv * 8 + j], ss[0][j]); }
    }
  } else {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int cv = tid + u * GN_THREADS;
      if (cv < NV) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { red[0][cv * 8 + j] = s[u][j]; red[1][cv * 8 + j] = ss[u][j]; }
      }
    }
  }
  __syncthreads();
  for (int g = tid; g < G; g += GN_THREADS) {
    const int c0 = g * Cg;
    float sm = 0.f, sq = 0.f;
    for (int c = c0; c < c0 + Cg; ++c) { sm += red[0][c]; sq += red[1][c]; }
    float n = (float)(p1 - p0) * (float)Cg;
    float mean = n > 0.f ? sm / n : 0.f;
    float m2 = fmaxf(sq - sm * mean, 0.f);
    float* o = part + (((size_t)b * nchunk + ck) * G + g) * 3;
    o[0] = n; o[1] = mean; o[2] = m2;
  }
}

__global__ __launch_bounds__(GN_THREADS) void gn_apply_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                              const float* __restrict__ part,
                                                              const bf16_t* __restrict__ gamma, const bf16_t* __restrict__ beta,
                                                              int P, int C, int G, int chunk, int nchunk, float eps, int silu) {
  __shared__ float sa[GN_MAXC], sb[GN_MAXC];
  __shared__ float smean[128], srstd[128];
  const int b = blockIdx.y, ck = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // 1) merge chunk partials per group (one wave per group)
  for (int g = wid; g < G; g += GN_THREADS / 64) {
    float n = 0.f, mean = 0.f, m2 = 0.f;
    for (int c = lane; c < nchunk; c += 64) {
      const float* pp = part + (((size_t)b * nchunk + c) * G + g) * 3;
      chan_combine(n, mean, m2, pp[0], pp[1], pp[2]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float n2 = __shfl_xor(n, o, 64), me2 = __shfl_xor(mean, o, 64), q2 = __shfl_xor(m2, o, 64);
      chan_combine(n, mean, m2, n2, me2, q2);
    }
    if (lane == 0) {
      smean[g] = mean;
      srstd[g] = rsqrtf(m2 / fmaxf(n, 1.f) + eps);
    }
  }
  __syncthreads();
  const int Cg = C / G;
  for (int c = tid; c < C; c += GN_THREADS) {
    int g = c / Cg;
    float a = bf2f(gamma[c]) * srstd[g];
    sa[c] = a;
    sb[c] = bf2f(beta[c]) - smean[g] * a;
  }
  __syncthreads();
  // 2) stream the chunk
  const int NV = C >> 3;
  const size_t base = ((size_t)b * P + (size_t)ck * chunk) * NV;
  const int p1 = min(P, (ck + 1) * chunk);
  const size_t nvec = (size_t)(p1 - ck * chunk) * NV;
  const uint4* xin = reinterpret_cast<const uint4*>(x) + base;
  uint4* yo = reinterpret_cast<uint4*>(y) + base;
  for (size_t i = tid; i < nvec; i += GN_THREADS) {
    int cv = (int)(i % NV);
    float f[8];
    unpack8(xin[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = f[j] * sa[cv * 8 + j] + sb[cv * 8 + j];
      f[j] = silu ? silu_f(v) : v;
    }
    yo[i] = pack8(f);
  }
}

CSK_API int csk_group_norm(void* y, const void* x, void* part, const void* gamma, const void* beta, int B, int P, int C,
                           int G, int chunk, int nchunk, float eps, int silu, hipStream_t stream) {
  if (C % 8 != 0 || C > GN_MAXC || G > 128 || C % G != 0) return (int)hipErrorInvalidValue;
  dim3 grid(nchunk, B);
  gn_stats_kernel<<<grid, GN_THREADS, 0, stream>>>((const bf16_t*)x, (float*)part, P, C, G, chunk, nchunk);
  gn_apply_kernel<<<grid, GN_THREADS, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const float*)part,
                                                   (const bf16_t*)gamma, (const bf16_t*)beta, P, C, G, chunk, nchunk,
                                                   eps, silu);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// LayerNorm: one wave per row, row held in registers (C <= 64*8*NVMAX).
// --------------------------------------------------------------------------
template <int NVMAX>
__global__ __launch_bounds__(256) void layer_norm_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         const bf16_t* __restrict__ gamma,
                                                         const bf16_t* __restrict__ beta, int rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int NV = C >> 3;
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * C);
  float f[NVMAX][8];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < NVMAX; ++u) {
    int cv = lane + 64 * u;
    if (cv < NV) {
      unpack8(xr[cv], f[u]);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[u][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[u][j] = 0.f;
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int u = 0; u < NVMAX; ++u) {
    int cv = lane + 64 * u;
    if (cv < NV) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { float d = f[u][j] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)C + eps);
  uint4* yr = reinterpret_cast<uint4*>(y + (size_t)row * C);
#pragma unroll
  for (int u = 0; u < NVMAX; ++u) {
    int cv = lane + 64 * u;
    if (cv < NV) {
      float gg[8], bb[8], o[8];
      unpack8(reinterpret_cast<const uint4*>(gamma)[cv], gg);
      unpack8(reinterpret_cast<const uint4*>(beta)[cv], bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (f[u][j] - mean) * rstd * gg[j] + bb[j];
      yr[cv] = pack8(o);
    }
  }
}

CSK_API int csk_layer_norm(void* y, const void* x, const void* gamma, const void* beta, int rows, int C, float eps,
                           hipStream_t stream) {
  if (C % 8 != 0) return (int)hipErrorInvalidValue;
  int nv = C / 8;
  dim3 grid((rows + 3) / 4);
  if (nv <= 64)
    layer_norm_kernel<1><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,
                                                    (const bf16_t*)beta, rows, C, eps);
  else if (nv <= 128)
    layer_norm_kernel<2><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,
                                                    (const bf16_t*)beta, rows, C, eps);
  else if (nv <= 256)
    layer_norm_kernel<4><<<grid, 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (const bf16_t*)gamma,
                                                    (const bf16_t*)beta, rows, C, eps);
  else
    return (int)hipErrorInvalidValue;
  CSK_CHECK_LAUNCH();
}
