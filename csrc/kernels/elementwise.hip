// Streaming kernels: SiLU, add, fused sampler step, VAE post-process
// to uint8 (K15), row softmax (VAE single-head attention), channel padding.
// All bf16 traffic is 16 bytes per lane (8 elements), grid-strided.
#include "common.h"
#include "gemm_common.h"  // apply_act

static inline int ew_grid(size_t nvec) {
  size_t g = (nvec + 255) / 256;
  return (int)(g < 4096 ? (g > 0 ? g : 1) : 4096);
}

// tails (n % 8 != 0): the last n % 8 elements go through a scalar loop in the
// same kernel, so every length runs on the GPU (no host-side torch fallback)
__global__ void silu_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, size_t nvec, const bf16_t* xs,
                            bf16_t* ys, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(x[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = silu_f(f[j]);
    y[i] = pack8(f);
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nvec * 8) {
    const size_t k = nvec * 8 + threadIdx.x;
    ys[k] = f2bf(silu_f(bf2f(xs[k])));
  }
}

CSK_API int csk_silu(void* y, const void* x, long long n, hipStream_t stream) {
  if (n <= 0) return 0;
  const size_t nv = n / 8;
  silu_kernel<<<ew_grid(nv > 0 ? nv : 1), 256, 0, stream>>>((const uint4*)x, (uint4*)y, nv, (const bf16_t*)x,
                                                             (bf16_t*)y, (size_t)n);
  CSK_CHECK_LAUNCH();
}

__global__ void add_kernel(const uint4* __restrict__ a, const uint4* __restrict__ b, uint4* __restrict__ y, size_t nvec,
                           const bf16_t* as, const bf16_t* bs, bf16_t* ys, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float fa[8], fb[8];
    unpack8(a[i], fa);
    unpack8(b[i], fb);
#pragma unroll
    for (int j = 0; j < 8; ++j) fa[j] += fb[j];
    y[i] = pack8(fa);
  }
  if (blockIdx.x == 0 && threadIdx.x < n - nvec * 8) {
    const size_t k = nvec * 8 + threadIdx.x;
    ys[k] = f2bf(bf2f(as[k]) + bf2f(bs[k]));
  }
}

// dst[r][:] = tab[*cur][:] for r < rows (bf16, width % 8 == 0): the step's row of
// a per-request table (the ResNet time projections of every timestep, computed
// once per job) broadcast to the batch inside the step graph
__global__ void row_bcast_kernel(uint4* __restrict__ dst, const uint4* __restrict__ tab, const int* __restrict__ cur,
                                 int rows, int wv, int n) {
  const int c = min(max(*cur, 0), n - 1);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rows * wv; i += gridDim.x * blockDim.x) {
    const int r = i / wv, v = i - r * wv;
    dst[(size_t)r * wv + v] = tab[(size_t)c * wv + v];
  }
}

CSK_API int csk_row_bcast(void* dst, const void* tab, const void* cur, int rows, int width, int n,
                          hipStream_t stream) {
  if (width % 8 != 0 || rows <= 0 || n <= 0) return (int)hipErrorInvalidValue;
  const int wv = width / 8;
  row_bcast_kernel<<<min((rows * wv + 255) / 256, 1024), 256, 0, stream>>>((uint4*)dst, (const uint4*)tab,
                                                                            (const int*)cur, rows, wv, n);
  CSK_CHECK_LAUNCH();
}

// y = [x; x] (a CFG-shared prefix result duplicated for both guidance halves):
// one read of x and two 16-byte stores per vector, one vector per thread over
// a full grid (a 4-vector-per-thread loop on a quarter grid ran at 1.4 TB/s)
__global__ void dup2_kernel(const uint4* __restrict__ x, uint4* __restrict__ y, size_t nvec) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = x[i];
    y[i] = v;
    y[nvec + i] = v;
  }
}

CSK_API int csk_dup2(void* y, const void* x, long long n, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n % 8 != 0 || (((size_t)x) & 15) != 0 || (((size_t)y) & 15) != 0) return (int)hipErrorInvalidValue;
  const size_t nv = n / 8;
  const size_t blocks = (nv + 255) / 256;
  dup2_kernel<<<(int)(blocks < 16384 ? blocks : 16384), 256, 0, stream>>>((const uint4*)x, (uint4*)y, nv);
  CSK_CHECK_LAUNCH();
}

CSK_API int csk_add(void* y, const void* a, const void* b, long long n, hipStream_t stream) {
  if (n <= 0) return 0;
  const size_t nv = n / 8;
  add_kernel<<<ew_grid(nv > 0 ? nv : 1), 256, 0, stream>>>((const uint4*)a, (const uint4*)b, (uint4*)y, nv,
                                                            (const bf16_t*)a, (const bf16_t*)b, (bf16_t*)y,
                                                            (size_t)n);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// Fused sampler step.  e: UNet output bf16 [(cfg?2:1)*n] (uncond half first),
// x, x0prev, noise: fp32 [n]; writes x_next fp32, x0 fp32.
//   e_g = e_u + g (e_c - e_u);  x0 = p x + q e_g;
//   x_next = A x + B x0 + C x0prev + D noise
// --------------------------------------------------------------------------
struct StepC {
  float p, q, A, B, C, D, g;
  int cfg, has_prev, has_noise;
};

__global__ void sched_step_kernel(const bf16_t* __restrict__ e, const float* __restrict__ x,
                                  const float* __restrict__ x0prev, const float* __restrict__ noise,
                                  float* __restrict__ xn, float* __restrict__ x0o, size_t n4, size_t n, StepC c) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 xv = reinterpret_cast<const float4*>(x)[i];
    uint2 eu = reinterpret_cast<const uint2*>(e)[i];
    float ev[4] = {__uint_as_float(eu.x << 16), __uint_as_float(eu.x & 0xffff0000u), __uint_as_float(eu.y << 16),
                   __uint_as_float(eu.y & 0xffff0000u)};
    if (c.cfg) {
      uint2 ec = reinterpret_cast<const uint2*>(e + n)[i];
      float cv[4] = {__uint_as_float(ec.x << 16), __uint_as_float(ec.x & 0xffff0000u), __uint_as_float(ec.y << 16),
                     __uint_as_float(ec.y & 0xffff0000u)};
#pragma unroll
      for (int j = 0; j < 4; ++j) ev[j] = ev[j] + c.g * (cv[j] - ev[j]);
    }
    float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    float pv[4] = {0, 0, 0, 0}, nz[4] = {0, 0, 0, 0};
    if (c.has_prev) {
      float4 t = reinterpret_cast<const float4*>(x0prev)[i];
      pv[0] = t.x; pv[1] = t.y; pv[2] = t.z; pv[3] = t.w;
    }
    if (c.has_noise) {
      float4 t = reinterpret_cast<const float4*>(noise)[i];
      nz[0] = t.x; nz[1] = t.y; nz[2] = t.z; nz[3] = t.w;
    }
    float o[4], z[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      z[j] = c.p * xs[j] + c.q * ev[j];
      o[j] = c.A * xs[j] + c.B * z[j] + c.C * pv[j] + c.D * nz[j];
    }
    reinterpret_cast<float4*>(xn)[i] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4*>(x0o)[i] = make_float4(z[0], z[1], z[2], z[3]);
  }
}

CSK_API int csk_sched_step(void* xn, void* x0o, const void* e, const void* x, const void* x0prev, const void* noise,
                           long long n, float p, float q, float A, float B, float C, float D, float g, int cfg,
                           hipStream_t stream) {
  if (n % 4) return (int)hipErrorInvalidValue;
  StepC c{p, q, A, B, C, D, g, cfg, x0prev != nullptr, noise != nullptr};
  size_t n4 = n / 4;
  sched_step_kernel<<<ew_grid(n4 / 2 + 1), 256, 0, stream>>>((const bf16_t*)e, (const float*)x, (const float*)x0prev,
                                                             (const float*)noise, (float*)xn, (float*)x0o, n4, n, c);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// Device-resident sampler loop (one hipGraph replay per denoising step, no
// host work between replays).  The per-step scalars live in a device table
// indexed by a device step counter:
//   loop_prologue (1 thread, head of the step graph): cur = counter++,
//     t_out = t_tab[cur]  -> the UNet's timestep input;
//   sched_loop (tail of the step graph): coefficients coef[cur] =
//     {p, q, A, B, C, D, s_next, g, g2, -, -, -} (g / g2: the request's guidance
//     scales, so one captured graph serves every guidance value), CFG combine (none / 2-way [u, c] /
//     3-way pix2pix [c, i, u]), x0 = p x + q e, x' = A x + B x0 + C x0prev +
//     D noise[cur], x and x0prev updated in place, and the NEXT UNet input
//     written directly: x_in[r] = bf16(s_next x') for every CFG replica r,
//     channels [0, 4) of a Cin-channel pixel (extra image-latent channels of
//     pix2pix / 9-channel inpaint stay as set up once per request).
// Replaces per step: x * s_in, bf16 cast, torch.cat of the CFG copies, the
// static-input copy, t.fill_ and the separate step launch.
// --------------------------------------------------------------------------
__global__ void loop_prologue_kernel(int* __restrict__ counter, int* __restrict__ cur,
                                     const float* __restrict__ t_tab, float* __restrict__ t_out, int n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int i = *counter;
    i = i < 0 ? 0 : (i >= n ? n - 1 : i);  // clamp: never index past the table
    *cur = i;
    *t_out = t_tab[i];
    *counter = i + 1;
  }
}

CSK_API int csk_loop_prologue(void* counter, void* cur, const void* t_tab, void* t_out, int n, hipStream_t stream) {
  if (n <= 0) return (int)hipErrorInvalidValue;
  loop_prologue_kernel<<<1, 64, 0, stream>>>((int*)counter, (int*)cur, (const float*)t_tab, (float*)t_out, n);
  CSK_CHECK_LAUNCH();
}

#define LOOP_COEF_STRIDE 12
__global__ void sched_loop_kernel(const bf16_t* __restrict__ e, float* __restrict__ x, float* __restrict__ x0prev,
                                  const float* __restrict__ noise_tab, const int* __restrict__ cur,
                                  const float* __restrict__ coef, bf16_t* __restrict__ xin, int cin, int nrep,
                                  size_t npix, int mode) {
  const int idx = *cur;
  const float* c = coef + (size_t)idx * LOOP_COEF_STRIDE;
  const float p = c[0], q = c[1], A = c[2], B = c[3], C = c[4], D = c[5], s = c[6], g = c[7], g2 = c[8];
  const float* nz = (noise_tab != nullptr && D != 0.f) ? noise_tab + (size_t)idx * npix * 4 : nullptr;
  const size_t n = npix * 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < npix; i += (size_t)gridDim.x * blockDim.x) {
    float4 xv = reinterpret_cast<const float4*>(x)[i];
    float4 pv = reinterpret_cast<const float4*>(x0prev)[i];
    uint2 e0 = reinterpret_cast<const uint2*>(e)[i];
    float ev[4] = {__uint_as_float(e0.x << 16), __uint_as_float(e0.x & 0xffff0000u), __uint_as_float(e0.y << 16),
                   __uint_as_float(e0.y & 0xffff0000u)};
    if (mode >= 1) {
      uint2 e1 = reinterpret_cast<const uint2*>(e + n)[i];
      float cv[4] = {__uint_as_float(e1.x << 16), __uint_as_float(e1.x & 0xffff0000u), __uint_as_float(e1.y << 16),
                     __uint_as_float(e1.y & 0xffff0000u)};
      if (mode == 1) {  // [u, c]: e = u + g (c - u)
#pragma unroll
        for (int j = 0; j < 4; ++j) ev[j] = ev[j] + g * (cv[j] - ev[j]);
      } else {  // [c, i, u]: e = u + g (c - i) + g2 (i - u)
        uint2 e2 = reinterpret_cast<const uint2*>(e + 2 * n)[i];
        float uv[4] = {__uint_as_float(e2.x << 16), __uint_as_float(e2.x & 0xffff0000u),
                       __uint_as_float(e2.y << 16), __uint_as_float(e2.y & 0xffff0000u)};
#pragma unroll
        for (int j = 0; j < 4; ++j) ev[j] = uv[j] + g * (ev[j] - cv[j]) + g2 * (cv[j] - uv[j]);
      }
    }
    float nv[4] = {0.f, 0.f, 0.f, 0.f};
    if (nz != nullptr) {
      float4 t = reinterpret_cast<const float4*>(nz)[i];
      nv[0] = t.x; nv[1] = t.y; nv[2] = t.z; nv[3] = t.w;
    }
    const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
    const float ps[4] = {pv.x, pv.y, pv.z, pv.w};
    float o[4], z[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      z[j] = p * xs[j] + q * ev[j];
      o[j] = A * xs[j] + B * z[j] + C * ps[j] + D * nv[j];
    }
    reinterpret_cast<float4*>(x)[i] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4*>(x0prev)[i] = make_float4(z[0], z[1], z[2], z[3]);
    const u32 lo = pack2(s * o[0], s * o[1]), hi = pack2(s * o[2], s * o[3]);
    for (int r = 0; r < nrep; ++r) {
      bf16_t* dst = xin + ((size_t)r * npix + i) * cin;
      if ((cin & 3) == 0) {
        *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
      } else {
        dst[0] = (bf16_t)(lo & 0xffffu); dst[1] = (bf16_t)(lo >> 16);
        dst[2] = (bf16_t)(hi & 0xffffu); dst[3] = (bf16_t)(hi >> 16);
      }
    }
  }
}

CSK_API int csk_sched_loop(const void* e, void* x, void* x0prev, const void* noise_tab, const void* cur,
                           const void* coef, void* xin, int cin, int nrep, long long npix, int mode,
                           hipStream_t stream) {
  // nrep = 1 with mode > 0: a CFG-parallel half (pipelines/sd.py _denoise_loop_split) combines the full
  // prediction but feeds only its own UNet half
  if (cin < 4 || nrep < 1 || nrep > 3 || npix <= 0 || mode < 0 || mode > 2 || (mode > 0 && nrep != 1 && mode + 1 != nrep))
    return (int)hipErrorInvalidValue;
  sched_loop_kernel<<<ew_grid((size_t)npix / 2 + 1), 256, 0, stream>>>(
      (const bf16_t*)e, (float*)x, (float*)x0prev, (const float*)noise_tab, (const int*)cur, (const float*)coef,
      (bf16_t*)xin, cin, nrep, (size_t)npix, mode);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// VAE post-process: NHWC bf16 [-1,1], C channels (3) -> uint8 NHWC.
// --------------------------------------------------------------------------
__global__ void vae_post_kernel(const bf16_t* __restrict__ x, unsigned char* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float v = bf2f(x[i]) * 0.5f + 0.5f;
    v = fminf(fmaxf(v, 0.f), 1.f);
    y[i] = (unsigned char)__float2int_rn(v * 255.f);
  }
}

CSK_API int csk_vae_post(void* y, const void* x, long long n, hipStream_t stream) {
  vae_post_kernel<<<ew_grid((size_t)n), 256, 0, stream>>>((const bf16_t*)x, (unsigned char*)y, (size_t)n);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// y = a*x + b*z  (RRDB residual scaling, ControlNet residual scale)
// --------------------------------------------------------------------------
__global__ void axpby_kernel(const uint4* __restrict__ x, const uint4* __restrict__ z, uint4* __restrict__ y, size_t nvec,
                             float a, float b) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nvec; i += (size_t)gridDim.x * blockDim.x) {
    float fx[8], fz[8];
    unpack8(x[i], fx);
    unpack8(z[i], fz);
#pragma unroll
    for (int j = 0; j < 8; ++j) fx[j] = a * fx[j] + b * fz[j];
    y[i] = pack8(fx);
  }
}

CSK_API int csk_axpby(void* y, const void* x, const void* z, long long n, float a, float b, hipStream_t stream) {
  if (n % 8) return (int)hipErrorInvalidValue;
  size_t nv = n / 8;
  axpby_kernel<<<ew_grid(nv), 256, 0, stream>>>((const uint4*)x, (const uint4*)z, (uint4*)y, nv, a, b);
  CSK_CHECK_LAUNCH();
}

// Strided NHWC form: y[p, c] = act(a*x[p, c] + b*z[p, c]) over P pixels x C
// channels, each operand with its own pixel stride (channel slices of wider
// buffers); z may be null.  Also the standalone activation op (HiFi-GAN
// pre-activations, multi-receptive-field averaging).
__global__ void axpby_nhwc_kernel(bf16_t* __restrict__ y, int ys, const bf16_t* __restrict__ x, int xs,
                                  const bf16_t* __restrict__ z, int zs, size_t P, int C, float a, float b, int act) {
  const int nv = C >> 3;
  const size_t total = P * nv;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t p = i / nv;
    const int c = (int)(i - p * nv) * 8;
    float fx[8], fz[8];
    unpack8(*reinterpret_cast<const uint4*>(x + p * xs + c), fx);
    if (z) {
      unpack8(*reinterpret_cast<const uint4*>(z + p * zs + c), fz);
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[j] = a * fx[j] + b * fz[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) fx[j] *= a;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) fx[j] = apply_act(act, fx[j]);
    *reinterpret_cast<uint4*>(y + p * ys + c) = pack8(fx);
  }
}

CSK_API int csk_axpby_nhwc(void* y, int ys, const void* x, int xs, const void* z, int zs, long long P, int C, float a,
                           float b, int act, hipStream_t stream) {
  if (C % 8 || ys % 8 || xs % 8 || zs % 8 || act == ACT_GEGLU) return (int)hipErrorInvalidValue;
  axpby_nhwc_kernel<<<ew_grid((size_t)P * (C / 8)), 256, 0, stream>>>((bf16_t*)y, ys, (const bf16_t*)x, xs,
                                                                       (const bf16_t*)z, zs, (size_t)P, C, a, b, act);
  CSK_CHECK_LAUNCH();
}

// --------------------------------------------------------------------------
// Channel pad: [R, Cin] -> [R, Cout] (zero fill), for Cin % 8 != 0 convs.
// --------------------------------------------------------------------------
__global__ void pad_channels_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, size_t rows, int cin, int cout) {
  size_t n = rows * cout;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    size_t r = i / cout;
    int c = (int)(i - r * cout);
    y[i] = c < cin ? x[r * cin + c] : (bf16_t)0;
  }
}

CSK_API int csk_pad_channels(void* y, const void* x, long long rows, int cin, int cout, hipStream_t stream) {
  pad_channels_kernel<<<ew_grid((size_t)rows * cout), 256, 0, stream>>>((const bf16_t*)x, (bf16_t*)y, (size_t)rows, cin,
                                                                         cout);
  CSK_CHECK_LAUNCH();
}

// Sinusoidal timestep embedding (diffusers `Timesteps`) in ONE launch
// (it was ~12 small torch kernels at the head of every UNet step):
//   freq_i = exp(-ln(max_period) * i / (half - shift)),  a = t[b] * freq_i
//   out[b] = flip ? [cos(a), sin(a)] : [sin(a), cos(a)]     (bf16)
// t: fp32 [B] with element stride ts (0 broadcasts one timestep over the batch).
__global__ void timestep_emb_kernel(bf16_t* __restrict__ y, const float* __restrict__ t, int ts, int B, int dim,
                                    int flip, float shift, float log_max_period) {
  const int half = dim / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * half) return;
  const int b = i / half, j = i - b * half;
  const float freq = expf(-log_max_period * (float)j / ((float)half - shift));
  const float a = t[(size_t)b * ts] * freq;
  const float s = sinf(a), c = cosf(a);
  bf16_t* yb = y + (size_t)b * dim;
  yb[j] = f2bf(flip ? c : s);
  yb[half + j] = f2bf(flip ? s : c);
}

CSK_API int csk_timestep_embedding(void* y, const void* t, int ts, int B, int dim, int flip, float shift,
                                   float max_period, hipStream_t stream) {
  if (dim % 2 != 0 || B <= 0) return (int)hipErrorInvalidValue;
  const int n = B * (dim / 2);
  timestep_emb_kernel<<<(n + 255) / 256, 256, 0, stream>>>((bf16_t*)y, (const float*)t, ts, B, dim, flip, shift,
                                                           logf(max_period));
  return (int)hipGetLastError();
}
