// Shared helpers for the gfx950 (CDNA4, wave64) kernels of chiaswarm_amd.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short bf16_t;  // storage type of bfloat16
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef unsigned int u32;

#define CSK_API extern "C" __attribute__((visibility("default")))

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((u32)x) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(bf16_t, b);
}

typedef float csk_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 csk_b2 __attribute__((ext_vector_type(2)));

// ONE v_cvt_pk_bf16_f32 (RNE) for both halves; packing two scalar conversions
// costs 4 VALU (2 cvt + shift + or), which the attention softmax and every
// epilogue / normalisation store paid per output pair.
__device__ __forceinline__ u32 pack2(float lo, float hi) {
  const csk_f2 v = {lo, hi};
  return __builtin_bit_cast(u32, __builtin_convertvector(v, csk_b2));
}

// 8 bf16 <-> 8 floats through a 16-byte vector
__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 v;
  v.x = pack2(f[0], f[1]); v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]); v.w = pack2(f[6], f[7]);
  return v;
}

// Activations on the VALU-issue-bound paths (GroupNorm+SiLU apply, GEGLU and
// GEMM epilogues): v_rcp_f32 instead of an IEEE divide (~10 instructions), and
// erf from Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7; GELU |err| <= 6.5e-7 over
// [-12, 12] against the exact form) instead of the branchy libm erff, whose two
// polynomial paths both run when a wave's lanes straddle |x| = 1.
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float gelu_f(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, z, 1.0f));
  float p = __builtin_fmaf(t, 1.061405429f, -1.453152027f);
  p = __builtin_fmaf(t, p, 1.421413741f);
  p = __builtin_fmaf(t, p, -0.284496736f);
  p = __builtin_fmaf(t, p, 0.254829592f);
  const float q = p * t * __expf(-z * z);  // erfc(|x| / sqrt 2)
  return 0.5f * x * (x >= 0.f ? 2.0f - q : q);
}
__device__ __forceinline__ float qgelu_f(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-1.702f * x)); }
// GELU of the GEGLU epilogues (the gate of every UNet feed-forward: 10-42 M
// evaluations per call, where the A-S erf form above made the epilogue VALU
// bound): the tanh form x * sigmoid(2 sqrt(2/pi) (x + 0.044715 x^3)) in
// 5 VALU + 2 transcendental ops instead of ~13 + 2.  |err| vs the exact GELU
// <= 4.7e-4 over [-12, 12] (near |x| ~ 2, relative ~2.4e-4): ~15x below the
// bf16 rounding of the product it feeds.
__device__ __forceinline__ float gelu_geglu(float x) {
  const float u = x * __builtin_fmaf(x * x, -0.1029432396f, -2.302208198f);  // -log2(e) * 1.59577 (x + 0.044715 x^3)
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u));
}

// Single-instruction max / add for values straight out of MFMA accumulators:
// hipcc inserts a canonicalising v_max before every fmaxf on them and SLP-packs
// adjacent f32 adds into v_pk_add_f32 (an anti-lever beside MFMAs,
// MI355X_MICROARCH.md constants table) — inline asm keeps each one instruction.
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vadd(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// vadd for operands that may be FRESH transcendental results (v_exp / v_rcp ...):
// CDNA3/4 need one wait state between a trans op and a VALU reading its result
// (trans forwarding hazard) and hipcc pads none before an inline-asm reader —
// a plain vadd scheduled right behind its v_exp reads the pre-exp value.
// (_build.py lints every kernel's assembly for that adjacency.)
__device__ __forceinline__ float vadd_t(float a, float b) {
  float r;
  asm("s_nop 0\n\tv_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// MFMA result -> inline-asm reader: hipcc pads no wait states for an asm
// statement (cdna_hip_programming.md §5.7 item 2), and the softmax's vmax3
// reads score accumulators straight out of the matrix cores.  This nop
// statement names the accumulators ("+v": ordered after the MFMAs that write
// them, before any reader) and covers the XDL write -> read distance: 12 states
// for the 8-pass 16x16x32, 18 for the 16-pass 32x32x16.
__device__ __forceinline__ void mfma_fence4(v4f& a, v4f& b, v4f& c, v4f& d) {
  asm volatile("s_nop 7\n\ts_nop 3" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
__device__ __forceinline__ void mfma_fence16(v16f& a, v16f& b) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 1" : "+v"(a), "+v"(b));
}
// max over lanes {l, l^16, l^32, l^48} (the four 16-lane row groups of a
// 16x16 MFMA fragment) with two permlane swaps: no LDS round trip (the
// ds_bpermute that __shfl_xor lowers to sat in the softmax's critical chain)
__device__ __forceinline__ float max_rowgroups(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float m = vmax3(__uint_as_float(a[0]), __uint_as_float(a[1]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return vmax3(__uint_as_float(b[0]), __uint_as_float(b[1]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Chan et al. parallel combination of (count, mean, M2) partial moments.
__device__ __forceinline__ void chan_combine(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  float nn = n + nb;
  if (nn <= 0.f) return;
  float d = meanb - mean;
  float r = nb / nn;
  mean += d * r;
  m2 += m2b + d * d * n * r;
  n = nn;
}

// Bijective XCD-aware remap of a linear workgroup id (MI355X: 8 XCDs, blocks
// dealt round-robin; consecutive remapped ids land on one XCD's L2).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int NX = 8;
  if (nwg < NX) return bid;
  int q = nwg / NX, r = nwg % NX, x = bid % NX;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / NX;
}

#define CSK_CHECK_LAUNCH() return (int)hipGetLastError()

// ---- CSK_DEBUG builds (python -m chiaswarm_amd._build --debug -> libcsk_debug.so) ----
// Device-side checks record the FIRST violation per translation unit into a
// device record {count, site, block.x, thread, value lo, value hi, limit,
// block.y} instead of trapping (a trap would take the GPU down with it); the
// host reads it after a synchronise (csk_debug_read_<tu>) and the GPU test
// suite fails any test that left a record (tests/conftest.py).  Release builds
// compile every check away.
#ifdef CSK_DEBUG
static __device__ unsigned int csk_dbg_rec[8];
static __device__ __noinline__ void csk_dbg_fail(int site, long long v, long long lim) {
  if (atomicAdd(&csk_dbg_rec[0], 1u) == 0u) {
    csk_dbg_rec[1] = (unsigned)site;
    csk_dbg_rec[2] = blockIdx.x;
    csk_dbg_rec[3] = threadIdx.x;
    csk_dbg_rec[4] = (unsigned)(v & 0xffffffffll);
    csk_dbg_rec[5] = (unsigned)(v >> 32);
    csk_dbg_rec[6] = (unsigned)lim;
    csk_dbg_rec[7] = blockIdx.y;
  }
}
#define CSK_DCHECK(cond, site, v, lim) \
  do {                                 \
    if (!(cond)) csk_dbg_fail((site), (long long)(v), (long long)(lim)); \
  } while (0)
#define CSK_DEBUG_EXPORT(tu)                                                                              \
  CSK_API int csk_debug_read_##tu(unsigned* out) {                                                      \
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(csk_dbg_rec), sizeof(csk_dbg_rec), 0, hipMemcpyDeviceToHost); \
  }                                                                                                     \
  CSK_API int csk_debug_clear_##tu() {                                                                  \
    const unsigned z[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                                     \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(csk_dbg_rec), z, sizeof(z), 0, hipMemcpyHostToDevice);     \
  }
#else
#define CSK_DCHECK(cond, site, v, lim) \
  do {                                 \
  } while (0)
#define CSK_DEBUG_EXPORT(tu)
#endif
