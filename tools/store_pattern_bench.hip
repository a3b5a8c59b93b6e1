// Store-shape microbenchmark: how fast does a wave write a [M][N] bf16 matrix
// when each 16-byte-per-lane store instruction covers R rows x (1024 / R) bytes?
// The GEMM direct epilogue (gemm_common.h) stores 16 rows x 64 B per
// instruction; this measures it against 8 rows x 128 B (full cache lines) on
// 128 x 64 output tiles at the UNet's K = 320 output shapes.
//   hipcc --offload-arch=gfx950 -O3 -o store_pattern_bench tools/store_pattern_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>

template <int R>
__global__ __launch_bounds__(256) void store_kernel(uint4* __restrict__ out, int M, int N16, int tiles_n) {
  // a workgroup writes a 128-row x 64-column tile (128 B of each row), 4 waves x 32 rows
  const int t = blockIdx.x;
  const int m0 = (t / tiles_n) * 128, c0 = (t % tiles_n) * 8;  // c0 in 16-B units (8 per 128 B)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint4 v = make_uint4(lane, t, 1, 2);
  // each wave: 32 rows x 8 chunks = 256 chunks = 4 instructions of 64 lanes
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = k * 64 + lane;           // chunk index within the wave's 32 x 8 block
    int row, chunk;
    if (R == 8) {                            // 8 rows x 8 chunks (128 B) per instruction
      row = idx / 8;
      chunk = idx % 8;
    } else {                                 // R = 16: 16 rows x 4 chunks per instruction
      const int half = k & 1, rb = k >> 1;   // instruction k: rows rb*16 .. +16, chunks half*4 .. +4
      row = rb * 16 + (lane & 15);
      chunk = half * 4 + (lane >> 4);
    }
    const int m = m0 + wave * 32 + row;
    if (m < M && c0 + chunk < N16) out[(size_t)m * N16 + c0 + chunk] = v;
  }
}

template <int R>
static float run(uint4* out, int M, int N) {
  const int N16 = N / 8, tiles_n = N16 / 8, grid = (M / 128) * tiles_n;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) store_kernel<R><<<grid, 256>>>(out, M, N16, tiles_n);
  hipEventRecord(a);
  const int it = 20;
  for (int i = 0; i < it; ++i) store_kernel<R><<<grid, 256>>>(out, M, N16, tiles_n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / it;
}

int main() {
  const int shapes[3][2] = {{32768, 320}, {32768, 960}, {8192, 1280}};
  uint4* out = nullptr;
  if (hipMalloc(&out, (size_t)32768 * 1280 * 2) != hipSuccess) return 1;
  for (auto& s : shapes) {
    const int M = s[0], N = s[1];
    const double mb = (double)M * N * 2 / 1e6;
    const float t16 = run<16>(out, M, N), t8 = run<8>(out, M, N);
    std::printf("M%d N%d (%.1f MB): 16 rows x 64 B %.1f us (%.2f TB/s)   8 rows x 128 B %.1f us (%.2f TB/s)\n", M, N,
                mb, t16, mb / t16, t8, mb / t8);
  }
  hipFree(out);
  return 0;
}
