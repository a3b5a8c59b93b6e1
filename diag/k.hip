#include <hip/hip_runtime.h>
__global__ void addone(float* x, int n) { int i = blockIdx.x * blockDim.x + threadIdx.x; if (i < n) x[i] += 1.0f; }
extern "C" int diag_launch(float* x, int n, hipStream_t s) {
  addone<<<(n + 255) / 256, 256, 0, s>>>(x, n);
  return (int)hipGetLastError();
}
extern "C" int diag_selftest() {
  float* d; hipMalloc(&d, 1024 * 4); hipMemset(d, 0, 4096);
  addone<<<4, 256>>>(d, 1024); float h[4]; hipMemcpy(h, d, 16, hipMemcpyDeviceToHost); hipFree(d);
  return (int)(h[0] * 100);
}
