// Canny edge detector for the ControlNet-canny preprocessor (reference:
// cv2.Canny(np.array(rgb_image), 100, 200) at swarm/controlnet/input_processor.py:
// 77-81, i.e. on the 3-CHANNEL image; SURVEY §2.2 "Canny as a small HIP
// kernel").  Same definitions as controlnet/preprocess.py::canny_np, following
// OpenCV's canny.cpp: 3x3 Sobel with BORDER_REPLICATE per channel; for a
// multi-channel image each pixel takes the dx/dy of the channel with the
// largest L1 magnitude (first channel on ties); direction quantised to
// 0/45/90/135 degrees; non-maximum suppression against zero-padded
// neighbours, strict against the previous neighbour (left / up / up-left or
// up-right) and >= against the next; double threshold; 8-connected
// hysteresis (weak pixels survive when their component holds a strong one).
//
//   canny_grad_kernel : gray u8 -> magnitude f32 + direction u8
//   canny_nms_kernel  : -> label u8 (0 none, 1 weak, 2 strong)
//   canny_hyst_kernel : 32x32 tiles iterate weak->strong promotion in LDS
//                       until the tile is stable; sets a global "changed"
//                       flag when a tile changed, the host relaunches until a
//                       pass changes nothing (edges rarely cross > 2 tiles)
//   canny_out_kernel  : label -> 0/255
#include "common.h"

__device__ __forceinline__ int clampi(int i, int n) { return i < 0 ? 0 : (i >= n ? n - 1 : i); }

__global__ void canny_grad_kernel(const unsigned char* __restrict__ g, float* __restrict__ mag,
                                  unsigned char* __restrict__ dir, int H, int W, int C) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= W || y >= H) return;
  float gx = 0.f, gy = 0.f, best = -1.f;
  for (int c = 0; c < C; ++c) {
    float p[3][3];
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
      for (int dx = -1; dx <= 1; ++dx)
        p[dy + 1][dx + 1] = (float)g[((size_t)clampi(y + dy, H) * W + clampi(x + dx, W)) * C + c];
    const float cx = (p[0][2] + 2.f * p[1][2] + p[2][2]) - (p[0][0] + 2.f * p[1][0] + p[2][0]);
    const float cy = (p[2][0] + 2.f * p[2][1] + p[2][2]) - (p[0][0] + 2.f * p[0][1] + p[0][2]);
    const float m = fabsf(cx) + fabsf(cy);
    if (m > best) { best = m; gx = cx; gy = cy; }
  }
  mag[y * W + x] = best;
  // q = round(atan2(gy, gx) / (pi/4)) mod 4
  const float a = atan2f(gy, gx) * 1.27323954473516f;  // 4/pi
  int q = (int)rintf(a);
  q = ((q % 4) + 4) % 4;
  dir[y * W + x] = (unsigned char)q;
}

__global__ void canny_nms_kernel(const float* __restrict__ mag, const unsigned char* __restrict__ dir,
                                 unsigned char* __restrict__ lab, int H, int W, float low, float high) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= W || y >= H) return;
  auto M = [&](int yy, int xx) -> float { return (yy < 0 || yy >= H || xx < 0 || xx >= W) ? 0.f : mag[yy * W + xx]; };
  const float c = mag[y * W + x];
  float a, b;
  // a: previous neighbour (strict), b: next neighbour (>=), as cv2's canny.cpp
  switch (dir[y * W + x]) {
    case 0: a = M(y, x - 1); b = M(y, x + 1); break;
    case 1: a = M(y - 1, x - 1); b = M(y + 1, x + 1); break;
    case 2: a = M(y - 1, x); b = M(y + 1, x); break;
    default: a = M(y - 1, x + 1); b = M(y + 1, x - 1); break;
  }
  const float n = (c > a && c >= b) ? c : 0.f;
  lab[y * W + x] = n > high ? 2 : (n > low ? 1 : 0);
}

#define CT 32
__global__ __launch_bounds__(256) void canny_hyst_kernel(unsigned char* __restrict__ lab, int H, int W,
                                                         int* __restrict__ changed) {
  __shared__ unsigned char t[CT + 2][CT + 2];
  __shared__ int dirty;
  const int x0 = blockIdx.x * CT, y0 = blockIdx.y * CT;
  for (int i = threadIdx.x; i < (CT + 2) * (CT + 2); i += 256) {
    const int ty = i / (CT + 2), tx = i % (CT + 2);
    const int y = y0 + ty - 1, x = x0 + tx - 1;
    t[ty][tx] = (y >= 0 && y < H && x >= 0 && x < W) ? lab[y * W + x] : 0;
  }
  int tile_changed = 0;
  for (;;) {
    if (threadIdx.x == 0) dirty = 0;
    __syncthreads();
    for (int i = threadIdx.x; i < CT * CT; i += 256) {
      const int ty = i / CT + 1, tx = i % CT + 1;
      if (t[ty][tx] == 1) {
        bool s = false;
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
          for (int dx = -1; dx <= 1; ++dx) s |= t[ty + dy][tx + dx] == 2;
        if (s) { t[ty][tx] = 2; dirty = 1; }
      }
    }
    __syncthreads();
    if (!dirty) break;
    tile_changed = 1;
    __syncthreads();
  }
  if (tile_changed) {
    for (int i = threadIdx.x; i < CT * CT; i += 256) {
      const int ty = i / CT, tx = i % CT;
      const int y = y0 + ty, x = x0 + tx;
      if (y < H && x < W) lab[y * W + x] = t[ty + 1][tx + 1];
    }
    if (threadIdx.x == 0) atomicOr(changed, 1);
  }
}

__global__ void canny_out_kernel(const unsigned char* __restrict__ lab, unsigned char* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = lab[i] == 2 ? 255 : 0;
}

// ws: >= canny_ws_bytes(H, W) of 256-byte aligned device workspace
CSK_API int csk_canny(void* out, const void* img, int H, int W, int C, float low, float high, void* ws,
                      hipStream_t stream) {
  if (C < 1 || C > 4) return (int)hipErrorInvalidValue;
  // workspace layout (every region 256-byte aligned): [changed flag][mag f32][dir u8][label u8]
  char* w = (char*)ws;
  if (((size_t)w) & 255) return (int)hipErrorInvalidValue;
  const size_t hw = (size_t)H * W, a4 = (hw * 4 + 255) & ~(size_t)255, a1 = (hw + 255) & ~(size_t)255;
  int* changed = (int*)w;
  float* mag = (float*)(w + 256);
  unsigned char* dir = (unsigned char*)(w + 256 + a4);
  unsigned char* lab = dir + a1;
  dim3 b2(16, 16), g2((W + 15) / 16, (H + 15) / 16);
  canny_grad_kernel<<<g2, b2, 0, stream>>>((const unsigned char*)img, mag, dir, H, W, C);
  canny_nms_kernel<<<g2, b2, 0, stream>>>(mag, dir, lab, H, W, low, high);
  dim3 gt((W + CT - 1) / CT, (H + CT - 1) / CT);
  for (int pass = 0; pass < 4 * (H + W); ++pass) {  // bounded: a pass that changes nothing ends it
    int h_changed = 0;
    hipMemsetAsync(changed, 0, sizeof(int), stream);
    canny_hyst_kernel<<<gt, 256, 0, stream>>>(lab, H, W, changed);
    hipMemcpyAsync(&h_changed, changed, sizeof(int), hipMemcpyDeviceToHost, stream);
    hipStreamSynchronize(stream);
    if (!h_changed) break;
  }
  canny_out_kernel<<<(H * W + 255) / 256, 256, 0, stream>>>(lab, (unsigned char*)out, H * W);
  CSK_CHECK_LAUNCH();
}
