// NHWC max pooling (the ResNet stem's 3x3 / stride 2 / pad 1) forward + backward.
//
// Forward: each thread owns 8 channels of one output pixel (16-B loads / stores), keeps the running max and
// the window position of the winner (uint8, 8 per thread = one 8-B store).
// Backward as a GATHER: each thread owns 8 channels of one INPUT pixel and sums dy over the (at most
// ceil(k/s)^2) output windows covering it whose recorded winner is this pixel -- no atomics, no zero fill,
// every dx element written exactly once.
#include <stdexcept>

#include "common.h"
#include "launchers.h"

namespace k8s_amd {

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                          int Ho, int Wo, int k, int s, int p) {
  // 32-bit index decode (the host guarantees total < 2^31): 64-bit division is a long software sequence on
  // CDNA and dominated these bandwidth-bound kernels
  const int cv = C / 8;
  const int total = N * Ho * Wo * cv;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c = (e % cv) * 8;
    int t = e / cv;
    const int wo = t % Wo;
    t /= Wo;
    const int ho = t % Ho;
    const int n = t / Ho;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      arg[j] = 255;
    }
    for (int dh = 0; dh < k; ++dh) {
      const int h = ho * s - p + dh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int dw = 0; dw < k; ++dw) {
        const int w = wo * s - p + dw;
        if ((unsigned)w >= (unsigned)W) continue;
        float v[8];
        load8(x + (((long)n * H + h) * W + w) * C + c, v);
        const uint8_t pos = (uint8_t)(dh * k + dw);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best[j] || (v[j] != v[j] && best[j] == best[j])) {  // NaN propagates like torch
            best[j] = v[j];
            arg[j] = pos;
          }
      }
    }
    store8(y + (long)e * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) packed |= (uint64_t)arg[j] << (8 * j);
    *reinterpret_cast<uint64_t*>(idx + (long)e * 8) = packed;
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx, uint16_t* __restrict__ dx,
                                                          int N, int H, int W, int C, int Ho, int Wo, int k, int s,
                                                          int p) {
  const int cv = C / 8;
  const int total = N * H * W * cv;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    const int c = (e % cv) * 8;
    int t = e / cv;
    const int w = t % W;
    t /= W;
    const int h = t % H;
    const int n = t / H;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    // output windows covering (h, w): ho*s - p <= h <= ho*s - p + k - 1
    const int ho0 = max(0, (h + p - k + s) / s), ho1 = min(Ho - 1, (h + p) / s);
    const int wo0 = max(0, (w + p - k + s) / s), wo1 = min(Wo - 1, (w + p) / s);
    for (int ho = ho0; ho <= ho1; ++ho) {
      const int dh = h - (ho * s - p);
      for (int wo = wo0; wo <= wo1; ++wo) {
        const int dw = w - (wo * s - p);
        const uint8_t pos = (uint8_t)(dh * k + dw);
        const long o = (((long)n * Ho + ho) * Wo + wo) * C + c;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        bool any = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) any |= ((packed >> (8 * j)) & 0xff) == pos;
        if (!any) continue;
        float g[8];
        load8(dy + o, g);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((packed >> (8 * j)) & 0xff) == pos) acc[j] += g[j];
      }
    }
    store8(dx + (long)e * 8, acc);
  }
}

void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                        int k, int s, int p, hipStream_t st) {
  const long total = (long)N * Ho * Wo * (C / 8);
  if ((long)N * H * W * C / 8 >= (1L << 31)) throw std::runtime_error("maxpool: tensor too large for 32-bit indexing");
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, x, y, idx, N, H, W, C, Ho,
                     Wo, k, s, p);
}

void launch_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int Ho,
                        int Wo, int k, int s, int p, hipStream_t st) {
  const long total = (long)N * H * W * (C / 8);
  if (total >= (1L << 31)) throw std::runtime_error("maxpool: tensor too large for 32-bit indexing");
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, dy, idx, dx, N, H, W, C,
                     Ho, Wo, k, s, p);
}

}  // namespace k8s_amd
