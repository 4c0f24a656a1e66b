// NHWC max pooling (the ResNet stem's 3x3 / stride 2 / pad 1) forward + backward.
//
// Forward: each thread owns 8 channels of one output pixel (16-B loads / stores), keeps the running max and
// the window position of the winner (uint8, 8 per thread = one 8-B store).
// Backward as a GATHER: each thread owns 8 channels of one INPUT pixel and sums dy over the (at most
// ceil(k/s)^2) output windows covering it whose recorded winner is this pixel -- no atomics, no zero fill,
// every dx element written exactly once.
// Both are flat launches (one 16-B vector per thread, no grid-stride loop: see batchnorm.hip's header for the
// measured streaming advantage) with the index decode as multiply-high FastDivs.
#include <stdexcept>

#include "common.h"
#include "launchers.h"

namespace k8s_amd {

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int H, int W, int C, int Ho,
                                                          int Wo, int k, int s, int p, int total, FastDiv fcv,
                                                          FastDiv fWo, FastDiv fHo) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  int t = fcv.div(e);
  const int c = (e - t * cv) * 8;
  int t2 = fWo.div(t);
  const int wo = t - t2 * Wo;
  const int n = fHo.div(t2);
  const int ho = t2 - n * Ho;
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

// k x k window known at compile time (the stem's 3 x 3): all k*k input vectors are loaded up front (clamped
// in-bounds addresses, out-of-image taps masked afterwards) so the loads are in flight together instead of one
// load -> compare round trip per tap; taps are compared in the same (dh, dw) order, so ties pick the same winner
template <int K>
__global__ void __launch_bounds__(256) maxpool_fwd_k_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                            uint8_t* __restrict__ idx, int H, int W, int C, int Ho,
                                                            int Wo, int s, int p, int total, FastDiv fcv, FastDiv fWo,
                                                            FastDiv fHo) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  int t = fcv.div(e);
  const int c = (e - t * cv) * 8;
  int t2 = fWo.div(t);
  const int wo = t - t2 * Wo;
  const int n = fHo.div(t2);
  const int ho = t2 - n * Ho;
  const int h0 = ho * s - p, w0 = wo * s - p;
  float v[K * K][8];
#pragma unroll
  for (int dh = 0; dh < K; ++dh)
#pragma unroll
    for (int dw = 0; dw < K; ++dw) {
      const int h = min(max(h0 + dh, 0), H - 1), w = min(max(w0 + dw, 0), W - 1);
      load8(x + (((long)n * H + h) * W + w) * C + c, v[dh * K + dw]);
    }
  float best[8];
  uint8_t arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    best[j] = -INFINITY;
    arg[j] = 255;
  }
#pragma unroll
  for (int dh = 0; dh < K; ++dh)
#pragma unroll
    for (int dw = 0; dw < K; ++dw) {
      if ((unsigned)(h0 + dh) >= (unsigned)H || (unsigned)(w0 + dw) >= (unsigned)W) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float u = v[dh * K + dw][j];
        if (u > best[j] || (u != u && best[j] == best[j])) {  // NaN propagates like torch
          best[j] = u;
          arg[j] = (uint8_t)(dh * K + dw);
        }
      }
    }
  store8(y + (long)e * 8, best);
  uint64_t packed = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) packed |= (uint64_t)arg[j] << (8 * j);
  *reinterpret_cast<uint64_t*>(idx + (long)e * 8) = packed;
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const uint16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx, uint16_t* __restrict__ dx,
                                                          int H, int W, int C, int Ho, int Wo, int k, int s, int p,
                                                          int total, FastDiv fcv, FastDiv fW, FastDiv fH) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  int t = fcv.div(e);
  const int c = (e - t * cv) * 8;
  int t2 = fW.div(t);
  const int w = t - t2 * W;
  const int n = fH.div(t2);
  const int h = t2 - n * H;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  // output windows covering (h, w): ho*s - p <= h <= ho*s - p + k - 1
  const int ho0 = max(0, (h + p - k + s) / s), ho1 = min(Ho - 1, (h + p) / s);
  const int wo0 = max(0, (w + p - k + s) / s), wo1 = min(Wo - 1, (w + p) / s);
  if (k <= 2 * s) {
    // at most 2 x 2 covering windows (the ResNet stem's 3x3 / s2): every window's winner bytes and dy vector are
    // loaded up front (8 independent loads in flight) instead of a dependent idx -> dy round trip per window
    uint64_t pk[4];
    float g[4][8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ho = ho0 + (q >> 1), wo = wo0 + (q & 1);
      const bool ok = ho <= ho1 && wo <= wo1;
      const long o = (((long)n * Ho + (ok ? ho : ho0)) * Wo + (ok ? wo : wo0)) * C + c;
      pk[q] = *reinterpret_cast<const uint64_t*>(idx + o);  // (clamped in-bounds address when !ok: not used)
      load8(dy + o, g[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int ho = ho0 + (q >> 1), wo = wo0 + (q & 1);
      if (ho > ho1 || wo > wo1) continue;
      const uint8_t pos = (uint8_t)((h - (ho * s - p)) * k + (w - (wo * s - p)));
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((pk[q] >> (8 * j)) & 0xff) == pos) acc[j] += g[q][j];
    }
    store8(dx + (long)e * 8, acc);
    return;
  }
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

// 3x3 / stride 2 / pad 1 (the ResNet stem) backward by 2x2 input-pixel cells: the cell (2k..2k+1, 2j..2j+1) is
// covered by exactly the windows (k..k+1, j..j+1), so one thread loads those 4 windows' winner bytes and dy
// vectors ONCE for its 4 pixels (24 B of L2 reads per 16-B output instead of 4 x 24 B when every pixel thread
// loads its own covering windows) and writes the 4 pixels. Window position of pixel (h, w) in window (ho, wo):
// (h - 2ho + 1) * 3 + (w - 2wo + 1).
__global__ void __launch_bounds__(256) maxpool_bwd_3s2_kernel(const uint16_t* __restrict__ dy,
                                                              const uint8_t* __restrict__ idx,
                                                              uint16_t* __restrict__ dx, int H, int W, int C, int Ho,
                                                              int Wo, int Hc, int Wc, int total, FastDiv fcv,
                                                              FastDiv fWc, FastDiv fHc) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  int t = fcv.div(e);
  const int c = (e - t * cv) * 8;
  int t2 = fWc.div(t);
  const int j = t - t2 * Wc;
  const int n = fHc.div(t2);
  const int k = t2 - n * Hc;
  uint64_t pk[2][2];
  float g[2][2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const bool ok = k + a < Ho && j + b < Wo;
      const long o = (((long)n * Ho + (ok ? k + a : k)) * Wo + (ok ? j + b : j)) * C + c;
      pk[a][b] = ok ? *reinterpret_cast<const uint64_t*>(idx + o) : ~0ull;  // 0xff: matches no position
      load8(dy + o, g[a][b]);
    }
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int h = 2 * k + dh, w = 2 * j + dw;
      if (h >= H || w >= W) continue;
      float acc[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] = 0.f;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          // pixel (h, w) lies in window (k + a, j + b) iff its offset inside the window is in 0..2
          const int oh = h - 2 * (k + a) + 1, ow = w - 2 * (j + b) + 1;
          if (oh < 0 || oh > 2 || ow < 0 || ow > 2) continue;  // compile-time after unrolling
          const uint8_t pos = (uint8_t)(oh * 3 + ow);
#pragma unroll
          for (int r = 0; r < 8; ++r)
            if (((pk[a][b] >> (8 * r)) & 0xff) == pos) acc[r] += g[a][b][r];
        }
      store8(dx + (((long)n * H + h) * W + w) * C + c, acc);
    }
}

void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                        int k, int s, int p, hipStream_t st) {
  const long total = (long)N * Ho * Wo * (C / 8);
  if ((long)N * H * W * C / 8 >= (1L << 31)) throw std::runtime_error("maxpool: tensor too large for 32-bit indexing");
  if (k == 3) {
    hipLaunchKernelGGL(maxpool_fwd_k_kernel<3>, dim3(cdiv(total, 256)), dim3(256), 0, st, x, y, idx, H, W, C, Ho, Wo,
                       s, p, (int)total, make_fastdiv(C / 8), make_fastdiv(Wo), make_fastdiv(Ho));
    return;
  }
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, x, y, idx, H, W, C, Ho, Wo, k, s,
                     p, (int)total, make_fastdiv(C / 8), make_fastdiv(Wo), make_fastdiv(Ho));
}

void launch_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int Ho,
                        int Wo, int k, int s, int p, hipStream_t st) {
  const long total = (long)N * H * W * (C / 8);
  if (total >= (1L << 31)) throw std::runtime_error("maxpool: tensor too large for 32-bit indexing");
  if (k == 3 && s == 2 && p == 1) {
    const int Hc = (H + 1) / 2, Wc = (W + 1) / 2;
    const long cells = (long)N * Hc * Wc * (C / 8);
    hipLaunchKernelGGL(maxpool_bwd_3s2_kernel, dim3(cdiv(cells, 256)), dim3(256), 0, st, dy, idx, dx, H, W, C, Ho,
                       Wo, Hc, Wc, (int)cells, make_fastdiv(C / 8), make_fastdiv(Wc), make_fastdiv(Hc));
    return;
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, dy, idx, dx, H, W, C, Ho, Wo, k, s,
                     p, (int)total, make_fastdiv(C / 8), make_fastdiv(W), make_fastdiv(H));
}

// Global average pool (the ResNet head): thread = (image, 8 channels) summing HW rows in fp32; backward writes
// dy / HW to every pixel, one 16-B vector per thread.
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          int N, int HW, int C, float inv) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int cv = C >> 3;
  if (e >= N * cv) return;
  const int n = e / cv, c = (e - n * cv) * 8;
  const uint16_t* p = x + (long)n * HW * C + c;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int i = 0;
  for (; i + 3 < HW; i += 4) {  // 4 rows in flight
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8(p + (long)(i + u) * C, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[u][j];
  }
  for (; i < HW; ++i) {
    float v[8];
    load8(p + (long)i * C, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= inv;
  store8(y + (long)n * C + c, acc);
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const uint16_t* __restrict__ dy, uint16_t* __restrict__ dx,
                                                          int total, int HW, int C, FastDiv fcv, FastDiv fhw,
                                                          float inv) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  const int pix = fcv.div(e), c = (e - pix * cv) * 8;
  const int n = fhw.div(pix);
  float v[8];
  load8(dy + (long)n * C + c, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= inv;
  store8(dx + (long)e * 8, v);
}

void launch_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t st) {
  if (C % 8 != 0) throw std::runtime_error("avgpool: C must be a multiple of 8");
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(cdiv((long)N * (C / 8), 256)), dim3(256), 0, st, x, y, N, HW, C,
                     1.f / (float)HW);
}

void launch_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st) {
  const long total = (long)N * HW * (C / 8);
  if (C % 8 != 0 || total >= (1L << 31)) throw std::runtime_error("avgpool: C % 8 != 0 or tensor too large");
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, dy, dx, (int)total, HW, C,
                     make_fastdiv(C / 8), make_fastdiv(HW), 1.f / (float)HW);
}

// Stride-s subsample of an NHWC tensor, y[n][i][j][:] = x[n][s i][s j][:] (the input of a 1x1 / stride-s / pad-0
// convolution, which then runs as a plain stride-1 GEMM on y: ResNet's downsample convolutions). One 16-B chunk per
// thread, grid-strided; the source rows are read as whole 16-B pieces.
__global__ void __launch_bounds__(256) subsample_nhwc_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                             long total, int Ho, int Wo, int H, int W, int C8,
                                                             int s) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long pix = e / C8;
    const int c = (int)(e - pix * C8);
    const long n = pix / ((long)Ho * Wo);
    const int r = (int)(pix - n * Ho * Wo), i = r / Wo, j = r - i * Wo;
    const long src = ((n * H + (long)i * s) * W + (long)j * s) * C8 + c;
    reinterpret_cast<bf16x8_t*>(y)[e] = reinterpret_cast<const bf16x8_t*>(x)[src];
  }
}

void launch_subsample_nhwc(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int s, hipStream_t st) {
  const int Ho = (H + s - 1) / s, Wo = (W + s - 1) / s;
  const long total = (long)N * Ho * Wo * (C / 8);
  hipLaunchKernelGGL(subsample_nhwc_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, x, y, total, Ho, Wo, H,
                     W, C / 8, s);
}

}  // namespace k8s_amd
