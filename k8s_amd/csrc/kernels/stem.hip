// ResNet stem as a space-to-depth convolution.
//
// The 7x7 / stride-2 / pad-3 stem over a 3-channel image is the same linear map as a 4x4 / stride-1 / pad-0
// convolution over the image's 2x2 space-to-depth transform (16 channels: 2x2 pixels x 4 channels, the 4th and
// the 8th tap row / column zero): 256 MACs per output channel instead of 392 on the 8-channel-padded 7x7 form,
// and 16-B units that cover two full taps. Measured at batch 1024 (scripts/stem_ab.py): forward 1.87 -> 1.22 ms,
// weight gradient 2.59 -> 1.36 ms. The master weight keeps the 7x7 layout [K][7][7][Cw] (checkpoints and the
// reference twin are unchanged): each step maps it to the 4x4 form, and the 4x4 weight gradient back.
//
//   x_s2d[n][i][j][(dy*2 + dx)*4 + c] = x[n][2i + dy - pad][2j + dx - pad][c]      (0 outside / for c >= Cin)
//   w4[k][i][j][(dy*2 + dx)*4 + c]    = w7[k][2i + dy][2j + dx][c]                 (0 for taps >= R, c >= 4)
//   dw7[k][r][s][c]                   = dw4[k][r/2][s/2][((r%2)*2 + s%2)*4 + c]    (0 for c >= 4)
#include <stdexcept>

#include "common.h"
#include "launchers.h"

namespace k8s_amd {

__global__ void __launch_bounds__(256) stem_s2d_input_kernel(const uint16_t* __restrict__ x, int Cin, int H, int W,
                                                             int pad, int Hs, int Ws, uint16_t* __restrict__ out,
                                                             int total) {
  const int e = blockIdx.x * 256 + threadIdx.x;  // output pixel (n, i, j)
  if (e >= total) return;
  const int j = e % Ws, t = e / Ws;
  const int i = t % Hs, n = t / Hs;
  bf16x8_t o[2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int dy = q >> 1, dx = q & 1;
    const int h = 2 * i + dy - pad, w = 2 * j + dx - pad;
    const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    const uint16_t* p = x + (((long)n * H + (in ? h : 0)) * W + (in ? w : 0)) * Cin;
#pragma unroll
    for (int c = 0; c < 4; ++c) o[q >> 1][(q & 1) * 4 + c] = (short)((in && c < Cin) ? p[c] : 0);
  }
  bf16x8_t* dst = reinterpret_cast<bf16x8_t*>(out + (long)e * 16);
  dst[0] = o[0];
  dst[1] = o[1];
}

__global__ void stem_w_s2d_kernel(const uint16_t* __restrict__ w7, int K, int R, int Cw, int Rs,
                                  uint16_t* __restrict__ w4) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // [K][Rs][Rs][16]
  if (e >= K * Rs * Rs * 16) return;
  const int ch = e & 15, t = e >> 4;
  const int j = t % Rs, t2 = t / Rs;
  const int i = t2 % Rs, k = t2 / Rs;
  const int q = ch >> 2, c = ch & 3, dy = q >> 1, dx = q & 1;
  const int r = 2 * i + dy, s = 2 * j + dx;
  w4[e] = (r < R && s < R && c < Cw) ? w7[(((long)k * R + r) * R + s) * Cw + c] : (uint16_t)0;
}

__global__ void stem_dw_s2d_kernel(const float* __restrict__ dw4, int K, int R, int Cw, int Rs,
                                   float* __restrict__ dw7) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // [K][R][R][Cw]
  if (e >= K * R * R * Cw) return;
  const int c = e % Cw, t = e / Cw;
  const int s = t % R, t2 = t / R;
  const int r = t2 % R, k = t2 / R;
  dw7[e] = c < 4 ? dw4[(((long)k * Rs + r / 2) * Rs + s / 2) * 16 + ((r & 1) * 2 + (s & 1)) * 4 + c] : 0.f;
}

void launch_stem_s2d_input(const uint16_t* x, int N, int H, int W, int Cin, int pad, uint16_t* out,
                           hipStream_t st) {
  if (Cin > 8 || (H + 2 * pad) % 2 || (W + 2 * pad) % 2) throw std::runtime_error("stem s2d: Cin <= 8, even padded size");
  const int Hs = (H + 2 * pad) / 2, Ws = (W + 2 * pad) / 2;
  const long total = (long)N * Hs * Ws;
  if (total >= (1L << 31)) throw std::runtime_error("stem s2d: too many pixels");
  hipLaunchKernelGGL(stem_s2d_input_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, x, Cin, H, W, pad, Hs, Ws, out,
                     (int)total);
}

void launch_stem_w_s2d(const uint16_t* w7, int K, int R, int Cw, uint16_t* w4, hipStream_t st) {
  const int Rs = (R + 1) / 2;
  hipLaunchKernelGGL(stem_w_s2d_kernel, dim3(cdiv((long)K * Rs * Rs * 16, 256)), dim3(256), 0, st, w7, K, R, Cw, Rs,
                     w4);
}

void launch_stem_dw_s2d(const float* dw4, int K, int R, int Cw, float* dw7, hipStream_t st) {
  const int Rs = (R + 1) / 2;
  hipLaunchKernelGGL(stem_dw_s2d_kernel, dim3(cdiv((long)K * R * R * Cw, 256)), dim3(256), 0, st, dw4, K, R, Cw, Rs,
                     dw7);
}

}  // namespace k8s_amd
