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
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

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

// ---------------------------------------------------------------- the s2d stem convolution, LDS-tiled
// y[n][h][w][k] = sum_{i,j<4, c<16} xs[n][h+i][w+j][c] * w4[k][i][j][c]  (4x4 / stride 1 over the s2d image), with the
// BatchNorm statistics of the stored bf16 outputs. The generic implicit-GEMM kernel gathers every 16-B tap unit
// from L2 (256 taps x channels per output pixel, 16x re-read); here a block stages the (RT + 3)-row input window of
// RT whole output rows in LDS once (LDS-DMA) and builds the MFMA operands from it (forward 940 -> 741 us at
// ResNet-50 b1024 with register staging).
//   block: 4 waves, wave w = output row r0 + w, all Wo (<= 112, % 16 == 0) pixels as Wo / 16 pixel tiles
//   MFMA:  C^T[k][px] += W[k][32 taps*ch] . im2col^T  (v_mfma_f32_16x16x32_bf16, A = weight rows from LDS,
//          B = 16 B of one position's channel half per lane) -> a lane holds 4 consecutive output channels of one
//          pixel, staged through LDS and stored as whole 128-B pixel rows
//   LDS:   input window [RT + 3][Ws][16] bf16 (32 B per position; halves swapped when (pos >> 3) & 1: lanes 8
//          positions apart hit different banks), weights [64][256] with 16-B chunk c of row k at c ^ (k & 15);
//          the same bytes then stage the bf16 output rows (the statistics reduction has its own 2 KB after them).
//   (A persistent variant -- weights loaded once per block, the next tile's window prefetched behind the MFMAs,
//   outputs stored straight from the accumulators as 8-B pieces since the staging area is then taken -- measured
//   797 us.)
constexpr int STEM_RT = 4, STEM_K = 64, STEM_WMAX = 112;
constexpr int STEM_WIN = (STEM_RT + 3) * (STEM_WMAX + 3) * 32;  // 25,760 B
// window + weights, then the same bytes as the output staging (4 waves x Wo rows of 128 B)
constexpr int STEM_OST = STEM_WIN + STEM_K * 256 * 2 > 4 * STEM_WMAX * 128 ? STEM_WIN + STEM_K * 256 * 2
                                                                             : 4 * STEM_WMAX * 128;
constexpr int STEM_LDS = STEM_OST + 4 * 2 * STEM_K * 4;  // + the statistics reduction [wave][2][64]

__device__ __forceinline__ int stem_xoff(int pos, int half) { return pos * 32 + ((half ^ ((pos >> 3) & 1)) << 4); }

template <int NMT>  // pixel tiles per row = Wo / 16
__global__ void __launch_bounds__(256, 2) stem_conv_fwd_kernel(const uint16_t* __restrict__ xs,
                                                              const uint16_t* __restrict__ w4,
                                                              uint16_t* __restrict__ y, float* __restrict__ stats,
                                                              int Hs, int Ws, int Ho, int tiles_per_img) {
  __shared__ __attribute__((aligned(1024))) char smem[STEM_LDS];
  char* const xw = smem;
  char* const wl = smem + STEM_WIN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = blockIdx.x / tiles_per_img, r0 = (blockIdx.x % tiles_per_img) * STEM_RT;
  constexpr int Wo = NMT * 16;
  // ---- stage the input window (rows r0 .. r0 + RT + 2, contiguous in xs) and the weights by LDS-DMA: chunk c of
  // an image lands at byte 16 c, its source is the logical chunk the read-side swizzle maps there
  const int rows = min(STEM_RT + 3, Hs - r0);
  const int nch = rows * Ws * 2;  // 16-B chunks
  const uint16_t* src = xs + ((long)n * Hs + r0) * Ws * 16;
#pragma unroll 1
  for (int c = tid; c - tid < nch; c += 256) {
    if (c < nch) {
      const int pos = c >> 1, lh = (c & 1) ^ ((pos >> 3) & 1);
      glds16(src + (long)pos * 16 + lh * 8, xw + __builtin_amdgcn_readfirstlane(c - lane) * 16);
    }
  }
#pragma unroll 1
  for (int i = 0; i < STEM_K * 32 / 256; ++i) {
    const int c = i * 256 + tid, k = c >> 5, lc = (c & 31) ^ (k & 15);
    glds16(w4 + (long)k * 256 + lc * 8, wl + __builtin_amdgcn_readfirstlane(c - lane) * 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4_t acc[4][NMT];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int mi = 0; mi < NMT; ++mi) acc[ni][mi] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, g = lane >> 4;
#pragma unroll 2
  for (int kk = 0; kk < 8; ++kk) {  // 32-deep k steps: taps 2kk, 2kk + 1 (i = kk >> 1, j = 2 (kk & 1) + {0, 1})
    mfma_bf16x8 af[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int k = ni * 16 + li, ch = kk * 4 + g;
      af[ni] = __builtin_bit_cast(mfma_bf16x8,
                                  *reinterpret_cast<const bf16x8_t*>(wl + k * 512 + ((ch ^ (k & 15)) << 4)));
    }
    const int tap = 2 * kk + (g >> 1), ti = tap >> 2, tj = tap & 3, half = g & 1;
    const int prow = (wid + ti) * Ws;
#pragma unroll
    for (int mi = 0; mi < NMT; ++mi) {
      const int pos = prow + mi * 16 + li + tj;
      const mfma_bf16x8 bf = __builtin_bit_cast(mfma_bf16x8,
                                                *reinterpret_cast<const bf16x8_t*>(xw + stem_xoff(pos, half)));
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[ni][mi] = mfma16(af[ni], bf, acc[ni][mi]);
    }
  }
  // ---- epilogue: bf16 outputs through LDS (wave-private [Wo][64] rows, 16-B chunk c of pixel p at c ^ (p & 7)),
  // statistics of the stored values (lane: channels 16 ni + 4 g .. +3 of pixel 16 mi + li)
  const int orow = r0 + wid;
  const bool live = orow < Ho;
  float ssum[4][4], ssq[4][4];
  __syncthreads();  // every wave is done with the window / weights
  char* const ost = smem + wid * (Wo * 128);
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
#pragma unroll
    for (int r = 0; r < 4; ++r) ssum[ni][r] = ssq[ni][r] = 0.f;
#pragma unroll
    for (int mi = 0; mi < NMT; ++mi) {
      const int px = mi * 16 + li;
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint16_t bv = f2bf(acc[ni][mi][r]);
        o[r] = (short)bv;
        const float v = bf2f(bv);
        ssum[ni][r] += v;
        ssq[ni][r] += v * v;
      }
      const int ch = 2 * ni + (g >> 1);
      *reinterpret_cast<bf16x4_t*>(ost + px * 128 + ((ch ^ (px & 7)) << 4) + (g & 1) * 8) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staging writes landed (wave-private region)
  if (live) {
    uint16_t* dst = y + (((long)n * Ho + orow) * Wo) * STEM_K;
#pragma unroll
    for (int it = 0; it < Wo * 8 / 64; ++it) {
      const int q = it * 64 + lane, px = q >> 3, c = q & 7;
      *reinterpret_cast<bf16x8_t*>(dst + (long)q * 8) =
          *reinterpret_cast<const bf16x8_t*>(ost + px * 128 + ((c ^ (px & 7)) << 4));
    }
  }
  // statistics: 16 pixel lanes -> DPP row sums, then the 4 waves through LDS, one atomic per (channel, moment)
  float* red = reinterpret_cast<float*>(smem + STEM_OST);  // [wave][2][64]
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = row16_sum(live ? ssum[ni][r] : 0.f), b = row16_sum(live ? ssq[ni][r] : 0.f);
      if (li == 0) {
        const int ch = ni * 16 + g * 4 + r;
        red[(wid * 2 + 0) * 64 + ch] = a;
        red[(wid * 2 + 1) * 64 + ch] = b;
      }
    }
  __syncthreads();
  if (tid < 128) {
    const int ch = tid & 63, which = tid >> 6;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) v += red[(w * 2 + which) * 64 + ch];
    atomicAdd(stats + (long)(blockIdx.x % kConvStatReplicas) * 2 * STEM_K + which * STEM_K + ch, v);
  }
}

// Wo <= 112: the 8-tile (Wo = 128) forward instantiation would spill (acc 4 x 8 f32x4 + the window prefetch)
bool stem_conv_fwd_ok(int K, int R, int C, int Wo) { return K == STEM_K && R == 4 && C == 16 && Wo % 16 == 0 && Wo <= 112; }

void launch_stem_conv_fwd(const uint16_t* xs, const uint16_t* w4, uint16_t* y, float* stats, int N, int Hs, int Ws,
                          hipStream_t st) {
  const int Ho = Hs - 3, Wo = Ws - 3;
  if (Wo % 16 || Wo > 112 || Wo < 16) throw std::runtime_error("stem conv: Wo must be a multiple of 16, <= 112");
  const int tpi = (Ho + STEM_RT - 1) / STEM_RT;
  if ((long)N * tpi >= (1L << 31)) throw std::runtime_error("stem conv: too many tiles");
  const dim3 grid((unsigned)(N * tpi)), blk(256);
  switch (Wo / 16) {
#define K8S_STEM_CASE(T) \
  case T: hipLaunchKernelGGL(stem_conv_fwd_kernel<T>, grid, blk, 0, st, xs, w4, y, stats, Hs, Ws, Ho, tpi); break;
    K8S_STEM_CASE(1) K8S_STEM_CASE(2) K8S_STEM_CASE(3) K8S_STEM_CASE(4)
    K8S_STEM_CASE(5) K8S_STEM_CASE(6) K8S_STEM_CASE(7)
#undef K8S_STEM_CASE
  }
}

// ---------------------------------------------------------------- the s2d stem weight gradient, LDS-tiled
// dw4[k][i][j][c] = sum_{n,h,w} dy[n][h][w][k] * xs[n][h+i][w+j][c]: a 64 x 256 product reduced over all N*Ho*Wo
// output pixels. Persistent blocks (3 per CU) sweep tiles of RT = 2 output rows; per tile the input window
// [RT + 3][Ws][16] and the dy rows [RT * Wo][64] are staged in LDS by LDS-DMA (register staging with the next
// tile prefetched behind the MFMAs measured 668 us at b1024), both operands are read transposed (ds_read_b64_tr_b16: 4 pixels x 16 channels per 16 lanes), and
// the block's fp32 partial stays in 64 accumulator registers per lane until its last tile; the partials are
// summed by splitk_reduce. (The generic split-K implicit GEMM gathers every 16-B tap unit from L2 and fills only
// half of its 128-row tiles with the 64 output channels.)
//   wave w: output columns q = 64 w .. 64 w + 63 (taps 4w .. 4w + 3 x 16 channels), all 64 k
constexpr int SWG_RT = 2;
constexpr int SWG_WIN = (SWG_RT + 3) * (STEM_WMAX + 3) * 32;   // 20,960 B
constexpr int SWG_DY = SWG_RT * STEM_WMAX * 128;               // 32 KB
__device__ __attribute__((aligned(64))) uint16_t g_stem_zero[64];  // source of dy rows past the image

__device__ __forceinline__ int swg_dyoff(int px, int ch16) { return px * 128 + ((ch16 ^ (px & 7)) << 4); }

template <int NMT>  // Wo / 16
__global__ void __launch_bounds__(256, 3) stem_wgrad_kernel(const uint16_t* __restrict__ xs,
                                                           const uint16_t* __restrict__ dy, float* __restrict__ ws,
                                                           int Hs, int Ws, int Ho, int tiles_per_img, int ntiles) {
  __shared__ __attribute__((aligned(1024))) char smem[SWG_WIN + SWG_DY];
  char* const xw = smem;
  char* const dl = smem + SWG_WIN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, G = lane >> 4, q4 = li >> 2, p4 = li & 3;
  constexpr int Wo = NMT * 16, PX = SWG_RT * Wo, NKS = PX / 32;
  // stage tile t by LDS-DMA (chunk c of an image at byte 16 c, sourced from the logical chunk the read swizzle maps
  // there; dy rows past Ho from the zero page); the CU's other blocks compute while one stages
  auto stage = [&](int t) {
    const int n = t / tiles_per_img, r0 = (t % tiles_per_img) * SWG_RT;
    // the whole window, rows past the image from the zero page: a partial last tile multiplies its zero dy rows by
    // these window rows, and stale LDS there (a NaN bit pattern from an earlier kernel) would make 0 * NaN = NaN
    const int nch = (SWG_RT + 3) * Ws * 2, nvalid = min(SWG_RT + 3, Hs - r0) * Ws * 2;
    const int npx = min(SWG_RT, Ho - r0) * Wo;
    const uint16_t* sx = xs + ((long)n * Hs + r0) * Ws * 16;
    const uint16_t* sd = dy + (((long)n * Ho + r0) * Wo) * STEM_K;
#pragma unroll 1
    for (int c = tid; c - tid < nch; c += 256) {
      if (c < nch) {
        const int pos = c >> 1, lh = (c & 1) ^ ((pos >> 3) & 1);
        glds16(c < nvalid ? (const void*)(sx + (long)pos * 16 + lh * 8) : (const void*)g_stem_zero,
               xw + __builtin_amdgcn_readfirstlane(c - lane) * 16);
      }
    }
#pragma unroll 1
    for (int c = tid; c - tid < PX * 8; c += 256) {
      if (c < PX * 8) {
        const int px = c >> 3, lc = (c & 7) ^ (px & 7);
        glds16(px < npx ? (const void*)(sd + (long)px * STEM_K + lc * 8) : (const void*)g_stem_zero,
               dl + __builtin_amdgcn_readfirstlane(c - lane) * 16);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  f32x4_t acc[4][4];  // [k tile][q tile]: lane holds out[16 kt + 4 G + r][64 wid + 16 qt + li]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    stage(t);
    __syncthreads();
#pragma unroll 1
    for (int ks = 0; ks < NKS; ++ks) {
      // k-step: pixels 32 ks + 8 G + (0..7) of the tile (row-major over RT x Wo; 8-pixel runs never straddle a row)
      const int pb = 32 * ks + 8 * G;
      mfma_bf16x8 af[4];  // dy^T: row = channel 16 kt + li, k = 8 pixels
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const int ch16 = 2 * kt + (p4 >> 1);
        const short4_t lo = tr16(dl + swg_dyoff(pb + q4, ch16) + (p4 & 1) * 8);
        const short4_t hi = tr16(dl + swg_dyoff(pb + 4 + q4, ch16) + (p4 & 1) * 8);
        af[kt] = join8(lo, hi);
      }
#pragma unroll
      for (int qt = 0; qt < 4; ++qt) {
        const int tap = 4 * wid + qt, ti = tap >> 2, tj = tap & 3;
        // X: rows = pixels (their input position shifted by the tap), column = channel 4 p4 .. of the tap
        const int p0 = pb + q4, p1 = pb + 4 + q4;
        const int pos0 = ((p0 / Wo) + ti) * Ws + (p0 % Wo) + tj;
        const int pos1 = ((p1 / Wo) + ti) * Ws + (p1 % Wo) + tj;
        const short4_t lo = tr16(xw + stem_xoff(pos0, p4 >> 1) + (p4 & 1) * 8);
        const short4_t hi = tr16(xw + stem_xoff(pos1, p4 >> 1) + (p4 & 1) * 8);
        const mfma_bf16x8 bf = join8(lo, hi);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt][qt] = mfma16(af[kt], bf, acc[kt][qt]);
      }
    }
    __syncthreads();  // every wave is done with this tile's LDS before the next stage
  }
  float* out = ws + (long)blockIdx.x * (STEM_K * 256);
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(kt * 16 + G * 4 + r) * 256 + wid * 64 + qt * 16 + li] = acc[kt][qt][r];
}

int stem_wgrad_blocks(int N, int Hs) {
  const long ntiles = (long)N * ((Hs - 3 + SWG_RT - 1) / SWG_RT);
  return (int)std::min<long>(ntiles, 3L * planner_cus());  // persistent: 3 blocks per CU (47 KB LDS, ~130 VGPRs)
}

void launch_stem_wgrad(const uint16_t* xs, const uint16_t* dy, float* ws, float* dw4, int N, int Hs, int Ws,
                       hipStream_t st) {
  const int Ho = Hs - 3, Wo = Ws - 3;
  if (Wo % 16 || Wo > 112 || Wo < 16) throw std::runtime_error("stem wgrad: Wo must be a multiple of 16, <= 112");
  const int tpi = (Ho + SWG_RT - 1) / SWG_RT;
  const long ntiles = (long)N * tpi;
  if (ntiles >= (1L << 31)) throw std::runtime_error("stem wgrad: too many tiles");
  const int nb = stem_wgrad_blocks(N, Hs);
  switch (Wo / 16) {
#define K8S_SWG_CASE(T)                                                                                            \
  case T:                                                                                                          \
    hipLaunchKernelGGL(stem_wgrad_kernel<T>, dim3(nb), dim3(256), 0, st, xs, dy, ws, Hs, Ws, Ho, tpi, (int)ntiles); \
    break;
    K8S_SWG_CASE(1) K8S_SWG_CASE(2) K8S_SWG_CASE(3) K8S_SWG_CASE(4)
    K8S_SWG_CASE(5) K8S_SWG_CASE(6) K8S_SWG_CASE(7)
#undef K8S_SWG_CASE
  }
  splitk_reduce(ws, nb, (long)STEM_K * 256, dw4, false, st);
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
