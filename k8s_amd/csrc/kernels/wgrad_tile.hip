// LDS-tiled weight gradient of the ResNet-50 stage-1 3x3 convolution (C = K = 64, 56 x 56, stride 1, pad 1).
//
//   dw[k][r][s][c] = sum_{n,h,w} dy[n][h][w][k] * x[n][h + r - 1][w + s - 1][c]        (a 64 x 576 product,
//                                                                                     reduced over N*H*W pixels)
// The generic split-K implicit GEMM (gemm.hip ConvWgB) ran this shape at ~270 TF/s: its 128-row tiles are half
// empty with 64 output channels, and every 16-B tap unit of im2col(x) is gathered from L2 nine times. Here
// persistent blocks (2 per CU) sweep tiles of RT = 4 output rows: the (RT + 2)-row zero-padded input window and
// the RT dy rows are staged in LDS once per tile and both MFMA operands are read from them transposed
// (ds_read_b64_tr_b16: 4 pixels x 16 channels per 16 lanes), staged by LDS-DMA; each block keeps its fp32 partial of the whole
// 64 x 576 gradient in accumulator registers (wave w: output columns 144 w .. 144 w + 143) until its last tile,
// and splitk_reduce sums the blocks' partials into dw.
//   LDS images: [position][64 ch] bf16, 128-B rows, 16-B chunk c of row p at c ^ (p & 7) (window and dy alike).
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {

namespace wg3 {
constexpr int RT = 4, C = 64, NQ = 9 * C;  // 576 output columns (tap, channel)
__device__ __attribute__((aligned(64))) uint16_t g_wg3_zero[64];  // source of the zero padding

__device__ __forceinline__ int off(int p, int ch16) { return p * 128 + ((ch16 ^ (p & 7)) << 4); }

template <int W>
__global__ void __launch_bounds__(256, 2) wgrad3x3_c64_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ dy, float* __restrict__ ws,
                                                             int H, int tiles_per_img, int ntiles) {
  constexpr int WP = W + 2, WIN = (RT + 2) * WP, PX = RT * W, NKS = PX / 32;
  static_assert(W % 8 == 0 && PX % 32 == 0, "8-pixel runs inside one row, whole 32-pixel k steps");
  __shared__ __attribute__((aligned(1024))) char smem[(WIN + PX) * 128];
  char* const xw = smem;
  char* const dl = smem + WIN * 128;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, G = lane >> 4, q4 = li >> 2, p4 = li & 3;

  f32x4_t acc[4][9];  // [k tile][q tile 9 wid + j]: lane holds dw[16 kt + 4 G + r][16 (9 wid + j) + li]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / tiles_per_img, h0 = (t % tiles_per_img) * RT;
    // ---- stage by LDS-DMA (global_load_lds, 16 B per lane, no VGPR round trip): window rows h0 - 1 .. h0 + RT,
    // columns -1 .. W (the zero page outside the image), then the RT dy rows. Chunk c of an image lands at LDS byte
    // 16 c (lane-linear per wave instruction); its source is logical chunk (c & 7) ^ (position & 7) of the position
    // (the read-side swizzle of off()).
    {
      constexpr int NW = (WIN * 8 + 255) / 256, ND = (PX * 8 + 255) / 256;
#pragma unroll 1
      for (int i = 0; i < NW; ++i) {
        const int c = i * 256 + tid;
        if (c < WIN * 8) {  // lanes past the image stay inactive (they would write into the dy image)
          const int p = c >> 3, lc = (c & 7) ^ (p & 7);
          const int wr = p / WP, wc = p - wr * WP, h = h0 - 1 + wr, w = wc - 1;
          const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
          const void* src = in ? (const void*)(x + (((long)n * H + h) * W + w) * C + lc * 8) : (const void*)g_wg3_zero;
          glds16(src, xw + __builtin_amdgcn_readfirstlane(i * 256 + wid * 64) * 16);
        }
      }
#pragma unroll 1
      for (int i = 0; i < ND; ++i) {
        const int c = i * 256 + tid;
        if (c < PX * 8) {
          const int p = c >> 3, lc = (c & 7) ^ (p & 7);
          const bool in = h0 + p / W < H;
          const void* src = in ? (const void*)(dy + (((long)n * H + h0) * W + p) * C + lc * 8) : (const void*)g_wg3_zero;
          glds16(src, dl + __builtin_amdgcn_readfirstlane(i * 256 + wid * 64) * 16);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
#pragma unroll 1
    for (int ks = 0; ks < NKS; ++ks) {
      const int pb = 32 * ks + 8 * G;  // this lane group's 8 pixels of the k step (one row: W % 8 == 0)
      mfma_bf16x8 af[4];               // dy^T: row = output channel 16 kt + li, k = 8 pixels
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const int ch16 = 2 * kt + (p4 >> 1);
        const short4_t lo = tr16(dl + off(pb + q4, ch16) + (p4 & 1) * 8);
        const short4_t hi = tr16(dl + off(pb + 4 + q4, ch16) + (p4 & 1) * 8);
        af[kt] = join8(lo, hi);
      }
      const int r0 = pb / W, c0 = pb - r0 * W;  // output row / column of the group's first pixel
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int qt = 9 * wid + j, tap = qt >> 2, cq = qt & 3, tr = tap / 3, ts = tap - tr * 3;
        // X: rows = the 8 pixels' window positions shifted by the tap, column = channel 16 cq + 4 p4 ..
        const int pos = (r0 + tr) * WP + c0 + ts + q4;
        const int ch16 = 2 * cq + (p4 >> 1);
        const short4_t lo = tr16(xw + off(pos, ch16) + (p4 & 1) * 8);
        const short4_t hi = tr16(xw + off(pos + 4, ch16) + (p4 & 1) * 8);
        const mfma_bf16x8 bf = join8(lo, hi);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt][j] = mfma16(af[kt], bf, acc[kt][j]);
      }
    }
    __syncthreads();  // every wave is done with this tile's LDS before the next stage
  }
  float* out = ws + (long)blockIdx.x * (C * NQ);
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(kt * 16 + G * 4 + r) * NQ + (9 * wid + j) * 16 + li] = acc[kt][j][r];
}
}  // namespace wg3

bool wgrad3x3_c64_ok(int C, int K, int R, int S, int stride, int pad, int W) {
  return C == 64 && K == 64 && R == 3 && S == 3 && stride == 1 && pad == 1 && (W == 56 || W == 16);
}

int wgrad3x3_c64_blocks(int N, int H) { return (int)std::min<long>((long)N * ((H + wg3::RT - 1) / wg3::RT), 512); }

void launch_wgrad3x3_c64(const uint16_t* x, const uint16_t* dy, float* ws, float* dw, int N, int H, int W,
                         bool accumulate, hipStream_t st) {
  const int tpi = (H + wg3::RT - 1) / wg3::RT;
  const long ntiles = (long)N * tpi;
  if (ntiles >= (1L << 31)) throw std::runtime_error("wgrad3x3_c64: too many tiles");
  const int nb = wgrad3x3_c64_blocks(N, H);
  if (W == 56)
    hipLaunchKernelGGL(wg3::wgrad3x3_c64_kernel<56>, dim3(nb), dim3(256), 0, st, x, dy, ws, H, tpi, (int)ntiles);
  else if (W == 16)
    hipLaunchKernelGGL(wg3::wgrad3x3_c64_kernel<16>, dim3(nb), dim3(256), 0, st, x, dy, ws, H, tpi, (int)ntiles);
  else
    throw std::runtime_error("wgrad3x3_c64: W must be 56 or 16");
  splitk_reduce(ws, nb, (long)wg3::C * wg3::NQ, dw, accumulate, st);
}

}  // namespace k8s_amd
