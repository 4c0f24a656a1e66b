// LDS-tiled weight gradient of the ResNet-50 stride-1 3x3 convolutions (C = K = 64 / 128 / 256 at 56 / 28 / 14
// pixels square, pad 1).
//
//   dw[k][r][s][c] = sum_{n,h,w} dy[n][h][w][k] * x[n][h + r - 1][w + s - 1][c]
// The generic split-K implicit GEMM (gemm.hip ConvWgB) gathers every 16-B tap unit of im2col(x) from L2 nine
// times and, at K = 64, fills half of its 128-row tiles (~270 TF/s at stage 1). Here the product is cut into
// 64 x 576 pieces -- output channels k0 .. k0 + 63 x (9 taps x input channels c0 .. c0 + 63), one piece per
// blockIdx.y -- and persistent blocks (2 per CU) sweep tiles of RT output rows: per tile the (RT + 2)-row
// zero-padded input window of the 64-channel slice and the RT dy rows of the 64-output slice are staged in LDS by
// LDS-DMA, both MFMA operands are read from them transposed (ds_read_b64_tr_b16: 4 pixels x 16 channels per 16
// lanes), and each block keeps its fp32 partial of the piece in accumulator registers (wave w: output columns
// 144 w .. 144 w + 143) until its last tile; wg3_reduce1/2 sum the blocks' partials into dw.
//   LDS images: [position][64 ch] bf16, 128-B rows, 16-B chunk c of row p at c ^ (p & 7) (window and dy alike).
//   Wave w computes q tiles 4 tap + w (channel group w of every tap), so a tap's row / column offsets are compile-time;
//   with the window pitch a multiple of 8, per k step each lane forms 3 addresses per pixel (column taps) and the row
//   taps are immediate offsets (round 6: the per-tap swizzle arithmetic was 3.3 VALU per MFMA).
//   tile: RT rows x W pixels, RT * W = 224 (7 k-steps of 32 pixels; a tile may run past the image: zero dy rows;
//   the W = 16 test shape: 2 rows)
#include <algorithm>
#include <stdexcept>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {

namespace wg3 {
constexpr int CS = 64, NQ = 9 * CS;  // a piece: 64 output channels x 576 (tap, input channel) columns
__device__ __attribute__((aligned(64))) uint16_t g_wg3_zero[64];  // source of the zero padding

__device__ __forceinline__ int off(int p, int ch16) { return p * 128 + ((ch16 ^ (p & 7)) << 4); }

// XF: the activation operand is relu(x * scale + shift) (BatchNorm normalised on load, xf = fp32 [2][C] scale |
// shift): each thread rewrites its staged window chunks in place once per tile, the zero padding left zero (the
// forward's conv3x3.hip does the same, so the bn1 apply pass is gone from both directions).
template <int W, int RT, bool XF = false>
__global__ void __launch_bounds__(256, 2) wgrad3x3_kernel(const uint16_t* __restrict__ x,
                                                         const uint16_t* __restrict__ dy, float* __restrict__ ws,
                                                         int H, int C, int K, int tiles_per_img, int ntiles,
                                                         const float* __restrict__ xf) {
  // window pitch a multiple of 8 positions: a position's swizzle (p & 7) is then the same for the three filter rows,
  // so the row taps are immediate LDS offsets of one per-(k step, column tap) address
  constexpr int WP = (W + 2 + 7) / 8 * 8, WIN = (RT + 2) * WP, PX = RT * W, NKS = PX / 32;
  static_assert(PX % 32 == 0, "whole 32-pixel k steps");
  __shared__ __attribute__((aligned(1024))) char smem[(WIN + PX) * 128];
  char* const xw = smem;
  char* const dl = smem + WIN * 128;
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, G = lane >> 4, q4 = li >> 2, p4 = li & 3;
  const int cpieces = C / CS, k0 = (blockIdx.y / cpieces) * CS, c0 = (blockIdx.y % cpieces) * CS;
  const int hb = (p4 & 1) * 8, c1 = p4 >> 1;
  // dy^T fragment offsets in the dy image, tile- and k-step-invariant: the k step's first pixel 32 ks + 8 G is a
  // multiple of 8, so the swizzle of pixel + q4 (+ 4) is q4 (+ 4); a k step adds 32 positions (4 KB, uniform)
  int aoff[4][2];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    const int ch16 = 2 * kt + c1;
    aoff[kt][0] = (8 * G + q4) * 128 + ((ch16 ^ q4) << 4) + hb;
    aoff[kt][1] = (8 * G + 4 + q4) * 128 + ((ch16 ^ (q4 + 4)) << 4) + hb;
  }
  const int cq5 = wid << 5;  // this wave's 16-channel group (q tile 4 tap + wid) as a swizzled-chunk XOR term

  f32x4_t acc[4][9];  // [k tile][tap j]: lane holds piece[16 kt + 4 G + r][16 (4 j + wid) + li]
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
          const void* src =
              in ? (const void*)(x + (((long)n * H + h) * W + w) * C + c0 + lc * 8) : (const void*)g_wg3_zero;
          glds16(src, xw + __builtin_amdgcn_readfirstlane(i * 256 + wid * 64) * 16);
        }
      }
#pragma unroll 1
      for (int i = 0; i < ND; ++i) {
        const int c = i * 256 + tid;
        if (c < PX * 8) {
          const int p = c >> 3, lc = (c & 7) ^ (p & 7);
          const bool in = h0 + p / W < H;
          const void* src =
              in ? (const void*)(dy + (((long)n * H + h0) * W + p) * K + k0 + lc * 8) : (const void*)g_wg3_zero;
          glds16(src, dl + __builtin_amdgcn_readfirstlane(i * 256 + wid * 64) * 16);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if constexpr (XF) {
      // a thread's window chunks c = i * 256 + tid all hold logical channels 8 * ((tid & 7) ^ ((tid >> 3) & 7)) + 0..7
      // (scale / shift re-read per tile from L1: kept live across the K loop they spill the 255-VGPR kernel)
      float xsc[8], xsh[8];
      const int ch = c0 + 8 * ((tid & 7) ^ ((tid >> 3) & 7));
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xsc[j] = xf[ch + j];
        xsh[j] = xf[C + ch + j];
      }
#pragma unroll 1
      for (int i = 0; i < (WIN * 8 + 255) / 256; ++i) {
        const int c = i * 256 + tid;
        if (c < WIN * 8) {
          const int p = c >> 3, wr = p / WP, wc = p - wr * WP, h = h0 - 1 + wr, w = wc - 1;
          if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
            bf16x8_t* q = reinterpret_cast<bf16x8_t*>(xw + c * 16);
            const bf16x8_t v = *q;
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = fmaxf(__builtin_fmaf(bf2f((uint16_t)v[j]), xsc[j], xsh[j]), 0.f);
            *q = pack_bf16x8(o);
          }
        }
      }
      __syncthreads();
    }
#pragma unroll  // (unrolled: the dy reads' k-step offsets are immediates, the window addresses tile-invariant)
    for (int ks = 0; ks < NKS; ++ks) {
      const lds_char* const dk = lds_ptr(dl) + ks * 4096;
      mfma_bf16x8 af[4];  // dy^T: row = output channel 16 kt + li, k = 8 pixels
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) af[kt] = join8(tr16l(dk, aoff[kt][0]), tr16l(dk, aoff[kt][1]));
      // window positions of this lane's two pixels (pb + q4, pb + 4 + q4) at tap (0, 0), and per column tap s the
      // byte address of this wave's 16-channel group there (row taps: + r WP 128, immediate)
      const int pa = 32 * ks + 8 * G + q4, pc = pa + 4;
      const int ra = pa / W, rc = pc / W;
      const int posa = ra * WP + (pa - ra * W), posc = rc * WP + (pc - rc * W);
      int za[3], zc[3];
#pragma unroll
      for (int s_ = 0; s_ < 3; ++s_) {
        const int qa = posa + s_, qc = posc + s_;
        za[s_] = qa * 128 + hb + (cq5 ^ (((qa & 7) ^ c1) << 4));
        zc[s_] = qc * 128 + hb + (cq5 ^ (((qc & 7) ^ c1) << 4));
        // opaque: otherwise the compiler re-associates the row-tap constants into the sums and adds per read
        asm volatile("" : "+v"(za[s_]), "+v"(zc[s_]));
      }
#pragma unroll
      for (int j = 0; j < 9; ++j) {  // tap j = 3 r + s (compile-time), channel group wid
        const int r_ = j / 3, s_ = j - 3 * r_;
        const lds_char* const xr = lds_ptr(xw) + r_ * WP * 128;  // (immediate)
        const mfma_bf16x8 bf = join8(tr16l(xr, za[s_]), tr16l(xr, zc[s_]));
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) acc[kt][j] = mfma16(af[kt], bf, acc[kt][j]);
      }
    }
    __syncthreads();  // every wave is done with this tile's LDS before the next stage
  }
  float* out = ws + ((long)blockIdx.y * gridDim.x + blockIdx.x) * (CS * NQ);
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(kt * 16 + G * 4 + r) * NQ + (4 * j + wid) * 16 + li] = acc[kt][j][r];
}

// Two-pass deterministic sum of the nb per-block partials of every piece: pass 1 (blockIdx.y = slab group s of SG)
// sums slabs s, s + SG, ... into part[s]; pass 2 sums the SG group partials and scatters the piece into
// dw[k0 + kk][tap][c0 + cc] (+)=. (One pass with a 512-slab serial loop per output ran 125 us at stage 1.)
__global__ void __launch_bounds__(256) wg3_reduce1_kernel(const float* __restrict__ ws, int nb, int pieces, int SG,
                                                          float* __restrict__ part) {
  const long n4 = (long)pieces * CS * NQ / 4;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;  // float4 index over [pieces][64][576]
  if (e >= n4) return;
  const int piece = (int)(e / (CS * NQ / 4));
  const long rem4 = e - (long)piece * (CS * NQ / 4);
  const float4* src = reinterpret_cast<const float4*>(ws) + (long)piece * nb * (CS * NQ / 4) + rem4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
  for (int b = blockIdx.y; b < nb; b += SG) {
    const float4 v = src[(long)b * (CS * NQ / 4)];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  reinterpret_cast<float4*>(part)[(long)blockIdx.y * n4 + e] = s;
}

__global__ void __launch_bounds__(256) wg3_reduce2_kernel(const float* __restrict__ part, int SG, int C, int pieces,
                                                          float* __restrict__ dw, int accumulate) {
  const long n4 = (long)pieces * CS * NQ / 4;
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n4) return;
  const int piece = (int)(e / (CS * NQ / 4));
  const int rem = (int)(e - (long)piece * (CS * NQ / 4)) * 4;
  const int kk = rem / NQ, q = rem - kk * NQ, tap = q / CS, cc = q - tap * CS;
  const int cpieces = C / CS, k0 = (piece / cpieces) * CS, c0 = (piece % cpieces) * CS;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g = 0; g < SG; ++g) {
    const float4 v = reinterpret_cast<const float4*>(part)[(long)g * n4 + e];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  float4* d = reinterpret_cast<float4*>(dw + ((long)(k0 + kk) * 9 + tap) * C + c0 + cc);
  if (accumulate) {
    const float4 o = *d;
    s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
  }
  *d = s;
}
}  // namespace wg3

// stride-1 / pad-1 3x3, C == K in {64, 128, 256} with the matching square image side (56 / 28 / 14), or the small
// W = 16 test shape at 64 channels
bool wgrad3x3_tiled_ok(int C, int K, int R, int S, int stride, int pad, int W) {
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || C != K) return false;
  return (C == 64 && (W == 56 || W == 16)) || (C == 128 && W == 28) || (C == 256 && W == 14);
}

static int wg3_rt(int W) { return W == 56 ? 4 : W == 28 ? 8 : W == 16 ? 2 : 16; }

int wgrad3x3_tiled_blocks(int N, int H, int W, int C) {
  const int pieces = (C / wg3::CS) * (C / wg3::CS);
  const long tiles = (long)N * ((H + wg3_rt(W) - 1) / wg3_rt(W));
  return (int)std::max<long>(1, std::min<long>(tiles, std::max(2 * planner_cus() / pieces, 32)));
}

static int wg3_groups(int nb) { return std::max(1, nb / 16); }

long wgrad3x3_tiled_workspace(int N, int H, int W, int C) {
  const long pieces = (long)(C / wg3::CS) * (C / wg3::CS);
  const int nb = wgrad3x3_tiled_blocks(N, H, W, C);
  return pieces * (nb + wg3_groups(nb)) * wg3::CS * wg3::NQ;  // block partials + slab-group partials
}

template <int W, int RT>
static void wg3_launch(dim3 grid, hipStream_t st, const uint16_t* x, const uint16_t* dy, float* ws, int H, int C,
                       int tpi, int ntiles, const float* xf) {
  if (xf)
    hipLaunchKernelGGL((wg3::wgrad3x3_kernel<W, RT, true>), grid, dim3(256), 0, st, x, dy, ws, H, C, C, tpi, ntiles, xf);
  else
    hipLaunchKernelGGL((wg3::wgrad3x3_kernel<W, RT>), grid, dim3(256), 0, st, x, dy, ws, H, C, C, tpi, ntiles, xf);
}

void launch_wgrad3x3_tiled(const uint16_t* x, const uint16_t* dy, float* ws, float* dw, int N, int H, int W, int C,
                           bool accumulate, hipStream_t st, const float* xform) {
  const int rt = wg3_rt(W), tpi = (H + rt - 1) / rt;
  const long ntiles = (long)N * tpi;
  if (ntiles >= (1L << 31)) throw std::runtime_error("wgrad3x3_tiled: too many tiles");
  const int pieces = (C / wg3::CS) * (C / wg3::CS);
  const int nb = wgrad3x3_tiled_blocks(N, H, W, C);
  const dim3 grid(nb, pieces);
  if (W == 56) wg3_launch<56, 4>(grid, st, x, dy, ws, H, C, tpi, (int)ntiles, xform);
  else if (W == 28) wg3_launch<28, 8>(grid, st, x, dy, ws, H, C, tpi, (int)ntiles, xform);
  else if (W == 16) wg3_launch<16, 2>(grid, st, x, dy, ws, H, C, tpi, (int)ntiles, xform);
  else if (W == 14) wg3_launch<14, 16>(grid, st, x, dy, ws, H, C, tpi, (int)ntiles, xform);
  else throw std::runtime_error("wgrad3x3_tiled: unsupported width");
  const long n4 = (long)pieces * wg3::CS * wg3::NQ / 4;
  const int SG = wg3_groups(nb);
  float* part = ws + (long)pieces * nb * wg3::CS * wg3::NQ;
  hipLaunchKernelGGL(wg3::wg3_reduce1_kernel, dim3(cdiv(n4, 256), SG), dim3(256), 0, st, ws, nb, pieces, SG, part);
  hipLaunchKernelGGL(wg3::wg3_reduce2_kernel, dim3(cdiv(n4, 256)), dim3(256), 0, st, part, SG, C, pieces, dw,
                     accumulate ? 1 : 0);
}

}  // namespace k8s_amd
