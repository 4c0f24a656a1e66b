// K2 weight gradient for tall-K / small-output convolutions (ResNet-50's 1x1 layers at 56x56 / 28x28, the
// strided 1x1 downsamples, and any RxS layer whose output tile count is small):
//
//   dW[k][(r, s, c)] (+)= sum_m dy[m][k] * x_im2col[m][(r, s, c)]      m = (n, ho, wo): N*Ho*Wo rows
//
// The reduction runs over millions of rows while dW is a few hundred KB, so the product is HBM-bound (reading
// dy and x once is the floor: e.g. 56x56x256 -> 64 at batch 1024 is 2 GB, ~0.33 ms). The generic 128 x 128 GEMM
// (gemm.hip) gets there through split-K slabs with one block per CU and a per-16-B im2col decode; MIOpen beat it
// on 11 of these shapes in round 1. Here instead:
//  * the grid is (output tiles) x (row chunks), sized to ~4 workgroups per CU, each 256-thread workgroup
//    streaming a contiguous run of 64-row k-steps through a 3-4 slot LDS ring filled by global_load_lds (16 B per
//    lane, lane-linear images, swizzle on the source address), so every CU keeps several stages of both operands
//    in flight -- enough bytes to cover HBM latency;
//  * the workgroups that share a row chunk (different output tiles) are placed on one XCD and adjacent in
//    dispatch order, so the operand they share is read from HBM once and from L2 after;
//  * partial sums leave through fp32 atomics (dW is zeroed by the launcher unless accumulating): a few tens of
//    KB per workgroup, far below the chip's ~1.3 TB/s atomic rate (MI355X_MICROARCH "Global float atomics");
//  * im2col is implicit: a k-step's 64 rows decode (n, ho, wo) once per lane, a tile's columns lie inside one
//    (r, s) tap because C % 64 == 0, and taps outside the image read a zero line.
// Both operands are consumed "MN-major" (the reduction index m is the row of dy and of x), through
// ds_read_b64_tr_b16 transposed fragment reads of v_mfma_f32_16x16x32_bf16.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {
namespace wgs {

constexpr int KS = 64;  // rows of the reduction per stage

__device__ __attribute__((aligned(64))) uint16_t g_zero16[64];

__device__ __forceinline__ int swz128(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }
__device__ __forceinline__ int swz256(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

// Transposed fragment of an [64 rows (m)][W cols] image (W = 64: 128-B rows, W = 128: 256-B rows):
// lane l holds col rb + (l & 15), rows kk*32 + 8*(l >> 4) + j. Issued as inline asm (tr16_asm: the builtin
// would make hipcc drain the LDS-DMA ring before every read); ready after the stage's lds tie.
struct TrRaw {
  short4_t lo, hi;
};
template <int W>
__device__ __forceinline__ void tr_load(TrRaw& r, const char* img, int rb, int kk, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int u = (rb >> 3) + (p >> 1);
  const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
  constexpr int RB = W * 2;
  int u0, u1;
  if constexpr (W == 64) {
    u0 = u ^ swz128(r0);
    u1 = u ^ swz128(r1);
  } else {
    u0 = u ^ swz256(r0);
    u1 = u ^ swz256(r1);
  }
  tr16_asm(r.lo, img + r0 * RB + (u0 << 4) + (p & 1) * 8);
  tr16_asm(r.hi, img + r1 * RB + (u1 << 4) + (p & 1) * 8);
}

// dy rows: m -> dy + m * K (plain [M][K] matrix), columns k0 .. k0 + W
struct DySrc {
  const uint16_t* p;
  int K, M;
};

// x rows through the implicit im2col of an NHWC input: row m = (n, ho, wo), columns (r, s, c) of one tap
struct XSrc {
  const uint16_t* x;
  int H, W, C, Ho, Wo, stride, pad, M;
  FastDiv fHW, fWo;
  int plain;  // 1x1 / stride 1 / pad 0: x is just the [M][C] matrix
};

struct Args {
  DySrc dy;
  XSrc xs;
  float* dw;   // [K][R*S*C] fp32
  int RSC;     // dW row length
  int S;       // kernel width (tap decode)
  int tiles_k, tiles_c;
  int chunk_steps;  // k-steps (64 rows) per workgroup
  int chunks;
};

// Tile KT (dW rows = dy columns) x CT (dW columns = im2col columns), WK x WC waves each owning a
// (KT / WK) x (CT / WC) piece, NSLOT-deep ring of 64-row stages:
//   <128,  64, 2, 2, 3>: 256 threads, 72 KB ring, 2 workgroups / CU -- 43.7 FLOP per L2->LDS byte
//   <128, 128, 2, 2, 2>: 256 threads, 64 KB ring, 2 workgroups / CU -- 64 FLOP / B
//   <256, 128, 4, 2, 3>: 512 threads, 144 KB ring, 1 workgroup / CU -- 87 FLOP / B
// L2 feeds LDS at ~70 GB/s per CU (MI355X_MICROARCH, "Indexed rows: gather into LDS"), so the FLOP/B of the
// tile caps the compute-bound (3x3) weight gradients at ~0.78 / 1.15 / 1.56 PFLOP/s.
//   <64, 64, 2, 2, 4>: K = 64 layers, 64 KB ring.
template <int KT, int CT, int WK, int WC, int NSLOT>
__global__ void __launch_bounds__(WK * WC * 64, WK * WC == 8 ? 1 : 2) wgrad_stream_kernel(Args a) {
  constexpr int THREADS = WK * WC * 64;
  constexpr int IMG_A = KS * KT * 2, IMG_B = KS * CT * 2, STAGE = IMG_A + IMG_B;
  __shared__ __attribute__((aligned(1024))) char smem[NSLOT * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wid / WC, wc = wid % WC;

  // tiles that share a chunk go to one XCD (bid % 8) and run back to back (bid / 8)
  const int T = a.tiles_k * a.tiles_c;
  const int bid = blockIdx.x;
  const int tile = (bid >> 3) % T;
  const int chunk = (bid & 7) + 8 * (bid / (8 * T));
  if (chunk >= a.chunks) return;
  const int tk = tile / a.tiles_c, tc = tile % a.tiles_c;
  const int k0 = tk * KT;
  const int col0 = tc * CT;  // dW column (r, s, c) of the tile's first column
  const int rs = col0 / a.xs.C, c0 = col0 - rs * a.xs.C;
  const int tap_r = rs / a.S, tap_s = rs - tap_r * a.S;
  const int step0 = chunk * a.chunk_steps;
  const int nsteps = min(a.chunk_steps, (a.dy.M + KS - 1) / KS - step0);
  if (nsteps <= 0) return;

  // ---- per-thread DMA sources. A image [64 m][KT k]: KT/8 units per row; B image [64 m][CT c].
  constexpr int UA = KT / 8, UB = CT / 8;               // 16-B units per row
  constexpr int LA = KS * UA / THREADS, LB = KS * UB / THREADS;  // glds per thread per stage
  static_assert(LA >= 1 && LB >= 1, "tile too small for 256 threads");
  const int dma_off = wid * 1024;
  static_assert(KT == 64 || KT == 128 || KT == 256, "KT");
  static_assert(CT == 64 || CT == 128, "CT");
  auto src_a = [&](int j, int m0) -> const void* {
    const int sl = j * THREADS + tid, row = sl / UA, up = sl % UA;
    const int u = KT == 64 ? (up ^ swz128(row)) : (up ^ swz256(row));
    const int m = m0 + row, k = k0 + u * 8;
    if (m >= a.dy.M || k >= a.dy.K) return g_zero16;
    return a.dy.p + (long)m * a.dy.K + k;
  };
  auto src_b = [&](int j, int m0) -> const void* {
    const int sl = j * THREADS + tid, row = sl / UB, up = sl % UB;
    const int u = CT == 64 ? (up ^ swz128(row)) : (up ^ swz256(row));
    const int m = m0 + row, c = c0 + u * 8;
    const XSrc& X = a.xs;
    if (m >= X.M || c >= X.C) return g_zero16;
    if (X.plain) return X.x + (long)m * X.C + c;
    const int n = X.fHW.div(m), rem = m - n * (X.Ho * X.Wo);
    const int ho = X.fWo.div(rem), wo = rem - ho * X.Wo;
    const int hi = ho * X.stride - X.pad + tap_r, wi = wo * X.stride - X.pad + tap_s;
    if ((unsigned)hi >= (unsigned)X.H || (unsigned)wi >= (unsigned)X.W) return g_zero16;
    return X.x + (((long)n * X.H + hi) * X.W + wi) * X.C + c;
  };
  auto issue = [&](int slot, int step) {
    char* st = smem + slot * STAGE;
    const int m0 = (step0 + step) * KS;
#pragma unroll
    for (int j = 0; j < LA; ++j) glds16(src_a(j, m0), st + j * (THREADS * 16) + dma_off);
#pragma unroll
    for (int j = 0; j < LB; ++j) glds16(src_b(j, m0), st + IMG_A + j * (THREADS * 16) + dma_off);
  };
  constexpr int PER = LA + LB;  // glds per thread per stage

  constexpr int RT = KT / WK / 16, CTT = CT / WC / 16;  // 16-wide tiles per wave
  f32x4_t acc[RT][CTT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < CTT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // prologue: up to NSLOT - 1 stages in flight
  const int pre = min(nsteps, NSLOT - 1);
  for (int s = 0; s < pre; ++s) issue(s, s);
  for (int s = 0; s < nsteps; ++s) {
    // stage s landed: the younger stages in flight are min(nsteps - 1, s + NSLOT - 2) - s
    const int younger = min(nsteps - 1, s + NSLOT - 2) - s;
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's DMA share of stage s is in LDS; stage s-1's reads are done
    asm volatile("" ::: "memory");
    if (s + NSLOT - 1 < nsteps) issue((s + NSLOT - 1) % NSLOT, s + NSLOT - 1);  // into the slot of stage s-1
    const char* st = smem + (s % NSLOT) * STAGE;
    TrRaw ar[2 * RT], br[2 * CTT];  // [kk * n + i]
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < RT; ++i) tr_load<KT>(ar[kk * RT + i], st, wk * (KT / WK) + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < CTT; ++j) tr_load<CT>(br[kk * CTT + j], st + IMG_A, wc * (CT / WC) + j * 16, kk, lane);
    }
    static_assert((2 * RT) % 4 == 0 && (2 * CTT) % 4 == 0, "tie groups of 4");
#pragma unroll
    for (int i = 0; i < 2 * RT; i += 4)
      K8S_LDS_TIE8("s_waitcnt lgkmcnt(0)", ar[i].lo, ar[i].hi, ar[i + 1].lo, ar[i + 1].hi, ar[i + 2].lo, ar[i + 2].hi,
                   ar[i + 3].lo, ar[i + 3].hi);
#pragma unroll
    for (int i = 0; i < 2 * CTT; i += 4)
      K8S_LDS_TIE8("s_waitcnt lgkmcnt(0)", br[i].lo, br[i].hi, br[i + 1].lo, br[i + 1].hi, br[i + 2].lo, br[i + 2].hi,
                   br[i + 3].lo, br[i + 3].hi);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < CTT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(join8(br[kk * CTT + j].lo, br[kk * CTT + j].hi),
                                                              join8(ar[kk * RT + i].lo, ar[kk * RT + i].hi),
                                                              acc[i][j], 0, 0, 0);
  }
  // acc[i][j]: lane holds dW[k = k0 + wk*KT/WK + i*16 + (lane & 15)][col0 + wc*CT/WC + j*16 + 4*(lane >> 4) + r]
#pragma unroll
  for (int i = 0; i < RT; ++i) {
    const int k = k0 + wk * (KT / WK) + i * 16 + (lane & 15);
    if (k >= a.dy.K) continue;
#pragma unroll
    for (int j = 0; j < CTT; ++j) {
      const int cl = wc * (CT / WC) + j * 16 + 4 * (lane >> 4);
      if (c0 + cl >= a.xs.C) continue;
      float* d = a.dw + (long)k * a.RSC + col0 + cl;
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(d + r, acc[i][j][r]);
    }
  }
}

}  // namespace wgs

// Tile choice: 128 x 64 (64 x 64 for K = 64). Measured (scripts/bench_wgrad_tiles.py, b1024): 128 x 128, 256 x 128
// are not faster on the shapes this kernel keeps (their rings leave one or two workgroups per CU).
struct WgsTile {
  int KT, CT;
};
static WgsTile wgs_tile(int K, int RSC) {
  (void)RSC;
  if (K % 128 == 0) return WgsTile{128, 64};
  return WgsTile{64, 64};
}

// Shapes this kernel takes: C % 64 == 0 (a tile's columns inside one tap), K % 64 == 0, and a 64-wide side of
// dW (K == 64 or R*S*C == 64: the memory-bound ResNet-50 layers at 56 x 56). Measured at batch 1024
// (scripts/bench_wgrad_tiles.py, profiles/r02_wgrad_tiles.jsonl) the generic split-K kernel is 5-60 % faster on
// every other ResNet-50 weight gradient, the 3x3 ones included.
bool wgrad_stream_eligible(int N, int Ho, int Wo, int C, int K, int R, int S) {
  if (C % 64 != 0 || K % 64 != 0) return false;
  const WgsTile t = wgs_tile(K, R * S * C);
  const long tiles = (long)(K / t.KT) * ((long)R * S * C / t.CT);
  const long rows = (long)N * Ho * Wo;
  const bool narrow = K == 64 || R * S * C == 64;
  return narrow && tiles <= 96 && rows >= 64L * 64;
}

void launch_wgrad_stream(const uint16_t* x, const uint16_t* dy, float* dw, int N, int H, int W, int C, int K, int R,
                         int S, int stride, int pad, int Ho, int Wo, bool accumulate, hipStream_t st) {
  using namespace wgs;
  if (C % 64 != 0 || K % 64 != 0) throw std::runtime_error("wgrad_stream: C and K must be multiples of 64");
  const int M = N * Ho * Wo, RSC = R * S * C;
  if (!accumulate) hipMemsetAsync(dw, 0, (size_t)K * RSC * sizeof(float), st);
  Args a;
  a.dy = DySrc{dy, K, M};
  a.xs = XSrc{x, H, W, C, Ho, Wo, stride, pad, M, make_fastdiv(Ho * Wo), make_fastdiv(Wo),
              (R == 1 && S == 1 && stride == 1 && pad == 0) ? 1 : 0};
  a.dw = dw;
  a.RSC = RSC;
  a.S = S;
  const WgsTile t = wgs_tile(K, RSC);
  a.tiles_k = K / t.KT;
  a.tiles_c = RSC / t.CT;
  const int T = a.tiles_k * a.tiles_c;
  const int steps = (M + KS - 1) / KS;
  // ~4 workgroups per CU in total, at least 8 k-steps each (prologue amortised), chunks a multiple of 8 so the
  // tiles of one chunk share an XCD
  const int per_cu = 4;
  int chunks = (per_cu * 256 + T - 1) / T;
  chunks = (chunks + 7) / 8 * 8;
  chunks = std::max(8, std::min(chunks, (steps + 7) / 8));
  a.chunk_steps = (steps + chunks - 1) / chunks;
  a.chunks = (steps + a.chunk_steps - 1) / a.chunk_steps;
  const int grid = ((a.chunks + 7) / 8) * 8 * T;
  if (t.KT == 128)
    hipLaunchKernelGGL((wgrad_stream_kernel<128, 64, 2, 2, 3>), dim3(grid), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((wgrad_stream_kernel<64, 64, 2, 2, 4>), dim3(grid), dim3(256), 0, st, a);
}

}  // namespace k8s_amd
