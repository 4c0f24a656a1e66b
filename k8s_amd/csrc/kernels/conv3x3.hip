// K2: staged-window 3 x 3 / stride-1 / pad-1 NHWC convolution for gfx950 (the ResNet-50 bottleneck conv2 of every
// block but the stage-entry ones, forward and -- with spatially flipped, in/out-swapped weights -- data gradient).
//
//   y[n][h][w][k] = sum_{r,s,c} x[n][h + r - 1][w + s - 1][c] * wt[k][r][s][c]
//
// The implicit GEMM of gemm.hip (ConvA) gathers im2col(x) through L2: every input element is fetched into LDS nine
// times, one 16-B LDS-DMA piece per (pixel, tap, 8 channels). Here a block owns RT whole image rows (RT * W output
// pixels) x KT output channels and stages the zero-padded (RT + 2) x (W + 2) input WINDOW of each 64-channel slice
// once; the nine taps read the MFMA A operand from that window at a shifted position. The slice's weights stream per
// tap ([KT][64] bf16, double-buffered, the next tap's DMA behind this tap's MFMAs).
//
// XF (BatchNorm + ReLU normalised on load, see gemm.hip XForm): after the window lands, each thread rewrites its
// window chunks in place as relu(x * scale + shift) -- ONCE per staged element, not once per tap (the implicit GEMM's
// on-load path re-applied it nine times) -- leaving the zero padding zero. The BN apply pass of bn1 (read x, write z)
// and the z tensor then disappear from the ResNet forward.
//
// Layout / tiling:
//  * 256 threads = 4 waves as 2 (pixels) x 2 (channels); wave piece = MF x 16 pixels x KT / 2 channels, MF x NF
//    tiles of v_mfma_f32_16x16x32_bf16 (operands swapped: each lane ends with 4 consecutive output channels).
//  * window: row wr (image row h0 - 1 + wr) at positions wr * WP + 8 + [0, W), WP = W rounded up to a multiple of 8
//    (64 / 32 / 16); the positions between rows are zero and serve as the left and right padding. Output pixel m =
//    (r, c) reads position pw + dr * WP + ds at tap (dr, ds), pw = r * WP + 7 + c. Because WP % 8 == 0 the swizzle
//    below is the same for all three dr, so a lane's A address is computed once per ds and the dr taps are
//    immediate offsets of the same ds_read_b128.
//  * LDS images [position][64 ch] (window) and [row][64 ch] (weights), 128-B rows, 16-B chunk c of row p stored at
//    c ^ (p & 6): with fragment lane group j reading chunk 4 kk + j, every ds_read_b128 lane group of 16 consecutive
//    positions -- starting at ANY position -- hits 16 distinct 16-B bank slots (searched exhaustively; the
//    (p >> 1) & 7 XOR of gemm.hip is conflict-free only for 16-aligned runs and cost 37-41 % of the LDS cycles here).
//    A fragment crossing a row end jumps by WP - W positions: 8 at W = 56 (still conflict-free), 4 / 2 at 28 / 14.
//  * NS weight slots: tap g + NS - 1 streams in while tap g computes.
//  * measured (profiles/r04_conv3x3_pmc.txt): 1.10-1.24x the implicit GEMM; the 56 x 56 layer runs at 28 % MFMA busy
//    and an ablation of its phases (staging, LDS reads, epilogue) shows no single one dominating -- the two blocks per
//    CU overlap their phases poorly. The swizzle, address and weight-ring changes above moved it by < 1 %.
//  * epilogue: the bf16 tile goes through LDS, leaves as 16-B row segments, and the per-channel sum / sum of squares
//    of the stored values are accumulated for the following BatchNorm (the [STAT_REPL][2][K] layout of gemm.hip).
//  * per-tile prologue (round 6): only the padding positions are zeroed (enumerated, 2 iterations at 56 x 56 instead
//    of a divide-and-test over all 12 window chunks per thread), the window and weight DMA addresses are a lane offset
//    fixed per tile plus a wave-uniform offset: 3-8.5 % per layer (profiles/r06_conv3x3_lean.jsonl).
//  * <= 80 KB LDS: 2 blocks per CU, so one block's window staging overlaps the other's MFMAs.
//  * the per-tap barrier is a raw s_barrier after explicit waits (__syncthreads() adds a release fence, i.e.
//    s_waitcnt vmcnt(0), which drained the in-flight weight tap every step): 2-5 % per layer (round 5).
//  * not kept (round 5, profiles/r05_conv3x3_c3p_ab.jsonl, r05_conv3x3_pmc.txt): a persistent form with one block
//    per CU walking a range of tiles, both windows and a 4-slot weight ring in flight, fragments read one k-half
//    ahead among the MFMAs (the g4 GEMM's schedule) and the epilogue stored from registers -- 0.63-0.76x this
//    kernel at 28 x 28 / 14 x 14. With 8 waves (2 per SIMD) it read 0.64 fragments per MFMA and saturated the LDS
//    (26-30 % MFMA busy); with 4 (one per SIMD) the loop ran ~60 % MFMA-busy cycles but the kernel still lost on
//    wall time to this one's two blocks per CU, and its register-direct epilogue with statistics cost ~25 %.
#include <stdexcept>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {

namespace c3 {
constexpr int THREADS = 256;
constexpr int STAT_REPL = 32;  // = gemm.hip STAT_REPL = kConvStatReplicas
__device__ __attribute__((aligned(64))) uint16_t g_c3_zero[64];  // source of the rows outside the image

__device__ __forceinline__ int swz(int p) { return p & 6; }

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int W, int RT, int KT, bool XF>
struct Geo {
  static constexpr int WP = (W + 7) / 8 * 8 + (W % 8 == 0 ? 8 : 0), P = RT * W;
  static constexpr int NPOS = (RT + 2) * WP + 8;  // + the right padding of the last row
  static constexpr int MF = (P + 31) / 32, NF = KT / 32;
  static constexpr int WIN_B = NPOS * 128, WT_B = KT * 128;
  static constexpr int NS = WIN_B + 3 * WT_B <= 80 * 1024 ? 3 : 2;  // 2 blocks per CU
  static constexpr int STAGE_B = 32 * MF * KT * 2;  // epilogue C tile
  static constexpr int LDS = (WIN_B + NS * WT_B) > STAGE_B ? (WIN_B + NS * WT_B) : STAGE_B;
  static_assert(WIN_B + NS * WT_B <= 80 * 1024, "two blocks per CU");
  static_assert(LDS >= THREADS * 16 * 4, "room for the statistics partials");
  static_assert(WP % 8 == 0 && WP > W, "pitch");
};

template <int W, int RT, int KT, bool XF>
__global__ void __launch_bounds__(THREADS, 2) conv3x3_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ wt, uint16_t* __restrict__ y,
                                                            float* __restrict__ stats, const float* __restrict__ xf,
                                                            int H, int C, int K, int tiles_per_img, BnBwdSums bb) {
  using G = Geo<W, RT, KT, XF>;
  constexpr int WP = G::WP, NPOS = G::NPOS, P = G::P, MF = G::MF, NF = G::NF, NS = G::NS;
  constexpr int WOPS = KT * 8 / THREADS;  // weight DMA instructions per thread per tap
  __shared__ __attribute__((aligned(1024))) char smem[G::LDS];
  char* const win = smem;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int tile = blockIdx.x;
  const int n = tile / tiles_per_img, h0 = (tile - n * tiles_per_img) * RT;
  const int k0 = blockIdx.y * KT;

  // window position of this lane's pixel for each fragment at tap (0, 0); pad lanes of a last fragment (m >= P, only
  // when P % 32 != 0) read what lies past the window -- their output rows are never stored
  int pw[MF];
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int m = (wm * MF + f) * 16 + (lane & 15), r = m / W;
    pw[f] = r * WP + 7 + (m - r * W);
  }
  int boff[2][NF];  // B operand byte offsets in a weight slot
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int r = wn * (KT / 2) + j * 16 + (lane & 15), ch = kk * 4 + (lane >> 4);
      boff[kk][j] = r * 128 + ((ch ^ swz(r)) << 4);
    }
  f32x4_t acc[MF][NF];
#pragma unroll
  for (int f = 0; f < MF; ++f)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // the padding positions (everything that is not image data) are zeroed once; the DMA never writes them
  constexpr int PADR = WP - W, NPAD = 8 + (RT + 2) * PADR;  // 8 leading positions + PADR after every window row
#pragma unroll
  for (int t0 = 0; t0 < NPAD * 8; t0 += THREADS) {  // only the padding positions, enumerated
    const int t = t0 + tid, pi = t >> 3;
    if (t < NPAD * 8) {
      const int r = (pi - 8) / PADR;
      const int pos = pi < 8 ? pi : 8 + r * WP + W + (pi - 8 - r * PADR);
      *reinterpret_cast<bf16x8_t*>(win + (pos * 8 + (t & 7)) * 16) = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  // window DMA: row wr, instruction i covers positions wr * WP + 8 + 8 i + [0, 8) (lane-linear 16-B pieces); the
  // logical chunk of a lane is fixed because every instruction's first position is a multiple of 8
  constexpr int IPR = (W * 8 + 63) / 64, NWI = (RT + 2) * IPR;
  const int lch = (lane & 7) ^ ((lane >> 3) & 6);
  // the lane's part of the address is fixed per tile (image n, pixel lane >> 3, chunk lch); per instruction only
  // a wave-uniform row / pixel-group offset is added
  const uint16_t* const xlane = x + ((long)n * H * W + (lane >> 3)) * C + lch * 8;
  auto load_window = [&](int c0) {
#pragma unroll 1
    for (int wi = wid; wi < NWI; wi += THREADS / 64) {  // wave-uniform
      const int wr = wi / IPR, i = wi - wr * IPR, h = h0 - 1 + wr;
      if (i * 8 + (lane >> 3) < W) {
        const void* src = (unsigned)h < (unsigned)H ? (const void*)(xlane + (h * W + i * 8) * C + c0)
                                                    : (const void*)g_c3_zero;
        glds16(src, win + (wr * WP + 8 + i * 8) * 128);
      }
    }
  };
  auto transform_window = [&](int c0) {  // XF: relu(x * scale + shift) in place, once per staged image element
    const int lc = (tid & 7) ^ ((tid >> 3) & 6);  // logical chunk of LDS chunk c = k * 256 + tid
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = xf[c0 + lc * 8 + j];
      sh[j] = xf[C + c0 + lc * 8 + j];
    }
#pragma unroll 1
    for (int c = tid; c < NPOS * 8; c += THREADS) {
      const int q = (c >> 3) - 8, wr = q / WP, h = h0 - 1 + wr;
      if (q >= 0 && q - wr * WP < W && wr < RT + 2 && (unsigned)h < (unsigned)H) {
        bf16x8_t* qp = reinterpret_cast<bf16x8_t*>(win + c * 16);
        const bf16x8_t v = *qp;
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaxf(__builtin_fmaf(bf2f((uint16_t)v[j]), sc[j], sh[j]), 0.f);
        *qp = pack_bf16x8(o);
      }
    }
    __syncthreads();
  };
  // per-thread weight source offsets (row k0 + row, chunk lc) computed once; a tap adds a uniform offset
  uint32_t wlane[WOPS];  // byte offsets (32-bit: the tap's uniform base + a lane offset, the saddr load form)
#pragma unroll
  for (int i = 0; i < WOPS; ++i) {
    const int c = i * THREADS + tid, row = c >> 3, lc = (c & 7) ^ swz(row);
    wlane[i] = (uint32_t)(((k0 + row) * 9 * C + lc * 8) * 2);
  }
  auto stage_w = [&](int tap, int c0, int slot) {
    char* d = smem + G::WIN_B + slot * G::WT_B;
#pragma unroll
    for (int i = 0; i < WOPS; ++i) {
      glds16(reinterpret_cast<const char*>(wt + tap * C + c0) + wlane[i], d + (i * THREADS + wid * 64) * 16);
    }
  };
  // steps g = slice * 9 + 3 ds + dr visit the taps ds-major; tap_of(k) for k = g % 9
  auto tap_of = [](int k) { return (k % 3) * 3 + k / 3; };

  // BatchNorm-backward sums (bb.sums, a data gradient): this thread's x chunks at its output positions. With a 64-wide
  // K tile (the 56 x 56 layers: 7 chunks, 28 VGPRs beside 186) they are loaded here, behind the first window DMA, so
  // the epilogue never waits on them (loaded at the epilogue, their latency was exposed once per tile: +0.5 ms per
  // 56 x 56 call); the 128-wide tiles have no such room and load them when the accumulators are freed.
  constexpr int CPR = KT / 8;
  constexpr int RSTEP = THREADS / CPR, NR = (P + RSTEP - 1) / RSTEP;
  constexpr bool XEARLY = KT == 64;
  const int c = tid % CPR, row0 = tid / CPR;
  const bool bst = bb.sums != nullptr;
  bf16x8_t xr[NR];
  auto load_xr = [&]() {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = row0 + i * RSTEP, hr = m / W, h = h0 + hr;
      xr[i] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      if (m < P && h < H)
        xr[i] = *reinterpret_cast<const bf16x8_t*>(bb.x + (((long)n * H + h) * W + (m - hr * W)) * K + k0 + c * 8);
    }
  };
  const int nsteps = (C >> 6) * 9;
  load_window(0);
  if (XEARLY && bst) load_xr();
#pragma unroll
  for (int g = 0; g < NS - 1; ++g)
    if (g < nsteps) stage_w(tap_of(g), 0, g);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (XF) transform_window(0);
#pragma unroll 1
  for (int cs = 0; cs < (C >> 6); ++cs) {
    if (cs) {  // next 64-channel slice: every wave is past the previous slice's last tap (barrier)
      load_window(cs * 64);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if constexpr (XF) transform_window(cs * 64);
    }
#pragma unroll 1
    for (int ds = 0; ds < 3; ++ds) {
      int aoff[2][MF];
#pragma unroll
      for (int f = 0; f < MF; ++f) {
        const int p = pw[f] + ds;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) aoff[kk][f] = p * 128 + (((kk * 4 + (lane >> 4)) ^ swz(p)) << 4);
      }
#pragma unroll
      for (int dr = 0; dr < 3; ++dr) {
        const int g = cs * 9 + ds * 3 + dr, gp = g + NS - 1;
        if (gp < nsteps) stage_w(tap_of(gp % 9), gp / 9 * 64, gp % NS);  // slot last read in step g - 1
        const char* ws = smem + G::WIN_B + (NS == 3 ? dr : g & 1) * G::WT_B;  // NS = 3: g % 3 == dr
        const char* wa = win + dr * WP * 128;
        if constexpr (NF == 2) {
          // both k-halves' fragments read up front, the first half's MFMAs waiting only for their own reads (the
          // compiler's own order waited for every read before the next: LDS latency exposed at 2 waves per SIMD)
          mfma_bf16x8 af[2][MF], bfr[2][NF];
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
            for (int f = 0; f < MF; ++f)
              af[kk][f] = __builtin_bit_cast(mfma_bf16x8, *reinterpret_cast<const bf16x8_t*>(wa + aoff[kk][f]));
#pragma unroll
            for (int j = 0; j < NF; ++j)
              bfr[kk][j] = __builtin_bit_cast(mfma_bf16x8, *reinterpret_cast<const bf16x8_t*>(ws + boff[kk][j]));
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            if (kk == 0) asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(MF + NF) : "memory");
            else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int f = 0; f < MF; ++f)
#pragma unroll
              for (int j = 0; j < NF; ++j)
                acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[kk][j], af[kk][f], acc[f][j], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {  // 112 accumulator VGPRs: no room for a second fragment set
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            mfma_bf16x8 af[MF], bfr[NF];
#pragma unroll
            for (int f = 0; f < MF; ++f)
              af[f] = __builtin_bit_cast(mfma_bf16x8, *reinterpret_cast<const bf16x8_t*>(wa + aoff[kk][f]));
#pragma unroll
            for (int j = 0; j < NF; ++j)
              bfr[j] = __builtin_bit_cast(mfma_bf16x8, *reinterpret_cast<const bf16x8_t*>(ws + boff[kk][j]));
#pragma unroll
            for (int f = 0; f < MF; ++f)
#pragma unroll
              for (int j = 0; j < NF; ++j)
                acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[f], acc[f][j], 0, 0, 0);
          }
        }
        // step g + 1's weights landed (step g + NS - 1's may still be in flight). A raw s_barrier: __syncthreads()
        // adds a workgroup release fence -- s_waitcnt vmcnt(0) -- which drained the in-flight weight tap every step
        if (NS > 2 && gp < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WOPS * (NS - 2)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
      }
    }
  }

  // ---- epilogue: [32 MF][KT] bf16 tile in LDS (16-B chunk c of row r at c ^ (r % CPR)), 16-B copy-out with the BN
  // statistics of the stored values -- or, as a data gradient (bb.sums), the BatchNorm-backward sums of the
  // non-residual BatchNorm + ReLU that produced the convolution's input: g = relu_on(x) ? dx : 0, sum g and
  // sum g (x - mean) per channel, x read at the output positions (prefetched here, into the registers the
  // accumulators free, so the loads overlap the staging)
  float bsc[8], bsh[8], bmu[8];
  if (bst) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = k0 + c * 8 + j;
      bmu[j] = bb.mean[col];
      bn_affine_regs(bb.gamma[col], bb.beta[col], bmu[j], bb.invstd[col], bsc[j], bsh[j]);
    }
    if (!XEARLY) load_xr();
  }
  uint16_t* const ctile = reinterpret_cast<uint16_t*>(smem);
#pragma unroll
  for (int f = 0; f < MF; ++f) {
    const int row = (wm * MF + f) * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int col = wn * (KT / 2) + j * 16 + (lane >> 4) * 4;
      const bf16x4_t o = __builtin_bit_cast(bf16x4_t, __builtin_convertvector(acc[f][j], bf16v4_t));
      *reinterpret_cast<bf16x4_t*>(ctile + row * KT + (((col >> 3) ^ (row % CPR)) << 3) + (col & 4)) = o;
    }
  }
  __syncthreads();
  f32x2_t s2[4], q2[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) s2[r] = q2[r] = f32x2_t{0.f, 0.f};
  if (bst) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = row0 + i * RSTEP, hr = m / W, h = h0 + hr;
      if (m < P && h < H) {
        const bf16x8_t o = *reinterpret_cast<const bf16x8_t*>(ctile + m * KT + ((c ^ (m % CPR)) << 3));
        *reinterpret_cast<bf16x8_t*>(y + (((long)n * H + h) * W + (m - hr * W)) * K + k0 + c * 8) = o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          f32x2_t g, d;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const float xv = bf2f((uint16_t)xr[i][2 * r + e]);
            g[e] = relu_on(xv, bsc[2 * r + e], bsh[2 * r + e]) ? bf2f((uint16_t)o[2 * r + e]) : 0.f;
            d[e] = xv - bmu[2 * r + e];
          }
          s2[r] += g;
          q2[r] = __builtin_elementwise_fma(g, d, q2[r]);
        }
      }
    }
  } else {
#pragma unroll 2
  for (int m = row0; m < P; m += RSTEP) {
    const int hr = m / W, h = h0 + hr;
    if (h < H) {
      const bf16x8_t o = *reinterpret_cast<const bf16x8_t*>(ctile + m * KT + ((c ^ (m % CPR)) << 3));
      *reinterpret_cast<bf16x8_t*>(y + (((long)n * H + h) * W + (m - hr * W)) * K + k0 + c * 8) = o;
      if (stats) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&o);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const f32x2_t v = {__uint_as_float(w[r] << 16), __uint_as_float(w[r] & 0xFFFF0000u)};
          s2[r] += v;
          q2[r] = __builtin_elementwise_fma(v, v, q2[r]);
        }
      }
    }
  }
  }
  if (stats || bst) {
    __syncthreads();
    float* part = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      part[tid * 16 + 2 * r] = s2[r][0];
      part[tid * 16 + 2 * r + 1] = s2[r][1];
      part[tid * 16 + 8 + 2 * r] = q2[r][0];
      part[tid * 16 + 8 + 2 * r + 1] = q2[r][1];
    }
    __syncthreads();
    if (tid < 2 * KT) {
      const int col = tid % KT, which = tid / KT, cc = col >> 3, r = col & 7;
      float v = 0.f;
#pragma unroll 4
      for (int t = cc; t < THREADS; t += CPR) v += part[t * 16 + which * 8 + r];
      atomicAdd((bst ? bb.sums : stats) + (long)(tile % STAT_REPL) * 2 * K + (long)which * K + k0 + col, v);
    }
  }
}


template <int W, int RT, int KT, bool XF>
static void launch(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const float* xf, int N, int H,
                   int C, int K, hipStream_t st, const BnBwdSums& bb) {
  const int tpi = (H + RT - 1) / RT;
  hipLaunchKernelGGL((conv3x3_kernel<W, RT, KT, XF>), dim3(N * tpi, K / KT), dim3(THREADS), 0, st, x, w, y, stats, xf,
                     H, C, K, tpi, bb);
}

template <int W, int RT, int KT>
static void launch_x(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const float* xf, int N, int H,
                     int C, int K, hipStream_t st, const BnBwdSums& bb) {
  if (xf) launch<W, RT, KT, true>(x, w, y, stats, xf, N, H, C, K, st, bb);
  else launch<W, RT, KT, false>(x, w, y, stats, xf, N, H, C, K, st, bb);
}
}  // namespace c3

// Shapes the staged-window kernel takes: 3 x 3, stride 1, pad 1, dilation 1, square 56 / 28 / 14 images (the
// stride-1 ResNet-50 3 x 3 layers and their data gradients), C and K multiples of 64 (K = 64 at 56 x 56, else a
// multiple of 128), bf16 output without bias / activation. $K8S_AMD_CONV3X3=0 keeps them on the implicit GEMM (A/B;
// read per call, both sides tested).
bool conv3x3_eligible(int H, int W, int C, int K, int R, int S, int stride, int pad, int dil) {
  const char* e = getenv("K8S_AMD_CONV3X3");
  if (e && e[0] == '0') return false;
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || dil != 1 || H != W || C % 64 != 0) return false;
  if (W == 56) return K == 64;
  return (W == 28 || W == 14) && K % 128 == 0;
}

void launch_conv3x3(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const float* xform, int N,
                    int H, int W, int C, int K, hipStream_t st, const BnBwdSums* bsums) {
  const BnBwdSums bb = bsums ? *bsums : BnBwdSums{};
  if (bb.sums && (stats || !bb.x || !bb.gamma || !bb.beta || !bb.mean || !bb.invstd))
    throw std::runtime_error("conv3x3: BatchNorm-backward sums need x / gamma / beta / mean / invstd, no statistics");
  if (W == 56 && K == 64) c3::launch_x<56, 4, 64>(x, w, y, stats, xform, N, H, C, K, st, bb);
  else if (W == 28 && K % 128 == 0) c3::launch_x<28, 8, 128>(x, w, y, stats, xform, N, H, C, K, st, bb);
  else if (W == 14 && K % 128 == 0) c3::launch_x<14, 14, 128>(x, w, y, stats, xform, N, H, C, K, st, bb);
  else throw std::runtime_error("conv3x3: shape outside the staged-window kernel's contract");
}

}  // namespace k8s_amd
