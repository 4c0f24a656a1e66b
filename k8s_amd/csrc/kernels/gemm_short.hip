// Short-K streaming GEMM: C[M][N] (bf16) = op(A)[M][K] . B^T for K in {64, 128, 256} and N % 128 == 0:
// the 1x1 convolutions of ResNet-50 as GEMMs (forward: A = the NHWC activation, B = w[Kout][C]; data gradient: A =
// dy, B = w read transposed), reference parity: the 1x1 conv2d calls of the reference's tf_cnn_benchmarks ResNet
// (SURVEY.md §2.6 K3 / BASELINE.json configs[1]).
//
// Why a separate kernel. These products move 2-8x more bytes through HBM than they take MFMA time (K = 64..256
// against M = 50k..3.2M rows), so the 128 x 128 tile kernel of gemm.hip spends each tile in load latency: one or
// two 64-deep K steps per tile, each a full HBM round trip, then the epilogue, with three blocks per CU to overlap
// them -- measured 0.3-0.45 of max(bytes / 8 TB/s, FLOP / 2.5 PF/s) on these layers (scripts/layer_roofline.py),
// and hipBLASLt is no faster there (scripts/gpurun/r4/c1x1.py). Here the operand that is small (the weights) stays
// resident and the big one streams:
//  * block = 4 waves owning one 128-wide column panel; the panel's B [128][K] is loaded once into LDS, in MFMA
//    fragment order (fragment (nb, kc) = 64 lanes x 16 B, lane-linear: conflict-free ds_read_b128);
//  * each wave walks its own 32-row tiles (persistent, grid = Cfg::OCC blocks per CU) and loads the A fragments of
//    a tile straight into VGPRs with raw buffer loads -- lane l's 16 B are row l & 15, k 8 (l >> 4) .. +7 of a
//    32-deep chunk, exactly the v_mfma_f32_16x16x32_bf16 operand, so A never touches LDS -- 1-2 tiles ahead;
//  * the 4 column panels that share rows are placed on one XCD (blockIdx % 8) and sweep the rows in step, so A
//    comes from HBM once and from that XCD's L2 for the other panels;
//  * the epilogue converts the 32 x 128 result to bf16, pairs column blocks with v_permlane16_swap (8 consecutive
//    columns per lane), passes the tile through a per-wave LDS staging area and stores it as 4 whole 256-B rows per
//    16-B store instruction; row tails past M are handled by the buffer descriptors' range checks (loads return 0,
//    stores are dropped), so there is no masking code;
//  * optional: per-column sum / sum of squares of the stored bf16 values (the BatchNorm statistics, kept in
//    registers for the whole sweep and reduced once), A normalised on load (relu(a * scale[k] + shift[k]), the
//    BatchNorm of the previous layer), and a bf16 addend -- the old C, or a second tensor with packed ReLU bits
//    (a residual gradient) -- prefetched as far ahead as the A fragments, in the copy-out layout.
// Measured (profiles/r04_gemm_short_final_ab.jsonl): 1.05-1.35x the tile kernel per ResNet-50 layer; ResNet-50 b1024
// 13.81k -> 14.15k img/s on one box.
#include <stdexcept>
#include <type_traits>
#include <utility>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {
namespace gsk {

constexpr int THREADS = 256;           // 4 waves
constexpr int BN = 128, NB = BN / 16;  // column panel of a block, 16-wide MFMA blocks
constexpr int REPL = kConvStatReplicas;

typedef __attribute__((ext_vector_type(2))) int i32x2;
typedef __attribute__((ext_vector_type(4))) int i32x4;

struct Args {
  const uint16_t* A;
  const uint16_t* B;
  uint16_t* C;
  const uint16_t* add;   // EPI 2: addend tensor [M][N]
  const uint8_t* mask;   // EPI 2: packed bits of the addend (bit j of byte e keeps element 8 e + j)
  const float* xf;       // XF: [2][K] scale | shift
  float* stats;          // STATS: [REPL][2][N]
  // EPI 3 / 4: BatchNorm-backward statistics of the stored output (see the kernel's epilogue)
  const uint16_t* bx;    // the BatchNorm's input [M][N]
  const uint16_t* bx2;   // EPI 4: the second BatchNorm's input [M][N]
  const uint8_t* bmask;  // the BatchNorm's packed ReLU bits [M][N / 8]
  const float* bmean;    // [N]
  const float* bmean2;   // EPI 4: [N]
  float* bst;            // [REPL][2][N]: sum g, sum g (x - mean)
  float* bst2;           // EPI 4: [REPL][2][N], slot 1: sum g (x2 - mean2)
  int M, N, lda, ldb;
  int P, G;              // column panels, row groups
};

// A-fragment ring depth (tiles in flight incl. the one being computed), tile rows and waves per SIMD: sized so the
// ring fits beside the accumulators, the statistics and (EPI > 0) the addend in 256 registers (2 waves per SIMD)
// EPI: 0 plain store, 1 accumulate onto C, 2 + a masked addend, 5 = 0 + the BatchNorm-backward statistics of the
// stored result (one BatchNorm: the first of two data gradients into a ResNet stage-entry input, see ops.conv),
// 3 = 2 + the BatchNorm-backward statistics of the
// stored result (one BatchNorm), 4 = 3 for two BatchNorms fed by the same masked gradient
template <int K, int EPI, bool XF, bool STATS>
struct Cfg {
  static constexpr int KC = K / 32;
  static constexpr bool HEAVY = EPI != 0 || (XF && STATS);  // the variants with the most live state
  // rows per wave tile: the heavy variants and K = 256 take 16-row tiles so they fit 2 waves per SIMD (MFMAs and
  // epilogues then overlap across the two waves; at one wave per SIMD with 32-row tiles they serialised)
  static constexpr int TM = HEAVY || K == 256 ? 16 : 32;
  static constexpr int OCC = 2;
  static constexpr int NBUF = (!HEAVY && K != 128) || (EPI != 0 && EPI < 3 && K <= 128) || (EPI == 3 && K == 64) ? 3 : 2;
};

__device__ __forceinline__ mfma_bf16x8 as_frag(i32x4 v) { return __builtin_bit_cast(mfma_bf16x8, v); }

// Vector-memory traffic: raw buffer loads / stores the compiler tracks (it places the vmcnt waits). A hand-counted
// inline-asm form was wrong: stores and loads may complete out of order with each other, so a load can only be
// waited for by draining the counter to the number of loads issued after it (what the compiler does). 16-B
// stores keep the per-tile operation count low.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void bload16(i32x4& d, uint32_t voff, const __amdgpu_buffer_rsrc_t& rs) {
  d = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, 0);
}
__device__ __forceinline__ void bstore16(const i32x4& d, uint32_t voff, const __amdgpu_buffer_rsrc_t& rs) {
  __builtin_amdgcn_raw_buffer_store_b128(d, rs, voff, 0, 0);
}

template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// relu(x * s + b) on 8 bf16, scale / shift from LDS (4 x 16 B, the same for the 16 lanes of a row group)
__device__ __forceinline__ mfma_bf16x8 xform8(i32x4 raw, const float* tab) {
  const f32x4_t s0 = *reinterpret_cast<const f32x4_t*>(tab), s1 = *reinterpret_cast<const f32x4_t*>(tab + 4);
  const f32x4_t b0 = *reinterpret_cast<const f32x4_t*>(tab + 8), b1 = *reinterpret_cast<const f32x4_t*>(tab + 12);
  float o[8];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t w = (uint32_t)raw[p];
    const f32x2_t v = {__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
    const f32x2_t s = p < 2 ? f32x2_t{s0[2 * p], s0[2 * p + 1]} : f32x2_t{s1[2 * p - 4], s1[2 * p - 3]};
    const f32x2_t b = p < 2 ? f32x2_t{b0[2 * p], b0[2 * p + 1]} : f32x2_t{b1[2 * p - 4], b1[2 * p - 3]};
    const f32x2_t y = __builtin_elementwise_max(__builtin_elementwise_fma(v, s, b), f32x2_t{0.f, 0.f});
    o[2 * p] = y[0];
    o[2 * p + 1] = y[1];
  }
  return __builtin_bit_cast(mfma_bf16x8, pack_bf16x8(o));
}

template <int K, bool BMN, bool XF, bool STATS, int EPI>
__global__ __launch_bounds__(THREADS, (Cfg<K, EPI, XF, STATS>::OCC)) void gemm_short_kernel(Args g) {
  constexpr int KC = Cfg<K, EPI, XF, STATS>::KC, NBUF = Cfg<K, EPI, XF, STATS>::NBUF;
  constexpr int TM = Cfg<K, EPI, XF, STATS>::TM, MB = TM / 16;
  constexpr int WBYTES = NB * KC * 1024;
  constexpr int XBYTES = XF ? KC * 4 * 64 : 0;
  constexpr int SBYTES = TM * 128;  // per-wave staging of half a bf16 output tile (64 columns; the copy-out)
  constexpr bool BST = EPI >= 3;
  constexpr bool ADD = EPI >= 2 && EPI <= 4;  // a masked addend
  constexpr int NS = EPI == 4 ? 3 : 2;  // BatchNorm-backward sums: g, g (x - mean) [, g (x2 - mean2)]
  constexpr int MBYTES = BST ? (NS - 1) * BN * 4 : 0;
  constexpr int STG = (WBYTES + XBYTES + MBYTES + 1023) / 1024 * 1024;
  constexpr int RBYTES = STATS ? 4 * 2 * BN * 4 : BST ? 4 * NS * BN * 4 : 0;
  constexpr int LDS = STG + 4 * SBYTES > RBYTES ? STG + 4 * SBYTES : RBYTES;
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x, xcd = bid & 7, jb = bid >> 3;
  const int panel = jb % g.P, group = xcd + 8 * (jb / g.P);
  const int n0 = panel * BN, N = g.N;

  // ---- the panel's B into LDS in fragment order: fragment f = nb * KC + kc, lane l holds
  //      B[n0 + 16 nb + (l & 15)][32 kc + 8 (l >> 4) .. +7]
  if constexpr (!BMN) {
    for (int f = wid; f < NB * KC; f += 4) {
      const int nb = f / KC, kc = f % KC;
      glds16(g.B + (long)(n0 + nb * 16 + (lane & 15)) * g.ldb + kc * 32 + (lane >> 4) * 8, smem + f * 1024);
    }
  } else {  // B stored [K][N] (the data gradient's w[Kout][C]): gathered, 8 strided bf16 per lane
    for (int c = tid; c < NB * KC * 64; c += THREADS) {
      const int f = c >> 6, l = c & 63, nb = f / KC, kc = f % KC;
      const int n = n0 + nb * 16 + (l & 15), k = kc * 32 + (l >> 4) * 8;
      bf16x8_t v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (short)g.B[(long)(k + e) * g.ldb + n];
      *reinterpret_cast<bf16x8_t*>(smem + c * 16) = v;
    }
  }
  if constexpr (XF) {  // [kc][row group q][scale 8 | shift 8]
    float* tab = reinterpret_cast<float*>(smem + WBYTES);
    for (int c = tid; c < KC * 64; c += THREADS) {
      const int kc = c >> 6, q = (c >> 4) & 3, e = c & 15;
      tab[c] = g.xf[(e >> 3) * K + kc * 32 + q * 8 + (e & 7)];
    }
  }
  float* const mtab = reinterpret_cast<float*>(smem + WBYTES + XBYTES);  // BST: [NS - 1][BN] means
  if constexpr (BST) {
    for (int c = tid; c < BN; c += THREADS) {
      mtab[c] = g.bmean[n0 + c];
      if constexpr (EPI == 4) mtab[BN + c] = g.bmean2[n0 + c];
    }
  }
  __builtin_amdgcn_s_waitcnt(0);  // the LDS DMA drained (a wait the compiler's own counter tracking sees)
  __syncthreads();

  // ---- this wave's row tiles: gw, gw + WG, gw + 2 WG, ... (tiles past M read zeros and store nothing)
  const int MT = (g.M + TM - 1) / TM, WG = g.G * 4, gw = group * 4 + wid;
  const int nt = gw < MT ? (MT - gw + WG - 1) / WG : 0;
  const __amdgpu_buffer_rsrc_t ra = rsrc(g.A, (uint32_t)((long)g.M * g.lda * 2));
  const __amdgpu_buffer_rsrc_t rc = rsrc(g.C, (uint32_t)((long)g.M * N * 2));
  const __amdgpu_buffer_rsrc_t radd = ADD ? rsrc(g.add, (uint32_t)((long)g.M * N * 2)) : rc;
  const __amdgpu_buffer_rsrc_t rmask = ADD ? rsrc(g.mask, (uint32_t)((long)g.M * N / 8)) : rc;
  const __amdgpu_buffer_rsrc_t rbx = BST ? rsrc(g.bx, (uint32_t)((long)g.M * N * 2)) : rc;
  const __amdgpu_buffer_rsrc_t rbx2 = EPI == 4 ? rsrc(g.bx2, (uint32_t)((long)g.M * N * 2)) : rc;
  const __amdgpu_buffer_rsrc_t rbm = BST ? rsrc(g.bmask, (uint32_t)((long)g.M * N / 8)) : rc;
  const int q = lane >> 4;
  const uint32_t la = (uint32_t)(((lane & 15) * g.lda + q * 8) * 2);
  const uint32_t lda16 = (uint32_t)(16 * g.lda * 2), rowA = (uint32_t)(WG * TM * g.lda * 2);
  // output / addend, in the copy-out layout: half h of the panel, row r0 + 8 k + (l >> 3), 8 columns from
  // n0 + 64 h + 8 (l & 7)
  const uint32_t lc = (uint32_t)(((lane >> 3) * N + n0 + 8 * (lane & 7)) * 2);
  const uint32_t n8 = (uint32_t)(8 * N * 2), rowC = (uint32_t)(WG * TM * N * 2);
  const uint32_t lm = (uint32_t)((((lane >> 3) * N + n0) >> 3) + (lane & 7));  // the lane's mask byte
  const uint32_t n8m = (uint32_t)N, rowM = (uint32_t)(WG * TM * N / 8);
  constexpr int NP = NB / 2, D = NBUF - 1, KO = TM / 8;  // column-block pairs; tiles ahead; copy-out rows / 8

  i32x4 abuf[NBUF][MB][KC];
  // the addend ring (EPI 1 / 2); with the BatchNorm sums (BST) the addend and its bits instead travel with x in the
  // one-slot, a-tile-ahead buffers of load_bx (registers for the second BatchNorm's operand at K >= 128)
  constexpr int AR = BST ? 1 : NBUF;
  i32x4 obuf[AR][EPI == 1 || ADD ? 2 : 1][EPI == 1 || ADD ? KO : 1];
  uint32_t mbuf[AR][ADD ? 2 : 1][ADD ? KO : 1];
  // BST: the BatchNorm input(s) and ReLU bits of the next tile, in the copy-out layout: one slot, loaded right after
  // a tile's stores (a whole tile period ahead of their use, in registers the A / addend ring does not hold)
  i32x4 xbuf[BST ? 2 : 1][BST ? KO : 1];
  i32x4 x2buf[EPI == 4 ? 2 : 1][EPI == 4 ? KO : 1];
  uint32_t bbuf[BST ? 2 : 1][BST ? KO : 1];
  auto load_a = [&](i32x4 (&dst)[MB][KC], int t) __attribute__((always_inline)) {
    const uint32_t base = (uint32_t)(gw * TM) * (uint32_t)(g.lda * 2) + (uint32_t)t * rowA + la;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) bload16(dst[mb][kc], base + mb * lda16 + kc * 64, ra);
  };
  auto load_add = [&](int slot, int t) __attribute__((always_inline)) {
    if constexpr (EPI != 0 && !BST) {
      const uint32_t base = (uint32_t)(gw * TM) * (uint32_t)(N * 2) + (uint32_t)t * rowC + lc;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < KO; ++k) bload16(obuf[slot][h][k], base + h * 128 + k * n8, EPI >= 2 ? radd : rc);
      if constexpr (ADD) {
        const uint32_t mrow = (uint32_t)(gw * TM) * (uint32_t)(N / 8) + (uint32_t)t * rowM + lm;
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int k = 0; k < KO; ++k)
            mbuf[slot][h][k] = __builtin_amdgcn_raw_buffer_load_b8(rmask, mrow + h * 8 + k * n8m, 0, 0);
      }
    }
  };
  auto load_bx = [&](int t) __attribute__((always_inline)) {
    if constexpr (BST) {
      const uint32_t base = (uint32_t)(gw * TM) * (uint32_t)(N * 2) + (uint32_t)t * rowC + lc;
      const uint32_t mrow = (uint32_t)(gw * TM) * (uint32_t)(N / 8) + (uint32_t)t * rowM + lm;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int k = 0; k < KO; ++k) {
          if constexpr (ADD) {
            bload16(obuf[0][h][k], base + h * 128 + k * n8, radd);
            mbuf[0][h][k] = __builtin_amdgcn_raw_buffer_load_b8(rmask, mrow + h * 8 + k * n8m, 0, 0);
          }
          bload16(xbuf[h][k], base + h * 128 + k * n8, rbx);
          if constexpr (EPI == 4) bload16(x2buf[h][k], base + h * 128 + k * n8, rbx2);
          bbuf[h][k] = __builtin_amdgcn_raw_buffer_load_b8(rbm, mrow + h * 8 + k * n8m, 0, 0);
        }
    }
  };

  f32x2_t s2[STATS ? NP : 1][4], q2[STATS ? NP : 1][4];
  if constexpr (STATS) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) s2[p][j] = q2[p][j] = f32x2_t{0.f, 0.f};
  }

  // BST: per lane, half h, dword j: columns 64 h + 8 (l & 7) + 2 j, + 1 -- sum g, sum g (x - mean) [, x2]
  f32x2_t bs[BST ? 2 : 1][4], bq[BST ? 2 : 1][4], bq2[EPI == 4 ? 2 : 1][4];
  if constexpr (BST) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bs[h][j] = bq[h][j] = f32x2_t{0.f, 0.f};
        if constexpr (EPI == 4) bq2[h][j] = f32x2_t{0.f, 0.f};
      }
  }

  const float* xtab = reinterpret_cast<const float*>(smem + WBYTES) + q * 16;
  // one tile; u = its ring slot (compile time)
  auto tile = [&](auto u_c, int t) __attribute__((always_inline)) {
    constexpr int u = decltype(u_c)::value;
    load_a(abuf[(u + D) % NBUF], t + D);
    load_add((u + D) % NBUF, t + D);
    // the prefetch is issued before this tile's first wait: stores may complete out of order with loads, so a
    // load is waited for by draining to the number of LOADS issued after it -- those must already be in flight
    __builtin_amdgcn_sched_barrier(0);
    f32x4_t acc[MB][NB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[mb][nb] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // weight fragments: one register set rolled across the 32-deep chunks; the scheduling barrier per chunk keeps
    // the compiler from hoisting every chunk's LDS reads to the top of the tile (KC x NB x 4 registers)
    mfma_bf16x8 wf[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) wf[nb] = *reinterpret_cast<const mfma_bf16x8*>(smem + (nb * KC * 64 + lane) * 16);
    // A operands: with XF the next chunk's normalisation is computed inside this chunk's region, so its VALU work
    // issues between this chunk's MFMAs instead of in front of the next chunk's
    mfma_bf16x8 af[MB];
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) af[mb] = XF ? xform8(abuf[u][mb][0], xtab) : as_frag(abuf[u][mb][0]);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      mfma_bf16x8 an[MB];
      if (kc + 1 < KC) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          an[mb] = XF ? xform8(abuf[u][mb][kc + 1], xtab + (kc + 1) * 64) : as_frag(abuf[u][mb][kc + 1]);
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][nb] = mfma16(wf[nb], af[mb], acc[mb][nb]);
        if (kc + 1 < KC)
          wf[nb] = *reinterpret_cast<const mfma_bf16x8*>(smem + ((nb * KC + kc + 1) * 64 + lane) * 16);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (kc + 1 < KC) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) af[mb] = an[mb];
      }
    }
    // ---- epilogue. Lane group q of column blocks (2p, 2p + 1) holds columns 32p + 4q and 32p + 16 + 4q (4 each);
    // one v_permlane16_swap per dword pair gives it the 8 consecutive columns 32p + 16 (q & 1) + 8 (q >> 1) .. +7.
    // Per 64-column half, the chunks go to this wave's staging rows (128 B, chunk XOR row: conflict-free both ways)
    // and come back row-contiguous: each 16-B store instruction then writes 8 whole 128-B row segments (straight
    // from the MFMA layout every instruction wrote 16 rows x 64 B: 1.1-1.2x slower on output-heavy shapes). The
    // statistics are taken from the same bf16 values before the round trip.
    char* stg = smem + STG + wid * SBYTES;
    const uint32_t cb = (uint32_t)(gw * TM) * (uint32_t)(N * 2) + (uint32_t)t * rowC + lc;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int r = mb * 16 + (lane & 15);
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          const int p = 2 * h + pp;
          i32x2 pa = __builtin_bit_cast(i32x2, __builtin_convertvector(acc[mb][2 * p], bf16v4_t));
          i32x2 pb = __builtin_bit_cast(i32x2, __builtin_convertvector(acc[mb][2 * p + 1], bf16v4_t));
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const auto rr = __builtin_amdgcn_permlane16_swap(pa[d], pb[d], false, false);
            pa[d] = rr[0];
            pb[d] = rr[1];
          }
          const i32x4 o = {pa[0], pa[1], pb[0], pb[1]};
          const int c = 4 * pp + 2 * (q & 1) + (q >> 1);
          *reinterpret_cast<i32x4*>(stg + r * 128 + ((c ^ (r & 7)) << 4)) = o;
          if constexpr (STATS) {
            // rows past M: A read as 0, but normalised on load that is relu(shift), not 0 -- keep them out
            const bool live = !XF || (gw + t * WG) * TM + r < g.M;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const uint32_t w = live ? (uint32_t)o[j] : 0u;
              const f32x2_t y = {__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
              s2[p][j] += y;
              q2[p][j] = __builtin_elementwise_fma(y, y, q2[p][j]);
            }
          }
        }
      }
#pragma unroll
      for (int k = 0; k < KO; ++k) {
        const int r = 8 * k + (lane >> 3), c = lane & 7;
        i32x4 o = *reinterpret_cast<const i32x4*>(stg + r * 128 + ((c ^ (r & 7)) << 4));
        if constexpr (EPI == 1 || ADD) {  // one more bf16 rounding on top of the stored product (<= 1 ulp)
          const i32x4 old = obuf[BST ? 0 : u][h][k];
          const uint32_t keep = ADD ? mbuf[BST ? 0 : u][h][k] : 0xFFu;
          float f[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t w = (uint32_t)o[j], ow = (uint32_t)old[j];
            f[2 * j] = __uint_as_float(w << 16) + (((keep >> (2 * j)) & 1u) ? __uint_as_float(ow << 16) : 0.f);
            f[2 * j + 1] = __uint_as_float(w & 0xFFFF0000u) +
                           (((keep >> (2 * j + 1)) & 1u) ? __uint_as_float(ow & 0xFFFF0000u) : 0.f);
          }
          o = __builtin_bit_cast(i32x4, pack_bf16x8(f));
        }
        if constexpr (BST) {  // g = the stored value where the BatchNorm's ReLU passed; rows past M load x = bits = 0
          const uint32_t bits = bbuf[h][k];
          const i32x4 xv = xbuf[h][k];
          const float* mt = mtab + 64 * h + 8 * (lane & 7);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t w = (uint32_t)o[j], xw = (uint32_t)xv[j];
            const f32x2_t gv = {((bits >> (2 * j)) & 1u) ? __uint_as_float(w << 16) : 0.f,
                                ((bits >> (2 * j + 1)) & 1u) ? __uint_as_float(w & 0xFFFF0000u) : 0.f};
            const f32x2_t mu = {mt[2 * j], mt[2 * j + 1]};
            const f32x2_t xd = f32x2_t{__uint_as_float(xw << 16), __uint_as_float(xw & 0xFFFF0000u)} - mu;
            bs[h][j] += gv;
            bq[h][j] = __builtin_elementwise_fma(gv, xd, bq[h][j]);
            if constexpr (EPI == 4) {
              const uint32_t x2w = (uint32_t)x2buf[h][k][j];
              const f32x2_t mu2 = {mt[BN + 2 * j], mt[BN + 2 * j + 1]};
              const f32x2_t xd2 = f32x2_t{__uint_as_float(x2w << 16), __uint_as_float(x2w & 0xFFFF0000u)} - mu2;
              bq2[h][j] = __builtin_elementwise_fma(gv, xd2, bq2[h][j]);
            }
          }
        }
        bstore16(o, cb + h * 128 + k * n8, rc);
      }
    }
    load_bx(t + 1);
  };

  // prologue: the loads of a round (A and addend of tiles 0 .. D - 1) in the loop's order; then whole
  // rounds with no branch inside (a skipped tile leaves its loads outstanding on one path, and the compiler's
  // wait state at the loop head -- the merge of all paths -- then drained the counter once per round); then the tail
  sfor<NBUF>([&](auto u) __attribute__((always_inline)) {
    constexpr int uu = decltype(u)::value;
    load_a(abuf[(uu + D) % NBUF], uu - NBUF + D);
    load_add((uu + D) % NBUF, uu - NBUF + D);
  });
  load_bx(0);
  int t0 = 0;
  for (; t0 + NBUF <= nt; t0 += NBUF) sfor<NBUF>([&](auto u) __attribute__((always_inline)) { tile(u, t0 + decltype(u)::value); });
  sfor<NBUF>([&](auto u) __attribute__((always_inline)) {
    if (t0 + decltype(u)::value < nt) tile(u, t0 + decltype(u)::value);
  });

  if constexpr (STATS) {
    // lanes with equal q hold the same columns: sum the 16 row lanes (DPP), the 4 waves through LDS, then one
    // atomic per (column, sum | square) per block into replica bid % REPL
    __syncthreads();  // every wave is past its last read of the weight panel
    float* red = reinterpret_cast<float*>(smem);  // [wave][2][BN]
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const float a = row16_sum(s2[p][j][e]), b = row16_sum(q2[p][j][e]);
          if ((lane & 15) == 0) {
            const int col = 32 * p + 16 * (q & 1) + 8 * (q >> 1) + 2 * j + e;
            red[(wid * 2 + 0) * BN + col] = a;
            red[(wid * 2 + 1) * BN + col] = b;
          }
        }
    __syncthreads();
    const int col = tid & (BN - 1), which = tid >> 7;
    const float v = red[which * BN + col] + red[(2 + which) * BN + col] + red[(4 + which) * BN + col] +
                    red[(6 + which) * BN + col];
    atomicAdd(g.stats + (long)(bid % REPL) * 2 * N + (long)which * N + n0 + col, v);
  }
  if constexpr (BST) {
    // lanes with equal l & 7 hold the same 16 columns: xor-sum over the 8 row lanes, the 4 waves through LDS, then
    // one atomic per (column, sum) per block into replica bid % REPL
    __syncthreads();  // every wave is past its last read of the weight panel and the mean table
    float* red = reinterpret_cast<float*>(smem);  // [wave][NS][BN]
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          float v[NS] = {bs[h][j][e], bq[h][j][e]};
          if constexpr (EPI == 4) v[NS - 1] = bq2[h][j][e];
#pragma unroll
          for (int s = 0; s < NS; ++s) {
            v[s] += __shfl_xor(v[s], 8);
            v[s] += __shfl_xor(v[s], 16);
            v[s] += __shfl_xor(v[s], 32);
          }
          if (lane < 8) {
            const int col = 64 * h + 8 * lane + 2 * j + e;
#pragma unroll
            for (int s = 0; s < NS; ++s) red[(wid * NS + s) * BN + col] = v[s];
          }
        }
    __syncthreads();
    for (int i = tid; i < NS * BN; i += THREADS) {
      const int col = i & (BN - 1), which = i >> 7;
      const float v = red[which * BN + col] + red[(NS + which) * BN + col] + red[(2 * NS + which) * BN + col] +
                      red[(3 * NS + which) * BN + col];
      float* dst = which < 2 ? g.bst + (long)which * N : g.bst2 + N;
      atomicAdd(dst + (long)(bid % REPL) * 2 * N + n0 + col, v);
    }
  }
}

}  // namespace gsk

// Shape contract (the caller falls back to gemm.hip otherwise): K-major A with contiguous rows of K in {64, 128,
// 256}, N % 128 == 0, bf16 C [M][N] contiguous, every operand < 2 GiB (32-bit buffer offsets). (K = 64 lost to
// gemm.hip's tile kernel while the epilogue stored straight from the MFMA layout; with the row-contiguous copy-out
// it wins on ResNet-50's 64-deep layers: bench 13.88k -> 13.93k img/s routed, scripts/gpurun/r4/gsk2.sh.)
bool gemm_short_ok(int M, int N, int K, long lda, long ldc) {
  const char* e = std::getenv("K8S_AMD_GEMM_SHORT");
  if (e && e[0] == '0') return false;
  return (K == 64 || K == 128 || K == 256) && N % 128 == 0 && lda == K && ldc == N && M > 0;
}

// Whether a masked-addend data gradient can also take the BatchNorm-backward statistics of one (dual = two) BatchNorms
// in its epilogue (K8S_AMD_BN_BSTATS=0 turns the fusion off for A/B runs).
bool gemm_short_bnstats_ok(int M, int N, int K, bool dual) {
  const char* e = std::getenv("K8S_AMD_BN_BSTATS");
  if (e && e[0] == '0') return false;
  // two BatchNorms up to K = 128 (the addend travels in the one-slot buffers; at K = 256 the second one spills)
  return gemm_short_ok(M, N, K, K, N) && (!dual || K <= 128);
}

// Rows per launch: every operand of one launch stays below 2 GiB (the kernel's 32-bit buffer offsets); larger
// products (batch >= 2048 at 56 x 56: a 3.3 GB activation) run as consecutive row ranges, the statistics epilogue
// accumulating across them. A multiple of 32 rows (whole tiles, whole mask bytes).
static int gemm_short_rows_per_launch(int M, int N, int K) {
  const long lim = (1L << 31) - (1L << 20);
  const long per_row = 2L * (N > K ? N : K);
  long rows = lim / per_row;
  if (const char* e = std::getenv("K8S_AMD_GEMM_SHORT_ROWS")) {  // tests: force the chunked path at small sizes
    const long r = std::atol(e);
    if (r >= 32 && r < rows) rows = r;
  }
  rows -= rows % 32;
  return (int)(rows < M ? rows : M);
}

// epi 0: C = op(A) B^T; 1: C += ...; 2: C = op(A) B^T + (mask ? add : 0). b_mn: B stored [K][N] (ldb) else [N][K].
void launch_gemm_short(const uint16_t* A, const uint16_t* B, long ldb, bool b_mn, uint16_t* C, const uint16_t* add,
                       const uint8_t* mask, const float* xf, float* stats, int M, int N, int K, int epi,
                       hipStream_t st, const GemmShortBnStats* bst) {
  if (!gemm_short_ok(M, N, K, K, N)) throw std::runtime_error("gemm_short: shape outside the kernel's contract");
  if ((long)K * N * 2 >= (1L << 31)) throw std::runtime_error("gemm_short: weight operand >= 2 GiB");
  const int rows = gemm_short_rows_per_launch(M, N, K);
  if (rows < M) {
    for (int r0 = 0; r0 < M; r0 += rows) {
      const int mr = M - r0 < rows ? M - r0 : rows;
      GemmShortBnStats sub;
      if (bst) {
        sub = *bst;
        sub.x += (long)r0 * N;
        if (sub.x2) sub.x2 += (long)r0 * N;
        sub.mask += (long)r0 * N / 8;
      }
      launch_gemm_short(A + (long)r0 * K, B, ldb, b_mn, C + (long)r0 * N, add ? add + (long)r0 * N : nullptr,
                        mask ? mask + (long)r0 * N / 8 : nullptr, xf, stats, mr, N, K, epi, st, bst ? &sub : nullptr);
    }
    return;
  }
  if ((epi == 2) != (add != nullptr) || (epi == 2 && !mask)) throw std::runtime_error("gemm_short: bad addend");
  if (epi != 0 && stats) throw std::runtime_error("gemm_short: statistics only with a plain store");
  if (bst && ((epi != 2 && epi != 0) || !b_mn || !bst->x || !bst->mask || !bst->mean || !bst->sums ||
              (bst->x2 && (epi != 2 || !bst->mean2 || !bst->sums2))))
    throw std::runtime_error("gemm_short: BatchNorm-backward statistics need a plain or masked-addend data gradient");
  gsk::Args g{A, B, C, add, mask, xf, stats,
              bst ? bst->x : nullptr, bst ? bst->x2 : nullptr, bst ? bst->mask : nullptr,
              bst ? bst->mean : nullptr, bst ? bst->mean2 : nullptr, bst ? bst->sums : nullptr,
              bst ? bst->sums2 : nullptr, M, N, K, (int)ldb, N / gsk::BN, 0};
  // Cfg::OCC blocks per CU; the P panels of one row group share an XCD, so blocks come in multiples of 8 P
  const int per_chip = 2 * planner_cus();  // Cfg::OCC = 2 blocks per CU
  const int gx = (per_chip / (8 * g.P)) > 1 ? per_chip / (8 * g.P) : 1;
  g.G = 8 * gx;
  const dim3 grid(8 * g.P * gx), block(gsk::THREADS);
#define K8S_GSK(KK, BM, XF, ST, EP) \
  hipLaunchKernelGGL((gsk::gemm_short_kernel<KK, BM, XF, ST, EP>), grid, block, 0, st, g)
#define K8S_GSK_K(BM, XF, ST, EP)    \
  do {                               \
    if (K == 64)                     \
      K8S_GSK(64, BM, XF, ST, EP);   \
    else if (K == 128)               \
      K8S_GSK(128, BM, XF, ST, EP);  \
    else                             \
      K8S_GSK(256, BM, XF, ST, EP);  \
  } while (0)
  if (!b_mn) {  // the convolution forward: statistics, optionally A normalised on load
    if (epi != 0) throw std::runtime_error("gemm_short: K-major B takes the plain store");
    if (xf && stats)
      K8S_GSK_K(false, true, true, 0);
    else if (xf)
      K8S_GSK_K(false, true, false, 0);
    else if (stats)
      K8S_GSK_K(false, false, true, 0);
    else
      K8S_GSK_K(false, false, false, 0);
  } else {  // the data gradient: plain, accumulating, or with a masked addend
    if (xf || stats) throw std::runtime_error("gemm_short: MN-major B takes no statistics / normalisation");
    if (epi == 0 && bst)
      K8S_GSK_K(true, false, false, 5);
    else if (epi == 0)
      K8S_GSK_K(true, false, false, 0);
    else if (epi == 1)
      K8S_GSK_K(true, false, false, 1);
    else if (bst && bst->x2) {
      // two BatchNorms' sums fit the register budget up to K = 128 (gemm_short_bnstats_ok)
      if (K == 64)
        K8S_GSK(64, true, false, false, 4);
      else if (K == 128)
        K8S_GSK(128, true, false, false, 4);
      else
        throw std::runtime_error("gemm_short: two-BatchNorm statistics need K <= 128");
    }
    else if (bst)
      K8S_GSK_K(true, false, false, 3);
    else
      K8S_GSK_K(true, false, false, 2);
  }
#undef K8S_GSK_K
#undef K8S_GSK
}

}  // namespace k8s_amd
