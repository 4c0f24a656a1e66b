// K3: NHWC BatchNorm (training statistics) fused with residual add + ReLU.
//
// Activations are [M = N*H*W, C] bf16 rows (channels_last); every pass reads / writes 16-B bf16x8 vectors.
//
//  fwd:  statistics: from the producing conv's epilogue (bn_finalize_sums) or a stats pass + final
//        -> mean, invstd, and the per-channel affine pair (scale = gamma*invstd, shift = beta - mean*scale)
//        apply  : y = relu(fma(x, scale, shift) [+ res])  (+ packed ReLU mask bits for a residual BN)
//  bwd:  reduce : sum(dy_eff), sum(dy_eff * xhat)  with dy_eff = dy * relu'(y)
//        final  : dgamma, dbeta (fp32, straight into the flat grad bucket) and the per-channel triple
//                 (sc, B, D): dx = sc*dy_eff + B*x + D
//        apply  : dx (and dres = dy_eff for a residual BN)
//
// The per-element passes (apply) are launched flat: ONE 16-B vector per thread, one 256-thread block per 4 KB
// of the tensor, no grid-stride loop. Measured on MI355X (scripts/microbench/stream_bw.hip, read-1-write-1 over
// 2 GB): that shape streams 6.25 TB/s where grid-stride loops reach 4.8-5.5 TB/s (2048-8192 blocks, 1-4 vectors
// per trip, temporal or non-temporal) -- short-lived waves dispatched in address order keep the DRAM pages hot.
// Per-thread channel parameters are therefore precomputed per channel (2-4 floats instead of 4-6 + math).
#include <cstdlib>
#include <stdexcept>

#include "common.h"
#include "launchers.h"

namespace k8s_amd {

// bn_affine_regs / bn_affine / relu_on: common.h (the 3x3 conv's BatchNorm-backward epilogue makes the same decision)

constexpr int BN_THREADS = 256;

struct BnGeom {
  int cgroups;        // C / 8
  int tpr;            // threads per row (channel groups handled per block column)
  int rows_per_iter;  // rows processed per block iteration
  int grid_y;         // channel slices
};

// Reduction geometry. Every row-block writes a [C][2] fp32 partial that the final kernel reads back, so the
// number of row-blocks is capped at M / 64 (partials <= ~6% of one pass over the data; the old fixed ~1024
// row-blocks made the partials 16% of the traffic at 7x7x2048). Parallelism lost that way is recovered by
// splitting the channels over more blocks (fewer threads per row, more rows per block iteration).
static inline BnGeom bn_geom(int C, long M) {
  BnGeom g;
  g.cgroups = C / 8;
  g.tpr = g.cgroups < BN_THREADS ? g.cgroups : BN_THREADS;
  const long cus = planner_cus();  // 4 row-blocks per CU at most, 3 per CU counted as full
  long nbx = M / 64;
  nbx = nbx < 1 ? 1 : (nbx > 4 * cus ? 4 * cus : nbx);
  for (;;) {
    g.grid_y = (g.cgroups + g.tpr - 1) / g.tpr;
    if (nbx * g.grid_y >= 3 * cus || g.tpr <= 8 || (g.tpr & 1)) break;
    g.tpr /= 2;
  }
  g.rows_per_iter = BN_THREADS / g.tpr;
  return g;
}

// Partial stats per block: part[(bx * C + c) * 2 + {0,1}] = (mean, M2) over the
// block's rows; count per block is derivable from rows_per_block.
__global__ void __launch_bounds__(BN_THREADS) bn_stats_kernel(const uint16_t* __restrict__ x, long M, int C,
                                                              int tpr, int rows_per_iter, long rows_per_block,
                                                              float* __restrict__ part) {
  __shared__ float sh[2][BN_THREADS][9];  // +1 pad
  const int t = threadIdx.x;
  const int r = t / tpr, cg_local = t % tpr;
  const int cg = blockIdx.y * tpr + cg_local;
  const bool active = (r < rows_per_iter) && (cg * 8 < C);
  const long r0 = blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  float shift[8];
  // shift by the first row of the block to avoid catastrophic cancellation
  if (active && r0 < M) {
    load8(x + r0 * C + cg * 8, shift);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) shift[j] = 0.f;
  }
  int n = 0;
  if (active) {
    long row = r0 + r;
    for (; row + 3 * rows_per_iter < r1; row += 4 * rows_per_iter) {
      float v4[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) load8(x + (row + u * rows_per_iter) * C + cg * 8, v4[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = v4[u][j] - shift[j];
          s[j] += d;
          q[j] += d * d;
        }
      n += 4;
    }
    for (; row < r1; row += rows_per_iter) {
      float v[8];
      load8(x + row * C + cg * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = v[j] - shift[j];
        s[j] += d;
        q[j] += d * d;
      }
      ++n;
    }
  }
  // per-thread (mean, M2) in shifted coordinates
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float mean = n ? s[j] / n : 0.f;
    sh[0][t][j] = mean;
    sh[1][t][j] = n ? (q[j] - s[j] * mean) : 0.f;
  }
  sh[0][t][8] = (float)n;
  __syncthreads();
  // combine rows (threads with the same cg_local) -- row 0 threads do it
  if (r == 0 && cg * 8 < C) {
    float cnt = sh[0][t][8];
    float mean[8], m2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mean[j] = sh[0][t][j]; m2[j] = sh[1][t][j]; }
    for (int rr = 1; rr < rows_per_iter; ++rr) {
      const int o = rr * tpr + cg_local;
      const float nb = sh[0][o][8];
      if (nb == 0.f) continue;
      const float tot = cnt + nb;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = sh[0][o][j] - mean[j];
        mean[j] += d * nb / tot;
        m2[j] += sh[1][o][j] + d * d * cnt * nb / tot;
      }
      cnt = tot;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long idx = ((long)blockIdx.x * C + cg * 8 + j) * 2;
      part[idx] = mean[j] + shift[j];
      part[idx + 1] = m2[j];
    }
  }
}

// Parallel finalize: a 256-thread block owns 32 channels; its 8 row groups
// Chan-combine strided subsets of the per-block partials (coalesced: 32
// consecutive channels = 256 contiguous bytes), then one LDS combine.
constexpr int FIN_CH = 32, FIN_RG = 8;

__device__ __forceinline__ void chan_merge(float& cnt, float& mean, float& m2, float nb, float bm, float bq) {
  if (nb == 0.f) return;
  const float tot = cnt + nb;
  const float d = bm - mean;
  mean += d * nb / tot;
  m2 += bq + d * d * cnt * nb / tot;
  cnt = tot;
}

__global__ void __launch_bounds__(256) bn_stats_final_kernel(const float* __restrict__ part, int nblocks, long M,
                                                             long rows_per_block, int C, float eps, float momentum,
                                                             float* __restrict__ mean_out,
                                                             float* __restrict__ invstd_out,
                                                             float* __restrict__ run_mean,
                                                             float* __restrict__ run_var,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             float* __restrict__ params) {
  __shared__ float sh[3][FIN_RG][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, rg = threadIdx.x / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  float cnt = 0.f, mean = 0.f, m2 = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int b = rg; b < nblocks; b += FIN_RG) {
      long rows = M - (long)b * rows_per_block;
      rows = rows > rows_per_block ? rows_per_block : rows;
      const float2 v = *reinterpret_cast<const float2*>(part + ((long)b * C + c) * 2);
      chan_merge(cnt, mean, m2, rows > 0 ? (float)rows : 0.f, v.x, v.y);
    }
  }
  sh[0][rg][cl] = cnt;
  sh[1][rg][cl] = mean;
  sh[2][rg][cl] = m2;
  __syncthreads();
  if (rg == 0 && c < C) {
    for (int r = 1; r < FIN_RG; ++r) chan_merge(cnt, mean, m2, sh[0][r][cl], sh[1][r][cl], sh[2][r][cl]);
    const float var = m2 / cnt;
    mean_out[c] = mean;
    invstd_out[c] = rsqrtf(var + eps);
    bn_affine(gamma[c], beta[c], mean, invstd_out[c], params + c, params + C + c);
    if (run_mean) {
      const float unbiased = cnt > 1.f ? m2 / (cnt - 1.f) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
    }
  }
}

// Statistics arrive as fp32 (sum, sum of squares) per channel, accumulated by the producing conv's
// epilogue (gemm.hip, Epi::stats): no extra pass over the activation.
__global__ void bn_finalize_sums_kernel(const float* __restrict__ sums, int nrep, int C, float count, float eps,
                                        float momentum, float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                        float* __restrict__ run_mean, float* __restrict__ run_var,
                                        const float* __restrict__ gamma, const float* __restrict__ beta,
                                        float* __restrict__ params) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, q = 0.f;
  // replicas written by the conv epilogue: all 2 x nrep loads in flight (a rolled loop waited ~32 round trips)
#pragma unroll 16
  for (int r = 0; r < nrep; ++r) {
    s += sums[(long)r * 2 * C + c];
    q += sums[(long)r * 2 * C + C + c];
  }
  const float mean = s / count;
  const float var = fmaxf(q / count - mean * mean, 0.f);
  mean_out[c] = mean;
  invstd_out[c] = rsqrtf(var + eps);
  bn_affine(gamma[c], beta[c], mean, invstd_out[c], params + c, params + C + c);
  if (run_mean) {
    const float unbiased = count > 1.f ? var * count / (count - 1.f) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
  }
}

// Packed ReLU mask: bit j of byte e = (bf16(y[8e + j]) > 0). A residual BN's backward reads these M*C/8 bytes
// instead of the bf16 output y (2 B/elem) in both its reduce and apply passes. A bf16 is > 0 iff its int16 bit
// pattern is > 0 (NaN aside).
__device__ __forceinline__ uint8_t relu_bits(const bf16x8_t& o) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) b |= (o[j] > 0 ? 1u : 0u) << j;
  return (uint8_t)b;
}

__device__ __forceinline__ void load_f8(const float* p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// Block -> 4-KB chunk order of the flat passes (see stream_order_mode below). rev 0: address order. rev 1 / 2: the tensor as
// 8 contiguous bands swept concurrently (consecutive blocks in different bands), each descending (1) or ascending
// (2) -- the shape in which the XCD-remapped GEMMs write their outputs (8 row bands in parallel, ascending); rev 3:
// plain descending address order.
__device__ __forceinline__ int bn_block_order(int b, int nb, int rev) {
  if (!rev) return b;
  if (rev == 3) return nb - 1 - b;  // plain descending
  const int band = b & 7, q = nb >> 3, r = nb & 7;
  const int size = q + (band < r ? 1 : 0);
  const int start = band < r ? band * (q + 1) : r * (q + 1) + (band - r) * q;
  const int local = b >> 3;
  return rev == 1 ? start + size - 1 - local : start + local;
}

// y = act(fma(x, scale, shift) [+ res]); params = [scale | shift] (fp32 [2][C]). One vector per thread.
// rparams: the residual is itself a BatchNorm input (a ResNet downsample branch) -- res is normalised here with its own
// [scale | shift] instead of by a separate apply pass that writes and re-reads the normalised tensor.
__global__ void __launch_bounds__(BN_THREADS) bn_apply_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ res,
                                                              const float* __restrict__ params,
                                                              const float* __restrict__ rparams,
                                                              uint16_t* __restrict__ y, uint8_t* __restrict__ mask,
                                                              int nvec, int C, FastDiv fcg, int relu, int rev,
                                                              uint16_t* __restrict__ ysub, FastDiv fW, FastDiv fH) {
  const int e = bn_block_order(blockIdx.x, gridDim.x, rev) * BN_THREADS + threadIdx.x;
  if (e >= nvec) return;
  const int cgroups = C >> 3;
  const int c0 = (e - fcg.div(e) * cgroups) * 8;
  const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + (long)e * 8);
  bf16x8_t rv;
  if (res) rv = *reinterpret_cast<const bf16x8_t*>(res + (long)e * 8);
  float sc[8], sh[8], v[8];
  load_f8(params + c0, sc);
  load_f8(params + C + c0, sh);
  if (rparams) {
    float rsc[8], rsh[8];
    load_f8(rparams + c0, rsc);
    load_f8(rparams + C + c0, rsh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float o = __builtin_fmaf(bf2f((uint16_t)xv[j]), sc[j], sh[j]) +
                      __builtin_fmaf(bf2f((uint16_t)rv[j]), rsc[j], rsh[j]);
      v[j] = relu ? fmaxf(o, 0.f) : o;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = __builtin_fmaf(bf2f((uint16_t)xv[j]), sc[j], sh[j]);
      if (res) o += bf2f((uint16_t)rv[j]);
      v[j] = relu ? fmaxf(o, 0.f) : o;
    }
  }
  const bf16x8_t ov = pack_bf16x8(v);
  *reinterpret_cast<bf16x8_t*>(y + (long)e * 8) = ov;
  if (mask) mask[e] = relu_bits(ov);
  if (ysub) {  // the stride-2 subsample of y (the next block's downsample-convolution input) written in the same pass
    const int pix = fcg.div(e), r = fW.div(pix), w = pix - r * (int)fW.d, n = fH.div(r), h = r - n * (int)fH.d;
    if (((h | w) & 1) == 0) {
      const int Ho = ((int)fH.d + 1) >> 1, Wo = ((int)fW.d + 1) >> 1;
      const long q = (((long)n * Ho + (h >> 1)) * Wo + (w >> 1)) * cgroups + (e - pix * cgroups);
      *reinterpret_cast<bf16x8_t*>(ysub + q * 8) = ov;
    }
  }
}

// Eval mode: the affine pair from the running statistics.
__global__ void bn_eval_prep_kernel(const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                    const float* __restrict__ gamma, const float* __restrict__ beta, int C, float eps,
                                    float* __restrict__ mean, float* __restrict__ invstd,
                                    float* __restrict__ params) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = run_mean[c];
  invstd[c] = rsqrtf(run_var[c] + eps);
  bn_affine(gamma[c], beta[c], mean[c], invstd[c], params + c, params + C + c);
}

// Backward reduce: part[(bx*C + c)*2] = sum dy_eff, [+1] = sum dy_eff * xhat.
// Rows are visited grid-stride (block bx takes row groups bx, bx + G, ... of rows_per_iter rows each): the
// blocks resident at any time then sweep one narrow window of the tensors front to back, which streams at
// 5.5-5.7 TB/s on MI355X against ~4.9 for one long contiguous run per block (scripts/microbench/stream_bw.hip).
// (Round 3 tried a flat variant -- short-lived blocks over 8 x 256-vector contiguous chunks, 6.0-6.3 TB/s in
// scripts/microbench/read_bw.hip -- with per-block partials and a parallel fold: 85.8 vs 81.7 ms per ResNet-50
// step, the fold of tens of thousands of partials plus the extra launches eating the bandwidth gain; with
// same-address atomics into 32 replicas instead, 88.1 vs 82.2. Not kept.)
// MASK: the ReLU mask comes from the packed bit mask (a separate instantiation, so the relu_x variant keeps its
// register budget and occupancy).
// DUAL (with MASK): a second BatchNorm input x2 (mean2 / invstd2) fed by the same masked dy -- the ResNet downsample
// block's bn3 and downsample BN after their fused forward -- reduced in the same sweep (dy and the mask read once);
// part2 gets (sum dy_eff, sum dy_eff * xhat2).
template <bool MASK, bool DUAL = false>
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy,
                                                                   const uint16_t* __restrict__ x,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ invstd,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta, int relu_x, long M,
                                                                   int C, int tpr, int rows_per_iter,
                                                                   float* __restrict__ part,
                                                                   const uint8_t* __restrict__ mask, int rev,
                                                                   const uint16_t* __restrict__ x2 = nullptr,
                                                                   const float* __restrict__ mean2 = nullptr,
                                                                   const float* __restrict__ invstd2 = nullptr,
                                                                   float* __restrict__ part2 = nullptr) {
  __shared__ float sh[DUAL ? 3 : 2][BN_THREADS][9];
  const int t = threadIdx.x;
  const int r = t / tpr, cg_local = t % tpr;
  const int cg = blockIdx.y * tpr + cg_local;
  const bool active = (r < rows_per_iter) && (cg * 8 < C);
  float sd[8], sx[8], mu[8], is[8], sc[8], bt[8];
  float sx2[DUAL ? 8 : 1], mu2[DUAL ? 8 : 1], is2[DUAL ? 8 : 1];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sd[j] = sx[j] = 0.f;
    mu[j] = active ? mean[cg * 8 + j] : 0.f;
    is[j] = active ? invstd[cg * 8 + j] : 0.f;
    sc[j] = 0.f;
    bt[j] = 0.f;
    if (active && relu_x) bn_affine_regs(gamma[cg * 8 + j], beta[cg * 8 + j], mu[j], is[j], sc[j], bt[j]);
    if constexpr (DUAL) {
      sx2[j] = 0.f;
      mu2[j] = active ? mean2[cg * 8 + j] : 0.f;
      is2[j] = active ? invstd2[cg * 8 + j] : 0.f;
    }
  }
  auto one = [&](const bf16x8_t& gv, const bf16x8_t& xw, uint32_t bits) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float xv = bf2f((uint16_t)xw[j]);
      bool on = (bits >> j) & 1u;
      if (!MASK && relu_x) on = relu_on(xv, sc[j], bt[j]);
      const float g = on ? bf2f((uint16_t)gv[j]) : 0.f;
      sd[j] += g;
      sx[j] += g * (xv - mu[j]) * is[j];
    }
  };
  auto two = [&](const bf16x8_t& gv, const bf16x8_t& xw, uint32_t bits) {  // DUAL: the second input's term
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (DUAL) {
        const float g = ((bits >> j) & 1u) ? bf2f((uint16_t)gv[j]) : 0.f;
        sx2[j] += g * (bf2f((uint16_t)xw[j]) - mu2[j]) * is2[j];
      }
    }
  };
  // rev: the rows as 8 bands (block bx sweeps band bx & 7), each visited descending -- the reverse of the
  // producing GEMM's write order (bn_block_order)
  long M_ = M, base = 0, nblk = gridDim.x, bx = blockIdx.x;
  if (rev) {
    const long bandlen = (M + 7) / 8, band = bx & 7;
    base = band * bandlen;
    M_ = M - base < bandlen ? M - base : bandlen;
    if (M_ < 0) M_ = 0;
    nblk = gridDim.x / 8;
    bx = bx >> 3;
  }
  const long stride = nblk * rows_per_iter;
  if (active) {
    long row = bx * rows_per_iter + r;
    // 4 row groups per trip: every 16-B load (and mask byte) of the trip is issued before any is used
    for (; row + 3 * stride < M_; row += 4 * stride) {
      bf16x8_t g4[4], x4[4], y4[DUAL ? 4 : 1];
      uint32_t b4[4] = {0xFFu, 0xFFu, 0xFFu, 0xFFu};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rw = row + u * stride;
        const long off = (rev ? base + M_ - 1 - rw : rw) * C + cg * 8;
        g4[u] = *reinterpret_cast<const bf16x8_t*>(dy + off);
        x4[u] = *reinterpret_cast<const bf16x8_t*>(x + off);
        if constexpr (DUAL) y4[u] = *reinterpret_cast<const bf16x8_t*>(x2 + off);
        if constexpr (MASK) b4[u] = mask[off >> 3];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        one(g4[u], x4[u], b4[u]);
        if constexpr (DUAL) two(g4[u], y4[u], b4[u]);
      }
    }
    for (; row < M_; row += stride) {
      const long off = (rev ? base + M_ - 1 - row : row) * C + cg * 8;
      const bf16x8_t gv = *reinterpret_cast<const bf16x8_t*>(dy + off);
      const uint32_t bits = MASK ? (uint32_t)mask[off >> 3] : 0xFFu;
      one(gv, *reinterpret_cast<const bf16x8_t*>(x + off), bits);
      if constexpr (DUAL) two(gv, *reinterpret_cast<const bf16x8_t*>(x2 + off), bits);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][t][j] = sd[j];
    sh[1][t][j] = sx[j];
    if constexpr (DUAL) sh[DUAL ? 2 : 0][t][j] = sx2[j];
  }
  __syncthreads();
  if (r == 0 && cg * 8 < C) {
    for (int rr = 1; rr < rows_per_iter; ++rr) {
      const int o = rr * tpr + cg_local;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += sh[0][o][j];
        sx[j] += sh[1][o][j];
        if constexpr (DUAL) sx2[j] += sh[DUAL ? 2 : 0][o][j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long idx = ((long)blockIdx.x * C + cg * 8 + j) * 2;
      part[idx] = sd[j];
      part[idx + 1] = sx[j];
      if constexpr (DUAL) {
        part2[idx] = sd[j];
        part2[idx + 1] = sx2[j];
      }
    }
  }
}

// Backward per-channel constants from the two reductions (sum dy_eff, sum dy_eff*xhat), M rows:
//   params = [sc | B | D | shift]:  dx = sc*dy_eff + B*x + D,  shift = the forward's affine shift (relu_x)
__device__ __forceinline__ void bn_bwd_consts(int c, int C, float s_dy, float s_dyxh, float inv_m,
                                              const float* __restrict__ mean, const float* __restrict__ invstd,
                                              const float* __restrict__ gamma, const float* __restrict__ beta,
                                              float* __restrict__ params) {
  float sc, shift;
  bn_affine_regs(gamma[c], beta ? beta[c] : 0.f, mean[c], invstd[c], sc, shift);
  const float k1 = s_dy * inv_m, k2 = s_dyxh * inv_m;  // mean(dy_eff), mean(dy_eff * xhat)
  const float B = -sc * invstd[c] * k2;
  params[c] = sc;
  params[C + c] = B;
  params[2 * C + c] = -sc * k1 - B * mean[c];
  params[3 * C + c] = shift;
}

__global__ void __launch_bounds__(256) bn_bwd_final_kernel(const float* __restrict__ part, int nblocks, int C,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float inv_m, const float* __restrict__ mean,
                                                           const float* __restrict__ invstd,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           float* __restrict__ params) {
  __shared__ float sh[2][FIN_RG][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, rg = threadIdx.x / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  float a = 0.f, b2 = 0.f;
  if (c < C) {
#pragma unroll 16
    for (int i = rg; i < nblocks; i += FIN_RG) {
      const float2 v = *reinterpret_cast<const float2*>(part + ((long)i * C + c) * 2);
      a += v.x;
      b2 += v.y;
    }
  }
  sh[0][rg][cl] = a;
  sh[1][rg][cl] = b2;
  __syncthreads();
  if (rg == 0 && c < C) {
    for (int r = 1; r < FIN_RG; ++r) {
      a += sh[0][r][cl];
      b2 += sh[1][r][cl];
    }
    if (dbeta) dbeta[c] = a;
    if (dgamma) dgamma[c] = b2;
    bn_bwd_consts(c, C, a, b2, inv_m, mean, invstd, gamma, beta, params);
  }
}

// bn_bwd_final_kernel for sums accumulated by a data-gradient epilogue (gemm_short.hip EPI 3 / 4): replicas
// [nrep][2][C], slot 0 of `sg` = sum g, slot 1 of `sd` = sum g (x - mean) (dual: the second BatchNorm's sums share g)
__global__ void __launch_bounds__(256) bn_bwd_final_sums_kernel(const float* __restrict__ sg,
                                                                const float* __restrict__ sd, int nrep, int C,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                float inv_m, const float* __restrict__ mean,
                                                                const float* __restrict__ invstd,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta,
                                                                float* __restrict__ params) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
#pragma unroll 16
  for (int r = 0; r < nrep; ++r) {
    a += sg[(long)r * 2 * C + c];
    b += sd[(long)r * 2 * C + C + c];
  }
  b *= invstd[c];
  if (dbeta) dbeta[c] = a;
  if (dgamma) dgamma[c] = b;
  bn_bwd_consts(c, C, a, b, inv_m, mean, invstd, gamma, beta, params);
}

// dx = sc*dy_eff + B*x + D; dres = dy_eff. dy_eff = dy masked by the packed bits (residual BN), by relu_on(x)
// (non-residual BN + ReLU) or not at all. One vector per thread (see the header).
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                                  const uint16_t* __restrict__ x,
                                                                  const uint8_t* __restrict__ mask,
                                                                  const float* __restrict__ params, int relu_x,
                                                                  uint16_t* __restrict__ dx,
                                                                  uint16_t* __restrict__ dres, int nvec, int C,
                                                                  FastDiv fcg, int rev) {
  const int e = bn_block_order(blockIdx.x, gridDim.x, rev) * BN_THREADS + threadIdx.x;
  if (e >= nvec) return;
  const int cgroups = C >> 3;
  const int c0 = (e - fcg.div(e) * cgroups) * 8;
  const bf16x8_t gv = *reinterpret_cast<const bf16x8_t*>(dy + (long)e * 8);
  const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + (long)e * 8);
  const uint32_t bits = mask ? (uint32_t)mask[e] : 0xFFu;
  float sc[8], B[8], D[8], g[8], o[8];
  load_f8(params + c0, sc);
  load_f8(params + C + c0, B);
  load_f8(params + 2 * C + c0, D);
  float sh[8];
  if (relu_x) load_f8(params + 3 * C + c0, sh);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float xf = bf2f((uint16_t)xv[j]);
    bool on = (bits >> j) & 1u;
    if (relu_x) on = relu_on(xf, sc[j], sh[j]);
    g[j] = on ? bf2f((uint16_t)gv[j]) : 0.f;
    o[j] = __builtin_fmaf(sc[j], g[j], __builtin_fmaf(B[j], xf, D[j]));
  }
  if (dres) *reinterpret_cast<bf16x8_t*>(dres + (long)e * 8) = pack_bf16x8(g);
  *reinterpret_cast<bf16x8_t*>(dx + (long)e * 8) = pack_bf16x8(o);
}

// Both BatchNorm backwards of a fused downsample-block forward (bn_apply_kernel with rparams): one masked dy, two
// inputs, two gradients; dy and the mask read once.
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_apply_dual_kernel(
    const uint16_t* __restrict__ dy, const uint8_t* __restrict__ mask, const uint16_t* __restrict__ x,
    const float* __restrict__ params, uint16_t* __restrict__ dx, const uint16_t* __restrict__ x2,
    const float* __restrict__ params2, uint16_t* __restrict__ dx2, int nvec, int C, FastDiv fcg, int rev) {
  const int e = bn_block_order(blockIdx.x, gridDim.x, rev) * BN_THREADS + threadIdx.x;
  if (e >= nvec) return;
  const int c0 = (e - fcg.div(e) * (C >> 3)) * 8;
  const bf16x8_t gv = *reinterpret_cast<const bf16x8_t*>(dy + (long)e * 8);
  const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + (long)e * 8);
  const bf16x8_t yv = *reinterpret_cast<const bf16x8_t*>(x2 + (long)e * 8);
  const uint32_t bits = mask[e];
  float g[8], o[8];
  {
    float sc[8], B[8], D[8];
    load_f8(params + c0, sc);
    load_f8(params + C + c0, B);
    load_f8(params + 2 * C + c0, D);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = ((bits >> j) & 1u) ? bf2f((uint16_t)gv[j]) : 0.f;
      o[j] = __builtin_fmaf(sc[j], g[j], __builtin_fmaf(B[j], bf2f((uint16_t)xv[j]), D[j]));
    }
    *reinterpret_cast<bf16x8_t*>(dx + (long)e * 8) = pack_bf16x8(o);
  }
  float sc[8], B[8], D[8];
  load_f8(params2 + c0, sc);
  load_f8(params2 + C + c0, B);
  load_f8(params2 + 2 * C + c0, D);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = __builtin_fmaf(sc[j], g[j], __builtin_fmaf(B[j], bf2f((uint16_t)yv[j]), D[j]));
  *reinterpret_cast<bf16x8_t*>(dx2 + (long)e * 8) = pack_bf16x8(o);
}


// ---------------------------------------------------------------- stem: BatchNorm + ReLU + 3x3 / s2 / p1 max pool
// The ResNet stem's bn1 -> ReLU -> max pool as one pass each way, so the 112 x 112 x 64 BN output is never stored:
//  forward : each thread owns 8 channels of one pooled pixel, normalises its 9 window taps on load
//            (z = bf16(relu(fma(x, scale, shift))), bit-identical to bn_apply_kernel's output) and keeps the max
//            and the winner's window position (uint8, as maxpool_fwd_k_kernel; ties -> first tap)
//  backward: the max-pool gradient of an input pixel (sum of dy over the covering windows whose winner it is)
//            is GATHERED inside the BatchNorm backward's reduce and apply passes, by 2 x 2 input cells (the four
//            windows covering a cell are loaded once for its 4 pixels, as maxpool_bwd_3s2_kernel), rounded to bf16
//            as the stored gradient would be, and masked by the ReLU recomputed from x.
// HBM bytes per step at ResNet-50 b1024 (x = 1.64 GB): forward 1 read of x + the pooled write instead of read x,
// write z, read z; backward 2 reads of x + the dx write instead of writing dz and reading it twice with x.
__global__ void __launch_bounds__(BN_THREADS) bn_relu_maxpool_fwd_kernel(
    const uint16_t* __restrict__ x, const float* __restrict__ params, uint16_t* __restrict__ y,
    uint8_t* __restrict__ idx, int H, int W, int C, int Ho, int Wo, int total, FastDiv fcv, FastDiv fWo, FastDiv fHo,
    uint16_t* __restrict__ xarg, uint8_t* __restrict__ ybits) {
  const int e = blockIdx.x * BN_THREADS + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  const int t = fcv.div(e);
  const int c = (e - t * cv) * 8;
  const int t2 = fWo.div(t);
  const int wo = t - t2 * Wo;
  const int n = fHo.div(t2);
  const int ho = t2 - n * Ho;
  const int h0 = 2 * ho - 1, w0 = 2 * wo - 1;
  float sc[8], sh[8];
  load_f8(params + c, sc);
  load_f8(params + C + c, sh);
  bf16x8_t v[9];
#pragma unroll
  for (int dh = 0; dh < 3; ++dh)
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      const int h = min(max(h0 + dh, 0), H - 1), w = min(max(w0 + dw, 0), W - 1);
      v[dh * 3 + dw] = *reinterpret_cast<const bf16x8_t*>(x + (((long)n * H + h) * W + w) * C + c);
    }
  float best[8];
  uint32_t arg[8];
  bf16x8_t bx = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};  // the winner's x (xarg)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    best[j] = -INFINITY;
    arg[j] = 255;
  }
#pragma unroll
  for (int dh = 0; dh < 3; ++dh)
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      if ((unsigned)(h0 + dh) >= (unsigned)H || (unsigned)(w0 + dw) >= (unsigned)W) continue;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float z = bf2f(f2bf(fmaxf(__builtin_fmaf(bf2f((uint16_t)v[dh * 3 + dw][j]), sc[j], sh[j]), 0.f)));
        if (z > best[j] || (z != z && best[j] == best[j])) {
          best[j] = z;
          arg[j] = (uint32_t)(dh * 3 + dw);
          bx[j] = v[dh * 3 + dw][j];
        }
      }
    }
  store8(y + (long)e * 8, best);
  uint64_t packed = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) packed |= (uint64_t)arg[j] << (8 * j);
  *reinterpret_cast<uint64_t*>(idx + (long)e * 8) = packed;
  // for the BatchNorm-backward sums in the consuming data gradients' epilogues (nn.BnStatLink): per pooled element
  // the winner's x and whether its ReLU passed (y > 0) -- g = bit ? dpool : 0 routes to exactly that x
  if (xarg) {
    *reinterpret_cast<bf16x8_t*>(xarg + (long)e * 8) = bx;
    uint32_t bits = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) bits |= (best[j] > 0.f ? 1u : 0u) << j;
    ybits[e] = (uint8_t)bits;
  }
}

// dz of the 4 pixels of input cell (n, kc, jc), channels c .. c+7: the max-pool gradient (bf16-rounded)
struct PoolCell {
  float dz[2][2][8];
};
__device__ __forceinline__ void pool_cell_grad(const uint16_t* __restrict__ dpool, const uint8_t* __restrict__ idx,
                                               int n, int kc, int jc, int c, int C, int Ho, int Wo, PoolCell& pc) {
  uint64_t pk[2][2];
  float g[2][2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const bool ok = kc + a < Ho && jc + b < Wo;
      const long o = (((long)n * Ho + (ok ? kc + a : kc)) * Wo + (ok ? jc + b : jc)) * C + c;
      pk[a][b] = ok ? *reinterpret_cast<const uint64_t*>(idx + o) : ~0ull;  // 0xff matches no position
      load8(dpool + o, g[a][b]);
    }
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      float acc[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) acc[r] = 0.f;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          // pixel (2kc + dh, 2jc + dw) lies in window (kc + a, jc + b) iff its offset there is in 0..2
          const int oh = dh - 2 * a + 1, ow = dw - 2 * b + 1;
          if (oh < 0 || oh > 2 || ow < 0 || ow > 2) continue;  // compile-time after unrolling
          const uint32_t pos = (uint32_t)(oh * 3 + ow);
#pragma unroll
          for (int r = 0; r < 8; ++r)
            if (((pk[a][b] >> (8 * r)) & 0xff) == pos) acc[r] += g[a][b][r];
        }
#pragma unroll
      for (int r = 0; r < 8; ++r) pc.dz[dh][dw][r] = bf2f(f2bf(acc[r]));
    }
}

// Backward reduce over input cells: part[(bx * C + c) * 2 + {0, 1}] = sum dz_eff, sum dz_eff * xhat (the layout of
// bn_bwd_reduce_kernel, finished by bn_bwd_final_kernel). Block = (256 / cv) cells x cv channel groups, cell-strided.
__global__ void __launch_bounds__(BN_THREADS) pool_bn_bwd_reduce_kernel(
    const uint16_t* __restrict__ dpool, const uint8_t* __restrict__ idx, const uint16_t* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int H, int W, int C, int Ho, int Wo, int Hc, int Wc, int ncells,
    float* __restrict__ part, FastDiv fWc, FastDiv fHc) {
  __shared__ float sh[2][BN_THREADS][9];
  const int t = threadIdx.x, cv = C >> 3;
  const int cg = t % cv, cl = t / cv, cpb = BN_THREADS / cv;
  const int c = cg * 8;
  float sd[8], sx[8], mu[8], is[8], sc[8], bt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sd[j] = sx[j] = 0.f;
    mu[j] = mean[c + j];
    is[j] = invstd[c + j];
    bn_affine_regs(gamma[c + j], beta[c + j], mu[j], is[j], sc[j], bt[j]);
  }
  for (int cell = blockIdx.x * cpb + cl; cell < ncells; cell += gridDim.x * cpb) {
    const int r2 = fWc.div(cell), jc = cell - r2 * Wc, n = fHc.div(r2), kc = r2 - n * Hc;
    PoolCell pc;
    pool_cell_grad(dpool, idx, n, kc, jc, c, C, Ho, Wo, pc);
#pragma unroll
    for (int dh = 0; dh < 2; ++dh)
#pragma unroll
      for (int dw = 0; dw < 2; ++dw) {
        const int h = 2 * kc + dh, w = 2 * jc + dw;
        if (h >= H || w >= W) continue;
        const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + (((long)n * H + h) * W + w) * C + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xf = bf2f((uint16_t)xv[j]);
          const float g = relu_on(xf, sc[j], bt[j]) ? pc.dz[dh][dw][j] : 0.f;
          sd[j] += g;
          sx[j] += g * (xf - mu[j]) * is[j];
        }
      }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][t][j] = sd[j];
    sh[1][t][j] = sx[j];
  }
  __syncthreads();
  if (cl == 0) {
    for (int rr = 1; rr < cpb; ++rr) {
      const int o = rr * cv + cg;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += sh[0][o][j];
        sx[j] += sh[1][o][j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long i = ((long)blockIdx.x * C + c + j) * 2;
      part[i] = sd[j];
      part[i + 1] = sx[j];
    }
  }
}

// dx = sc * dz_eff + B * x + D for the 4 pixels of one cell, 8 channels per thread (params = [sc | B | D | shift])
__global__ void __launch_bounds__(BN_THREADS) pool_bn_bwd_apply_kernel(
    const uint16_t* __restrict__ dpool, const uint8_t* __restrict__ idx, const uint16_t* __restrict__ x,
    const float* __restrict__ params, uint16_t* __restrict__ dx, int H, int W, int C, int Ho, int Wo, int total,
    FastDiv fcv, FastDiv fWc, FastDiv fHc) {
  const int e = blockIdx.x * BN_THREADS + threadIdx.x;
  if (e >= total) return;
  const int cv = C >> 3;
  const int t = fcv.div(e);
  const int c = (e - t * cv) * 8;
  const int t2 = fWc.div(t);
  const int jc = t - t2 * (int)fWc.d;
  const int n = fHc.div(t2);
  const int kc = t2 - n * (int)fHc.d;
  PoolCell pc;
  pool_cell_grad(dpool, idx, n, kc, jc, c, C, Ho, Wo, pc);
  float sc[8], B[8], D[8], shf[8];
  load_f8(params + c, sc);
  load_f8(params + C + c, B);
  load_f8(params + 2 * C + c, D);
  load_f8(params + 3 * C + c, shf);
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw) {
      const int h = 2 * kc + dh, w = 2 * jc + dw;
      if (h >= H || w >= W) continue;
      const long o = (((long)n * H + h) * W + w) * C + c;
      const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + o);
      float r[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xf = bf2f((uint16_t)xv[j]);
        const float g = relu_on(xf, sc[j], shf[j]) ? pc.dz[dh][dw][j] : 0.f;
        r[j] = __builtin_fmaf(sc[j], g, __builtin_fmaf(B[j], xf, D[j]));
      }
      store8(dx + o, r);
    }
}

// ---------------------------------------------------------------- launchers
// Traversal order of the streaming passes, chosen so that each pass starts where its producer stopped: the bytes
// the producer touched last are still in the 256 MiB Infinity Cache (a line stays resident while it plus every
// byte streamed since its last use fits, MI355X_MICROARCH.md "Infinity Cache"). The XCD-remapped GEMMs write their
// outputs as 8 row bands in parallel, each ascending; so the passes sweep 8 bands concurrently too
// (bn_block_order), in the direction opposite to their producer's.
// Measured (ResNet-50 b1024, scripts/gpurun/env_ab.sh, round 3): 12.36-12.38k img/s in plain address order,
// 12.61-12.64k with these fixed BatchNorm directions (forward apply descending behind its ascending conv, backward
// reduce descending behind its dgrad, backward apply ascending behind the reduce), 12.51-12.53k when every streaming
// launch, the GEMMs included, alternated direction (the GEMMs' reversed tile order costs more than the reuse buys).
int stream_order_mode() { return 1; }
int stream_dir(int fixed) { return fixed; }

static long bn_rows_per_block(long M, const BnGeom& g) {
  // ~1024 blocks in total (4 per CU: enough loads in flight to cover HBM latency), at most M / 64 row-blocks,
  // >= 4 row trips per block
  long blocks_x = 4L * planner_cus() / g.grid_y;
  const long cap = M / 64;
  if (blocks_x > cap) blocks_x = cap;
  if (blocks_x < 1) blocks_x = 1;
  long rpb = (M + blocks_x - 1) / blocks_x;
  long minr = (long)g.rows_per_iter * 4;
  if (rpb < minr) rpb = minr;
  rpb = (rpb + g.rows_per_iter - 1) / g.rows_per_iter * g.rows_per_iter;
  return rpb;
}

// grid-stride reduction blocks along the rows: ~1024 in total (4 per CU)
static int bn_reduce_blocks(long M, const BnGeom& g) {
  long nb = 4L * planner_cus() / g.grid_y;
  const long groups = (M + g.rows_per_iter - 1) / g.rows_per_iter;
  if (nb > groups) nb = groups;
  if (stream_order_mode()) nb = nb < 8 ? 8 : nb & ~7L;  // banded order: a multiple of 8 blocks (one band each)
  return (int)(nb < 1 ? 1 : nb);
}

int bn_workspace_floats(long M, int C) {
  BnGeom g = bn_geom(C, M);
  long rpb = bn_rows_per_block(M, g);
  long nb = (M + rpb - 1) / rpb;  // forward statistics pass
  const long nr = bn_reduce_blocks(M, g);
  return (int)((nb > nr ? nb : nr) * C * 2);
}

static void launch_bn_apply(const uint16_t* x, const uint16_t* res, const float* params, uint16_t* y, uint8_t* mask,
                            long M, int C, bool relu, hipStream_t st, const float* rparams = nullptr,
                            uint16_t* ysub = nullptr, int H = 1, int W = 1) {
  const long nvec = M * C / 8;
  if (nvec >= (1L << 31)) throw std::runtime_error("BatchNorm tensor too large (>= 2^31 vectors)");
  if (ysub && (M % ((long)H * W) != 0)) throw std::runtime_error("bn_apply subsample: M must be N * H * W");
  hipLaunchKernelGGL(bn_apply_kernel, dim3(cdiv(nvec, BN_THREADS)), dim3(BN_THREADS), 0, st, x, res, params, rparams,
                     y, mask, (int)nvec, C, make_fastdiv(C / 8), (int)relu,
                     stream_order_mode() ? (stream_dir(1) ? 1 : 2) : 0, ysub, make_fastdiv(W), make_fastdiv(H));
}

void launch_bn_fwd(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta, uint16_t* y,
                   float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* work, float* params,
                   long M, int C, float eps, float momentum, bool training, bool relu, hipStream_t st,
                   uint8_t* mask) {
  if (training) {
    BnGeom g = bn_geom(C, M);
    long rpb = bn_rows_per_block(M, g);
    int nb = (int)((M + rpb - 1) / rpb);
    hipLaunchKernelGGL(bn_stats_kernel, dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, x, M, C, g.tpr,
                       g.rows_per_iter, rpb, work);
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work, nb, M, rpb, C, eps,
                       momentum, save_mean, save_invstd, run_mean, run_var, gamma, beta, params);
  } else {
    hipLaunchKernelGGL(bn_eval_prep_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, run_mean, run_var, gamma, beta, C,
                       eps, save_mean, save_invstd, params);
  }
  launch_bn_apply(x, res, params, y, mask, M, C, relu, st);
}

void launch_bn_fwd_from_sums(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                             uint16_t* y, const float* sums, int nrep, float* save_mean, float* save_invstd,
                             float* run_mean, float* run_var, float* params, long M, int C, float eps, float momentum,
                             bool relu, hipStream_t st, uint8_t* mask, uint16_t* ysub, int H, int W) {
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, nrep, C, (float)M, eps,
                     momentum, save_mean, save_invstd, run_mean, run_var, gamma, beta, params);
  launch_bn_apply(x, res, params, y, mask, M, C, relu, st, nullptr, ysub, H, W);
}

// y = relu(BN(x) + BN_r(xr)), both BatchNorms' statistics from their convs' epilogue sums (a ResNet downsample
// block's bn3 and downsample BN): the downsample BN's output is never written (it was stored by its own apply pass
// and read back once by bn3's). mask = the packed ReLU mask of y.
void launch_bn_fwd_from_sums_dual(const uint16_t* x, const float* gamma, const float* beta, const float* sums,
                                  int nrep, float* save_mean, float* save_invstd, float* run_mean, float* run_var,
                                  float* params, const uint16_t* xr, const float* gamma_r, const float* beta_r,
                                  const float* sums_r, int nrep_r, float* save_mean_r, float* save_invstd_r,
                                  float* run_mean_r, float* run_var_r, float* params_r, uint16_t* y, uint8_t* mask,
                                  long M, int C, float eps, float momentum, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, nrep, C, (float)M, eps,
                     momentum, save_mean, save_invstd, run_mean, run_var, gamma, beta, params);
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums_r, nrep_r, C, (float)M, eps,
                     momentum, save_mean_r, save_invstd_r, run_mean_r, run_var_r, gamma_r, beta_r, params_r);
  launch_bn_apply(x, xr, params, y, mask, M, C, true, st, params_r);
}

// Statistics finalize only (mean, invstd, running stats, [scale | shift]): the apply happens in the consuming
// convolution's operand load (gemm.hip XForm, normalize on load).
void launch_bn_finalize_sums(const float* gamma, const float* beta, const float* sums, int nrep, float* save_mean,
                             float* save_invstd, float* run_mean, float* run_var, float* params, long M, int C,
                             float eps, float momentum, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, nrep, C, (float)M, eps,
                     momentum, save_mean, save_invstd, run_mean, run_var, gamma, beta, params);
}

static void launch_bn_bwd_apply(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* params,
                                bool relu_x, uint16_t* dx, uint16_t* dres, long M, int C, hipStream_t st,
                                int order = -1) {
  const long nvec = M * C / 8;
  if (nvec >= (1L << 31)) throw std::runtime_error("BatchNorm tensor too large (>= 2^31 vectors)");
  if (order < 0) order = stream_order_mode() ? (stream_dir(0) ? 1 : 2) : 0;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(cdiv(nvec, BN_THREADS)), dim3(BN_THREADS), 0, st, dy, x, mask, params,
                     (int)relu_x, dx, dres, (int)nvec, C, make_fastdiv(C / 8), order);
}

void launch_bn_bwd(const uint16_t* dy, const uint16_t* x, const float* mean, const float* invstd, const float* gamma,
                   const float* beta, bool relu_x, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta,
                   float* work, float* params, long M, int C, hipStream_t st, const uint8_t* mask) {
  BnGeom g = bn_geom(C, M);
  const int nb = bn_reduce_blocks(M, g);
  // (round 3: the residual-BN reduce in address order, and its apply descending behind it, measured slower than
  // the producer-opposite banded order -- 12.92k vs 13.06k img/s -- and were dropped)
  const int rdir = stream_dir(1);
  if (mask)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, dy, x, mean, invstd,
                       gamma, beta, (int)relu_x, M, C, g.tpr, g.rows_per_iter, work, mask, rdir);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, dy, x, mean, invstd,
                       gamma, beta, (int)relu_x, M, C, g.tpr, g.rows_per_iter, work, mask, rdir);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work, nb, C, dgamma, dbeta,
                     1.f / (float)M, mean, invstd, gamma, beta, params);
  launch_bn_bwd_apply(dy, x, mask, params, relu_x, dx, dres, M, C, st);
}

// launch_bn_bwd with the reduce done by dy's producer (the sums of bn_bwd_final_sums_kernel): the final and apply
// passes only. mask: the packed ReLU bits (residual BatchNorm).
void launch_bn_bwd_from_sums(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* sums, int nrep,
                             const float* mean, const float* invstd, const float* gamma, const float* beta,
                             uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, float* params, long M, int C,
                             hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_final_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, sums, nrep, C, dgamma,
                     dbeta, 1.f / (float)M, mean, invstd, gamma, beta, params);
  launch_bn_bwd_apply(dy, x, mask, params, false, dx, dres, M, C, st);
}

void launch_bn_bwd_relu_from_sums(const uint16_t* dy, const uint16_t* x, const float* sums, int nrep,
                                  const float* mean, const float* invstd, const float* gamma, const float* beta,
                                  uint16_t* dx, float* dgamma, float* dbeta, float* params, long M, int C,
                                  hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_final_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, sums, nrep, C, dgamma,
                     dbeta, 1.f / (float)M, mean, invstd, gamma, beta, params);
  launch_bn_bwd_apply(dy, x, nullptr, params, true, dx, nullptr, M, C, st);
}

void launch_bn_bwd_dual_from_sums(const uint16_t* dy, const uint8_t* mask, const uint16_t* x, const float* sums,
                                  int nrep, const float* mean, const float* invstd, const float* gamma,
                                  const float* beta, uint16_t* dx, float* dgamma, float* dbeta, float* params,
                                  const uint16_t* x2, const float* sums2, const float* mean2, const float* invstd2,
                                  const float* gamma2, const float* beta2, uint16_t* dx2, float* dgamma2,
                                  float* dbeta2, float* params2, long M, int C, hipStream_t st) {
  hipLaunchKernelGGL(bn_bwd_final_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, sums, nrep, C, dgamma,
                     dbeta, 1.f / (float)M, mean, invstd, gamma, beta, params);
  hipLaunchKernelGGL(bn_bwd_final_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, sums2, nrep, C, dgamma2,
                     dbeta2, 1.f / (float)M, mean2, invstd2, gamma2, beta2, params2);
  const long nvec = M * C / 8;
  if (nvec >= (1L << 31)) throw std::runtime_error("BatchNorm tensor too large (>= 2^31 vectors)");
  hipLaunchKernelGGL(bn_bwd_apply_dual_kernel, dim3(cdiv(nvec, BN_THREADS)), dim3(BN_THREADS), 0, st, dy, mask, x,
                     params, dx, x2, params2, dx2, (int)nvec, C, make_fastdiv(C / 8),
                     stream_order_mode() ? (stream_dir(0) ? 1 : 2) : 0);
}

// Backward of launch_bn_fwd_from_sums_dual: both BatchNorms' (dgamma, dbeta, dx) from one masked dy in one reduce
// sweep and one apply pass (work / work2: bn_workspace_floats each; params / params2: fp32 [4][C] each).
void launch_bn_bwd_dual(const uint16_t* dy, const uint8_t* mask, const uint16_t* x, const float* mean,
                        const float* invstd, const float* gamma, const float* beta, uint16_t* dx, float* dgamma,
                        float* dbeta, float* work, float* params, const uint16_t* x2, const float* mean2,
                        const float* invstd2, const float* gamma2, const float* beta2, uint16_t* dx2, float* dgamma2,
                        float* dbeta2, float* work2, float* params2, long M, int C, hipStream_t st) {
  BnGeom g = bn_geom(C, M);
  const int nb = bn_reduce_blocks(M, g);
  const int rdir = stream_dir(1);
  hipLaunchKernelGGL((bn_bwd_reduce_kernel<true, true>), dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, dy, x, mean,
                     invstd, gamma, beta, 0, M, C, g.tpr, g.rows_per_iter, work, mask, rdir, x2, mean2, invstd2, work2);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work, nb, C, dgamma, dbeta,
                     1.f / (float)M, mean, invstd, gamma, beta, params);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work2, nb, C, dgamma2, dbeta2,
                     1.f / (float)M, mean2, invstd2, gamma2, beta2, params2);
  const long nvec = M * C / 8;
  if (nvec >= (1L << 31)) throw std::runtime_error("BatchNorm tensor too large (>= 2^31 vectors)");
  hipLaunchKernelGGL(bn_bwd_apply_dual_kernel, dim3(cdiv(nvec, BN_THREADS)), dim3(BN_THREADS), 0, st, dy, mask, x,
                     params, dx, x2, params2, dx2, (int)nvec, C, make_fastdiv(C / 8),
                     stream_order_mode() ? (stream_dir(0) ? 1 : 2) : 0);
}

// ---- stem BatchNorm + ReLU + 3x3 / s2 / p1 max pool (see bn_relu_maxpool_fwd_kernel)
void launch_bn_relu_maxpool_fwd(const uint16_t* x, const float* gamma, const float* beta, const float* sums, int nrep,
                                float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* params,
                                uint16_t* y, uint8_t* idx, int N, int H, int W, int C, float eps, float momentum,
                                hipStream_t st, uint16_t* xarg, uint8_t* ybits) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;  // (H + 2 - 3) / 2 + 1
  const long total = (long)N * Ho * Wo * (C / 8);
  if ((long)N * H * W * C / 8 >= (1L << 31)) throw std::runtime_error("bn_relu_maxpool: tensor too large");
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, nrep, C,
                     (float)((long)N * H * W), eps, momentum, save_mean, save_invstd, run_mean, run_var, gamma, beta,
                     params);
  hipLaunchKernelGGL(bn_relu_maxpool_fwd_kernel, dim3(cdiv(total, BN_THREADS)), dim3(BN_THREADS), 0, st, x, params,
                     y, idx, H, W, C, Ho, Wo, (int)total, make_fastdiv(C / 8), make_fastdiv(Wo), make_fastdiv(Ho),
                     xarg, ybits);
}

int pool_bn_workspace_floats(int C) { return 4096 * C * 2; }

void launch_pool_bn_bwd(const uint16_t* dpool, const uint8_t* idx, const uint16_t* x, const float* mean,
                        const float* invstd, const float* gamma, const float* beta, uint16_t* dx, float* dgamma,
                        float* dbeta, float* work, float* params, int N, int H, int W, int C, hipStream_t st) {
  if (C % 8 || BN_THREADS % (C / 8)) throw std::runtime_error("pool_bn_bwd: C / 8 must divide 256");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const long ncells = (long)N * Hc * Wc;
  if (ncells * (C / 8) >= (1L << 31)) throw std::runtime_error("pool_bn_bwd: tensor too large");
  const int cpb = BN_THREADS / (C / 8);
  long nb = (ncells + cpb - 1) / cpb;
  nb = std::min(nb, 16L * planner_cus());  // ~16 blocks per CU: enough loads in flight (a 1024-block grid ran at half the roof)
  hipLaunchKernelGGL(pool_bn_bwd_reduce_kernel, dim3((unsigned)nb), dim3(BN_THREADS), 0, st, dpool, idx, x, mean,
                     invstd, gamma, beta, H, W, C, Ho, Wo, Hc, Wc, (int)ncells, work, make_fastdiv(Wc),
                     make_fastdiv(Hc));
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work, (int)nb, C, dgamma, dbeta,
                     1.f / (float)((long)N * H * W), mean, invstd, gamma, beta, params);
  const long total = ncells * (C / 8);
  hipLaunchKernelGGL(pool_bn_bwd_apply_kernel, dim3(cdiv(total, BN_THREADS)), dim3(BN_THREADS), 0, st, dpool, idx, x,
                     params, dx, H, W, C, Ho, Wo, (int)total, make_fastdiv(C / 8), make_fastdiv(Wc),
                     make_fastdiv(Hc));
}

// launch_pool_bn_bwd with the sums taken by the data gradients into the pooled output (the winner's x and ReLU bit
// per pooled element, bn_relu_maxpool_fwd_kernel's xarg / ybits): the final and apply passes only
void launch_pool_bn_bwd_from_sums(const uint16_t* dpool, const uint8_t* idx, const uint16_t* x, const float* mean,
                                  const float* invstd, const float* gamma, const float* beta, uint16_t* dx,
                                  float* dgamma, float* dbeta, const float* sums, int nrep, float* params, int N,
                                  int H, int W, int C, hipStream_t st) {
  if (C % 8 || BN_THREADS % (C / 8)) throw std::runtime_error("pool_bn_bwd: C / 8 must divide 256");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2, Hc = (H + 1) / 2, Wc = (W + 1) / 2;
  const long ncells = (long)N * Hc * Wc;
  if (ncells * (C / 8) >= (1L << 31)) throw std::runtime_error("pool_bn_bwd: tensor too large");
  hipLaunchKernelGGL(bn_bwd_final_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, sums, nrep, C, dgamma,
                     dbeta, 1.f / (float)((long)N * H * W), mean, invstd, gamma, beta, params);
  const long total = ncells * (C / 8);
  hipLaunchKernelGGL(pool_bn_bwd_apply_kernel, dim3(cdiv(total, BN_THREADS)), dim3(BN_THREADS), 0, st, dpool, idx, x,
                     params, dx, H, W, C, Ho, Wo, (int)total, make_fastdiv(C / 8), make_fastdiv(Wc),
                     make_fastdiv(Hc));
}

__global__ void __launch_bounds__(BN_THREADS) relu_mask_kernel(const uint16_t* __restrict__ y,
                                                               uint8_t* __restrict__ mask, int nvec) {
  const int e = blockIdx.x * BN_THREADS + threadIdx.x;
  if (e < nvec) mask[e] = relu_bits(*reinterpret_cast<const bf16x8_t*>(y + (long)e * 8));
}

void launch_relu_mask(const uint16_t* y, uint8_t* mask, long nvec, hipStream_t st) {
  if (nvec >= (1L << 31)) throw std::runtime_error("tensor too large (>= 2^31 vectors)");
  hipLaunchKernelGGL(relu_mask_kernel, dim3(cdiv(nvec, BN_THREADS)), dim3(BN_THREADS), 0, st, y, mask, (int)nvec);
}

// out = bit ? src : 0: a residual gradient handed over as (dy, ReLU mask) materialised for a consumer whose
// epilogue cannot read the pair itself (GEMM Epi::addmask covers the 1x1 identity-block dgrad)
__global__ void __launch_bounds__(BN_THREADS) mask_apply_kernel(const uint16_t* __restrict__ src,
                                                                const uint8_t* __restrict__ mask,
                                                                uint16_t* __restrict__ out, int nvec) {
  const int e = blockIdx.x * BN_THREADS + threadIdx.x;
  if (e >= nvec) return;
  bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(src + (long)e * 8);
  const uint32_t bits = mask[e];
#pragma unroll
  for (int r = 0; r < 8; ++r) v[r] = ((bits >> r) & 1u) ? v[r] : (short)0;
  *reinterpret_cast<bf16x8_t*>(out + (long)e * 8) = v;
}

void launch_mask_apply(const uint16_t* src, const uint8_t* mask, uint16_t* out, long n, hipStream_t st) {
  if (n % 8) throw std::runtime_error("mask_apply: element count must be a multiple of 8");
  const long nvec = n / 8;
  if (nvec >= (1L << 31)) throw std::runtime_error("tensor too large (>= 2^31 vectors)");
  hipLaunchKernelGGL(mask_apply_kernel, dim3(cdiv(nvec, BN_THREADS)), dim3(BN_THREADS), 0, st, src, mask, out,
                     (int)nvec);
}

}  // namespace k8s_amd
