// K3: NHWC BatchNorm (training statistics) fused with residual add + ReLU.
//
// Activations are [M = N*H*W, C] bf16 rows (channels_last). Every kernel
// reads/writes 16-B bf16x8 vectors; a thread owns 8 consecutive channels.
//
//  fwd:  stats  : per-block Welford/Chan partials (count-weighted mean, M2)
//        final  : combine partials -> mean, invstd; update running stats
//        apply  : y = relu(x*scale + shift [+ res])    (scale/shift per channel)
//  bwd:  reduce : sum(dy_eff), sum(dy_eff * xhat)  with dy_eff = dy * (y > 0)
//        final  : dgamma, dbeta (fp32, written straight into the flat grad bucket)
//        apply  : dx = gamma*invstd*(dy_eff - sum_dy/M - xhat*sum_dyxh/M), dres = dy_eff
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace k8s_amd {

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
  long nbx = M / 64;
  nbx = nbx < 1 ? 1 : (nbx > 1024 ? 1024 : nbx);
  for (;;) {
    g.grid_y = (g.cgroups + g.tpr - 1) / g.tpr;
    if (nbx * g.grid_y >= 768 || g.tpr <= 8 || (g.tpr & 1)) break;
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
                                                             float* __restrict__ run_var) {
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
                                        float* __restrict__ run_mean, float* __restrict__ run_var) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f, q = 0.f;
  for (int r = 0; r < nrep; ++r) {  // replicas written by the conv epilogue
    s += sums[(long)r * 2 * C + c];
    q += sums[(long)r * 2 * C + C + c];
  }
  const float mean = s / count;
  const float var = fmaxf(q / count - mean * mean, 0.f);
  mean_out[c] = mean;
  invstd_out[c] = rsqrtf(var + eps);
  if (run_mean) {
    const float unbiased = count > 1.f ? var * count / (count - 1.f) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
  }
}

// Packed ReLU mask: bit j of byte e = (bf16(y[8e + j]) > 0). A residual BN's backward reads these M*C/8 bytes
// instead of the bf16 output y (2 B/elem) in both its reduce and apply passes.
__device__ __forceinline__ uint8_t relu_bits(const float (&v)[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) b |= (bf2f(f2bf(v[j])) > 0.f ? 1u : 0u) << j;
  return (uint8_t)b;
}

// y = act((x - mean) * (gamma * invstd) + beta [+ res]).
// The grid is sized so (gridDim.x * blockDim.x) % cgroups == 0: every thread then keeps ONE channel group
// for the whole grid-stride loop and holds its 8 channels' parameters in registers. U vectors per trip: all
// U (or 2U with a residual) 16-B loads are issued before the first is used, so each wave keeps several HBM
// requests in flight instead of one load -> use -> store chain per trip.
template <int U>
__global__ void __launch_bounds__(BN_THREADS) bn_apply_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ res,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ invstd,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta,
                                                              uint16_t* __restrict__ y, uint8_t* __restrict__ mask,
                                                              long nvec, int cgroups, int relu) {
  const long e0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const int cg = (int)(e0 % cgroups);
  float mu[8], sc[8], bt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    mu[j] = mean[c];
    sc[j] = gamma[c] * invstd[c];
    bt[j] = beta[c];
  }
  long e = e0;
  for (; e + (U - 1) * stride < nvec; e += U * stride) {
    bf16x8_t xv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = *reinterpret_cast<const bf16x8_t*>(x + (e + u * stride) * 8);
    if (res) {
#pragma unroll
      for (int u = 0; u < U; ++u) rv[u] = *reinterpret_cast<const bf16x8_t*>(res + (e + u * stride) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float o = (bf2f((uint16_t)xv[u][j]) - mu[j]) * sc[j] + bt[j];
        if (res) o += bf2f((uint16_t)rv[u][j]);
        if (relu) o = fmaxf(o, 0.f);
        v[j] = o;
      }
      store8(y + (e + u * stride) * 8, v);
      if (mask) mask[e + u * stride] = relu_bits(v);
    }
  }
  for (; e < nvec; e += stride) {
    float v[8];
    load8(x + e * 8, v);
    float rv[8];
    if (res) load8(res + e * 8, rv);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float o = (v[j] - mu[j]) * sc[j] + bt[j];
      if (res) o += rv[j];
      if (relu) o = fmaxf(o, 0.f);
      v[j] = o;
    }
    store8(y + e * 8, v);
    if (mask) mask[e] = relu_bits(v);
  }
}

// Eval-mode: same apply with running stats (mean/invstd precomputed on host side kernel below).
__global__ void bn_eval_prep_kernel(const float* __restrict__ run_mean, const float* __restrict__ run_var, int C,
                                    float eps, float* __restrict__ mean, float* __restrict__ invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = run_mean[c];
  invstd[c] = rsqrtf(run_var[c] + eps);
}

// Backward reduce: part[(bx*C + c)*2] = sum dy_eff, [+1] = sum dy_eff * xhat
// MASK: the ReLU mask comes from the packed bit mask (a separate instantiation, so the y / relu_x variant keeps
// its register budget and occupancy).
template <bool MASK>
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_reduce_kernel(const uint16_t* __restrict__ dy,
                                                                   const uint16_t* __restrict__ x,
                                                                   const uint16_t* __restrict__ y,
                                                                   const float* __restrict__ mean,
                                                                   const float* __restrict__ invstd,
                                                                   const float* __restrict__ gamma,
                                                                   const float* __restrict__ beta, int relu_x, long M,
                                                                   int C, int tpr, int rows_per_iter,
                                                                   long rows_per_block, float* __restrict__ part,
                                                                   const uint8_t* __restrict__ mask) {
  __shared__ float sh[2][BN_THREADS][9];
  const int t = threadIdx.x;
  const int r = t / tpr, cg_local = t % tpr;
  const int cg = blockIdx.y * tpr + cg_local;
  const bool active = (r < rows_per_iter) && (cg * 8 < C);
  const long r0 = blockIdx.x * rows_per_block;
  long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float sd[8], sx[8], mu[8], is[8], sc[8], bt[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sd[j] = sx[j] = 0.f;
    mu[j] = active ? mean[cg * 8 + j] : 0.f;
    is[j] = active ? invstd[cg * 8 + j] : 0.f;
    sc[j] = (active && relu_x) ? gamma[cg * 8 + j] * is[j] : 0.f;
    bt[j] = (active && relu_x) ? beta[cg * 8 + j] : 0.f;
  }
  if (active) {
    // 4 rows per trip: 8-12 independent 16-B loads in flight per thread before any is used
    long row = r0 + r;
    for (; row + 3 * rows_per_iter < r1; row += 4 * rows_per_iter) {
      float g4[4][8], x4[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long off = (row + u * rows_per_iter) * C + cg * 8;
        load8(dy + off, g4[u]);
        load8(x + off, x4[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float* g = g4[u];
        const float* xv = x4[u];
        if constexpr (MASK) {
          const uint32_t bits = mask[((row + u * rows_per_iter) * C + cg * 8) >> 3];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (!((bits >> j) & 1u)) g[j] = 0.f;
        } else if (y) {
          bf16x8_t yv = *reinterpret_cast<const bf16x8_t*>(y + (row + u * rows_per_iter) * C + cg * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (bf2f((uint16_t)yv[j]) <= 0.f) g[j] = 0.f;
        } else if (relu_x) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (bf2f(f2bf((xv[j] - mu[j]) * sc[j] + bt[j])) <= 0.f) g[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sd[j] += g[j];
          sx[j] += g[j] * (xv[j] - mu[j]) * is[j];
        }
      }
    }
    for (; row < r1; row += rows_per_iter) {
      const long off = row * C + cg * 8;
      float g[8], xv[8];
      load8(dy + off, g);
      load8(x + off, xv);
      if constexpr (MASK) {
        const uint32_t bits = mask[off >> 3];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (!((bits >> j) & 1u)) g[j] = 0.f;
      } else if (y) {
        bf16x8_t yv = *reinterpret_cast<const bf16x8_t*>(y + off);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (bf2f((uint16_t)yv[j]) <= 0.f) g[j] = 0.f;
      } else if (relu_x) {  // ReLU mask recomputed from x: no read of y (non-residual BN)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (bf2f(f2bf((xv[j] - mu[j]) * sc[j] + bt[j])) <= 0.f) g[j] = 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += g[j];
        sx[j] += g[j] * (xv[j] - mu[j]) * is[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][t][j] = sd[j];
    sh[1][t][j] = sx[j];
  }
  __syncthreads();
  if (r == 0 && cg * 8 < C) {
    for (int rr = 1; rr < rows_per_iter; ++rr) {
      const int o = rr * tpr + cg_local;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sd[j] += sh[0][o][j];
        sx[j] += sh[1][o][j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const long idx = ((long)blockIdx.x * C + cg * 8 + j) * 2;
      part[idx] = sd[j];
      part[idx + 1] = sx[j];
    }
  }
}

__global__ void __launch_bounds__(256) bn_bwd_final_kernel(const float* __restrict__ part, int nblocks, int C,
                                                           float* __restrict__ sums, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta) {
  __shared__ float sh[2][FIN_RG][FIN_CH];
  const int cl = threadIdx.x % FIN_CH, rg = threadIdx.x / FIN_CH;
  const int c = blockIdx.x * FIN_CH + cl;
  float a = 0.f, b2 = 0.f;
  if (c < C) {
#pragma unroll 4
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
    sums[c] = a;
    sums[C + c] = b2;
    if (dbeta) dbeta[c] = a;
    if (dgamma) dgamma[c] = b2;
  }
}

// dx = gamma*invstd*(dy_eff - mean(dy_eff) - xhat*mean(dy_eff*xhat)); dres = dy_eff. U vectors per trip
// with every load of the trip issued up front (see bn_apply_kernel).
template <int U>
__global__ void __launch_bounds__(BN_THREADS) bn_bwd_apply_kernel(const uint16_t* __restrict__ dy,
                                                                  const uint16_t* __restrict__ x,
                                                                  const uint16_t* __restrict__ y,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ invstd,
                                                                  const float* __restrict__ beta, int relu_x,
                                                                  const float* __restrict__ gamma,
                                                                  const float* __restrict__ sums,
                                                                  uint16_t* __restrict__ dx,
                                                                  uint16_t* __restrict__ dres, long nvec,
                                                                  int cgroups, int C, float inv_m,
                                                                  const uint8_t* __restrict__ mask) {
  const long e0 = blockIdx.x * (long)blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  const int cg = (int)(e0 % cgroups);  // fixed per thread: grid sized so (grid*block) % cgroups == 0
  float mu[8], is[8], sc[8], bt[8], k1[8], k2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    mu[j] = mean[c];
    is[j] = invstd[c];
    sc[j] = gamma[c] * is[j];
    bt[j] = beta ? beta[c] : 0.f;
    k1[j] = sums[c] * inv_m;      // mean(dy_eff)
    k2[j] = sums[C + c] * inv_m;  // mean(dy_eff * xhat)
  }
  // B = -gamma*invstd^2*mean(dy_eff*xhat), D = -gamma*invstd*mean(dy_eff) - B*mean: dx = sc*g + B*x + D
  float B[8], D[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    B[j] = -sc[j] * is[j] * k2[j];
    D[j] = -sc[j] * k1[j] - B[j] * mu[j];
  }
  auto one = [&](bf16x8_t gv, bf16x8_t xvv, bool has_y, bf16x8_t yv, long e) {
    float g[8], xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = bf2f((uint16_t)gv[j]);
      xv[j] = bf2f((uint16_t)xvv[j]);
    }
    if (mask) {
      const uint32_t bits = mask[e];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (!((bits >> j) & 1u)) g[j] = 0.f;
    } else if (has_y) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (bf2f((uint16_t)yv[j]) <= 0.f) g[j] = 0.f;
    } else if (relu_x) {  // ReLU mask recomputed from x: no read of y (non-residual BN)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (bf2f(f2bf((xv[j] - mu[j]) * sc[j] + bt[j])) <= 0.f) g[j] = 0.f;
    }
    if (dres) store8(dres + e * 8, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = sc[j] * g[j] + B[j] * xv[j] + D[j];
    store8(dx + e * 8, xv);
  };
  long e = e0;
  for (; e + (U - 1) * stride < nvec; e += U * stride) {
    bf16x8_t gv[U], xv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) yv[u] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      gv[u] = *reinterpret_cast<const bf16x8_t*>(dy + (e + u * stride) * 8);
      xv[u] = *reinterpret_cast<const bf16x8_t*>(x + (e + u * stride) * 8);
    }
    if (y) {
#pragma unroll
      for (int u = 0; u < U; ++u) yv[u] = *reinterpret_cast<const bf16x8_t*>(y + (e + u * stride) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(gv[u], xv[u], y != nullptr, yv[u], e + u * stride);
  }
  for (; e < nvec; e += stride) {
    const bf16x8_t gv = *reinterpret_cast<const bf16x8_t*>(dy + e * 8);
    const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(x + e * 8);
    bf16x8_t yv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (y) yv = *reinterpret_cast<const bf16x8_t*>(y + e * 8);
    one(gv, xv, y != nullptr, yv, e);
  }
}

// Loads per trip for the per-element BN kernels. $K8S_AMD_BN_UNROLL (1, 2 or 4) exists for A/B runs; the
// default stays 1: on the ResNet-50 b512 shapes one 16-B load per trip already streams 4.4-5.3 TB/s and 2 or 4
// per trip measured 0-12 % slower (lower occupancy), ResNet-50 8151 / 8097 / 8028 img/s for U = 1 / 2 / 4
// (profiles/r01_bn_unroll_ab.md).
static int bn_unroll() {
  static int u = [] {
    const char* s = getenv("K8S_AMD_BN_UNROLL");
    const int v = s ? atoi(s) : 1;
    return (v == 2 || v == 4) ? v : 1;
  }();
  return u;
}

static void launch_bn_apply(const uint16_t* x, const uint16_t* res, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, uint16_t* y, uint8_t* mask, long nvec,
                            int cgroups, int relu, hipStream_t st);
static void launch_bn_bwd_apply(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean,
                                const float* invstd, const float* beta, int relu_x, const float* gamma,
                                const float* sums, uint16_t* dx, uint16_t* dres, long nvec, int cgroups, int C,
                                float inv_m, const uint8_t* mask, hipStream_t st);

// ---------------------------------------------------------------- launchers
static long bn_rows_per_block(long M, const BnGeom& g) {
  // ~1024 blocks in total (4 per CU: enough loads in flight to cover HBM latency), at most M / 64 row-blocks,
  // >= 4 row trips per block
  long blocks_x = 1024 / g.grid_y;
  const long cap = M / 64;
  if (blocks_x > cap) blocks_x = cap;
  if (blocks_x < 1) blocks_x = 1;
  long rpb = (M + blocks_x - 1) / blocks_x;
  long minr = (long)g.rows_per_iter * 4;
  if (rpb < minr) rpb = minr;
  rpb = (rpb + g.rows_per_iter - 1) / g.rows_per_iter * g.rows_per_iter;
  return rpb;
}

// grid for the per-element kernels: (grid * BN_THREADS) % cgroups == 0 keeps each thread on one channel group
static int bn_elem_grid(long nvec, int cgroups) {
  int g = stream_grid(nvec, BN_THREADS);
  if ((BN_THREADS % cgroups) != 0) {
    // cgroups does not divide the block: round the grid up to a multiple of cgroups / gcd(cgroups, BN_THREADS)
    int a = cgroups, b = BN_THREADS;
    while (b) { int t = a % b; a = b; b = t; }
    const int step = cgroups / a;
    g = (g + step - 1) / step * step;
  }
  return g;
}

static void launch_bn_apply(const uint16_t* x, const uint16_t* res, const float* mean, const float* invstd,
                            const float* gamma, const float* beta, uint16_t* y, uint8_t* mask, long nvec,
                            int cgroups, int relu, hipStream_t st) {
  const dim3 grid(bn_elem_grid(nvec, cgroups)), block(BN_THREADS);
  switch (bn_unroll()) {
    case 4:
      hipLaunchKernelGGL(bn_apply_kernel<4>, grid, block, 0, st, x, res, mean, invstd, gamma, beta, y, mask, nvec,
                         cgroups, relu);
      break;
    case 2:
      hipLaunchKernelGGL(bn_apply_kernel<2>, grid, block, 0, st, x, res, mean, invstd, gamma, beta, y, mask, nvec,
                         cgroups, relu);
      break;
    default:
      hipLaunchKernelGGL(bn_apply_kernel<1>, grid, block, 0, st, x, res, mean, invstd, gamma, beta, y, mask, nvec,
                         cgroups, relu);
  }
}

static void launch_bn_bwd_apply(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean,
                                const float* invstd, const float* beta, int relu_x, const float* gamma,
                                const float* sums, uint16_t* dx, uint16_t* dres, long nvec, int cgroups, int C,
                                float inv_m, const uint8_t* mask, hipStream_t st) {
  const dim3 grid(bn_elem_grid(nvec, cgroups)), block(BN_THREADS);
  switch (bn_unroll()) {
    case 4:
      hipLaunchKernelGGL(bn_bwd_apply_kernel<4>, grid, block, 0, st, dy, x, y, mean, invstd, beta, relu_x, gamma,
                         sums, dx, dres, nvec, cgroups, C, inv_m, mask);
      break;
    case 2:
      hipLaunchKernelGGL(bn_bwd_apply_kernel<2>, grid, block, 0, st, dy, x, y, mean, invstd, beta, relu_x, gamma,
                         sums, dx, dres, nvec, cgroups, C, inv_m, mask);
      break;
    default:
      hipLaunchKernelGGL(bn_bwd_apply_kernel<1>, grid, block, 0, st, dy, x, y, mean, invstd, beta, relu_x, gamma,
                         sums, dx, dres, nvec, cgroups, C, inv_m, mask);
  }
}

int bn_workspace_floats(long M, int C) {
  BnGeom g = bn_geom(C, M);
  long rpb = bn_rows_per_block(M, g);
  long nb = (M + rpb - 1) / rpb;
  return (int)(nb * C * 2);
}

void launch_bn_fwd(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta, uint16_t* y,
                   float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* work, long M, int C,
                   float eps, float momentum, bool training, bool relu, hipStream_t st, uint8_t* mask) {
  if (training) {
    BnGeom g = bn_geom(C, M);
    long rpb = bn_rows_per_block(M, g);
    int nb = (int)((M + rpb - 1) / rpb);
    hipLaunchKernelGGL(bn_stats_kernel, dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, x, M, C, g.tpr,
                       g.rows_per_iter, rpb, work);
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work, nb, M, rpb, C, eps,
                       momentum, save_mean, save_invstd, run_mean, run_var);
  } else {
    hipLaunchKernelGGL(bn_eval_prep_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, run_mean, run_var, C, eps,
                       save_mean, save_invstd);
  }
  const long nvec = M * C / 8;
  launch_bn_apply(x, res, save_mean, save_invstd, gamma, beta, y, mask, nvec, C / 8, (int)relu, st);
}

void launch_bn_fwd_from_sums(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                             uint16_t* y, const float* sums, int nrep, float* save_mean, float* save_invstd,
                             float* run_mean, float* run_var, long M, int C, float eps, float momentum, bool relu,
                             hipStream_t st, uint8_t* mask) {
  hipLaunchKernelGGL(bn_finalize_sums_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, sums, nrep, C, (float)M, eps,
                     momentum, save_mean, save_invstd, run_mean, run_var);
  const long nvec = M * C / 8;
  launch_bn_apply(x, res, save_mean, save_invstd, gamma, beta, y, mask, nvec, C / 8, (int)relu, st);
}

// Fold the conv-epilogue replicas [nrep][2][C] of (sum g*mask, sum g*mask*xhat) into sums / dgamma / dbeta.
__global__ void __launch_bounds__(256) bn_bwd_fold_reps_kernel(const float* __restrict__ reps, int nrep, int C,
                                                               float* __restrict__ sums, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int r = 0; r < nrep; ++r) {
    a += reps[((long)r * 2) * C + c];
    b += reps[((long)r * 2 + 1) * C + c];
  }
  sums[c] = a;
  sums[C + c] = b;
  if (dbeta) dbeta[c] = a;
  if (dgamma) dgamma[c] = b;
}

// BN backward whose reduction already happened in the epilogue of the kernel that produced dy.
void launch_bn_bwd_from_sums(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean,
                             const float* invstd, const float* gamma, const float* beta, bool relu_x, uint16_t* dx,
                             uint16_t* dres, float* dgamma, float* dbeta, const float* reps, int nrep, float* sums,
                             long M, int C, hipStream_t st, const uint8_t* mask) {
  hipLaunchKernelGGL(bn_bwd_fold_reps_kernel, dim3(cdiv(C, 256)), dim3(256), 0, st, reps, nrep, C, sums, dgamma,
                     dbeta);
  const long nvec = M * C / 8;
  launch_bn_bwd_apply(dy, x, y, mean, invstd, beta, (int)relu_x, gamma, sums, dx, dres, nvec, C / 8, C,
                      1.f / (float)M, mask, st);
}

void launch_bn_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean, const float* invstd,
                   const float* gamma, const float* beta, bool relu_x, uint16_t* dx, uint16_t* dres, float* dgamma,
                   float* dbeta, float* work, float* sums, long M, int C, hipStream_t st, const uint8_t* mask) {
  BnGeom g = bn_geom(C, M);
  long rpb = bn_rows_per_block(M, g);
  int nb = (int)((M + rpb - 1) / rpb);
  if (mask)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, dy, x, y, mean,
                       invstd, gamma, beta, (int)relu_x, M, C, g.tpr, g.rows_per_iter, rpb, work, mask);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(nb, g.grid_y), dim3(BN_THREADS), 0, st, dy, x, y, mean,
                       invstd, gamma, beta, (int)relu_x, M, C, g.tpr, g.rows_per_iter, rpb, work, mask);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(cdiv(C, FIN_CH)), dim3(256), 0, st, work, nb, C, sums, dgamma, dbeta);
  const long nvec = M * C / 8;
  launch_bn_bwd_apply(dy, x, y, mean, invstd, beta, (int)relu_x, gamma, sums, dx, dres, nvec, C / 8, C,
                      1.f / (float)M, mask, st);
}

}  // namespace k8s_amd
