// K4: LayerNorm and RMSNorm, forward and backward, bf16 rows, fp32 math.
//
// One 64-lane wave owns one row; the row stays in registers between the
// statistics and the normalisation (CPL = 16-byte chunks per lane, so a row of
// D = CPL*64*8 elements is at most one global read and one write). Four waves
// per 256-thread block. Optional fused residual add (x = a + r, sum written
// out) covers the transformer "add & norm" step.
//
// Backward: per-row dx in registers; dgamma/dbeta are per-block partial sums
// over the block's rows ([nblocks, D] fp32) folded by a column-reduce kernel,
// so no float atomics are needed and results are reproducible.
#include "common.h"
#include "launchers.h"

namespace k8s_amd {

constexpr int NORM_WAVES = 4;

template <int CPL, bool RMS>
__global__ void __launch_bounds__(256) norm_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ res,
                                                       uint16_t* __restrict__ xsum, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, uint16_t* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       long R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * NORM_WAVES + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nch = D / 8;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      load8(x + row * D + ch * 8, v[c]);
      if (res) {
        float r[8];
        load8(res + row * D + ch * 8, r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] += r[j];
        store8(xsum + row * D + ch * 8, v[c]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[c][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[c][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
  if (lane == 0) {
    if (!RMS) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = ch * 8 + j;
        o[j] = (v[c][j] - mean) * rstd * gamma[k] + (RMS ? 0.f : beta[k]);
      }
      store8(y + row * D + ch * 8, o);
    }
  }
}

// rows_per_block rows per block (waves stride over rows); writes partial dgamma/dbeta per block.
template <int CPL, bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x,
                                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const uint16_t* __restrict__ dres,
                                                       uint16_t* __restrict__ dx, float* __restrict__ part, long R,
                                                       int D, int rows_per_block) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nch = D / 8;
  float pg[CPL][8], pb[CPL][8];
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) pg[c][j] = pb[c][j] = 0.f;
  const long r0 = (long)blockIdx.x * rows_per_block;
  for (long row = r0 + w; row < r0 + rows_per_block && row < R; row += NORM_WAVES) {
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float a = 0.f, b = 0.f;  // sum(dy*gamma), sum(dy*gamma*xhat)
    // pass 1: row reductions + parameter-gradient partials (kept in registers across rows)
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float g[8], xh[8];
        load8(dy + row * D + ch * 8, g);
        load8(x + row * D + ch * 8, xh);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = ch * 8 + j;
          xh[j] = (xh[j] - mu) * rs;
          pg[c][j] += g[j] * xh[j];
          pb[c][j] += g[j];
          const float gg = g[j] * gamma[k];
          a += gg;
          b += gg * xh[j];
        }
      }
    }
    a = wave_sum(a) / D;
    b = wave_sum(b) / D;
    // pass 2: re-read the (L1/L2-hot) row and write dx
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float g[8], xh[8], o[8];
        load8(dy + row * D + ch * 8, g);
        load8(x + row * D + ch * 8, xh);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = ch * 8 + j;
          const float xn = (xh[j] - mu) * rs;
          o[j] = rs * (g[j] * gamma[k] - (RMS ? 0.f : a) - xn * b);
        }
        if (dres) {
          float r[8];
          load8(dres + row * D + ch * 8, r);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += r[j];
        }
        store8(dx + row * D + ch * 8, o);
      }
    }
  }
  // block partials: waves write their own slice [blockIdx][w][D] then a column reduce folds waves too
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float* pgp = part + (((long)blockIdx.x * NORM_WAVES + w) * 2) * D + ch * 8;
      float* pbp = pgp + D;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pgp[j] = pg[c][j];
        pbp[j] = pb[c][j];
      }
    }
  }
}

// fold partial rows: part [P][2][D] -> dgamma[D], dbeta[D]. Block = 32 columns x 8 row slices (coalesced
// 128-B rows, 4 independent loads in flight per thread), LDS combine of the slices. P is ~1k partials: a
// thread-per-column serial loop here was latency-bound at ~260 us per call.
__global__ void __launch_bounds__(256) norm_colsum_kernel(const float* __restrict__ part, int P, int D,
                                                          float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float sh[2][8][33];
  const int col = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int k = blockIdx.x * 32 + col;
  float a = 0.f, b = 0.f;
  if (k < D) {
    int p = sl;
    for (; p + 24 < P; p += 32) {
      float av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = part[((long)(p + 8 * u) * 2) * D + k];
        bv[u] = part[((long)(p + 8 * u) * 2 + 1) * D + k];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a += av[u];
        b += bv[u];
      }
    }
    for (; p < P; p += 8) {
      a += part[((long)p * 2) * D + k];
      b += part[((long)p * 2 + 1) * D + k];
    }
  }
  sh[0][sl][col] = a;
  sh[1][sl][col] = b;
  __syncthreads();
  if (sl == 0 && k < D) {
#pragma unroll
    for (int i = 1; i < 8; ++i) {
      a += sh[0][i][col];
      b += sh[1][i][col];
    }
    if (dgamma) dgamma[k] = a;
    if (dbeta) dbeta[k] = b;
  }
}

template <bool RMS>
static void norm_fwd_dispatch(int cpl, dim3 g, hipStream_t st, const uint16_t* x, const uint16_t* res,
                              uint16_t* xsum, const float* gamma, const float* beta, uint16_t* y, float* mean,
                              float* rstd, long R, int D, float eps) {
#define NF(C) hipLaunchKernelGGL((norm_fwd_kernel<C, RMS>), g, dim3(256), 0, st, x, res, xsum, gamma, beta, y, mean, rstd, R, D, eps)
  switch (cpl) {
    case 1: NF(1); break;
    case 2: NF(2); break;
    case 4: NF(4); break;
    case 8: NF(8); break;
    default: NF(16); break;
  }
#undef NF
}

static int norm_cpl(int D) {
  const int nch = (D / 8 + 63) / 64;
  return nch <= 1 ? 1 : nch <= 2 ? 2 : nch <= 4 ? 4 : nch <= 8 ? 8 : 16;
}

void launch_norm_fwd(bool rms, const uint16_t* x, const uint16_t* res, uint16_t* xsum, const float* gamma,
                     const float* beta, uint16_t* y, float* mean, float* rstd, long R, int D, float eps,
                     hipStream_t st) {
  dim3 g(cdiv(R, NORM_WAVES));
  const int cpl = norm_cpl(D);
  if (rms)
    norm_fwd_dispatch<true>(cpl, g, st, x, res, xsum, gamma, beta, y, mean, rstd, R, D, eps);
  else
    norm_fwd_dispatch<false>(cpl, g, st, x, res, xsum, gamma, beta, y, mean, rstd, R, D, eps);
}

int norm_bwd_blocks(long R) {
  long b = (R + 31) / 32;  // 32 rows per block
  if (b > 256) b = 256;
  if (b < 1) b = 1;
  return (int)b;
}

int norm_workspace_floats(long R, int D) { return norm_bwd_blocks(R) * NORM_WAVES * 2 * D; }

void launch_norm_bwd(bool rms, const uint16_t* dy, const uint16_t* x, const float* gamma, const float* mean,
                     const float* rstd, const uint16_t* dres, uint16_t* dx, float* dgamma, float* dbeta, float* work,
                     long R, int D, hipStream_t st) {
  const int nb = norm_bwd_blocks(R);
  const int rpb = (int)((R + nb - 1) / nb);
  const int cpl = norm_cpl(D);
#define NB(C)                                                                                                    \
  if (rms)                                                                                                       \
    hipLaunchKernelGGL((norm_bwd_kernel<C, true>), dim3(nb), dim3(256), 0, st, dy, x, gamma, mean, rstd, dres, dx, \
                       work, R, D, rpb);                                                                         \
  else                                                                                                           \
    hipLaunchKernelGGL((norm_bwd_kernel<C, false>), dim3(nb), dim3(256), 0, st, dy, x, gamma, mean, rstd, dres,    \
                       dx, work, R, D, rpb);
  switch (cpl) {
    case 1: NB(1); break;
    case 2: NB(2); break;
    case 4: NB(4); break;
    case 8: NB(8); break;
    default: NB(16); break;
  }
#undef NB
  hipLaunchKernelGGL(norm_colsum_kernel, dim3(cdiv(D, 32)), dim3(256), 0, st, work, nb * NORM_WAVES, D, dgamma,
                     rms ? nullptr : dbeta);
}

}  // namespace k8s_amd
