// K4: LayerNorm and RMSNorm, forward and backward, bf16 rows, fp32 math.
//
// One 64-lane wave owns one row; the row stays in registers between the
// statistics and the normalisation (CPL = 16-byte chunks per lane, so a row of
// D = CPL*64*8 elements is at most one global read and one write). Four waves
// per 256-thread block. Optional fused residual add (x = a + r, sum written
// out) covers the transformer "add & norm" step.
//
// Backward: per-row dx in registers (one wave per row); dgamma/dbeta are
// per-64-row-block partial sums ([nblocks, 2, D] fp32) from a column kernel,
// folded by a column-reduce kernel, so no float atomics are needed and results
// are reproducible.
#include <stdexcept>

#include <type_traits>

#include <cstdlib>

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
  // the affine parameters are loaded with the row (in flight together) rather than after the two reductions,
  // where they were a dependent L2 round trip at the end of every wave (one wave per row = a single round of waves);
  // rows of up to 2048 only: at CPL 8 the extra 64-128 registers would cost waves per SIMD
  constexpr bool kPre = CPL <= 4;
  float gm[kPre ? CPL : 1][8], bt[kPre ? CPL : 1][8];
  if constexpr (kPre) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int cc = min(lane + c * 64, nch - 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        gm[c][j] = gamma[cc * 8 + j];
        bt[c][j] = RMS ? 0.f : beta[cc * 8 + j];
      }
    }
  }
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
        if constexpr (kPre) {
          o[j] = (v[c][j] - mean) * rstd * gm[c][j] + bt[c][j];
        } else {
          const int k = ch * 8 + j;
          o[j] = (v[c][j] - mean) * rstd * gamma[k] + (RMS ? 0.f : beta[k]);
        }
      }
      store8(y + row * D + ch * 8, o);
    }
  }
}

// rows_per_block rows per block (waves stride over rows); writes partial dgamma/dbeta per block.
// Backward as two independent launches (measured: the former one-kernel form, 8 rows per wave in sequence with a
// dy/x re-read for the second pass and per-block dgamma/dbeta partials, ran 0.9-1.7 TB/s: latency-bound, 2
// waves per CU on Llama-3-8B's 4096 rows):
//  * norm_bwd_dx_kernel: one wave per row, all of the row's dy / x (/ dres) loads issued up front and kept in
//    registers as raw bf16 across both passes -> every row in flight at once;
//  * norm_bwd_param_kernel: dgamma / dbeta column partials over 64-row blocks (8 columns per thread, 4 rows per
//    trip, mean / rstd broadcast per row), folded by norm_colsum_kernel.
template <int CPL, bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_dx_kernel(const uint16_t* __restrict__ dy,
                                                          const uint16_t* __restrict__ x,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const uint16_t* __restrict__ dres,
                                                          uint16_t* __restrict__ dx, float* __restrict__ rowab, long R,
                                                          int D) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * NORM_WAVES + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nch = D / 8;
  bf16x8_t gr[CPL], xr[CPL], rr[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    const int cc = ch < nch ? ch : nch - 1;  // clamped (unused) load instead of a branch per chunk
    gr[c] = *reinterpret_cast<const bf16x8_t*>(dy + row * D + cc * 8);
    xr[c] = *reinterpret_cast<const bf16x8_t*>(x + row * D + cc * 8);
    // the residual gradient addend too: loaded after the reductions it was a dependent round trip per wave
    if (dres) rr[c] = *reinterpret_cast<const bf16x8_t*>(dres + row * D + cc * 8);
  }
  const float mu = RMS ? 0.f : mean[row];
  const float rs = rstd[row];
  float a = 0.f, b = 0.f;  // sum(dy*gamma), sum(dy*gamma*xhat)
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gg = bf2f((uint16_t)gr[c][j]) * gamma[ch * 8 + j];
        a += gg;
        b += gg * ((bf2f((uint16_t)xr[c][j]) - mu) * rs);
      }
    }
  }
  a = wave_sum(a) / D;
  b = wave_sum(b) / D;
  if (rowab && lane == 0) {  // the row's dx coefficients, for the column sums of dx (upstream linear's bias grad)
    rowab[2 * row] = a;
    rowab[2 * row + 1] = b;
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xn = (bf2f((uint16_t)xr[c][j]) - mu) * rs;
        o[j] = rs * (bf2f((uint16_t)gr[c][j]) * gamma[ch * 8 + j] - (RMS ? 0.f : a) - xn * b);
      }
      if (dres) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += bf2f((uint16_t)rr[c][j]);
      }
      store8(dx + row * D + ch * 8, o);
    }
  }
}

constexpr int NORM_PARAM_ROWS = 64;  // rows per column-partial block (at least; norm_param_rows)
// rows per column-partial block: 64, or enough that at most 512 partial rows remain for the fold, whose D / 32 blocks
// walk them serially (BERT-base at 131k tokens: 2,048 partials took the fold 49 us per call, 1.3 ms per step)
static int norm_param_rows(long R) {
  long rows = (R + 511) / 512;
  rows = (rows + 31) / 32 * 32;
  return (int)(rows < NORM_PARAM_ROWS ? NORM_PARAM_ROWS : rows);
}

// part[blockIdx.x][0][k] = sum dy * xhat, part[blockIdx.x][1][k] = sum dy over the block's rows; block = 32 column
// chunks (256 columns) x 8 row groups, LDS combine of the row groups
// With rowab (the dx kernel's per-row a, b): also part[..][2][k] = sum dx, dx recomputed from dy, x and the row
// coefficients -- the bias gradient of the linear whose output this norm read (no separate column-sum pass).
template <bool RMS>
__global__ void __launch_bounds__(256) norm_bwd_param_kernel(const uint16_t* __restrict__ dy,
                                                             const uint16_t* __restrict__ x,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ rowab,
                                                             const float* __restrict__ gamma,
                                                             float* __restrict__ part, long R, int D, int prows) {
  const int nch = D / 8;
  const int ch = blockIdx.y * 32 + (threadIdx.x & 31), rg = threadIdx.x >> 5;
  float pg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pb[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float gm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (rowab && ch < nch) {
#pragma unroll
    for (int j = 0; j < 8; ++j) gm[j] = gamma[ch * 8 + j];
  }
  if (ch < nch) {
    const long r0 = (long)blockIdx.x * prows;
    const long r1 = r0 + prows < R ? r0 + prows : R;
    for (long r = r0 + rg; r < r1; r += 32) {  // 4 rows per trip, loads first (clamped, zero-weighted tail)
      float g[4][8], xv[4][8], mu[4], rs[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = r + 8 * u < r1 ? r + 8 * u : r1 - 1;
        load8(dy + rr * D + ch * 8, g[u]);
        load8(x + rr * D + ch * 8, xv[u]);
        mu[u] = RMS ? 0.f : mean[rr];
        rs[u] = r + 8 * u < r1 ? rstd[rr] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float wgt = r + 8 * u < r1 ? 1.f : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pg[j] += g[u][j] * ((xv[u][j] - mu[u]) * rs[u]);
          pb[j] += g[u][j] * wgt;
        }
      }
      if (rowab) {  // sum dx = rs * (dy * gamma - a - xhat * b) (rs = 0 on the clamped tail rows)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long rr = r + 8 * u < r1 ? r + 8 * u : r1 - 1;
          const float ra = RMS ? 0.f : rowab[2 * rr], rb = rowab[2 * rr + 1];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            pd[j] += rs[u] * (g[u][j] * gm[j] - ra - (xv[u][j] - mu[u]) * rs[u] * rb);
        }
      }
    }
  }
  __shared__ float sh[3][8][32][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][rg][threadIdx.x & 31][j] = pg[j];
    sh[1][rg][threadIdx.x & 31][j] = pb[j];
    sh[2][rg][threadIdx.x & 31][j] = pd[j];
  }
  __syncthreads();
  if (rg == 0 && ch < nch) {
    for (int q = 1; q < 8; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pg[j] += sh[0][q][threadIdx.x][j];
        pb[j] += sh[1][q][threadIdx.x][j];
        pd[j] += sh[2][q][threadIdx.x][j];
      }
    float* pgp = part + ((long)blockIdx.x * 3) * D + ch * 8;
    float* pbp = pgp + D;
    float* pdp = pbp + D;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      pgp[j] = pg[j];
      pbp[j] = pb[j];
      pdp[j] = pd[j];
    }
  }
}

// fold partial rows: part [P][2][D] -> dgamma[D], dbeta[D]. Block = 32 columns x 8 row slices (coalesced
// 128-B rows, 4 independent loads in flight per thread), LDS combine of the slices. P = R / 64 partial rows; a
// thread-per-column serial loop here was latency-bound at ~260 us per call with ~1k partials.
// (pstep: partial row p at part + p * pstep * 3 * D -- the group sums of a first-level fold, launch_colsum_group)
__global__ void __launch_bounds__(256) norm_colsum_kernel(const float* __restrict__ part, int P, int D,
                                                          float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                          float* __restrict__ dsum, int pstep = 1) {
  __shared__ float sh[3][8][33];
  const int col = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int k = blockIdx.x * 32 + col;
  float a = 0.f, b = 0.f, d = 0.f;
  if (k < D) {
    int p = sl;
    for (; p + 24 < P; p += 32) {
      float av[4], bv[4], dv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        av[u] = part[((long)(p + 8 * u) * pstep * 3) * D + k];
        bv[u] = part[((long)(p + 8 * u) * pstep * 3 + 1) * D + k];
        dv[u] = dsum ? part[((long)(p + 8 * u) * pstep * 3 + 2) * D + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a += av[u];
        b += bv[u];
        d += dv[u];
      }
    }
    for (; p < P; p += 8) {
      a += part[((long)p * pstep * 3) * D + k];
      b += part[((long)p * pstep * 3 + 1) * D + k];
      if (dsum) d += part[((long)p * pstep * 3 + 2) * D + k];
    }
  }
  sh[0][sl][col] = a;
  sh[1][sl][col] = b;
  sh[2][sl][col] = d;
  __syncthreads();
  if (sl == 0 && k < D) {
#pragma unroll
    for (int i = 1; i < 8; ++i) {
      a += sh[0][i][col];
      b += sh[1][i][col];
      d += sh[2][i][col];
    }
    if (dgamma) dgamma[k] = a;
    if (dbeta) dbeta[k] = b;
    if (dsum) dsum[k] = d;
  }
}

// Many short rows (BERT-base: 131k rows of 768): the dx kernel and the column partials in ONE pass. Each wave walks
// RPW consecutive rows with the next row's dy / x (/ dres) loads issued before this row's math, keeps the per-column
// sums of dy * xhat, dy and dx (the upstream linear's bias gradient) in registers, and the block's 4 waves combine them
// in LDS into one partial row [3][D]. The separate column kernel re-read dy and x (91 us per BERT call) and its
// 64-row partials made a 2,048-row fold. CPL <= 2 (D <= 1024).
// NS: register slots of the row prefetch (2: the next row's loads in flight during this row's math; 3: two rows ahead,
// no residual gradient operand -- its slots would push D = 768 past 256 VGPRs)
constexpr int NORM_FUSED_RPW = 32;
template <int CPL, bool RMS, int NS = 2>
__global__ void __launch_bounds__(256) norm_bwd_fused_kernel(const uint16_t* __restrict__ dy,
                                                             const uint16_t* __restrict__ x,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const uint16_t* __restrict__ dres,
                                                             uint16_t* __restrict__ dx, float* __restrict__ part,
                                                             long R, int D, int want_dsum) {
  static_assert(CPL <= 2, "short rows only");
  constexpr int RPW = NORM_FUSED_RPW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long row0 = ((long)blockIdx.x * NORM_WAVES + wave) * RPW;
  const int nch = D / 8;
  float gm[CPL][8], pg[CPL][8], pb[CPL][8], pd[CPL][8];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int ch = lane + c * 64;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      gm[c][j] = ch < nch ? gamma[ch * 8 + j] : 0.f;
      pg[c][j] = pb[c][j] = pd[c][j] = 0.f;
    }
  }
  bf16x8_t gr[NS][CPL], xr[NS][CPL], rr[NS == 2 ? NS : 1][CPL];
  if constexpr (NS != 2) dres = nullptr;
  auto load = [&](auto slot_c, long row) {
    constexpr int sl = decltype(slot_c)::value;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      const int cc = ch < nch ? ch : nch - 1;
      gr[sl][c] = *reinterpret_cast<const bf16x8_t*>(dy + row * D + cc * 8);
      xr[sl][c] = *reinterpret_cast<const bf16x8_t*>(x + row * D + cc * 8);
      if constexpr (NS == 2) {
        if (dres) rr[sl][c] = *reinterpret_cast<const bf16x8_t*>(dres + row * D + cc * 8);
      }
    }
  };
  auto step = [&](auto slot_c, long row) {
    constexpr int sl = decltype(slot_c)::value;
    const float mu = RMS ? 0.f : mean[row];
    const float rs = rstd[row];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (lane + c * 64 < nch) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gg = bf2f((uint16_t)gr[sl][c][j]) * gm[c][j];
          a += gg;
          b += gg * ((bf2f((uint16_t)xr[sl][c][j]) - mu) * rs);
        }
      }
    }
    a = wave_sum(a) / D;
    b = wave_sum(b) / D;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const int ch = lane + c * 64;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float g = bf2f((uint16_t)gr[sl][c][j]);
          const float xn = (bf2f((uint16_t)xr[sl][c][j]) - mu) * rs;
          o[j] = rs * (g * gm[c][j] - (RMS ? 0.f : a) - xn * b);
          pg[c][j] += g * xn;
          pb[c][j] += g;
          pd[c][j] += o[j];
        }
        if constexpr (NS == 2) {
          if (dres) {
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] += bf2f((uint16_t)rr[sl][c][j]);
          }
        }
        store8(dx + row * D + ch * 8, o);
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, NS == 3 ? 2 : 0>;
  const long rend = row0 + RPW < R ? row0 + RPW : R;
  if constexpr (NS == 2) {
    if (row0 < R) load(S0{}, row0);
    for (int i = 0; i < RPW; i += 2) {  // two rows per trip: the register slots stay compile-time
      const long r = row0 + i;
      if (r >= R) break;
      if (r + 1 < R) load(S1{}, r + 1);
      step(S0{}, r);
      if (r + 1 >= R) break;
      if (i + 2 < RPW && r + 2 < R) load(S0{}, r + 2);
      step(S1{}, r + 1);
    }
  } else {
    if (row0 < rend) load(S0{}, row0);
    if (row0 + 1 < rend) load(S1{}, row0 + 1);
    for (long r = row0; r < rend; r += 3) {  // three rows per trip, each slot refilled three rows ahead
      if (r + 2 < rend) load(S2{}, r + 2);
      step(S0{}, r);
      if (r + 1 >= rend) break;
      if (r + 3 < rend) load(S0{}, r + 3);
      step(S1{}, r + 1);
      if (r + 2 >= rend) break;
      if (r + 4 < rend) load(S1{}, r + 4);
      step(S2{}, r + 2);
    }
  }
  // the block's 4 waves -> one partial row [3][D] (sum dy * xhat | sum dy | sum dx)
  __shared__ float sh[NORM_WAVES][3][CPL * 512];
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = (lane + c * 64) * 8 + j;
      sh[wave][0][k] = pg[c][j];
      sh[wave][1][k] = pb[c][j];
      sh[wave][2][k] = pd[c][j];
    }
  __syncthreads();
  for (int k = threadIdx.x; k < 3 * D; k += 256) {
    const int which = k / D, col = k - which * D;
    if (which == 2 && !want_dsum) continue;
    part[(long)blockIdx.x * 3 * D + k] =
        (sh[0][which][col] + sh[1][which][col]) + (sh[2][which][col] + sh[3][which][col]);
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

static int norm_param_blocks(long R) { return (int)((R + norm_param_rows(R) - 1) / norm_param_rows(R)); }

// the fused one-pass backward for many short rows (norm_bwd_fused_kernel)
static bool norm_fused_ok(long R, int D) { return norm_cpl(D) <= 2 && R >= 16384; }
static int norm_fused_blocks(long R) { return (int)((R + NORM_WAVES * NORM_FUSED_RPW - 1) / (NORM_WAVES * NORM_FUSED_RPW)); }

// [nblocks][3][D] partials + [R][2] row coefficients
int norm_workspace_floats(long R, int D) {
  const long two = norm_param_blocks(R) * 3L * D + 2 * R;
  const long one = norm_fused_ok(R, D) ? norm_fused_blocks(R) * 3L * D : 0;
  return (int)(two > one ? two : one);
}

void launch_norm_bwd(bool rms, const uint16_t* dy, const uint16_t* x, const float* gamma, const float* mean,
                     const float* rstd, const uint16_t* dres, uint16_t* dx, float* dgamma, float* dbeta, float* work,
                     long R, int D, hipStream_t st, float* dsum) {
  if (dsum && dres) throw std::runtime_error("norm_bwd: the dx column sums exclude a residual gradient");
  const int cpl = norm_cpl(D);
  if (norm_fused_ok(R, D)) {
    const int nbf = norm_fused_blocks(R);
    static const bool deep = [] {  // K8S_AMD_NORM_PREFETCH=2 keeps the two-slot form
      const char* e = std::getenv("K8S_AMD_NORM_PREFETCH");
      return !(e && e[0] == '2');
    }();
#define NBF(C, RM)                                                                                                    \
  if (deep && !dres)                                                                                                  \
    hipLaunchKernelGGL((norm_bwd_fused_kernel<C, RM, 3>), dim3(nbf), dim3(256), 0, st, dy, x, gamma, mean, rstd, dres, \
                       dx, work, R, D, dsum ? 1 : 0);                                                                 \
  else                                                                                                                \
    hipLaunchKernelGGL((norm_bwd_fused_kernel<C, RM, 2>), dim3(nbf), dim3(256), 0, st, dy, x, gamma, mean, rstd, dres, \
                       dx, work, R, D, dsum ? 1 : 0)
    if (cpl == 1) {
      if (rms) NBF(1, true); else NBF(1, false);
    } else {
      if (rms) NBF(2, true); else NBF(2, false);
    }
#undef NBF
    // 1,024 partial rows at BERT b1024: folded in groups of 32 first (24 blocks walking them took 20 us a call)
    constexpr int GS = 32;
    if (nbf > 4 * GS) {
      launch_colsum_group(work, nbf, 3 * D, GS, st);
      hipLaunchKernelGGL(norm_colsum_kernel, dim3(cdiv(D, 32)), dim3(256), 0, st, work, (nbf + GS - 1) / GS, D,
                         dgamma, rms ? nullptr : dbeta, dsum, GS);
    } else {
      hipLaunchKernelGGL(norm_colsum_kernel, dim3(cdiv(D, 32)), dim3(256), 0, st, work, nbf, D, dgamma,
                         rms ? nullptr : dbeta, dsum, 1);
    }
    return;
  }
  const dim3 g(cdiv(R, NORM_WAVES));
  const int nb = norm_param_blocks(R);
  float* const rowab = dsum ? work + (long)nb * 3 * D : nullptr;
#define NB(C)                                                                                                     \
  if (rms)                                                                                                        \
    hipLaunchKernelGGL((norm_bwd_dx_kernel<C, true>), g, dim3(256), 0, st, dy, x, gamma, mean, rstd, dres, dx, \
                       rowab, R, D);                                                                             \
  else                                                                                                            \
    hipLaunchKernelGGL((norm_bwd_dx_kernel<C, false>), g, dim3(256), 0, st, dy, x, gamma, mean, rstd, dres, dx, \
                       rowab, R, D);
  switch (cpl) {
    case 1: NB(1); break;
    case 2: NB(2); break;
    case 4: NB(4); break;
    case 8: NB(8); break;
    default: NB(16); break;
  }
#undef NB
  const dim3 gp(nb, cdiv(D / 8, 32));
  if (rms)
    hipLaunchKernelGGL(norm_bwd_param_kernel<true>, gp, dim3(256), 0, st, dy, x, mean, rstd, rowab, gamma, work, R,
                       D, norm_param_rows(R));
  else
    hipLaunchKernelGGL(norm_bwd_param_kernel<false>, gp, dim3(256), 0, st, dy, x, mean, rstd, rowab, gamma, work, R,
                       D, norm_param_rows(R));
  hipLaunchKernelGGL(norm_colsum_kernel, dim3(cdiv(D, 32)), dim3(256), 0, st, work, nb, D, dgamma,
                     rms ? nullptr : dbeta, dsum);
}

}  // namespace k8s_amd
