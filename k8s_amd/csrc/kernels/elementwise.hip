// K9: transformer elementwise fusions, bf16 16-byte vectors, fp32 math.
//
//  * SwiGLU   y = silu(g) * u over a fused [T, 2F] gate|up GEMM output, and its backward
//  * RoPE     rotary embedding on [T, H, D] q/k in place of the usual 4 elementwise passes
//             (cos/sin from a precomputed fp32 table, host-built once -- no device trig)
//  * GELU(tanh) backward from the saved pre-activation
//  * column sums (bias gradients) without atomics: block partials + fold
#include "common.h"
#include "launchers.h"

namespace k8s_amd {

__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
// tanh(u) = 1 - 2 / (1 + 2^(2u log2 e)) on v_exp_f32 / v_rcp_f32 (libm tanhf is a long polynomial + branch path);
// saturates to +-1 for large |u|, absolute error ~1e-7 near 0
__device__ __forceinline__ float ftanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(2.8853900817779268f * u));
}

// gu: [T, 2F] (gate in [:, :F], up in [:, F:]) -> y: [T, F]
// Flat launches, one 16-B vector per thread: grid (T rows, F/8 / 256 column blocks), so no 64-bit index division
// (the former grid-stride form divided by F/8 per vector)
// gu column layout: blk == 0 -> [gate F | up F]; blk > 0 -> blocks of blk gate columns then blk up columns (the layout
// the gate|up GEMM's fused SwiGLU epilogue produces, gemm256.hip copy_out_swiglu): gate j at (j / blk) 2 blk + j % blk
__device__ __forceinline__ int swiglu_gcol(int c, int F, int blk) { return blk ? (c / blk) * 2 * blk + c % blk : c; }

__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ y,
                                                         long T, int F, int blk) {
  const int cvec = blockIdx.y * 256 + threadIdx.x;
  if (cvec >= F / 8) return;
  const long t = blockIdx.x;
  const int c = cvec * 8, gc = swiglu_gcol(c, F, blk), uo = blk ? blk : F;
  float g[8], u[8], o[8];
  load8(gu + t * 2 * F + gc, g);
  load8(gu + t * 2 * F + gc + uo, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = silu(g[j]) * u[j];
  store8(y + t * F + c, o);
}

// dgu[:, :F] = dy * u * silu'(g),  dgu[:, F:] = dy * silu(g)
__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const uint16_t* __restrict__ gu,
                                                         const uint16_t* __restrict__ dy, uint16_t* __restrict__ dgu,
                                                         long T, int F, int blk) {
  const int cvec = blockIdx.y * 256 + threadIdx.x;
  if (cvec >= F / 8) return;
  const long t = blockIdx.x;
  const int c = cvec * 8, gc = swiglu_gcol(c, F, blk), uo = blk ? blk : F;
  float g[8], u[8], d[8], dg[8], du[8];
  load8(gu + t * 2 * F + gc, g);
  load8(gu + t * 2 * F + gc + uo, u);
  load8(dy + t * F + c, d);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-g[j]));
    const float sl = g[j] * s;
    du[j] = d[j] * sl;
    dg[j] = d[j] * u[j] * (s * (1.f + g[j] * (1.f - s)));
  }
  store8(dgu + t * 2 * F + gc, dg);
  store8(dgu + t * 2 * F + gc + uo, du);
}

// x: [T, H, D] bf16 (row stride ld elements between tokens), pos: [T] int32, table: [maxpos, D/2] (cos, sin)
// rotate-half convention (x1 = x[:D/2], x2 = x[D/2:]): out1 = x1 c - x2 s, out2 = x2 c + x1 s.
// sign = -1 applies the inverse rotation (backward).
__global__ void __launch_bounds__(256) rope_kernel(uint16_t* __restrict__ x, long ld, const int* __restrict__ pos,
                                                   const float2* __restrict__ table, long T, int H, int D, float sign) {
  const int half = D / 2, hv = half / 8;
  const long total = T * H * hv;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long th = e / hv;
    const int c = (int)(e - th * hv) * 8;
    const long t = th / H;
    const int h = (int)(th - t * H);
    uint16_t* row = x + t * ld + (long)h * D;
    const float2* tb = table + (long)pos[t] * half + c;
    float a[8], b[8];
    load8(row + c, a);
    load8(row + half + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float cs = tb[j].x, sn = sign * tb[j].y;
      const float x1 = a[j], x2 = b[j];
      a[j] = __builtin_fmaf(x1, cs, -(x2 * sn));  // explicit fmas: the rounding gemm256.hip copy_out_rope repeats
      b[j] = __builtin_fmaf(x2, cs, x1 * sn);
    }
    store8(row + c, a);
    store8(row + half + c, b);
  }
}

__global__ void __launch_bounds__(256) gelu_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ pre,
                                                       uint16_t* __restrict__ dx, long nvec) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < nvec; e += (long)gridDim.x * blockDim.x) {
    float d[8], x[8];
    load8(dy + e * 8, d);
    load8(pre + e * 8, x);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float u = k0 * (x[j] + k1 * x[j] * x[j] * x[j]);
      const float t = ftanh(u);
      const float g = 0.5f * (1.f + t) + 0.5f * x[j] * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x[j] * x[j]);
      d[j] *= g;
    }
    store8(dx + e * 8, d);
  }
}

// relu backward with the mask taken from the (post-ReLU) output y
__global__ void __launch_bounds__(256) relu_bwd_kernel(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ y,
                                                       uint16_t* __restrict__ dx, long nvec) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < nvec; e += (long)gridDim.x * blockDim.x) {
    float d[8], v[8];
    load8(dy + e * 8, d);
    load8(y + e * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = v[j] > 0.f ? d[j] : 0.f;
    store8(dx + e * 8, d);
  }
}

// column sums of a [R, C] bf16 matrix -> fp32 [C] (written, or added when accumulate)
__global__ void __launch_bounds__(256) colsum_partial_kernel(const uint16_t* __restrict__ x, long R, int C, long rpb,
                                                             float* __restrict__ part) {
  const int cv = C / 8;
  const int cg = blockIdx.y * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;  // 8 row groups
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cg < cv) {
    const long r0 = blockIdx.x * rpb;
    const long r1 = r0 + rpb < R ? r0 + rpb : R;
    // 4 rows per trip, all loads issued before the adds (clamped address + zero weight past the end: no
    // per-load branch, which would serialise the loads behind vmcnt(0) waits)
    for (long r = r0 + rg; r < r1; r += 32) {
      float v[4][8], wgt[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = r + 8 * u;
        wgt[u] = rr < r1 ? 1.f : 0.f;
        load8(x + (rr < r1 ? rr : r1 - 1) * C + cg * 8, v[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += v[u][j] * wgt[u];
    }
  }
  __shared__ float sh[8][32][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[rg][threadIdx.x & 31][j] = s[j];
  __syncthreads();
  if (rg == 0 && cg < cv) {
    for (int g = 1; g < 8; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += sh[g][threadIdx.x][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) part[(long)blockIdx.x * C + cg * 8 + j] = s[j];
  }
}

// Activation backward fused with the column sums of its output (the bias gradient of the linear whose activation
// it is): g = dy * act'(pre) stored bf16 and summed per column exactly as colsum_partial_kernel sums a stored
// tensor (ACT 1 ReLU with pre = the ReLU output, 2 GELU(tanh) with pre = the pre-activation).
template <int ACT>
__global__ void __launch_bounds__(256) act_bwd_colsum_partial_kernel(const uint16_t* __restrict__ dy,
                                                                     const uint16_t* __restrict__ pre,
                                                                     uint16_t* __restrict__ g, long R, int C, long rpb,
                                                                     float* __restrict__ part) {
  const int cv = C / 8;
  const int cg = blockIdx.y * 32 + (threadIdx.x & 31);
  const int rg = threadIdx.x >> 5;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cg < cv) {
    const long r0 = blockIdx.x * rpb;
    const long r1 = r0 + rpb < R ? r0 + rpb : R;
    for (long r = r0 + rg; r < r1; r += 32) {
      float d[4][8], x[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long rr = r + 8 * u < r1 ? r + 8 * u : r1 - 1;
        load8(dy + rr * C + cg * 8, d[u]);
        load8(pre + rr * C + cg * 8, x[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float gd;
          if (ACT == 1) {
            gd = x[u][j] > 0.f ? 1.f : 0.f;
          } else {
            const float k0 = 0.7978845608028654f, k1 = 0.044715f;
            const float t = ftanh(k0 * (x[u][j] + k1 * x[u][j] * x[u][j] * x[u][j]));
            gd = 0.5f * (1.f + t) + 0.5f * x[u][j] * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x[u][j] * x[u][j]);
          }
          o[j] = d[u][j] * gd;
        }
        const bf16x8_t ob = pack_bf16x8(o);
        if (r + 8 * u < r1) {
          *reinterpret_cast<bf16x8_t*>(g + (r + 8 * u) * C + cg * 8) = ob;
#pragma unroll
          for (int j = 0; j < 8; ++j) s[j] += bf2f((uint16_t)ob[j]);
        }
      }
    }
  }
  __shared__ float sh[8][32][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[rg][threadIdx.x & 31][j] = s[j];
  __syncthreads();
  if (rg == 0 && cg < cv) {
    for (int q = 1; q < 8; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += sh[q][threadIdx.x][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) part[(long)blockIdx.x * C + cg * 8 + j] = s[j];
  }
}

// fold of the P partial rows: block = 64 columns x 4 partial-row groups (a wave each), LDS combine. P is up to
// 256 rows of L2-resident partials: 4 waves x P/4 independent loads per lane instead of one lane walking all P.
// Rows are ldp floats apart. With gridDim.y > 1 (the first level of a two-level fold of many rows): block y sums
// rows [y gs, min(P, (y + 1) gs)) and writes the result over row y gs (only this block reads that group).
__global__ void __launch_bounds__(256) colsum_fold_kernel(const float* part, int P, int C, float* out, int accumulate,
                                                          long ldp = 0,
                                                          int gs = 0) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), pg = threadIdx.x >> 6;
  if (ldp == 0) ldp = C;
  if (gridDim.y > 1) {
    part += (long)blockIdx.y * gs * ldp;
    P = min(gs, P - (int)blockIdx.y * gs);
    out = const_cast<float*>(part);
    accumulate = 0;
  }
  float s = 0.f;
  if (c < C) {
    int p = pg;
    for (; p + 12 < P; p += 16) {  // 4 loads in flight per lane
      const float a = part[(long)p * ldp + c], b = part[(long)(p + 4) * ldp + c];
      const float d = part[(long)(p + 8) * ldp + c], e = part[(long)(p + 12) * ldp + c];
      s += (a + b) + (d + e);
    }
    for (; p < P; p += 4) s += part[(long)p * ldp + c];
  }
  __shared__ float sh[4][64];
  sh[pg][threadIdx.x & 63] = s;
  __syncthreads();
  if (pg == 0 && c < C) {
    s = (sh[0][threadIdx.x] + sh[1][threadIdx.x]) + (sh[2][threadIdx.x] + sh[3][threadIdx.x]);
    out[c] = accumulate ? out[c] + s : s;  // (two-level first pass: every read of this group was before the barrier)
  }
}

// ----------------------------------------------------------------------------- launchers
void launch_swiglu_fwd(const uint16_t* gu, uint16_t* y, long T, int F, int blk, hipStream_t st) {
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(T, cdiv(F / 8, 256)), dim3(256), 0, st, gu, y, T, F, blk);
}
void launch_swiglu_bwd(const uint16_t* gu, const uint16_t* dy, uint16_t* dgu, long T, int F, int blk, hipStream_t st) {
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(T, cdiv(F / 8, 256)), dim3(256), 0, st, gu, dy, dgu, T, F, blk);
}
void launch_rope(uint16_t* x, long ld, const int* pos, const float* table, long T, int H, int D, bool inverse,
                 hipStream_t st) {
  hipLaunchKernelGGL(rope_kernel, dim3(stream_grid(T * H * (D / 16), 256)), dim3(256), 0, st, x, ld, pos,
                     (const float2*)table, T, H, D, inverse ? -1.f : 1.f);
}
void launch_gelu_bwd(const uint16_t* dy, const uint16_t* pre, uint16_t* dx, long n, hipStream_t st) {
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(stream_grid(n / 8, 256)), dim3(256), 0, st, dy, pre, dx, n / 8);
}
void launch_relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, hipStream_t st) {
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(stream_grid(n / 8, 256)), dim3(256), 0, st, dy, y, dx, n / 8);
}
// Row blocks of 32 rows (4 per thread, 8 row groups), at most 256 of them: a [8192, 768] gradient launches
// 256 x 3 = 768 blocks (was 32 x 3 with 256-row blocks: 96 blocks on 256 CUs, 0.9 TB/s).
static long colsum_row_blocks(long R) {
  long nb = (R + 31) / 32;
  return nb > 256 ? 256 : nb;
}
int colsum_workspace_floats(long R, int C) { return (int)(colsum_row_blocks(R) * C); }
void launch_act_bwd_colsum(int act, const uint16_t* dy, const uint16_t* pre, uint16_t* g, long R, int C, float* work,
                           float* out, bool accumulate, hipStream_t st) {
  const long nb = colsum_row_blocks(R);
  const long rpb = (R + nb - 1) / nb;
  dim3 grid((unsigned)nb, (unsigned)((C / 8 + 31) / 32));
  if (act == 1)
    hipLaunchKernelGGL(act_bwd_colsum_partial_kernel<1>, grid, dim3(256), 0, st, dy, pre, g, R, C, rpb, work);
  else
    hipLaunchKernelGGL(act_bwd_colsum_partial_kernel<2>, grid, dim3(256), 0, st, dy, pre, g, R, C, rpb, work);
  hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(C, 64)), dim3(256), 0, st, work, (int)nb, C, out, (int)accumulate,
                     0L, 0);
}
// P > 256 rows (per-128-row GEMM partials, per-sequence attention partials: 1,024 at BERT b1024) fold in two levels:
// groups of 32 rows in place, then the group results (36-48 blocks walking 1,024 rows took 29 us a fold)
void launch_colsum_fold(float* part, int P, int C, float* out, bool accumulate, hipStream_t st) {
  if (P > 256) {
    constexpr int GS = 32;
    const int G = (P + GS - 1) / GS;
    hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(C, 64), G), dim3(256), 0, st, part, P, C, part, 0, (long)C, GS);
    hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(C, 64)), dim3(256), 0, st, part, G, C, out, (int)accumulate,
                       (long)GS * C, 0);
    return;
  }
  hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(C, 64)), dim3(256), 0, st, part, P, C, out, (int)accumulate, 0L,
                     0);
}
// first level alone: rows [g gs, (g + 1) gs) of part summed into row g gs (a strided fold of the result follows)
void launch_colsum_group(float* part, int P, int C, int gs, hipStream_t st) {
  hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(C, 64), (P + gs - 1) / gs), dim3(256), 0, st, part, P, C, part, 0,
                     (long)C, gs);
}
void launch_colsum(const uint16_t* x, long R, int C, float* work, float* out, bool accumulate, hipStream_t st) {
  const long nb = colsum_row_blocks(R);
  const long rpb = (R + nb - 1) / nb;
  dim3 g((unsigned)nb, (unsigned)((C / 8 + 31) / 32));
  hipLaunchKernelGGL(colsum_partial_kernel, g, dim3(256), 0, st, x, R, C, rpb, work);
  hipLaunchKernelGGL(colsum_fold_kernel, dim3(cdiv(C, 64)), dim3(256), 0, st, work, (int)nb, C, out, (int)accumulate,
                     0L, 0);
}

}  // namespace k8s_amd
