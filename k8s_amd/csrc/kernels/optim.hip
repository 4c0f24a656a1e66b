// Fused multi-tensor optimizers (K7 fused SGD+momentum, K8 fused Adam/AdamW)
// and gradient-norm utilities.
//
// "Multi-tensor" on this framework means FLAT: every parameter of a model
// lives in one contiguous fp32 master buffer (64-element aligned slots, see
// k8s_amd/parallel/flat.py), its optimizer state in same-shaped buffers and
// its gradients in one contiguous buffer that is also the all-reduce bucket
// storage. One launch therefore updates the whole model: no per-tensor
// launches, no pointer tables, and every access is a 16-B vector access.
//
// Weight decay is selected per 64-element chunk by `decay_mask` (one byte per
// chunk; parameter slots are 64-aligned, so a chunk never straddles two
// parameters). A null mask means "decay everything".
//
// An optional device-side scale pointer (gradient clip factor / loss-scale
// inverse) keeps the step free of host synchronisation so the whole step can
// be captured in a hipGraph. `hyper` (device fp32 [lr, step], optional) does
// the same for the values that change every step: a captured graph replays
// with the learning-rate schedule and Adam's bias correction read on device
// (utils/graph.py).
#include "common.h"
#include "launchers.h"

namespace k8s_amd {

template <typename GT>
__device__ __forceinline__ void load_grad4(const GT* g, long i, float (&o)[4]);

template <>
__device__ __forceinline__ void load_grad4<float>(const float* g, long i, float (&o)[4]) {
  float4 v = *reinterpret_cast<const float4*>(g + i);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
__device__ __forceinline__ void load_grad4<uint16_t>(const uint16_t* g, long i, float (&o)[4]) {
  bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(g + i);
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = bf2f((uint16_t)v[j]);
}

__device__ __forceinline__ void store_bf4(uint16_t* p, long i, const float4& v) {
  bf16x4_t o;
  o[0] = (short)f2bf(v.x); o[1] = (short)f2bf(v.y); o[2] = (short)f2bf(v.z); o[3] = (short)f2bf(v.w);
  *reinterpret_cast<bf16x4_t*>(p + i) = o;
}

template <typename GT>
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, float* __restrict__ mom,
                                                  const GT* __restrict__ g, uint16_t* __restrict__ pbf,
                                                  long n4, const uint8_t* __restrict__ decay_mask, float lr, float mu, float wd,
                                                  float scale, const float* __restrict__ scale_ptr,
                                                  const float* __restrict__ hyper, int nesterov, int first_step) {
  // a zero device factor = non-finite gradients (clip_factor_kernel): skip the step, leave every buffer
  // bit-identical (NaN * 0 is NaN, so scaling by 0 would poison the momentum / moments / weights)
  if (scale_ptr && *scale_ptr == 0.f) return;
  const float s = scale * (scale_ptr ? *scale_ptr : 1.f);
  if (hyper) lr = hyper[0];
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n4; q += (long)gridDim.x * blockDim.x) {
    const long i = q * 4;
    float gv[4];
    load_grad4<GT>(g, i, gv);
    float4 pv = *reinterpret_cast<float4*>(p + i);
    float4 mv = *reinterpret_cast<float4*>(mom + i);
    float* pp = &pv.x;
    float* mp = &mv.x;
    const float w = (!decay_mask || decay_mask[i >> 6]) ? wd : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float d = gv[j] * s + w * pp[j];
      float m = first_step ? d : mu * mp[j] + d;
      mp[j] = m;
      pp[j] -= lr * (nesterov ? d + mu * m : m);
    }
    *reinterpret_cast<float4*>(p + i) = pv;
    *reinterpret_cast<float4*>(mom + i) = mv;
    if (pbf) store_bf4(pbf, i, pv);
  }
}

template <typename GT>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, float* __restrict__ m1,
                                                   float* __restrict__ m2, const GT* __restrict__ g,
                                                   uint16_t* __restrict__ pbf, long n4, const uint8_t* __restrict__ decay_mask,
                                                   float lr, float b1, float b2, float eps, float wd,
                                                   float scale, const float* __restrict__ scale_ptr,
                                                   const float* __restrict__ hyper, float bc1, float bc2,
                                                   int decoupled) {
  if (scale_ptr && *scale_ptr == 0.f) return;  // non-finite gradients: skipped step (see sgd_kernel)
  const float s = scale * (scale_ptr ? *scale_ptr : 1.f);
  if (hyper) {
    lr = hyper[0];
    bc1 = 1.f - powf(b1, hyper[1]);
    bc2 = 1.f - powf(b2, hyper[1]);
  }
  const float step1 = lr / bc1;
  const float rbc2 = 1.f / sqrtf(bc2);
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q < n4; q += (long)gridDim.x * blockDim.x) {
    const long i = q * 4;
    float gv[4];
    load_grad4<GT>(g, i, gv);
    float4 pv = *reinterpret_cast<float4*>(p + i);
    float4 av = *reinterpret_cast<float4*>(m1 + i);
    float4 bv = *reinterpret_cast<float4*>(m2 + i);
    float* pp = &pv.x;
    float* ap = &av.x;
    float* bp = &bv.x;
    const float w = (!decay_mask || decay_mask[i >> 6]) ? wd : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = gv[j] * s;
      if (!decoupled) gr += w * pp[j];
      float a = b1 * ap[j] + (1.f - b1) * gr;
      float b = b2 * bp[j] + (1.f - b2) * gr * gr;
      ap[j] = a;
      bp[j] = b;
      float upd = step1 * a / (sqrtf(b) * rbc2 + eps);
      if (decoupled) pp[j] -= lr * w * pp[j];
      pp[j] -= upd;
    }
    *reinterpret_cast<float4*>(p + i) = pv;
    *reinterpret_cast<float4*>(m1 + i) = av;
    *reinterpret_cast<float4*>(m2 + i) = bv;
    if (pbf) store_bf4(pbf, i, pv);
  }
}

// Sum of squares of a flat buffer into out[0] (fp32, atomics once per block);
// also counts non-finite values into out[1]. out must be zeroed beforehand.
// A read-only stream: each thread keeps U independent 16-B (fp32) loads in flight per trip (U = 4: 64 B per lane),
// the tail is a plain one-vector loop. One vector per trip with 512 blocks measured 3.75 TB/s on Llama-3-8B's
// 32 GB fp32 gradient (profiles/r02_llama3_8b_seq4096_v2.md).
template <typename GT>
__global__ void __launch_bounds__(256) sumsq_kernel(const GT* __restrict__ g, long n4, float* __restrict__ out) {
  constexpr int U = 4;
  __shared__ float red[8];
  float acc = 0.f, bad = 0.f;
  const long stride = (long)gridDim.x * blockDim.x;
  long q = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; q + (U - 1) * stride < n4; q += U * stride) {
    float gv[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) load_grad4<GT>(g, (q + u * stride) * 4, gv[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc += gv[u][j] * gv[u][j];
        bad += isfinite(gv[u][j]) ? 0.f : 1.f;
      }
  }
  for (; q < n4; q += stride) {
    float gv[4];
    load_grad4<GT>(g, q * 4, gv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc += gv[j] * gv[j];
      bad += isfinite(gv[j]) ? 0.f : 1.f;
    }
  }
  acc = block_sum(acc, red);
  bad = block_sum(bad, red);
  if (threadIdx.x == 0) {
    atomicAdd(out, acc);
    atomicAdd(out + 1, bad);
  }
}

// clip factor = min(1, max_norm / (sqrt(sumsq) + 1e-6)); 0 if non-finite grads: the update kernels then skip
// the step entirely (no decay, no state change), like a loss-scaler's overflow skip.
__global__ void clip_factor_kernel(const float* __restrict__ stats, float max_norm, float* __restrict__ factor) {
  float norm = sqrtf(stats[0]);
  float f = max_norm / (norm + 1e-6f);
  f = f < 1.f ? f : 1.f;
  if (stats[1] > 0.f || !isfinite(norm)) f = 0.f;
  factor[0] = f;
}

// ---------------------------------------------------------------- bf16 gradient transport (parallel/ddp.py, ps.py)
// Sum of the `world` bf16 chunks [world][n] an all-to-all delivered for one gradient bucket, in rank order with fp32
// accumulation (deterministic, the same sum on every owner), into fp32 `out` (the owner's gradient slice) and/or
// bf16 `out_bf` (the reduced slice an all-gather returns to every rank). One pass, 16-B loads: replaces
// recv.float().sum(0).to(bf16) (an fp32 copy of the whole receive buffer plus two more passes).
__global__ void __launch_bounds__(256) slice_sum_kernel(const uint16_t* __restrict__ in, long n, int world,
                                                        float* __restrict__ out, uint16_t* __restrict__ out_bf) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q * 8 < n; q += (long)gridDim.x * blockDim.x) {
    const long i = q * 8;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (i + 8 <= n && (n & 7) == 0) {
      for (int r = 0; r < world; ++r) {
        const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(in + (long)r * n + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f((uint16_t)v[j]);
      }
      if (out) {
        *reinterpret_cast<float4*>(out + i) = make_float4(acc[0], acc[1], acc[2], acc[3]);
        *reinterpret_cast<float4*>(out + i + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
      }
      if (out_bf) *reinterpret_cast<bf16x8_t*>(out_bf + i) = pack_bf16x8(acc);
    } else {  // ragged slice length: element by element
      for (int j = 0; j < 8 && i + j < n; ++j) {
        float a = 0.f;
        for (int r = 0; r < world; ++r) a += bf2f(in[(long)r * n + i + j]);
        if (out) out[i + j] = a;
        if (out_bf) out_bf[i + j] = f2bf(a);
      }
    }
  }
}

// fp32 -> bf16 (round to nearest even) of a gradient bucket before the all-to-all, 16-B stores
__global__ void __launch_bounds__(256) cast_bf16_kernel(const float* __restrict__ in, uint16_t* __restrict__ out,
                                                        long n) {
  for (long q = blockIdx.x * (long)blockDim.x + threadIdx.x; q * 8 < n; q += (long)gridDim.x * blockDim.x) {
    const long i = q * 8;
    if (i + 8 <= n && (n & 7) == 0) {
      const float4 a = *reinterpret_cast<const float4*>(in + i), b = *reinterpret_cast<const float4*>(in + i + 4);
      const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      *reinterpret_cast<bf16x8_t*>(out + i) = pack_bf16x8(v);
    } else {
      for (int j = 0; j < 8 && i + j < n; ++j) out[i + j] = f2bf(in[i + j]);
    }
  }
}

// ---------------------------------------------------------------- launchers
void launch_slice_sum(const uint16_t* in, long n, int world, float* out, uint16_t* out_bf, hipStream_t st) {
  const int grid = stream_grid((n + 7) / 8, 256);
  hipLaunchKernelGGL(slice_sum_kernel, dim3(grid), dim3(256), 0, st, in, n, world, out, out_bf);
}

void launch_cast_bf16(const float* in, uint16_t* out, long n, hipStream_t st) {
  const int grid = stream_grid((n + 7) / 8, 256);
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid), dim3(256), 0, st, in, out, n);
}

void launch_sgd(float* p, float* mom, const void* g, bool g_bf16, uint16_t* pbf, long n, const uint8_t* decay_mask,
                float lr, float mu, float wd, float scale, const float* scale_ptr, const float* hyper, bool nesterov,
                bool first_step, hipStream_t st) {
  const long n4 = n / 4;
  const int grid = stream_grid(n4, 256);
  if (g_bf16)
    hipLaunchKernelGGL(sgd_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, p, mom, (const uint16_t*)g, pbf, n4,
                       decay_mask, lr, mu, wd, scale, scale_ptr, hyper, (int)nesterov, (int)first_step);
  else
    hipLaunchKernelGGL(sgd_kernel<float>, dim3(grid), dim3(256), 0, st, p, mom, (const float*)g, pbf, n4, decay_mask,
                       lr, mu, wd, scale, scale_ptr, hyper, (int)nesterov, (int)first_step);
}

void launch_adam(float* p, float* m1, float* m2, const void* g, bool g_bf16, uint16_t* pbf, long n, const uint8_t* decay_mask,
                 float lr, float b1, float b2, float eps, float wd, float scale, const float* scale_ptr,
                 const float* hyper, float bc1, float bc2, bool decoupled, hipStream_t st) {
  const long n4 = n / 4;
  const int grid = stream_grid(n4, 256);
  if (g_bf16)
    hipLaunchKernelGGL(adam_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, p, m1, m2, (const uint16_t*)g, pbf, n4,
                       decay_mask, lr, b1, b2, eps, wd, scale, scale_ptr, hyper, bc1, bc2, (int)decoupled);
  else
    hipLaunchKernelGGL(adam_kernel<float>, dim3(grid), dim3(256), 0, st, p, m1, m2, (const float*)g, pbf, n4,
                       decay_mask, lr, b1, b2, eps, wd, scale, scale_ptr, hyper, bc1, bc2, (int)decoupled);
}

void launch_sumsq(const void* g, bool g_bf16, long n, float* out, hipStream_t st) {
  const long n4 = n / 4;
  // 8 blocks of 256 per CU (stream_grid's cap): enough loads in flight to stream, few enough atomics
  const int grid = stream_grid(n4, 256);
  if (g_bf16)
    hipLaunchKernelGGL(sumsq_kernel<uint16_t>, dim3(grid), dim3(256), 0, st, (const uint16_t*)g, n4, out);
  else
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(grid), dim3(256), 0, st, (const float*)g, n4, out);
}

void launch_clip_factor(const float* stats, float max_norm, float* factor, hipStream_t st) {
  hipLaunchKernelGGL(clip_factor_kernel, dim3(1), dim3(1), 0, st, stats, max_norm, factor);
}

}  // namespace k8s_amd
