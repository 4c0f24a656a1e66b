// K6: fused softmax cross-entropy (fwd + bwd), large-vocab friendly.
//
// One 256-thread block per row. The forward streams the row once with an
// online (max, sum-exp) per thread, combines across the block and writes the
// per-row loss and log-sum-exp. The backward recomputes softmax from the saved
// LSE and writes dlogits = (softmax - onehot) * dloss[row] in one pass, so the
// [rows, vocab] probability matrix is never materialised.
#include "common.h"
#include "launchers.h"

namespace k8s_amd {

template <typename T>
__device__ __forceinline__ void load8_any(const T* p, float (&o)[8]);
template <>
__device__ __forceinline__ void load8_any<uint16_t>(const uint16_t* p, float (&o)[8]) { load8(p, o); }
template <>
__device__ __forceinline__ void load8_any<float>(const float* p, float (&o)[8]) {
  float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <typename T>
__device__ __forceinline__ float load1(const T* p);
template <>
__device__ __forceinline__ float load1<uint16_t>(const uint16_t* p) { return bf2f(*p); }
template <>
__device__ __forceinline__ float load1<float>(const float* p) { return *p; }

template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       long V, long ld, float* __restrict__ loss,
                                                       float* __restrict__ lse_out, long ignore_index,
                                                       float smoothing) {
  __shared__ float red[8];
  const long row = blockIdx.x;
  const T* x = logits + row * ld;
  float m = -INFINITY, s = 0.f, sumx = 0.f;
  const long V8 = ((ld & 7) == 0 && (((uintptr_t)logits) & 15) == 0) ? (V / 8) * 8 : 0;
  for (long i = threadIdx.x * 8; i < V8; i += 256 * 8) {
    float v[8];
    load8_any<T>(x + i, v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    const float nm = fmaxf(m, lm);
    float acc = s * __expf(m - nm);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      acc += __expf(v[j] - nm);
      sumx += v[j];
    }
    s = acc;
    m = nm;
  }
  for (long i = V8 + threadIdx.x; i < V; i += 256) {
    const float v = load1<T>(x + i);
    const float nm = fmaxf(m, v);
    s = s * __expf(m - nm) + __expf(v - nm);
    m = nm;
    sumx += v;
  }
  const float gm = block_max(m, red);
  float sc = (m == -INFINITY) ? 0.f : s * __expf(m - gm);
  const float gs = block_sum(sc, red);
  const float gsumx = smoothing > 0.f ? block_sum(sumx, red) : 0.f;
  if (threadIdx.x == 0) {
    const float lse = gm + __logf(gs);
    lse_out[row] = lse;
    const long lab = labels[row];
    if (lab == ignore_index) {
      loss[row] = 0.f;
    } else {
      const float xl = load1<T>(x + lab);
      float l = lse - xl;
      if (smoothing > 0.f) l = (1.f - smoothing) * l + smoothing * (lse - gsumx / (float)V);
      loss[row] = l;
    }
  }
}

template <typename T>
__device__ __forceinline__ void store8_any(T* p, const float (&o)[8]);
template <>
__device__ __forceinline__ void store8_any<uint16_t>(uint16_t* p, const float (&o)[8]) { store8(p, o); }
template <>
__device__ __forceinline__ void store8_any<float>(float* p, const float (&o)[8]) {
  reinterpret_cast<float4*>(p)[0] = make_float4(o[0], o[1], o[2], o[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(o[4], o[5], o[6], o[7]);
}
template <typename T>
__device__ __forceinline__ void store1(T* p, float v);
template <>
__device__ __forceinline__ void store1<uint16_t>(uint16_t* p, float v) { *p = f2bf(v); }
template <>
__device__ __forceinline__ void store1<float>(float* p, float v) { *p = v; }

// dscale: per-row multiplier pointer (dloss/n_valid broadcast) -> scale = dscale[0] (scalar mean reduction)
template <typename T>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse, const float* __restrict__ dscale,
                                                       int per_row, long V, long ld, T* __restrict__ dlogits,
                                                       long ignore_index, float smoothing) {
  const long row = blockIdx.x;
  const T* x = logits + row * ld;
  T* dx = dlogits + row * ld;
  const long lab = labels[row];
  const float sc = (lab == ignore_index) ? 0.f : dscale[per_row ? row : 0];
  const float l = lse[row];
  const float off = smoothing / (float)V;
  const float on = 1.f - smoothing;
  const long V8 = ((ld & 7) == 0 && (((uintptr_t)logits) & 15) == 0) ? (V / 8) * 8 : 0;
  for (long i = threadIdx.x * 8; i < V8; i += 256 * 8) {
    float v[8];
    load8_any<T>(x + i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float p = __expf(v[j] - l) - off;
      if (i + j == lab) p -= on;
      v[j] = p * sc;
    }
    store8_any<T>(dx + i, v);
  }
  for (long i = V8 + threadIdx.x; i < V; i += 256) {
    float p = __expf(load1<T>(x + i) - l) - off;
    if (i == lab) p -= on;
    store1<T>(dx + i, p * sc);
  }
  // padded columns [V, ld) of the gradient are written here, so the caller never zero-fills the whole matrix
  for (long i = V + threadIdx.x; i < ld; i += 256) store1<T>(dx + i, 0.f);
}

void launch_xent_fwd(const void* logits, bool bf16, const int64_t* labels, long R, long V, long ld, float* loss,
                     float* lse, long ignore_index, float smoothing, hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL(xent_fwd_kernel<uint16_t>, dim3(R), dim3(256), 0, st, (const uint16_t*)logits, labels, V, ld,
                       loss, lse, ignore_index, smoothing);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(R), dim3(256), 0, st, (const float*)logits, labels, V, ld, loss,
                       lse, ignore_index, smoothing);
}

void launch_xent_bwd(const void* logits, bool bf16, const int64_t* labels, const float* lse, const float* dscale,
                     bool per_row, long R, long V, long ld, void* dlogits, long ignore_index, float smoothing,
                     hipStream_t st) {
  if (bf16)
    hipLaunchKernelGGL(xent_bwd_kernel<uint16_t>, dim3(R), dim3(256), 0, st, (const uint16_t*)logits, labels, lse,
                       dscale, (int)per_row, V, ld, (uint16_t*)dlogits, ignore_index, smoothing);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(R), dim3(256), 0, st, (const float*)logits, labels, lse, dscale,
                       (int)per_row, V, ld, (float*)dlogits, ignore_index, smoothing);
}

}  // namespace k8s_amd
