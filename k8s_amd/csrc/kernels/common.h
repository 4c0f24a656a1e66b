// Shared device helpers for the gfx950 (CDNA4) kernels of k8s_amd.
//
// Everything here is written for a 64-lane wavefront: reductions use
// __shfl_xor over 64 lanes, vector types are sized for 16-byte global
// accesses (bf16x8 / float4), and bf16 conversion is round-to-nearest-even.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace k8s_amd {

constexpr int kWave = 64;

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // 8 bf16 = 16 B
typedef __attribute__((ext_vector_type(4))) short bf16x4_t;   // 4 bf16 = 8 B
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;
typedef uint16_t bf16_raw;

__device__ __forceinline__ float bf2f(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

typedef __attribute__((ext_vector_type(8))) __bf16 bf16v8_t;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16v4_t;
typedef __attribute__((ext_vector_type(8))) float f32x8_t;

// fp32 -> bf16, round-to-nearest-even, NaN kept as a quiet NaN: gfx950's v_cvt_pk_bf16_f32 (one instruction per
// PAIR of values) instead of the 7-instruction integer rounding sequence -- the per-element passes (BatchNorm,
// GEMM epilogues) were VALU-bound on that sequence at ~4.5 TB/s
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

// The forward's affine pair; the backward recomputes it with the same operations, so the ReLU decision
// relu_on(x) below is bit-identical in every pass that makes it.
__device__ __forceinline__ void bn_affine_regs(float gamma, float beta, float mean, float invstd, float& scale,
                                               float& shift) {
  scale = gamma * invstd;
  shift = __builtin_fmaf(-mean, scale, beta);
}
__device__ __forceinline__ void bn_affine(float gamma, float beta, float mean, float invstd, float* scale,
                                          float* shift) {
  float a, b;
  bn_affine_regs(gamma, beta, mean, invstd, a, b);
  *scale = a;
  *shift = b;
}
// y > 0 for a non-residual BN + ReLU, from its input: the stored bf16 of fma(x, scale, shift) is positive
__device__ __forceinline__ bool relu_on(float x, float scale, float shift) {
  return bf2f(f2bf(__builtin_fmaf(x, scale, shift))) > 0.f;
}

// 8 floats -> 8 bf16 (4 v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16x8_t pack_bf16x8(const float (&o)[8]) {
  const f32x8_t f = {o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]};
  return __builtin_bit_cast(bf16x8_t, __builtin_convertvector(f, bf16v8_t));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum; `red` must hold blockDim.x/64 floats. Result broadcast to all threads.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

// Load 8 bf16 as floats.
__device__ __forceinline__ void load8(const uint16_t* p, float (&o)[8]) {
  bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f((uint16_t)v[j]);
}

__device__ __forceinline__ void store8(uint16_t* p, const float (&o)[8]) {
  *reinterpret_cast<bf16x8_t*>(p) = pack_bf16x8(o);
}

// Division by a runtime-invariant divisor as multiply-high + shift (valid for 0 <= n < 2^31).
struct FastDiv {
  uint32_t d, m, s;
  __device__ __forceinline__ int div(int n) const { return (int)((__umulhi((uint32_t)n, m) + (uint32_t)n) >> s); }
};
inline FastDiv make_fastdiv(int d) {
  FastDiv f;
  f.d = (uint32_t)d;
  f.s = 0;
  while ((1u << f.s) < f.d) ++f.s;
  f.m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << f.s) - f.d)) / f.d + 1);
  return f;
}

inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// CUs the launch planners size their grids for (wave quantisation, persistent grids, stream-K tails, split-K
// fill targets, grid-stride caps). Default: the current device's hipDeviceAttributeMultiprocessorCount (256 on
// MI355X), queried once per device. An override (set_planner_cus, or $K8S_AMD_PLANNER_CUS read on first use)
// replaces it for every device: a rank whose CUs are partly taken by concurrently running RCCL kernels can plan
// for fewer, and the GPU tests force odd budgets to check that every planner stays correct off the 256 grid.
// Defined in ops_binding.cpp's translation unit set (planner.cpp) so all kernels share one value.
int planner_cus();
void set_planner_cus(int n);  // n <= 0: back to the device's count

// Memory-bound launch sizing: at most 8 blocks per CU, grid-stride beyond that.
inline int stream_grid(long work_items, int block) {
  long g = (work_items + block - 1) / block;
  const long cap = 8L * planner_cus();
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace k8s_amd
