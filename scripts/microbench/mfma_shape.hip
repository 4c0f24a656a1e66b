// Which bf16 MFMA shape should a gfx950 GEMM / attention inner loop use: v_mfma_f32_16x16x32_bf16 or
// v_mfma_f32_32x32x16_bf16? (VERDICT round 2 asked for a 32x32x16 variant of the 256 x 256 GEMM.)
//
// Both loops compute the same per-wave output tile (128 x 64, the 256 x 256 GEMM's wave tile) over the same K, with
// every operand fragment re-read from LDS by ds_read_b128 each K step (as the GEMM does), on random data (MFMA
// power and therefore clock depend on the operand bits: zero data would rank the shapes by cycles only), one block
// of 8 waves per CU, 2 waves per SIMD, grid = 256 x 4 blocks. Reports wall time and TFLOP/s for each shape.
//   hipcc --offload-arch=gfx950 -O3 mfma_shape.hip -o mfma_shape && ./mfma_shape
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                      \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef __attribute__((ext_vector_type(8))) __bf16 bf8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(16))) float f16v;

constexpr int KSTEPS = 2048;  // 32-deep K steps per wave

// 16x16x32: wave tile 128 x 64 = 8 x 4 accumulators (f32x4), per K step 8 A + 4 B fragments, 32 MFMAs
__global__ void __launch_bounds__(512, 1) k16(const bf8* __restrict__ src, float* __restrict__ out) {
  __shared__ bf8 lds[512 * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 512 * 4; i += 512) lds[i] = src[(blockIdx.x * 2048 + i) & 65535];
  __syncthreads();
  f4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0, 0, 0, 0};
  for (int s = 0; s < KSTEPS; ++s) {
    bf8 a[8], b[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = lds[(i * 64 + lane + s) & 2047];
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = lds[(1024 + j * 64 + lane + s) & 2047];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) t += acc[i][j].x + acc[i][j].y + acc[i][j].z + acc[i][j].w;
  out[blockIdx.x * 512 + tid] = t;
}

// 32x32x16: the same 128 x 64 wave tile = 4 x 2 accumulators (f32x16); a 32-deep K step is two 16-deep MFMA k
// steps: per step 4 A + 2 B fragments per half, 16 MFMAs
__global__ void __launch_bounds__(512, 1) k32(const bf8* __restrict__ src, float* __restrict__ out) {
  __shared__ bf8 lds[512 * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < 512 * 4; i += 512) lds[i] = src[(blockIdx.x * 2048 + i) & 65535];
  __syncthreads();
  f16v acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f16v{};
  for (int s = 0; s < KSTEPS; ++s) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf8 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = lds[(h * 512 + i * 64 + lane + s) & 2047];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = lds[(1024 + h * 256 + j * 64 + lane + s) & 2047];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) t += acc[i][j][r];
  out[blockIdx.x * 512 + tid] = t;
}

int main() {
  const int blocks = 256 * 4;
  std::vector<__bf16> h(65536 * 8);
  srand(1);
  for (auto& v : h) v = (__bf16)((float)rand() / RAND_MAX * 2.f - 1.f);
  bf8* src;
  float* out;
  CK(hipMalloc(&src, h.size() * 2));
  CK(hipMalloc(&out, blocks * 512 * 4));
  CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // FLOPs per launch: blocks x 8 waves x (128 x 64 x 32 x 2) per K step x KSTEPS
  const double flops = (double)blocks * 8 * 128 * 64 * 32 * 2 * KSTEPS;
  for (int rep = 0; rep < 3; ++rep) {
    for (int which = 0; which < 2; ++which) {
      for (int w = 0; w < 2; ++w) {  // warm-up launch
        if (which == 0) hipLaunchKernelGGL(k16, dim3(blocks), dim3(512), 0, 0, src, out);
        else hipLaunchKernelGGL(k32, dim3(blocks), dim3(512), 0, 0, src, out);
      }
      CK(hipEventRecord(a));
      const int it = 5;
      for (int i = 0; i < it; ++i) {
        if (which == 0) hipLaunchKernelGGL(k16, dim3(blocks), dim3(512), 0, 0, src, out);
        else hipLaunchKernelGGL(k32, dim3(blocks), dim3(512), 0, 0, src, out);
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= it;
      printf("{\"shape\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"tflops\": %.1f}\n",
             which == 0 ? "16x16x32" : "32x32x16", rep, ms, flops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
