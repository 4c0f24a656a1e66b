// Read-only streaming study for gfx950: which launch shape reaches HBM peak when a pass only READS (the BatchNorm
// backward reduction reads dy and x, writes a few KB of partial sums).
//   hipcc --offload-arch=gfx950 -O3 read_bw.hip -o read_bw && ./read_bw [GB per tensor]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f4;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float fold(const f4& v) { return v.x + v.y + v.z + v.w; }

// two tensors, U vectors of each per thread; block b covers a contiguous chunk of 256*U vectors (no grid stride);
// one float per block written (negligible traffic)
template <int U>
__global__ void __launch_bounds__(256) k_chunk2(const f4* __restrict__ a, const f4* __restrict__ b, long n,
                                                float* __restrict__ out) {
  const long base = (long)blockIdx.x * 256 * U + threadIdx.x;
  f4 va[U], vb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long i = base + u * 256;
    va[u] = i < n ? a[i] : f4{0, 0, 0, 0};
    vb[u] = i < n ? b[i] : f4{0, 0, 0, 0};
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) s += fold(va[u]) * fold(vb[u]);
  if (s == 1234.5f) out[blockIdx.x] = s;  // keeps the loads live without a store per block
}

// grid-stride: G blocks, U vectors of each tensor per trip, all loads of a trip issued first
template <int U>
__global__ void __launch_bounds__(256) k_gs2(const f4* __restrict__ a, const f4* __restrict__ b, long n,
                                             float* __restrict__ out) {
  const long stride = (long)gridDim.x * 256;
  float s = 0.f;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      va[u] = a[i + u * stride];
      vb[u] = b[i + u * stride];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s += fold(va[u]) * fold(vb[u]);
  }
  for (; i < n; i += stride) s += fold(a[i]) * fold(b[i]);
  if (s == 1234.5f) out[blockIdx.x] = s;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 1.0;
  const long n = (long)(gb * (1L << 30) / 16);
  f4 *a, *b;
  float* out;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMalloc(&out, 1 << 24));
  CK(hipMemset(a, 0, n * 16));
  CK(hipMemset(b, 0, n * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 9; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"kernel\": \"%s\", \"GB\": %.2f, \"ms\": %.4f, \"read_tbps\": %.2f}\n", name, 2 * gb, ts[4],
           2.0 * n * 16 / ts[4] / 1e9);
    fflush(stdout);
  };
  run("chunk2_u1", [&] { hipLaunchKernelGGL(k_chunk2<1>, dim3((n + 255) / 256), dim3(256), 0, 0, a, b, n, out); });
  run("chunk2_u2", [&] { hipLaunchKernelGGL(k_chunk2<2>, dim3((n + 511) / 512), dim3(256), 0, 0, a, b, n, out); });
  run("chunk2_u4", [&] { hipLaunchKernelGGL(k_chunk2<4>, dim3((n + 1023) / 1024), dim3(256), 0, 0, a, b, n, out); });
  run("chunk2_u8", [&] { hipLaunchKernelGGL(k_chunk2<8>, dim3((n + 2047) / 2048), dim3(256), 0, 0, a, b, n, out); });
  for (int g : {1024, 2048, 4096}) {
    char nm[64];
    snprintf(nm, 64, "gs2_g%d_u4", g);
    run(nm, [&] { hipLaunchKernelGGL(k_gs2<4>, dim3(g), dim3(256), 0, 0, a, b, n, out); });
    snprintf(nm, 64, "gs2_g%d_u8", g);
    run(nm, [&] { hipLaunchKernelGGL(k_gs2<8>, dim3(g), dim3(256), 0, 0, a, b, n, out); });
  }
  return 0;
}
