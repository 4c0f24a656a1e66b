// Streaming-kernel shape study for gfx950: which launch / access pattern reaches HBM peak for a
// read-one-write-one bf16 pass (the shape of every BatchNorm / elementwise pass).
//   hipcc --offload-arch=gfx950 -O3 stream_bw.hip -o stream_bw && ./stream_bw [GB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(8))) short v8;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// (a) grid-stride, one 16-B vector per trip
__global__ void __launch_bounds__(256) k_gs(const v8* __restrict__ x, v8* __restrict__ y, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    v8 v = x[i];
    v[0] += 1;
    y[i] = v;
  }
}
// (b) grid-stride, U vectors per trip, loads first
template <int U>
__global__ void __launch_bounds__(256) k_gsu(const v8* __restrict__ x, v8* __restrict__ y, long n) {
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    v8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) { v[u][0] += 1; y[i + u * stride] = v[u]; }
  }
  for (; i < n; i += stride) { v8 v = x[i]; v[0] += 1; y[i] = v; }
}
// (c) one block per contiguous chunk: block b handles vectors [b*CH, (b+1)*CH), U per trip, no grid stride
template <int U>
__global__ void __launch_bounds__(256) k_chunk(const v8* __restrict__ x, v8* __restrict__ y, long n, long ch) {
  const long b0 = blockIdx.x * ch, b1 = b0 + ch < n ? b0 + ch : n;
  for (long i = b0 + threadIdx.x; i < b1; i += 256 * U) {
    v8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + u * 256 < b1) v[u] = x[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) if (i + u * 256 < b1) { v[u][0] += 1; y[i + u * 256] = v[u]; }
  }
}
// (d) non-temporal variant of (b)
template <int U>
__global__ void __launch_bounds__(256) k_nt(const v8* __restrict__ x, v8* __restrict__ y, long n) {
  const long stride = (long)gridDim.x * 256;
  long i = blockIdx.x * 256L + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    v8 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) { v[u][0] += 1; __builtin_nontemporal_store(v[u], y + i + u * stride); }
  }
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 2.0;
  const long n = (long)(gb * (1L << 30) / 16);
  v8 *x, *y;
  CK(hipMalloc(&x, n * 16));
  CK(hipMalloc(&y, n * 16));
  CK(hipMemset(x, 0, n * 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 9; ++r) {
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"kernel\": \"%s\", \"GB\": %.2f, \"ms\": %.4f, \"tbps\": %.2f}\n", name, gb, ts[4], 2.0 * n * 16 / ts[4] / 1e9);
    fflush(stdout);
  };
  run("flat_1per_thread", [&] { hipLaunchKernelGGL(k_gs, dim3((n + 255) / 256), dim3(256), 0, 0, x, y, n); });
  for (long ch : {256L, 512L, 1024L, 2048L, 4096L}) {
    char nm[64];
    snprintf(nm, 64, "chunk%ld_u1", ch);
    run(nm, [&] { hipLaunchKernelGGL(k_chunk<1>, dim3((n + ch - 1) / ch), dim3(256), 0, 0, x, y, n, ch); });
    snprintf(nm, 64, "chunk%ld_u2", ch);
    run(nm, [&] { hipLaunchKernelGGL(k_chunk<2>, dim3((n + ch - 1) / ch), dim3(256), 0, 0, x, y, n, ch); });
    snprintf(nm, 64, "chunk%ld_u4", ch);
    run(nm, [&] { hipLaunchKernelGGL(k_chunk<4>, dim3((n + ch - 1) / ch), dim3(256), 0, 0, x, y, n, ch); });
  }
  run("gs_grid512", [&] { hipLaunchKernelGGL(k_gs, dim3(512), dim3(256), 0, 0, x, y, n); });
  run("gs_grid768", [&] { hipLaunchKernelGGL(k_gs, dim3(768), dim3(256), 0, 0, x, y, n); });
  run("gs_grid1024", [&] { hipLaunchKernelGGL(k_gs, dim3(1024), dim3(256), 0, 0, x, y, n); });
  return 0;
}
