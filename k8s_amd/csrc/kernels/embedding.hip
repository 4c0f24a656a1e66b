// K9: token-embedding gather (sum of up to 3 tables: BERT word + position + token type; Llama: 1) and its
// scatter-add backward into the fp32 flat-gradient slots.
//
//   fwd: out[t][:] = sum_i W_i[row_i(t)][:]            (bf16 tables, fp32 sum, bf16 out)
//   bwd: dW_i[row_i(t)][:] += g[t][:]                    (fp32 atomics straight into the gradient slot)
// row_i(t) = ids_i[t] (int64), or t % S for a position table (no [B, S] position-id tensor).
// Flat launches, one 16-B vector (8 columns) of one token per thread (batchnorm.hip header: the streaming
// shape MI355X serves fastest). Tables with at most 4 rows (BERT's token types) are reduced per thread over a
// run of tokens in registers first: every token adding into the same 2 rows would serialize the atomics on a
// handful of addresses (MI355X_MICROARCH "Global float atomics": one hot row is ~14x slower).
#include <stdexcept>

#include "common.h"
#include "launchers.h"

namespace k8s_amd {

struct EmbTab {
  const uint16_t* w;    // [V][D] bf16 (forward)
  float* g;             // [V][D] fp32 gradient slot (backward)
  const int64_t* ids;   // [T] or null for a position table
  int V;
};
struct EmbArgs {
  EmbTab t[3];
  int ntab, T, D, S;  // S: sequence length (position rows = t % S)
};

__device__ __forceinline__ int emb_row(const EmbTab& e, int t, int S) {
  if (!e.ids) return t % S;
  const long r = e.ids[t];
  return (int)(r < 0 ? 0 : (r >= e.V ? e.V - 1 : r));  // out-of-range ids clamp (torch raises; we never fault)
}

__global__ void __launch_bounds__(256) embed_fwd_kernel(EmbArgs a, uint16_t* __restrict__ out, int nvec) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= nvec) return;
  const int cv = a.D >> 3;
  const int t = e / cv, c = (e - t * cv) * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= a.ntab) break;
    const int row = emb_row(a.t[i], t, a.S);
    float v[8];
    load8(a.t[i].w + (long)row * a.D + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  store8(out + (long)e * 8, acc);
}

// large tables: one wave per token, lane l adding column 64 i + l -- every atomic wave-instruction covers 256
// contiguous bytes of the gradient row, the shape the chip's atomic rate is quoted for (MI355X_MICROARCH "Global float
// atomics": ~1.3 TB/s of added bytes). The first form (a thread per 8 columns, 8 atomics each) put 64 lanes 32 B apart
// in every instruction and ran BERT-base's word-embedding backward (131k tokens x 768) in 2.7 ms.
// The wave walks its token's row 256 columns at a time: lane l loads columns 64 k + l (k = 0..3) first, then adds them.
__global__ void __launch_bounds__(256) embed_bwd_kernel(EmbArgs a, const uint16_t* __restrict__ g, int tab_mask) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= a.T) return;
  const uint16_t* gr = g + (long)t * a.D;
  float* dst[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    dst[i] = nullptr;
    if (i < a.ntab && ((tab_mask >> i) & 1)) {
      dst[i] = a.t[i].g + (long)emb_row(a.t[i], t, a.S) * a.D;
    }
  }
  for (int c0 = 0; c0 < a.D; c0 += 256) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // loads of the 4 columns first, then the atomics
      const int c = c0 + 64 * k + lane;
      v[k] = c < a.D ? bf2f(gr[c]) : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (!dst[i]) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = c0 + 64 * k + lane;
        if (c < a.D) atomicAdd(dst[i] + c, v[k]);
      }
    }
  }
}

// position tables (row = t % S): thread = (position p, 8 columns) sums the T / S tokens at that position in
// registers (loads of 8 tokens in flight) and adds once -- no atomics: each (row, column) has one owner. Through the
// atomic kernel every position row took T / S same-address atomics (64 per element at BERT's 8192 tokens / 128),
// which serialised it (~340 us of BERT-base's embedding backward).
__global__ void __launch_bounds__(256) embed_bwd_pos_kernel(EmbArgs a, const uint16_t* __restrict__ g, int tab,
                                                            int nthreads) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= nthreads) return;
  const int cv = a.D >> 3;
  const int p = e / cv, c = (e - p * cv) * 8;
  const EmbTab& tb = a.t[tab];
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  int t = p;
  for (; t + 7 * a.S < a.T; t += 8 * a.S) {
    float v[8][8];
#pragma unroll
    for (int u = 0; u < 8; ++u) load8(g + (long)(t + u * a.S) * a.D + c, v[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[u][j];
  }
  for (; t < a.T; t += a.S) {
    float v[8];
    load8(g + (long)t * a.D + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
  float* dst = tb.g + (long)p * a.D + c;
#pragma unroll
  for (int j = 0; j < 8; ++j) dst[j] += acc[j];
}

// small tables (V <= 4, BERT's token types): block = 32 column groups (8 columns each) x 8 token lanes over a chunk
// of EMB_CHUNK tokens; per-row sums in registers (8 tokens' ids and 16-B loads issued per trip), folded over the 8
// token lanes in LDS, then one atomic per (row, column) per block. (A thread per 64-token run with its own atomics
// put 2,048 adds on each of the 2 x 768 addresses at BERT's 131k tokens: 463 us, atomic-bound.)
constexpr int EMB_CHUNK = 512;
__global__ void __launch_bounds__(256) embed_bwd_small_kernel(EmbArgs a, const uint16_t* __restrict__ g, int tab) {
  const int cgl = threadIdx.x & 31, tl = threadIdx.x >> 5;
  const int cg = blockIdx.x * 32 + cgl, c = cg * 8;
  const bool on = c < a.D;
  const EmbTab& tb = a.t[tab];
  float acc[4][8];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[r][j] = 0.f;
  const int t0 = blockIdx.y * EMB_CHUNK, t1 = min(a.T, t0 + EMB_CHUNK);
  if (on) {
    int t = t0 + tl;
    for (; t + 56 < t1; t += 64) {  // 8 tokens of this lane per trip, all loads first
      int rows[8];
      bf16x8_t raw[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        rows[u] = emb_row(tb, t + 8 * u, a.S);
        raw[u] = *reinterpret_cast<const bf16x8_t*>(g + (long)(t + 8 * u) * a.D + c);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float w = rows[u] == r ? 1.f : 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[r][j] = __builtin_fmaf(w, bf2f((uint16_t)raw[u][j]), acc[r][j]);
        }
    }
    for (; t < t1; t += 8) {
      const int row = emb_row(tb, t, a.S);
      float v[8];
      load8(g + (long)t * a.D + c, v);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (row == r) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[r][j] += v[j];
        }
    }
  }
  __shared__ float sh[8][32][33];  // [token lane][column group][row * 8 + j] (+1 pad)
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[tl][cgl][r * 8 + j] = acc[r][j];
  __syncthreads();
  // 256 threads: (column group, 4 of the 32 (row, j) slots each) sum the 8 token lanes and add once
  const int k0 = tl * 4;
  if (on) {
#pragma unroll
    for (int k = k0; k < k0 + 4; ++k) {
      const int r = k >> 3, j = k & 7;
      if (r >= tb.V) continue;
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) v += sh[q][cgl][k];
      atomicAdd(tb.g + (long)r * a.D + c + j, v);
    }
  }
}

static EmbArgs emb_args(const EmbTable* tabs, int ntab, int T, int D, int S) {
  if (ntab < 1 || ntab > 3) throw std::runtime_error("embedding: 1 to 3 tables");
  if (D % 8 != 0) throw std::runtime_error("embedding: width must be a multiple of 8");
  if ((long)T * (D / 8) >= (1L << 31)) throw std::runtime_error("embedding: too many elements");
  EmbArgs a;
  for (int i = 0; i < 3; ++i) a.t[i] = EmbTab{nullptr, nullptr, nullptr, 1};
  for (int i = 0; i < ntab; ++i) a.t[i] = EmbTab{tabs[i].w, tabs[i].g, tabs[i].ids, tabs[i].V};
  a.ntab = ntab;
  a.T = T;
  a.D = D;
  a.S = S;
  return a;
}

void launch_embed_fwd(const EmbTable* tabs, int ntab, int T, int D, int S, uint16_t* out, hipStream_t st) {
  const EmbArgs a = emb_args(tabs, ntab, T, D, S);
  const int nvec = T * (D / 8);
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(cdiv(nvec, 256)), dim3(256), 0, st, a, out, nvec);
}

void launch_embed_bwd(const EmbTable* tabs, int ntab, int T, int D, int S, const uint16_t* g, hipStream_t st) {
  const EmbArgs a = emb_args(tabs, ntab, T, D, S);
  int big = 0;
  for (int i = 0; i < ntab; ++i) {
    if (tabs[i].V <= 4) {
      hipLaunchKernelGGL(embed_bwd_small_kernel, dim3(cdiv(D / 8, 32), cdiv(T, EMB_CHUNK)), dim3(256), 0, st, a, g,
                         i);
    } else if (!tabs[i].ids && S > 0 && S <= tabs[i].V) {  // position table: rows 0 .. S-1, one owner each
      const int nthreads = S * (D / 8);
      hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(cdiv(nthreads, 256)), dim3(256), 0, st, a, g, i, nthreads);
    } else {
      big |= 1 << i;
    }
  }
  if (big) hipLaunchKernelGGL(embed_bwd_kernel, dim3(cdiv(T, 4)), dim3(256), 0, st, a, g, big);
}

}  // namespace k8s_amd
