// K1 large-tile GEMM for gfx950: 256 x 256 output tile, 8 waves, LDS-ring pipelined K loop.
//
//   C[M,N] (+)= alpha * op(A) . op(B) (+ bias, ReLU / GELU epilogue)   bf16 in, fp32 accumulate
//
// The hot path of the transformer linear layers (BERT / Llama-3-8B fwd, dgrad and wgrad) when the output has
// enough 256 x 256 tiles to fill the chip (gemm256_eligible); the 128 x 128 kernel of gemm.hip (2 blocks/CU)
// takes the rest and the convolutions.
//
// Design (cdna_hip_programming.md §5, MI355X_MICROARCH "Two waves per SIMD"):
//  * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 piece = 8 x 4 tiles of
//    v_mfma_f32_16x16x32_bf16 (128 accumulator VGPRs), ~200 VGPRs -> 2 waves per SIMD, 1 workgroup per CU.
//  * K is streamed in 32-deep stages (A 256 x 32 + B 256 x 32 = 32 KB) through a 5-slot LDS ring (160 KB) by
//    global_load_lds (16 B per lane, no VGPR round trip); each stage is issued THREE phases ahead of its use and
//    the counted `s_waitcnt vmcnt(8)` never drains the ring inside the loop. (A first design staged whole
//    64-deep K tiles in 2 buffers; with its operand DMA removed it ran 1.72 PF/s at 8192^3 against 1.24 with
//    it: slabs issued one phase before use stalled it. See profiles/r02_gemm256.md.)
//  * Half-phase stagger: waves 4-7 (the partner of wave w on its SIMD is w + 4) run one barrier behind waves
//    0-3, so on every SIMD one wave's MFMA cluster overlaps its partner's LDS reads and DMA issue.
//  * LDS images are lane-linear (global_load_lds writes base + lane*16): bank-conflict swizzles are applied to
//    the per-lane SOURCE address and the same XOR on the read (rule 21). MN-major operands (dgrad's weight,
//    both wgrad operands) are read in place with ds_read_b64_tr_b16: no transposes anywhere.
//  * Operands swapped in the MFMA (B fragment as the instruction's A) so each lane holds 4 consecutive output
//    columns; a plain bf16 output is staged through LDS and written as whole 16-B row segments.
//  * XCD-aware bijective block remap + grouped (8 M-tiles) order: tiles sharing an A row panel / B column panel
//    run on one XCD's L2.
#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {

namespace g256 {

constexpr int THREADS = 512;

__device__ __forceinline__ int mn128_swz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

struct Epi {
  void* c;
  long ldc;
  const float* bias;  // [N] fp32 or null
  uint16_t* pre;      // bf16 pre-activation copy (GELU backward) or null
  int out_f32;
  int act;            // 0 none, 1 relu, 2 gelu(tanh)
  int accumulate;     // C += result
  float alpha;
  long slab;          // split-K: split z writes plain fp32 at c + z * slab (0: no split)
};

// GELU(tanh) = x * sigmoid(2u): v_exp_f32 + v_rcp_f32 (see gemm.hip's gelu_tanh)
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));
}

__device__ __forceinline__ void barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// ---- epilogue shared by both 256 x 256 kernels: wave (wr, wc) holds acc[a][j] = C[m][n..n+3] with
// m = m0 + wr*128 + a*16 + (lane & 15), n = n0 + wc*64 + j*16 + 4*(lane >> 4).
__device__ __forceinline__ void epilogue256(const f32x4_t (&acc)[8][4], const Epi& E, char* smem, int M, int N,
                                            int m0, int n0, int wid, int wr, int wc, int lane) {
  const float alpha = E.alpha;
  if (!E.out_f32 && !E.pre && !E.accumulate) {
    // bf16 tile through LDS: each wave stages its 128 x 64 piece (16 KB) and stores whole 128-B row segments.
    barrier();  // every wave is past its last LDS read of the K loop
    uint16_t* st = reinterpret_cast<uint16_t*>(smem) + wid * (128 * 64);  // [128 rows][64 cols], row 128 B
#pragma unroll
    for (int a = 0; a < 8; ++a) {
      const int lr = a * 16 + (lane & 15);  // wave-local row (ph*32 + i*16 == a*16)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int lc = j * 16 + 4 * (lane >> 4);
        const int n = n0 + wc * 64 + lc;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[a][j][r] * alpha;
          if (E.bias) v[r] += (n + r < N) ? E.bias[n + r] : 0.f;
          if (E.act == 1) v[r] = fmaxf(v[r], 0.f);
          else if (E.act == 2) v[r] = gelu_tanh(v[r]);
        }
        bf16x4_t o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
        // 16-B chunk (lc / 8) of row lr, XOR-swizzled by the row to spread the banks
        const int ch = (lc >> 3) ^ (lr & 7);
        *reinterpret_cast<bf16x4_t*>(reinterpret_cast<char*>(st) + lr * 128 + ch * 16 + (lc & 4) * 2) = o;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's staging writes landed (wave-private region)
    asm volatile("" ::: "memory");
    // 128 rows x 8 chunks of 16 B = 1024 chunks, 16 per lane
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int idx = it * 64 + lane;
      const int lr = idx >> 3, ch = idx & 7;
      const int m = m0 + wr * 128 + lr;
      const int n = n0 + wc * 64 + ch * 8;
      const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(reinterpret_cast<const char*>(st) + lr * 128 +
                                                            ((ch ^ (lr & 7)) << 4));
      if (m < M && n < N) {
        uint16_t* cp = reinterpret_cast<uint16_t*>(E.c) + (long)m * E.ldc + n;
        if (n + 8 <= N && (E.ldc & 7) == 0) {
          *reinterpret_cast<bf16x8_t*>(cp) = v;
        } else {
          for (int r = 0; r < 8 && n + r < N; ++r) cp[r] = (uint16_t)v[r];
        }
      }
    }
    return;
  }
  if (E.out_f32 && !E.pre && !E.bias && E.act == 0 && (E.ldc & 3) == 0) {
    // fp32 tile (the weight gradients, written or accumulated into the flat fp32 slots) through LDS in two
    // 64-row halves per wave (16 KB each, wave-private): the copy-out stores whole 256-B row segments (4 rows per
    // wave-instruction) instead of 16 rows x 64 B per instruction from the MFMA fragment layout.
    barrier();  // every wave is past its last LDS read of the K loop
    float* st = reinterpret_cast<float*>(smem) + wid * (64 * 64);  // [64 rows][64 cols], 256-B rows
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half) {
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of the first half are done
        asm volatile("" ::: "memory");
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int lr = a * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ch = (j * 4 + (lane >> 4)) ^ (lr & 15);  // 16-B chunk, XOR-swizzled by the row
          const f32x4_t v = acc[half * 4 + a][j] * alpha;
          *reinterpret_cast<f32x4_t*>(reinterpret_cast<char*>(st) + lr * 256 + ch * 16) = v;
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the staging writes landed (wave-private region)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int idx = it * 64 + lane;
        const int lr = idx >> 4, ch = idx & 15;
        const int m = m0 + wr * 128 + half * 64 + lr;
        const int n = n0 + wc * 64 + ch * 4;
        f32x4_t v = *reinterpret_cast<const f32x4_t*>(reinterpret_cast<const char*>(st) + lr * 256 +
                                                      ((ch ^ (lr & 15)) << 4));
        if (m < M && n < N) {  // N % 4 == 0 (gemm256_eligible)
          float* cp = reinterpret_cast<float*>(E.c) + (long)m * E.ldc + n;
          if (E.accumulate) v += *reinterpret_cast<const f32x4_t*>(cp);
          *reinterpret_cast<f32x4_t*>(cp) = v;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    const int m = m0 + wr * 128 + a * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wc * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= N) continue;
      const bool full = n + 3 < N;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[a][j][r] * alpha;
        if (E.bias) v[r] += (n + r < N) ? E.bias[n + r] : 0.f;
      }
      if (E.pre) {
        uint16_t* pp = E.pre + (long)m * E.ldc + n;
        if (full) {
          bf16x4_t o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
          *reinterpret_cast<bf16x4_t*>(pp) = o;
        } else {
          for (int r = 0; r < 4 && n + r < N; ++r) pp[r] = f2bf(v[r]);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (E.act == 1) v[r] = fmaxf(v[r], 0.f);
        else if (E.act == 2) v[r] = gelu_tanh(v[r]);
      }
      if (E.out_f32) {
        float* cp = reinterpret_cast<float*>(E.c) + (long)m * E.ldc + n;
        if (full) {
          float4 o = make_float4(v[0], v[1], v[2], v[3]);
          if (E.accumulate) {
            const float4 old = *reinterpret_cast<const float4*>(cp);
            o.x += old.x; o.y += old.y; o.z += old.z; o.w += old.w;
          }
          *reinterpret_cast<float4*>(cp) = o;
        } else {
          for (int r = 0; r < 4 && n + r < N; ++r) cp[r] = (E.accumulate ? cp[r] : 0.f) + v[r];
        }
      } else {
        uint16_t* cp = reinterpret_cast<uint16_t*>(E.c) + (long)m * E.ldc + n;
        if (full) {
          bf16x4_t o;
          if (E.accumulate) {
            const bf16x4_t old = *reinterpret_cast<const bf16x4_t*>(cp);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += bf2f((uint16_t)old[r]);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
          *reinterpret_cast<bf16x4_t*>(cp) = o;
        } else {
          for (int r = 0; r < 4 && n + r < N; ++r) cp[r] = f2bf(v[r] + (E.accumulate ? bf2f(cp[r]) : 0.f));
        }
      }
    }
  }
}

}  // namespace g256

// ============================================================================ the kernel
//   phase h: ds_read this wave's 8 A + 4 B fragments of stage h; issue stage h+3 into slot (h+3) % 5 (4 x 16 B
//   per thread); vmcnt(8) = stage h+1 landed (two younger stages stay in flight); barrier; 32 MFMAs; barrier.
//   RAW: stage h+1 is waited in phase h and read in phase h+1 (the barrier between makes every wave's DMA share
//   visible). WAR: slot (h+3) % 5 last held stage h-2, whose reads finished >= 2 phases earlier (safe under the
//   half-phase stagger, where one group runs one barrier behind the other).
// Images (lane-linear DMA, swizzles on the source address and the read):
//   K-major  [256 rows][32 k], 64-B rows: chunk c of row r at c ^ ((r >> 3) & 1) * 2 -> conflict-free b128 reads
//   MN-major 4 sub-images [32 k][64 mn], 128-B rows: 16-B unit u of k-row r at u ^ h(r),
//            h(r) = 2 * (((r >> 1) & 1) | ((r >> 3) & 1) << 1)        -> conflict-free ds_read_b64_tr_b16
namespace g256r {
constexpr int KS = 32;
constexpr int STAGE_A = 256 * KS * 2;  // 16 KB
constexpr int STAGE = 2 * STAGE_A;     // 32 KB
constexpr int NSLOT = 5;
constexpr int LDS_BYTES = NSLOT * STAGE;  // 160 KB

__device__ __forceinline__ int km_swz(int r) { return ((r >> 3) & 1) << 1; }

struct KMaj {
  const uint16_t* p;
  long ld;
  int rows;
  static constexpr bool kmajor = true;
  // glds j (0, 1) of thread tid: 16 B of row s >> 2, chunk (s & 3) ^ swz, s = j * 512 + tid
  __device__ __forceinline__ const uint16_t* cursor(int tid, int j, int o0) const {
    const int sl = j * 512 + tid, row = sl >> 2, c = (sl & 3) ^ km_swz(row);
    int r = o0 + row;
    r = r < rows ? r : rows - 1;
    return p + (long)r * ld + c * 8;
  }
  __device__ __forceinline__ long step() const { return KS; }
  // fragment in two steps: load() issues the LDS read, fin() yields the MFMA operand after the phase's wait
  using Raw = bf16x8_t;
  __device__ __forceinline__ static void load(Raw& r, const char* img, int rb, int lane) {
    const int row = rb + (lane & 15), c = lane >> 4;
    r = *reinterpret_cast<const bf16x8_t*>(img + row * 64 + ((c ^ km_swz(row)) << 4));
  }
  __device__ __forceinline__ static mfma_bf16x8 fin(const Raw& r) { return __builtin_bit_cast(mfma_bf16x8, r); }
};

struct MNMaj {
  const uint16_t* p;
  long ld;
  int cols;
  static constexpr bool kmajor = false;
  // glds j of thread tid fills sub-image 2j + (tid >> 8): k-row s >> 3, 16-B unit (s & 7) ^ h(k-row), s = tid & 255
  __device__ __forceinline__ const uint16_t* cursor(int tid, int j, int o0) const {
    const int sub = 2 * j + (tid >> 8), sl = tid & 255, kr = sl >> 3;
    const int lc = ((sl & 7) ^ g256::mn128_swz(kr)) * 8;
    int c = o0 + sub * 64 + lc;
    c = c < cols ? c : cols - 8;
    return p + (long)kr * ld + c;
  }
  __device__ __forceinline__ long step() const { return (long)KS * ld; }
  struct Raw {
    short4_t lo, hi;
  };
  // transposed reads as inline asm (see tr16_asm): the destinations are tied to the phase's lgkmcnt wait
  __device__ __forceinline__ static void load(Raw& r, const char* img, int rb, int lane) {
    const char* sub = img + (rb >> 6) * 4096;
    const int cb = rb & 63;
    const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
    const int u = (cb >> 3) + (pp >> 1);
    const int r0 = 8 * g + q, r1 = r0 + 4;
    tr16_asm(r.lo, sub + r0 * 128 + ((u ^ g256::mn128_swz(r0)) << 4) + (pp & 1) * 8);
    tr16_asm(r.hi, sub + r1 * 128 + ((u ^ g256::mn128_swz(r1)) << 4) + (pp & 1) * 8);
  }
  __device__ __forceinline__ static mfma_bf16x8 fin(const Raw& r) { return join8(r.lo, r.hi); }
};

// Ties every asm-read destination of a phase to one lgkmcnt(0) wait (no-op for compiler-read K-major frags).
template <class S, int N>
__device__ __forceinline__ void tie(typename S::Raw (&r)[N]) {
  if constexpr (!S::kmajor) {
    static_assert(N % 4 == 0, "tie groups of 4 fragments");
#pragma unroll
    for (int i = 0; i < N; i += 4)
      K8S_LDS_TIE8("s_waitcnt lgkmcnt(0)", r[i].lo, r[i].hi, r[i + 1].lo, r[i + 1].hi, r[i + 2].lo, r[i + 2].hi,
                   r[i + 3].lo, r[i + 3].hi);
  }
}

// XCD-aware bijective remap of block b of n (blocks b and b + 8 share an XCD): consecutive results share one
__device__ __forceinline__ int xcd_remap(int b, int n) {
  const int xcd = b & 7, q = n >> 3, r = n & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Stream-K tail (g256::Plan): blocks [0, full) each own one whole tile (the full waves); the remaining tiles are split
// `sk` ways along K, one block per (tile, split), so a 1.5-wave grid runs as 1 + 1/sk waves instead of 2.
struct SkArgs {
  int full;      // tiles computed whole (a multiple of the CU count), in tile order [0, full)
  int sk;        // K splits of each remaining tile (1: none)
  float* slabs;  // [tail tiles][sk][256 x 256] fp32 partials, fragment-native order
  int* sync;     // [tail tiles][1 + sk]: arrival ticket, then one published flag per split (self-resetting)
};

// Deterministic in-kernel split-K fix-up of one stream-K tile (cdna_hip_programming.md §5 "In-launch split-K
// reduction", §6 Guideline 16). Each split takes an arrival ticket FIRST; every split but the last arriver writes
// its fp32 partial (plain 16-B stores, fragment-native order: coalesced both ways), drains, and publishes it with an
// agent-scope release + a flag; the last arriver waits only for blocks that already took a ticket (they are running
// and never wait themselves: no residency assumption), acquires, and sums the partials in a FIXED order -- for two
// splits own + other (IEEE addition commutes: bit-identical whoever arrives last), for more splits every split's
// slab in split order (the reducer writes its own too) -- then resets the ticket and flags for the next launch and
// runs the normal epilogue. Returns true in the reducer (which goes on to the epilogue).
template <int NJ = 4, int NT = 512, int LDS = LDS_BYTES>
__device__ __forceinline__ bool sk_fixup(f32x4_t (&acc)[8][NJ], const SkArgs& SK, int slot, int split, char* smem,
                                      int tid) {
  const int sk = SK.sk;
  int* cnt = SK.sync + (long)slot * (1 + sk);
  int* flg = cnt + 1;
  int* bcast = reinterpret_cast<int*>(smem + LDS - 16);  // the K loop's reads are all done
  __syncthreads();
  if (tid == 0) bcast[0] = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool last = bcast[0] == sk - 1;
  // this tile's slabs through one buffer resource: the lane offset is one VGPR (tid * 16 B) and each 8 KB piece's
  // offset an SGPR, so the 32 stores / loads add no address registers next to the 128 accumulators
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(SK.slabs + (long)slot * sk * 65536, (short)0, sk * 262144, 0x00020000);
  const int voff = tid * 16;
  if (!last || sk > 2) {
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(acc[a][j], rs, voff, split * 262144 + (a * NJ + j) * NT * 16, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // keep: the compiler may drop the fence's own wait
      __hip_atomic_store(flg + split, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!last) return false;
  }
  if (tid == 0) {
    for (int z = 0; z < sk; ++z)
      if (z != split)
        while (__hip_atomic_load(flg + z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // slab reads in chunks of 8 x 16 B per lane (the sched_barrier keeps the compiler from hoisting all 32 loads of
  // a slab ahead of the adds: 128 more live VGPRs next to the accumulators would spill)
  for (int z = sk == 2 ? 1 - split : 0; z < sk; z += (sk == 2 ? 2 : 1)) {
    const bool assign = sk > 2 && z == 0;
#pragma unroll
    for (int a = 0; a < 8; a += 8 / NJ) {
      constexpr int R = 8 / NJ;  // accumulator rows per chunk: 8 loads of 16 B per lane
      f32x4_t v[R][NJ];
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          v[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, z * 262144 + ((a + i) * NJ + j) * NT * 16, 0);
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[a + i][j] = assign ? v[i][j] : acc[a + i][j] + v[i][j];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if (tid == 0) {  // every split has taken its ticket and published: reset for the next launch (stream-ordered)
    __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int z = 0; z < sk; ++z) __hip_atomic_store(flg + z, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return true;
}

template <class AS, class BS>
__global__ void __launch_bounds__(g256::THREADS, 2) gemm256r_kernel(AS A, BS B, g256::Epi E, int M, int N, int K,
                                                                   int kps, SkArgs SK) {
  using namespace g256;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int bid = blockIdx.x;
  int wg, split = 0, sk_slot = -1, ysplit = 0;
  if (gridDim.y > 1) {
    // tall-K split over blockIdx.y (no stream-K): remap the LINEAR dispatch id (XCD = id % 8) so every tile of one
    // split shares an XCD and the operand those tiles share is read once into its L2 (gemm.hip does the same)
    const int L = bid + gridDim.x * blockIdx.y;
    const int lam = xcd_remap(L, gridDim.x * gridDim.y);
    ysplit = lam / gridDim.x;
    wg = lam - ysplit * gridDim.x;
  } else if (bid < SK.full) {
    wg = xcd_remap(bid, SK.full);
  } else {  // stream-K tail: a tile's splits are consecutive after the remap, so they share an XCD's L2
    const int j = xcd_remap(bid - SK.full, gridDim.x - SK.full);
    sk_slot = j / SK.sk;
    split = j - sk_slot * SK.sk;
    wg = SK.full + sk_slot;
  }
  const int group = 8 * tiles_n;
  const int first_m = (wg / group) * 8;
  const int gm = min(tiles_m - first_m, 8);
  const int tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  const int m0 = tm * 256, n0 = tn * 256;

  // split-K: blockIdx.y (tall-K products, fp32 slabs combined by splitk_reduce) or the stream-K split; this block
  // reduces K range [koff, koff + kps)
  if (bid < SK.full && SK.sk > 1) kps = K;  // a whole tile of a stream-K launch: the full K range
  const long koff = (long)(ysplit + split) * kps;
  if (E.slab) E.c = reinterpret_cast<float*>(E.c) + ysplit * E.slab;
  const uint16_t* ca0 = A.cursor(tid, 0, m0) + (AS::kmajor ? koff : koff * A.ld);
  const uint16_t* ca1 = A.cursor(tid, 1, m0) + (AS::kmajor ? koff : koff * A.ld);
  const uint16_t* cb0 = B.cursor(tid, 0, n0) + (BS::kmajor ? koff : koff * B.ld);
  const uint16_t* cb1 = B.cursor(tid, 1, n0) + (BS::kmajor ? koff : koff * B.ld);
  const long sa = A.step(), sb = B.step();
  const int dma_off = wid * 1024;
  auto issue = [&](int slot) {
    char* d = smem + slot * STAGE + dma_off;
    glds16(ca0, d);
    glds16(ca1, d + 8192);
    glds16(cb0, d + STAGE_A);
    glds16(cb1, d + STAGE_A + 8192);
    ca0 += sa; ca1 += sa; cb0 += sb; cb1 += sb;
  };

  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)(min((long)K, koff + kps) - koff) / KS;
  issue(0);
  if (nk > 1) issue(1);
  if (nk > 2) issue(2);
  if (nk > 2) vmwait<8>();
  else if (nk > 1) vmwait<4>();
  else vmwait<0>();
  barrier();
  const bool lag = wr == 1;  // half-phase stagger (header)
  if (lag) barrier();

  int slot = 0, islot = 3;  // slot of stage h, slot for stage h + 3
  for (int h = 0; h < nk; ++h) {
    const char* st = smem + slot * STAGE;
    typename AS::Raw ar[8];
    typename BS::Raw br[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) BS::load(br[j], st + STAGE_A, wc * 64 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) AS::load(ar[i], st, wr * 128 + i * 16, lane);
    if (h + 3 < nk) {
      issue(islot);
      vmwait<8>();
    } else if (h + 2 < nk) {
      vmwait<4>();
    } else {
      vmwait<0>();
    }
    barrier();
    tie<BS>(br);
    tie<AS>(ar);
    mfma_bf16x8 afr[8], bfr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = BS::fin(br[j]);
#pragma unroll
    for (int i = 0; i < 8; ++i) afr[i] = AS::fin(ar[i]);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], afr[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    slot = slot == NSLOT - 1 ? 0 : slot + 1;
    islot = islot == NSLOT - 1 ? 0 : islot + 1;
  }
  if (!lag) barrier();
  if (sk_slot >= 0 && !sk_fixup(acc, SK, sk_slot, split, smem, tid)) return;
  epilogue256(acc, E, smem, M, N, m0, n0, wid, wr, wc, lane);
}
}  // namespace g256r


namespace g256 {
template <class AS, class BS>
static void launch_ring(const AS& a, const BS& b, const Epi& e, int M, int N, int K, int splits,
                        const Gemm256Plan& plan, float* sk_slabs, int* sk_sync, hipStream_t st) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int kps = K / splits;  // a multiple of 64 (gemm256_choose_splits)
  int blocks = tiles;
  if (splits == 1 && plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  const dim3 grid(blocks, splits);
  hipLaunchKernelGGL((g256r::gemm256r_kernel<AS, BS>), grid, dim3(THREADS), 0, st, a, b, e, M, N, K, kps, sk);
}

}  // namespace g256

// ============================================================================ 4-wave kernel
// Every operand layout (K-major rows, or MN-major through the ring kernel's MNMaj sub-images and ds_read_b64_tr_b16)
// with a plain bf16 or fp32 (stored / accumulated) output -- the forward, data-gradient and weight-gradient products
// of the transformer linears whose grids fill the chip -- on the schedule hipBLASLt's MT256x256x64 kernel
// uses on gfx950 (its disassembly: 4 waves, 128 MFMAs + 32 ds_read_b128 + 16 LDS-DMA per 64-deep stage, 2 stages,
// accumulators in AGPRs). The ring kernel above reached 0.78-0.85x hipBLASLt on the forward form
// (profiles/r04_gemm_all_vs_hipblaslt.jsonl) with 2x its L2 requests -- its 32-deep stages read half cache lines
// of a K-major row per DMA piece; it keeps the products outside this kernel's contract (w4_ok).
//  * 256 threads = 4 waves as 2 x 2, each wave a 128 x 128 piece = 8 x 8 tiles of v_mfma_f32_16x16x32_bf16: 0.25
//    LDS reads per MFMA (the 8-wave ring: 0.375). The 64 accumulators live in AGPRs: the MFMAs are inline asm with
//    "+a" operands (the builtin's register choice moved the 256 accumulator registers between AGPRs and VGPRs every
//    phase in a first 4-wave version, 0.97 vs 1.25 PF/s).
//  * 64-deep stages (A 256 x 64 + B 256 x 64 = 64 KB), 2 in LDS; a K-major row's 64 k are one 128-B line, an
//    MN-major k-row's 64 columns of a sub-image too, read by 8 lanes of one DMA instruction. Stage s + 2 is issued
//    in the half after the barrier in the middle of stage s, a whole stage (128 MFMAs per wave, one wave per SIMD)
//    ahead of its wait.
//  * fragments double-buffered in VGPRs: the next k-half read while this half's 64 MFMAs run; the transposed reads
//    of MN-major operands are inline asm (the builtin draws a vmcnt(0) drain in front of it) tied to an explicit
//    lgkmcnt(0) at each half's end.
//  * K-major LDS images [256 rows][64 k], 128-B rows, 16-B chunk c of row r at c ^ (r & 6): conflict-free
//    ds_read_b128 for 16-row fragment groups (the conv3x3 swizzle); a lane's row & 6 is lane & 6, so every fragment
//    address is one of two per-lane bases plus an immediate.
//  * stream-K tail (gemm256_plan) with a slab-sum epilogue; bf16 output staged through LDS in 16-B row segments,
//    fp32 output (stored or accumulated) straight from the fragments.
namespace g4 {
constexpr int THREADS = 256, KS = 64;
constexpr int STAGE_A = 256 * KS * 2;  // 32 KB
constexpr int STAGE = 2 * STAGE_A;     // 64 KB
constexpr int LDS_BYTES = 2 * STAGE;   // 128 KB

#define K8S_G4_MFMA(acc, b, a) \
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a))

// X: the transformer linears' bf16 epilogue extras -- bias (fp32, added before the one rounding of the staged
// value), ReLU / GELU of the staged pre-activation, its copy to `pre` (what the activation backward reads) and a bf16
// accumulate (C = result + old C; a residual's second gradient contribution) -- in the row-contiguous copy-out. Its
// own instantiation so the plain kernels keep their code and registers.
// Tall-K split (gridDim.y > 1, the weight gradients of outputs with fewer tiles than CUs): split y reduces K range
// [y kps, min(K, (y + 1) kps)) into the fp32 slab at C + y * slab (plain store), combined by splitk_reduce; the last
// split may be shorter, so the split count is free to fill the chip (9 BERT tiles x 28 splits = 252 blocks).
// GELU(tanh) of 8 values, 2 at a time on the packed fp32 ALU (v_pk_mul / v_pk_fma): x * 1 / (1 + 2^(c (x + k1 x^3)))
__device__ __forceinline__ void gelu8(float (&f)[8]) {
  const f32x2_t k1 = {0.044715f, 0.044715f};
  const f32x2_t c = {-2.8853900817779268f * 0.7978845608028654f, -2.8853900817779268f * 0.7978845608028654f};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f32x2_t x = {f[2 * p], f[2 * p + 1]};
    const f32x2_t u = __builtin_elementwise_fma(x * x * k1, x, x) * c;
    const f32x2_t d = {1.f + __builtin_amdgcn_exp2f(u[0]), 1.f + __builtin_amdgcn_exp2f(u[1])};
    const f32x2_t y = x * f32x2_t{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    f[2 * p] = y[0];
    f[2 * p + 1] = y[1];
  }
}

// the X copy-out (8 groups of 4 chunks of this wave's staged 128 x 128 tile): pre-activation copy, ACT (0 none, 1 ReLU,
// 2 GELU) and ACC (C = result + old C, the old C of group g + 1 loaded before group g is processed, so each group
// waits for loads issued a group earlier)
// d/dx GELU(tanh) (elementwise.hip's act_bwd form: t = tanh(k0 (x + k1 x^3)) on v_exp / v_rcp)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(2.8853900817779268f * k0 *
                                                                                  (x + k1 * x * x * x)));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
}

// f *= GELU'(x) for 8 values, 2 at a time on the packed fp32 ALU (the gelu_tanh_grad formula)
__device__ __forceinline__ void gelu_grad_mul8(float (&f)[8], const float (&xs)[8]) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const f32x2_t one = {1.f, 1.f}, half = {0.5f, 0.5f};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f32x2_t x = {xs[2 * p], xs[2 * p + 1]};
    const f32x2_t x2 = x * x;
    const f32x2_t u = x * __builtin_elementwise_fma(x2, f32x2_t{k1, k1}, one) *
                      f32x2_t{2.8853900817779268f * k0, 2.8853900817779268f * k0};  // 2 log2(e) k0 (x + k1 x^3)
    const f32x2_t d = {1.f + __builtin_amdgcn_exp2f(u[0]), 1.f + __builtin_amdgcn_exp2f(u[1])};
    const f32x2_t r = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    const f32x2_t t = __builtin_elementwise_fma(r, f32x2_t{-2.f, -2.f}, one);  // tanh
    const f32x2_t a = __builtin_elementwise_fma(t, half, half);
    const f32x2_t b = x * __builtin_elementwise_fma(-t, t, one) * __builtin_elementwise_fma(x2, f32x2_t{3.f * k1, 3.f * k1}, one) *
                      f32x2_t{0.5f * k0, 0.5f * k0};
    const f32x2_t y = f32x2_t{f[2 * p], f[2 * p + 1]} * (a + b);
    f[2 * p] = y[0];
    f[2 * p + 1] = y[1];
  }
}

// ACT < 0: the data gradient of a linear whose input is an activation's output, fused with that activation's
// backward (-1 ReLU: `pre` holds the ReLU output; -2 GELU: the pre-activation): C = dgrad * act'(pre), and the
// per-column sums of the stored bf16 C (the producing linear's bias gradient) -- this wave's 128 columns summed over
// its 128 rows into one partial row of `cpart` (folded by colsum_fold_kernel). `pre` is read a group ahead, as the
// accumulate's old C.
// ACT = -3: SwiGLU backward (Llama's down-projection data gradient): C / pre are the [M][2F] dgu / gu buffers
// (ldc = 2F), the GEMM's N = F columns are the gate half; with d = this data gradient, g = gate (pre at off), u = up
// (pre at off + fo): dgate = d u silu'(g) at off, dup = d silu(g) at off + fo -- elementwise.hip's swiglu_bwd_kernel
// formula on the same bf16 inputs, so the fused result is bit-identical to the two-pass one.
template <int ACT, bool ACC, class Off, class Stg>
__device__ __forceinline__ void copy_out_x(uint16_t* __restrict__ C, uint16_t* __restrict__ pre, const char* stg,
                                           const Off& coff, const Stg& staged, float* __restrict__ cpart = nullptr,
                                           long fo = 0) {
  (void)stg;
  static_assert(!(ACT < 0 && ACC), "activation backward without accumulate");
  constexpr bool RD = ACC || ACT < 0;  // a bf16 operand per chunk read a group ahead (old C, or pre)
  constexpr bool SW = ACT == -3;
  bf16x8_t oldc[2][4], oldu[SW ? 2 : 1][SW ? 4 : 1];
  const uint16_t* rsrc = ACT < 0 ? pre : C;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (RD) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      oldc[0][q] = *reinterpret_cast<const bf16x8_t*>(rsrc + coff(q));
      if constexpr (SW) oldu[0][q] = *reinterpret_cast<const bf16x8_t*>(rsrc + coff(q) + fo);
    }
  }
#pragma unroll
  for (int grp = 0; grp < 8; ++grp) {
    if constexpr (RD) {
      if (grp + 1 < 8) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          oldc[(grp + 1) & 1][q] = *reinterpret_cast<const bf16x8_t*>(rsrc + coff((grp + 1) * 4 + q));
          if constexpr (SW)
            oldu[(grp + 1) & 1][q] = *reinterpret_cast<const bf16x8_t*>(rsrc + coff((grp + 1) * 4 + q) + fo);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int it = grp * 4 + q;
      const long off = coff(it);
      bf16x8_t v = staged(it);
      if constexpr (SW) {
        float dg[8], du[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float gg = bf2f((uint16_t)oldc[grp & 1][q][r]), uu = bf2f((uint16_t)oldu[grp & 1][q][r]);
          const float d = bf2f((uint16_t)v[r]);
          const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-gg));
          du[r] = d * (gg * sg);
          dg[r] = d * uu * (sg * (1.f + gg * (1.f - sg)));
        }
        *reinterpret_cast<bf16x8_t*>(C + off) = pack_bf16x8(dg);
        *reinterpret_cast<bf16x8_t*>(C + off + fo) = pack_bf16x8(du);
        continue;
      } else if constexpr (ACT < 0) {
        float f[8], x[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          x[r] = bf2f((uint16_t)oldc[grp & 1][q][r]);
          f[r] = bf2f((uint16_t)v[r]);
        }
        if constexpr (ACT == -1) {
#pragma unroll
          for (int r = 0; r < 8; ++r) f[r] = x[r] > 0.f ? f[r] : 0.f;
        } else {
          gelu_grad_mul8(f, x);
        }
        v = pack_bf16x8(f);
#pragma unroll
        for (int r = 0; r < 8; ++r) cs[r] += bf2f((uint16_t)v[r]);
        *reinterpret_cast<bf16x8_t*>(C + off) = v;
        continue;
      }
      if (pre) *reinterpret_cast<bf16x8_t*>(pre + off) = v;  // the staged pre-activation (bias included)
      if constexpr (ACT != 0 || ACC) {
        float f[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) f[r] = bf2f((uint16_t)v[r]);
        if constexpr (ACT == 1) {
#pragma unroll
          for (int r = 0; r < 8; ++r) f[r] = fmaxf(f[r], 0.f);
        } else if constexpr (ACT == 2) {
          gelu8(f);
        }
        if constexpr (ACC) {  // one more bf16 rounding on top of the staged value (<= 1 ulp), as gemm.hip's lean path
#pragma unroll
          for (int r = 0; r < 8; ++r) f[r] += bf2f((uint16_t)oldc[grp & 1][q][r]);
        }
        v = pack_bf16x8(f);
      }
      *reinterpret_cast<bf16x8_t*>(C + off) = v;
    }
  }
  if constexpr (ACT < 0 && !SW) {
    // lanes l, l ^ 16, l ^ 32, l ^ 48 hold the same 8 columns (chunk l & 15) of different rows
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      cs[r] += __shfl_xor(cs[r], 16);
      cs[r] += __shfl_xor(cs[r], 32);
    }
    if ((threadIdx.x & 63) < 16) {
      float* d = cpart + (threadIdx.x & 15) * 8;
#pragma unroll
      for (int r = 0; r < 8; ++r) d[r] = cs[r];
    }
  }
}

// ACT = 3: the gate|up projection with its SwiGLU in the epilogue (Llama). The weight's rows are laid out in blocks of
// 64 gate rows then the 64 matching up rows, so each wave's staged 128 columns hold gate block b in columns 0-63 and up
// block b in 64-127 (the rotate-half pairing of copy_out_rope): chunk c's partner is chunk c + 8 of the same staged
// row, no other wave's piece is read and no barrier is needed. Every wave stores its staged piece to C (= gu [M][2F],
// what the backward reads), then h = silu(g) u (elementwise.hip swiglu_fwd_kernel's formula on the same bf16 inputs:
// bit-identical) to `hout` [M][F] at column (n0 + wc 128) / 2 -- the separate SwiGLU pass (read gu, write h) is gone.
template <class Off, class Stg>
__device__ __forceinline__ void copy_out_swiglu(uint16_t* __restrict__ C, uint16_t* __restrict__ hout, const char* stg,
                                                const Off& coff, const Stg& staged, int row0, int hcol0, int N) {
  const int lane = threadIdx.x & 63;
#pragma unroll 4
  for (int it = 0; it < 32; ++it) *reinterpret_cast<bf16x8_t*>(C + coff(it)) = staged(it);
  const long F = N / 2;
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 64 + lane, lr = idx >> 3, c = idx & 7;
    const bf16x8_t g = *reinterpret_cast<const bf16x8_t*>(stg + lr * 256 + ((c ^ (lr & 15)) << 4));
    const bf16x8_t u = *reinterpret_cast<const bf16x8_t*>(stg + lr * 256 + (((c + 8) ^ (lr & 15)) << 4));
    float h[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float gg = bf2f((uint16_t)g[r]);
      h[r] = gg * __builtin_amdgcn_rcpf(1.f + __expf(-gg)) * bf2f((uint16_t)u[r]);
    }
    *reinterpret_cast<bf16x8_t*>(hout + (long)(row0 + lr) * F + hcol0 + c * 8) = pack_bf16x8(h);
  }
}

// ACT = 4: the QKV projection with the rotary embedding of its q / k heads in the copy-out (Llama). A wave's staged
// 128 columns are exactly one head of D = 128; the rotate-half partner of chunk ch (8 columns) is chunk ch ^ 8 of the
// same staged row, the angle table row is pos[row]. elementwise.hip rope_kernel's formula (explicit fmas, the same
// rounding), so the fused output is bit-identical to the projection + the in-place rope pass it replaces. `rot`: this
// wave's head is a q / k head (columns < rcols); the v heads are stored as staged.
__device__ __forceinline__ void copy_out_rope(uint16_t* __restrict__ C, const char* stg, long cbase, long ldc,
                                              bool rot, const int* __restrict__ rpos, const float* __restrict__ rtab,
                                              int row0) {
  const int lane = threadIdx.x & 63;
  if (!rot) {
#pragma unroll 4
    for (int it = 0; it < 32; ++it) {
      const int idx = it * 64 + lane, lr = idx >> 4, ch = idx & 15;
      *reinterpret_cast<bf16x8_t*>(C + cbase + lr * ldc + ch * 8) =
          *reinterpret_cast<const bf16x8_t*>(stg + lr * 256 + ((ch ^ (lr & 15)) << 4));
    }
    return;
  }
  // each lane rotates one (x1 chunk c, x2 chunk c + 8) pair of a row: one table read and one LDS read per operand
#pragma unroll 2
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 64 + lane, lr = idx >> 3, c = idx & 7;
    const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(stg + lr * 256 + ((c ^ (lr & 15)) << 4));
    const bf16x8_t w = *reinterpret_cast<const bf16x8_t*>(stg + lr * 256 + (((c + 8) ^ (lr & 15)) << 4));
    const f32x4_t* tb = reinterpret_cast<const f32x4_t*>(rtab + ((long)rpos[row0 + lr] * 64 + c * 8) * 2);
    float o1[8], o2[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4_t t = tb[q];  // (cos, sin) of elements 2q, 2q + 1
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float cs = t[2 * e], sn = t[2 * e + 1];
        const float x1 = bf2f((uint16_t)v[2 * q + e]), x2 = bf2f((uint16_t)w[2 * q + e]);
        o1[2 * q + e] = __builtin_fmaf(x1, cs, -(x2 * sn));  // rope_kernel's formula
        o2[2 * q + e] = __builtin_fmaf(x2, cs, x1 * sn);
      }
    }
    uint16_t* d = C + cbase + lr * ldc + c * 8;
    *reinterpret_cast<bf16x8_t*>(d) = pack_bf16x8(o1);
    *reinterpret_cast<bf16x8_t*>(d + 64) = pack_bf16x8(o2);
  }
}

// ACT = 5: the BatchNorm statistics of the stored bf16 values (per-column sum / sum of squares -- the conv epilogue
// statistics of gemm.hip, [kConvStatReplicas][2][N]) for ResNet's deep-reduction 1x1 convolutions. Every lane keeps the
// sums of its fixed 8 columns (chunk lane & 15) over its rows; lanes l, l ^ 16, l ^ 32, l ^ 48 are folded by shuffles,
// each wave parks its 128 + 128 partials at the head of its own (already copied-out) staged region, and after one
// barrier thread t adds the two wave rows' partials of column t % 128 of wave column t / 128: 2 full-wave atomic
// instructions per wave.
template <class Off, class Stg>
__device__ __forceinline__ void copy_out_stats(uint16_t* __restrict__ C, float* __restrict__ stats, char* smem,
                                               char* stg, const Off& coff, const Stg& staged, int rep, int N, int n0) {
  const int lane = threadIdx.x & 63;
  float sm[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, sq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int it = 0; it < 32; ++it) {
    const bf16x8_t v = staged(it);
    *reinterpret_cast<bf16x8_t*>(C + coff(it)) = v;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float f = bf2f((uint16_t)v[r]);
      sm[r] += f;
      sq[r] = __builtin_fmaf(f, f, sq[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    sm[r] += __shfl_xor(sm[r], 16);
    sm[r] += __shfl_xor(sm[r], 32);
    sq[r] += __shfl_xor(sq[r], 16);
    sq[r] += __shfl_xor(sq[r], 32);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's staged reads are done: reuse its region
  if (lane < 16) {
    float* part = reinterpret_cast<float*>(stg);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      part[lane * 8 + r] = sm[r];
      part[128 + lane * 8 + r] = sq[r];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g256::barrier();
  const int t = threadIdx.x, wcol = t >> 7, c = t & 127;
  const float* p0 = reinterpret_cast<const float*>(smem + (0 * 2 + wcol) * 32768);  // wave (wr 0, wc)
  const float* p1 = reinterpret_cast<const float*>(smem + (1 * 2 + wcol) * 32768);  // wave (wr 1, wc)
  float* d = stats + (long)rep * 2 * N + n0 + wcol * 128 + c;
  atomicAdd(d, p0[c] + p1[c]);
  atomicAdd(d + N, p0[128 + c] + p1[128 + c]);
}

// ACT = 6 (a data gradient dx = dy . w): the BatchNorm-backward sums of dx for the relu(BN(x)) that produced the
// convolution's input (launchers.h BnBwdSums): g = relu_on(x) ? dx : 0, sums[rep][0][c] += sum g, [1][c] += sum g (x -
// mean). x is read at the output positions (same layout), in two halves of 16 rows per lane, each half's loads issued
// before the previous half is consumed; tab = [gamma | beta | mean | invstd] fp32 [4][N].
template <class Off, class Stg>
__device__ __forceinline__ void copy_out_bnbwd(uint16_t* __restrict__ C, const uint16_t* __restrict__ x,
                                               const float* __restrict__ tab, float* __restrict__ sums, char* smem,
                                               char* stg, const Off& coff, const Stg& staged, int rep, int N,
                                               int n0, int col0) {
  const int lane = threadIdx.x & 63, col = col0 + (lane & 15) * 8;
  float sc[8], sh[8], mu[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    mu[r] = tab[2 * N + col + r];
    bn_affine_regs(tab[col + r], tab[N + col + r], mu[r], tab[3 * N + col + r], sc[r], sh[r]);
  }
  float sm[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, sq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  bf16x8_t xv[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) xv[it] = *reinterpret_cast<const bf16x8_t*>(x + coff(it));
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const bf16x8_t v = staged(it);
    *reinterpret_cast<bf16x8_t*>(C + coff(it)) = v;
    const bf16x8_t xx = xv[it & 15];
    if (it < 16) xv[it] = *reinterpret_cast<const bf16x8_t*>(x + coff(it + 16));
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float xf = bf2f((uint16_t)xx[r]);
      const float g = relu_on(xf, sc[r], sh[r]) ? bf2f((uint16_t)v[r]) : 0.f;
      sm[r] += g;
      sq[r] = __builtin_fmaf(g, xf - mu[r], sq[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    sm[r] += __shfl_xor(sm[r], 16);
    sm[r] += __shfl_xor(sm[r], 32);
    sq[r] += __shfl_xor(sq[r], 16);
    sq[r] += __shfl_xor(sq[r], 32);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's staged reads are done: reuse its region
  if (lane < 16) {
    float* part = reinterpret_cast<float*>(stg);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      part[lane * 8 + r] = sm[r];
      part[128 + lane * 8 + r] = sq[r];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  g256::barrier();
  const int t = threadIdx.x, wcol = t >> 7, c = t & 127;
  const float* p0 = reinterpret_cast<const float*>(smem + (0 * 2 + wcol) * 32768);  // wave (wr 0, wc)
  const float* p1 = reinterpret_cast<const float*>(smem + (1 * 2 + wcol) * 32768);  // wave (wr 1, wc)
  float* d = sums + (long)rep * 2 * N + n0 + wcol * 128 + c;
  atomicAdd(d, p0[c] + p1[c]);
  atomicAdd(d + N, p0[128 + c] + p1[128 + c]);
}

template <bool AMN, bool BMN, bool X>
__global__ void __launch_bounds__(THREADS, 1) gemm_w4_kernel(const uint16_t* __restrict__ A, long lda,
                                                             const uint16_t* __restrict__ B, long ldb, void* Cv,
                                                             long ldc, int M, int N, int K, float alpha, int kps,
                                                             g256r::SkArgs SK, int out_f32, int accumulate,
                                                             const float* __restrict__ bias, int act,
                                                             uint16_t* __restrict__ pre, long slab,
                                                             float* __restrict__ cpart, const int* __restrict__ rpos,
                                                             const float* __restrict__ rtab, int rcols) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const int tiles_m = M >> 8, tiles_n = N >> 8;
  // whole tiles [0, SK.full), then the stream-K tail: (tile, split) pairs of K range kps (as gemm256r_kernel)
  const int bid = blockIdx.x;
  int wg, split = 0, sk_slot = -1;
  if (gridDim.y > 1) {  // tall-K split: the linear (tile, split) id remapped so a split's tiles share an XCD
    const int lam = g256r::xcd_remap(bid + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    split = lam / gridDim.x;
    wg = lam - split * gridDim.x;
    Cv = reinterpret_cast<float*>(Cv) + (long)split * slab;
  } else if (bid < SK.full) {
    wg = g256r::xcd_remap(bid, SK.full);
    kps = K;
  } else {
    const int j = g256r::xcd_remap(bid - SK.full, gridDim.x - SK.full);
    sk_slot = j / SK.sk;
    split = j - sk_slot * SK.sk;
    wg = SK.full + sk_slot;
  }
  const long koff = (long)split * kps;
  const int group = 8 * tiles_n;
  const int first_m = (wg / group) * 8;
  const int gm = min(tiles_m - first_m, 8);
  const int m0 = (first_m + (wg % group) % gm) * 256, n0 = ((wg % group) / gm) * 256;

  // DMA (buffer_load ... lds: the per-instruction row offset in an SGPR, no per-lane address arithmetic):
  // instruction q = wid + 4 i of an operand's stage covers rows 8 q .. 8 q + 7 (1 KB of LDS); lane l loads row
  // 8 q + l / 8, logical chunk (l & 7) ^ (row & 6) = (l & 7) ^ ((l >> 3) & 6)
  const int drow = wid * 8 + (lane >> 3), lch = (lane & 7) ^ ((lane >> 3) & 6);
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(AMN ? A + koff * lda + m0 : A + (long)m0 * lda + koff), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(BMN ? B + koff * ldb + n0 : B + (long)n0 * ldb + koff), (short)0, 0x7fffffff, 0x00020000);
  const int va = AMN ? ((drow * (int)lda) + (((lane & 7) ^ g256::mn128_swz(drow)) * 8)) * 2
                     : (drow * (int)lda + lch * 8) * 2;
  // B MN-major ([K][N], the data gradient's weight): the stage is 8 sub-images [32 k][64 n] (k-half p >> 2, column
  // block p & 3) of 128-B rows, 16-B unit u of k-row r at u ^ h(r) (the ring kernel's MNMaj image, read by
  // ds_read_b64_tr_b16). Piece p of wave w is sub-image p's k-rows 8 w .. 8 w + 7: lane l loads k-row 8 w + l / 8,
  // unit (l & 7) ^ h(that row) -- per wave, one lane offset.
  const int vb = BMN ? ((drow * (int)ldb) + (((lane & 7) ^ g256::mn128_swz(drow)) * 8)) * 2
                     : (drow * (int)ldb + lch * 8) * 2;
  const int sa = 64 * (int)lda, sb = 64 * (int)ldb;  // K-major: bytes between instruction i and i + 1 (32 rows)
  // piece p (0-7: A instruction p, 8-15: B instruction p - 8) of stage t into buffer dbuf
  auto dma = [&](int p, int t, int dbuf) {
    char* d = smem + dbuf * STAGE + wid * 1024 + (p & 7) * 4096 + (p >> 3) * STAGE_A;
    auto* l = (__attribute__((address_space(3))) void*)d;
    if (p < 8) {
      if constexpr (AMN)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, l, 16, va, ((p >> 2) * 32 * (int)lda + (p & 3) * 64) * 2 +
                                                                     t * (KS * 2) * (int)lda, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, l, 16, va, p * sa + t * (KS * 2), 0, 0);
    } else if constexpr (BMN) {
      const int q = p - 8;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, l, 16, vb, ((q >> 2) * 32 * (int)ldb + (q & 3) * 64) * 2 +
                                                                   t * (KS * 2) * (int)ldb, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, l, 16, vb, (p - 8) * sb + t * (KS * 2), 0, 0);
    }
  };
  // B MN-major fragment j of k-half kk (ring kernel's MNMaj::load): two transposed reads at k-rows r0 = 8 g + q_
  // and r0 + 4 of sub-image (2 wc + j / 4), unit 2 (j & 3) + pp / 2; the per-lane parts precomputed for j & 3
  int bmo[2][4], amo[2][4];  // (A MN-major: the same with the wave's rows, sub-image 2 wr + f / 4)
  {
    const int li_ = lane & 15, q_ = li_ >> 2, pp = li_ & 3, r0 = 8 * (lane >> 4) + q_;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = r0 + 4 * h;
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4) {
        const int u = (((2 * j4 + (pp >> 1)) ^ g256::mn128_swz(r)) << 4) + (pp & 1) * 8 + r * 128;
        bmo[h][j4] = STAGE_A + wc * 2 * 4096 + u;
        amo[h][j4] = wr * 2 * 4096 + u;
      }
    }
  }
  // fragment f of the wave's A piece: row wr * 128 + 16 f + (lane & 15), chunk 4 kk + (lane >> 4)
  const int li = lane & 15, g = lane >> 4, sw = lane & 6;
  const int ra = (wr * 128 + li) * 128, rb = STAGE_A + (wc * 128 + li) * 128;
  const int co0 = (g ^ sw) << 4, co1 = ((4 + g) ^ sw) << 4;
  auto frag = [&](int buf, int kk, int off) {
    return __builtin_bit_cast(
        mfma_bf16x8, *reinterpret_cast<const bf16x8_t*>(smem + buf * STAGE + (kk ? co1 : co0) + off));
  };

  f32x4_t acc[8][8];
#pragma unroll
  for (int f = 0; f < 8; ++f)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[f][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // MFMAs [lo, hi) of the 64 on (af, bf): after MFMA x with x % 4 == 1 the next k-half's fragment x / 4 is read
  // into (na, nb) when `rd` (the eight B fragments first: the next half's first eight MFMAs use all of them), after
  // x % 4 == 3 DMA piece x / 4 of stage `dt` is issued into buffer `dbuf` when `dm`. An LDS-DMA piece costs its wave
  // 60-185 issue cycles beside MFMAs (MI355X_MICROARCH constants table): spread one per four MFMAs the 16 pieces ran
  // 5-7 % faster than packed one per two MFMAs into the half's second quarter (gate_up 730 -> 677 us, same box;
  // moving the A pieces into the first halves measured slower again, 691 -> 722). rd_c / dm_c are
  // std::integral_constant<bool, ...>, so the sequence carries no branches.
  short4_t blo[8], bhi[8], alo[8], ahi[8];  // MN-major operands: the next k-half's raw transposed reads (tied and
                                           // joined after a wait)
  auto tra = [&](int nbuf, int nkk, int f, int h) {
    tr16_asm(h ? ahi[f] : alo[f], smem + nbuf * STAGE + nkk * 16384 + (f >> 2) * 4096 + amo[h][f & 3]);
  };
  auto trb = [&](int nbuf, int nkk, int j, int h) {
    tr16_asm(h ? bhi[j] : blo[j], smem + nbuf * STAGE + nkk * 16384 + (j >> 2) * 4096 + bmo[h][j & 3]);
  };
  auto mm = [&](int lo, int hi, const mfma_bf16x8 (&af)[8], const mfma_bf16x8 (&bf)[8], mfma_bf16x8 (&na)[8],
                mfma_bf16x8 (&nb)[8], auto rd_c, int nbuf, int nkk, auto dm_c, int dt, int dbuf) {
    constexpr bool rd = decltype(rd_c)::value, dm = decltype(dm_c)::value;
#pragma unroll
    for (int x = lo; x < hi; ++x) {
      K8S_G4_MFMA(acc[x >> 3][x & 7], bf[x & 7], af[x >> 3]);
      const int k = x >> 2;
      if constexpr (rd) {
        if constexpr (AMN && BMN) {  // 32 transposed reads, one after each MFMA of the first half (A, then B)
          if (x < 32) {
            if (x < 16) tra(nbuf, nkk, x >> 1, x & 1);
            else trb(nbuf, nkk, (x - 16) >> 1, x & 1);
          }
        } else if constexpr (BMN) {  // 16 transposed B reads after the odd MFMAs of the first half, 8 A reads after
          if ((x & 1) && x < 32) trb(nbuf, nkk, x >> 2, (x >> 1) & 1);
          if ((x & 3) == 1 && x >= 32) na[k - 8] = frag(nbuf, nkk, ra + (k - 8) * 2048);
        } else if constexpr (AMN) {  // 16 transposed A reads after the odd MFMAs of the first half, 8 B reads after
          if ((x & 1) && x < 32) tra(nbuf, nkk, x >> 2, (x >> 1) & 1);
          if ((x & 3) == 1 && x >= 32) nb[k - 8] = frag(nbuf, nkk, rb + (k - 8) * 2048);
        } else if ((x & 3) == 1) {
          if (k < 8) nb[k] = frag(nbuf, nkk, rb + k * 2048);
          else na[k - 8] = frag(nbuf, nkk, ra + (k - 8) * 2048);
        }
      }
      if constexpr (dm) {
        if ((x & 3) == 3) dma(k, dt, dbuf);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // MN-major operands: after an lgkmcnt(0) wait, make the raw transposed reads MFMA operands (tied to the wait)
  auto joins = [&](mfma_bf16x8 (&na)[8], mfma_bf16x8 (&nb)[8]) {
    if constexpr (AMN) {
      K8S_LDS_TIE8("", alo[0], alo[1], alo[2], alo[3], alo[4], alo[5], alo[6], alo[7]);
      K8S_LDS_TIE8("", ahi[0], ahi[1], ahi[2], ahi[3], ahi[4], ahi[5], ahi[6], ahi[7]);
#pragma unroll
      for (int f = 0; f < 8; ++f) na[f] = join8(alo[f], ahi[f]);
    }
    if constexpr (BMN) {
      K8S_LDS_TIE8("", blo[0], blo[1], blo[2], blo[3], blo[4], blo[5], blo[6], blo[7]);
      K8S_LDS_TIE8("", bhi[0], bhi[1], bhi[2], bhi[3], bhi[4], bhi[5], bhi[6], bhi[7]);
#pragma unroll
      for (int j = 0; j < 8; ++j) nb[j] = join8(blo[j], bhi[j]);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  const int nst = (int)(((long)K - koff < kps ? (long)K - koff : (long)kps) / KS);  // a tall-K split's last range
  // X: this lane's bias columns (4 per 16-wide block j), loaded once here and held through the K loop -- loaded per
  // fragment in the epilogue, each load's wait was exposed 64 times per tile (QKV forward 31 us per tile vs 26.5)
  f32x4_t bj[X ? 8 : 1];
  if constexpr (X) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      bj[j] = bias ? *reinterpret_cast<const f32x4_t*>(bias + n0 + wc * 128 + j * 16 + 4 * (lane >> 4))
                   : f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(p, 0, 0);
  if (nst > 1) {
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(p, 1, 1);
    g256::vmwait<16>();  // stage 0 landed, stage 1 in flight
  } else {
    g256::vmwait<0>();
  }
  g256::barrier();
  mfma_bf16x8 a0[8], b0[8], a1[8], b1[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    if constexpr (AMN) {
      tra(0, 0, f, 0);
      tra(0, 0, f, 1);
    } else {
      a0[f] = frag(0, 0, ra + f * 2048);
    }
    if constexpr (BMN) {
      trb(0, 0, f, 0);
      trb(0, 0, f, 1);
    } else {
      b0[f] = frag(0, 0, rb + f * 2048);
    }
  }
  if constexpr (AMN || BMN) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    joins(a0, b0);
  }
  // first k-half of stage s (+ its second half's reads), the stage's hand-over -- stage s + 1 landed and visible,
  // every wave done with stage s's buffer -- with the last two MFMAs of the half around it
  auto first = [&](int s) {
    mm(0, 62, a0, b0, a1, b1, T_{}, s & 1, 1, F_{}, 0, 0);
    g256::vmwait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    joins(a1, b1);
    mm(62, 63, a0, b0, a1, b1, F_{}, 0, 0, F_{}, 0, 0);
    g256::barrier();
    mm(63, 64, a0, b0, a1, b1, F_{}, 0, 0, F_{}, 0, 0);
  };
  auto second_done = [&]() {  // MN-major operands: the next first half's fragments
    if constexpr (AMN || BMN) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      joins(a0, b0);
    }
  };
  int s = 0;
  for (; s + 2 < nst; ++s) {
    first(s);
    mm(0, 64, a1, b1, a0, b0, T_{}, (s & 1) ^ 1, 0, T_{}, s + 2, s & 1);  // + stage s + 1's reads, stage s + 2's DMA
    second_done();
  }
  if (s + 1 < nst) {  // stage nst - 2: no DMA left
    first(s);
    mm(0, 64, a1, b1, a0, b0, T_{}, (s & 1) ^ 1, 0, F_{}, 0, 0);
    second_done();
    ++s;
  }
  mm(0, 64, a0, b0, a1, b1, T_{}, s & 1, 1, F_{}, 0, 0);  // the last stage
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  joins(a1, b1);
  mm(0, 64, a1, b1, a0, b0, F_{}, 0, 0, F_{}, 0, 0);

  // stream-K tail: every split stores its fp32 partial (fragment-native order, the slab layout of sk_fixup), takes a
  // ticket and publishes; the last arriver sums the tile's slabs in split order inside the epilogue -- fixed order,
  // so bit-identical whoever arrives last. The accumulators are only read here (updating them in place would pull
  // all 256 out of the AGPRs).
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      SK.slabs + (long)(sk_slot < 0 ? 0 : sk_slot) * SK.sk * 65536, (short)0, SK.sk * 262144, 0x00020000);
  if (sk_slot >= 0) {
    const int sk = SK.sk;
    int* cnt = SK.sync + (long)sk_slot * (1 + sk);
    int* flg = cnt + 1;
    int* bcast = reinterpret_cast<int*>(smem + LDS_BYTES - 16);
#pragma unroll
    for (int f = 0; f < 8; ++f)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(acc[f][j], srs, tid * 16, split * 262144 + (f * 8 + j) * THREADS * 16,
                                               0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // also: every wave is past its last fragment read (bcast lives in the stage buffers)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(flg + split, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bcast[0] = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (bcast[0] != sk - 1) return;
    if (tid == 0) {  // the others published before taking their tickets
      for (int z = 0; z < sk; ++z)
        while (__hip_atomic_load(flg + z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reset for the next launch
      for (int z = 0; z < sk; ++z) __hip_atomic_store(flg + z, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  if (out_f32) {  // fp32 (the weight gradients, stored or accumulated into the flat slots): straight from the
                  // fragments, 16 B per lane (4 lanes = one 64-B row piece)
    float* C = reinterpret_cast<float*>(Cv);
#pragma unroll
    for (int f = 0; f < 8; ++f) {
      const long m = m0 + wr * 128 + f * 16 + li;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        f32x4_t v = acc[f][j];
        if (sk_slot >= 0) {
          v = __builtin_amdgcn_raw_buffer_load_b128(srs, tid * 16, (f * 8 + j) * THREADS * 16, 0);
          for (int z = 1; z < SK.sk; ++z)
            v += __builtin_amdgcn_raw_buffer_load_b128(srs, tid * 16, z * 262144 + (f * 8 + j) * THREADS * 16, 0);
        }
        v *= alpha;
        f32x4_t* cp = reinterpret_cast<f32x4_t*>(C + m * ldc + n0 + wc * 128 + j * 16 + 4 * g);
        if (accumulate) v += *cp;
        *cp = v;
      }
    }
    return;
  }
  uint16_t* C = reinterpret_cast<uint16_t*>(Cv);
  // epilogue: each wave stages its 128 x 128 bf16 piece (32 KB, wave-private; 256-B rows, 16-B chunk c of row r at
  // c ^ (r & 15)) and stores whole 16-B row segments
  g256::barrier();  // every wave is past its last fragment read
  char* stg = smem + wid * 32768;
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    const int lr = f * 16 + li;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int lc = j * 16 + 4 * g;
      f32x4_t v = acc[f][j];
      if (sk_slot >= 0) {
        v = __builtin_amdgcn_raw_buffer_load_b128(srs, tid * 16, (f * 8 + j) * THREADS * 16, 0);
        for (int z = 1; z < SK.sk; ++z)
          v += __builtin_amdgcn_raw_buffer_load_b128(srs, tid * 16, z * 262144 + (f * 8 + j) * THREADS * 16, 0);
      }
      f32x4_t b4 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (X) b4 = bj[j];
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(__builtin_fmaf(v[r], alpha, b4[r]));
      *reinterpret_cast<bf16x4_t*>(stg + lr * 256 + (((lc >> 3) ^ (lr & 15)) << 4) + (lc & 4) * 2) = o;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private region: no barrier needed
  auto coff = [&](int it) {
    const int idx = it * 64 + lane, lr = idx >> 4, ch = idx & 15;
    return (long)(m0 + wr * 128 + lr) * ldc + n0 + wc * 128 + ch * 8;
  };
  auto staged = [&](int it) {
    const int idx = it * 64 + lane, lr = idx >> 4, ch = idx & 15;
    return *reinterpret_cast<const bf16x8_t*>(stg + lr * 256 + ((ch ^ (lr & 15)) << 4));
  };
  if (!X || (act == 0 && !accumulate && !pre)) {  // (a bias alone was added while staging: the plain copy)
#pragma unroll 4
    for (int it = 0; it < 32; ++it) *reinterpret_cast<bf16x8_t*>(C + coff(it)) = staged(it);
  } else if constexpr (X) {
    // the activation and the accumulate are compile-time in the loop body (copy_out<ACT, ACC>): with them as run-time
    // values the compiler branched per ELEMENT and serialised every GELU chain (exp -> add -> rcp -> mul, s_nop
    // between): BERT-base's FFN1 forward took 1013 us against 543 us for the bias-only QKV forward of 3/4 its FLOPs
    if (act < 0) {  // activation backward (data-gradient form only): a partial row of column sums per (tile, wave row)
      if constexpr (!AMN && BMN) {
        if (act == -3) {  // SwiGLU backward: no column sums; the up half `slab` columns to the right
          copy_out_x<-3, false>(C, pre, stg, coff, staged, nullptr, slab);
        } else if (act == -4) {  // the same on the 64-blocked gate|up layout (copy_out_swiglu): h column j is gate
                                 // column (j / 64) 128 + j % 64, its up column 64 further
          auto coff_b = [&](int it) {
            const int idx = it * 64 + lane, lr = idx >> 4, ch = idx & 15;
            return (long)(m0 + wr * 128 + lr) * ldc + 2 * (n0 + wc * 128) + (ch >> 3) * 128 + (ch & 7) * 8;
          };
          copy_out_x<-3, false>(C, pre, stg, coff_b, staged, nullptr, 64);
        } else {
          float* const cp = cpart + (long)((m0 >> 8) * 2 + wr) * N + n0 + wc * 128;
          if (act == -2) copy_out_x<-2, false>(C, pre, stg, coff, staged, cp);
          else copy_out_x<-1, false>(C, pre, stg, coff, staged, cp);
        }
      }
    } else if (act == 3) {
      copy_out_swiglu(C, pre, stg, coff, staged, m0 + wr * 128, (n0 + wc * 128) / 2, N);
    } else if (act == 5) {
      copy_out_stats(C, cpart, smem, stg, coff, staged, (m0 >> 8) % kConvStatReplicas, N, n0);
    } else if (act == 6) {
      copy_out_bnbwd(C, pre, rtab, cpart, smem, stg, coff, staged, (m0 >> 8) % kConvStatReplicas, N, n0,
                     n0 + wc * 128);
    } else if (act == 4) {
      copy_out_rope(C, stg, (long)(m0 + wr * 128) * ldc + n0 + wc * 128, ldc, n0 + wc * 128 < rcols, rpos, rtab,
                    m0 + wr * 128);
    } else if (act == 2) {
      if (accumulate) copy_out_x<2, true>(C, pre, stg, coff, staged); else copy_out_x<2, false>(C, pre, stg, coff, staged);
    } else if (act == 1) {
      if (accumulate) copy_out_x<1, true>(C, pre, stg, coff, staged); else copy_out_x<1, false>(C, pre, stg, coff, staged);
    } else {
      if (accumulate) copy_out_x<0, true>(C, pre, stg, coff, staged); else copy_out_x<0, false>(C, pre, stg, coff, staged);
    }
  }
}
#undef K8S_G4_MFMA
}  // namespace g4

// The 4-wave kernel's contract: any operand layout, whole 256 x 256 tiles (M, N % 256), K % 64, 16-B aligned rows;
// a bf16 output with the X extras (bias / ReLU / GELU / pre-activation copy / bf16 accumulate) or an fp32 one (stored or
// accumulated, alpha allowed); at least one wave of tiles (a partial last wave takes the stream-K tail) -- or, as a
// tall-K split of a plain fp32 product, one wave of (tile, split) blocks. $K8S_AMD_GEMM_W4=0 keeps such products on
// the ring kernel (A/B; read per call, both sides tested).
static bool w4_enabled() {
  const char* e = getenv("K8S_AMD_GEMM_W4");
  return !(e && e[0] == '0');
}
static bool w4_ok(bool a_kmajor, bool b_kmajor, bool c_f32, int M, int N, int K, long lda, long ldb, long ldc,
                  const float* bias, int act, const uint16_t* pre, bool accumulate, int splits, int sk) {
  if (!w4_enabled()) return false;
  (void)sk;
  (void)a_kmajor;  // every operand layout: K-major (read as rows) or MN-major (transposed reads)
  (void)b_kmajor;
  const bool extras = bias || act != 0 || pre || (accumulate && !c_f32);
  if (c_f32 && extras) return false;             // fp32 outputs: plain store / accumulate
  if (reinterpret_cast<uintptr_t>(bias) % 16 != 0) return false;  // the epilogue reads the bias as 16-B vectors
  if (splits > 1 && (!c_f32 || accumulate)) return false;  // split slabs: plain fp32 stores
  if (M % 256 != 0 || N % 256 != 0 || K % 64 != 0 || (lda | ldb | ldc) % 8 != 0) return false;
  const long tiles = (long)(M / 256) * (N / 256);
  return splits > 1 ? tiles * splits >= 3L * planner_cus() / 4 : tiles >= planner_cus();
}
// K range per split of a tall-K split on the 4-wave kernel (whole 64-deep stages; the last split takes the rest)
static int w4_split_kps(int K, int splits) { return (K / 64 + splits - 1) / splits * 64; }

// Data gradient fused with the backward of the activation that produced the GEMM's input (see copy_out_x, ACT < 0):
// C[M][N] = (A . B) * act'(pre), db[N] = column sums of C (fp32, written or added), A K-major [M][K], B [K][N]
// (the linear's weight). 4-wave kernel shapes only (w4_dact_ok); `part` holds (M / 128) x N floats.
bool gemm_w4_dact_ok(int M, int N, int K, long lda, long ldb, long ldc) {
  return w4_enabled() && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && (lda | ldb | ldc) % 8 == 0 &&
         (long)(M / 256) * (N / 256) >= planner_cus();
}
long gemm_w4_dact_part_floats(int M, int N) { return (long)(M / 128) * N; }
void launch_gemm_w4_dact(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* C, long ldc, int M, int N,
                         int K, const uint16_t* pre, int act, float* part, float* db, bool db_accumulate,
                         float* sk_slabs, int* sk_sync, hipStream_t st) {
  if (!gemm_w4_dact_ok(M, N, K, lda, ldb, ldc) || (act != 1 && act != 2) || ldc != N)
    throw std::runtime_error("gemm_w4_dact: shape / activation outside the 4-wave kernel's contract");
  Gemm256Plan plan = gemm256_plan(M, N, K);
  if (!sk_slabs || !sk_sync) plan.sk = 1;
  const int tiles = (M / 256) * (N / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int blocks = tiles, kps = K;
  if (plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  hipLaunchKernelGGL((g4::gemm_w4_kernel<false, true, true>), dim3(blocks), dim3(g4::THREADS), 0, st, A, lda, B, ldb,
                     (void*)C, ldc, M, N, K, 1.f, kps, sk, 0, 0, nullptr, -act, const_cast<uint16_t*>(pre), 0L, part,
                     nullptr, nullptr, 0);
  launch_colsum_fold(part, M / 128, N, db, db_accumulate, st);
}

// Llama's down-projection data gradient fused with the SwiGLU backward (copy_out_x ACT = -3): dgu [M][2F] from
// g [M][K] (K-major) . w [K][F] (MN-major) and gu [M][2F]; the 4-wave kernel's whole-tile shapes (N = F).
bool gemm_w4_swiglu_ok(int M, int F, int K, long lda, long ldb) {
  return gemm_w4_dact_ok(M, F, K, lda, ldb, 2L * F);
}
void launch_gemm_w4_swiglu_bwd(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* dgu,
                               const uint16_t* gu, int M, int F, int K, int blk, float* sk_slabs, int* sk_sync,
                               hipStream_t st) {
  if (!gemm_w4_swiglu_ok(M, F, K, lda, ldb) || (blk != 0 && blk != 64))
    throw std::runtime_error("gemm_w4_swiglu_bwd: shape outside the 4-wave kernel's contract");
  Gemm256Plan plan = gemm256_plan(M, F, K);
  if (!sk_slabs || !sk_sync) plan.sk = 1;
  const int tiles = (M / 256) * (F / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int blocks = tiles, kps = K;
  if (plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  // C = dgu (row stride 2F, gate half at column 0), pre = gu, slab = F: the up half's column offset (blk = 64: the
  // blocked layout, act -4)
  hipLaunchKernelGGL((g4::gemm_w4_kernel<false, true, true>), dim3(blocks), dim3(g4::THREADS), 0, st, A, lda, B, ldb,
                     (void*)dgu, 2L * F, M, F, K, 1.f, kps, sk, 0, 0, nullptr, blk ? -4 : -3,
                     const_cast<uint16_t*>(gu), (long)F, nullptr, nullptr, nullptr, 0);
}

// Llama's gate|up projection with the SwiGLU in the epilogue (copy_out_swiglu): gu [M][2F] = A [M][K] . B [2F][K]^T
// (both K-major; B's rows in the 64-blocked gate|up order) and h [M][F] = silu(gate) up. Whole 256 x 256 tiles.
bool gemm_w4_swiglu_fwd_ok(int M, int F, int K, long lda, long ldb) {
  return w4_enabled() && M % 256 == 0 && F % 128 == 0 && K % 64 == 0 && (lda | ldb) % 8 == 0 &&
         (long)(M / 256) * (2 * F / 256) >= planner_cus();  // (2F % 256: whole tiles, each 2 gate|up block pairs)
}
void launch_gemm_w4_swiglu_fwd(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* gu, uint16_t* h,
                               int M, int F, int K, float* sk_slabs, int* sk_sync, hipStream_t st) {
  if (!gemm_w4_swiglu_fwd_ok(M, F, K, lda, ldb))
    throw std::runtime_error("gemm_w4_swiglu_fwd: shape outside the 4-wave kernel's contract");
  const int N = 2 * F;
  Gemm256Plan plan = gemm256_plan(M, N, K);
  if (!sk_slabs || !sk_sync) plan.sk = 1;
  const int tiles = (M / 256) * (N / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int blocks = tiles, kps = K;
  if (plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  hipLaunchKernelGGL((g4::gemm_w4_kernel<false, false, true>), dim3(blocks), dim3(g4::THREADS), 0, st, A, lda, B, ldb,
                     (void*)gu, (long)N, M, N, K, 1.f, kps, sk, 0, 0, nullptr, 3, h, 0L, nullptr, nullptr, nullptr, 0);
}

// Llama's QKV projection with the rotary embedding of the q / k heads (columns < rot_cols, head dim 128) in the
// copy-out (copy_out_rope): y [M][N] = A [M][K] . B [N][K]^T, both K-major; pos [M] int32, table [maxpos][64][2].
bool gemm_w4_rope_ok(int M, int N, int K, long lda, long ldb, int rot_cols) {
  return w4_enabled() && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && (lda | ldb) % 8 == 0 && rot_cols % 128 == 0 &&
         rot_cols <= N && (long)(M / 256) * (N / 256) >= planner_cus();
}
void launch_gemm_w4_rope(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* y, int M, int N, int K,
                         const int* pos, const float* table, int rot_cols, float* sk_slabs, int* sk_sync,
                         hipStream_t st) {
  if (!gemm_w4_rope_ok(M, N, K, lda, ldb, rot_cols))
    throw std::runtime_error("gemm_w4_rope: shape outside the 4-wave kernel's contract");
  Gemm256Plan plan = gemm256_plan(M, N, K);
  if (!sk_slabs || !sk_sync) plan.sk = 1;
  const int tiles = (M / 256) * (N / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int blocks = tiles, kps = K;
  if (plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  hipLaunchKernelGGL((g4::gemm_w4_kernel<false, false, true>), dim3(blocks), dim3(g4::THREADS), 0, st, A, lda, B, ldb,
                     (void*)y, (long)N, M, N, K, 1.f, kps, sk, 0, 0, nullptr, 4, nullptr, 0L, nullptr, pos, table,
                     rot_cols);
}

// ResNet's deep-reduction 1x1 convolution forwards with the BatchNorm statistics epilogue (copy_out_stats):
// y [M][N] = x [M][K] . w [N][K]^T, stats [kConvStatReplicas][2][N] (zeroed by the caller). $K8S_AMD_W4_STATS=0 keeps
// them on the 128 x 128 tile kernel (A/B; read per call); K8S_AMD_W4_STATS_MINK (default 512) is the smallest
// reduction taken.
bool gemm_w4_stats_ok(int M, int N, int K) {
  const char* e = getenv("K8S_AMD_W4_STATS");
  if (e && e[0] == '0') return false;
  const char* mk = getenv("K8S_AMD_W4_STATS_MINK");
  const int mink = mk ? atoi(mk) : 512;
  return w4_enabled() && K >= mink && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 &&
         (long)(M / 256) * (N / 256) >= planner_cus();
}
void launch_gemm_w4_stats(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* y, int M, int N, int K,
                          float* stats, float* sk_slabs, int* sk_sync, hipStream_t st) {
  Gemm256Plan plan = gemm256_plan(M, N, K);
  if (!sk_slabs || !sk_sync) plan.sk = 1;
  const int tiles = (M / 256) * (N / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int blocks = tiles, kps = K;
  if (plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  hipLaunchKernelGGL((g4::gemm_w4_kernel<false, false, true>), dim3(blocks), dim3(g4::THREADS), 0, st, A, lda, B, ldb,
                     (void*)y, (long)N, M, N, K, 1.f, kps, sk, 0, 0, nullptr, 5, nullptr, 0L, stats, nullptr, nullptr,
                     0);
}

// A data gradient dx [M][N] = dy [M][K] . w [K][N] (w stored MN-major, the 1x1 convolution's [Kout][Cin]) with the
// BatchNorm-backward sums of dx in the epilogue (copy_out_bnbwd); whole 256 x 256 tiles, stream-K tail with a workspace.
bool gemm_w4_dgrad_bnstats_ok(int M, int N, int K) {
  return w4_enabled() && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && (long)(M / 256) * (N / 256) >= planner_cus();
}
void launch_gemm_w4_dgrad_bnstats(const uint16_t* A, const uint16_t* B, uint16_t* y, int M, int N, int K,
                                  const uint16_t* x, const float* tab, float* sums, float* sk_slabs, int* sk_sync,
                                  hipStream_t st) {
  if (!gemm_w4_dgrad_bnstats_ok(M, N, K)) throw std::runtime_error("w4 dgrad BatchNorm sums: outside the contract");
  Gemm256Plan plan = gemm256_plan(M, N, K);
  if (!sk_slabs || !sk_sync) plan.sk = 1;
  const int tiles = (M / 256) * (N / 256);
  g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
  int blocks = tiles, kps = K;
  if (plan.sk > 1) {
    sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
    kps = plan.kps;
    blocks = plan.full + (tiles - plan.full) * plan.sk;
  }
  hipLaunchKernelGGL((g4::gemm_w4_kernel<false, true, true>), dim3(blocks), dim3(g4::THREADS), 0, st, A, (long)K, B,
                     (long)N, (void*)y, (long)N, M, N, K, 1.f, kps, sk, 0, 0, nullptr, 6, const_cast<uint16_t*>(x), 0L,
                     sums, nullptr, tab, 0);
}

// Stream-K tail plan for a grid of 256 x 256 tiles on P = planner_cus() CUs (one block per CU; 256 on MI355X): with
// T = w * P + r tiles and 0 < r <= P / 2, the last r tiles are split sk = min(P / r, 4) ways along K (each split a multiple of 64 deep and
// >= 512), so the tail costs ~1/sk of a wave (+ the fix-up) instead of a whole one. Not for grids of 8+ waves (the
// tail is then a small fraction) or when the split would be too shallow.
Gemm256Plan gemm256_plan(int M, int N, int K) {
  Gemm256Plan p;
  p.tiles = ((M + 255) / 256) * ((N + 255) / 256);
  p.full = p.tiles;
  p.sk = 1;
  p.kps = K;
  const int P = planner_cus();
  const int waves = p.tiles / P, r = p.tiles % P;
  // sub-wave grids (waves == 0, e.g. BERT's M = 8192 x N = 768 products, 96 tiles) stay on the 128 x 128 kernel:
  // split 2 ways onto this kernel they measured 72-82 us per call in the BERT step against 51-62 us there
  // (profiles/r04_bert_b64.md, first run)
  if (r == 0 || waves == 0 || waves >= 8 || r > P / 2) return p;
  const char* e = getenv("K8S_AMD_GEMM256_SK");  // =0: no stream-K tail (A/B knob, read per call; tests run both)
  if (e && e[0] == '0') return p;
  int s = std::min(P / r, 4);
  while (s > 1 && (K % (64 * s) != 0 || K / s < 512)) --s;
  if (s > 1) {
    p.full = waves * P;
    p.sk = s;
    p.kps = K / s;
  }
  return p;
}
long gemm256_sk_slab_floats(const Gemm256Plan& p) { return p.sk > 1 ? (long)(p.tiles - p.full) * p.sk * 65536 : 0; }
long gemm256_sk_sync_ints(const Gemm256Plan& p) { return p.sk > 1 ? (long)(p.tiles - p.full) * (1 + p.sk) : 0; }

// Shape gate for the 256 x 256 kernel: K >= 768 and a multiple of 64, MN-major extents multiples of 8, and a wave-
// quantisation cost model against the 128 x 128 kernel of gemm.hip (2 blocks/CU). Per output element the 256
// kernel runs ~1.25x the 128 kernel's rate (measured, scripts/bench_gemm256.py), but with one 256-tile per CU
// a 1.5-wave grid (e.g. 384 tiles) idles a third of the chip in its last round:
//   t256 ~ ceil(T256 / 256) * 256^2 / 1.25     t128 ~ ceil(T128 / 512) * 2 * 128^2
bool gemm256_eligible(int M, int N, int K, bool a_kmajor, bool b_kmajor) {
  // short reductions (ResNet's 1x1 convolutions as GEMMs, K = 64..512) leave the 5-stage ring mostly in its
  // prologue/epilogue; the 128 x 128 kernel's single-buffered 3-blocks/CU variant is built for them
  if (K % 64 != 0) return false;
  if (K < 768) {
    // K = 512 (8 stages): the 4-wave kernel's 2-stage pipeline, not the ring, when it takes the whole-tile grid --
    // K8S_AMD_GEMM256_MINK (default 768: off) for the A/B
    const char* e = getenv("K8S_AMD_GEMM256_MINK");
    const int mink = e ? atoi(e) : 768;
    if (K < mink || !w4_enabled() || M % 256 != 0 || N % 256 != 0 ||
        (long)(M / 256) * (N / 256) < planner_cus())
      return false;
  }
  if (!a_kmajor && M % 8 != 0) return false;
  if (!b_kmajor && N % 8 != 0) return false;
  if (N % 4 != 0) return false;
  const Gemm256Plan plan = gemm256_plan(M, N, K);
  const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
  const long P = planner_cus();
  // waves of P tiles, the stream-K tail counted as 1/sk of a wave (+5 % for its fix-up)
  const double w256 = plan.sk > 1 ? plan.full / P + 1.05 / plan.sk : (double)((plan.tiles + P - 1) / P);
  const double c256 = w256 * 65536.0 / 1.25;
  const double c128 = (double)((t128 + 2 * P - 1) / (2 * P)) * 32768.0;
  return c256 <= c128;
}

// Split-K for the tall-K fp32 products (weight gradients of small output, e.g. ResNet's 1x1 layers: 256 x 1024
// outputs over 200k pixels): the smallest split count that puts >= 192 blocks on the chip, each split a multiple of
// 64 deep and >= 1024 (the ring's prologue / epilogue), at most 64 splits. 1 when the tiles alone fill the chip.
// ("Fill" = 3/4 of planner_cus(): 192 blocks on MI355X's 256 CUs.)
int gemm256_choose_splits(int M, int N, int K) {
  const long tiles = (long)((M + 255) / 256) * ((N + 255) / 256);
  const long fill = 3L * planner_cus() / 4;
  if (w4_enabled() && M % 256 == 0 && N % 256 == 0 && K % 64 == 0) {
    // the 4-wave kernel takes uneven splits: as many as fit one wave of (tile, split) blocks at one block per CU,
    // each >= 512 deep (8 stages) -- BERT-base's weight gradients at 131k tokens: 9 tiles x 28, 27 x 9, 36 x 7
    long s = planner_cus() / tiles;
    s = s > 64 ? 64 : s;
    while (s > 1 && K / s < 512) --s;
    if (s >= 2 && tiles * s >= fill) {  // (w4_ok's split condition)
      const int kps = w4_split_kps(K, (int)s);
      return (K + kps - 1) / kps;  // splits actually launched (every one non-empty)
    }
    if (tiles >= fill) return 1;
  }
  int best = 1;
  for (int s = 2; s <= 64; ++s) {
    if (tiles * (s / 2) >= fill) break;  // the previous s already filled the chip
    if (K % (64 * s) != 0 || K / s < 1024) continue;
    best = s;
    if (tiles * s >= fill) break;
  }
  return best;
}

void launch_gemm256(const uint16_t* A, long lda, bool a_kmajor, const uint16_t* B, long ldb, bool b_kmajor, void* C,
                    long ldc, bool c_f32, int M, int N, int K, const float* bias, int act, uint16_t* pre,
                    bool accumulate, float alpha, hipStream_t st, int splits, float* ws, float* sk_slabs,
                    int* sk_sync) {
  if (K % 64 != 0) throw std::runtime_error("gemm256: K must be a multiple of 64");
  if (splits < 1) splits = 1;
  if (splits > 1 && (!c_f32 || bias || act || pre || !ws || ldc != N))
    throw std::runtime_error("gemm256 split-K: plain fp32 output and a workspace");
  g256::Epi e{splits > 1 ? (void*)ws : C, ldc, bias, pre, c_f32 ? 1 : 0, act, (splits == 1 && accumulate) ? 1 : 0,
              alpha, splits > 1 ? (long)M * N : 0};
  Gemm256Plan plan = gemm256_plan(M, N, K);
  if (splits > 1 || !sk_slabs || !sk_sync) plan.sk = 1;  // tall-K split, or no stream-K workspace given
  using namespace g256r;
  if (w4_ok(a_kmajor, b_kmajor, c_f32, M, N, K, lda, ldb, ldc, bias, act, pre, splits > 1 ? false : accumulate,
            splits, plan.sk)) {
    const int tiles = (M / 256) * (N / 256);
    g256r::SkArgs sk{tiles, 1, nullptr, nullptr};
    int blocks = tiles, kps = K, ysplits = 1;
    if (splits > 1) {  // tall-K split: slabs of ws, then splitk_reduce (which also applies `accumulate`)
      kps = w4_split_kps(K, splits);
      ysplits = (K + kps - 1) / kps;
    } else if (plan.sk > 1) {  // the stream-K tail (gemm256_plan), fixed up in-kernel as in the ring kernel
      sk = g256r::SkArgs{plan.full, plan.sk, sk_slabs, sk_sync};
      kps = plan.kps;
      blocks = plan.full + (tiles - plan.full) * plan.sk;
    }
    const bool x = bias || act != 0 || pre || (accumulate && !c_f32);
    void* const cv = splits > 1 ? (void*)ws : C;
    const int acc = splits > 1 ? 0 : (accumulate ? 1 : 0);
#define K8S_W4L(AM, BM, XX)                                                                                         \
  hipLaunchKernelGGL((g4::gemm_w4_kernel<AM, BM, XX>), dim3(blocks, ysplits), dim3(g4::THREADS), 0, st, A, lda, B, \
                     ldb, cv, ldc, M, N, K, alpha, kps, sk, c_f32 ? 1 : 0, acc, bias, act, pre, (long)M * N, nullptr,   \
                     nullptr, nullptr, 0)
#define K8S_W4X(AM, BM)       \
  do {                        \
    if (x)                    \
      K8S_W4L(AM, BM, true);  \
    else                      \
      K8S_W4L(AM, BM, false); \
  } while (0)
    if (a_kmajor && b_kmajor) K8S_W4X(false, false);
    else if (a_kmajor) K8S_W4X(false, true);
    else if (b_kmajor) K8S_W4X(true, false);
    else K8S_W4X(true, true);
#undef K8S_W4X
#undef K8S_W4L
    if (splits > 1) splitk_reduce(ws, ysplits, (long)M * N, reinterpret_cast<float*>(C), accumulate, st);
    return;
  }
  while (splits > 1 && K % (64 * splits) != 0) --splits;  // the ring kernel takes even splits only (ws holds more)
  e.slab = splits > 1 ? (long)M * N : 0;
  if (splits == 1) {
    e.c = C;
    e.accumulate = accumulate ? 1 : 0;
  }
  if (a_kmajor && b_kmajor)
    g256::launch_ring(KMaj{A, lda, M}, KMaj{B, ldb, N}, e, M, N, K, splits, plan, sk_slabs, sk_sync, st);
  else if (a_kmajor && !b_kmajor)
    g256::launch_ring(KMaj{A, lda, M}, MNMaj{B, ldb, N}, e, M, N, K, splits, plan, sk_slabs, sk_sync, st);
  else if (!a_kmajor && b_kmajor)
    g256::launch_ring(MNMaj{A, lda, M}, KMaj{B, ldb, N}, e, M, N, K, splits, plan, sk_slabs, sk_sync, st);
  else
    g256::launch_ring(MNMaj{A, lda, M}, MNMaj{B, ldb, N}, e, M, N, K, splits, plan, sk_slabs, sk_sync, st);
  if (splits > 1) splitk_reduce(ws, splits, (long)M * N, reinterpret_cast<float*>(C), accumulate, st);
}

}  // namespace k8s_amd
