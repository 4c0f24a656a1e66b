// K5: flash attention forward / backward for gfx950 (bf16 in, fp32 softmax/accumulate).
//
// Layout: token-major q [B, Sq, Hq, D], k/v [B, Sk, Hkv, D] with arbitrary batch / token / head
// strides (q, k, v are usually column slices of one fused QKV GEMM output -- no copies), D in
// {64, 128}, GQA (Hq % Hkv == 0), causal (bottom-right aligned) and per-batch key lengths.
//
// Forward (one block = 4 waves = 128 queries, KV tiles of 64 keys, double-buffered in LDS via
// global_load_lds):
//   S^T = K . Q^T    MFMA(first = K fragment, second = Q fragment held in VGPRs): each lane ends
//                    with ONE query (lane & 15) and 4 keys per 16-key subtile.
//   online softmax   per query column: row max = in-lane max + 2 xor-shuffles; the running sum
//                    stays lane-partial until the end (exp2 domain, scale * log2(e) folded in).
//   O^T += V^T . P^T P^T is consumed straight from the S^T accumulators: the MFMA's k order is
//                    permuted (keys 4g..4g+3 | 16+4g..16+4g+3 for lane group g) and V^T is read
//                    with the SAME permutation through ds_read_b64_tr_b16 -- no register shuffle,
//                    no LDS round trip for P.
//   writes O (bf16) and lse2 = m + log2(l) (fp32, [B, Hq, Sq]) for the backward.
//   (Round 3 measured two 8-wave v_mfma_f32_32x32x16_bf16 forwards against this kernel at Llama-3-8B s4096 D128:
//   one phase per 64-key tile, register-staged K/V -- 519 TF/s causal / 829 non-causal vs 596 / 833; and a
//   ping-pong with group B one barrier behind group A so the softmax VALU of one wave overlaps its partner's PV
//   MFMAs -- 519 / 787 vs 667 / 842 after the masking fix below. Neither kept. Later in round 3, same-box A/Bs:
//   8-wave / 256-query blocks (each K/V tile staged once per 256 queries) with a 3-stage ring 258 us causal / 312 us
//   non-causal, with 2 stages 235 / 291, vs this kernel 205 / 302 (scripts/gpurun/r3_attn7.sh); the row sums of P
//   on the matrix cores (ones^T P^T, 4 extra MFMAs per tile instead of 32 v_add_f32) measured neutral; an
//   unconditional rescale (one basic block per tile for the scheduler) 196 / 305 vs 188-194 / 294 us. Round 4: a
//   software pipeline over the full tiles -- S(t+1) = K(t+1) Q^T computed next to tile t's softmax, K streamed one tile
//   ahead of V in the same 64 KB -- spilled at D = 128 (a second S tile beside 233 VGPRs) and at D = 64 ran slower
//   on every shape: BERT s128 16 vs 13 us, s512 32 vs 26.5 us, Llama-1B s2048 84 vs 74.5 us (same box, alternating
//   processes, scripts/gpurun/r4/fapipe.sh); not kept.)
//
// Backward (FA2 order, dK/dV kernel: one block = 64 keys of one KV head, looping over every query tile
// of every query head of its GQA group, so dK/dV accumulate in VGPRs without atomics):
//   S = Q K^T, dP = dO V^T       (K, V fragments of the wave's 16 keys stay in VGPRs)
//   P = exp2(S*c - lse2), dS = P (dP - delta)
//   dV^T += dO^T P, dK^T += Q^T dS  (P / dS consumed in place through the permuted-k trick,
//                                   dO^T / Q^T read transposed from LDS)
//   dQ in a second kernel shaped like the forward (per query block: S^T, dP^T recomputed, dQ^T += K^T dS^T),
//   so no fp32 atomics; delta = rowsum(dO * O) is a tiny kernel ahead of both. lse / delta rows are padded
//   to a multiple of 64 so a query tile's 256 B of each can be staged by one global_load_lds.
#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {

constexpr int FA_BM = 128, FA_THREADS = 256;
constexpr int FB_BN = 64;
// Per-iteration tiles scale with 1/D so every K/V (forward, dQ) or Q/dO (dK/dV) step carries the same MFMA work
// per barrier: 64 keys / queries at D = 128, 128 at D = 64.
// (host side picks TILE = 128 for D = 64 only when the sequence is long enough to keep the grid full)

// 16-B unit swizzles of the attention LDS tiles, chosen so every fragment read is bank-conflict free on gfx950
// (ds_read_b128: 4 lane groups of 16; ds_read_b64_tr_b16: 2 groups of 32; 64 banks). The transposed reads take
// rows 4g + q_ (+16, +32 s2) per 32-lane group: 8 rows whose swizzles must pick 8 different unit pairs. The GEMM
// tiles' swizzles (mn_swz, row/2 mod 8) give those rows only 4 distinct pairs (2-way conflicts on every transposed
// read; rocprofv3 measured 31 % LDS bank-conflict cycles in the forward).
// V tile ([keys][D] rows of 2D bytes, read transposed in the forward's O^T += V^T P^T)
template <int D>
__device__ __forceinline__ int v_swz(int r) {
  return D == 128 ? 2 * (r & 7) : 2 * ((r >> 1) & 3);
}
// K-major-halves tiles ([rows][64] halves of 128-B rows): read as MFMA fragments (ds_read_b128) AND transposed
// (dK/dV: Q^T, dO^T; dQ: K^T)
__device__ __forceinline__ int kh_swz(int row) { return row & 6; }

// operand fragment of a K-major-halves tile: row rb + (lane & 15), k = kk*32 + 8*(lane>>4) .. +7
__device__ __forceinline__ mfma_bf16x8 frag_kh(const char* tile, int rb, int kk, int lane) {
  const int row = rb + (lane & 15);
  const int c = kk * 4 + (lane >> 4);
  const bf16x8_t v = *reinterpret_cast<const bf16x8_t*>(tile + row * 128 + ((c ^ kh_swz(row)) << 4));
  return __builtin_bit_cast(mfma_bf16x8, v);
}

// 2^x on v_exp_f32 alone: exp2f adds a denormal-range rescale (compare, select, ldexp) around every call;
// softmax probabilities below 2^-126 flush to zero, and -inf still gives 0
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// XCD-aware bijective remap of a linear block id (blocks sharing K/V land on the same XCD / L2)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// K-major-halves tile: [rows][D] stored as D/64 halves of [rows][64] with 128-B swizzled rows.
// Byte address of (row, column d .. d+3) for the transposed reads.
__device__ __forceinline__ const char* kh_addr(const char* tile, int rows, int row, int d) {
  const int half = d >> 6, c = (d & 63) >> 3;
  return tile + half * rows * 128 + row * 128 + ((c ^ kh_swz(row)) << 4) + (d & 7) * 2;
}

// global source of unit s (16 B) of a K-major-halves tile with `rows` rows starting at row0
__device__ __forceinline__ const uint16_t* kh_src(const uint16_t* base, long rstride, int rows, int row0, int nrows,
                                                  int s) {
  const int per_half = rows * 8;
  const int half = s / per_half, rem = s - half * per_half;
  const int row = rem >> 3, cp = rem & 7;
  const int c = cp ^ kh_swz(row);
  int gr = row0 + row;
  gr = gr < nrows ? gr : nrows - 1;
  return base + (long)gr * rstride + half * 64 + c * 8;
}

// =============================================================================== forward
// NB: K/V stage buffers (1: every key in one tile, Sk <= TILE -- the short-sequence form, no second buffer).
// QS: 16-query sets per wave (2: 128-query blocks. 1 -- 64-query blocks, 110 VGPRs / 4 blocks per CU -- measured
// slower on BERT s128 b1024: 200 vs 182 us, scripts/gpurun/r5/faqs.sh)
template <int D, int TILE, int NB = 2, int QS = 2>
__global__ void __launch_bounds__(FA_THREADS, NB == 1 ? (QS == 1 ? 4 : 3) : 2) flash_fwd_kernel(AttnFwdArgs a) {
  constexpr int BM = 64 * QS;  // queries per block
  constexpr int FA_BN = TILE;  // keys per iteration
  constexpr int NI = FA_BN / 16;       // 16-key subtiles
  constexpr int KT = FA_BN * D * 2;    // bytes of one K (or V) tile
  constexpr int UPR = D / 8;         // 16-B units per V row
  constexpr int ND = D / 16, NK = D / 32;
  __shared__ __attribute__((aligned(1024))) char smem[NB * 2 * KT];  // [buf][K | V]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int nqb = (a.Sq + BM - 1) / BM;
  const int nwg = nqb * a.Hq * a.B;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int qb = nqb - 1 - (wg % nqb);  // heavier (causal) query blocks first
  const int h = (wg / nqb) % a.Hq;
  const int b = wg / (nqb * a.Hq);
  const int hk = h / (a.Hq / a.Hkv);
  const int q0 = qb * BM, q0w = q0 + wid_u * 16 * QS;  // wave-uniform (SGPR): per-wave skip / mask tests branch on scc
  const int off = a.Sk - a.Sq;
  int kv_end = a.Sk;
  if (a.kv_lens) kv_end = min(kv_end, a.kv_lens[b]);
  int kv_stop = kv_end;
  if (a.causal) kv_stop = min(kv_stop, q0 + BM + off);
  const int ntiles = kv_stop > 0 ? (kv_stop + FA_BN - 1) / FA_BN : 0;

  const uint16_t* qp = a.q + (long)b * a.sqb + (long)h * a.sqh;
  const uint16_t* kp = a.k + (long)b * a.skb + (long)hk * a.skh;
  const uint16_t* vp = a.v + (long)b * a.svb + (long)hk * a.svh;

  // Q fragments (operand "B" of S^T = K Q^T): query q0w + 16*qs + li, d = 32*kk + 8*g
  mfma_bf16x8 qf[QS][NK];
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int qi = q0w + qs * 16 + li;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      bf16x8_t v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qi < a.Sq) v = *reinterpret_cast<const bf16x8_t*>(qp + (long)qi * a.sqs + kk * 32 + g * 8);
      qf[qs][kk] = __builtin_bit_cast(mfma_bf16x8, v);
    }
  }

  f32x4_t oacc[ND][QS];
  float m[QS], l[QS];
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
#pragma unroll
    for (int i = 0; i < ND; ++i) oacc[i][qs] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    m[qs] = -1e30f;
    l[qs] = 0.f;
  }

  // Staging geometry, fixed across tiles: round rd moves K unit s = rd * 256 + tid (tile row, element offset inside
  // the row) and V unit s. The element offsets row * stride + column are computed once -- for full tiles and, rows
  // clamped to Sk - 1, for the block's last tile -- so every LDS-DMA source is one 64-bit add off a wave-uniform tile
  // base (the per-tile index math was ~40 % of the loop's VALU; rocprofv3: 5.5 VALU per MFMA).
  constexpr int NRD = KT / (16 * FA_THREADS);
  int koff[NRD], voff[NRD], koffL[NRD], voffL[NRD];
  {
    const int lim = a.Sk - 1 - (ntiles > 0 ? (ntiles - 1) * FA_BN : 0);  // last tile's highest valid row
#pragma unroll
    for (int rd = 0; rd < NRD; ++rd) {
      const int s_ = rd * FA_THREADS + tid;
      const int per_half = FA_BN * 8, half = s_ / per_half, rem = s_ - half * per_half;
      const int kr = rem >> 3, kc = half * 64 + (((rem & 7) ^ kh_swz(kr)) * 8);  // kh_src's image
      const int vr = s_ / UPR, vc = ((s_ - vr * UPR) ^ v_swz<D>(vr)) * 8;
      koff[rd] = kr * (int)a.sks + kc;
      voff[rd] = vr * (int)a.svs + vc;
      koffL[rd] = min(kr, lim) * (int)a.sks + kc;
      voffL[rd] = min(vr, lim) * (int)a.svs + vc;
    }
  }
  auto stage = [&](int buf, int key0) {
    char* tk = smem + buf * 2 * KT;
    char* tv = tk + KT;
    const uint16_t* kt = kp + (long)key0 * a.sks;
    const uint16_t* vt = vp + (long)key0 * a.svs;
    const bool last = key0 + FA_BN > a.Sk;
#pragma unroll
    for (int rd = 0; rd < NRD; ++rd) {
      const size_t wb = (size_t)(rd * FA_THREADS + wid_u * 64) * 16;  // this wave's 1 KB of the round
      glds16(kt + (last ? koffL[rd] : koff[rd]), tk + wb);
      glds16(vt + (last ? voffL[rd] : voff[rd]), tv + wb);
    }
  };

  if (ntiles > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // one key tile; MASKED: causal / key-length masking and whole-tile skips (only the block's last tiles need it,
  // so the main loop carries no masking code -- as one loop, the compiler if-converted the mask selects into every
  // tile)
  auto tile = [&](const int t, auto masked_tag) {
    constexpr bool MASKED = decltype(masked_tag)::value;
    const int cur = NB > 1 ? (t & 1) : 0, key0 = t * FA_BN;
    if (NB > 1 && t + 1 < ntiles) stage(cur ^ 1, key0 + FA_BN);
    const char* tk = smem + cur * 2 * KT;
    const char* tv = tk + KT;
    const bool skip = MASKED && a.causal && key0 > q0w + 16 * QS - 1 + off;  // whole tile masked for this wave
    if (!skip) {
      // ---- S^T = K Q^T
      f32x4_t s[NI][QS];
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) s[i][qs] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const mfma_bf16x8 kf = frag_kh(tk + (kk >> 1) * (FA_BN * 128), i * 16, kk & 1, lane);
#pragma unroll
          for (int qs = 0; qs < QS; ++qs) s[i][qs] = mfma16(kf, qf[qs][kk], s[i][qs]);
        }
      }
      // ---- online softmax (per query column = lane & 15)
      const bool need_mask = MASKED && ((key0 + FA_BN > kv_end) || (a.causal && key0 + FA_BN - 1 > q0w + off));
#pragma unroll
      for (int qs = 0; qs < QS; ++qs) {
        const int qi = q0w + qs * 16 + li;
        // max over the raw scores (scale_log2 > 0 commutes with max), the scale folded into the exponent's fma
        if (need_mask) {  // wave-uniform; one compare per score against min(kv_end - 1, causal diagonal)
          const int klim = a.causal ? min(kv_end - 1, qi + off) : kv_end - 1;
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[i][qs][r] = key0 + i * 16 + g * 4 + r > klim ? -INFINITY : s[i][qs][r];
        }
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[i][qs][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mn = fmaxf(m[qs], mx * a.scale_log2);
        const float alpha = fexp2(m[qs] - mn);
        float rs = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = fexp2(fmaf(s[i][qs][r], a.scale_log2, -mn));
            s[i][qs][r] = p;
            rs += p;
          }
        l[qs] = l[qs] * alpha + rs;
        // rescale only when some row's running max moved (wave-uniform branch; late key tiles rarely move it)
        if (__any(mn != m[qs])) {
#pragma unroll
          for (int d = 0; d < ND; ++d)
#pragma unroll
            for (int r = 0; r < 4; ++r) oacc[d][qs][r] *= alpha;
        }
        m[qs] = mn;
      }
      // ---- O^T += V^T P^T (k = keys in the permuted order of the S^T accumulators)
#pragma unroll
      for (int s2 = 0; s2 < NI / 2; ++s2) {
        mfma_bf16x8 pf[QS];
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) {
          const float lo[4] = {s[2 * s2][qs][0], s[2 * s2][qs][1], s[2 * s2][qs][2], s[2 * s2][qs][3]};
          const float hi[4] = {s[2 * s2 + 1][qs][0], s[2 * s2 + 1][qs][1], s[2 * s2 + 1][qs][2], s[2 * s2 + 1][qs][3]};
          pf[qs] = pack8(lo, hi);
        }
        const int q_ = li >> 2, p = li & 3;
        const int r0 = 32 * s2 + 4 * g + q_, r1 = r0 + 16;
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          const int u = 2 * d + (p >> 1);
          const char* a0 = tv + r0 * (2 * D) + ((u ^ v_swz<D>(r0)) << 4) + (p & 1) * 8;
          const char* a1 = tv + r1 * (2 * D) + ((u ^ v_swz<D>(r1)) << 4) + (p & 1) * 8;
          const mfma_bf16x8 vf = join8(tr16(a0), tr16(a1));
#pragma unroll
          for (int qs = 0; qs < QS; ++qs) oacc[d][qs] = mfma16(vf, pf[qs], oacc[d][qs]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  };
  // tiles whose every key is valid for every query of the block: below kv_end and (causal) at or below the block's
  // first query's diagonal
  int tfull = kv_end / FA_BN;
  if (a.causal) tfull = min(tfull, max(0, q0 + off + 1) / FA_BN);
  tfull = min(tfull, ntiles);
  int t = 0;
  for (; t < tfull; ++t) tile(t, std::false_type{});
  for (; t < ntiles; ++t) tile(t, std::true_type{});

  // ---- epilogue: O = O^T / l, lse2 = m + log2(l)
  uint16_t* op = a.o + (long)b * a.sob + (long)h * a.soh;
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    float lt = l[qs];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int qi = q0w + qs * 16 + li;
    if (qi >= a.Sq) continue;
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      bf16x4_t o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(oacc[d][qs][r] * inv);
      *reinterpret_cast<bf16x4_t*>(op + (long)qi * a.sos + d * 16 + g * 4) = o;
    }
    if (g == 0) a.lse[((long)b * a.Hq + h) * a.lse_ld + qi] = lt > 0.f ? m[qs] + log2f(lt) : INFINITY;
  }
}


// =============================================================================== backward
// delta[b, h, q] = sum_d dO * O  (D/8 lanes per row, 8 elements per lane); rows of stride lse_ld
template <int D>
__global__ void __launch_bounds__(256) flash_delta_kernel(const uint16_t* o, long sob, long sos, long soh,
                                                         const uint16_t* dO, long sdb, long sds, long sdh,
                                                         float* delta, int B, int Sq, int Hq, long ld) {
  constexpr int LPR = D / 8;  // lanes per row
  const long row = ((long)blockIdx.x * blockDim.x + threadIdx.x) / LPR;
  const int part = threadIdx.x % LPR;
  const long R = (long)B * Sq * Hq;
  float acc = 0.f;
  int b = 0, q = 0, h = 0;
  if (row < R) {
    b = (int)(row / ((long)Sq * Hq));
    const int rem = (int)(row - (long)b * Sq * Hq);
    q = rem / Hq;
    h = rem - q * Hq;
    float x[8], y[8];
    load8(o + b * sob + q * sos + h * soh + part * 8, x);
    load8(dO + b * sdb + q * sds + h * sdh + part * 8, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += x[j] * y[j];
  }
#pragma unroll
  for (int w = LPR / 2; w > 0; w >>= 1) acc += __shfl_xor(acc, w, 64);
  if (row < R && part == 0) delta[((long)b * Hq + h) * ld + q] = acc;
}

// ---- dK, dV: one block = 64 keys of one KV head (wave w: keys k0 + 16w .. +15, K/V fragments in VGPRs),
// looping over every (query head of the GQA group, 64-query tile); Q / dO / lse / delta tiles double-buffered
// in LDS through global_load_lds. Lane layout of S, dP, P, dS: key = li, query = 16*qs + 4*g + r.
template <int D, int TILE>
__global__ void __launch_bounds__(FA_THREADS, 2) flash_bwd_dkv_kernel(AttnBwdArgs a) {
  constexpr int ND = D / 16, NK = D / 32;
  constexpr int FB_BM = TILE;              // queries per iteration
  constexpr int NQ = FB_BM / 16;           // 16-query subtiles
  constexpr int TQ = FB_BM * D * 2;        // Q / dO tile bytes
  constexpr int STAGE = 2 * TQ + 1024;     // Q | dO | lse (256 B) delta (256 B) pad
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int nkb = (a.Sk + FB_BN - 1) / FB_BN;
  const int nsp = a.dkv_split;  // blocks per (key block, KV head): contiguous chunks of its (head, query tile) walk
  const int nwg = nkb * a.Hkv * a.B * nsp;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int sp = wg % nsp;  // the chunks of one key block dispatch together (heavy causal key blocks first)
  const int kb = (wg / nsp) % nkb;
  const int hk = (wg / (nsp * nkb)) % a.Hkv;
  const int b = wg / (nsp * nkb * a.Hkv);
  const int rep = a.Hq / a.Hkv;
  const int k0 = kb * FB_BN, kw = k0 + wid_u * 16;
  const int off = a.Sk - a.Sq;
  int kv_end = a.Sk;
  if (a.kv_lens) kv_end = min(kv_end, a.kv_lens[b]);

  const uint16_t* kp = a.k + (long)b * a.skb + (long)hk * a.skh;
  const uint16_t* vp = a.v + (long)b * a.svb + (long)hk * a.svh;

  f32x4_t dka[ND], dva[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dka[i] = dva[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  const int qt0 = a.causal ? max(0, k0 - off) / FB_BM : 0;
  const int nqt = (a.Sq + FB_BM - 1) / FB_BM;
  const int per_head = nqt - qt0;
  const int total = (k0 < kv_end && per_head > 0) ? rep * per_head : 0;
  // this block's chunk [it0, it1) of the walk; causal key blocks differ in work by up to Sq / 64 x, so one block
  // per key block left the chip waiting on the first ones (load imbalance, not throughput, bounded the kernel)
  const int it0 = (int)((long)total * sp / nsp), it1 = (int)((long)total * (sp + 1) / nsp);
  if (it1 > it0) {
    mfma_bf16x8 kf[NK], vf[NK];
    {
      const int key = kw + li;
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        bf16x8_t x = {0, 0, 0, 0, 0, 0, 0, 0}, y = {0, 0, 0, 0, 0, 0, 0, 0};
        if (key < a.Sk) {
          x = *reinterpret_cast<const bf16x8_t*>(kp + (long)key * a.sks + kk * 32 + g * 8);
          y = *reinterpret_cast<const bf16x8_t*>(vp + (long)key * a.svs + kk * 32 + g * 8);
        }
        kf[kk] = __builtin_bit_cast(mfma_bf16x8, x);
        vf[kk] = __builtin_bit_cast(mfma_bf16x8, y);
      }
    }
    // per-thread staging offsets of the Q / dO units (kh_src's image without the row clamp; only a ragged last
    // query tile takes the clamped path)
    constexpr int NRQ = TQ / (16 * FA_THREADS);
    int qoff[NRQ], doff[NRQ];
#pragma unroll
    for (int rd = 0; rd < NRQ; ++rd) {
      const int s_ = rd * FA_THREADS + tid, half = s_ / (FB_BM * 8), rem = s_ - half * (FB_BM * 8);
      const int row = rem >> 3, col = half * 64 + (((rem & 7) ^ kh_swz(row)) * 8);
      qoff[rd] = row * (int)a.sqs + col;
      doff[rd] = row * (int)a.sds + col;
    }
    auto stage = [&](int buf, int h, int q0) {
      const uint16_t* qp = a.q + (long)b * a.sqb + (long)h * a.sqh;
      const uint16_t* dop = a.dO + (long)b * a.sdb + (long)h * a.sdh;
      char* base = smem + buf * STAGE;
      if (q0 + FB_BM <= a.Sq) {
        const uint16_t* qt = qp + (long)q0 * a.sqs;
        const uint16_t* dt = dop + (long)q0 * a.sds;
#pragma unroll
        for (int rd = 0; rd < NRQ; ++rd) {
          const size_t wb = (size_t)(rd * FA_THREADS + wid_u * 64) * 16;
          glds16(qt + qoff[rd], base + wb);
          glds16(dt + doff[rd], base + TQ + wb);
        }
      } else {
#pragma unroll
        for (int rd = 0; rd < NRQ; ++rd) {
          const int s = rd * FA_THREADS + tid;
          const size_t wb = (size_t)(rd * FA_THREADS + wid_u * 64) * 16;
          glds16(kh_src(qp, a.sqs, FB_BM, q0, a.Sq, s), base + wb);
          glds16(kh_src(dop, a.sds, FB_BM, q0, a.Sq, s), base + TQ + wb);
        }
      }
      if (wid_u == 0) {  // lse | delta of the tile's queries (rows padded to lse_ld, so never out of bounds)
        constexpr int L4 = FB_BM / 4;  // lanes per 4-float row piece
        const long row = ((long)b * a.Hq + h) * a.lse_ld + q0;
        const float* src = lane < L4 ? a.lse + row + lane * 4
                                     : (lane < 2 * L4 ? a.delta + row + (lane - L4) * 4 : a.lse + row);
        glds16(src, base + 2 * TQ);
      }
    };
    int hh = hk * rep + it0 / per_head, qt = qt0 + it0 % per_head;
    stage(0, hh, qt * FB_BM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int key = kw + li;
    // (head, query tile) walk by counters (no per-step division)
    for (int it = it0; it < it1; ++it) {
      const int cur = (it - it0) & 1, q0 = qt * FB_BM;
      if (++qt == nqt) {
        qt = qt0;
        ++hh;
      }
      if (it + 1 < it1) stage(cur ^ 1, hh, qt * FB_BM);
      const char* tq = smem + cur * STAGE;
      const char* tdo = tq + TQ;
      const float* tl = reinterpret_cast<const float*>(tq + 2 * TQ);
      // ---- S = Q K^T, dP = dO V^T
      f32x4_t sv[NQ], dp[NQ];
#pragma unroll
      for (int i = 0; i < NQ; ++i) sv[i] = dp[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
#pragma unroll
        for (int qs = 0; qs < NQ; ++qs) {
          const mfma_bf16x8 qa = frag_kh(tq + (kk >> 1) * (FB_BM * 128), qs * 16, kk & 1, lane);
          const mfma_bf16x8 da = frag_kh(tdo + (kk >> 1) * (FB_BM * 128), qs * 16, kk & 1, lane);
          sv[qs] = mfma16(qa, kf[kk], sv[qs]);
          dp[qs] = mfma16(da, vf[kk], dp[qs]);
        }
      }
      // ---- P = exp2(S c - lse2), dS = P (dP - delta)
      const bool need_mask = q0 + FB_BM > a.Sq || k0 + FB_BN > kv_end || (a.causal && k0 + FB_BN - 1 > q0 + off);
#pragma unroll
      for (int qs = 0; qs < NQ; ++qs) {
        f32x4_t l4 = *reinterpret_cast<const f32x4_t*>(tl + qs * 16 + g * 4);
        f32x4_t d4 = *reinterpret_cast<const f32x4_t*>(tl + FB_BM + qs * 16 + g * 4);
        // masked scores -> -inf (exp2 -> 0) and their lse / delta -> 0 (padded rows are uninitialised): cheap
        // selects in a uniform branch taken only by diagonal / ragged steps, one exponent path for every step
        if (need_mask) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int qi = q0 + qs * 16 + g * 4 + r;
            const bool ok = qi < a.Sq && key < kv_end && !(a.causal && key > qi + off);
            sv[qs][r] = ok ? sv[qs][r] : -INFINITY;
            l4[r] = ok ? l4[r] : 0.f;
            d4[r] = ok ? d4[r] : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fexp2(sv[qs][r] * a.scale_log2 - l4[r]);
          sv[qs][r] = p;
          dp[qs][r] = p * (dp[qs][r] - d4[r]);
        }
      }
      // ---- dV^T += dO^T P, dK^T += Q^T dS   (k = queries in the permuted order of the accumulators)
      const int q_ = li >> 2, pp = li & 3;
#pragma unroll
      for (int s2 = 0; s2 < NQ / 2; ++s2) {
        const float p0[4] = {sv[2 * s2][0], sv[2 * s2][1], sv[2 * s2][2], sv[2 * s2][3]};
        const float p1[4] = {sv[2 * s2 + 1][0], sv[2 * s2 + 1][1], sv[2 * s2 + 1][2], sv[2 * s2 + 1][3]};
        const float d0[4] = {dp[2 * s2][0], dp[2 * s2][1], dp[2 * s2][2], dp[2 * s2][3]};
        const float d1[4] = {dp[2 * s2 + 1][0], dp[2 * s2 + 1][1], dp[2 * s2 + 1][2], dp[2 * s2 + 1][3]};
        const mfma_bf16x8 pf = pack8(p0, p1), dsf = pack8(d0, d1);
        const int r0 = 32 * s2 + 4 * g + q_, r1 = r0 + 16;
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          const int dc = d * 16 + pp * 4;
          const mfma_bf16x8 dot = join8(tr16(kh_addr(tdo, FB_BM, r0, dc)), tr16(kh_addr(tdo, FB_BM, r1, dc)));
          const mfma_bf16x8 qtf = join8(tr16(kh_addr(tq, FB_BM, r0, dc)), tr16(kh_addr(tq, FB_BM, r1, dc)));
          dva[d] = mfma16(dot, pf, dva[d]);
          dka[d] = mfma16(qtf, dsf, dka[d]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  const int key = kw + li;
  if (key < a.Sk && nsp > 1) {  // fp32 partials [split][dk | dv][b][hk][key][D], summed by flash_dkv_reduce_kernel
    const long plane = (long)a.B * a.Hkv * a.Sk * D;
    float* wk = a.dkv_ws + (long)sp * 2 * plane + (((long)b * a.Hkv + hk) * a.Sk + key) * D;
    float* wv = wk + plane;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      *reinterpret_cast<f32x4_t*>(wk + d * 16 + g * 4) = dka[d];
      *reinterpret_cast<f32x4_t*>(wv + d * 16 + g * 4) = dva[d];
    }
  } else if (key < a.Sk) {
    uint16_t* dkp = a.dk + b * a.sgkb + key * a.sgks + hk * a.sgkh;
    uint16_t* dvp = a.dv + b * a.sgvb + key * a.sgvs + hk * a.sgvh;
#pragma unroll
    for (int d = 0; d < ND; ++d) {
      bf16x4_t x, y;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        x[r] = (short)f2bf(dka[d][r] * a.scale);
        y[r] = (short)f2bf(dva[d][r]);
      }
      *reinterpret_cast<bf16x4_t*>(dkp + d * 16 + g * 4) = x;
      *reinterpret_cast<bf16x4_t*>(dvp + d * 16 + g * 4) = y;
    }
  }
}

// sum of the dK / dV chunk partials (fp32), dK scaled, written as bf16 at the gradient strides; 8 columns per thread
template <int D>
__global__ void __launch_bounds__(256) flash_dkv_reduce_kernel(AttnBwdArgs a) {
  constexpr int CPR = D / 8;  // 8-column pieces per row
  const long rows = (long)a.B * a.Hkv * a.Sk;
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  if (t >= rows * CPR) return;
  const long row = t / CPR;
  const int c = (int)(t - row * CPR) * 8;
  const int key = (int)(row % a.Sk);
  const int hk = (int)((row / a.Sk) % a.Hkv);
  const int b = (int)(row / ((long)a.Sk * a.Hkv));
  const long plane = rows * D;
  const float* src = a.dkv_ws + row * D + c;
  f32x4_t k0 = {0.f, 0.f, 0.f, 0.f}, k1 = k0, v0 = k0, v1 = k0;
  for (int sp = 0; sp < a.dkv_split; ++sp) {
    const float* pk = src + (long)sp * 2 * plane;
    k0 += *reinterpret_cast<const f32x4_t*>(pk);
    k1 += *reinterpret_cast<const f32x4_t*>(pk + 4);
    v0 += *reinterpret_cast<const f32x4_t*>(pk + plane);
    v1 += *reinterpret_cast<const f32x4_t*>(pk + plane + 4);
  }
  bf16x8_t xk, xv;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    xk[r] = (short)f2bf(k0[r] * a.scale);
    xk[4 + r] = (short)f2bf(k1[r] * a.scale);
    xv[r] = (short)f2bf(v0[r]);
    xv[4 + r] = (short)f2bf(v1[r]);
  }
  *reinterpret_cast<bf16x8_t*>(a.dk + b * a.sgkb + key * a.sgks + hk * a.sgkh + c) = xk;
  *reinterpret_cast<bf16x8_t*>(a.dv + b * a.sgvb + key * a.sgvs + hk * a.sgvh + c) = xv;
}

// ---- dQ: one block = 4 waves x 16 queries of one head (the forward's structure): K/V tiles of 64 keys
// double-buffered in LDS, S^T = K Q^T and dP^T = V dO^T recomputed (lane: query = li, keys 4g+r), and
// dQ^T += K^T dS^T with dS^T consumed in place (permuted k) and K^T read transposed from the K tile.
// No atomics: each block owns its queries.
template <int D, int TILE, int QS>
__global__ void __launch_bounds__(FA_THREADS, (QS == 2 && D * TILE >= 8192) ? 1 : 2) flash_bwd_dq_kernel(AttnBwdArgs a) {
  constexpr int ND = D / 16, NK = D / 32;
  constexpr int FB_BN = TILE;  // keys per iteration
  constexpr int NI = FB_BN / 16;
  constexpr int KT = FB_BN * D * 2;
  constexpr int QW = 16 * QS;     // queries per wave (QS 16-query sets share every K / V / K^T fragment read)
  constexpr int BMQ = 4 * QW;
  __shared__ __attribute__((aligned(1024))) char smem[4 * KT];  // [buf][K | V], both K-major halves
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int nqb = (a.Sq + BMQ - 1) / BMQ;
  const int nwg = nqb * a.Hq * a.B;
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int qb = nqb - 1 - (wg % nqb);
  const int h = (wg / nqb) % a.Hq;
  const int b = wg / (nqb * a.Hq);
  const int hk = h / (a.Hq / a.Hkv);
  const int q0 = qb * BMQ, q0w = q0 + wid * QW;  // (wid, not wid_u: a scalar skip branch made the compiler copy all of acc on every tile)
  const int off = a.Sk - a.Sq;
  int kv_end = a.Sk;
  if (a.kv_lens) kv_end = min(kv_end, a.kv_lens[b]);
  int kv_stop = kv_end;
  if (a.causal) kv_stop = min(kv_stop, q0 + BMQ + off);
  const int ntiles = kv_stop > 0 ? (kv_stop + FB_BN - 1) / FB_BN : 0;

  const uint16_t* qp = a.q + (long)b * a.sqb + (long)h * a.sqh;
  const uint16_t* dop = a.dO + (long)b * a.sdb + (long)h * a.sdh;
  const uint16_t* kp = a.k + (long)b * a.skb + (long)hk * a.skh;
  const uint16_t* vp = a.v + (long)b * a.svb + (long)hk * a.svh;

  // query of set qs on this lane: q0w + 16 qs + li
  mfma_bf16x8 qf[QS][NK], df[QS][NK];
  float lq[QS], dq_[QS];
  const long lrow = ((long)b * a.Hq + h) * a.lse_ld;
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int qi = q0w + 16 * qs + li;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      bf16x8_t x = {0, 0, 0, 0, 0, 0, 0, 0}, y = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qi < a.Sq) {
        x = *reinterpret_cast<const bf16x8_t*>(qp + (long)qi * a.sqs + kk * 32 + g * 8);
        y = *reinterpret_cast<const bf16x8_t*>(dop + (long)qi * a.sds + kk * 32 + g * 8);
      }
      qf[qs][kk] = __builtin_bit_cast(mfma_bf16x8, x);
      df[qs][kk] = __builtin_bit_cast(mfma_bf16x8, y);
    }
    lq[qs] = qi < a.Sq ? a.lse[lrow + qi] : INFINITY;
    dq_[qs] = qi < a.Sq ? a.delta[lrow + qi] : 0.f;
  }

  f32x4_t acc[QS][ND];
#pragma unroll
  for (int qs = 0; qs < QS; ++qs)
#pragma unroll
    for (int i = 0; i < ND; ++i) acc[qs][i] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // per-thread staging offsets (kh_src's image without the row clamp; only a ragged last key tile is clamped)
  constexpr int NRK = KT / (16 * FA_THREADS);
  int kof[NRK], vof[NRK];
#pragma unroll
  for (int rd = 0; rd < NRK; ++rd) {
    const int s_ = rd * FA_THREADS + tid, half = s_ / (FB_BN * 8), rem = s_ - half * (FB_BN * 8);
    const int row = rem >> 3, col = half * 64 + (((rem & 7) ^ kh_swz(row)) * 8);
    kof[rd] = row * (int)a.sks + col;
    vof[rd] = row * (int)a.svs + col;
  }
  auto stage = [&](int buf, int key0) {
    char* tk = smem + buf * 2 * KT;
    if (key0 + FB_BN <= a.Sk) {
      const uint16_t* kt = kp + (long)key0 * a.sks;
      const uint16_t* vt = vp + (long)key0 * a.svs;
#pragma unroll
      for (int rd = 0; rd < NRK; ++rd) {
        const size_t wb = (size_t)(rd * FA_THREADS + wid_u * 64) * 16;
        glds16(kt + kof[rd], tk + wb);
        glds16(vt + vof[rd], tk + KT + wb);
      }
    } else {
#pragma unroll
      for (int rd = 0; rd < NRK; ++rd) {
        const int s = rd * FA_THREADS + tid;
        const size_t wb = (size_t)(rd * FA_THREADS + wid_u * 64) * 16;
        glds16(kh_src(kp, a.sks, FB_BN, key0, a.Sk, s), tk + wb);
        glds16(kh_src(vp, a.svs, FB_BN, key0, a.Sk, s), tk + KT + wb);
      }
    }
  };
  if (ntiles > 0) {
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int q_ = li >> 2, pp = li & 3;
  for (int t = 0; t < ntiles; ++t) {
    const int cur = t & 1, key0 = t * FB_BN;
    if (t + 1 < ntiles) stage(cur ^ 1, key0 + FB_BN);
    const char* tk = smem + cur * 2 * KT;
    const char* tv = tk + KT;
    if (!(a.causal && key0 > q0w + QW - 1 + off)) {
      f32x4_t s[NI][QS], dp[NI][QS];
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) s[i][qs] = dp[i][qs] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const mfma_bf16x8 kf = frag_kh(tk + (kk >> 1) * (FB_BN * 128), i * 16, kk & 1, lane);
          const mfma_bf16x8 vf = frag_kh(tv + (kk >> 1) * (FB_BN * 128), i * 16, kk & 1, lane);
#pragma unroll
          for (int qs = 0; qs < QS; ++qs) {
            s[i][qs] = mfma16(kf, qf[qs][kk], s[i][qs]);
            dp[i][qs] = mfma16(vf, df[qs][kk], dp[i][qs]);
          }
        }
      }
      // masked scores -> -inf before the exponent (exp2(-inf) = 0): a select per score in masked tiles only, no
      // branch around each exponent (the per-element `ok ? exp : 0` form compiled to 72 exec-mask branches)
      if ((key0 + FB_BN > kv_end) || (a.causal && key0 + FB_BN - 1 > q0w + off)) {
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) {
          const int qi = q0w + 16 * qs + li;
          const int klim = a.causal ? min(kv_end - 1, qi + off) : kv_end - 1;
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) s[i][qs][r] = key0 + i * 16 + g * 4 + r > klim ? -INFINITY : s[i][qs][r];
        }
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int qs = 0; qs < QS; ++qs)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = fexp2(s[i][qs][r] * a.scale_log2 - lq[qs]);
            dp[i][qs][r] = p * (dp[i][qs][r] - dq_[qs]);
          }
#pragma unroll
      for (int s2 = 0; s2 < NI / 2; ++s2) {
        mfma_bf16x8 dsf[QS];
#pragma unroll
        for (int qs = 0; qs < QS; ++qs) {
          const float d0[4] = {dp[2 * s2][qs][0], dp[2 * s2][qs][1], dp[2 * s2][qs][2], dp[2 * s2][qs][3]};
          const float d1[4] = {dp[2 * s2 + 1][qs][0], dp[2 * s2 + 1][qs][1], dp[2 * s2 + 1][qs][2],
                               dp[2 * s2 + 1][qs][3]};
          dsf[qs] = pack8(d0, d1);
        }
        const int r0 = 32 * s2 + 4 * g + q_, r1 = r0 + 16;
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          const int dc = d * 16 + pp * 4;
          const mfma_bf16x8 kt = join8(tr16(kh_addr(tk, FB_BN, r0, dc)), tr16(kh_addr(tk, FB_BN, r1, dc)));
#pragma unroll
          for (int qs = 0; qs < QS; ++qs) acc[qs][d] = mfma16(kt, dsf[qs], acc[qs][d]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int qs = 0; qs < QS; ++qs) {
    const int qi = q0w + 16 * qs + li;
    if (qi < a.Sq) {
      uint16_t* dqp = a.dq + b * a.sgqb + qi * a.sgqs + h * a.sgqh;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        bf16x4_t x;
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = (short)f2bf(acc[qs][d][r] * a.scale);
        *reinterpret_cast<bf16x4_t*>(dqp + d * 16 + g * 4) = x;
      }
    }
  }
}

// ---- short sequences (Sq, Sk <= 128, D = 64, one KV head per query head): the whole backward of one (batch, head)
// in one block. Prologue: Q, dO, K staged by global_load_lds, lse loaded and delta = rowsum(dO * O) computed into LDS.
// Per 64-key chunk: the dK/dV kernel's body (wave w: keys 16w .. +15 of the chunk, K fragments from the LDS tile,
// V fragments from global; S, dP, P, dS for all queries in 64-query halves; dV^T += dO^T P, dK^T += Q^T dS), dS of the
// chunk parked in LDS as bf16 [query][key], then dQ^T += K^T dS^T over the chunk (wave w: queries 32w .. +31, K^T read
// transposed from the K tile, dS^T rows read straight: lane = query, two 8-B reads per 32 keys in the permuted k order).
// BERT s128: the delta / dK-dV / dQ kernels each re-read Q, dO, K, V (664 us per layer at ~3.7 TB/s); here every input
// is read once and nothing round-trips through HBM (no delta array).
constexpr int FS_S = 128;   // longest sequence of the one-block form
constexpr int FS_DSR = 72;  // dS row stride in bf16: 64 keys + 8 pad (row r at bank 36 r: the dQ reads of 16 query rows
                            // x 2 lane groups cover the 64 banks once; the dS writes of 4g-apart rows land 16 banks apart)
__global__ void __launch_bounds__(FA_THREADS, 2) flash_bwd_short_kernel(AttnBwdArgs a, const uint16_t* o, long sob,
                                                                       long sos, long soh) {
  constexpr int NK = 2, ND = 4, TQ = FS_S * 64 * 2;  // Q / dO / K tile bytes (16 KB, one K-major half)
  __shared__ __attribute__((aligned(1024))) char smem[3 * TQ + FS_S * FS_DSR * 2 + 2 * FS_S * 4];
  char* tq = smem;
  char* tdo = smem + TQ;
  char* tk = smem + 2 * TQ;
  uint16_t* dsl = reinterpret_cast<uint16_t*>(smem + 3 * TQ);
  float* tl = reinterpret_cast<float*>(smem + 3 * TQ + FS_S * FS_DSR * 2);  // lse [128] | delta [128]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, li = lane & 15;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int b = blockIdx.x / a.Hq, h = blockIdx.x - b * a.Hq;
  const int off = a.Sk - a.Sq;
  int kv_end = a.Sk;
  if (a.kv_lens) kv_end = min(kv_end, a.kv_lens[b]);

  const uint16_t* qp = a.q + (long)b * a.sqb + (long)h * a.sqh;
  const uint16_t* dop = a.dO + (long)b * a.sdb + (long)h * a.sdh;
  const uint16_t* kp = a.k + (long)b * a.skb + (long)h * a.skh;
  const uint16_t* vp = a.v + (long)b * a.svb + (long)h * a.svh;
  const uint16_t* op = o + (long)b * sob + (long)h * soh;

  // ---- prologue: tiles (rows past the sequence clamped to its last row; their P / dS are masked to 0)
#pragma unroll
  for (int rd = 0; rd < TQ / (16 * FA_THREADS); ++rd) {
    const int s = rd * FA_THREADS + tid;
    const size_t wb = (size_t)(rd * FA_THREADS + wid_u * 64) * 16;
    glds16(kh_src(qp, a.sqs, FS_S, 0, a.Sq, s), tq + wb);
    glds16(kh_src(dop, a.sds, FS_S, 0, a.Sq, s), tdo + wb);
    glds16(kh_src(kp, a.sks, FS_S, 0, a.Sk, s), tk + wb);
  }
  if (tid < FS_S) tl[tid] = tid < a.Sq ? a.lse[((long)b * a.Hq + h) * a.lse_ld + tid] : 0.f;
  {
    const int q = tid >> 1, c0 = (tid & 1) * 32;  // two lanes per query, 32 columns each
    float acc = 0.f;
    if (q < a.Sq) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x[8], y[8];
        load8(op + (long)q * sos + c0 + 8 * j, x);
        load8(dop + (long)q * a.sds + c0 + 8 * j, y);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc += x[e] * y[e];
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    if ((tid & 1) == 0) tl[FS_S + q] = acc;
  }
  // V fragments of this wave's keys in both chunks, in flight with the tiles (loaded per chunk, each chunk's first
  // MFMAs waited on them)
  mfma_bf16x8 vfc[2][NK];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int key = c * 64 + wid_u * 16 + li;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      bf16x8_t y = {0, 0, 0, 0, 0, 0, 0, 0};
      if (key < a.Sk) y = *reinterpret_cast<const bf16x8_t*>(vp + (long)key * a.svs + kk * 32 + g * 8);
      vfc[c][kk] = __builtin_bit_cast(mfma_bf16x8, y);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int q_ = li >> 2, pp = li & 3;
  const int nqh = (a.Sq + 63) / 64, nkc = (a.Sk + 63) / 64;
  f32x4_t dqa[2][ND], dks[ND], dvs[ND];  // dks / dvs: this lane's dK / dV column sums over its chunk keys (cpart)
#pragma unroll
  for (int d = 0; d < ND; ++d) {
    dqa[0][d] = dqa[1][d] = dks[d] = dvs[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }

  for (int kc = 0; kc < nkc; ++kc) {
    const int kw = kc * 64 + wid_u * 16, key = kw + li;
    mfma_bf16x8 kf[NK], vf[NK];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      kf[kk] = frag_kh(tk, kw, kk, lane);
      vf[kk] = kc ? vfc[1][kk] : vfc[0][kk];
    }
    f32x4_t dka[ND], dva[ND];
#pragma unroll
    for (int d = 0; d < ND; ++d) dka[d] = dva[d] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int qh = 0; qh < nqh; ++qh) {
      const int q0 = qh * 64;
      f32x4_t sv[4], dp[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = dp[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < NK; ++kk)
#pragma unroll
        for (int qs = 0; qs < 4; ++qs) {
          sv[qs] = mfma16(frag_kh(tq, q0 + qs * 16, kk, lane), kf[kk], sv[qs]);
          dp[qs] = mfma16(frag_kh(tdo, q0 + qs * 16, kk, lane), vf[kk], dp[qs]);
        }
      const bool need_mask = q0 + 64 > a.Sq || kc * 64 + 64 > kv_end || (a.causal && kc * 64 + 63 > q0 + off);
#pragma unroll
      for (int qs = 0; qs < 4; ++qs) {
        f32x4_t l4 = *reinterpret_cast<const f32x4_t*>(tl + q0 + qs * 16 + g * 4);
        f32x4_t d4 = *reinterpret_cast<const f32x4_t*>(tl + FS_S + q0 + qs * 16 + g * 4);
        if (need_mask) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int qi = q0 + qs * 16 + g * 4 + r;
            const bool ok = qi < a.Sq && key < kv_end && !(a.causal && key > qi + off);
            sv[qs][r] = ok ? sv[qs][r] : -INFINITY;
            l4[r] = ok ? l4[r] : 0.f;
            d4[r] = ok ? d4[r] : 0.f;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = fexp2(sv[qs][r] * a.scale_log2 - l4[r]);
          sv[qs][r] = p;
          dp[qs][r] = p * (dp[qs][r] - d4[r]);
          dsl[(q0 + qs * 16 + g * 4 + r) * FS_DSR + wid_u * 16 + li] = f2bf(dp[qs][r]);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const float p0[4] = {sv[2 * s2][0], sv[2 * s2][1], sv[2 * s2][2], sv[2 * s2][3]};
        const float p1[4] = {sv[2 * s2 + 1][0], sv[2 * s2 + 1][1], sv[2 * s2 + 1][2], sv[2 * s2 + 1][3]};
        const float d0[4] = {dp[2 * s2][0], dp[2 * s2][1], dp[2 * s2][2], dp[2 * s2][3]};
        const float d1[4] = {dp[2 * s2 + 1][0], dp[2 * s2 + 1][1], dp[2 * s2 + 1][2], dp[2 * s2 + 1][3]};
        const mfma_bf16x8 pf = pack8(p0, p1), dsf = pack8(d0, d1);
        const int r0 = q0 + 32 * s2 + 4 * g + q_, r1 = r0 + 16;
        // transposed reads as asm tied to an explicit LDS wait: the builtin form made the compiler drain vmcnt
        // (the dK / dV / dQ stores in flight) in front of every read
        short4_t ol[ND], oh[ND], ql[ND], qh4[ND];
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          const int dc = d * 16 + pp * 4;
          tr16_asm(ol[d], kh_addr(tdo, FS_S, r0, dc));
          tr16_asm(oh[d], kh_addr(tdo, FS_S, r1, dc));
          tr16_asm(ql[d], kh_addr(tq, FS_S, r0, dc));
          tr16_asm(qh4[d], kh_addr(tq, FS_S, r1, dc));
        }
        K8S_LDS_TIE8("s_waitcnt lgkmcnt(0)", ol[0], ol[1], ol[2], ol[3], oh[0], oh[1], oh[2], oh[3]);
        K8S_LDS_TIE8("", ql[0], ql[1], ql[2], ql[3], qh4[0], qh4[1], qh4[2], qh4[3]);
#pragma unroll
        for (int d = 0; d < ND; ++d) {
          dva[d] = mfma16(join8(ol[d], oh[d]), pf, dva[d]);
          dka[d] = mfma16(join8(ql[d], qh4[d]), dsf, dka[d]);
        }
      }
    }
    if (key < a.Sk) {
      uint16_t* dkp = a.dk + b * a.sgkb + key * a.sgks + h * a.sgkh;
      uint16_t* dvp = a.dv + b * a.sgvb + key * a.sgvs + h * a.sgvh;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        bf16x4_t x, y;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          x[r] = (short)f2bf(dka[d][r] * a.scale);
          y[r] = (short)f2bf(dva[d][r]);
        }
        *reinterpret_cast<bf16x4_t*>(dkp + d * 16 + g * 4) = x;
        *reinterpret_cast<bf16x4_t*>(dvp + d * 16 + g * 4) = y;
      }
    }
    if (a.cpart) {  // (keys past the sequence carry zero P / dS, so zero dK / dV)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        dks[d] += dka[d];
        dvs[d] += dva[d];
      }
    }
    __syncthreads();  // the chunk's dS complete
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      mfma_bf16x8 dsf[2];
#pragma unroll
      for (int qs = 0; qs < 2; ++qs) {
        const uint16_t* row = dsl + (wid_u * 32 + qs * 16 + li) * FS_DSR + 32 * s2 + 4 * g;
        dsf[qs] = join8(*reinterpret_cast<const short4_t*>(row), *reinterpret_cast<const short4_t*>(row + 16));
      }
      const int r0 = kc * 64 + 32 * s2 + 4 * g + q_, r1 = r0 + 16;
      short4_t kl[ND], kh4[ND];
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const int dc = d * 16 + pp * 4;
        tr16_asm(kl[d], kh_addr(tk, FS_S, r0, dc));
        tr16_asm(kh4[d], kh_addr(tk, FS_S, r1, dc));
      }
      K8S_LDS_TIE8("s_waitcnt lgkmcnt(0)", kl[0], kl[1], kl[2], kl[3], kh4[0], kh4[1], kh4[2], kh4[3]);
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        const mfma_bf16x8 kt = join8(kl[d], kh4[d]);
#pragma unroll
        for (int qs = 0; qs < 2; ++qs) dqa[qs][d] = mfma16(kt, dsf[qs], dqa[qs][d]);
      }
    }
    __syncthreads();  // dS reads done before the next chunk overwrites it
  }
#pragma unroll
  for (int qs = 0; qs < 2; ++qs) {
    const int qi = wid_u * 32 + qs * 16 + li;
    if (qi < a.Sq) {
      uint16_t* dqp = a.dq + b * a.sgqb + qi * a.sgqs + h * a.sgqh;
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        bf16x4_t x;
#pragma unroll
        for (int r = 0; r < 4; ++r) x[r] = (short)f2bf(dqa[qs][d][r] * a.scale);
        *reinterpret_cast<bf16x4_t*>(dqp + d * 16 + g * 4) = x;
      }
    }
  }
  if (a.cpart) {
    // column sums of the block's dQ / dK / dV rows: each 16-lane row sums its lanes (DPP; lane = query or key), the
    // 4 waves combine through LDS (the Q tile, free since the last chunk's closing barrier)
    float* red = reinterpret_cast<float*>(smem);  // [dq | dk | dv][wave][64 columns]
    const bool v0 = wid_u * 32 + li < a.Sq, v1 = wid_u * 32 + 16 + li < a.Sq;  // dS rows past Sq may be unwritten
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sq = row16_sum((v0 ? dqa[0][d][r] : 0.f) + (v1 ? dqa[1][d][r] : 0.f));
        const float sk = row16_sum(dks[d][r]), sv = row16_sum(dvs[d][r]);
        if (li == 0) {
          const int c = d * 16 + g * 4 + r;
          red[wid_u * 64 + c] = sq * a.scale;
          red[(4 + wid_u) * 64 + c] = sk * a.scale;
          red[(8 + wid_u) * 64 + c] = sv;
        }
      }
    __syncthreads();
    if (tid < 192) {
      const int part = tid >> 6, c = tid & 63;
      const float* rp = red + part * 256 + c;
      const float s = (rp[0] + rp[64]) + (rp[128] + rp[192]);
      a.cpart[(long)b * a.cpart_ld + (part * a.Hq + h) * 64 + c] = s;  // q, k, v column blocks (Hkv == Hq)
    }
  }
}

bool flash_bwd_one_block(int D, int Sq, int Sk, int Hq, int Hkv, int dkv_split) {
  static const bool on = [] {
    const char* e = std::getenv("K8S_AMD_FA_SHORT_BWD");
    return !(e && e[0] == '0');
  }();
  return on && D == 64 && Sq > 0 && Sk > 0 && Sq <= FS_S && Sk <= FS_S && Hq == Hkv && dkv_split == 1;
}

// =============================================================================== launchers
// D = 64 with long sequences: 128-wide key / query steps (same MFMA work per barrier as D = 128)
static bool big_tile(int D, int S) { return D == 64 && S >= 1024; }



// dK/dV chunks per key block: causal key blocks carry from 1 to Sq / 64 query tiles of work, so with one block per
// key block the first ones ran long after the rest of the chip had drained. Split each key block's (head, query tile)
// walk into chunks (fp32 partials + a reduce pass) while the grid stays small enough for the partials to be cheap.
int flash_dkv_splits(int B, int Sq, int Sk, int Hkv, int causal) {
  if (!causal) return 1;
  const long nblk = (long)((Sk + FB_BN - 1) / FB_BN) * Hkv * B;
  const int per_block = (Sq + 63) / 64;  // query tiles of the heaviest key block (per query head)
  if (per_block < 8) return 1;
  // measured at 512 key blocks (Llama-3-8B s4096 / s2048 b2): 2 chunks 585 / 357 us, 4 chunks 601 / 367, 8 chunks 668 / 435
  const long cus = planner_cus();  // thresholds measured on 256 CUs: 1024 and 384 key blocks
  return nblk >= 4 * cus ? 1 : (2 * nblk >= 3 * cus ? 2 : 4);
}

// D = 64, Sk <= 128: every key in one 128-key tile, one stage buffer (K8S_AMD_FA_ONE_TILE=0 keeps the 64-key tiles)
static bool fwd_one_tile() {
  static const bool on = [] {
    const char* e = std::getenv("K8S_AMD_FA_ONE_TILE");
    return !(e && e[0] == '0');
  }();
  return on;
}

void launch_flash_fwd(const AttnFwdArgs& a, int D, hipStream_t st) {
  const int nqb = (a.Sq + FA_BM - 1) / FA_BM;
  const dim3 grid(nqb * a.Hq * a.B), blk(FA_THREADS);
  if (D == 128) hipLaunchKernelGGL((flash_fwd_kernel<128, 64>), grid, blk, 0, st, a);
  else if (big_tile(D, a.Sk)) hipLaunchKernelGGL((flash_fwd_kernel<64, 128>), grid, blk, 0, st, a);
  else if (a.Sk <= 128 && fwd_one_tile()) hipLaunchKernelGGL((flash_fwd_kernel<64, 128, 1>), grid, blk, 0, st, a);
  else hipLaunchKernelGGL((flash_fwd_kernel<64, 64>), grid, blk, 0, st, a);
}

void launch_flash_bwd(const AttnBwdArgs& a, int D, const uint16_t* o, long sob, long sos, long soh,
                      hipStream_t st) {
  if (flash_bwd_one_block(D, a.Sq, a.Sk, a.Hq, a.Hkv, a.dkv_split)) {
    if ((long)a.B * a.Hq > 0)
      hipLaunchKernelGGL(flash_bwd_short_kernel, dim3((unsigned)(a.B * a.Hq)), dim3(FA_THREADS), 0, st, a, o, sob,
                         sos, soh);
    return;
  }
  const long R = (long)a.B * a.Sq * a.Hq;
  const int lpr = D / 8;
  const dim3 dgrid((unsigned)((R * lpr + 255) / 256));
  if (D == 128)
    hipLaunchKernelGGL(flash_delta_kernel<128>, dgrid, dim3(256), 0, st, o, sob, sos, soh, a.dO, a.sdb, a.sds, a.sdh,
                       a.delta, a.B, a.Sq, a.Hq, a.lse_ld);
  else
    hipLaunchKernelGGL(flash_delta_kernel<64>, dgrid, dim3(256), 0, st, o, sob, sos, soh, a.dO, a.sdb, a.sds, a.sdh,
                       a.delta, a.B, a.Sq, a.Hq, a.lse_ld);
  // dK/dV blocks own 64 keys at any D, split into a.dkv_split chunks (flash_dkv_splits)
  const dim3 gkv(((a.Sk + FB_BN - 1) / FB_BN) * a.Hkv * a.B * a.dkv_split);
  // dQ: QS = 2 (32 queries per wave, 128 per block) when the grid still fills the chip. With D x TILE = 8192
  // (D = 128, or D = 64 on 128-key tiles) that form needs ~320 VGPRs (one wave per SIMD) and measured slower there
  // (round 3), so those keep QS = 1.
  const bool small = D == 64 && !big_tile(D, a.Sq);
  const bool qs2 = small && (long)((a.Sq + 127) / 128) * a.Hq * a.B >= 2L * planner_cus();
  const dim3 gq(((a.Sq + (qs2 ? 127 : 63)) / (qs2 ? 128 : 64)) * a.Hq * a.B), blk(FA_THREADS);
  if (D == 128) {
    hipLaunchKernelGGL((flash_bwd_dkv_kernel<128, 64>), gkv, blk, 0, st, a);
    hipLaunchKernelGGL((flash_bwd_dq_kernel<128, 64, 1>), gq, blk, 0, st, a);
  } else if (big_tile(D, a.Sq)) {
    hipLaunchKernelGGL((flash_bwd_dkv_kernel<64, 128>), gkv, blk, 0, st, a);
    hipLaunchKernelGGL((flash_bwd_dq_kernel<64, 128, 1>), gq, blk, 0, st, a);
  } else {
    hipLaunchKernelGGL((flash_bwd_dkv_kernel<64, 64>), gkv, blk, 0, st, a);
    if (qs2) hipLaunchKernelGGL((flash_bwd_dq_kernel<64, 64, 2>), gq, blk, 0, st, a);
    else hipLaunchKernelGGL((flash_bwd_dq_kernel<64, 64, 1>), gq, blk, 0, st, a);
  }
  if (a.dkv_split > 1) {
    const long n = (long)a.B * a.Hkv * a.Sk * (D / 8);
    const dim3 rg((unsigned)((n + 255) / 256));
    if (D == 128) hipLaunchKernelGGL(flash_dkv_reduce_kernel<128>, rg, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(flash_dkv_reduce_kernel<64>, rg, dim3(256), 0, st, a);
  }
}

}  // namespace k8s_amd
