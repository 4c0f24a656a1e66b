// K1 + K2: MFMA GEMM and NHWC implicit-GEMM convolution for gfx950.
//
//   C[M,N] (+)= A[M,K] . B[K,N]   bf16 in, fp32 accumulate, bf16/fp32 out
//
// One kernel template, four operand "sources":
//   KMajor   : operand stored row-major with K contiguous   (activations x[m][k], weights w[n][k])
//   MNMajor  : operand stored with M (or N) contiguous      (dY^T in wgrad, w[k][n] in dgrad)
//   ConvA    : implicit im2col of an NHWC input, K = (r, s, c), K contiguous per (r, s)
//   ConvWgB  : implicit im2col used as the N-major B operand of the weight-gradient GEMM
//
// Design (MI355X_MICROARCH / cdna_hip_programming guide):
//  * 128x128 block tile, BK = 64, 256 threads = 4 waves (2x2), each wave 64x64 = 4x4
//    v_mfma_f32_16x16x32_bf16 tiles (64 accumulator VGPRs).
//  * global -> LDS with 16-byte global_load_lds (no VGPR round trip); the LDS image is
//    lane-linear, so bank-conflict swizzles are applied to the per-lane SOURCE address and
//    the same XOR on the read (rule 21):
//      K-major   [128 rows][64 k]  : 16-B chunk c of row r stored at c ^ ((r >> 1) & 7)
//                                    -> conflict-free ds_read_b128 fragment reads
//      MN-major  [64 k][128 mn]    : 16-B unit u of k-row r stored at u ^ h(r),
//                                    h(r) = 2 * ((r & 3) | ((r >> 3 & 1) << 2))
//                                    -> conflict-free ds_read_b64_tr_b16 transposed reads
//  * double-buffered LDS (2 x 32 KB), next tile's loads issued before the current tile's MFMAs.
//  * operands swapped in the MFMA (B tile as the "A" operand) so each lane ends with 4
//    CONSECUTIVE output columns: 8-byte bf16 / 16-byte fp32 stores in the epilogue.
//  * XCD-aware, bijective block remap + grouped tile order so blocks sharing an A or B panel
//    run on the same XCD (private L2).
//  * epilogue: bias, ReLU / GELU(tanh), pre-activation side output, fp32 accumulate, split-K
//    fp32 atomics (for the tall-K weight gradients).
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace k8s_amd {

constexpr int BM = 128, BN = 128, BK = 64;  // the general tile (split-K sizing); see gemm_bf16_kernel
constexpr int GEMM_THREADS = 256;

// 16-byte zero line for out-of-image implicit-GEMM loads
__device__ __attribute__((aligned(64))) uint16_t g_zero_page[64];

// BatchNorm + ReLU applied to an operand as it is staged into LDS ("normalize on load"): the operand is a BN
// layer's raw input x and the GEMM consumes z = relu(fma(x, scale, shift)) -- bit-identical to what
// batchnorm.hip's bn_apply_kernel would have written -- so the BN forward's apply pass (read x, write z) and the z
// tensor disappear. p = fp32 [2][C] (scale | shift, from bn_finalize); an operand element's channel is its K index
// (A, K-major) or its column (B, MN-major) modulo C. Zero padding (taps outside the image, split-K / tile tails)
// stays zero: those loads are recognised by their zero-page source address and not transformed.
struct XForm {
  const float* p;
  int C;
  FastDiv fC;
};

__device__ __forceinline__ bf16x8_t bn_relu8(const bf16x8_t& v, const float (&sc)[8], const float (&sh)[8],
                                             bool valid) {
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = fmaxf(__builtin_fmaf(bf2f((uint16_t)v[j]), sc[j], sh[j]), 0.f);
  const bf16x8_t r = pack_bf16x8(o);
  return valid ? r : bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
}

__device__ __forceinline__ void load_f8g(const float* p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

// ----------------------------------------------------------------------------- operand sources
// stage(): called for round 0..3, writes slot s = round*256 + tid of a 16 KB tile.
struct KMajor {
  const uint16_t* p;
  long ld;    // elements between rows
  int rows;   // valid rows (M or N)
  int ktot = 1 << 30;  // valid K (a K % 64 tail reads zeros instead of the next row / past the end)
  // row-major [rows][K]; tile rows start at r0, k at k0
  __device__ __forceinline__ const void* src(int s, int r0, int k0) const {
    const int row = s >> 3, cp = s & 7;
    const int c = cp ^ ((row >> 1) & 7);
    int gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    if (k0 + c * 8 >= ktot) return g_zero_page;
    return p + (long)gr * ld + k0 + c * 8;
  }
  // Hoisted per-thread cursor: row, swizzled chunk and the 64-bit row address are loop-invariant, a tile only
  // adds k0 (rocprofv3 showed ~5 VALU instructions per MFMA with the per-tile derivation).
  struct Cursor { const uint16_t* p; int c8; };
  __device__ __forceinline__ Cursor cursor(int s, int r0) const {
    const int row = s >> 3, cp = s & 7;
    const int c = cp ^ ((row >> 1) & 7);
    int gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    return Cursor{p + (long)gr * ld + c * 8, c * 8};
  }
  __device__ __forceinline__ const void* at(const Cursor& q, int k0) const {
    return k0 + q.c8 >= ktot ? (const void*)g_zero_page : (const void*)(q.p + k0);
  }
  // per-K-step uniform part of the address (identity here; see ConvA)
  __device__ __forceinline__ int tap(int k0) const { return k0; }
  // channel of K index k0 (a 1x1 convolution's activation: K is the channel)
  __device__ __forceinline__ int chan0(int k0) const { return k0; }
  static constexpr bool kmajor = true;
};

struct MNMajor {
  const uint16_t* p;
  long ld;   // elements between k rows
  int cols;  // valid M (or N) extent; must be a multiple of 8
  __device__ __forceinline__ const void* src(int s, int c0, int k0) const {
    const int krow = s >> 4, up = s & 15;
    const int u = up ^ mn_swz(krow);
    int col = c0 + u * 8;
    col = col < cols ? col : cols - 8;
    return p + (long)(k0 + krow) * ld + col;
  }
  // no hoisted cursor: every tile re-derives the address from the slot index
  struct Cursor { int s, base; };
  __device__ __forceinline__ Cursor cursor(int s, int base) const { return Cursor{s, base}; }
  __device__ __forceinline__ const void* at(const Cursor& c, int k0) const { return src(c.s, c.base, k0); }
  // per-K-step uniform part of the address (identity here; see ConvA)
  __device__ __forceinline__ int tap(int k0) const { return k0; }
  static constexpr bool kmajor = false;
};

// Implicit im2col of NHWC input x[N][H][W][C] for a KRSC weight: row m = (n, ho, wo), k = (r, s, c).
// Requires C % 64 == 0 so one 64-wide k tile lies inside a single (r, s).
struct ConvA {
  const uint16_t* x;
  int N, H, W, C, Ho, Wo, S, stride, pad, dil;
  int rows;  // N*Ho*Wo
  FastDiv fC, fS, fHW, fWo;
  __device__ __forceinline__ const void* src(int s, int r0, int k0) const {
    const int row = s >> 3, cp = s & 7;
    const int c = cp ^ ((row >> 1) & 7);
    int m = r0 + row;
    m = m < rows ? m : rows - 1;
    const int rs = fC.div(k0), c0 = k0 - rs * C;
    const int r = fS.div(rs), sx = rs - r * S;
    const int n = fHW.div(m), rem = m - n * (Ho * Wo);
    const int ho = fWo.div(rem), wo = rem - ho * Wo;
    const int hi = ho * stride - pad + r * dil, wi = wo * stride - pad + sx * dil;
    if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) return g_zero_page;
    return x + (((long)n * H + hi) * W + wi) * C + c0 + c * 8;
  }
  // Hoisted cursor: the output pixel (n, ho, wo) of a thread's rows is fixed for the whole K loop; a tile only
  // decodes its (r, s, c0) -- wave-uniform, so scalar -- and bounds-checks the tap per lane.
  struct Cursor { const uint16_t* p; int hs, ws; };
  __device__ __forceinline__ Cursor cursor(int s, int r0) const {
    const int row = s >> 3, cp = s & 7;
    const int c = cp ^ ((row >> 1) & 7);
    int m = r0 + row;
    m = m < rows ? m : rows - 1;
    const int n = fHW.div(m), rem = m - n * (Ho * Wo);
    const int ho = fWo.div(rem), wo = rem - ho * Wo;
    const int hs = ho * stride - pad, ws = wo * stride - pad;
    return Cursor{x + (((long)n * H + hs) * W + ws) * C + c * 8, hs, ws};
  }
  // The (r, s, c0) decode of a K step is wave-uniform: done once per stage (tap) instead of once per load -- the
  // four loads' repeated scalar divisions were ~120 SALU per K step in the ISA, issued ahead of the MFMAs.
  struct Tap {
    int dh, dw;
    long off;
  };
  __device__ __forceinline__ Tap tap(int k0) const {
    const int rs = fC.div(k0), c0 = k0 - rs * C;
    const int r = fS.div(rs), sx = rs - r * S;
    return Tap{r * dil, sx * dil, ((long)(r * dil) * W + sx * dil) * C + c0};
  }
  __device__ __forceinline__ const void* at(const Cursor& q, const Tap& t) const {
    const int hi = q.hs + t.dh, wi = q.ws + t.dw;
    if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) return g_zero_page;
    return q.p + t.off;
  }
  // channel of K index k0 = (r, s, c0): c0 (a K step lies inside one tap, C % 64 == 0)
  __device__ __forceinline__ int chan0(int k0) const { return k0 - fC.div(k0) * C; }
  static constexpr bool kmajor = true;
};

// Implicit im2col for any C % 8 == 0 (the 8-channel ResNet stem): every 16-B unit decodes its own
// (r, s, c) and the K = R*S*C tail (K % 64 != 0) reads zeros.
struct ConvAG {
  const uint16_t* x;
  int N, H, W, C, Ho, Wo, S, stride, pad, dil;
  int rows;  // N*Ho*Wo
  int ktot;  // R*S*C
  FastDiv fC, fS, fHW, fWo;
  __device__ __forceinline__ const void* src(int s, int r0, int k0) const {
    const int row = s >> 3, cp = s & 7;
    const int c = cp ^ ((row >> 1) & 7);
    int m = r0 + row;
    m = m < rows ? m : rows - 1;
    const int k = k0 + c * 8;
    if (k >= ktot) return g_zero_page;
    const int rs = fC.div(k), c0 = k - rs * C;
    const int r = fS.div(rs), sx = rs - r * S;
    const int n = fHW.div(m), rem = m - n * (Ho * Wo);
    const int ho = fWo.div(rem), wo = rem - ho * Wo;
    const int hi = ho * stride - pad + r * dil, wi = wo * stride - pad + sx * dil;
    if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) return g_zero_page;
    return x + (((long)n * H + hi) * W + wi) * C + c0;
  }
  // no hoisted cursor: every tile re-derives the address from the slot index
  struct Cursor { int s, base; };
  __device__ __forceinline__ Cursor cursor(int s, int base) const { return Cursor{s, base}; }
  __device__ __forceinline__ const void* at(const Cursor& c, int k0) const { return src(c.s, c.base, k0); }
  // per-K-step uniform part of the address (identity here; see ConvA)
  __device__ __forceinline__ int tap(int k0) const { return k0; }
  static constexpr bool kmajor = true;
};

// B operand of the weight gradient: B[k' = m][n' = (r, s, c)] = x[n][ho*st-pad+r][wo*st-pad+s][c]
// (N-major: 8 consecutive c per 16-B unit). Requires C % 8 == 0.
struct ConvWgB {
  const uint16_t* x;
  int N, H, W, C, Ho, Wo, S, stride, pad, dil;
  int cols;  // R*S*C
  int mtot;  // N*Ho*Wo
  FastDiv fC, fS, fHW, fWo;
  __device__ __forceinline__ const void* src(int s, int c0, int k0) const {
    const int krow = s >> 4, up = s & 15;
    const int u = up ^ mn_swz(krow);
    int col = c0 + u * 8;
    if (col >= cols) return g_zero_page;
    const int m = k0 + krow;
    if (m >= mtot) return g_zero_page;
    const int rs = fC.div(col), c = col - rs * C;
    const int r = fS.div(rs), sx = rs - r * S;
    const int n = fHW.div(m), rem = m - n * (Ho * Wo);
    const int ho = fWo.div(rem), wo = rem - ho * Wo;
    const int hi = ho * stride - pad + r * dil, wi = wo * stride - pad + sx * dil;
    if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) return g_zero_page;
    return x + (((long)n * H + hi) * W + wi) * C + c;
  }
  // Hoisted cursor: a thread's column (r, s, c) -- and so its tap offsets -- is fixed for the whole K loop; a K
  // step only decodes its row m = k0 + krow into (n, ho, wo) (two multiply-high divisions).
  struct Cursor {
    int krow, dh, dw, coff;  // dh/dw: r*dil - pad, s*dil - pad; krow < 0 marks a padding column
  };
  __device__ __forceinline__ Cursor cursor(int s, int c0) const {
    const int krow = s >> 4, up = s & 15;
    const int u = up ^ mn_swz(krow);
    const int col = c0 + u * 8;
    if (col >= cols) return Cursor{-(1 << 30), 0, 0, 0};
    const int rs = fC.div(col), c = col - rs * C;
    const int r = fS.div(rs), sx = rs - r * S;
    return Cursor{krow, r * dil - pad, sx * dil - pad, c};
  }
  __device__ __forceinline__ const void* at(const Cursor& q, int k0) const {
    const int m = k0 + q.krow;
    if (q.krow < 0 || m >= mtot) return g_zero_page;
    const int n = fHW.div(m), rem = m - n * (Ho * Wo);
    const int ho = fWo.div(rem), wo = rem - ho * Wo;
    const int hi = ho * stride + q.dh, wi = wo * stride + q.dw;
    if ((unsigned)hi >= (unsigned)H || (unsigned)wi >= (unsigned)W) return g_zero_page;
    return x + (((long)n * H + hi) * W + wi) * C + q.coff;
  }
  // per-K-step uniform part of the address (identity here; see ConvA)
  __device__ __forceinline__ int tap(int k0) const { return k0; }
  static constexpr bool kmajor = false;
};

// MN-major operand whose K rows may run past the end (split-K tails): zero rows beyond mtot.
struct MNMajorK {
  const uint16_t* p;
  long ld;
  int cols, ktot;
  __device__ __forceinline__ const void* src(int s, int c0, int k0) const {
    const int krow = s >> 4, up = s & 15;
    const int u = up ^ mn_swz(krow);
    int col = c0 + u * 8;
    if (col >= cols || k0 + krow >= ktot) return g_zero_page;
    return p + (long)(k0 + krow) * ld + col;
  }
  struct Cursor { const uint16_t* p; int krow; };  // krow = -inf marks a padding column
  __device__ __forceinline__ Cursor cursor(int s, int c0) const {
    const int krow = s >> 4, up = s & 15;
    const int u = up ^ mn_swz(krow);
    const int col = c0 + u * 8;
    return Cursor{p + (long)krow * ld + col, col >= cols ? -(1 << 30) : krow};
  }
  __device__ __forceinline__ const void* at(const Cursor& q, int k0) const {
    return (q.krow < 0 || k0 + q.krow >= ktot) ? (const void*)g_zero_page : (const void*)(q.p + (long)k0 * ld);
  }
  // per-K-step uniform part of the address (identity here; see ConvA)
  __device__ __forceinline__ int tap(int k0) const { return k0; }
  static constexpr bool kmajor = false;
};

// ----------------------------------------------------------------------------- fragment reads
__device__ __forceinline__ mfma_bf16x8 frag_mnmajor(const char* tile, int cb, int kk, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int u = (cb >> 3) + (p >> 1);
  const int r0 = kk * 32 + 8 * g + q;
  const int r1 = r0 + 4;
  const char* a0 = tile + r0 * 256 + ((u ^ mn_swz(r0)) << 4) + (p & 1) * 8;
  const char* a1 = tile + r1 * 256 + ((u ^ mn_swz(r1)) << 4) + (p & 1) * 8;
  short4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0));
  short4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a1));
  bf16x8_t v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(mfma_bf16x8, v);
}

template <class Src>
__device__ __forceinline__ mfma_bf16x8 frag(const char* tile, int b, int kk, int lane) {
  if constexpr (Src::kmajor) return frag_kmajor(tile, b, kk, lane);
  else return frag_mnmajor(tile, b, kk, lane);
}

// ----------------------------------------------------------------------------- epilogue
struct Epi {
  void* c;           // output (bf16 or fp32)
  long ldc;
  const float* bias;  // [N] or null
  uint16_t* pre;      // bf16 pre-activation copy or null
  int out_f32;        // 1: fp32 output
  int act;            // 0 none, 1 relu, 2 gelu(tanh)
  int mode;           // 0 store, 1 accumulate (fp32 C += acc), 2 atomic add (fp32),
                      // 3 split-K slab: split z stores plain fp32 at c + z * slab (reduced by splitk_reduce)
  long slab;
  float alpha;
  float* stats;       // [STAT_REPL][2][N] fp32 per-column sum / sum of squares of the stored outputs
                      // (BN fusion) or null; tile row tm adds into replica tm % STAT_REPL so the atomics
                      // spread over STAT_REPL x 2N addresses instead of contending on 2N
  // Sub-grid output (stride-s data gradient by output parity): GEMM row m = (n, i, j) over an rHo x rWo grid
  // is stored at output row (n, i*rst + ra, j*rst + rb) of an rH x rW image. rst == 0: identity.
  int rst, rHo, rWo, rH, rW, ra, rb;
  // accumulate (mode 1, lean epilogue) onto addsrc instead of C's old value, with the elements whose packed bit in
  // addmask is clear taken as zero: C = acc + (bit ? addsrc : 0). A ResNet identity block's input gradient is
  // conv1's dgrad plus the block output's gradient masked by its ReLU -- read here from dy and the forward's
  // 1-bit mask instead of from a materialised residual gradient.
  const uint16_t* addsrc;
  const uint8_t* addmask;
  // BST instantiation (lean fast path, identity rows, ldc == N): the BatchNorm-backward sums of the stored output
  // for the relu(BN(x)) that produced this data gradient's input (launchers.h BnBwdSums), into bb.sums
  BnBwdSums bb;
};
constexpr int STAT_REPL = 32;

// GELU(tanh) as x * sigmoid(2u), u = k0 (x + k1 x^3): sigmoid(2u) = (1 + tanh u) / 2 = 1 / (1 + 2^(-2u log2 e)),
// one v_exp_f32 + one v_rcp_f32 (both ~1 ulp) instead of tanhf's polynomial. The epilogue runs it serially per
// thread over the whole tile, so its cost is not hidden: BERT-base FFN1 forward 89 -> 76 us per call.
__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-2.8853900817779268f * u));
}

// ----------------------------------------------------------------------------- the kernel
// NBUF = 2: double-buffered K loop (the next tile's loads in flight during this tile's MFMAs), 64 KB LDS,
// 2 blocks/CU. NBUF = 1: single buffer, 32 KB LDS, 3 blocks/CU -- for short K ranges (K <= 128: the
// memory-bound 1x1 convolutions of the early ResNet stages), where there is no next tile to prefetch and
// block-level overlap is what hides HBM latency.
//
// WM x WN waves (WM * WN = 4), each owning a 64 x 64 piece: 128 x 128 tiles (2 x 2) in general, 256 x 64
// (4 x 1) when N = 64 (the early ResNet convolutions and the stem) so no MFMA work is spent on padding.
// Only K-major sources may sit on a 64-wide side (the MN-major swizzle assumes 256-B rows).
// LEAN: the staged bf16 epilogue (also the only one with the BN-statistics reduction).
// (Rounds 2-3 also had a BatchNorm-BACKWARD statistics epilogue for the data gradients, the BN input tile DMA'd
// into LDS beside the operands; it measured a net loss on ResNet-50 both rounds and was removed -- ops/conv.py.)
// XEPI (lean only): bias / ReLU / GELU / pre-activation copy in the staged epilogue (the transformer linears'
// forward); its own instantiation so the convolutions' lean kernels stay as small as before (the extra epilogue
// code compiled into every lean kernel cost ResNet-50 1.1 %, measured new/old/new/old on one box).
// F32S (general epilogue only): fp32 outputs without bias / activation / statistics / row remap -- the weight
// gradients and their split-K slabs -- go through LDS and leave as whole 256-B row segments; its own instantiation
// for the weight-gradient operand pairs.
// XF (normalize on load, see XForm): 1 = the A operand (K-major: a convolution's activation), 2 = the B operand
// (MN-major: a weight gradient's im2col / activation operand) is loaded through VGPRs, transformed and written to
// its LDS slot by ds_write instead of by LDS-DMA (same lane-linear image, same swizzle). The staging registers of
// the next K step are filled behind this step's MFMAs and written after them, before the step's barrier.
// BST (lean only): the BatchNorm-backward sums epilogue of a data gradient (Epi::bb) instead of the statistics.
template <class ASrc, class BSrc, int NBUF, int WM = 2, int WN = 2, bool LEAN = false, bool XEPI = false,
          bool F32S = false, int XF = 0, bool BST = false>
__global__ void __launch_bounds__(GEMM_THREADS, (NBUF == 1 && (XF == 0 || (XF == 1 && WM == 2))) ? 3 : 2)
gemm_bf16_kernel(ASrc A, BSrc B, Epi E, int M, int N, int K, int k_per_split, XForm X) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int TA = BM * BK * 2, TB = BN * BK * 2;  // operand tile bytes
  static_assert(WM * WN == 4, "4 waves");
  static_assert((WM == 2 || ASrc::kmajor) && (WN == 2 || BSrc::kmajor), "MN-major operands need a 128 side");
  static_assert(BM * BN * 2 <= TA + TB, "the C tile fits one operand buffer");
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * (TA + TB)];  // [buf][A|B]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  // ---- XCD-aware bijective remap over the whole (tile, split) grid, then grouped (GROUP_M = 8) tile order. The
  // hardware hands workgroups to the 8 XCDs round-robin in dispatch order (x fastest, then z); remapping the LINEAR
  // id puts every tile of one K split on one XCD, so a split-K weight gradient with few output tiles (ResNet's 1x1
  // layers: 4 tiles of 128 x 128 over 800k pixels) reads the operand the tiles share from that XCD's L2 once instead
  // of from HBM once per tile (remapping x alone spread a split's 4 tiles over 4 XCDs)
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  int wg, zsplit;
  {
    const int L = blockIdx.x + nwg * blockIdx.z, tot = nwg * gridDim.z;
    const int xcd = L & 7, q = tot >> 3, r = tot & 7;
    const int lam = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
    zsplit = lam / nwg;
    wg = lam - zsplit * nwg;
  }
  const int group = 8 * tiles_n;
  const int first_m = (wg / group) * 8;
  const int gm = min(tiles_m - first_m, 8);
  const int tm = first_m + (wg % group) % gm;
  const int tn = (wg % group) / gm;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = zsplit * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nt = (kend - kbeg + BK - 1) / BK;

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  // BST: this thread's BatchNorm-input chunks for the epilogue's fast path (chunk column c, rows row0 + i RSTEP),
  // the first XE of them loaded before the K loop so their latency hides behind it, the rest at the epilogue's start.
  // All in the epilogue: the latency was exposed once per tile (+0.35 ms per ResNet-50 stage-1 call); all before the K
  // loop (32 VGPRs): the single-buffer kernel fell to 2 blocks per CU and gained nothing; 2 of 8 rows (8 VGPRs) keep
  // its 3 blocks per CU: +0.4 % ResNet-50 b3072 against the separate reduction (profiles/r06_notes.md)
  constexpr int XCPR = BN / 8, XRSTEP = GEMM_THREADS / XCPR, XR = BST ? BM / XRSTEP : 1;
  constexpr int XE = BST ? (NBUF == 1 ? XR / 4 : XR) : 0;
  bf16x8_t bxr[XR];
  auto load_bxr = [&](int i0, int i1) {
    const int c = tid % XCPR, row0 = tid / XCPR, n = n0 + c * 8;
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const int m = m0 + row0 + i * XRSTEP;
      bxr[i] = bf16x8_t{0, 0, 0, 0, 0, 0, 0, 0};
      if (n < N && m < M) bxr[i] = *reinterpret_cast<const bf16x8_t*>(E.bb.x + (long)m * N + n);
    }
  };
  if constexpr (BST) {
    if (!E.rst) load_bxr(0, XE);  // (the identity-row fast path; the sub-grid correction reads x itself)
  }

  const int wid_u = __builtin_amdgcn_readfirstlane(wid);  // provably wave-uniform for the M0 (LDS base) operand
  constexpr int RA = TA / (16 * GEMM_THREADS), RB = TB / (16 * GEMM_THREADS);
  // hoisted cursors cost ~4 VGPRs per load slot and pay off over many K tiles: the 3-blocks/CU single-buffer
  // kernels (<= 2 K tiles, 168-VGPR budget) keep the per-tile derivation
  constexpr bool HOIST = NBUF != 1;
  typename ASrc::Cursor ca[HOIST ? RA : 1];
  typename BSrc::Cursor cb[HOIST ? RB : 1];
  if constexpr (HOIST) {
#pragma unroll
    for (int rd = 0; rd < RA; ++rd) ca[rd] = A.cursor(rd * GEMM_THREADS + tid, m0);
#pragma unroll
    for (int rd = 0; rd < RB; ++rd) cb[rd] = B.cursor(rd * GEMM_THREADS + tid, n0);
  }
  static_assert(XF == 0 || (XF == 1 && ASrc::kmajor) || (XF == 2 && !BSrc::kmajor),
                "normalize-on-load: K-major A or MN-major B");
  // LDS-DMA staging of the operands that are not transformed
  auto stage = [&](int buf, int k0) {
    char* ta = smem + buf * (TA + TB);
    char* tb = ta + TA;
    if constexpr (HOIST) {
      const auto tpa = A.tap(k0);
      const auto tpb = B.tap(k0);
      if constexpr (XF != 1) {
#pragma unroll
        for (int rd = 0; rd < RA; ++rd) glds16(A.at(ca[rd], tpa), ta + (rd * GEMM_THREADS + wid_u * 64) * 16);
      }
      if constexpr (XF != 2) {
#pragma unroll
        for (int rd = 0; rd < RB; ++rd) glds16(B.at(cb[rd], tpb), tb + (rd * GEMM_THREADS + wid_u * 64) * 16);
      }
    } else {
      if constexpr (XF != 1) {
#pragma unroll
        for (int rd = 0; rd < RA; ++rd)
          glds16(A.src(rd * GEMM_THREADS + tid, m0, k0), ta + (rd * GEMM_THREADS + wid_u * 64) * 16);
      }
      if constexpr (XF != 2) {
#pragma unroll
        for (int rd = 0; rd < RB; ++rd)
          glds16(B.src(rd * GEMM_THREADS + tid, n0, k0), tb + (rd * GEMM_THREADS + wid_u * 64) * 16);
      }
    }
  };
  // ---- normalize on load: the transformed operand goes global -> VGPR (xload) -> transform -> LDS (xstore)
  constexpr int RX = XF == 1 ? RA : (XF == 2 ? RB : 1);
  bf16x8_t xr[RX];
  bool xok[RX];
  float xsc[8], xsh[8];
  // a thread's 16-B slots all cover the same 8 channels: K-major chunk (tid & 7) ^ ((tid >> 4) & 7) of the K step
  // (A), or MN-major unit (tid & 15) ^ mn_swz(tid >> 4) of the tile's columns (B) -- fixed for the whole kernel
  if constexpr (XF == 2) {
    const int col = n0 + (((tid & 15) ^ mn_swz(tid >> 4)) << 3);
    const int ch = col < N ? col - X.fC.div(col) * X.C : 0;
    load_f8g(X.p + ch, xsc);
    load_f8g(X.p + X.C + ch, xsh);
  }
  auto xload = [&](int k0) {
    if constexpr (XF == 1) {
      const int ch = A.chan0(k0) + (((tid & 7) ^ ((tid >> 4) & 7)) << 3);
      load_f8g(X.p + ch, xsc);
      load_f8g(X.p + X.C + ch, xsh);
      if constexpr (HOIST) {
        const auto tpa = A.tap(k0);
#pragma unroll
        for (int rd = 0; rd < RA; ++rd) {
          const void* q = A.at(ca[rd], tpa);
          xok[rd] = q != (const void*)g_zero_page;
          xr[rd] = *reinterpret_cast<const bf16x8_t*>(q);
        }
      } else {
#pragma unroll
        for (int rd = 0; rd < RA; ++rd) {
          const void* q = A.src(rd * GEMM_THREADS + tid, m0, k0);
          xok[rd] = q != (const void*)g_zero_page;
          xr[rd] = *reinterpret_cast<const bf16x8_t*>(q);
        }
      }
    } else if constexpr (XF == 2) {
      if constexpr (HOIST) {
        const auto tpb = B.tap(k0);
#pragma unroll
        for (int rd = 0; rd < RB; ++rd) {
          const void* q = B.at(cb[rd], tpb);
          xok[rd] = q != (const void*)g_zero_page;
          xr[rd] = *reinterpret_cast<const bf16x8_t*>(q);
        }
      } else {
#pragma unroll
        for (int rd = 0; rd < RB; ++rd) {
          const void* q = B.src(rd * GEMM_THREADS + tid, n0, k0);
          xok[rd] = q != (const void*)g_zero_page;
          xr[rd] = *reinterpret_cast<const bf16x8_t*>(q);
        }
      }
    }
  };
  auto xstore = [&](int buf) {
    if constexpr (XF != 0) {
      char* t = smem + buf * (TA + TB) + (XF == 1 ? 0 : TA);
#pragma unroll
      for (int rd = 0; rd < RX; ++rd)
        *reinterpret_cast<bf16x8_t*>(t + (rd * GEMM_THREADS + tid) * 16) = bn_relu8(xr[rd], xsc, xsh, xok[rd]);
    }
  };

  constexpr int CPR = BN / 8;  // 16-B chunks per output-tile row
  if (nt > 0) {
    stage(0, kbeg);
    xload(kbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    xstore(0);
    __syncthreads();
  }
  for (int t = 0; t < nt; ++t) {
    const int cur = NBUF == 1 ? 0 : (t & 1);
    if (NBUF == 1) {
      if (t > 0) {  // the previous tile's reads are done (barrier at the end of the last iteration)
        stage(0, kbeg + t * BK);
        xload(kbeg + t * BK);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        xstore(0);
        __syncthreads();
      }
    } else if (t + 1 < nt) {
      stage(cur ^ 1, kbeg + (t + 1) * BK);
      xload(kbeg + (t + 1) * BK);
    }
    const char* ta = smem + cur * (TA + TB);
    const char* tb = ta + TA;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      mfma_bf16x8 af[4], bfv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<ASrc>(ta, wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfv[j] = frag<BSrc>(tb, wn * 64 + j * 16, kk, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfv[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (NBUF == 2 && t + 1 < nt) xstore(cur ^ 1);  // the idle buffer: its last reader finished before the last barrier
    __syncthreads();
  }

  // ---- epilogue: lane holds C[m][n..n+3]
  // locals, not writes into the by-value kernarg struct: mutating E makes the compiler copy the whole
  // (large) Epi into scratch memory
  void* const ec = E.mode == 3 ? (void*)(reinterpret_cast<float*>(E.c) + (long)zsplit * E.slab) : E.c;
  const int emode = E.mode == 3 ? 0 : E.mode;  // mode 3 = this split's private fp32 slab, plain stores
  // LEAN (bf16 C, no bias / activation / pre-activation copy, mode store or accumulate; the convolution forward
  // and the data gradients): the tile goes through LDS and leaves as 16-B row-contiguous stores, and none of the
  // general epilogue's run-time branches are compiled in (the general instantiations are ~85 KB of code, more
  // than the instruction cache). LDS image [BM][BN] bf16, 16-B chunk c of row r at c ^ (r % (BN / 8)).
  uint16_t* const ctile = reinterpret_cast<uint16_t*>(smem);
  float st_s[4][4], st_q[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) st_s[j][r] = st_q[j][r] = 0.f;
  if constexpr (LEAN) {
    if constexpr (BST && XE < XR) {
      if (!E.rst) load_bxr(XE, XR);
    }
    // bias (fp32, added before the one bf16 rounding of the staged value): this lane's 4 columns of each j
    float bj[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) bj[j][r] = (XEPI && E.bias && n + r < N) ? E.bias[n + r] : 0.f;
    }
    // alpha is 1 for every convolution and data gradient: the scaling pass runs only when it is not (one
    // wave-uniform branch instead of 64 multiplies per lane on every tile)
    if (XEPI || E.alpha != 1.f) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[i][j][r] = XEPI ? __builtin_fmaf(acc[i][j][r], E.alpha, bj[j][r]) : acc[i][j][r] * E.alpha;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + (lane >> 4) * 4;
        // 4 fp32 -> 4 bf16: two v_cvt_pk_bf16_f32, no per-element packing
        const bf16x4_t o = __builtin_bit_cast(bf16x4_t, __builtin_convertvector(acc[i][j], bf16v4_t));
        *reinterpret_cast<bf16x4_t*>(ctile + row * BN + (((col >> 3) ^ (row % CPR)) << 3) + (col & 4)) = o;
      }
    }
    __syncthreads();
    // copy-out: thread t always handles 16-B chunk c = t % CPR of its rows (GEMM_THREADS % CPR == 0), so it
    // also accumulates the BN statistics (sum, sum of squares) of those 8 columns from the bf16 values it stores
    float* const stat_out = BST ? E.bb.sums : E.stats;
    float ps[8], pq[8], pq2[BST ? 8 : 1];
#pragma unroll
    for (int r = 0; r < 8; ++r) ps[r] = pq[r] = 0.f;
    if constexpr (BST) {
#pragma unroll
      for (int r = 0; r < 8; ++r) pq2[r] = 0.f;
    }
    constexpr int CHUNKS = BM * CPR;
    // fast path (convolution forward with statistics, plain and accumulating data gradients): identity rows. A
    // thread's chunk column is fixed and its rows advance by GEMM_THREADS / CPR per trip, so the
    // output pointer is one 64-bit add per trip; the statistics use packed fp32 adds / FMAs on the unpacked pairs.
    if (!XEPI && !E.rst) {
      constexpr int RSTEP = GEMM_THREADS / CPR;
      const int c = tid % CPR, row0 = tid / CPR;
      const int n = n0 + c * 8;
      if (n < N) {
        const long ldc = E.ldc;
        const long off0 = (long)(m0 + row0) * ldc + n;
        uint16_t* cp = reinterpret_cast<uint16_t*>(ec) + off0;
        // accumulate mode: the addend (C's old value, or addsrc masked by addmask -- a ResNet identity block's
        // residual gradient) walks with the output
        const uint16_t* ap = emode == 1 ? (E.addsrc ? E.addsrc + off0 : cp) : nullptr;
        const uint8_t* mp = emode == 1 && E.addmask ? E.addmask + (off0 >> 3) : nullptr;
        const uint16_t* lp = ctile + row0 * BN;
        f32x2_t s2[4], q2[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) s2[r] = q2[r] = f32x2_t{0.f, 0.f};
        // BST: this thread's 8 columns' ReLU affine (the forward's, recomputed bit-identically) and means; x walks
        // with the output (ldc == N). Mask kind (bb.mask, a BatchNorm whose ReLU bits are stored: the stem pool's
        // output): g = bit ? dx : 0, and the product may accumulate onto C (an unmasked addend: the first of two
        // data gradients into the same tensor)
        // Two-BatchNorm form (bb.x2, mask kind only): bsh holds the second BN's means, q2b its sum g (x2 - mean2).
        float bsc[BST ? 8 : 1], bsh[BST ? 8 : 1], bmu[BST ? 8 : 1];
        if constexpr (BST) {
          const bool mk = E.bb.mask != nullptr;
          const uint16_t* const x2p = E.bb.x2 ? E.bb.x2 + off0 : nullptr;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            bmu[j] = E.bb.mean[n + j];
            bsc[j] = 0.f;
            bsh[j] = x2p ? E.bb.mean2[n + j] : 0.f;
            if (!mk) bn_affine_regs(E.bb.gamma[n + j], E.bb.beta[n + j], bmu[j], E.bb.invstd[n + j], bsc[j], bsh[j]);
          }
#pragma unroll
          for (int i = 0; i < XR; ++i) {  // whole tile, unrolled: the prefetched x registers indexed statically
            const int row = row0 + i * RSTEP;
            if (m0 + row < M) {
              bf16x8_t o = *reinterpret_cast<const bf16x8_t*>(lp + i * RSTEP * BN + ((c ^ (row % CPR)) << 3));
              if (ap) {  // (the general path's rounding: the staged bf16 value + old C, one more rounding)
                const bf16x8_t old = *reinterpret_cast<const bf16x8_t*>(ap + (long)i * RSTEP * ldc);
                const uint32_t abits = mp ? (uint32_t)mp[((long)i * RSTEP * ldc) >> 3] : 0xFFu;
                float f[8];
#pragma unroll
                for (int r = 0; r < 8; ++r)
                  f[r] = bf2f((uint16_t)o[r]) + (((abits >> r) & 1u) ? bf2f((uint16_t)old[r]) : 0.f);
                o = pack_bf16x8(f);
              }
              *reinterpret_cast<bf16x8_t*>(cp + (long)i * RSTEP * ldc) = o;
              const uint32_t bits = mk ? (uint32_t)E.bb.mask[(off0 + (long)i * RSTEP * ldc) >> 3] : 0u;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                f32x2_t g, d;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                  const float xf = bf2f((uint16_t)bxr[i][2 * r + e]);
                  const bool on = mk ? ((bits >> (2 * r + e)) & 1u) != 0 : relu_on(xf, bsc[2 * r + e], bsh[2 * r + e]);
                  g[e] = on ? bf2f((uint16_t)o[2 * r + e]) : 0.f;
                  d[e] = xf - bmu[2 * r + e];
                }
                s2[r] += g;
                q2[r] = __builtin_elementwise_fma(g, d, q2[r]);
              }
              if (x2p) {
                const bf16x8_t x2v = *reinterpret_cast<const bf16x8_t*>(x2p + (long)i * RSTEP * ldc);
#pragma unroll
                for (int r = 0; r < 8; ++r) {
                  const float g = ((bits >> r) & 1u) ? bf2f((uint16_t)o[r]) : 0.f;
                  pq2[r] = __builtin_fmaf(g, bf2f((uint16_t)x2v[r]) - bsh[r], pq2[r]);
                }
              }
            }
          }
        } else {
#pragma unroll 4
        for (int row = row0; row < BM; row += RSTEP) {
          if (m0 + row < M) {
            bf16x8_t o = *reinterpret_cast<const bf16x8_t*>(lp + ((c ^ (row % CPR)) << 3));
            if (ap) {  // one extra bf16 rounding on top of the staged value (<= 1 ulp), as the general path
              const bf16x8_t old = *reinterpret_cast<const bf16x8_t*>(ap);
              const uint32_t bits = mp ? (uint32_t)*mp : 0xFFu;
              float f[8];
#pragma unroll
              for (int r = 0; r < 8; ++r)
                f[r] = bf2f((uint16_t)o[r]) + (((bits >> r) & 1u) ? bf2f((uint16_t)old[r]) : 0.f);
              o = pack_bf16x8(f);
            }
            *reinterpret_cast<bf16x8_t*>(cp) = o;
            if (stat_out) {
              const uint32_t* w = reinterpret_cast<const uint32_t*>(&o);
#pragma unroll
              for (int r = 0; r < 4; ++r) {  // pair r = elements (2r, 2r+1): bf16 -> fp32 is a shift / a mask
                const f32x2_t v = {__uint_as_float(w[r] << 16), __uint_as_float(w[r] & 0xFFFF0000u)};
                s2[r] += v;
                q2[r] = __builtin_elementwise_fma(v, v, q2[r]);
              }
            }
          }
          cp += (long)RSTEP * ldc;
          lp += RSTEP * BN;
          if (ap) ap += (long)RSTEP * ldc;
          if (mp) mp += ((long)RSTEP * ldc) >> 3;
        }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ps[2 * r] = s2[r][0];
          ps[2 * r + 1] = s2[r][1];
          pq[2 * r] = q2[r][0];
          pq[2 * r + 1] = q2[r][1];
        }
      }
    } else {
    // BST on the row-remapped (sub-grid) path: the correction of a residual BatchNorm's backward sums (packed ReLU
    // bits bb.mask) for the elements this accumulating product changes -- sum bit (new - old), sum bit (new - old)
    // (x - mean) -- the first data gradient into the same tensor having counted the old values (ops.conv)
    // Relu kind (no bb.mask, a plain store: the parities of a stride-2 3x3 data gradient, each writing its own
    // pixels): g = relu_on(x) ? dx : 0 from the BatchNorm's affine, sum g and sum g (x - mean) of the stored values.
    float gmu[BST ? 8 : 1], gsc[BST ? 8 : 1], gsh[BST ? 8 : 1];
    if constexpr (BST) {
      const int nt = n0 + (tid % CPR) * 8;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        gmu[r] = nt + r < N ? E.bb.mean[nt + r] : 0.f;
        gsc[r] = gsh[r] = 0.f;
        if (!E.bb.mask && nt + r < N)
          bn_affine_regs(E.bb.gamma[nt + r], E.bb.beta[nt + r], gmu[r], E.bb.invstd[nt + r], gsc[r], gsh[r]);
      }
    }
#pragma unroll 2
    for (int q = tid; q < CHUNKS; q += GEMM_THREADS) {
      const int row = q / CPR, c = q % CPR;
      const int m = m0 + row, n = n0 + c * 8;
      if (m >= M || n >= N) continue;
      long orow = m;
      if (E.rst) {
        const int hw = E.rHo * E.rWo;
        const int nimg = m / hw, rem = m - nimg * hw;
        const int ii = rem / E.rWo, jj = rem - ii * E.rWo;
        orow = ((long)nimg * E.rH + ii * E.rst + E.ra) * E.rW + jj * E.rst + E.rb;
      }
      bf16x8_t o = *reinterpret_cast<const bf16x8_t*>(ctile + row * BN + ((c ^ (row % CPR)) << 3));
      uint16_t* cp = reinterpret_cast<uint16_t*>(ec) + orow * E.ldc + n;
      if constexpr (XEPI) {
        if (E.pre) *reinterpret_cast<bf16x8_t*>(E.pre + orow * E.ldc + n) = o;  // pre-activation (+ bias), bf16
        if (E.act) {  // activation of the staged bf16 pre-activation (what the GELU / ReLU backward reads)
          float a8[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const float v = bf2f((uint16_t)o[r]);
            a8[r] = E.act == 1 ? fmaxf(v, 0.f) : gelu_tanh(v);
          }
          o = pack_bf16x8(a8);
        }
      }
      if (emode == 1) {  // accumulate onto bf16 C: the staged value is already bf16 (two roundings, <= 1 ulp more)
        const long aoff = orow * E.ldc + n;
        bf16x8_t old = *reinterpret_cast<const bf16x8_t*>(E.addsrc ? E.addsrc + aoff : cp);
        if (E.addmask) {
          const uint32_t abits = E.addmask[aoff >> 3];
#pragma unroll
          for (int r = 0; r < 8; ++r) old[r] = ((abits >> r) & 1u) ? old[r] : (short)0;
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) o[r] = (short)f2bf(bf2f((uint16_t)o[r]) + bf2f((uint16_t)old[r]));
        if constexpr (BST) {
          const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(E.bb.x + aoff);
          const uint32_t bits = E.bb.mask[aoff >> 3];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const float d = ((bits >> r) & 1u) ? bf2f((uint16_t)o[r]) - bf2f((uint16_t)old[r]) : 0.f;
            ps[r] += d;
            pq[r] = __builtin_fmaf(d, bf2f((uint16_t)xv[r]) - gmu[r], pq[r]);
          }
        }
      }
      if constexpr (BST) {
        if (!E.bb.mask) {
          const bf16x8_t xv = *reinterpret_cast<const bf16x8_t*>(E.bb.x + orow * E.ldc + n);
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const float xf = bf2f((uint16_t)xv[r]);
            const float g = relu_on(xf, gsc[r], gsh[r]) ? bf2f((uint16_t)o[r]) : 0.f;
            ps[r] += g;
            pq[r] = __builtin_fmaf(g, xf - gmu[r], pq[r]);
          }
        }
      }
      *reinterpret_cast<bf16x8_t*>(cp) = o;
      if (!BST && stat_out) {  // (BST: stat_out is the BatchNorm sums, corrected above)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const float v = bf2f((uint16_t)o[r]);
          ps[r] += v;
          pq[r] += v * v;
        }
      }
    }
    }
    if (stat_out) {
      // partials [GEMM_THREADS][16] in LDS, then thread (which, col) sums the GEMM_THREADS / CPR partials of its
      // column: one atomic per (column, sum | sum of squares) per block
      __syncthreads();
      float* part = reinterpret_cast<float*>(smem);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        part[tid * 16 + r] = ps[r];
        part[tid * 16 + 8 + r] = pq[r];
      }
      __syncthreads();
      if (tid < 2 * BN) {
        const int col = tid % BN, which = tid / BN;
        const int n = n0 + col;
        if (n < N) {
          const int c = col >> 3, r = col & 7;
          float v = 0.f;
#pragma unroll 4
          for (int t = c; t < GEMM_THREADS; t += CPR) v += part[t * 16 + which * 8 + r];
          atomicAdd(stat_out + (long)(tm % STAT_REPL) * 2 * N + (long)which * N + n, v);
        }
      }
      if constexpr (BST) {
        if (E.bb.x2) {  // the second BatchNorm's sum g (x2 - mean2) into sums2[.][1] (its sum g is the first's)
          __syncthreads();
#pragma unroll
          for (int r = 0; r < 8; ++r) part[tid * 16 + r] = pq2[r];
          __syncthreads();
          if (tid < BN) {
            const int n = n0 + tid;
            if (n < N) {
              const int c = tid >> 3, r = tid & 7;
              float v = 0.f;
#pragma unroll 4
              for (int t = c; t < GEMM_THREADS; t += CPR) v += part[t * 16 + r];
              atomicAdd(E.bb.sums2 + (long)(tm % STAT_REPL) * 2 * N + N + n, v);
            }
          }
        }
      }
    }
    return;
  } else {
    if constexpr (F32S && WM == 2 && WN == 2) {
      if (E.out_f32 && emode != 2 && !E.bias && !E.pre && E.act == 0 && !E.stats && !E.rst && (E.ldc & 3) == 0 &&
          (N & 3) == 0) {
        __syncthreads();  // every wave is past its last K-loop LDS read
        // wave (wm, wn): its 64 x 64 piece in two 32-row halves, [32 rows][64 cols] fp32 (8 KB, wave-private)
        float* const st = reinterpret_cast<float*>(smem) + (wm * WN + wn) * (32 * 64);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          if (h) {
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's reads of the first half are done
            asm volatile("" ::: "memory");
          }
#pragma unroll
          for (int i2 = 0; i2 < 2; ++i2) {
            const int lr = i2 * 16 + (lane & 15);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int ch = (j * 4 + (lane >> 4)) ^ (lr & 15);  // 16-B chunk, XOR-swizzled by the row
              *reinterpret_cast<f32x4_t*>(reinterpret_cast<char*>(st) + lr * 256 + ch * 16) =
                  acc[2 * h + i2][j] * E.alpha;
            }
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the staging writes landed
          asm volatile("" ::: "memory");
#pragma unroll
          for (int it = 0; it < 8; ++it) {
            const int idx = it * 64 + lane;
            const int lr = idx >> 4, ch = idx & 15;
            const int m = m0 + wm * 64 + h * 32 + lr, n = n0 + wn * 64 + ch * 4;
            f32x4_t v = *reinterpret_cast<const f32x4_t*>(reinterpret_cast<const char*>(st) + lr * 256 +
                                                          ((ch ^ (lr & 15)) << 4));
            if (m < M && n < N) {
              float* cp = reinterpret_cast<float*>(ec) + (long)m * E.ldc + n;
              if (emode == 1) v += *reinterpret_cast<const f32x4_t*>(cp);
              *reinterpret_cast<f32x4_t*>(cp) = v;
            }
          }
        }
        return;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + (lane & 15);
      if (m >= M) continue;
      long orow = m;
      if (E.rst) {
        const int hw = E.rHo * E.rWo;
        const int nimg = m / hw, rem = m - nimg * hw;
        const int ii = rem / E.rWo, jj = rem - ii * E.rWo;
        orow = ((long)nimg * E.rH + ii * E.rst + E.ra) * E.rW + jj * E.rst + E.rb;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
        if (n >= N) continue;
        float v[4] = {acc[i][j][0] * E.alpha, acc[i][j][1] * E.alpha, acc[i][j][2] * E.alpha,
                      acc[i][j][3] * E.alpha};
        const bool full = (n + 3 < N);
        if (E.bias) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < N) v[r] += E.bias[n + r];
        }
        if (E.pre) {
          uint16_t* pp = E.pre + orow * E.ldc + n;
          if (full) {
            bf16x4_t o;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
            *reinterpret_cast<bf16x4_t*>(pp) = o;
          } else {
            for (int r = 0; r < 4 && n + r < N; ++r) pp[r] = f2bf(v[r]);
          }
        }
        if (E.act == 1) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        } else if (E.act == 2) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
        }
        if (E.stats) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float vr = E.out_f32 ? v[r] : bf2f(f2bf(v[r]));  // statistics of what is stored
            const bool ok = n + r < N;
            st_s[j][r] += ok ? vr : 0.f;
            st_q[j][r] += ok ? vr * vr : 0.f;
          }
        }
        if (E.out_f32) {
          float* cp = reinterpret_cast<float*>(ec) + orow * E.ldc + n;
          if (emode == 2) {
            for (int r = 0; r < 4 && n + r < N; ++r) atomicAdd(cp + r, v[r]);
          } else if (full) {
            float4 o = make_float4(v[0], v[1], v[2], v[3]);
            if (emode == 1) {
              const float4 old = *reinterpret_cast<const float4*>(cp);
              o.x += old.x; o.y += old.y; o.z += old.z; o.w += old.w;
            }
            *reinterpret_cast<float4*>(cp) = o;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < N) cp[r] = (emode == 1 ? cp[r] : 0.f) + v[r];
          }
        } else {
          uint16_t* cp = reinterpret_cast<uint16_t*>(ec) + orow * E.ldc + n;
          if (full) {
            bf16x4_t o;
            if (emode == 1) {
              const bf16x4_t old = *reinterpret_cast<const bf16x4_t*>(cp);
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] += bf2f((uint16_t)old[r]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) o[r] = (short)f2bf(v[r]);
            *reinterpret_cast<bf16x4_t*>(cp) = o;
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {  // static r: keeps st_s/st_q in registers (a dynamic bound spills them)
              if (n + r >= N) continue;
              const uint16_t o = f2bf(v[r] + (emode == 1 ? bf2f(cp[r]) : 0.f));
              cp[r] = o;
            }
          }
        }
      }
    }
  }
  float* const stat_out = E.stats;
  if (stat_out) {
    // lanes with equal (lane >> 4) hold the same 4 columns: reduce over the 16 row lanes (DPP), then over the
    // row-waves through LDS, so the block issues 2 * BN / 64 full-wave atomic instructions instead of 128
    // quarter-empty ones -- float atomics cost ~50 ns per wave-instruction per CU.
    float* red = reinterpret_cast<float*>(smem);  // [wm][2][BN]; the K loop's last barrier freed the tiles
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = row16_sum(st_s[j][r]), b = row16_sum(st_q[j][r]);
        if ((lane & 15) == 0) {
          const int col = wn * 64 + j * 16 + (lane >> 4) * 4 + r;
          red[(wm * 2 + 0) * BN + col] = a;
          red[(wm * 2 + 1) * BN + col] = b;
        }
      }
    }
    __syncthreads();
    if (tid < 2 * BN) {
      const int col = tid % BN, which = tid / BN;
      const int n = n0 + col;
      if (n < N) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) v += red[(w * 2 + which) * BN + col];
        atomicAdd(stat_out + (long)(tm % STAT_REPL) * 2 * N + (long)which * N + n, v);
      }
    }
  }
}

// ----------------------------------------------------------------------------- host side
// Single-buffered (3 blocks / CU) kernel up to this K range per block, double-buffered (2 blocks / CU) above.
// Measured on the ResNet-50 b1024 step (round 1, one box, 2 rounds): 128 -> 12.20k img/s, 256 -> 12.46k,
// 512 -> 12.57k, 1024 -> 12.57k, 2304 -> 12.54k, all -> 12.44k: a third block per CU hides more load latency than a
// second LDS buffer does on these short / memory-bound K loops.
constexpr int kSingleBufMaxK = 8 * BK;
static int single_buf_maxk() { return kSingleBufMaxK; }

// splits actually launched for a requested count (each split a whole number of BK tiles)
static int effective_splits(int K, int splits) {
  if (splits <= 1) return 1;
  const int kps = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  return (K + kps - 1) / kps;
}

template <class ASrc, class BSrc, int WM, int WN, bool LEAN, bool XEPI = false, bool F32S = false, int XF = 0,
          bool BST = false>
static void launch_tiles2(const ASrc& a, const BSrc& b, const Epi& e, int M, int N, int K, int kps, int splits,
                          hipStream_t st, const XForm& x = XForm{nullptr, 0, FastDiv{}}) {
  const int tiles = ((M + 64 * WM - 1) / (64 * WM)) * ((N + 64 * WN - 1) / (64 * WN));
  if (kps <= single_buf_maxk())
    hipLaunchKernelGGL((gemm_bf16_kernel<ASrc, BSrc, 1, WM, WN, LEAN, XEPI, F32S, XF, BST>), dim3(tiles, 1, splits),
                       dim3(GEMM_THREADS), 0, st, a, b, e, M, N, K, kps, x);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<ASrc, BSrc, 2, WM, WN, LEAN, XEPI, F32S, XF, BST>), dim3(tiles, 1, splits),
                       dim3(GEMM_THREADS), 0, st, a, b, e, M, N, K, kps, x);
}

// the lean epilogue applies: bf16 C (16-B aligned rows), store or accumulate, no atomics; bias / ReLU / GELU /
// pre-activation copy in store mode on identity rows without statistics (the transformer linears: measured on
// BERT-base's QKV / FFN1 forward 81 / 105 us per call through the general per-lane epilogue)
static bool epi_extra(const Epi& e) { return e.bias || e.pre || e.act != 0; }
static bool lean_epi(const Epi& e, int N, bool allow_extra) {
  if (epi_extra(e) && (!allow_extra || e.mode != 0 || e.rst || e.stats || e.addsrc ||
                       (reinterpret_cast<uintptr_t>(e.pre) & 15) != 0))
    return false;
  return !e.out_f32 && (e.mode == 0 || e.mode == 1) && (e.ldc & 7) == 0 && (N & 7) == 0 &&
         (reinterpret_cast<uintptr_t>(e.c) & 15) == 0;
}

template <class ASrc, class BSrc, int WM, int WN>
static void launch_tiles(const ASrc& a, const BSrc& b, const Epi& e, int M, int N, int K, int kps, int splits,
                         hipStream_t st, const XForm* xf = nullptr) {
  // normalize-on-load instantiations: the convolution forward (A = the BN input, lean epilogue with statistics) and
  // the weight gradients (B = the BN input, fp32 output or split-K slab through the F32S epilogue)
  if (xf) {
    if constexpr ((std::is_same_v<ASrc, ConvA> || std::is_same_v<ASrc, KMajor>) && std::is_same_v<BSrc, KMajor>) {
      if (lean_epi(e, N, false) && !e.rst && !e.addsrc) {
        launch_tiles2<ASrc, BSrc, WM, WN, true, false, false, 1>(a, b, e, M, N, K, kps, splits, st, *xf);
        return;
      }
    }
    if constexpr (std::is_same_v<ASrc, MNMajorK> && (std::is_same_v<BSrc, ConvWgB> || std::is_same_v<BSrc, MNMajorK>) &&
                  WM == 2 && WN == 2) {
      if (e.out_f32 && e.mode != 2 && !epi_extra(e) && !e.stats && !e.rst) {
        launch_tiles2<ASrc, BSrc, WM, WN, false, false, true, 2>(a, b, e, M, N, K, kps, splits, st, *xf);
        return;
      }
    }
    throw std::runtime_error("normalize-on-load: no instantiation for this operand pair / epilogue");
  }
  // a data gradient (K-major dy, MN-major w) with the BatchNorm-backward sums of its output
  if (e.bb.sums) {
    if constexpr (std::is_same_v<ASrc, KMajor> && std::is_same_v<BSrc, MNMajorK> && WM == 2 && WN == 2) {
      if (lean_epi(e, N, false) && (e.mode == 0 || (e.mode == 1 && e.bb.mask)) && !e.stats && !e.rst &&
          (!e.addmask || e.addsrc) && splits == 1 && e.ldc == N) {
        launch_tiles2<ASrc, BSrc, WM, WN, true, false, false, 0, true>(a, b, e, M, N, K, kps, splits, st);
        return;
      }
    }
    // the row-remapped (sub-grid) data gradients: a 1x1 parity accumulating a residual BatchNorm's correction (mask
    // kind), or a parity of a stride-2 convolution's data gradient storing with a BatchNorm + ReLU's sums (relu kind;
    // the 1x1 parity on the K-major source, the others on the implicit GEMM)
    if constexpr ((std::is_same_v<ASrc, KMajor> || std::is_same_v<ASrc, ConvA>) && std::is_same_v<BSrc, KMajor> &&
                  WM == 2 && WN == 2) {
      if (lean_epi(e, N, false) && !e.stats && e.rst && !e.addsrc && !e.addmask && splits == 1 &&
          ((e.mode == 1 && e.bb.mask && std::is_same_v<ASrc, KMajor>) || (e.mode == 0 && !e.bb.mask))) {
        launch_tiles2<ASrc, BSrc, WM, WN, true, false, false, 0, true>(a, b, e, M, N, K, kps, splits, st);
        return;
      }
    }
    throw std::runtime_error("BatchNorm-backward sums epilogue: a plain bf16 data gradient (K-major dy, MN-major w)");
  }
  // the linear forward (both operands K-major) is the one pair with a bias / activation epilogue instantiation
  constexpr bool kXepi = std::is_same_v<ASrc, KMajor> && std::is_same_v<BSrc, KMajor>;
  if constexpr (kXepi) {
    if (epi_extra(e) && lean_epi(e, N, true)) {
      launch_tiles2<ASrc, BSrc, WM, WN, true, true>(a, b, e, M, N, K, kps, splits, st);
      return;
    }
  }
  if constexpr (!std::is_same_v<BSrc, ConvWgB>) {
    if (lean_epi(e, N, false)) {
      launch_tiles2<ASrc, BSrc, WM, WN, true>(a, b, e, M, N, K, kps, splits, st);
      return;
    }
  }
  if (e.addsrc || e.addmask) throw std::runtime_error("a separate (masked) addend needs the lean epilogue");
  // weight gradients (both operands MN-major: dense or im2col) with an fp32 output or split-K slab
  constexpr bool kWgrad = std::is_same_v<ASrc, MNMajorK> &&
                          (std::is_same_v<BSrc, MNMajorK> || std::is_same_v<BSrc, ConvWgB>);
  if constexpr (kWgrad && WM == 2 && WN == 2) {
    if (e.out_f32 && e.mode != 2 && !epi_extra(e) && !e.stats && !e.rst) {
      launch_tiles2<ASrc, BSrc, WM, WN, false, false, true>(a, b, e, M, N, K, kps, splits, st);
      return;
    }
  }
  launch_tiles2<ASrc, BSrc, WM, WN, false>(a, b, e, M, N, K, kps, splits, st);
}

template <class ASrc, class BSrc>
static void launch(const ASrc& a, const BSrc& b, const Epi& e, int M, int N, int K, int splits, hipStream_t st,
                   const XForm* xf = nullptr) {
  const int kps = ((K + splits - 1) / splits + BK - 1) / BK * BK;
  splits = (K + kps - 1) / kps;
  if constexpr (ASrc::kmajor && BSrc::kmajor) {
    if (N <= 64) {  // 256 x 64 tiles: no half-empty 128-wide column tile
      launch_tiles<ASrc, BSrc, 4, 1>(a, b, e, M, N, K, kps, splits, st, xf);
      return;
    }
  }
  launch_tiles<ASrc, BSrc, 2, 2>(a, b, e, M, N, K, kps, splits, st, xf);
}

static Epi make_epi(void* c, long ldc, bool out_f32, const float* bias, int act, uint16_t* pre, int mode,
                    float alpha) {
  Epi e;
  e.c = c;
  e.ldc = ldc;
  e.bias = bias;
  e.pre = pre;
  e.out_f32 = out_f32;
  e.act = act;
  e.mode = mode;
  e.alpha = alpha;
  e.stats = nullptr;
  e.slab = 0;
  e.rst = e.rHo = e.rWo = e.rH = e.rW = e.ra = e.rb = 0;
  e.addsrc = nullptr;
  e.addmask = nullptr;
  e.bb = BnBwdSums{};
  // (Issuing the next K step's loads behind the first MFMA half sped up the isolated 56x56 / 28x28 3x3 convolutions
  // 7-12 % but cost the ResNet-50 step 1.5 % at any K threshold -- round 2, scripts/gpurun/bench_ab.sh; removed.)
  return e;
}

// Choose split-K for small-MN / tall-K products (weight gradients) with a wave-quantisation cost model:
//   T(s) = ceil(tiles * s / slots) * ceil(ktiles / s)            -- block rounds x K tiles per block
//        + s * M * N * 8 B / HBM BW / t_ktile                     -- fp32 slab write + reduce read per split
// slots = resident blocks on the chip's CUs (planner_cus(); 2 per CU double-buffered, 3 single-buffered). The previous rule
// (double s until tiles * s >= 512) landed most ResNet-50 3x3 weight gradients on 576 blocks = 1.125
// rounds; measured on MI355X (scripts/sweep_wgrad_splits.py) the model's choice is 1.3-1.5x faster there.
// At most 256 splits: measured with up to 1024, the single-tile 64x64 1x1 weight gradient got slower (134 ->
// 189 us) -- the combine kernel's per-thread serial loop over the splits dominates.
int gemm_choose_splits(int M, int N, int K) {
  const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int ktiles = (K + BK - 1) / BK;
  const double slab_cost = (double)M * N * 8.0 / 5.0e12 / 2.0e-6;  // in units of one K tile (~2 us / block)
  const long cus = planner_cus();
  int best_s = 1;
  double best = 1e30;
  for (int s = 1; s <= 256 && s <= ktiles; ++s) {
    const int kpt = (ktiles + s - 1) / s;       // K tiles per split
    if ((ktiles + kpt - 1) / kpt != s) continue;  // same kps as a smaller s
    const long slots = kpt * BK <= single_buf_maxk() ? 3 * cus : 2 * cus;
    const long rounds = (tiles * s + slots - 1) / slots;
    const double t = (double)rounds * kpt + (s > 1 ? s * slab_cost : 0.0);
    if (t < best * 0.999) {
      best = t;
      best_s = s;
    }
  }
  return best_s;
}

// out[i] (+)= sum_z ws[z][i]  -- the split-K combine (float4 over MN, MN % 4 == 0)
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int splits, long mn4, float* __restrict__ out,
                                     int accumulate) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < mn4; i += (long)gridDim.x * blockDim.x) {
    float4 acc = accumulate ? reinterpret_cast<const float4*>(out)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int z = 0; z < splits; ++z) {  // slab loads of up to 8 splits in flight
      const float4 v = reinterpret_cast<const float4*>(ws)[(long)z * mn4 + i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
}

void splitk_reduce(const float* ws, int splits, long mn, float* out, bool accumulate, hipStream_t st) {
  const long mn4 = mn / 4;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(stream_grid(mn4, 256)), dim3(256), 0, st, ws, splits, mn4, out,
                     accumulate ? 1 : 0);
}

long gemm_splitk_workspace(int M, int N, int splits) { return splits > 1 ? (long)splits * M * N : 0; }

// C[M,N] = act(alpha * op(A) op(B) + bias)
//  a_kmajor: A stored [M][K] (lda) else [K][M];  b_kmajor: B stored [N][K] (ldb) else [K][N]
//  mode 0 store / 1 accumulate; with splits > 1 (fp32 C, plain epilogue) the K range is split over
//  blockIdx.z, each split writes an fp32 slab of `ws` and a reduce kernel combines them into C.
void launch_gemm(const uint16_t* A, long lda, bool a_kmajor, const uint16_t* B, long ldb, bool b_kmajor, void* C,
                 long ldc, bool c_f32, int M, int N, int K, const float* bias, int act, uint16_t* pre, int mode,
                 float alpha, int splits, float* ws, hipStream_t st, const AddEpi* add,
                 const float* xform_b, int xform_c) {
  splits = effective_splits(K, splits);
  // the data-gradient form (K-major dy, MN-major w) of a short reduction: the streaming kernel of gemm_short.hip
  if (a_kmajor && !b_kmajor && !c_f32 && !bias && act == 0 && !pre && (mode == 0 || mode == 1) && splits == 1 &&
      alpha == 1.f && !xform_b && ldb == N && (!add || add->mask) && gemm_short_ok(M, N, K, lda, ldc)) {
    launch_gemm_short(A, B, ldb, true, reinterpret_cast<uint16_t*>(C), add ? add->src : nullptr,
                      add ? add->mask : nullptr, nullptr, nullptr, M, N, K, add ? 2 : mode, st);
    return;
  }
  const bool slab = splits > 1;
  Epi e = make_epi(slab ? (void*)ws : C, slab ? (long)N : ldc, c_f32, bias, act, pre, slab ? 3 : mode, alpha);
  e.slab = (long)M * N;
  if (add) {
    if (slab || mode != 1) throw std::runtime_error("a separate addend needs accumulate mode and no split-K");
    e.addsrc = add->src;
    e.addmask = add->mask;
  }
  if (xform_b) {  // B = relu(bn(x)) normalised on load: the plain (1x1) weight gradient
    if (a_kmajor || b_kmajor) throw std::runtime_error("normalize-on-load GEMM: MN-major A and B");
    const XForm xf{xform_b, xform_c, make_fastdiv(xform_c)};
    launch(MNMajorK{A, lda, M, K}, MNMajorK{B, ldb, N, K}, e, M, N, K, splits, st, &xf);
  } else if (a_kmajor && b_kmajor)
    launch(KMajor{A, lda, M, K}, KMajor{B, ldb, N, K}, e, M, N, K, splits, st);
  else if (a_kmajor && !b_kmajor)
    launch(KMajor{A, lda, M, K}, MNMajorK{B, ldb, N, K}, e, M, N, K, splits, st);
  else if (!a_kmajor && b_kmajor)
    launch(MNMajorK{A, lda, M, K}, KMajor{B, ldb, N, K}, e, M, N, K, splits, st);
  else
    launch(MNMajorK{A, lda, M, K}, MNMajorK{B, ldb, N, K}, e, M, N, K, splits, st);
  if (slab) splitk_reduce(ws, splits, (long)M * N, reinterpret_cast<float*>(C), mode == 1, st);
}

// dx[M, N] = dy[M, K] . w[K, N] (bf16, the 1x1 data gradient) on the tile kernel with the BatchNorm-backward sums
// of dx for the relu(BN(x)) that produced the convolution's input (Epi::bb, BST instantiation).
void launch_gemm_dgrad_bnstats(const uint16_t* A, const uint16_t* B, uint16_t* C, int M, int N, int K,
                               const BnBwdSums& bb, hipStream_t st, bool accumulate, const uint16_t* add_src,
                               const uint8_t* add_mask) {
  // relu kind: x / gamma / beta / mean / invstd; mask kind (bb.mask): x / mean, and C may be accumulated onto
  if (bb.x2 && (!bb.mask || !bb.mean2 || !bb.sums2))
    throw std::runtime_error("gemm dgrad BatchNorm sums: the two-BatchNorm form is mask kind with mean2 / sums2");
  if (!bb.sums || !bb.x || !bb.mean || N % 8 || (!bb.mask && (!bb.gamma || !bb.beta || !bb.invstd || accumulate)))
    throw std::runtime_error("gemm dgrad BatchNorm-backward sums: x / mean / sums (+ gamma / beta / invstd without a "
                             "mask; accumulate only with one), N % 8 == 0");
  if ((add_src || add_mask) && !accumulate) throw std::runtime_error("gemm dgrad BatchNorm sums: an addend accumulates");
  Epi e = make_epi(C, N, false, nullptr, 0, nullptr, accumulate ? 1 : 0, 1.f);
  e.bb = bb;
  e.addsrc = add_src;  // out = product + (add_mask bit ? add_src : 0) (a ResNet identity block's residual gradient)
  e.addmask = add_mask;
  launch(KMajor{A, (long)K, M, K}, MNMajorK{B, (long)N, N, K}, e, M, N, K, 1, st);
}

// NHWC conv forward: y[N,Ho,Wo,K] = conv(x[N,H,W,C], w[K,R,S,C]); C % 64 == 0 takes the per-tile (r, s)
// decode, any other C % 8 == 0 the per-unit one.
void launch_conv_fwd(const uint16_t* x, const uint16_t* w, void* y, bool y_f32, int N, int H, int W, int C, int K,
                     int R, int S, int stride, int pad, int dil, int Ho, int Wo, const float* bias, int act,
                     int mode, float* stats, hipStream_t st, const SubGrid* sg,
                     const float* xform, const BnBwdSums* bb) {
  if (bb && bb->mask &&
      (!sg || mode != 1 || R != 1 || S != 1 || stride != 1 || pad != 0 || y_f32 || stats || xform || !bb->x ||
       !bb->mean || !bb->sums))
    throw std::runtime_error("conv: BatchNorm-sum corrections only on an accumulating 1x1 sub-grid data gradient");
  // relu kind: a sub-grid parity's plain store (a stride-2 data gradient) on the tile kernel, C % 64 == 0, K > 64
  if (bb && !bb->mask &&
      (!sg || mode != 0 || y_f32 || stats || xform || bias || act || C % 64 || K <= 64 || !bb->x || !bb->mean ||
       !bb->sums || !bb->gamma || !bb->beta || !bb->invstd))
    throw std::runtime_error("conv: BatchNorm + ReLU sums only on a stored sub-grid data gradient (C % 64, K > 64)");
  if (!bb && !sg && !y_f32 && !bias && act == 0 && mode == 0 && conv3x3_eligible(H, W, C, K, R, S, stride, pad, dil)) {
    launch_conv3x3(x, w, reinterpret_cast<uint16_t*>(y), stats, xform, N, H, W, C, K, st);  // staged window
    return;
  }
  const int M = N * Ho * Wo, RSC = R * S * C;
  KMajor b{w, (long)RSC, K, RSC};
  Epi e = make_epi(y, K, y_f32, bias, act, nullptr, mode, 1.f);
  e.stats = stats;
  if (bb) e.bb = *bb;
  if (sg) {
    if (stats) throw std::runtime_error("sub-grid output takes no statistics epilogue");
    e.rst = sg->stride;
    e.rHo = Ho;
    e.rWo = Wo;
    e.rH = sg->H;
    e.rW = sg->W;
    e.ra = sg->a;
    e.rb = sg->b;
  }
  if (xform && C % 64 != 0) throw std::runtime_error("normalize-on-load convolution needs C % 64 == 0");
  if (R == 1 && S == 1 && stride == 1 && pad == 0 && (!sg || (Ho == H && Wo == W)) && C % 64 == 0) {
    // a plain 1x1 convolution is the GEMM y[M][K] = x[M][C] . w[K][C]^T: the K-major source needs no im2col
    // decode (ConvA's per-row (n, ho, wo) cursors were ~1/4 of the VALU of these memory-bound kernels); short
    // reductions stream through gemm_short.hip. The live parity of a strided 1x1 data gradient (a sub-grid output,
    // scattered by the epilogue) takes the same source: 2-4 % faster per layer than ConvA (scripts/gpurun/r4/sgkm.sh)
    if (!sg && !y_f32 && !bias && act == 0 && mode == 0 && gemm_short_ok(M, K, C, C, K)) {
      launch_gemm_short(x, w, C, false, reinterpret_cast<uint16_t*>(y), nullptr, nullptr, xform, stats, M, K, C, 0,
                        st);
      return;
    }
    // deep reductions (C >= 512: ResNet stage-3/4 conv1 / conv3) with whole 256 x 256 tiles filling the chip: the
    // 4-wave kernel with the statistics epilogue (gemm256.hip copy_out_stats). Stream-K tails are not taken here
    // (no workspace): such grids stay on the tile kernel.
    if (!sg && !xform && !y_f32 && !bias && act == 0 && mode == 0 && stats && gemm_w4_stats_ok(M, K, C) &&
        gemm256_plan(M, K, C).sk == 1) {
      launch_gemm_w4_stats(x, C, w, C, reinterpret_cast<uint16_t*>(y), M, K, C, stats, nullptr, nullptr, st);
      return;
    }
    KMajor a{x, (long)C, M};
    if (xform) {
      const XForm xf{xform, C, make_fastdiv(C)};
      launch(a, b, e, M, K, RSC, 1, st, &xf);
    } else {
      launch(a, b, e, M, K, RSC, 1, st);
    }
  } else if (C % 64 == 0) {
    ConvA a{x, N, H, W, C, Ho, Wo, S, stride, pad, dil, M,
            make_fastdiv(C), make_fastdiv(S), make_fastdiv(Ho * Wo), make_fastdiv(Wo)};
    if (xform) {
      const XForm xf{xform, C, make_fastdiv(C)};
      launch(a, b, e, M, K, RSC, 1, st, &xf);
    } else {
      launch(a, b, e, M, K, RSC, 1, st);
    }
  } else {
    ConvAG a{x, N, H, W, C, Ho, Wo, S, stride, pad, dil, M, RSC,
             make_fastdiv(C), make_fastdiv(S), make_fastdiv(Ho * Wo), make_fastdiv(Wo)};
    launch(a, b, e, M, K, RSC, 1, st);
  }
}

// Weight gradient: dw[K][R*S*C] fp32 (+)= dY^T . im2col(x); split-K through fp32 slabs in `ws`
void launch_conv_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int N, int H, int W, int C, int K, int R,
                       int S, int stride, int pad, int dil, int Ho, int Wo, int splits, bool accumulate, float* ws,
                       hipStream_t st, const float* xform) {
  const int M = N * Ho * Wo;  // reduction dim
  MNMajorK a{dy, (long)K, K, M};
  ConvWgB b{x, N, H, W, C, Ho, Wo, S, stride, pad, dil, R * S * C, M,
            make_fastdiv(C), make_fastdiv(S), make_fastdiv(Ho * Wo), make_fastdiv(Wo)};
  splits = effective_splits(M, splits);
  const int RSC = R * S * C;
  const bool slab = splits > 1;
  Epi e = make_epi(slab ? (void*)ws : (void*)dw, (long)RSC, true, nullptr, 0, nullptr, slab ? 3 : (accumulate ? 1 : 0),
                   1.f);
  e.slab = (long)K * RSC;
  if (xform) {
    const XForm xf{xform, C, make_fastdiv(C)};
    launch(a, b, e, K, RSC, M, splits, st, &xf);
  } else {
    launch(a, b, e, K, RSC, M, splits, st);
  }
  if (slab) splitk_reduce(ws, splits, (long)K * RSC, dw, accumulate, st);
}

// dgrad weight transform: w2[c][r][s][k] = w[k][R-1-r][S-1-s][c]
__global__ void conv_dgrad_wtrans_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ w2, int K, int R,
                                         int S, int C) {
  const long total = (long)K * R * S * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    long t = i / K;
    const int s = (int)(t % S);
    t /= S;
    const int r = (int)(t % R);
    const int c = (int)(t / R);
    w2[i] = w[(((long)k * R + (R - 1 - r)) * S + (S - 1 - s)) * C + c];
  }
}

void launch_conv_dgrad_wtrans(const uint16_t* w, uint16_t* w2, int K, int R, int S, int C, hipStream_t st) {
  const long total = (long)K * R * S * C;
  hipLaunchKernelGGL(conv_dgrad_wtrans_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, st, w, w2, K, R, S, C);
}

// Stride-s data gradient, per-parity sub-weights in one launch: parity p (grid.y) gets
//   out[off_p + (c * T_p + t) * K + k] = w[k][rs_p[t]][c]          ([C][T_p][K], T_p = its taps, rs = r*S + s)
// replacing a stack / permute / contiguous chain of ATen copies per parity (ops/conv.py _dgrad_strided_hip).
__global__ void conv_dgrad_wsub_kernel(const uint16_t* __restrict__ w, uint16_t* __restrict__ out, int K, int RS,
                                       int C, DgradTaps taps) {
  const int p = blockIdx.y;
  const int T = taps.n[p];
  const long total = (long)C * T * K;
  uint16_t* o = out + taps.off[p];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int k = (int)(i % K);
    const long ct = i / K;
    const int t = (int)(ct % T);
    const int c = (int)(ct / T);
    o[i] = w[((long)k * RS + taps.rs[p][t]) * C + c];
  }
}

void launch_conv_dgrad_wsub(const uint16_t* w, uint16_t* out, int K, int RS, int C, const DgradTaps& taps, int np,
                            hipStream_t st) {
  int maxt = 1;
  for (int p = 0; p < np; ++p) maxt = taps.n[p] > maxt ? taps.n[p] : maxt;
  const long total = (long)C * maxt * K;
  hipLaunchKernelGGL(conv_dgrad_wsub_kernel, dim3(stream_grid(total, 256), np), dim3(256), 0, st, w, out, K, RS, C,
                     taps);
}

}  // namespace k8s_amd
