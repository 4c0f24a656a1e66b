// Host-side launcher declarations for every gfx950 kernel translation unit.
// The kernels themselves are compiled without any PyTorch headers (fast,
// parallel builds); only ops_binding.cpp sees torch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace k8s_amd {

// planner.hip: the CU count every launch planner sizes its grid for (see common.h)
int planner_cus();
void set_planner_cus(int n);

// optim.hip
void launch_sgd(float* p, float* mom, const void* g, bool g_bf16, uint16_t* pbf, long n, const uint8_t* decay_mask, float lr,
                float mu, float wd, float scale, const float* scale_ptr, const float* hyper, bool nesterov,
                bool first_step, hipStream_t st);
void launch_adam(float* p, float* m1, float* m2, const void* g, bool g_bf16, uint16_t* pbf, long n, const uint8_t* decay_mask,
                 float lr, float b1, float b2, float eps, float wd, float scale, const float* scale_ptr,
                 const float* hyper, float bc1, float bc2, bool decoupled, hipStream_t st);
void launch_sumsq(const void* g, bool g_bf16, long n, float* out, hipStream_t st);
void launch_clip_factor(const float* stats, float max_norm, float* factor, hipStream_t st);
void launch_slice_sum(const uint16_t* in, long n, int world, float* out, uint16_t* out_bf, hipStream_t st);
void launch_cast_bf16(const float* in, uint16_t* out, long n, hipStream_t st);

// batchnorm.hip
int bn_workspace_floats(long M, int C);
// params: fp32 workspace, [2][C] for the forward (scale, shift), [4][C] for the backward (sc, B, D, shift)
void launch_bn_fwd(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta, uint16_t* y,
                   float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* work, float* params,
                   long M, int C, float eps, float momentum, bool training, bool relu, hipStream_t st,
                   uint8_t* mask = nullptr);
void launch_bn_fwd_from_sums(const uint16_t* x, const uint16_t* res, const float* gamma, const float* beta,
                             uint16_t* y, const float* sums, int nrep, float* save_mean, float* save_invstd,
                             float* run_mean, float* run_var, float* params, long M, int C, float eps, float momentum,
                             bool relu, hipStream_t st, uint8_t* mask = nullptr, uint16_t* ysub = nullptr,
                             int H = 1, int W = 1);
void launch_bn_fwd_from_sums_dual(const uint16_t* x, const float* gamma, const float* beta, const float* sums,
                                  int nrep, float* save_mean, float* save_invstd, float* run_mean, float* run_var,
                                  float* params, const uint16_t* xr, const float* gamma_r, const float* beta_r,
                                  const float* sums_r, int nrep_r, float* save_mean_r, float* save_invstd_r,
                                  float* run_mean_r, float* run_var_r, float* params_r, uint16_t* y, uint8_t* mask,
                                  long M, int C, float eps, float momentum, hipStream_t st);
void launch_bn_bwd_from_sums(const uint16_t* dy, const uint16_t* x, const uint8_t* mask, const float* sums, int nrep,
                             const float* mean, const float* invstd, const float* gamma, const float* beta,
                             uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, float* params, long M, int C,
                             hipStream_t st);
void launch_bn_bwd_relu_from_sums(const uint16_t* dy, const uint16_t* x, const float* sums, int nrep,
                                  const float* mean, const float* invstd, const float* gamma, const float* beta,
                                  uint16_t* dx, float* dgamma, float* dbeta, float* params, long M, int C,
                                  hipStream_t st);
void launch_bn_bwd_dual_from_sums(const uint16_t* dy, const uint8_t* mask, const uint16_t* x, const float* sums,
                                  int nrep, const float* mean, const float* invstd, const float* gamma,
                                  const float* beta, uint16_t* dx, float* dgamma, float* dbeta, float* params,
                                  const uint16_t* x2, const float* sums2, const float* mean2, const float* invstd2,
                                  const float* gamma2, const float* beta2, uint16_t* dx2, float* dgamma2,
                                  float* dbeta2, float* params2, long M, int C, hipStream_t st);
void launch_bn_bwd_dual(const uint16_t* dy, const uint8_t* mask, const uint16_t* x, const float* mean,
                        const float* invstd, const float* gamma, const float* beta, uint16_t* dx, float* dgamma,
                        float* dbeta, float* work, float* params, const uint16_t* x2, const float* mean2,
                        const float* invstd2, const float* gamma2, const float* beta2, uint16_t* dx2, float* dgamma2,
                        float* dbeta2, float* work2, float* params2, long M, int C, hipStream_t st);
void launch_bn_finalize_sums(const float* gamma, const float* beta, const float* sums, int nrep, float* save_mean,
                             float* save_invstd, float* run_mean, float* run_var, float* params, long M, int C,
                             float eps, float momentum, hipStream_t st);
constexpr int kConvStatReplicas = 32;  // must match STAT_REPL in gemm.hip
void launch_bn_bwd(const uint16_t* dy, const uint16_t* x, const float* mean, const float* invstd, const float* gamma,
                   const float* beta, bool relu_x, uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta,
                   float* work, float* params, long M, int C, hipStream_t st, const uint8_t* mask = nullptr);
// packed ReLU bits of a bf16 tensor (bit j of byte e = y[8e + j] > 0), nvec = numel / 8
void launch_relu_mask(const uint16_t* y, uint8_t* mask, long nvec, hipStream_t st);

// norm.hip
void launch_norm_fwd(bool rms, const uint16_t* x, const uint16_t* res, uint16_t* xsum, const float* gamma,
                     const float* beta, uint16_t* y, float* mean, float* rstd, long R, int D, float eps,
                     hipStream_t st);
int norm_workspace_floats(long R, int D);
void launch_norm_bwd(bool rms, const uint16_t* dy, const uint16_t* x, const float* gamma, const float* mean,
                     const float* rstd, const uint16_t* dres, uint16_t* dx, float* dgamma, float* dbeta, float* work,
                     long R, int D, hipStream_t st, float* dsum = nullptr);

// xent.hip
void launch_xent_fwd(const void* logits, bool bf16, const int64_t* labels, long R, long V, long ld, float* loss,
                     float* lse, long ignore_index, float smoothing, hipStream_t st);
void launch_xent_bwd(const void* logits, bool bf16, const int64_t* labels, const float* lse, const float* dscale,
                     bool per_row, long R, long V, long ld, void* dlogits, long ignore_index, float smoothing,
                     hipStream_t st);

// gemm.hip
int gemm_choose_splits(int M, int N, int K);
// accumulate-mode addend read from src (same layout as C) instead of C, elements with a clear bit in the packed
// mask (bit j of byte e = element 8e + j; null = all set) taken as zero (see Epi::addsrc in gemm.hip)
struct AddEpi {
  const uint16_t* src;
  const uint8_t* mask;
};
// gemm_short.hip: the short-K streaming GEMM (K in {64, 128, 256}, N % 128 == 0; see its header)
bool gemm_short_ok(int M, int N, int K, long lda, long ldc);
bool gemm_short_bnstats_ok(int M, int N, int K, bool dual);
// The BatchNorm-backward statistics a masked-addend data gradient can take in its epilogue: for the stored result g'
// of the BatchNorm y = relu(BN(x) + ...) whose packed ReLU bits are `mask`, g = mask ? g' : 0 and
//   sums[r][0][c] += sum g,  sums[r][1][c] += sum g (x - mean)   (r = the block's replica of kConvStatReplicas)
// and for a second BatchNorm fed by the same masked gradient (x2: sums2[r][1][c] += sum g (x2 - mean2)).
// The BatchNorm-backward sums a data-gradient epilogue accumulates for the non-residual BatchNorm + ReLU
// z = relu(BN(x)) that produced the convolution's input: g = relu_on(x) ? dx : 0 (the forward's ReLU decision, from
// gamma / beta / mean / invstd), sums[r][0][c] += sum g, sums[r][1][c] += sum g (x - mean). sums == nullptr: off.
struct BnBwdSums {
  const uint16_t* x = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  float* sums = nullptr;
  // mask kind (a residual BatchNorm's packed ReLU bits instead of the affine ReLU decision): the row-remapped
  // accumulating data gradient's correction (gemm.hip BST sub-grid path); gamma / beta / invstd unused
  const uint8_t* mask = nullptr;
  // mask kind, the two-BatchNorm form (a ResNet downsample block's output: bn3 and the downsample BN share g):
  // sums2[.][1] += sum g (x2 - mean2) (identity-row path only)
  const uint16_t* x2 = nullptr;
  const float* mean2 = nullptr;
  float* sums2 = nullptr;
};
struct GemmShortBnStats {
  const uint16_t* x = nullptr;
  const uint8_t* mask = nullptr;
  const float* mean = nullptr;
  float* sums = nullptr;
  const uint16_t* x2 = nullptr;
  const float* mean2 = nullptr;
  float* sums2 = nullptr;
};
void launch_gemm_short(const uint16_t* A, const uint16_t* B, long ldb, bool b_mn, uint16_t* C, const uint16_t* add,
                       const uint8_t* mask, const float* xf, float* stats, int M, int N, int K, int epi,
                       hipStream_t st, const GemmShortBnStats* bst = nullptr);
void launch_gemm_dgrad_bnstats(const uint16_t* A, const uint16_t* B, uint16_t* C, int M, int N, int K,
                               const BnBwdSums& bb, hipStream_t st, bool accumulate = false,
                               const uint16_t* add_src = nullptr, const uint8_t* add_mask = nullptr);
void launch_gemm(const uint16_t* A, long lda, bool a_kmajor, const uint16_t* B, long ldb, bool b_kmajor, void* C,
                 long ldc, bool c_f32, int M, int N, int K, const float* bias, int act, uint16_t* pre, int mode,
                 float alpha, int splits, float* ws, hipStream_t st, const AddEpi* add = nullptr,
                 const float* xform_b = nullptr, int xform_c = 0);
// out = bit ? src : 0 per element (bf16, n % 8 == 0; mask packed as above)
void launch_mask_apply(const uint16_t* src, const uint8_t* mask, uint16_t* out, long n, hipStream_t st);
long gemm_splitk_workspace(int M, int N, int splits);  // fp32 elements of the split-K slab workspace
// conv3x3.hip: staged-window 3 x 3 / stride-1 / pad-1 NHWC convolution (optional BN + ReLU on load: xform =
// fp32 [2][C] scale | shift), bf16 output, optional BN statistics [kConvStatReplicas][2][K]
bool conv3x3_eligible(int H, int W, int C, int K, int R, int S, int stride, int pad, int dil);
void launch_conv3x3(const uint16_t* x, const uint16_t* w, uint16_t* y, float* stats, const float* xform, int N,
                    int H, int W, int C, int K, hipStream_t st,
                    const BnBwdSums* bsums = nullptr);
// gemm256.hip: 256 x 256-tile, 8-wave phased MFMA GEMM for the large (transformer) products
bool gemm256_eligible(int M, int N, int K, bool a_kmajor, bool b_kmajor);
// split count for the tall-K fp32 products on the 256 x 256 kernel (1 = none)
int gemm256_choose_splits(int M, int N, int K);
// gemm256.hip: data gradient fused with the backward of the activation that produced the GEMM's input (4-wave kernel)
bool gemm_w4_dact_ok(int M, int N, int K, long lda, long ldb, long ldc);
long gemm_w4_dact_part_floats(int M, int N);
void launch_gemm_w4_dact(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* C, long ldc, int M, int N,
                         int K, const uint16_t* pre, int act, float* part, float* db, bool db_accumulate,
                         float* sk_slabs, int* sk_sync, hipStream_t st);
// the down-projection data gradient fused with the SwiGLU backward: dgu [M][2F] (gemm256.hip copy_out_x ACT = -3)
bool gemm_w4_swiglu_ok(int M, int F, int K, long lda, long ldb);
void launch_gemm_w4_swiglu_bwd(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* dgu,
                               const uint16_t* gu, int M, int F, int K, int blk, float* sk_slabs, int* sk_sync,
                               hipStream_t st);
bool gemm_w4_stats_ok(int M, int N, int K);
bool gemm_w4_dgrad_bnstats_ok(int M, int N, int K);
void launch_gemm_w4_dgrad_bnstats(const uint16_t* A, const uint16_t* B, uint16_t* y, int M, int N, int K,
                                  const uint16_t* x, const float* tab, float* sums, float* sk_slabs, int* sk_sync,
                                  hipStream_t st);
void launch_gemm_w4_stats(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* y, int M, int N, int K,
                          float* stats, float* sk_slabs, int* sk_sync, hipStream_t st);
bool gemm_w4_rope_ok(int M, int N, int K, long lda, long ldb, int rot_cols);
void launch_gemm_w4_rope(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* y, int M, int N, int K,
                         const int* pos, const float* table, int rot_cols, float* sk_slabs, int* sk_sync,
                         hipStream_t st);
bool gemm_w4_swiglu_fwd_ok(int M, int F, int K, long lda, long ldb);
void launch_gemm_w4_swiglu_fwd(const uint16_t* A, long lda, const uint16_t* B, long ldb, uint16_t* gu, uint16_t* h,
                               int M, int F, int K, float* sk_slabs, int* sk_sync, hipStream_t st);
// stream-K tail plan (gemm256.hip): tiles [full, tiles) are split sk ways along K (sk == 1: none), kps deep each
struct Gemm256Plan {
  int tiles, full, sk, kps;
};
Gemm256Plan gemm256_plan(int M, int N, int K);
long gemm256_sk_slab_floats(const Gemm256Plan& p);  // fp32 partial slabs the stream-K tail needs
long gemm256_sk_sync_ints(const Gemm256Plan& p);    // zeroed ints (ticket + flags) it needs; left zeroed after
void launch_gemm256(const uint16_t* A, long lda, bool a_kmajor, const uint16_t* B, long ldb, bool b_kmajor, void* C,
                    long ldc, bool c_f32, int M, int N, int K, const float* bias, int act, uint16_t* pre,
                    bool accumulate, float alpha, hipStream_t st, int splits = 1, float* ws = nullptr,
                    float* sk_slabs = nullptr, int* sk_sync = nullptr);
// Output written to the (a, b) parity sub-grid of an H x W image: GEMM row (n, i, j) -> (n, i*stride+a,
// j*stride+b). Used for stride-s data gradients decomposed by output parity (ops/conv.py _dgrad_strided_hip).
struct SubGrid {
  int H, W, stride, a, b;
};
void launch_conv_fwd(const uint16_t* x, const uint16_t* w, void* y, bool y_f32, int N, int H, int W, int C, int K,
                     int R, int S, int stride, int pad, int dil, int Ho, int Wo, const float* bias, int act,
                     int mode, float* stats, hipStream_t st, const SubGrid* sg = nullptr, const float* xform = nullptr,
                     const BnBwdSums* bb = nullptr);
// xform (here and in launch_gemm / launch_wgrad_stream): fp32 [2][C] BatchNorm (scale | shift): the activation
// operand x is consumed as relu(x * scale + shift), normalised as it is loaded (gemm.hip XForm)
void launch_conv_wgrad(const uint16_t* x, const uint16_t* dy, float* dw, int N, int H, int W, int C, int K, int R,
                       int S, int stride, int pad, int dil, int Ho, int Wo, int splits, bool accumulate, float* ws,
                       hipStream_t st, const float* xform = nullptr);
// wgrad_stream.hip: tall-K weight gradient (few output tiles, millions of rows), fp32 atomics into dw
bool wgrad_stream_eligible(int N, int Ho, int Wo, int C, int K, int R, int S);
void launch_wgrad_stream(const uint16_t* x, const uint16_t* dy, float* dw, int N, int H, int W, int C, int K, int R,
                         int S, int stride, int pad, int Ho, int Wo, bool accumulate, hipStream_t st);
void launch_conv_dgrad_wtrans(const uint16_t* w, uint16_t* w2, int K, int R, int S, int C, hipStream_t st);
// per-output-parity sub-weights of a stride-s dgrad (up to 16 parities x 16 taps), packed at off[p]
struct DgradTaps {
  int n[16];
  long off[16];
  int rs[16][16];
};
void launch_conv_dgrad_wsub(const uint16_t* w, uint16_t* out, int K, int RS, int C, const DgradTaps& taps, int np,
                            hipStream_t st);

// elementwise.hip
void launch_swiglu_fwd(const uint16_t* gu, uint16_t* y, long T, int F, int blk, hipStream_t st);
void launch_swiglu_bwd(const uint16_t* gu, const uint16_t* dy, uint16_t* dgu, long T, int F, int blk, hipStream_t st);
void launch_rope(uint16_t* x, long ld, const int* pos, const float* table, long T, int H, int D, bool inverse,
                 hipStream_t st);
void launch_gelu_bwd(const uint16_t* dy, const uint16_t* pre, uint16_t* dx, long n, hipStream_t st);
void launch_relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, hipStream_t st);
int colsum_workspace_floats(long R, int C);
void launch_colsum(const uint16_t* x, long R, int C, float* work, float* out, bool accumulate, hipStream_t st);
// the fold of P partial rows of column sums (colsum_fold_kernel)
// (P > 256: two levels, overwriting part)
void launch_colsum_fold(float* part, int P, int C, float* out, bool accumulate, hipStream_t st);
// the first level of that fold alone: the sum of rows [g gs, (g + 1) gs) written over row g gs
void launch_colsum_group(float* part, int P, int C, int gs, hipStream_t st);
// g = dy * act'(pre) (1 ReLU, pre = its output; 2 GELU(tanh), pre = the pre-activation) and out = column sums of g
void launch_act_bwd_colsum(int act, const uint16_t* dy, const uint16_t* pre, uint16_t* g, long R, int C, float* work,
                           float* out, bool accumulate, hipStream_t st);

// ---- K5 flash attention (attention.hip). q [B,Sq,Hq,D], k/v [B,Sk,Hkv,D] (strided, last dim contiguous)
struct AttnFwdArgs {
  const uint16_t *q, *k, *v;
  uint16_t* o;
  float* lse;          // [B, Hq, lse_ld]: m + log2(l) in the exp2 domain (scores scaled by scale*log2(e))
  const int* kv_lens;  // [B] or null
  long sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sob, sos, soh;
  long lse_ld;         // row stride of lse (Sq rounded up to 64)
  int B, Sq, Sk, Hq, Hkv, causal;
  float scale_log2;
};
struct AttnBwdArgs {
  const uint16_t *q, *k, *v, *dO;
  const float* lse;
  float* delta;       // [B, Hq, lse_ld] scratch
  uint16_t* dq;       // [B, Sq, Hq, D] at strides (sgqb, sgqs, sgqh)
  uint16_t *dk, *dv;  // [B, Sk, Hkv, D] at strides (sgkb, sgks, sgkh) / (sgvb, sgvs, sgvh)
  const int* kv_lens;
  long sqb, sqs, sqh, skb, sks, skh, svb, svs, svh, sdb, sds, sdh;
  // output strides: a packed [B*S, (Hq + 2*Hkv) * D] gradient of a fused QKV projection is written in place
  long sgqb, sgqs, sgqh, sgkb, sgks, sgkh, sgvb, sgvs, sgvh;
  long lse_ld;
  int B, Sq, Sk, Hq, Hkv, causal;
  float scale_log2, scale;
  // dK/dV split into dkv_split chunks per key block (flash_dkv_splits): fp32 partials [dkv_split][2][B][Hkv][Sk][D]
  int dkv_split = 1;
  float* dkv_ws = nullptr;
  // one-block short-sequence form only (flash_bwd_one_block): per-batch column sums of the packed QKV gradient,
  // fp32 [B][cpart_ld] (the projection's bias gradient once folded over B)
  float* cpart = nullptr;
  int cpart_ld = 0;
};
int flash_dkv_splits(int B, int Sq, int Sk, int Hkv, int causal);
// the whole backward of one (batch, head) in one block (flash_bwd_short_kernel) applies to this shape
bool flash_bwd_one_block(int D, int Sq, int Sk, int Hq, int Hkv, int dkv_split);
// ResNet stem BatchNorm + ReLU + 3x3 / s2 / p1 max pool, fused (batchnorm.hip): forward from the conv's epilogue sums
// (params = fp32 [2][C] scale | shift, idx = winner byte per pooled element); backward into dx of the conv output
// (params = fp32 [4][C] workspace, work = pool_bn_workspace_floats(C))
void launch_bn_relu_maxpool_fwd(const uint16_t* x, const float* gamma, const float* beta, const float* sums, int nrep,
                                float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* params,
                                uint16_t* y, uint8_t* idx, int N, int H, int W, int C, float eps, float momentum,
                                hipStream_t st, uint16_t* xarg = nullptr, uint8_t* ybits = nullptr);
void launch_pool_bn_bwd_from_sums(const uint16_t* dpool, const uint8_t* idx, const uint16_t* x, const float* mean,
                                  const float* invstd, const float* gamma, const float* beta, uint16_t* dx,
                                  float* dgamma, float* dbeta, const float* sums, int nrep, float* params, int N,
                                  int H, int W, int C, hipStream_t st);
int pool_bn_workspace_floats(int C);
void launch_pool_bn_bwd(const uint16_t* dpool, const uint8_t* idx, const uint16_t* x, const float* mean,
                        const float* invstd, const float* gamma, const float* beta, uint16_t* dx, float* dgamma,
                        float* dbeta, float* work, float* params, int N, int H, int W, int C, hipStream_t st);

// Streaming-order state (batchnorm.hip): direction (0 ascending, 1 descending, as 8 concurrent bands) of the next
// streaming launch; `fixed` is the direction used in the fixed-BatchNorm mode.
int stream_order_mode();
int stream_dir(int fixed);

void launch_flash_fwd(const AttnFwdArgs& a, int D, hipStream_t st);
void launch_flash_bwd(const AttnBwdArgs& a, int D, const uint16_t* o, long sob, long sos, long soh, hipStream_t st);

// ---- embedding.hip: sum of up to 3 table gathers (fwd) / fp32 atomic scatter-add into gradient slots (bwd)
struct EmbTable {
  const uint16_t* w;   // [V][D] bf16 table (forward)
  float* g;            // [V][D] fp32 gradient (backward; accumulated into)
  const int64_t* ids;  // [T] row ids, or null: row = token % S (position table)
  int V;
};
void launch_embed_fwd(const EmbTable* tabs, int ntab, int T, int D, int S, uint16_t* out, hipStream_t st);
void launch_embed_bwd(const EmbTable* tabs, int ntab, int T, int D, int S, const uint16_t* g, hipStream_t st);

// ---- NHWC average pooling over H*W (pool.hip): y[n][c] = mean_hw x[n][hw][c] (fp32 accumulate, bf16 out)
void launch_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t st);
void launch_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t st);

// ---- stem.hip: 7x7 / stride-2 stem as a 4x4 conv over the 2x2 space-to-depth image (16 channels)
void launch_stem_s2d_input(const uint16_t* x, int N, int H, int W, int Cin, int pad, uint16_t* out, hipStream_t st);
void launch_stem_w_s2d(const uint16_t* w7, int K, int R, int Cw, uint16_t* w4, hipStream_t st);
// the s2d stem conv (K = 64, 4x4 taps, 16 channels) LDS-tiled, BN statistics into stats [kConvStatReplicas][2][64]
bool stem_conv_fwd_ok(int K, int R, int C, int Wo);
void launch_stem_conv_fwd(const uint16_t* xs, const uint16_t* w4, uint16_t* y, float* stats, int N, int Hs, int Ws,
                          hipStream_t st);
// out[i] (+)= sum over `splits` fp32 slabs of mn elements (gemm.hip)
void splitk_reduce(const float* ws, int splits, long mn, float* out, bool accumulate, hipStream_t st);
// LDS-tiled 3x3 / s1 / p1 weight gradient (wgrad_tile.hip), C == K in 64 pieces; ws = wgrad3x3_tiled_workspace floats
bool wgrad3x3_tiled_ok(int C, int K, int R, int S, int stride, int pad, int W);
int wgrad3x3_tiled_blocks(int N, int H, int W, int C);
long wgrad3x3_tiled_workspace(int N, int H, int W, int C);
void launch_wgrad3x3_tiled(const uint16_t* x, const uint16_t* dy, float* ws, float* dw, int N, int H, int W, int C,
                           bool accumulate, hipStream_t st, const float* xform = nullptr);
// the s2d stem weight gradient (LDS-tiled, persistent blocks; ws = stem_wgrad_blocks(N, Hs) x 64 x 256 fp32 partials)
int stem_wgrad_blocks(int N, int Hs);
void launch_stem_wgrad(const uint16_t* xs, const uint16_t* dy, float* ws, float* dw4, int N, int Hs, int Ws,
                       hipStream_t st);
void launch_stem_dw_s2d(const float* dw4, int K, int R, int Cw, float* dw7, hipStream_t st);

// ---- NHWC max pooling (pool.hip): idx = winning window position per output element (uint8)
void launch_subsample_nhwc(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int s, hipStream_t st);
void launch_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo,
                        int k, int s, int p, hipStream_t st);
void launch_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int Ho,
                        int Wo, int k, int s, int p, hipStream_t st);

}  // namespace k8s_amd
