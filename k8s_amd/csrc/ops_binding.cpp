// Python bindings of the k8s_amd gfx950 kernels (module k8s_amd._C).
//
// Every entry point validates device, dtype, contiguity and shape on the host
// before launching, so a mis-shaped call raises a Python exception instead of
// faulting the GPU. Kernels are launched on PyTorch's current HIP stream so
// they compose with torch ops, streams and hipGraph capture.
#include <cstdlib>

#include <torch/extension.h>

#include <map>
#include <mutex>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "kernels/launchers.h"

namespace {

using at::Tensor;

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_dtype(const Tensor& t, at::ScalarType d, const char* name) {
  TORCH_CHECK(t.scalar_type() == d, name, " has dtype ", t.scalar_type(), ", expected ", d);
}
void check_aligned(const Tensor& t, const char* name) {
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
}
uint16_t* bf(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }
const uint16_t* cbf(const Tensor& t) { return reinterpret_cast<const uint16_t*>(t.data_ptr()); }
float* f32(const Tensor& t) { return t.data_ptr<float>(); }
const float* optf(const c10::optional<Tensor>& t) { return t.has_value() ? t->data_ptr<float>() : nullptr; }

// ------------------------------------------------------------------ optimizers
const uint8_t* mask_ptr(const c10::optional<Tensor>& m, long n) {
  if (!m) return nullptr;
  TORCH_CHECK(m->is_cuda() && m->scalar_type() == at::kByte && m->is_contiguous(), "decay_mask must be uint8 GPU");
  TORCH_CHECK(m->numel() * 64 >= n, "decay_mask must have one byte per 64 elements");
  return m->data_ptr<uint8_t>();
}

// device fp32 [lr, step] read by the optimizer kernels instead of the host scalars (hipGraph replay)
static const float* hyper_ptr(const c10::optional<Tensor>& h) {
  if (!h) return nullptr;
  check_cuda(*h, "hyper");
  check_dtype(*h, at::kFloat, "hyper");
  TORCH_CHECK(h->numel() >= 2 && h->is_contiguous(), "hyper must be a contiguous fp32 [lr, step] tensor");
  return h->data_ptr<float>();
}

void fused_sgd(Tensor p, Tensor mom, Tensor g, c10::optional<Tensor> pbf, c10::optional<Tensor> decay_mask, double lr, double mu,
               double wd, double scale, c10::optional<Tensor> scale_t, bool nesterov, bool first_step,
               c10::optional<Tensor> hyper) {
  check_cuda(p, "param"); check_cuda(mom, "momentum"); check_cuda(g, "grad");
  check_dtype(p, at::kFloat, "param"); check_dtype(mom, at::kFloat, "momentum");
  const long n = p.numel();
  TORCH_CHECK(n % 4 == 0, "flat buffer length must be a multiple of 4");
  TORCH_CHECK(mom.numel() == n && g.numel() == n, "size mismatch");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "grad must be fp32 or bf16");
  if (pbf) { check_cuda(*pbf, "param_bf16"); check_dtype(*pbf, at::kBFloat16, "param_bf16"); TORCH_CHECK(pbf->numel() == n); }
  const uint8_t* dm = mask_ptr(decay_mask, n);
  k8s_amd::launch_sgd(f32(p), f32(mom), g.data_ptr(), g.scalar_type() == at::kBFloat16, pbf ? bf(*pbf) : nullptr, n,
                      dm, (float)lr, (float)mu, (float)wd, (float)scale, optf(scale_t), hyper_ptr(hyper), nesterov,
                      first_step, cur_stream());
}

void fused_adam(Tensor p, Tensor m1, Tensor m2, Tensor g, c10::optional<Tensor> pbf, c10::optional<Tensor> decay_mask, double lr,
                double b1, double b2, double eps, double wd, double scale, c10::optional<Tensor> scale_t, int64_t step,
                bool decoupled, c10::optional<Tensor> hyper) {
  check_cuda(p, "param"); check_cuda(m1, "exp_avg"); check_cuda(m2, "exp_avg_sq"); check_cuda(g, "grad");
  const long n = p.numel();
  TORCH_CHECK(n % 4 == 0, "flat buffer length must be a multiple of 4");
  TORCH_CHECK(m1.numel() == n && m2.numel() == n && g.numel() == n, "size mismatch");
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "grad must be fp32 or bf16");
  if (pbf) { check_cuda(*pbf, "param_bf16"); check_dtype(*pbf, at::kBFloat16, "param_bf16"); TORCH_CHECK(pbf->numel() == n); }
  const float bc1 = 1.f - std::pow((float)b1, (float)step);
  const float bc2 = 1.f - std::pow((float)b2, (float)step);
  k8s_amd::launch_adam(f32(p), f32(m1), f32(m2), g.data_ptr(), g.scalar_type() == at::kBFloat16,
                       pbf ? bf(*pbf) : nullptr, n, mask_ptr(decay_mask, n), (float)lr, (float)b1, (float)b2, (float)eps, (float)wd,
                       (float)scale, optf(scale_t), hyper_ptr(hyper), bc1, bc2, decoupled, cur_stream());
}

Tensor grad_sumsq(Tensor g) {
  check_cuda(g, "grad");
  TORCH_CHECK(g.numel() % 4 == 0);
  auto out = torch::zeros({2}, g.options().dtype(at::kFloat));
  k8s_amd::launch_sumsq(g.data_ptr(), g.scalar_type() == at::kBFloat16, g.numel(), f32(out), cur_stream());
  return out;
}

Tensor clip_factor(Tensor stats, double max_norm) {
  auto f = torch::empty({1}, stats.options());
  k8s_amd::launch_clip_factor(f32(stats), (float)max_norm, f32(f), cur_stream());
  return f;
}

// ------------------------------------------------------------------ bf16 gradient transport
// recv: bf16 [world * n] (all-to-all receive buffer of one bucket) -> fp32 out [n] and/or bf16 out_bf [n]
void slice_sum(Tensor recv, int64_t world, c10::optional<Tensor> out, c10::optional<Tensor> out_bf) {
  check_cuda(recv, "recv"); check_dtype(recv, at::kBFloat16, "recv");
  TORCH_CHECK(recv.is_contiguous() && world > 0 && recv.numel() % world == 0, "recv must be [world * n]");
  const long n = recv.numel() / world;
  float* o = nullptr;
  uint16_t* ob = nullptr;
  if (out && out->defined()) {
    check_dtype(*out, at::kFloat, "out");
    TORCH_CHECK(out->is_contiguous() && out->numel() == n, "out must be [n] fp32");
    o = f32(*out);
  }
  if (out_bf && out_bf->defined()) {
    check_dtype(*out_bf, at::kBFloat16, "out_bf");
    TORCH_CHECK(out_bf->is_contiguous() && out_bf->numel() == n, "out_bf must be [n] bf16");
    ob = reinterpret_cast<uint16_t*>(out_bf->data_ptr());
  }
  TORCH_CHECK(o || ob, "slice_sum: no output");
  k8s_amd::launch_slice_sum(reinterpret_cast<const uint16_t*>(recv.data_ptr()), n, (int)world, o, ob, cur_stream());
}

Tensor cast_bf16(Tensor x, c10::optional<Tensor> out) {
  check_cuda(x, "x"); check_dtype(x, at::kFloat, "x");
  TORCH_CHECK(x.is_contiguous(), "x must be contiguous");
  Tensor o = (out && out->defined()) ? *out : torch::empty({x.numel()}, x.options().dtype(at::kBFloat16));
  check_dtype(o, at::kBFloat16, "out");
  TORCH_CHECK(o.is_contiguous() && o.numel() == x.numel(), "out size mismatch");
  k8s_amd::launch_cast_bf16(f32(x), reinterpret_cast<uint16_t*>(o.data_ptr()), x.numel(), cur_stream());
  return o;
}

// ------------------------------------------------------------------ batchnorm (NHWC)
// want_mask: also return the packed ReLU mask (uint8 [M*C/8], bit j of byte e = y[8e+j] > 0) for the backward
static Tensor relu_mask_for(const Tensor& x, bool want_mask) {
  return want_mask ? torch::empty({x.numel() / 8}, x.options().dtype(at::kByte)) : Tensor();
}

static const uint8_t* cmask(const c10::optional<Tensor>& m) {
  if (!m || !m->defined()) return nullptr;
  TORCH_CHECK(m->is_cuda() && m->scalar_type() == at::kByte && m->is_contiguous(), "mask must be contiguous uint8");
  return m->data_ptr<uint8_t>();
}

std::vector<Tensor> bn_fwd(Tensor x, c10::optional<Tensor> res, Tensor gamma, Tensor beta, Tensor run_mean,
                           Tensor run_var, bool training, double momentum, double eps, bool relu, bool want_mask) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x"); check_aligned(x, "x");
  const int C = (int)x.size(-1);
  TORCH_CHECK(C % 8 == 0, "channels must be a multiple of 8");
  const long M = x.numel() / C;
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  check_dtype(gamma, at::kFloat, "gamma");
  if (res) { check_cuda(*res, "res"); TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch"); }
  auto y = torch::empty_like(x);
  auto mean = torch::empty({C}, gamma.options());
  auto invstd = torch::empty({C}, gamma.options());
  auto params = torch::empty({2 * C}, gamma.options());
  Tensor work = training ? torch::empty({k8s_amd::bn_workspace_floats(M, C)}, gamma.options()) : mean;
  Tensor mask = relu_mask_for(x, want_mask);
  k8s_amd::launch_bn_fwd(cbf(x), res ? cbf(*res) : nullptr, f32(gamma), f32(beta), bf(y), f32(mean), f32(invstd),
                         f32(run_mean), f32(run_var), f32(work), f32(params), M, C, (float)eps, (float)momentum,
                         training, relu, cur_stream(), want_mask ? mask.data_ptr<uint8_t>() : nullptr);
  if (want_mask) return {y, mean, invstd, mask};
  return {y, mean, invstd};
}

std::vector<Tensor> bn_fwd_from_sums(Tensor x, c10::optional<Tensor> res, Tensor gamma, Tensor beta, Tensor sums,
                                     Tensor run_mean, Tensor run_var, double momentum, double eps, bool relu,
                                     bool want_mask, bool want_sub2) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x"); check_aligned(x, "x");
  const int C = (int)x.size(-1);
  TORCH_CHECK(C % 8 == 0, "channels must be a multiple of 8");
  const long M = x.numel() / C;
  TORCH_CHECK(sums.numel() % (2 * C) == 0 && sums.scalar_type() == at::kFloat, "sums must be fp32 [R, 2, C]");
  const int nrep = (int)(sums.numel() / (2 * C));
  if (res) { check_cuda(*res, "res"); TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch"); }
  auto y = torch::empty_like(x);
  auto mean = torch::empty({C}, gamma.options());
  auto invstd = torch::empty({C}, gamma.options());
  auto params = torch::empty({2 * C}, gamma.options());
  Tensor mask = relu_mask_for(x, want_mask);
  // want_sub2: also y[:, ::2, ::2, :] (the next block's downsample input), written by the same pass
  Tensor ysub;
  int H = 1, W = 1;
  if (want_sub2) {
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "want_sub2: contiguous NHWC x");
    H = (int)x.size(1);
    W = (int)x.size(2);
    ysub = torch::empty({x.size(0), (H + 1) / 2, (W + 1) / 2, C}, x.options());
  }
  k8s_amd::launch_bn_fwd_from_sums(cbf(x), res ? cbf(*res) : nullptr, f32(gamma), f32(beta), bf(y), f32(sums),
                                   nrep, f32(mean), f32(invstd), f32(run_mean), f32(run_var), f32(params), M, C,
                                   (float)eps, (float)momentum, relu, cur_stream(),
                                   want_mask ? mask.data_ptr<uint8_t>() : nullptr, want_sub2 ? bf(ysub) : nullptr, H,
                                   W);
  std::vector<Tensor> out = {y, mean, invstd};
  if (want_mask) out.push_back(mask);
  if (want_sub2) out.push_back(ysub);
  return out;
}

// y = relu(BN(x) + BN_r(xr)) with both BatchNorms' statistics from conv epilogue sums (ResNet downsample block:
// bn3 + the downsample BN in one apply pass). Returns (y, mean, invstd, packed ReLU mask, mean_r, invstd_r).
std::vector<Tensor> bn_fwd_from_sums_dual(Tensor x, Tensor sums, Tensor gamma, Tensor beta, Tensor run_mean,
                                          Tensor run_var, Tensor xr, Tensor sums_r, Tensor gamma_r, Tensor beta_r,
                                          Tensor run_mean_r, Tensor run_var_r, double momentum, double eps) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x"); check_aligned(x, "x");
  check_cuda(xr, "xr"); check_dtype(xr, at::kBFloat16, "xr"); check_aligned(xr, "xr");
  TORCH_CHECK(x.is_contiguous() && xr.is_contiguous() && xr.sizes() == x.sizes(), "x / xr: same contiguous shape");
  const int C = (int)x.size(-1);
  TORCH_CHECK(C % 8 == 0, "channels must be a multiple of 8");
  const long M = x.numel() / C;
  for (const Tensor* t : {&gamma, &beta, &run_mean, &run_var, &gamma_r, &beta_r, &run_mean_r, &run_var_r})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_cuda(), "per-channel fp32 vectors of C");
  for (const Tensor* t : {&sums, &sums_r})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() % (2 * C) == 0,
                "sums must be fp32 [R, 2, C]");
  auto y = torch::empty_like(x);
  auto mean = torch::empty({C}, gamma.options()), invstd = torch::empty({C}, gamma.options());
  auto mean_r = torch::empty({C}, gamma.options()), invstd_r = torch::empty({C}, gamma.options());
  auto params = torch::empty({2 * C}, gamma.options()), params_r = torch::empty({2 * C}, gamma.options());
  Tensor mask = relu_mask_for(x, true);
  k8s_amd::launch_bn_fwd_from_sums_dual(
      cbf(x), f32(gamma), f32(beta), f32(sums), (int)(sums.numel() / (2 * C)), f32(mean), f32(invstd), f32(run_mean),
      f32(run_var), f32(params), cbf(xr), f32(gamma_r), f32(beta_r), f32(sums_r), (int)(sums_r.numel() / (2 * C)),
      f32(mean_r), f32(invstd_r), f32(run_mean_r), f32(run_var_r), f32(params_r), bf(y), mask.data_ptr<uint8_t>(), M,
      C, (float)eps, (float)momentum, cur_stream());
  return {y, mean, invstd, mask, mean_r, invstd_r};
}

// BatchNorm statistics of a conv output from its epilogue sums, WITHOUT the apply pass: returns (mean, invstd,
// params = fp32 [2][C] scale | shift) for a consumer that normalises on load (conv_fwd / conv_wgrad / gemm xform).
std::vector<Tensor> bn_finalize(Tensor sums, Tensor gamma, Tensor beta, Tensor run_mean, Tensor run_var,
                                int64_t count, double momentum, double eps) {
  const int C = (int)gamma.numel();
  check_dtype(gamma, at::kFloat, "gamma");
  TORCH_CHECK(sums.is_cuda() && sums.numel() % (2 * C) == 0 && sums.scalar_type() == at::kFloat &&
                  sums.is_contiguous(), "sums must be fp32 [R, 2, C]");
  TORCH_CHECK(beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  const int nrep = (int)(sums.numel() / (2 * C));
  auto mean = torch::empty({C}, gamma.options());
  auto invstd = torch::empty({C}, gamma.options());
  auto params = torch::empty({2 * C}, gamma.options());
  k8s_amd::launch_bn_finalize_sums(f32(gamma), f32(beta), f32(sums), nrep, f32(mean), f32(invstd), f32(run_mean),
                                   f32(run_var), f32(params), (long)count, C, (float)eps, (float)momentum,
                                   cur_stream());
  return {mean, invstd, params};
}

// ResNet stem: BatchNorm (statistics from the conv epilogue sums) + ReLU + 3x3 / s2 / p1 max pool in one pass; the
// BN output is never stored. Returns (pooled y, winner idx, mean, invstd); with `want_link` also (xarg, ybits): the
// winner's x and packed ReLU bits per pooled element (the BatchNorm-backward sums in the consumers' dgrad epilogues).
std::vector<Tensor> bn_relu_maxpool(Tensor x, Tensor sums, Tensor gamma, Tensor beta, Tensor run_mean, Tensor run_var,
                                    double momentum, double eps, bool want_link) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "x must be a contiguous NHWC tensor");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "C / 8 must divide 256");
  check_dtype(gamma, at::kFloat, "gamma");
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() && sums.numel() % (2 * C) == 0,
              "sums must be fp32 [R, 2, C]");
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  auto y = torch::empty({N, Ho, Wo, C}, x.options());
  auto idx = torch::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  auto mean = torch::empty({C}, gamma.options());
  auto invstd = torch::empty({C}, gamma.options());
  auto params = torch::empty({2 * C}, gamma.options());
  Tensor xarg, ybits;
  if (want_link) {
    xarg = torch::empty({N, Ho, Wo, C}, x.options());
    ybits = torch::empty({(long)N * Ho * Wo * C / 8}, x.options().dtype(at::kByte));
  }
  k8s_amd::launch_bn_relu_maxpool_fwd(cbf(x), f32(gamma), f32(beta), f32(sums), (int)(sums.numel() / (2 * C)),
                                      f32(mean), f32(invstd), f32(run_mean), f32(run_var), f32(params), bf(y),
                                      idx.data_ptr<uint8_t>(), N, H, W, C, (float)eps, (float)momentum, cur_stream(),
                                      want_link ? bf(xarg) : nullptr,
                                      want_link ? ybits.data_ptr<uint8_t>() : nullptr);
  if (want_link) return {y, idx, mean, invstd, xarg, ybits};
  return {y, idx, mean, invstd};
}

// pool_bn_bwd with the BatchNorm-backward sums already taken (fp32 [conv_stat_replicas, 2, C] over g = bit ? dpool :
// 0 at the winners' x, by the data gradients into the pooled output): the final and apply passes only.
Tensor pool_bn_bwd_from_sums(Tensor dpool, Tensor idx, Tensor x, Tensor mean, Tensor invstd, Tensor gamma,
                             Tensor beta, Tensor dgamma, Tensor dbeta, Tensor sums) {
  check_cuda(dpool, "dpool"); check_dtype(dpool, at::kBFloat16, "dpool");
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  check_dtype(idx, at::kByte, "idx");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && dpool.is_contiguous() && idx.is_contiguous());
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(dpool.sizes() == idx.sizes() && dpool.size(0) == N && dpool.size(1) == (H + 1) / 2 &&
                  dpool.size(2) == (W + 1) / 2 && dpool.size(3) == C, "dpool / idx shape mismatch");
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.is_contiguous() && dbeta.is_contiguous());
  check_dtype(dgamma, at::kFloat, "dgamma"); check_dtype(dbeta, at::kFloat, "dbeta");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() &&
                  sums.numel() == (long)k8s_amd::kConvStatReplicas * 2 * C, "sums: fp32 [conv_stat_replicas, 2, C]");
  auto dx = torch::empty_like(x);
  auto params = torch::empty({4 * C}, gamma.options());
  k8s_amd::launch_pool_bn_bwd_from_sums(cbf(dpool), idx.data_ptr<uint8_t>(), cbf(x), f32(mean), f32(invstd),
                                        f32(gamma), f32(beta), bf(dx), f32(dgamma), f32(dbeta), f32(sums),
                                        k8s_amd::kConvStatReplicas, f32(params), N, H, W, C, cur_stream());
  return dx;
}

// Backward of bn_relu_maxpool: dx of the conv output; dgamma / dbeta written into the given fp32 tensors.
Tensor pool_bn_bwd(Tensor dpool, Tensor idx, Tensor x, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta,
                   Tensor dgamma, Tensor dbeta) {
  check_cuda(dpool, "dpool"); check_dtype(dpool, at::kBFloat16, "dpool");
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  check_dtype(idx, at::kByte, "idx");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && dpool.is_contiguous() && idx.is_contiguous());
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(dpool.sizes() == idx.sizes() && dpool.size(0) == N && dpool.size(1) == (H + 1) / 2 &&
                  dpool.size(2) == (W + 1) / 2 && dpool.size(3) == C, "dpool / idx shape mismatch");
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.is_contiguous() && dbeta.is_contiguous());
  check_dtype(dgamma, at::kFloat, "dgamma"); check_dtype(dbeta, at::kFloat, "dbeta");
  auto dx = torch::empty_like(x);
  auto params = torch::empty({4 * C}, gamma.options());
  auto work = torch::empty({k8s_amd::pool_bn_workspace_floats(C)}, gamma.options());
  k8s_amd::launch_pool_bn_bwd(cbf(dpool), idx.data_ptr<uint8_t>(), cbf(x), f32(mean), f32(invstd), f32(gamma),
                              f32(beta), bf(dx), f32(dgamma), f32(dbeta), f32(work), f32(params), N, H, W, C,
                              cur_stream());
  return dx;
}

static const float* xform_ptr(const c10::optional<Tensor>& xf, long C) {
  if (!xf || !xf->defined()) return nullptr;
  TORCH_CHECK(xf->is_cuda() && xf->scalar_type() == at::kFloat && xf->is_contiguous() && xf->numel() == 2 * C,
              "xform must be fp32 [2 * C] (BatchNorm scale | shift)");
  TORCH_CHECK(C % 8 == 0, "xform channels must be a multiple of 8");
  return xf->data_ptr<float>();
}

// returns dx, dres (or empty), writes dgamma/dbeta into the given (flat-bucket view) tensors. The ReLU of the
// forward comes from the packed `mask` (residual BN), is recomputed from x (`relu_x`), or -- given the BN output
// `y` -- is packed from y first (compatibility; the trainer passes the mask).
std::vector<Tensor> bn_bwd(Tensor dy, Tensor x, c10::optional<Tensor> y, Tensor mean, Tensor invstd, Tensor gamma,
                           Tensor beta, bool relu_x, Tensor dgamma, Tensor dbeta, bool want_dres,
                           c10::optional<Tensor> mask) {
  check_cuda(dy, "dy"); check_cuda(x, "x");
  check_dtype(dy, at::kBFloat16, "dy"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(dy.sizes() == x.sizes());
  const int C = (int)x.size(-1);
  const long M = x.numel() / C;
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.is_contiguous() && dbeta.is_contiguous());
  check_dtype(dgamma, at::kFloat, "dgamma");
  TORCH_CHECK(!(relu_x && y), "relu mask from x and y are exclusive");
  Tensor ymask;
  if (y) {
    check_cuda(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes() && !mask, "y: same shape as x, exclusive with mask");
    ymask = torch::empty({x.numel() / 8}, x.options().dtype(at::kByte));
    k8s_amd::launch_relu_mask(cbf(y->contiguous()), ymask.data_ptr<uint8_t>(), x.numel() / 8, cur_stream());
  }
  auto dx = torch::empty_like(x);
  Tensor dres = want_dres ? torch::empty_like(x) : Tensor();
  auto params = torch::empty({4 * C}, gamma.options());
  const uint8_t* mk = y ? ymask.data_ptr<uint8_t>() : cmask(mask);
  TORCH_CHECK(!mk || (!relu_x && (y || mask->numel() == x.numel() / 8)),
              "packed mask: M*C/8 bytes, exclusive with relu_x");
  auto work = torch::empty({k8s_amd::bn_workspace_floats(M, C)}, gamma.options());
  k8s_amd::launch_bn_bwd(cbf(dy), cbf(x), f32(mean), f32(invstd), f32(gamma), f32(beta), relu_x, bf(dx),
                         want_dres ? bf(dres) : nullptr, f32(dgamma), f32(dbeta), f32(work), f32(params), M, C,
                         cur_stream(), mk);
  return {dx, dres};
}

// Backward of bn_fwd_from_sums_dual: (dx, dx2) and both BatchNorms' dgamma / dbeta from one masked dy (dy and the
// packed ReLU mask read once per pass).
std::vector<Tensor> bn_bwd_dual(Tensor dy, Tensor mask, Tensor x, Tensor mean, Tensor invstd, Tensor gamma,
                                Tensor beta, Tensor dgamma, Tensor dbeta, Tensor x2, Tensor mean2, Tensor invstd2,
                                Tensor gamma2, Tensor beta2, Tensor dgamma2, Tensor dbeta2) {
  for (const Tensor* t : {&dy, &x, &x2}) {
    check_cuda(*t, "dy / x / x2"); check_dtype(*t, at::kBFloat16, "dy / x / x2");
    TORCH_CHECK(t->is_contiguous() && t->sizes() == x.sizes(), "dy / x / x2: same contiguous shape");
  }
  const int C = (int)x.size(-1);
  const long M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0, "channels must be a multiple of 8");
  for (const Tensor* t : {&mean, &invstd, &gamma, &beta, &dgamma, &dbeta, &mean2, &invstd2, &gamma2, &beta2, &dgamma2,
                          &dbeta2})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "per-channel fp32 of C");
  TORCH_CHECK(mask.numel() == x.numel() / 8, "packed mask: M*C/8 bytes");
  auto dx = torch::empty_like(x), dx2 = torch::empty_like(x);
  auto params = torch::empty({4 * C}, gamma.options()), params2 = torch::empty({4 * C}, gamma.options());
  auto work = torch::empty({k8s_amd::bn_workspace_floats(M, C)}, gamma.options());
  auto work2 = torch::empty({k8s_amd::bn_workspace_floats(M, C)}, gamma.options());
  k8s_amd::launch_bn_bwd_dual(cbf(dy), cmask(mask), cbf(x), f32(mean), f32(invstd), f32(gamma), f32(beta), bf(dx),
                              f32(dgamma), f32(dbeta), f32(work), f32(params), cbf(x2), f32(mean2), f32(invstd2),
                              f32(gamma2), f32(beta2), bf(dx2), f32(dgamma2), f32(dbeta2), f32(work2), f32(params2), M,
                              C, cur_stream());
  return {dx, dx2};
}

// ------------------------------------------------------------------ layernorm / rmsnorm
std::vector<Tensor> norm_fwd(Tensor x, c10::optional<Tensor> res, Tensor gamma, c10::optional<Tensor> beta, double eps,
                             bool rms) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x"); check_aligned(x, "x");
  const int D = (int)x.size(-1);
  TORCH_CHECK(D % 8 == 0 && D <= 8192, "norm row length must be a multiple of 8 and <= 8192");
  const long R = x.numel() / D;
  TORCH_CHECK(gamma.numel() == D); check_dtype(gamma, at::kFloat, "gamma");
  if (!rms) TORCH_CHECK(beta.has_value() && beta->numel() == D, "layernorm needs beta");
  if (res) { check_cuda(*res, "res"); TORCH_CHECK(res->sizes() == x.sizes()); }
  auto y = torch::empty_like(x);
  Tensor xsum = res ? torch::empty_like(x) : Tensor();
  auto mean = torch::empty({rms ? 1 : R}, gamma.options());
  auto rstd = torch::empty({R}, gamma.options());
  k8s_amd::launch_norm_fwd(rms, cbf(x), res ? cbf(*res) : nullptr, res ? bf(xsum) : nullptr, f32(gamma),
                           beta ? beta->data_ptr<float>() : nullptr, bf(y), f32(mean), f32(rstd), R, D, (float)eps,
                           cur_stream());
  return {y, mean, rstd, xsum};
}

// dsum (optional, fp32 [D]): also the column sums of dx -- the bias gradient of the linear that produced x's
// first summand (no residual gradient allowed)
Tensor norm_bwd(Tensor dy, Tensor x, Tensor gamma, Tensor mean, Tensor rstd, c10::optional<Tensor> dres,
                Tensor dgamma, c10::optional<Tensor> dbeta, bool rms, c10::optional<Tensor> dsum) {
  check_cuda(dy, "dy"); check_cuda(x, "x");
  check_dtype(dy, at::kBFloat16, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes());
  const int D = (int)x.size(-1);
  const long R = x.numel() / D;
  TORCH_CHECK(dgamma.numel() == D && dgamma.is_contiguous());
  if (!rms) TORCH_CHECK(dbeta.has_value() && dbeta->numel() == D);
  if (dres) TORCH_CHECK(dres->sizes() == x.sizes() && dres->is_contiguous());
  if (dsum) TORCH_CHECK(!dres && dsum->is_cuda() && dsum->scalar_type() == at::kFloat && dsum->is_contiguous() &&
                            dsum->numel() == D, "dsum: contiguous fp32 [D], no residual gradient");
  auto dx = torch::empty_like(x);
  auto work = torch::empty({k8s_amd::norm_workspace_floats(R, D)}, gamma.options());
  k8s_amd::launch_norm_bwd(rms, cbf(dy), cbf(x), f32(gamma), f32(mean), f32(rstd), dres ? cbf(*dres) : nullptr,
                           bf(dx), f32(dgamma), dbeta ? dbeta->data_ptr<float>() : nullptr, f32(work), R, D,
                           cur_stream(), dsum ? dsum->data_ptr<float>() : nullptr);
  return dx;
}

// ------------------------------------------------------------------ cross entropy
std::vector<Tensor> xent_fwd(Tensor logits, Tensor labels, int64_t ignore_index, double smoothing) {
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits must be [R, V] row-major");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat);
  check_cuda(labels, "labels"); check_dtype(labels, at::kLong, "labels");
  const long R = logits.size(0), V = logits.size(1);
  TORCH_CHECK(labels.numel() == R);
  auto opt = logits.options().dtype(at::kFloat);
  auto loss = torch::empty({R}, opt);
  auto lse = torch::empty({R}, opt);
  k8s_amd::launch_xent_fwd(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, labels.data_ptr<int64_t>(), R, V,
                           logits.stride(0), f32(loss), f32(lse), ignore_index, (float)smoothing, cur_stream());
  return {loss, lse};
}

// logits [R, Vpad] dense; classes are the first V columns; returns dlogits [R, Vpad] (pad columns zero)
Tensor xent_bwd(Tensor logits, Tensor labels, Tensor lse, Tensor dscale, int64_t ignore_index, double smoothing,
                int64_t V) {
  const long R = logits.size(0), Vpad = logits.size(1);
  TORCH_CHECK(logits.is_contiguous(), "xent_bwd expects dense logits");
  TORCH_CHECK(V > 0 && V <= Vpad);
  TORCH_CHECK(dscale.numel() == 1 || dscale.numel() == R);
  auto d = dscale.to(at::kFloat).contiguous();
  auto dl = torch::empty({R, Vpad}, logits.options());  // the kernel zeroes the pad columns itself
  k8s_amd::launch_xent_bwd(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, labels.data_ptr<int64_t>(),
                           f32(lse), f32(d), d.numel() == R, R, V, Vpad, dl.data_ptr(), ignore_index,
                           (float)smoothing, cur_stream());
  return dl;
}

// ------------------------------------------------------------------ GEMM / conv (MFMA)
void check_bf16_operand(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1, name, " must be a 2-D row-major GPU tensor");
  check_dtype(t, at::kBFloat16, name);
  check_aligned(t, name);
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " leading dimension must be a multiple of 8 elements");
}

// a: [M,K] if a_kmajor else [K,M];  b: [N,K] if b_kmajor else [K,N];  returns / writes C[M,N]
// K8S_AMD_GEMM256=0 routes every product to the 128 x 128 kernel, =2 every product the 256 x 256 kernel can take
// (A/B comparisons, debugging); read per call, so one process can A/B both kernels
static int gemm256_mode() {
  const char* e = std::getenv("K8S_AMD_GEMM256");
  return e ? atoi(e) : 1;
}
static bool use_gemm256(long M, long N, long K, bool a_kmajor, bool b_kmajor) {
  const int m = gemm256_mode();
  if (m == 2)
    return K % 64 == 0 && N % 4 == 0 && (a_kmajor || M % 8 == 0) && (b_kmajor || N % 8 == 0);
  return m != 0 && k8s_amd::gemm256_eligible((int)M, (int)N, (int)K, a_kmajor, b_kmajor);
}

// Zero-initialised int words for the stream-K tickets / flags, one buffer per (device, stream), grown on demand.
// The kernel leaves every word it used at zero again, so no per-call clear is needed; launches on one stream are
// ordered, so they never share the words concurrently, and two streams (a side stream, user streams) get their own.
static int* sk_sync_words(long n, const c10::Device& dev) {
  static std::mutex mu;
  static std::map<std::pair<int, int64_t>, Tensor> bufs;
  const int64_t sid = at::hip::getCurrentHIPStream(dev.index()).id();
  std::lock_guard<std::mutex> g(mu);
  Tensor& t = bufs[{dev.index(), sid}];
  if (!t.defined() || t.numel() < n)
    t = torch::zeros({std::max<long>(n, 1 << 16)}, torch::TensorOptions().dtype(at::kInt).device(dev));
  return t.data_ptr<int>();
}

Tensor mask_apply(Tensor src, Tensor mask) {
  check_cuda(src, "src");
  check_dtype(src, at::kBFloat16, "src");
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.is_contiguous() &&
                  mask.numel() * 8 == src.numel(), "mask: packed uint8, one bit per element");
  Tensor out = torch::empty_like(src);
  k8s_amd::launch_mask_apply(cbf(src), mask.data_ptr<uint8_t>(), bf(out), src.numel(), cur_stream());
  return out;
}

// 1x1 data gradient dx[M, N] = gy[M, K] . w[K, N] + (add_mask ? add_src : 0) that also accumulates the
// BatchNorm-backward statistics of dx for the BatchNorm(s) that produced the convolution's input (gemm_short.hip
// EPI 3 / 4): sums[r][0][c] += sum g, sums[r][1][c] += sum g (x - mean), g = bit ? dx : 0 with the BatchNorm's packed
// ReLU bits `mask`; with x2 (a ResNet downsample block's second BatchNorm) sums2[r][1][c] += sum g (x2 - mean2).
// sums / sums2: zeroed fp32 [conv_stat_replicas, 2, N].
Tensor dgrad_short_bnstats(Tensor gy, Tensor w, c10::optional<Tensor> add_opt, c10::optional<Tensor> add_mask_opt,
                           Tensor x, Tensor mask, Tensor mean, Tensor sums, c10::optional<Tensor> x2,
                           c10::optional<Tensor> mean2, c10::optional<Tensor> sums2) {
  // no addend (add_src None): the plain data gradient + the sums (EPI 5), one BatchNorm only
  const bool has_add = add_opt.has_value();
  TORCH_CHECK(has_add == add_mask_opt.has_value() && (has_add || !x2), "add_src / add_mask together; x2 needs them");
  Tensor add_src = has_add ? *add_opt : x;
  Tensor add_mask = has_add ? *add_mask_opt : mask;
  for (const Tensor* t : {&gy, &w, &add_src, &x}) {
    check_cuda(*t, "gy / w / add_src / x");
    check_dtype(*t, at::kBFloat16, "gy / w / add_src / x");
    TORCH_CHECK(t->is_contiguous() && t->dim() == 2, "gy / w / add_src / x: contiguous 2-d");
  }
  const long M = gy.size(0), K = gy.size(1), N = w.size(1);
  TORCH_CHECK(w.size(0) == K && add_src.sizes() == x.sizes() && x.size(0) == M && x.size(1) == N,
              "shapes: gy [M, K], w [K, N], add_src / x [M, N]");
  TORCH_CHECK(M < (1L << 31) && k8s_amd::gemm_short_bnstats_ok((int)M, (int)N, (int)K, x2.has_value()),
              "dgrad_short_bnstats: shape outside the kernel's contract (gemm_short_bnstats_ok)");
  for (const Tensor* t : {&add_mask, &mask})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kByte && t->is_contiguous() && t->numel() * 8 == M * N,
                "masks: packed uint8, one bit per element");
  const long nrep = k8s_amd::kConvStatReplicas;
  auto chk_sums = [&](const Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == nrep * 2 * N,
                "sums: zeroed fp32 [conv_stat_replicas, 2, N]");
  };
  chk_sums(sums);
  TORCH_CHECK(mean.numel() == N && mean.scalar_type() == at::kFloat && mean.is_cuda(), "mean: fp32 [N]");
  k8s_amd::GemmShortBnStats b;
  b.x = cbf(x);
  b.mask = mask.data_ptr<uint8_t>();
  b.mean = f32(mean);
  b.sums = f32(sums);
  if (x2) {
    TORCH_CHECK(mean2 && sums2, "x2 needs mean2 and sums2");
    check_cuda(*x2, "x2");
    check_dtype(*x2, at::kBFloat16, "x2");
    TORCH_CHECK(x2->is_contiguous() && x2->sizes() == x.sizes(), "x2: the shape of x");
    TORCH_CHECK(mean2->numel() == N && mean2->scalar_type() == at::kFloat, "mean2: fp32 [N]");
    chk_sums(*sums2);
    b.x2 = cbf(*x2);
    b.mean2 = f32(*mean2);
    b.sums2 = f32(*sums2);
  }
  Tensor out = torch::empty({M, N}, gy.options());
  k8s_amd::launch_gemm_short(cbf(gy), cbf(w), N, true, bf(out), has_add ? cbf(add_src) : nullptr,
                             has_add ? add_mask.data_ptr<uint8_t>() : nullptr, nullptr, nullptr, (int)M, (int)N,
                             (int)K, has_add ? 2 : 0, cur_stream(), &b);
  return out;
}

// 3x3 / stride-1 / pad-1 data gradient dx = conv(gy, wt) on the staged-window kernel (wt = conv_dgrad_wtrans(w))
// that also accumulates the BatchNorm-backward sums of dx for the non-residual BatchNorm + ReLU relu(BN(x)) that
// produced the convolution's input (conv3x3.hip epilogue): sums[r][0][c] += sum g, sums[r][1][c] += sum g (x - mean),
// g = relu_on(x) ? dx : 0. sums: zeroed fp32 [conv_stat_replicas, 2, C].
Tensor conv3x3_dgrad_bnstats(Tensor gy, Tensor wt, Tensor x, Tensor gamma, Tensor beta, Tensor mean, Tensor invstd,
                             Tensor sums) {
  for (const Tensor* t : {&gy, &wt, &x}) {
    check_cuda(*t, "gy / wt / x");
    check_dtype(*t, at::kBFloat16, "gy / wt / x");
    TORCH_CHECK(t->is_contiguous() && t->dim() == 4, "gy / wt / x: contiguous NHWC / KRSC");
  }
  const int N = (int)gy.size(0), H = (int)gy.size(1), W = (int)gy.size(2), Kc = (int)gy.size(3);
  const int C = (int)wt.size(0);
  TORCH_CHECK(wt.size(1) == 3 && wt.size(2) == 3 && wt.size(3) == Kc, "wt: [C, 3, 3, K]");
  TORCH_CHECK(x.size(0) == N && x.size(1) == H && x.size(2) == W && x.size(3) == C, "x: the shape of dx");
  TORCH_CHECK(k8s_amd::conv3x3_eligible(H, W, Kc, C, 3, 3, 1, 1, 1), "conv3x3_dgrad_bnstats: outside the kernel");
  for (const Tensor* t : {&gamma, &beta, &mean, &invstd})
    TORCH_CHECK(t->is_cuda() && t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(),
                "per-channel fp32 [C]");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() &&
                  sums.numel() == (long)k8s_amd::kConvStatReplicas * 2 * C,
              "sums: zeroed fp32 [conv_stat_replicas, 2, C]");
  Tensor dx = torch::empty({N, H, W, C}, gy.options());
  k8s_amd::BnBwdSums bb;
  bb.x = cbf(x);
  bb.gamma = f32(gamma);
  bb.beta = f32(beta);
  bb.mean = f32(mean);
  bb.invstd = f32(invstd);
  bb.sums = f32(sums);
  k8s_amd::launch_conv3x3(cbf(gy), cbf(wt), bf(dx), nullptr, nullptr, N, H, W, Kc, C, cur_stream(), &bb);
  return dx;
}

// 1x1 data gradient dx[M, N] = gy[M, K] . w[K, N] on the tile kernel with the BatchNorm-backward sums of dx for the
// relu(BN(x)) that produced the convolution's input (gemm.hip BST epilogue); for shapes the 4-wave kernel does not
// take (gemm_dgrad_bnstats_ok). sums: zeroed fp32 [conv_stat_replicas, 2, N].
Tensor gemm_dgrad_bnstats(Tensor gy, Tensor w, Tensor x, Tensor gamma, Tensor beta, Tensor mean, Tensor invstd,
                          Tensor sums) {
  for (const Tensor* t : {&gy, &w, &x}) {
    check_cuda(*t, "gy / w / x");
    check_dtype(*t, at::kBFloat16, "gy / w / x");
    TORCH_CHECK(t->is_contiguous() && t->dim() == 2, "gy / w / x: contiguous 2-d");
  }
  const long M = gy.size(0), K = gy.size(1), N = w.size(1);
  TORCH_CHECK(w.size(0) == K && x.size(0) == M && x.size(1) == N, "shapes: gy [M, K], w [K, N], x [M, N]");
  TORCH_CHECK(N % 8 == 0 && M < (1L << 31), "N % 8 == 0");
  for (const Tensor* t : {&gamma, &beta, &mean, &invstd})
    TORCH_CHECK(t->is_cuda() && t->numel() == N && t->scalar_type() == at::kFloat && t->is_contiguous(),
                "per-channel fp32 [N]");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() &&
                  sums.numel() == (long)k8s_amd::kConvStatReplicas * 2 * N,
              "sums: zeroed fp32 [conv_stat_replicas, 2, N]");
  Tensor out = torch::empty({M, N}, gy.options());
  if (use_gemm256(M, N, K, true, false)) {  // the product's regular path is the 256 x 256 kernel: its epilogue
    TORCH_CHECK(k8s_amd::gemm_w4_dgrad_bnstats_ok((int)M, (int)N, (int)K), "gemm_dgrad_bnstats: 4-wave contract");
    Tensor tab = torch::cat({gamma, beta, mean, invstd});
    const k8s_amd::Gemm256Plan plan = k8s_amd::gemm256_plan((int)M, (int)N, (int)K);
    Tensor slabs;
    int* sync = nullptr;
    if (plan.sk > 1) {
      slabs = torch::empty({k8s_amd::gemm256_sk_slab_floats(plan)}, gy.options().dtype(at::kFloat));
      sync = sk_sync_words(k8s_amd::gemm256_sk_sync_ints(plan), gy.device());
    }
    k8s_amd::launch_gemm_w4_dgrad_bnstats(cbf(gy), cbf(w), bf(out), (int)M, (int)N, (int)K, cbf(x), f32(tab),
                                          f32(sums), sync ? f32(slabs) : nullptr, sync, cur_stream());
    return out;
  }
  k8s_amd::BnBwdSums bb;
  bb.x = cbf(x);
  bb.gamma = f32(gamma);
  bb.beta = f32(beta);
  bb.mean = f32(mean);
  bb.invstd = f32(invstd);
  bb.sums = f32(sums);
  k8s_amd::launch_gemm_dgrad_bnstats(cbf(gy), cbf(w), bf(out), (int)M, (int)N, (int)K, bb, cur_stream());
  return out;
}

// out[M, N] += gy[M, K] . w[K, N] on the tile kernel, also accumulating the BatchNorm-backward sums of the final out
// for a BatchNorm whose ReLU bits are stored (mask kind: g = bit ? out : 0, sum g, sum g (x - mean)) -- the second
// of two data gradients into that BatchNorm's output (the stem pool's, nn.BnStatLink.last_full). Returns out.
// With add_src / add_mask (a ResNet identity block's residual gradient as (dy, packed ReLU bits)): out = product +
// (bit ? add_src : 0), out's old values unread.
// x2 / mean2 / sums2: the two-BatchNorm form (a ResNet downsample block's output), sums2[.][1] += sum g (x2 - mean2).
Tensor gemm_dgrad_bnstats_mask(Tensor gy, Tensor w, Tensor out, Tensor x, Tensor mask, Tensor mean, Tensor sums,
                               c10::optional<Tensor> add_src, c10::optional<Tensor> add_mask,
                               c10::optional<Tensor> x2, c10::optional<Tensor> mean2, c10::optional<Tensor> sums2) {
  for (const Tensor* t : {&gy, &w, &out, &x}) {
    check_cuda(*t, "gy / w / out / x");
    check_dtype(*t, at::kBFloat16, "gy / w / out / x");
    TORCH_CHECK(t->is_contiguous() && t->dim() == 2, "gy / w / out / x: contiguous 2-d");
  }
  const long M = gy.size(0), K = gy.size(1), N = w.size(1);
  TORCH_CHECK(w.size(0) == K && x.size(0) == M && x.size(1) == N && out.sizes() == x.sizes(),
              "shapes: gy [M, K], w [K, N], out / x [M, N]");
  TORCH_CHECK(N % 8 == 0 && M < (1L << 31), "N % 8 == 0");
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.numel() * 8 == M * N, "mask: packed bits");
  TORCH_CHECK(mean.is_cuda() && mean.numel() == N && mean.scalar_type() == at::kFloat, "mean: fp32 [N]");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.is_contiguous() &&
                  sums.numel() == (long)k8s_amd::kConvStatReplicas * 2 * N,
              "sums: zeroed fp32 [conv_stat_replicas, 2, N]");
  k8s_amd::BnBwdSums bb;
  bb.x = cbf(x);
  bb.mask = mask.data_ptr<uint8_t>();
  bb.mean = f32(mean);
  bb.sums = f32(sums);
  TORCH_CHECK(x2.has_value() == mean2.has_value() && x2.has_value() == sums2.has_value(), "x2 / mean2 / sums2 together");
  if (x2) {
    check_dtype(*x2, at::kBFloat16, "x2");
    TORCH_CHECK(x2->is_cuda() && x2->is_contiguous() && x2->sizes() == x.sizes(), "x2: the shape of x");
    TORCH_CHECK(mean2->is_cuda() && mean2->numel() == N && mean2->scalar_type() == at::kFloat, "mean2: fp32 [N]");
    TORCH_CHECK(sums2->is_cuda() && sums2->scalar_type() == at::kFloat && sums2->is_contiguous() &&
                    sums2->numel() == (long)k8s_amd::kConvStatReplicas * 2 * N, "sums2: fp32 [conv_stat_replicas, 2, N]");
    bb.x2 = cbf(*x2);
    bb.mean2 = f32(*mean2);
    bb.sums2 = f32(*sums2);
  }
  TORCH_CHECK(add_src.has_value() == add_mask.has_value(), "add_src and add_mask together");
  if (add_src) {
    check_dtype(*add_src, at::kBFloat16, "add_src");
    TORCH_CHECK(add_src->is_cuda() && add_src->is_contiguous() && add_src->numel() == M * N, "add_src: [M, N]");
    TORCH_CHECK(add_mask->is_cuda() && add_mask->scalar_type() == at::kByte && add_mask->numel() * 8 == M * N,
                "add_mask: packed bits");
  }
  k8s_amd::launch_gemm_dgrad_bnstats(cbf(gy), cbf(w), bf(out), (int)M, (int)N, (int)K, bb, cur_stream(), true,
                                     add_src ? cbf(*add_src) : nullptr,
                                     add_src ? add_mask->data_ptr<uint8_t>() : nullptr);
  return out;
}

// bn_bwd (relu_x: the ReLU recomputed from x) with the reduction done by dy's producer.
std::vector<Tensor> bn_bwd_relu_from_sums(Tensor dy, Tensor x, Tensor sums, Tensor mean, Tensor invstd, Tensor gamma,
                                          Tensor beta, Tensor dgamma, Tensor dbeta) {
  check_cuda(dy, "dy"); check_cuda(x, "x");
  check_dtype(dy, at::kBFloat16, "dy"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.is_contiguous() && x.is_contiguous(), "dy / x: same contiguous shape");
  const int C = (int)x.size(-1);
  const long M = x.numel() / C;
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.numel() % (2 * C) == 0, "sums: fp32 [R, 2, C]");
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.is_contiguous() && dbeta.is_contiguous());
  auto dx = torch::empty_like(x);
  auto params = torch::empty({4 * C}, gamma.options());
  k8s_amd::launch_bn_bwd_relu_from_sums(cbf(dy), cbf(x), f32(sums), (int)(sums.numel() / (2 * C)), f32(mean),
                                        f32(invstd), f32(gamma), f32(beta), bf(dx), f32(dgamma), f32(dbeta),
                                        f32(params), M, C, cur_stream());
  return {dx};
}

// BatchNorm backward (dx, dres) with the reduction already done by dy's producer (dgrad_short_bnstats sums).
std::vector<Tensor> bn_bwd_from_sums(Tensor dy, Tensor x, Tensor mask, Tensor sums, Tensor mean, Tensor invstd,
                                     Tensor gamma, Tensor beta, Tensor dgamma, Tensor dbeta, bool want_dres) {
  check_cuda(dy, "dy"); check_cuda(x, "x");
  check_dtype(dy, at::kBFloat16, "dy"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.is_contiguous() && x.is_contiguous(), "dy / x: same contiguous shape");
  const int C = (int)x.size(-1);
  const long M = x.numel() / C;
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.numel() * 8 == x.numel(), "mask: packed bits");
  TORCH_CHECK(sums.is_cuda() && sums.scalar_type() == at::kFloat && sums.numel() % (2 * C) == 0, "sums: fp32 [R, 2, C]");
  TORCH_CHECK(dgamma.numel() == C && dbeta.numel() == C && dgamma.is_contiguous() && dbeta.is_contiguous());
  auto dx = torch::empty_like(x);
  Tensor dres = want_dres ? torch::empty_like(x) : Tensor();
  auto params = torch::empty({4 * C}, gamma.options());
  k8s_amd::launch_bn_bwd_from_sums(cbf(dy), cbf(x), mask.data_ptr<uint8_t>(), f32(sums), (int)(sums.numel() / (2 * C)),
                                   f32(mean), f32(invstd), f32(gamma), f32(beta), bf(dx),
                                   want_dres ? bf(dres) : nullptr, f32(dgamma), f32(dbeta), f32(params), M, C,
                                   cur_stream());
  return {dx, dres};
}

// bn_bwd_dual with the reduction done by dy's producer: sums (sum g, sum g (x - mean)) and sums2 (slot 1:
// sum g (x2 - mean2)).
std::vector<Tensor> bn_bwd_dual_from_sums(Tensor dy, Tensor mask, Tensor x, Tensor mean, Tensor invstd, Tensor gamma,
                                          Tensor beta, Tensor dgamma, Tensor dbeta, Tensor sums, Tensor x2,
                                          Tensor mean2, Tensor invstd2, Tensor gamma2, Tensor beta2, Tensor dgamma2,
                                          Tensor dbeta2, Tensor sums2) {
  for (const Tensor* t : {&dy, &x, &x2}) {
    check_cuda(*t, "dy / x / x2"); check_dtype(*t, at::kBFloat16, "dy / x / x2");
    TORCH_CHECK(t->is_contiguous() && t->sizes() == x.sizes(), "dy / x / x2: same contiguous shape");
  }
  const int C = (int)x.size(-1);
  const long M = x.numel() / C;
  for (const Tensor* t : {&mean, &invstd, &gamma, &beta, &dgamma, &dbeta, &mean2, &invstd2, &gamma2, &beta2, &dgamma2,
                          &dbeta2})
    TORCH_CHECK(t->numel() == C && t->scalar_type() == at::kFloat && t->is_contiguous(), "per-channel fp32 of C");
  TORCH_CHECK(mask.numel() == x.numel() / 8 && mask.scalar_type() == at::kByte, "packed mask: M*C/8 bytes");
  for (const Tensor* t : {&sums, &sums2})
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == sums.numel() && t->numel() % (2 * C) == 0,
                "sums / sums2: fp32 [R, 2, C]");
  auto dx = torch::empty_like(x), dx2 = torch::empty_like(x);
  auto params = torch::empty({4 * C}, gamma.options()), params2 = torch::empty({4 * C}, gamma.options());
  k8s_amd::launch_bn_bwd_dual_from_sums(cbf(dy), mask.data_ptr<uint8_t>(), cbf(x), f32(sums),
                                        (int)(sums.numel() / (2 * C)), f32(mean), f32(invstd), f32(gamma), f32(beta),
                                        bf(dx), f32(dgamma), f32(dbeta), f32(params), cbf(x2), f32(sums2), f32(mean2),
                                        f32(invstd2), f32(gamma2), f32(beta2), bf(dx2), f32(dgamma2), f32(dbeta2),
                                        f32(params2), M, C, cur_stream());
  return {dx, dx2};
}

Tensor gemm(Tensor a, bool a_kmajor, Tensor b, bool b_kmajor, c10::optional<Tensor> out, bool out_f32,
            c10::optional<Tensor> bias, int64_t act, c10::optional<Tensor> pre, bool accumulate, double alpha,
            int64_t splits, c10::optional<Tensor> add_src, c10::optional<Tensor> add_mask, c10::optional<Tensor> xform_b,
            int64_t xform_c) {
  check_bf16_operand(a, "A");
  check_bf16_operand(b, "B");
  const long M = a_kmajor ? a.size(0) : a.size(1), K = a_kmajor ? a.size(1) : a.size(0);
  const long N = b_kmajor ? b.size(0) : b.size(1), Kb = b_kmajor ? b.size(1) : b.size(0);
  TORCH_CHECK(K == Kb, "inner dimensions differ: ", K, " vs ", Kb);
  // a K-major operand's K % 64 tail reads zeros (KMajor::ktot; e.g. the 1000-class head's data gradient)
  if (a_kmajor || b_kmajor) TORCH_CHECK(K % 8 == 0, "K-major operands need K % 8 == 0 (got ", K, ")");
  if (!a_kmajor) TORCH_CHECK(M % 8 == 0, "M-major A needs M % 8 == 0");
  if (!b_kmajor) TORCH_CHECK(N % 8 == 0, "N-major B needs N % 8 == 0");
  TORCH_CHECK(N % 4 == 0, "N must be a multiple of 4");
  Tensor c;
  if (out) {
    c = *out;
    TORCH_CHECK(c.is_cuda() && c.is_contiguous() && c.numel() == M * N, "out must be a contiguous [M,N] tensor");
    TORCH_CHECK(c.scalar_type() == (out_f32 ? at::kFloat : at::kBFloat16), "out dtype mismatch");
  } else {
    c = torch::empty({M, N}, a.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  }
  if (bias) TORCH_CHECK(bias->numel() == N && bias->scalar_type() == at::kFloat && bias->is_contiguous());
  if (pre) TORCH_CHECK(pre->numel() == M * N && pre->scalar_type() == at::kBFloat16 && pre->is_contiguous());
  const int mode = accumulate ? 1 : 0;
  k8s_amd::AddEpi add{nullptr, nullptr};
  if (add_src) {
    TORCH_CHECK(accumulate && !out_f32, "add_src: a bf16 accumulate-mode output");
    TORCH_CHECK(add_src->is_cuda() && add_src->scalar_type() == at::kBFloat16 && add_src->is_contiguous() &&
                    add_src->numel() == M * N, "add_src must be a contiguous bf16 tensor of the output's size");
    add.src = cbf(*add_src);
    if (add_mask) {
      TORCH_CHECK(add_mask->is_cuda() && add_mask->scalar_type() == at::kByte && add_mask->is_contiguous() &&
                      add_mask->numel() * 8 == M * N, "add_mask: packed uint8, one bit per output element");
      add.mask = add_mask->data_ptr<uint8_t>();
    }
  } else {
    TORCH_CHECK(!add_mask, "add_mask needs add_src");
  }
  const float* xfb = xform_ptr(xform_b, xform_c);
  if (xfb) TORCH_CHECK(!a_kmajor && !b_kmajor && out_f32 && !bias && act == 0 && !pre && !add_src &&
                           N % xform_c == 0, "normalize-on-load GEMM: the plain weight-gradient form only");
  if (!xfb && !add_src && use_gemm256(M, N, K, a_kmajor, b_kmajor)) {
    // stream-K tail of a partial-wave grid: fp32 partial slabs (caching allocator, stream-ordered) and the
    // self-resetting ticket / flag words
    const k8s_amd::Gemm256Plan plan = k8s_amd::gemm256_plan((int)M, (int)N, (int)K);
    Tensor slabs;
    int* sync = nullptr;
    if (plan.sk > 1) {
      slabs = torch::empty({k8s_amd::gemm256_sk_slab_floats(plan)}, a.options().dtype(at::kFloat));
      sync = sk_sync_words(k8s_amd::gemm256_sk_sync_ints(plan), a.device());
    }
    k8s_amd::launch_gemm256(cbf(a), a.stride(0), a_kmajor, cbf(b), b.stride(0), b_kmajor, c.data_ptr(), N, out_f32,
                            (int)M, (int)N, (int)K, bias ? bias->data_ptr<float>() : nullptr, (int)act,
                            pre ? bf(*pre) : nullptr, accumulate, (float)alpha, cur_stream(), 1, nullptr,
                            sync ? f32(slabs) : nullptr, sync);
    return c;
  }
  // tall-K fp32 products whose output is too small for the 256 x 256 kernel alone (the ResNet 1x1 weight gradients):
  // split-K on the 256 kernel
  if (!xfb && !add_src && splits != 1 && out_f32 && !bias && act == 0 && !pre && gemm256_mode() != 0 &&
      K % 64 == 0 && (a_kmajor || M % 8 == 0) && (b_kmajor || N % 8 == 0) && N % 4 == 0) {
    const int s256 = k8s_amd::gemm256_choose_splits((int)M, (int)N, (int)K);
    const long t256 = ((M + 255) / 256) * ((N + 255) / 256);
    if (s256 > 1 && t256 * s256 >= 128) {
      auto ws = torch::empty({(long)s256 * M * N}, c.options());
      k8s_amd::launch_gemm256(cbf(a), a.stride(0), a_kmajor, cbf(b), b.stride(0), b_kmajor, c.data_ptr(), N, true,
                              (int)M, (int)N, (int)K, nullptr, 0, nullptr, accumulate, (float)alpha, cur_stream(), s256,
                              f32(ws));
      return c;
    }
  }
  int sp = (int)splits;
  if (sp != 1 && out_f32 && !bias && act == 0 && !pre && N % 4 == 0) {
    if (sp <= 0) sp = k8s_amd::gemm_choose_splits((int)M, (int)N, (int)K);
  } else {
    sp = 1;
  }
  Tensor ws;
  if (sp > 1) ws = torch::empty({k8s_amd::gemm_splitk_workspace((int)M, (int)N, sp)}, a.options().dtype(at::kFloat));
  k8s_amd::launch_gemm(cbf(a), a.stride(0), a_kmajor, cbf(b), b.stride(0), b_kmajor, c.data_ptr(), N, out_f32,
                       (int)M, (int)N, (int)K, bias ? bias->data_ptr<float>() : nullptr, (int)act,
                       pre ? bf(*pre) : nullptr, mode, (float)alpha, sp, sp > 1 ? f32(ws) : nullptr, cur_stream(),
                       add_src ? &add : nullptr, xfb, (int)xform_c);
  return c;
}

// dx = (g . W) * act'(pre) and db (+)= column sums of dx: the data gradient of a linear whose input is the output of
// an activation (1 ReLU: pre = the ReLU output, 2 GELU: the pre-activation), fused with that activation's backward and
// Llama's down-projection data gradient fused with the SwiGLU backward: dgu [M, 2F] = swiglu_bwd(gu, g . w),
// g [M, K] bf16, w [K, F] bf16 (the down weight [out, in], read MN-major), gu [M, 2F] bf16 (gate | up).
bool gemm_swiglu_bwd_ok(int64_t M, int64_t F, int64_t K) {
  return k8s_amd::gemm_w4_swiglu_ok((int)M, (int)F, (int)K, K, F);
}
Tensor gemm_swiglu_bwd(Tensor g, Tensor w, Tensor gu, int64_t blk) {
  check_bf16_operand(g, "g");
  check_bf16_operand(w, "w");
  check_bf16_operand(gu, "gu");
  const long M = g.size(0), K = g.size(1), F = w.size(1);
  TORCH_CHECK(w.size(0) == K, "g [M, K] . w [K, F]");
  TORCH_CHECK(gu.is_contiguous() && gu.size(0) == M && gu.size(1) == 2 * F, "gu must be a contiguous [M, 2F]");
  TORCH_CHECK(k8s_amd::gemm_w4_swiglu_ok((int)M, (int)F, (int)K, g.stride(0), w.stride(0)),
              "gemm_swiglu_bwd: shape outside the 4-wave kernel's contract");
  Tensor dgu = torch::empty({M, 2 * F}, g.options());
  const k8s_amd::Gemm256Plan plan = k8s_amd::gemm256_plan((int)M, (int)F, (int)K);
  Tensor slabs;
  int* sync = nullptr;
  if (plan.sk > 1) {
    slabs = torch::empty({k8s_amd::gemm256_sk_slab_floats(plan)}, g.options().dtype(at::kFloat));
    sync = sk_sync_words(k8s_amd::gemm256_sk_sync_ints(plan), g.device());
  }
  TORCH_CHECK(blk == 0 || blk == 64, "gemm_swiglu_bwd: blk is 0 (gate | up halves) or 64 (blocked layout)");
  k8s_amd::launch_gemm_w4_swiglu_bwd(cbf(g), g.stride(0), cbf(w), w.stride(0), bf(dgu), cbf(gu), (int)M, (int)F,
                                     (int)K, (int)blk, sync ? f32(slabs) : nullptr, sync, cur_stream());
  return dgu;
}

// Llama's QKV projection with the rotary embedding of its q / k heads (the first rot_cols columns, head dim 128) in
// the epilogue: y [M, N] = x [M, K] . w [N, K]^T, pos [M] int32, table [maxpos, 64, 2] fp32 (gemm256.hip copy_out_rope)
bool gemm_rope_ok(int64_t M, int64_t N, int64_t K, int64_t rot_cols) {
  return k8s_amd::gemm_w4_rope_ok((int)M, (int)N, (int)K, K, K, (int)rot_cols);
}
Tensor gemm_rope(Tensor x, Tensor w, Tensor pos, Tensor table, int64_t rot_cols) {
  check_bf16_operand(x, "x");
  check_bf16_operand(w, "w");
  const long M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && x.stride(1) == 1 && w.stride(1) == 1, "x [M, K] . w [N, K]^T, row-major");
  TORCH_CHECK(pos.is_cuda() && pos.scalar_type() == at::kInt && pos.is_contiguous() && pos.numel() == M, "pos: [M] int32");
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kFloat && table.is_contiguous() && table.dim() == 3 &&
                  table.size(1) == 64 && table.size(2) == 2, "table: [maxpos, 64, 2] fp32 (head dim 128)");
  TORCH_CHECK(k8s_amd::gemm_w4_rope_ok((int)M, (int)N, (int)K, x.stride(0), w.stride(0), (int)rot_cols),
              "gemm_rope: shape outside the 4-wave kernel's contract");
  Tensor y = torch::empty({M, N}, x.options());
  const k8s_amd::Gemm256Plan plan = k8s_amd::gemm256_plan((int)M, (int)N, (int)K);
  Tensor slabs;
  int* sync = nullptr;
  if (plan.sk > 1) {
    slabs = torch::empty({k8s_amd::gemm256_sk_slab_floats(plan)}, x.options().dtype(at::kFloat));
    sync = sk_sync_words(k8s_amd::gemm256_sk_sync_ints(plan), x.device());
  }
  k8s_amd::launch_gemm_w4_rope(cbf(x), x.stride(0), cbf(w), w.stride(0), bf(y), (int)M, (int)N, (int)K,
                               pos.data_ptr<int>(), f32(table), (int)rot_cols, sync ? f32(slabs) : nullptr, sync,
                               cur_stream());
  return y;
}

// Llama's gate|up projection with the SwiGLU in the epilogue: returns (gu [M, 2F], h [M, F] = silu(gate) up) from
// x [M, K] bf16 and w [2F, K] bf16 whose rows are in the 64-blocked gate|up order (gemm256.hip copy_out_swiglu).
bool gemm_swiglu_fwd_ok(int64_t M, int64_t F, int64_t K) {
  return k8s_amd::gemm_w4_swiglu_fwd_ok((int)M, (int)F, (int)K, K, K);
}
std::vector<Tensor> gemm_swiglu_fwd(Tensor x, Tensor w) {
  check_bf16_operand(x, "x");
  check_bf16_operand(w, "w");
  const long M = x.size(0), K = x.size(1), F2 = w.size(0);
  TORCH_CHECK(w.size(1) == K && F2 % 2 == 0, "x [M, K] . w [2F, K]^T");
  TORCH_CHECK(x.stride(1) == 1 && w.stride(1) == 1, "x and w must be row-major");
  const long F = F2 / 2;
  TORCH_CHECK(k8s_amd::gemm_w4_swiglu_fwd_ok((int)M, (int)F, (int)K, x.stride(0), w.stride(0)),
              "gemm_swiglu_fwd: shape outside the 4-wave kernel's contract");
  Tensor gu = torch::empty({M, F2}, x.options());
  Tensor h = torch::empty({M, F}, x.options());
  const k8s_amd::Gemm256Plan plan = k8s_amd::gemm256_plan((int)M, (int)F2, (int)K);
  Tensor slabs;
  int* sync = nullptr;
  if (plan.sk > 1) {
    slabs = torch::empty({k8s_amd::gemm256_sk_slab_floats(plan)}, x.options().dtype(at::kFloat));
    sync = sk_sync_words(k8s_amd::gemm256_sk_sync_ints(plan), x.device());
  }
  k8s_amd::launch_gemm_w4_swiglu_fwd(cbf(x), x.stride(0), cbf(w), w.stride(0), bf(gu), bf(h), (int)M, (int)F, (int)K,
                                     sync ? f32(slabs) : nullptr, sync, cur_stream());
  return {gu, h};
}

// the producing linear's bias gradient in the 4-wave GEMM's epilogue (gemm256.hip copy_out_x, ACT < 0).
// g [M, N_out] bf16, w [N_out, K_in] bf16 (read MN-major), pre [M, K_in] bf16, db fp32 [K_in].
bool gemm_dact_ok(int64_t M, int64_t N, int64_t K) { return k8s_amd::gemm_w4_dact_ok((int)M, (int)N, (int)K, K, N, N); }
Tensor gemm_dact(Tensor g, Tensor w, Tensor pre, int64_t act, Tensor db, bool db_accumulate) {
  check_bf16_operand(g, "g");
  check_bf16_operand(w, "w");
  check_bf16_operand(pre, "pre");
  const long M = g.size(0), K = g.size(1), N = w.size(1);
  TORCH_CHECK(w.size(0) == K, "g [M, K] . w [K, N]");
  TORCH_CHECK(pre.is_contiguous() && pre.size(0) == M && pre.size(1) == N, "pre must be a contiguous [M, N]");
  TORCH_CHECK(db.is_cuda() && db.scalar_type() == at::kFloat && db.is_contiguous() && db.numel() == N,
              "db: contiguous fp32 [N]");
  TORCH_CHECK(act == 1 || act == 2, "act: 1 ReLU, 2 GELU(tanh)");
  TORCH_CHECK(k8s_amd::gemm_w4_dact_ok((int)M, (int)N, (int)K, g.stride(0), w.stride(0), N),
              "gemm_dact: shape outside the 4-wave kernel's contract");
  Tensor c = torch::empty({M, N}, g.options());
  Tensor part = torch::empty({k8s_amd::gemm_w4_dact_part_floats((int)M, (int)N)}, db.options());
  const k8s_amd::Gemm256Plan plan = k8s_amd::gemm256_plan((int)M, (int)N, (int)K);
  Tensor slabs;
  int* sync = nullptr;
  if (plan.sk > 1) {
    slabs = torch::empty({k8s_amd::gemm256_sk_slab_floats(plan)}, db.options());
    sync = sk_sync_words(k8s_amd::gemm256_sk_sync_ints(plan), g.device());
  }
  k8s_amd::launch_gemm_w4_dact(cbf(g), g.stride(0), cbf(w), w.stride(0), bf(c), N, (int)M, (int)N, (int)K, cbf(pre),
                               (int)act, f32(part), f32(db), db_accumulate, sync ? f32(slabs) : nullptr, sync,
                               cur_stream());
  return c;
}

static inline int conv_out(int in, int k, int st, int pad, int dil) { return (in + 2 * pad - dil * (k - 1) - 1) / st + 1; }

Tensor conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad, int64_t dil, bool out_f32, c10::optional<Tensor> bias,
                int64_t act, c10::optional<Tensor> stats, c10::optional<Tensor> xform) {
  check_cuda(x, "x"); check_cuda(w, "w");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "x [N,H,W,C], w [K,R,S,C]");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = w.size(0), R = w.size(1), S = w.size(2);
  TORCH_CHECK(w.size(3) == C, "channel mismatch");
  TORCH_CHECK(C % 8 == 0, "implicit-GEMM conv needs C % 8 == 0");
  TORCH_CHECK(K % 8 == 0, "output channels must be a multiple of 8");
  const int Ho = conv_out(H, R, stride, pad, dil), Wo = conv_out(W, S, stride, pad, dil);
  auto y = torch::empty({N, Ho, Wo, K}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  if (stats) TORCH_CHECK(stats->numel() == (long)k8s_amd::kConvStatReplicas * 2 * K &&
                             stats->scalar_type() == at::kFloat && stats->is_contiguous(),
                         "stats must be zeroed fp32 [conv_stat_replicas, 2, K]");
  const float* xf = xform_ptr(xform, C);
  if (xf) TORCH_CHECK(C % 64 == 0 && !out_f32 && !bias && act == 0,
                      "normalize-on-load convolution: C % 64 == 0, bf16 output, no bias / activation");
  k8s_amd::launch_conv_fwd(cbf(x), cbf(w), y.data_ptr(), out_f32, N, H, W, C, K, R, S, (int)stride, (int)pad,
                           (int)dil, Ho, Wo, bias ? bias->data_ptr<float>() : nullptr, (int)act, 0,
                           stats ? f32(*stats) : nullptr, cur_stream(), nullptr, xf);
  return y;
}

// One output-parity piece of a stride-s data gradient: out[n, i*s+a, j*s+b, :] = conv(dy, wsub, stride 1, pad)
// over an Hs x Ws grid (i < Hs, j < Ws). wsub [C, Tr, Ts, K] holds the taps of that parity
// (ops/conv.py _dgrad_strided_hip builds it); out is the full bf16 dx [N, H, W, C].
// out[n, i*stride + a, j*stride + b, :] (+)= conv(x, w)[n, i, j, :]: one output parity of a strided dgrad;
// `accumulate` adds onto out in the epilogue (out already holds the residual branch's gradient).
void conv_fwd_subgrid(Tensor x, Tensor w, int64_t pad, int64_t Hs, int64_t Ws, Tensor out, int64_t stride, int64_t a,
                      int64_t b, bool accumulate, c10::optional<Tensor> bn_x, c10::optional<Tensor> bn_mask,
                      c10::optional<Tensor> bn_mean, c10::optional<Tensor> bn_sums, c10::optional<Tensor> bn_gamma,
                      c10::optional<Tensor> bn_beta, c10::optional<Tensor> bn_invstd) {
  check_cuda(x, "x"); check_cuda(w, "w"); check_cuda(out, "out");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(w, at::kBFloat16, "w"); check_dtype(out, at::kBFloat16, "out");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && out.dim() == 4 && out.is_contiguous());
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = w.size(0), R = w.size(1), S = w.size(2);
  TORCH_CHECK(w.size(3) == C && C % 8 == 0 && K % 8 == 0, "sub-grid conv needs C % 8 == 0, K % 8 == 0");
  TORCH_CHECK(out.size(0) == N && out.size(3) == K, "out shape");
  const int OH = out.size(1), OW = out.size(2);
  TORCH_CHECK(stride >= 1 && a >= 0 && a < stride && b >= 0 && b < stride, "parity out of range");
  TORCH_CHECK(Hs >= 1 && Ws >= 1 && (Hs - 1) * stride + a < OH && (Ws - 1) * stride + b < OW,
              "sub-grid exceeds the output image");
  k8s_amd::SubGrid sg{OH, OW, (int)stride, (int)a, (int)b};
  // bn_*: the correction of a residual BatchNorm's backward sums for the elements this accumulating product changes
  // (gemm.hip BST sub-grid path; the first data gradient into `out` took the sums over its values)
  k8s_amd::BnBwdSums bb;
  // relu kind (bn_gamma / bn_beta / bn_invstd, no bn_mask, a plain store): the sums of a BatchNorm + ReLU over this
  // parity's stored pixels (a stride-2 data gradient; the parities partition the output)
  if (bn_sums) {
    const bool relu_kind = !bn_mask;
    TORCH_CHECK(bn_x && bn_mean, "bn sums: bn_x and bn_mean");
    TORCH_CHECK(relu_kind ? (bn_gamma && bn_beta && bn_invstd && !accumulate) : accumulate,
                "bn sums: bn_mask + accumulate (a correction) or bn_gamma / bn_beta / bn_invstd + a plain store");
    check_dtype(*bn_x, at::kBFloat16, "bn_x");
    TORCH_CHECK(bn_x->sizes() == out.sizes() && bn_x->is_contiguous(), "bn_x: the shape of out");
    TORCH_CHECK(relu_kind || (bn_mask->scalar_type() == at::kByte && bn_mask->numel() * 8 == out.numel()),
                "bn_mask: packed bits");
    TORCH_CHECK(bn_mean->numel() == K && bn_mean->scalar_type() == at::kFloat, "bn_mean: fp32 [K]");
    TORCH_CHECK(bn_sums->numel() == (long)k8s_amd::kConvStatReplicas * 2 * K && bn_sums->scalar_type() == at::kFloat,
                "bn_sums: fp32 [conv_stat_replicas, 2, K]");
    bb.x = cbf(*bn_x);
    bb.mean = f32(*bn_mean);
    bb.sums = f32(*bn_sums);
    if (relu_kind) {
      for (const c10::optional<Tensor>* t : {&bn_gamma, &bn_beta, &bn_invstd})
        TORCH_CHECK((*t)->numel() == K && (*t)->scalar_type() == at::kFloat && (*t)->is_contiguous(),
                    "bn_gamma / bn_beta / bn_invstd: fp32 [K]");
      bb.gamma = f32(*bn_gamma);
      bb.beta = f32(*bn_beta);
      bb.invstd = f32(*bn_invstd);
    } else {
      bb.mask = bn_mask->data_ptr<uint8_t>();
    }
  }
  k8s_amd::launch_conv_fwd(cbf(x), cbf(w), out.data_ptr(), false, N, H, W, C, K, R, S, 1, (int)pad, 1, (int)Hs,
                           (int)Ws, nullptr, 0, accumulate ? 1 : 0, nullptr, cur_stream(), &sg, nullptr,
                           bn_sums ? &bb : nullptr);
}

// dw[K,R,S,C] fp32 (+)= dy^T . im2col(x)
void conv_wgrad(Tensor x, Tensor dy, Tensor dw, int64_t stride, int64_t pad, int64_t dil, int64_t splits,
                bool accumulate, c10::optional<Tensor> xform) {
  check_cuda(x, "x"); check_cuda(dy, "dy"); check_cuda(dw, "dw");
  check_dtype(x, at::kBFloat16, "x"); check_dtype(dy, at::kBFloat16, "dy"); check_dtype(dw, at::kFloat, "dw");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = dw.size(0), R = dw.size(1), S = dw.size(2);
  TORCH_CHECK(dw.size(3) == C && C % 8 == 0 && K % 8 == 0);
  const int Ho = conv_out(H, R, stride, pad, dil), Wo = conv_out(W, S, stride, pad, dil);
  TORCH_CHECK(dy.size(0) == N && dy.size(1) == Ho && dy.size(2) == Wo && dy.size(3) == K, "dy shape mismatch");
  const float* xf = xform_ptr(xform, C);
  if (dil == 1 && dy.is_contiguous() && x.is_contiguous() && Ho == H &&
      Wo == W && H == W && k8s_amd::wgrad3x3_tiled_ok(C, K, R, S, (int)stride, (int)pad, W)) {
    auto wsp = torch::empty({k8s_amd::wgrad3x3_tiled_workspace(N, H, W, C)}, dw.options());
    k8s_amd::launch_wgrad3x3_tiled(cbf(x), cbf(dy), f32(wsp), f32(dw), N, H, W, C, accumulate, cur_stream(), xf);
    return;
  }
  if (!xf && dil == 1 && dy.is_contiguous() && x.is_contiguous() &&
      k8s_amd::wgrad_stream_eligible(N, Ho, Wo, C, K, R, S)) {
    k8s_amd::launch_wgrad_stream(cbf(x), cbf(dy), f32(dw), N, H, W, C, K, R, S, (int)stride, (int)pad, Ho, Wo,
                                 accumulate, cur_stream());
    return;
  }
  int sp = splits <= 0 ? k8s_amd::gemm_choose_splits(K, R * S * C, N * Ho * Wo) : (int)splits;
  Tensor ws;
  if (sp > 1) ws = torch::empty({k8s_amd::gemm_splitk_workspace(K, R * S * C, sp)}, dw.options());
  if (xf) TORCH_CHECK(C % 64 == 0, "normalize-on-load weight gradient needs C % 64 == 0");
  k8s_amd::launch_conv_wgrad(cbf(x), cbf(dy), f32(dw), N, H, W, C, K, R, S, (int)stride, (int)pad, (int)dil, Ho, Wo,
                             sp, accumulate, sp > 1 ? f32(ws) : nullptr, cur_stream(), xf);
}

// taps: per parity, the list of r*S + s tap indices (row-major over its [Tr][Ts] grid); returns one packed bf16
// buffer with parity p's [C, T_p, K] sub-weight at the element offset offsets[p]
std::vector<Tensor> conv_dgrad_wsub(Tensor w, std::vector<std::vector<int64_t>> taps) {
  check_cuda(w, "w"); check_dtype(w, at::kBFloat16, "w");
  const int K = w.size(0), R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(!taps.empty() && taps.size() <= 16, "1-16 parities");
  k8s_amd::DgradTaps t{};
  long off = 0;
  std::vector<int64_t> offs;
  for (size_t p = 0; p < taps.size(); ++p) {
    TORCH_CHECK(!taps[p].empty() && taps[p].size() <= 16, "1-16 taps per parity");
    t.n[p] = (int)taps[p].size();
    t.off[p] = off;
    offs.push_back(off);
    for (size_t i = 0; i < taps[p].size(); ++i) {
      TORCH_CHECK(taps[p][i] >= 0 && taps[p][i] < R * S, "tap index out of range");
      t.rs[p][i] = (int)taps[p][i];
    }
    off += (long)C * t.n[p] * K;
    off = (off + 7) / 8 * 8;  // keep every parity's sub-weight 16-B aligned
  }
  auto out = torch::empty({off}, w.options());
  k8s_amd::launch_conv_dgrad_wsub(cbf(w), bf(out), K, R * S, C, t, (int)taps.size(), cur_stream());
  return {out, torch::tensor(offs)};
}

Tensor conv_dgrad_wtrans(Tensor w) {
  check_cuda(w, "w"); check_dtype(w, at::kBFloat16, "w");
  const int K = w.size(0), R = w.size(1), S = w.size(2), C = w.size(3);
  auto w2 = torch::empty({C, R, S, K}, w.options());
  k8s_amd::launch_conv_dgrad_wtrans(cbf(w), bf(w2), K, R, S, C, cur_stream());
  return w2;
}

// ------------------------------------------------------------------ elementwise (K9)
Tensor swiglu_fwd(Tensor gu, int64_t blk) {
  check_cuda(gu, "gu"); check_dtype(gu, at::kBFloat16, "gu");
  const long F2 = gu.size(-1);
  TORCH_CHECK(F2 % 16 == 0, "2F must be a multiple of 16");
  const long T = gu.numel() / F2;
  auto sizes = gu.sizes().vec();
  sizes.back() = F2 / 2;
  auto y = torch::empty(sizes, gu.options());
  TORCH_CHECK(blk == 0 || (blk % 8 == 0 && (F2 / 2) % blk == 0), "swiglu: blk must divide F (multiple of 8)");
  k8s_amd::launch_swiglu_fwd(cbf(gu), bf(y), T, (int)(F2 / 2), (int)blk, cur_stream());
  return y;
}
Tensor swiglu_bwd(Tensor gu, Tensor dy, int64_t blk) {
  check_cuda(gu, "gu"); check_cuda(dy, "dy");
  const long F2 = gu.size(-1);
  TORCH_CHECK(dy.numel() * 2 == gu.numel());
  auto dgu = torch::empty_like(gu);
  TORCH_CHECK(blk == 0 || (blk % 8 == 0 && (F2 / 2) % blk == 0), "swiglu: blk must divide F (multiple of 8)");
  k8s_amd::launch_swiglu_bwd(cbf(gu), cbf(dy), bf(dgu), gu.numel() / F2, (int)(F2 / 2), (int)blk, cur_stream());
  return dgu;
}
// in place on x [T, H*D]: contiguous, or a 2-D column slice of a wider row-major tensor (row stride = its
// leading dimension -- the q and k heads of a packed QKV projection rotated without a copy)
void rope_(Tensor x, Tensor pos, Tensor table, bool inverse) {
  TORCH_CHECK(x.is_cuda(), "x must be a GPU tensor"); check_dtype(x, at::kBFloat16, "x");
  check_cuda(pos, "pos"); check_dtype(pos, at::kInt, "pos");
  check_cuda(table, "table"); check_dtype(table, at::kFloat, "table");
  const int D = (int)table.size(1) * 2;
  TORCH_CHECK(D % 16 == 0, "head dim must be a multiple of 16");
  const long T = pos.numel();
  long ld;
  int H;
  if (x.is_contiguous()) {
    TORCH_CHECK(x.numel() % (T * D) == 0, "x must be [T, H*D]");
    H = (int)(x.numel() / (T * D));
    ld = (long)H * D;
  } else {
    TORCH_CHECK(x.dim() == 2 && x.size(0) == T && x.stride(1) == 1 && x.size(1) % D == 0 && x.stride(0) % 8 == 0,
                "strided x must be a [T, H*D] column slice with unit column stride");
    check_aligned(x, "x");
    H = (int)(x.size(1) / D);
    ld = x.stride(0);
  }
  k8s_amd::launch_rope(bf(x), ld, pos.data_ptr<int>(), f32(table), T, H, D, inverse, cur_stream());
}
Tensor gelu_bwd(Tensor dy, Tensor pre) {
  check_cuda(dy, "dy"); check_cuda(pre, "pre");
  TORCH_CHECK(dy.numel() == pre.numel() && dy.numel() % 8 == 0);
  auto dx = torch::empty_like(dy);
  k8s_amd::launch_gelu_bwd(cbf(dy), cbf(pre), bf(dx), dy.numel(), cur_stream());
  return dx;
}
Tensor relu_bwd(Tensor dy, Tensor y) {
  check_cuda(dy, "dy"); check_cuda(y, "y");
  TORCH_CHECK(dy.numel() == y.numel() && dy.numel() % 8 == 0);
  auto dx = torch::empty_like(dy);
  k8s_amd::launch_relu_bwd(cbf(dy), cbf(y), bf(dx), dy.numel(), cur_stream());
  return dx;
}
// column sums of a [R, C] bf16 matrix in fp32; `out` (optional, fp32 [C] contiguous, e.g. a bias's flat gradient
// slot) is written in place instead of a new tensor
Tensor colsum(Tensor x, c10::optional<Tensor> out_) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  const int C = (int)x.size(-1);
  TORCH_CHECK(C % 8 == 0);
  const long R = x.numel() / C;
  Tensor out;
  if (out_) {
    out = *out_;
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == C,
                "colsum out: contiguous fp32 [C]");
  } else {
    out = torch::empty({C}, x.options().dtype(at::kFloat));
  }
  auto work = torch::empty({k8s_amd::colsum_workspace_floats(R, C)}, out.options());
  k8s_amd::launch_colsum(cbf(x), R, C, f32(work), f32(out), false, cur_stream());
  return out;
}

// activation backward + the column sums of its result (a linear's bias gradient); returns [g, db]
std::vector<Tensor> act_bwd_colsum(Tensor dy, Tensor pre, int64_t act, c10::optional<Tensor> out_) {
  check_cuda(dy, "dy"); check_cuda(pre, "pre");
  check_dtype(dy, at::kBFloat16, "dy"); check_dtype(pre, at::kBFloat16, "pre");
  TORCH_CHECK(act == 1 || act == 2, "act: 1 ReLU, 2 GELU(tanh)");
  TORCH_CHECK(dy.sizes() == pre.sizes() && dy.is_contiguous() && pre.is_contiguous());
  const int C = (int)dy.size(-1);
  TORCH_CHECK(C % 8 == 0);
  const long R = dy.numel() / C;
  Tensor out;
  if (out_) {
    out = *out_;
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == C,
                "act_bwd_colsum out: contiguous fp32 [C]");
  } else {
    out = torch::empty({C}, dy.options().dtype(at::kFloat));
  }
  auto g = torch::empty_like(dy);
  auto work = torch::empty({k8s_amd::colsum_workspace_floats(R, C)}, out.options());
  k8s_amd::launch_act_bwd_colsum((int)act, cbf(dy), cbf(pre), bf(g), R, C, f32(work), f32(out), false, cur_stream());
  return {g, out};
}

// ------------------------------------------------------------------ flash attention (K5)
void check_attn_operand(const Tensor& t, const char* name, long D) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  check_dtype(t, at::kBFloat16, name);
  TORCH_CHECK(t.dim() == 4, name, " must be [B, S, H, D]");
  TORCH_CHECK(t.size(3) == D && t.stride(3) == 1, name, " must have a contiguous head dim of ", D);
  for (int i = 0; i < 3; ++i) TORCH_CHECK(t.stride(i) % 8 == 0, name, " strides must be multiples of 8 elements");
  check_aligned(t, name);
}

const int* kv_lens_ptr(const c10::optional<Tensor>& kv_lens, long B) {
  if (!kv_lens) return nullptr;
  TORCH_CHECK(kv_lens->is_cuda() && kv_lens->scalar_type() == at::kInt && kv_lens->is_contiguous() &&
                  kv_lens->numel() == B, "kv_lens must be an int32 GPU tensor of length B");
  return kv_lens->data_ptr<int>();
}

std::vector<Tensor> flash_fwd(Tensor q, Tensor k, Tensor v, bool causal, c10::optional<Tensor> kv_lens,
                              double scale) {
  const long D = q.size(-1);
  TORCH_CHECK(D == 64 || D == 128, "head dim must be 64 or 128");
  check_attn_operand(q, "q", D); check_attn_operand(k, "k", D); check_attn_operand(v, "v", D);
  const long B = q.size(0), Sq = q.size(1), Hq = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && v.size(1) == Sk && v.size(2) == Hkv, "k/v shape mismatch");
  TORCH_CHECK(Hkv > 0 && Hq % Hkv == 0, "Hq must be a multiple of Hkv");
  TORCH_CHECK(Sq > 0 && Sk > 0, "empty sequence");
  auto o = torch::empty({B, Sq, Hq, D}, q.options());
  const long ld = (Sq + 127) / 128 * 128;  // padded rows: the backward stages 64/128-query slices with 16-B copies
  auto lse = torch::empty({B, Hq, ld}, q.options().dtype(at::kFloat));
  k8s_amd::AttnFwdArgs a;
  a.q = cbf(q); a.k = cbf(k); a.v = cbf(v); a.o = bf(o); a.lse = f32(lse); a.kv_lens = kv_lens_ptr(kv_lens, B);
  a.sqb = q.stride(0); a.sqs = q.stride(1); a.sqh = q.stride(2);
  a.skb = k.stride(0); a.sks = k.stride(1); a.skh = k.stride(2);
  a.svb = v.stride(0); a.svs = v.stride(1); a.svh = v.stride(2);
  a.sob = o.stride(0); a.sos = o.stride(1); a.soh = o.stride(2);
  a.lse_ld = ld;
  a.B = B; a.Sq = Sq; a.Sk = Sk; a.Hq = Hq; a.Hkv = Hkv; a.causal = causal;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  k8s_amd::launch_flash_fwd(a, (int)D, cur_stream());
  return {o, lse};
}

// dq / dk / dv are new contiguous tensors, or -- with `dqkv` given -- views into that [B*S, (Hq + 2*Hkv) * D]
// buffer laid out like the packed QKV projection q / k / v were sliced from (q at column 0, k at Hq*D, v at
// (Hq + Hkv)*D): the fused projection's gradient is written in place, no concatenation afterwards.
std::vector<Tensor> flash_bwd(Tensor dO, Tensor q, Tensor k, Tensor v, Tensor o, Tensor lse, bool causal,
                              c10::optional<Tensor> kv_lens, double scale, c10::optional<Tensor> dqkv,
                              c10::optional<Tensor> dbias) {
  const long D = q.size(-1);
  TORCH_CHECK(D == 64 || D == 128, "head dim must be 64 or 128");
  check_attn_operand(q, "q", D); check_attn_operand(k, "k", D); check_attn_operand(v, "v", D);
  check_attn_operand(o, "o", D); check_attn_operand(dO, "dO", D);
  const long B = q.size(0), Sq = q.size(1), Hq = q.size(2), Sk = k.size(1), Hkv = k.size(2);
  TORCH_CHECK(dO.sizes() == q.sizes() && o.sizes() == q.sizes(), "dO / o must match q");
  TORCH_CHECK(Hq % Hkv == 0, "Hq must be a multiple of Hkv");
  check_cuda(lse, "lse"); check_dtype(lse, at::kFloat, "lse");
  const long ld = (Sq + 127) / 128 * 128;
  TORCH_CHECK(lse.dim() == 3 && lse.size(0) == B && lse.size(1) == Hq && lse.size(2) == ld,
              "lse must be the [B, Hq, round_up(Sq, 128)] tensor flash_fwd returned");
  auto delta = torch::empty({B, Hq, ld}, q.options().dtype(at::kFloat));
  Tensor dq, dk, dv;
  if (dqkv) {
    TORCH_CHECK(Sq == Sk, "packed QKV gradient needs self-attention (Sq == Sk)");
    const long W = (Hq + 2 * Hkv) * D;
    check_cuda(*dqkv, "dqkv"); check_dtype(*dqkv, at::kBFloat16, "dqkv");
    TORCH_CHECK(dqkv->is_contiguous() && dqkv->numel() == B * Sq * W, "dqkv must be contiguous [B*S, (Hq+2*Hkv)*D]");
    auto g = dqkv->view({B, Sq, Hq + 2 * Hkv, D});
    dq = g.narrow(2, 0, Hq);
    dk = g.narrow(2, Hq, Hkv);
    dv = g.narrow(2, Hq + Hkv, Hkv);
  } else {
    dq = torch::empty({B, Sq, Hq, D}, q.options());
    dk = torch::empty({B, Sk, Hkv, D}, q.options());
    dv = torch::empty({B, Sk, Hkv, D}, q.options());
  }
  k8s_amd::AttnBwdArgs a;
  a.q = cbf(q); a.k = cbf(k); a.v = cbf(v); a.dO = cbf(dO); a.lse = f32(lse); a.delta = f32(delta);
  a.dq = bf(dq); a.dk = bf(dk); a.dv = bf(dv); a.kv_lens = kv_lens_ptr(kv_lens, B);
  a.lse_ld = ld;
  a.sqb = q.stride(0); a.sqs = q.stride(1); a.sqh = q.stride(2);
  a.skb = k.stride(0); a.sks = k.stride(1); a.skh = k.stride(2);
  a.svb = v.stride(0); a.svs = v.stride(1); a.svh = v.stride(2);
  a.sdb = dO.stride(0); a.sds = dO.stride(1); a.sdh = dO.stride(2);
  a.sgqb = dq.stride(0); a.sgqs = dq.stride(1); a.sgqh = dq.stride(2);
  a.sgkb = dk.stride(0); a.sgks = dk.stride(1); a.sgkh = dk.stride(2);
  a.sgvb = dv.stride(0); a.sgvs = dv.stride(1); a.sgvh = dv.stride(2);
  TORCH_CHECK(dq.stride(3) == 1 && dk.stride(3) == 1 && dv.stride(3) == 1, "gradient rows must be contiguous");
  a.B = B; a.Sq = Sq; a.Sk = Sk; a.Hq = Hq; a.Hkv = Hkv; a.causal = causal;
  a.scale_log2 = (float)(scale * 1.4426950408889634);
  a.scale = (float)scale;
  a.dkv_split = k8s_amd::flash_dkv_splits((int)B, (int)Sq, (int)Sk, (int)Hkv, causal);
  Tensor dkv_ws;
  if (a.dkv_split > 1) {
    dkv_ws = torch::empty({a.dkv_split, 2, B, Hkv, Sk, D}, q.options().dtype(at::kFloat));
    a.dkv_ws = f32(dkv_ws);
  }
  Tensor cpart;
  if (dbias) {  // the packed projection's bias gradient from the one-block kernel's column partials
    const long W = (Hq + 2 * Hkv) * D;
    TORCH_CHECK(dqkv && k8s_amd::flash_bwd_one_block((int)D, (int)Sq, (int)Sk, (int)Hq, (int)Hkv, a.dkv_split),
                "dbias needs the packed gradient and a one-block shape (flash_bwd_one_block)");
    check_cuda(*dbias, "dbias"); check_dtype(*dbias, at::kFloat, "dbias");
    TORCH_CHECK(dbias->is_contiguous() && dbias->numel() == W, "dbias must be fp32 [(Hq+2*Hkv)*D]");
    cpart = torch::empty({B, W}, q.options().dtype(at::kFloat));
    a.cpart = f32(cpart);
    a.cpart_ld = (int)W;
  }
  k8s_amd::launch_flash_bwd(a, (int)D, cbf(o), o.stride(0), o.stride(1), o.stride(2), cur_stream());
  if (dbias) k8s_amd::launch_colsum_fold(a.cpart, (int)B, a.cpart_ld, f32(*dbias), false, cur_stream());
  return {dq, dk, dv};
}

// ------------------------------------------------------------------ max pooling (NHWC)
std::vector<Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t s, int64_t p) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "x must be NHWC with C % 8 == 0");
  TORCH_CHECK(k <= 15 && p < k, "window too large");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int Ho = (H + 2 * p - k) / s + 1, Wo = (W + 2 * p - k) / s + 1;
  auto y = torch::empty({N, Ho, Wo, C}, x.options());
  auto idx = torch::empty({N, Ho, Wo, C}, x.options().dtype(at::kByte));
  k8s_amd::launch_maxpool_fwd(cbf(x), bf(y), idx.data_ptr<uint8_t>(), N, H, W, C, Ho, Wo, (int)k, (int)s, (int)p,
                              cur_stream());
  return {y, idx};
}

Tensor maxpool_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t p) {
  check_cuda(dy, "dy"); check_dtype(dy, at::kBFloat16, "dy");
  check_cuda(idx, "idx"); check_dtype(idx, at::kByte, "idx");
  TORCH_CHECK(dy.sizes() == idx.sizes() && dy.dim() == 4 && dy.size(3) % 8 == 0, "dy / idx mismatch");
  const int N = dy.size(0), Ho = dy.size(1), Wo = dy.size(2), C = dy.size(3);
  TORCH_CHECK(Ho == (H + 2 * p - k) / s + 1 && Wo == (W + 2 * p - k) / s + 1, "input size mismatch");
  auto dx = torch::empty({N, H, W, C}, dy.options());
  k8s_amd::launch_maxpool_bwd(cbf(dy), idx.data_ptr<uint8_t>(), bf(dx), N, (int)H, (int)W, C, Ho, Wo, (int)k,
                              (int)s, (int)p, cur_stream());
  return dx;
}

// ------------------------------------------------------------------ embedding (sum of gathers) / avg pool
// tables: list of (weight bf16 [V, D], ids int64 [T] or None = position table) ; returns bf16 [T, D]
Tensor embed_fwd(std::vector<Tensor> weights, std::vector<c10::optional<Tensor>> ids, int64_t T, int64_t S) {
  TORCH_CHECK(!weights.empty() && weights.size() <= 3 && weights.size() == ids.size(), "1-3 tables, one ids each");
  const long D = weights[0].size(1);
  k8s_amd::EmbTable tabs[3];
  for (size_t i = 0; i < weights.size(); ++i) {
    const Tensor& w = weights[i];
    check_cuda(w, "weight"); check_dtype(w, at::kBFloat16, "weight");
    TORCH_CHECK(w.dim() == 2 && w.size(1) == D && D % 8 == 0, "tables must be [V, D] with one D % 8 == 0");
    const int64_t* ip = nullptr;
    if (ids[i]) {
      check_cuda(*ids[i], "ids"); check_dtype(*ids[i], at::kLong, "ids");
      TORCH_CHECK(ids[i]->numel() == T, "ids must have T entries");
      ip = ids[i]->data_ptr<int64_t>();
    } else {
      TORCH_CHECK(S > 0 && T % S == 0 && w.size(0) >= S, "position table needs T % S == 0 and >= S rows");
    }
    tabs[i] = k8s_amd::EmbTable{cbf(w), nullptr, ip, (int)w.size(0)};
  }
  auto out = torch::empty({T, D}, weights[0].options());
  k8s_amd::launch_embed_fwd(tabs, (int)weights.size(), (int)T, (int)D, (int)S, bf(out), cur_stream());
  return out;
}

// grads: fp32 [V, D] slots accumulated into (zero them first for a fresh gradient)
void embed_bwd(Tensor g, std::vector<Tensor> grads, std::vector<c10::optional<Tensor>> ids, int64_t S) {
  check_cuda(g, "g"); check_dtype(g, at::kBFloat16, "g");
  TORCH_CHECK(!grads.empty() && grads.size() <= 3 && grads.size() == ids.size(), "1-3 tables, one ids each");
  const long T = g.size(0), D = g.size(1);
  k8s_amd::EmbTable tabs[3];
  for (size_t i = 0; i < grads.size(); ++i) {
    const Tensor& gr = grads[i];
    check_cuda(gr, "grad"); check_dtype(gr, at::kFloat, "grad");
    TORCH_CHECK(gr.dim() == 2 && gr.size(1) == D, "grad slots must be [V, D]");
    const int64_t* ip = nullptr;
    if (ids[i]) {
      check_cuda(*ids[i], "ids"); check_dtype(*ids[i], at::kLong, "ids");
      TORCH_CHECK(ids[i]->numel() == T);
      ip = ids[i]->data_ptr<int64_t>();
    } else {
      TORCH_CHECK(S > 0 && T % S == 0 && gr.size(0) >= S, "position table needs T % S == 0");
    }
    tabs[i] = k8s_amd::EmbTable{nullptr, f32(gr), ip, (int)gr.size(0)};
  }
  k8s_amd::launch_embed_bwd(tabs, (int)grads.size(), (int)T, (int)D, (int)S, cbf(g), cur_stream());
}

// ------------------------------------------------------------------ space-to-depth stem
// y[n][i][j] = x[n][s i][s j]: the input of a 1x1 / stride-s / pad-0 convolution as a contiguous tensor
Tensor subsample_nhwc(Tensor x, int64_t s) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.size(3) % 8 == 0 && s >= 1, "x: contiguous NHWC, C % 8 == 0");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  auto y = torch::empty({N, (H + s - 1) / s, (W + s - 1) / s, C}, x.options());
  k8s_amd::launch_subsample_nhwc(cbf(x), bf(y), N, H, W, C, (int)s, cur_stream());
  return y;
}

Tensor stem_s2d_input(Tensor x, int64_t pad) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) <= 8, "x must be NHWC with <= 8 channels");
  const int N = x.size(0), H = x.size(1), W = x.size(2);
  auto out = torch::empty({N, (H + 2 * pad) / 2, (W + 2 * pad) / 2, 16}, x.options());
  k8s_amd::launch_stem_s2d_input(cbf(x), N, H, W, (int)x.size(3), (int)pad, bf(out), cur_stream());
  return out;
}
Tensor stem_w_s2d(Tensor w7) {
  check_cuda(w7, "w7"); check_dtype(w7, at::kBFloat16, "w7");
  TORCH_CHECK(w7.dim() == 4 && w7.size(1) == w7.size(2), "w7 must be [K, R, R, C]");
  const int K = w7.size(0), R = w7.size(1), Rs = (R + 1) / 2;
  auto w4 = torch::empty({K, Rs, Rs, 16}, w7.options());
  k8s_amd::launch_stem_w_s2d(cbf(w7), K, R, (int)w7.size(3), bf(w4), cur_stream());
  return w4;
}
// the s2d stem convolution on its LDS-tiled kernel (stem.hip): y [N, Hs-3, Ws-3, 64] + BN statistics into `stats`
Tensor stem_conv_fwd(Tensor xs, Tensor w4, Tensor stats) {
  check_cuda(xs, "xs"); check_dtype(xs, at::kBFloat16, "xs"); check_dtype(w4, at::kBFloat16, "w4");
  TORCH_CHECK(xs.dim() == 4 && xs.size(3) == 16 && xs.is_contiguous(), "xs must be a contiguous [N, Hs, Ws, 16] image");
  TORCH_CHECK(w4.dim() == 4 && w4.is_contiguous() && k8s_amd::stem_conv_fwd_ok((int)w4.size(0), (int)w4.size(1),
              (int)w4.size(3), (int)xs.size(2) - 3) && w4.size(2) == 4, "stem conv: w4 [64, 4, 4, 16], Wo % 16 == 0");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.is_contiguous() &&
              stats.numel() == (long)k8s_amd::kConvStatReplicas * 2 * 64, "stats must be zeroed fp32 [R, 2, 64]");
  const int N = xs.size(0), Hs = xs.size(1), Ws = xs.size(2);
  auto y = torch::empty({N, Hs - 3, Ws - 3, 64}, xs.options());
  k8s_amd::launch_stem_conv_fwd(cbf(xs), cbf(w4), bf(y), f32(stats), N, Hs, Ws, cur_stream());
  return y;
}

// the s2d stem weight gradient (stem.hip): dw4 fp32 [64, 4, 4, 16] from the image xs and the output gradient dy
void stem_wgrad(Tensor xs, Tensor dy, Tensor dw4) {
  check_cuda(xs, "xs"); check_dtype(xs, at::kBFloat16, "xs"); check_dtype(dy, at::kBFloat16, "dy");
  TORCH_CHECK(xs.dim() == 4 && xs.size(3) == 16 && xs.is_contiguous() && dy.is_contiguous(), "xs [N, Hs, Ws, 16]");
  const int N = xs.size(0), Hs = xs.size(1), Ws = xs.size(2);
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == Hs - 3 && dy.size(2) == Ws - 3 && dy.size(3) == 64 &&
              k8s_amd::stem_conv_fwd_ok(64, 4, 16, Ws - 3), "dy [N, Hs-3, Ws-3, 64], Wo % 16 == 0");
  TORCH_CHECK(dw4.is_cuda() && dw4.scalar_type() == at::kFloat && dw4.is_contiguous() && dw4.numel() == 64 * 256);
  auto ws = torch::empty({(long)k8s_amd::stem_wgrad_blocks(N, Hs) * 64 * 256}, dw4.options());
  k8s_amd::launch_stem_wgrad(cbf(xs), cbf(dy), f32(ws), f32(dw4), N, Hs, Ws, cur_stream());
}

void stem_dw_s2d(Tensor dw4, Tensor dw7) {
  check_cuda(dw4, "dw4"); check_cuda(dw7, "dw7");
  check_dtype(dw4, at::kFloat, "dw4"); check_dtype(dw7, at::kFloat, "dw7");
  const int K = dw7.size(0), R = dw7.size(1), Rs = (R + 1) / 2;
  TORCH_CHECK(dw4.numel() == (long)K * Rs * Rs * 16, "dw4 must be [K, Rs, Rs, 16]");
  k8s_amd::launch_stem_dw_s2d(f32(dw4), K, R, (int)dw7.size(3), f32(dw7), cur_stream());
}

Tensor avgpool_fwd(Tensor x) {
  check_cuda(x, "x"); check_dtype(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "x must be NHWC with C % 8 == 0");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto y = torch::empty({N, C}, x.options());
  k8s_amd::launch_avgpool_fwd(cbf(x), bf(y), N, HW, C, cur_stream());
  return y;
}

Tensor avgpool_bwd(Tensor dy, int64_t H, int64_t W) {
  check_cuda(dy, "dy"); check_dtype(dy, at::kBFloat16, "dy");
  TORCH_CHECK(dy.dim() == 2 && dy.size(1) % 8 == 0, "dy must be [N, C] with C % 8 == 0");
  const int N = dy.size(0), C = dy.size(1);
  auto dx = torch::empty({N, H, W, C}, dy.options());
  k8s_amd::launch_avgpool_bwd(cbf(dy), bf(dx), N, (int)(H * W), C, cur_stream());
  return dx;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "k8s_amd gfx950 (MI355X) HIP kernels";
  m.def("fused_sgd", &fused_sgd, py::arg("p"), py::arg("mom"), py::arg("g"), py::arg("pbf"), py::arg("decay_mask"),
        py::arg("lr"), py::arg("mu"), py::arg("wd"), py::arg("scale"), py::arg("scale_t"), py::arg("nesterov"),
        py::arg("first_step"), py::arg("hyper") = py::none());
  m.def("fused_adam", &fused_adam, py::arg("p"), py::arg("m1"), py::arg("m2"), py::arg("g"), py::arg("pbf"),
        py::arg("decay_mask"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"),
        py::arg("scale"), py::arg("scale_t"), py::arg("step"), py::arg("decoupled"), py::arg("hyper") = py::none());
  m.def("grad_sumsq", &grad_sumsq);
  m.def("clip_factor", &clip_factor);
  m.def("slice_sum", &slice_sum, py::arg("recv"), py::arg("world"), py::arg("out") = py::none(),
        py::arg("out_bf") = py::none(), "fp32 rank-order sum of an all-to-all's bf16 chunks");
  m.def("cast_bf16", &cast_bf16, py::arg("x"), py::arg("out") = py::none());
  m.def("bn_fwd", &bn_fwd, py::arg("x"), py::arg("res"), py::arg("gamma"), py::arg("beta"), py::arg("run_mean"),
        py::arg("run_var"), py::arg("training"), py::arg("momentum"), py::arg("eps"), py::arg("relu"),
        py::arg("want_mask") = false);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("mean"), py::arg("invstd"),
        py::arg("gamma"), py::arg("beta"), py::arg("relu_x"), py::arg("dgamma"), py::arg("dbeta"), py::arg("want_dres"),
        py::arg("mask") = py::none());
  m.def("bn_fwd_from_sums", &bn_fwd_from_sums, py::arg("x"), py::arg("res"), py::arg("gamma"), py::arg("beta"),
        py::arg("sums"), py::arg("run_mean"), py::arg("run_var"), py::arg("momentum"), py::arg("eps"),
        py::arg("relu"), py::arg("want_mask") = false, py::arg("want_sub2") = false);
  m.def("norm_fwd", &norm_fwd);
  m.def("norm_bwd", &norm_bwd, py::arg("dy"), py::arg("x"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("dres"), py::arg("dgamma"), py::arg("dbeta"), py::arg("rms"), py::arg("dsum") = py::none());
  m.def("xent_fwd", &xent_fwd);
  m.def("xent_bwd", &xent_bwd);
  m.def("wgrad_stream_eligible", &k8s_amd::wgrad_stream_eligible, "tall-K weight-gradient kernel takes this shape");
  m.def("gemm", &gemm, py::arg("a"), py::arg("a_kmajor"), py::arg("b"), py::arg("b_kmajor"), py::arg("out"),
        py::arg("out_f32"), py::arg("bias"), py::arg("act"), py::arg("pre"), py::arg("accumulate"), py::arg("alpha"),
        py::arg("splits"),
        py::arg("add_src") = py::none(), py::arg("add_mask") = py::none(), py::arg("xform_b") = py::none(),
        py::arg("xform_c") = 0);
  m.def("bn_bwd_dual", &bn_bwd_dual, "both BatchNorm backwards of bn_fwd_from_sums_dual from one masked dy");
  m.def("bn_fwd_from_sums_dual", &bn_fwd_from_sums_dual, "relu(BN(x) + BN_r(xr)), statistics from conv sums");
  m.def("bn_finalize", &bn_finalize, py::arg("sums"), py::arg("gamma"), py::arg("beta"), py::arg("run_mean"),
        py::arg("run_var"), py::arg("count"), py::arg("momentum"), py::arg("eps"));
  m.def("dgrad_short_bnstats", &dgrad_short_bnstats, py::arg("gy"), py::arg("w"), py::arg("add_src"),
        py::arg("add_mask"), py::arg("x"), py::arg("mask"), py::arg("mean"), py::arg("sums"),
        py::arg("x2") = py::none(), py::arg("mean2") = py::none(), py::arg("sums2") = py::none(),
        "1x1 masked-addend data gradient with the BatchNorm-backward statistics of its result (gemm_short EPI 3/4)");
  m.def("gemm_short_bnstats_ok", [](int64_t M, int64_t N, int64_t K, bool dual) {
    return M < (1L << 31) && k8s_amd::gemm_short_bnstats_ok((int)M, (int)N, (int)K, dual);
  });
  m.def("conv3x3_dgrad_bnstats", &conv3x3_dgrad_bnstats,
        "3x3 stride-1 data gradient with the BatchNorm-backward sums of a relu(BN(x)) input (conv3x3.hip)");
  m.def("gemm_dgrad_bnstats", &gemm_dgrad_bnstats,
        "1x1 data gradient with the BatchNorm-backward sums of a relu(BN(x)) input (gemm.hip BST epilogue)");
  m.def("gemm_dgrad_bnstats_ok", [](int64_t M, int64_t N, int64_t K) {
    const char* e = std::getenv("K8S_AMD_BN_BSTATS");
    if (e && e[0] == '0') return false;
    if (M >= (1L << 31) || N % 8 != 0) return false;
    if (use_gemm256(M, N, K, true, false)) {
      const char* g = std::getenv("K8S_AMD_BN_BSTATS_W4");
      return !(g && g[0] == '0') && k8s_amd::gemm_w4_dgrad_bnstats_ok((int)M, (int)N, (int)K);
    }
    return !k8s_amd::gemm_short_ok((int)M, (int)N, (int)K, K, N);
  }, "whether a 1x1 data gradient takes gemm_dgrad_bnstats (on its regular kernel: the 4-wave or the tile kernel)");
  m.def("bn_bwd_relu_from_sums", &bn_bwd_relu_from_sums, "relu_x BatchNorm backward from a producer's sums");
  m.def("bn_bwd_from_sums", &bn_bwd_from_sums, "BatchNorm backward from a producer's reduction sums (final + apply)");
  m.def("bn_bwd_dual_from_sums", &bn_bwd_dual_from_sums, "bn_bwd_dual from a producer's reduction sums");
  m.def("mask_apply", &mask_apply, "out = bit ? src : 0 (packed 1-bit mask per element)");
  m.def("swiglu_fwd", &swiglu_fwd, py::arg("gu"), py::arg("blk") = 0);
  m.def("swiglu_bwd", &swiglu_bwd, py::arg("gu"), py::arg("dy"), py::arg("blk") = 0);
  m.def("rope_", &rope_);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("act_bwd_colsum", &act_bwd_colsum, py::arg("dy"), py::arg("pre"), py::arg("act"),
        py::arg("out") = py::none());
  m.def("relu_bwd", &relu_bwd);
  m.def("colsum", &colsum, py::arg("x"), py::arg("out") = py::none());
  m.def("gemm_dact", &gemm_dact, "linear data gradient fused with the input activation's backward and bias gradient",
        py::arg("g"), py::arg("w"), py::arg("pre"), py::arg("act"), py::arg("db"), py::arg("db_accumulate"));
  m.def("gemm_dact_ok", &gemm_dact_ok, py::arg("M"), py::arg("N"), py::arg("K"));
  m.def("gemm_swiglu_bwd", &gemm_swiglu_bwd, "down-projection data gradient fused with the SwiGLU backward (dgu)",
        py::arg("g"), py::arg("w"), py::arg("gu"), py::arg("blk") = 0);
  m.def("gemm_swiglu_fwd", &gemm_swiglu_fwd, "gate|up projection with the SwiGLU in the epilogue: (gu, h)");
  m.def("gemm_swiglu_fwd_ok", &gemm_swiglu_fwd_ok, py::arg("M"), py::arg("F"), py::arg("K"));
  m.def("gemm_rope", &gemm_rope, "QKV projection with the q / k rotary embedding in the epilogue");
  m.def("gemm_rope_ok", &gemm_rope_ok, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("rot_cols"));
  m.def("gemm_swiglu_bwd_ok", &gemm_swiglu_bwd_ok, py::arg("M"), py::arg("F"), py::arg("K"));
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("stride"), py::arg("pad"), py::arg("dil"),
        py::arg("out_f32"), py::arg("bias"), py::arg("act"), py::arg("stats"),
        py::arg("xform") = py::none());
  m.def("conv3x3_staged_ok", [](int H, int W, int C, int K, int R, int S, int stride, int pad) {
    // the staged-window forward / data gradient (conv3x3.hip) and the tiled weight gradient (wgrad_tile.hip) both
    // take this layer: BatchNorm + ReLU can be normalised on load in all three products
    return k8s_amd::conv3x3_eligible(H, W, C, K, R, S, stride, pad, 1) &&
           k8s_amd::conv3x3_eligible(H, W, K, C, R, S, stride, pad, 1) &&
           k8s_amd::wgrad3x3_tiled_ok(C, K, R, S, stride, pad, W);
  });
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("stride"), py::arg("pad"),
        py::arg("dil"), py::arg("splits"), py::arg("accumulate"), py::arg("xform") = py::none());
  m.def("conv_fwd_subgrid", &conv_fwd_subgrid, py::arg("x"), py::arg("w"), py::arg("pad"), py::arg("Hs"),
        py::arg("Ws"), py::arg("out"), py::arg("stride"), py::arg("a"), py::arg("b"), py::arg("accumulate") = false,
        py::arg("bn_x") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bn_mean") = py::none(),
        py::arg("bn_sums") = py::none(), py::arg("bn_gamma") = py::none(), py::arg("bn_beta") = py::none(),
        py::arg("bn_invstd") = py::none());
  m.def("conv_dgrad_wtrans", &conv_dgrad_wtrans);
  m.def("conv_dgrad_wsub", &conv_dgrad_wsub);
  m.def("flash_fwd", &flash_fwd);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("bn_relu_maxpool", &bn_relu_maxpool, py::arg("x"), py::arg("sums"), py::arg("gamma"), py::arg("beta"),
        py::arg("run_mean"), py::arg("run_var"), py::arg("momentum"), py::arg("eps"), py::arg("want_link") = false);
  m.def("pool_bn_bwd_from_sums", &pool_bn_bwd_from_sums);
  m.def("gemm_dgrad_bnstats_mask", &gemm_dgrad_bnstats_mask, py::arg("gy"), py::arg("w"), py::arg("out"), py::arg("x"),
        py::arg("mask"), py::arg("mean"), py::arg("sums"), py::arg("add_src") = py::none(),
        py::arg("add_mask") = py::none(), py::arg("x2") = py::none(), py::arg("mean2") = py::none(),
        py::arg("sums2") = py::none());
  m.def("pool_bn_bwd", &pool_bn_bwd, py::arg("dpool"), py::arg("idx"), py::arg("x"), py::arg("mean"),
        py::arg("invstd"), py::arg("gamma"), py::arg("beta"), py::arg("dgamma"), py::arg("dbeta"));
  m.def("embed_fwd", &embed_fwd);
  m.def("embed_bwd", &embed_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("stem_s2d_input", &stem_s2d_input);
  m.def("subsample_nhwc", &subsample_nhwc, py::arg("x"), py::arg("s"));
  m.def("stem_w_s2d", &stem_w_s2d);
  m.def("stem_conv_fwd", &stem_conv_fwd);
  m.def("stem_wgrad", &stem_wgrad);
  m.def("stem_dw_s2d", &stem_dw_s2d);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("flash_bwd", &flash_bwd, py::arg("dO"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("causal"), py::arg("kv_lens"), py::arg("scale"), py::arg("dqkv") = py::none(),
        py::arg("dbias") = py::none());
  m.def("flash_bwd_one_block", [](int64_t D, int64_t Sq, int64_t Sk, int64_t Hq, int64_t Hkv, bool causal, int64_t B) {
          return k8s_amd::flash_bwd_one_block((int)D, (int)Sq, (int)Sk, (int)Hq, (int)Hkv,
                                              k8s_amd::flash_dkv_splits((int)B, (int)Sq, (int)Sk, (int)Hkv, causal));
        }, "whether flash_bwd runs as the one-block short-sequence kernel (which can also emit the packed bias gradient)");
  m.attr("conv_stat_replicas") = k8s_amd::kConvStatReplicas;
  m.def("gemm_short_ok", [](int64_t M, int64_t N, int64_t K) { return k8s_amd::gemm_short_ok((int)M, (int)N, (int)K, K, N); },
        "whether C[M,N] = A[M,K] . B^T (contiguous) takes the short-K streaming kernel (gemm_short.hip)");
  m.def("planner_cus", &k8s_amd::planner_cus,
        "CUs the launch planners size grids for (the device's multiprocessor count unless overridden)");
  m.def("set_planner_cus", &k8s_amd::set_planner_cus, py::arg("n"),
        "override the planners' CU budget for every device (n <= 0: back to the device's count)");
  m.attr("arch") = "gfx950";
}
