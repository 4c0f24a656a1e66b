"""Plain-PyTorch fp32 reference implementations of every fused kernel.

These are (a) the numerics oracles the GPU tests compare the HIP kernels
against and (b) the CPU execution path used by the CPU-only test tier and by
CPU rehearsals of the distributed code (gloo). They are written from the
mathematical definitions, in fp32, with no fusion.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch


# --------------------------------------------------------------------------- batchnorm (NHWC)
def bn_fwd(x, res, gamma, beta, run_mean, run_var, training, momentum, eps, relu):
    C = x.shape[-1]
    xf = x.float().reshape(-1, C)
    if training:
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        if run_mean is not None:
            n = xf.shape[0]
            unb = var * n / max(n - 1, 1)
            run_mean.mul_(1 - momentum).add_(momentum * mean)
            run_var.mul_(1 - momentum).add_(momentum * unb)
    else:
        mean, var = run_mean.float(), run_var.float()
    invstd = torch.rsqrt(var + eps)
    y = (xf - mean) * invstd * gamma.float() + beta.float()
    if res is not None:
        y = y + res.float().reshape(-1, C)
    if relu:
        y = torch.relu(y)
    return y.reshape(x.shape).to(x.dtype), mean, invstd


def bn_bwd(dy, x, y, mean, invstd, gamma):
    C = x.shape[-1]
    g = dy.float().reshape(-1, C)
    if y is not None:
        g = g * (y.float().reshape(-1, C) > 0)
    xh = (x.float().reshape(-1, C) - mean) * invstd
    M = g.shape[0]
    sd = g.sum(0)
    sx = (g * xh).sum(0)
    dx = gamma.float() * invstd * (g - sd / M - xh * sx / M)
    return dx.reshape(x.shape).to(x.dtype), g.reshape(x.shape).to(x.dtype), sx, sd


# --------------------------------------------------------------------------- layernorm / rmsnorm
def norm_fwd(x, res, gamma, beta, eps, rms):
    xs = x.float() if res is None else x.float() + res.float()
    if rms:
        mean = torch.zeros(1)
        rstd = torch.rsqrt(xs.pow(2).mean(-1) + eps)
        y = xs * rstd.unsqueeze(-1) * gamma.float()
    else:
        mean = xs.mean(-1)
        var = (xs - mean.unsqueeze(-1)).pow(2).mean(-1)
        rstd = torch.rsqrt(var + eps)
        y = (xs - mean.unsqueeze(-1)) * rstd.unsqueeze(-1) * gamma.float() + beta.float()
    xsum = xs.to(x.dtype) if res is not None else None
    return y.to(x.dtype), mean.reshape(-1), rstd.reshape(-1), xsum


def norm_bwd(dy, x, gamma, mean, rstd, dres, rms):
    D = x.shape[-1]
    g = dy.float().reshape(-1, D)
    xf = x.float().reshape(-1, D)
    r = rstd.reshape(-1, 1)
    mu = 0.0 if rms else mean.reshape(-1, 1)
    xh = (xf - mu) * r
    gg = g * gamma.float()
    a = gg.mean(-1, keepdim=True)
    b = (gg * xh).mean(-1, keepdim=True)
    dx = r * (gg - (0.0 if rms else a) - xh * b)
    if dres is not None:
        dx = dx + dres.float().reshape(-1, D)
    dgamma = (g * xh).sum(0)
    dbeta = g.sum(0)
    return dx.reshape(x.shape).to(x.dtype), dgamma, dbeta


# --------------------------------------------------------------------------- cross entropy
def xent_fwd(logits, labels, ignore_index=-100, smoothing=0.0):
    lf = logits.float()
    lse = torch.logsumexp(lf, -1)
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    picked = lf.gather(-1, safe.unsqueeze(-1)).squeeze(-1)
    loss = lse - picked
    if smoothing > 0:
        loss = (1 - smoothing) * loss + smoothing * (lse - lf.mean(-1))
    loss = torch.where(valid, loss, torch.zeros_like(loss))
    return loss, lse


def xent_bwd(logits, labels, lse, dscale, ignore_index=-100, smoothing=0.0):
    lf = logits.float()
    V = lf.shape[-1]
    p = torch.exp(lf - lse.unsqueeze(-1)) - smoothing / V
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    p.scatter_add_(-1, safe.unsqueeze(-1), torch.full_like(p[:, :1], -(1 - smoothing)))
    sc = dscale.float().reshape(-1)
    sc = sc.expand(lf.shape[0]) if sc.numel() == 1 else sc
    sc = torch.where(valid, sc, torch.zeros_like(sc))
    return (p * sc.unsqueeze(-1)).to(logits.dtype)


# --------------------------------------------------------------------------- optimizers
def _decay_vec(mask, n, wd, device):
    if mask is None:
        return torch.full((n,), wd, device=device)
    return mask.to(device).repeat_interleave(64)[:n].float() * wd


def _skipped(scale_t) -> bool:
    """A zero clip factor marks non-finite gradients: the step is skipped, all buffers untouched."""
    return scale_t is not None and float(scale_t.reshape(-1)[0]) == 0.0


def sgd(p, mom, g, pbf, mask, lr, mu, wd, scale, scale_t, nesterov, first_step):
    if _skipped(scale_t):
        return
    s = scale * (float(scale_t.reshape(-1)[0]) if scale_t is not None else 1.0)
    d = g.float() * s + _decay_vec(mask, p.numel(), wd, p.device) * p
    m = d.clone() if first_step else mom * mu + d
    mom.copy_(m)
    p.sub_(lr * (d + mu * m if nesterov else m))
    if pbf is not None:
        pbf.copy_(p)


def adam(p, m1, m2, g, pbf, mask, lr, b1, b2, eps, wd, scale, scale_t, step, decoupled):
    if _skipped(scale_t):
        return
    s = scale * (float(scale_t.reshape(-1)[0]) if scale_t is not None else 1.0)
    w = _decay_vec(mask, p.numel(), wd, p.device)
    gr = g.float() * s
    if not decoupled:
        gr = gr + w * p
    m1.mul_(b1).add_((1 - b1) * gr)
    m2.mul_(b2).add_((1 - b2) * gr * gr)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    upd = (lr / bc1) * m1 / (m2.sqrt() / math.sqrt(bc2) + eps)
    if decoupled:
        p.sub_(lr * w * p)
    p.sub_(upd)
    if pbf is not None:
        pbf.copy_(p)


def grad_sumsq(g):
    gf = g.float()
    return torch.stack([(gf * gf).sum(), (~torch.isfinite(gf)).sum().float()])
