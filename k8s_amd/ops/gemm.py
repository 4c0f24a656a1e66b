"""GEMM entry points (K1) used by linear layers.

``linear_fwd(x, w, b, act)`` computes ``act(x @ w^T + b)`` and
``linear_bwd`` the three backward products (dgrad NN, wgrad TN, bias
reduction). The gfx950 MFMA kernels (``csrc/kernels/gemm.hip``) serve GPU
tensors; CPU tensors use the fp32 reference.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _act_fwd(y, act):
    if act is None:
        return y
    if act == "relu":
        return torch.relu(y)
    if act == "gelu":
        return F.gelu(y, approximate="tanh")
    raise ValueError(act)


def _act_bwd(gy, pre, act):
    if act is None:
        return gy
    if act == "relu":
        return gy * (pre > 0)
    if act == "gelu":
        with torch.enable_grad():
            p = pre.detach().float().requires_grad_(True)
            (g,) = torch.autograd.grad(F.gelu(p, approximate="tanh"), p, gy.float())
        return g.to(gy.dtype)
    raise ValueError(act)


def linear_fwd(x, w, b, act=None):
    pre = torch.matmul(x, w.t())
    if b is not None:
        pre = pre + b.to(pre.dtype)
    y = _act_fwd(pre, act)
    return y, (pre if act is not None else None)


def linear_bwd(gy, x, w, pre, act, has_bias):
    g = _act_bwd(gy, pre, act)
    dx = torch.matmul(g, w)
    dw = torch.matmul(g.t(), x)
    db = g.float().sum(0) if has_bias else None
    return dx, dw, db
