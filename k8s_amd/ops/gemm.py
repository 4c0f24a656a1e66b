"""GEMM entry points (K1) for linear layers, on the gfx950 MFMA kernels.

``mm(a, b, a_kmajor, b_kmajor, ...)`` is the raw kernel (bf16 in, fp32 acc,
bf16/fp32 out, bias / ReLU / GELU epilogue, fp32 accumulate, split-K).
``linear_fwd`` / ``linear_bwd`` express a Linear layer's three products with
it WITHOUT materialising any transpose:

    fwd    y  = x . W^T          A = x   [M,K] K-major,  B = W [N,K] K-major
    dgrad  dx = g . W            A = g   [M,N] K-major,  B = W [N,K] read N-major
    wgrad  dW = g^T . x          A = g   read M-major,   B = x read N-major  (fp32 out straight into the
                                                             flat gradient slot, accumulated for tied weights)

Every product runs on our kernels: the 256 x 256 LDS-ring kernel (csrc/kernels/gemm256.hip) when the output
fills the chip, else the 128 x 128 kernel (gemm.hip); the choice is a wave-quantisation cost model in C++
(``gemm256_eligible``), not a timing race against a vendor library. CPU tensors use plain PyTorch; GPU shapes
the kernels do not take (K not a multiple of 8, N not a multiple of 4) go through PyTorch too and are counted in
``FALLBACKS`` (reported by the trainer), never silently; M and the K tail are masked in-kernel.
"""
from __future__ import annotations

import warnings
from typing import Dict

import torch
import torch.nn.functional as F

from k8s_amd.ops._ext import load as _load

ACT = {None: 0, "relu": 1, "gelu": 2}
FALLBACKS: Dict[str, int] = {}


def _fallback(key: str):
    if key not in FALLBACKS:
        warnings.warn("k8s_amd GEMM: %s is outside the MFMA kernels' shape contract; using PyTorch" % key)
    FALLBACKS[key] = FALLBACKS.get(key, 0) + 1


def hip_ok(*ts) -> bool:
    return all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


def mm(a, b, a_kmajor=True, b_kmajor=True, out=None, out_f32=False, bias=None, act=None, pre=None,
       accumulate=False, alpha=1.0, splits=1):
    return _load().gemm(a, a_kmajor, b, b_kmajor, out, out_f32, bias, ACT[act], pre, accumulate, alpha, splits)


def _shape_ok(M, N, K) -> bool:
    """The kernels' contract for a Linear layer's products: any M (the row tails are masked in-kernel); the K-major
    reduction dims (K forward, N in the data gradient) and the MN-major extents (N and K in the weight gradient)
    in whole 16-B units -- K % 8 and N % 8 -- and N % 4 for the forward epilogue. A ragged N runs on zero-padded
    weight rows (forward: ``_hip_fwd``; backward: ``linear_bwd``), so only K % 8 is required."""
    return K % 8 == 0


def _act_fwd(y, act):
    if act is None:
        return y
    if act == "relu":
        return torch.relu(y)
    if act == "gelu":
        return F.gelu(y, approximate="tanh")
    raise ValueError(act)


def _act_bwd(gy, pre_or_out, act):
    if act is None:
        return gy
    if gy.is_cuda and gy.dtype == torch.bfloat16 and gy.numel() % 8 == 0 and act in ("relu", "gelu"):
        C = _load()
        g = gy.contiguous()
        return C.relu_bwd(g, pre_or_out.contiguous()) if act == "relu" else C.gelu_bwd(g, pre_or_out.contiguous())
    if act == "relu":
        return gy * (pre_or_out > 0)
    if act == "gelu":
        x = pre_or_out.float()
        k0, k1 = 0.7978845608028654, 0.044715
        t = torch.tanh(k0 * (x + k1 * x ** 3))
        d = 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)
        return (gy.float() * d).to(gy.dtype)
    raise ValueError(act)


def _hip_fwd(x, w, b, act):
    M, N = x.shape[0], w.shape[0]
    if N % 4:  # ragged N (e.g. a 10-class head): zero weight rows up to a 16-B unit, the padded columns cut off
        n8 = (N + 7) // 8 * 8
        y, saved = _hip_fwd(x, F.pad(w, (0, 0, 0, n8 - N)), None if b is None else F.pad(b, (0, n8 - N)), act)
        return y[:, :N].contiguous(), (None if saved is None else saved[:, :N].contiguous())
    pre = torch.empty((M, N), device=x.device, dtype=torch.bfloat16) if act == "gelu" else None
    y = mm(x, w, True, True, bias=b, act=act, pre=pre)
    return y, (pre if act == "gelu" else (y if act == "relu" else None))


def linear_fwd(x, w, b, act=None):
    """Returns (y, saved) where saved is what linear_bwd needs for the activation derivative."""
    M, K = x.shape
    N = w.shape[0]
    if hip_ok(x, w) and _shape_ok(M, N, K) and x.stride(1) == 1:
        return _hip_fwd(x, w, b, act)
    if x.is_cuda:
        _fallback("linear_fwd %dx%dx%d" % (M, N, K))
    y = torch.matmul(x, w.t())
    if b is not None:
        y = y + b.to(y.dtype)
    pre = y
    y = _act_fwd(y, act)
    return y, (pre if act == "gelu" else (y if act == "relu" else None))


def dact_ok(x, w, dx_addend=None, gy=None) -> bool:
    """Whether a linear's data gradient can take its input activation's backward in the GEMM epilogue (``linear_bwd``
    ``dx_act``): the 4-wave kernel's whole-tile shapes, GPU bf16 operands (x, w and the incoming gradient gy), no
    second gradient contribution to add."""
    M, K = x.shape
    N = w.shape[0]
    return (dx_addend is None and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and (gy is None or gy.dtype == torch.bfloat16) and N % 8 == 0 and bool(_load().gemm_dact_ok(M, K, N)))


def swiglu_ok(x, w, dx_addend=None, gy=None) -> bool:
    """Whether a linear whose input is a SwiGLU output can return the SwiGLU's input gradient (dgu) from its data
    gradient's epilogue (``linear_bwd`` ``dx_swiglu``): GPU bf16, the 4-wave kernel's whole-tile shapes."""
    M, F = x.shape
    K = w.shape[0]
    return (dx_addend is None and x.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and (gy is None or gy.dtype == torch.bfloat16) and K % 8 == 0 and bool(_load().gemm_swiglu_bwd_ok(M, F, K)))


def _dgrad_act(g, w, dx_act):
    """dx = (g . w) * act'(pre) with the producing linear's bias gradient (column sums of dx) deposited into its flat
    slot -- ``dx_act`` = (pre, act, pb, store) -- in one 4-wave GEMM launch (+ the column-sum fold)."""
    pre, act, pb, store = dx_act
    C = _load()
    slot = store.slot_for_write(pb)
    if slot is not None:
        dx = C.gemm_dact(g, w, pre.contiguous(), ACT[act], slot.view(-1), False)
        store.mark_written(pb)
    else:  # already written this step (tied bias): add the column sums onto it
        dx = C.gemm_dact(g, w, pre.contiguous(), ACT[act], pb.grad.view(-1), True)
        store._notify(pb)
    return dx


def linear_bwd(gy, x, w, saved, act, pw=None, store=None, need_db=True, dx_addend=None, pb=None, dx_act=None,
               dx_swiglu=None, swiglu_blk=0):
    """dx and the parameter gradient. With (pw, store) on GPU the weight gradient is written
    (or accumulated) straight into the flat fp32 gradient slot; returns (dx, dw_or_None, db).
    ``dx_addend`` (bf16, x's shape): another gradient contribution of x, accumulated in the dgrad epilogue (it is
    overwritten and returned as dx). With ``pb`` the bias gradient goes straight into its flat slot on first use
    (db is then returned as None). ``dx_act`` = (pre, act, producer bias param, its store): x is the output of that
    activation and dx is returned already through its backward, the producer's bias gradient deposited
    (``dact_ok`` must hold). ``dx_swiglu`` = gu: x = swiglu(gu), and the gradient of gu ([M, 2F]) is returned in
    dx's place (``swiglu_ok`` must hold).

    The two fused forms exist only on the whole-tile HIP branch: a call that asks for one and would take any other
    path (ragged N, the torch.matmul fallback) raises instead of returning a gradient WITHOUT the activation /
    SwiGLU backward applied (the caller marks the producer's backward as done on return)."""
    M, K = x.shape
    N = w.shape[0]
    db = None
    if (dx_act is not None or dx_swiglu is not None) and not (
            gy.dtype == torch.bfloat16 and hip_ok(gy, x, w) and _shape_ok(M, N, K) and N % 8 == 0):
        raise RuntimeError("linear_bwd: fused %s backward requested on a path without it (%dx%dx%d, gy %s)"
                           % ("activation" if dx_act is not None else "SwiGLU", M, N, K, gy.dtype))
    if (need_db and act in ("relu", "gelu") and gy.is_cuda and gy.dtype == torch.bfloat16 and N % 8 == 0
            and saved is not None and saved.dtype == torch.bfloat16):
        # activation backward and the bias gradient (its column sums) in one pass
        slot = store.slot_for_write(pb) if (pb is not None and store is not None) else None
        g, db = _load().act_bwd_colsum(gy.reshape(-1, N).contiguous(), saved.reshape(-1, N).contiguous(), ACT[act],
                                       slot)
        if slot is not None:
            store.mark_written(pb)
            db = None
        need_db = False
    else:
        g = _act_bwd(gy, saved, act)
    if not need_db:
        pass
    elif g.is_cuda and g.dtype == torch.bfloat16 and N % 8 == 0:
        slot = store.slot_for_write(pb) if (pb is not None and store is not None) else None
        db = _load().colsum(g.contiguous(), slot)
        if slot is not None:
            store.mark_written(pb)
            db = None
    else:
        db = g.float().sum(0)
    if hip_ok(g, x, w) and _shape_ok(M, N, K):
        g = g.contiguous()
        if N % 8:  # ragged N (e.g. 12 classes): zero-pad g's columns and w's rows to whole 16-B units
            n8 = (N + 7) // 8 * 8
            g = F.pad(g, (0, n8 - N))
            w = F.pad(w, (0, 0, 0, n8 - N))
            dx = mm(g, w, True, False)
            if dx_addend is not None:
                dx = dx + dx_addend.reshape(dx.shape).to(dx.dtype)
            dw = mm(g, x, False, False, out_f32=True, splits=0)[:N]
            if pw is not None and store is not None and pw.grad.dtype == torch.float32:
                store.deposit(pw, dw)
                return dx, None, db
            return dx, dw, db
        acc = dx_addend is not None and dx_addend.is_contiguous() and dx_addend.dtype == torch.bfloat16
        # dgrad reduces over N; a ragged N (e.g. the 1000-class head) is masked by the kernel's K tail (zeros)
        if dx_act is not None:
            dx = _dgrad_act(g, w, dx_act)
        elif dx_swiglu is not None:
            dx = _load().gemm_swiglu_bwd(g, w, dx_swiglu.contiguous(), swiglu_blk)
        else:
            dx = mm(g, w, True, False, out=dx_addend if acc else None, accumulate=acc)
        if dx_addend is not None and not acc:
            dx = dx + dx_addend
        if pw is not None and store is not None and pw.grad.dtype == torch.float32:
            acc = pw.written
            mm(g, x, False, False, out=pw.grad, out_f32=True, accumulate=acc, splits=0)
            if acc:
                store._notify(pw)
            else:
                store.mark_written(pw)
            return dx, None, db
        dw = mm(g, x, False, False, out_f32=True, splits=0)
        return dx, dw, db
    if g.is_cuda:
        _fallback("linear_bwd %dx%dx%d" % (M, N, K))
    dx = torch.matmul(g, w)
    if dx_addend is not None:
        dx = dx + dx_addend.reshape(dx.shape).to(dx.dtype)
    dw = torch.matmul(g.t(), x)
    return dx, dw, db
