"""Attention (K5) entry point.

``attention(q, k, v, causal, kv_lens)`` with token-major layouts:
q [B, S, Hq, D], k/v [B, S, Hkv, D] (GQA: Hq % Hkv == 0), bf16.

GPU: the gfx950 flash-attention kernels (``csrc/kernels/attention.hip``:
online-softmax forward writing the log-sum-exp, recompute backward with
dK/dV in registers and atomically accumulated dQ). q/k/v may be strided
views (e.g. column slices of the fused QKV projection) -- no copies. Head
dims other than 64/128 and CPU tensors use an explicit matmul/softmax
reference (no SDPA dispatch, so no Triton-built kernels run).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from k8s_amd.ops._ext import load as _load


def _flash_ok(q, k, v) -> bool:
    if not (q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128)):
        return False
    ok = all(t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:3]) and t.data_ptr() % 16 == 0
             for t in (q, k, v))
    return ok and hasattr(_load(), "flash_fwd")  # _load() raises if the extension is missing on a GPU box


def attention_reference(q, k, v, causal: bool, kv_lens: Optional[torch.Tensor] = None, scale: Optional[float] = None):
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    scale = scale or 1.0 / math.sqrt(D)
    qh = q.permute(0, 2, 1, 3).float()
    kh = k.permute(0, 2, 1, 3).float().repeat_interleave(rep, dim=1)
    vh = v.permute(0, 2, 1, 3).float().repeat_interleave(rep, dim=1)
    s = torch.matmul(qh, kh.transpose(-1, -2)) * scale
    Sk = k.shape[1]
    if causal:
        mask = torch.ones(S, Sk, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    if kv_lens is not None:
        keymask = torch.arange(Sk, device=q.device)[None, :] >= kv_lens[:, None].to(q.device)
        s = s.masked_fill(keymask[:, None, None, :], float("-inf"))
    p = torch.softmax(s, -1)
    o = torch.matmul(p, vh)
    return o.permute(0, 2, 1, 3).to(q.dtype)


class _Flash(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, kv_lens, scale):
        C = _load()
        if kv_lens is not None:
            kv_lens = kv_lens.to(device=q.device, dtype=torch.int32).contiguous()
        o, lse = C.flash_fwd(q, k, v, causal, kv_lens, scale)
        ctx.save_for_backward(q, k, v, o, lse, kv_lens if kv_lens is not None else torch.empty(0))
        ctx.causal, ctx.scale, ctx.has_lens = causal, scale, kv_lens is not None
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, lens = ctx.saved_tensors
        C = _load()
        dq, dk, dv = C.flash_bwd(do.contiguous(), q, k, v, o, lse, ctx.causal, lens if ctx.has_lens else None,
                                 ctx.scale)
        return dq, dk, dv, None, None, None


class _Reference(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, kv_lens, scale):
        ctx.save_for_backward(q, k, v)
        ctx.causal, ctx.kv_lens, ctx.scale = causal, kv_lens, scale
        with torch.no_grad():
            return attention_reference(q, k, v, causal, kv_lens, scale)

    @staticmethod
    def backward(ctx, do):
        q, k, v = ctx.saved_tensors
        with torch.enable_grad():
            qq, kk, vv = (t.detach().float().requires_grad_(True) for t in (q, k, v))
            o = attention_reference(qq, kk, vv, ctx.causal, ctx.kv_lens, ctx.scale)
            dq, dk, dv = torch.autograd.grad(o, (qq, kk, vv), do.float())
        return dq.to(q.dtype), dk.to(k.dtype), dv.to(v.dtype), None, None, None


def attention(q, k, v, causal: bool = False, kv_lens: Optional[torch.Tensor] = None, scale: Optional[float] = None):
    scale = scale or 1.0 / math.sqrt(q.shape[-1])
    if _flash_ok(q, k, v):
        return _Flash.apply(q, k, v, causal, kv_lens, scale)
    return _Reference.apply(q, k, v, causal, kv_lens, scale)


class _FlashQKV(torch.autograd.Function):
    """Self-attention straight off a fused QKV projection [T = B*S, (H + 2*Hkv)*D]: q / k / v are strided views,
    the optional rotary embedding rotates the q and k columns of one copy in place, and the backward writes the
    packed gradient in place (flash_bwd ``dqkv``) and un-rotates it in place -- no split / concatenation / rope
    copies on either pass."""

    @staticmethod
    def forward(ctx, qkv, B, S, H, Hkv, D, causal, kv_lens, scale, pos, table, bias_link=None, rope_in_place=False,
                rope_applied=False):
        C = _load()
        if kv_lens is not None:
            kv_lens = kv_lens.to(device=qkv.device, dtype=torch.int32).contiguous()
        x = qkv.contiguous()
        if pos is not None and not rope_applied:  # (applied: the projection's epilogue rotated q / k, ops.nn.linear_rope)
            if not rope_in_place:  # (in place: the caller's qkv is a temporary nothing else reads)
                x = x.clone() if x.data_ptr() == qkv.data_ptr() else x
            # (in place, the raw-pointer rotation does not bump autograd's version counter -- and cannot: qkv is
            # the view output of the projection's custom Function, where autograd forbids in-place modification
            # outright. Contract, see ``attention_qkv``: nothing else may hold the projection output.)
            C.rope_(x[:, : (H + Hkv) * D], pos, table, False)
        g = x.view(B, S, H + 2 * Hkv, D)
        q, k, v = g.narrow(2, 0, H), g.narrow(2, H, Hkv), g.narrow(2, H + Hkv, Hkv)
        o, lse = C.flash_fwd(q, k, v, causal, kv_lens, scale)
        ctx.save_for_backward(x, o, lse, kv_lens if kv_lens is not None else torch.empty(0),
                              pos if pos is not None else torch.empty(0), table if table is not None else torch.empty(0))
        ctx.meta = (B, S, H, Hkv, D, causal, scale, kv_lens is not None, pos is not None)
        ctx.bias_link = bias_link
        return o

    @staticmethod
    def backward(ctx, do):
        x, o, lse, lens, pos, table = ctx.saved_tensors
        B, S, H, Hkv, D, causal, scale, has_lens, has_rope = ctx.meta
        C = _load()
        g = x.view(B, S, H + 2 * Hkv, D)
        q, k, v = g.narrow(2, 0, H), g.narrow(2, H, Hkv), g.narrow(2, H + Hkv, Hkv)
        dqkv = torch.empty_like(x)
        # the projection's bias gradient (column sums of dqkv) from the one-block kernel (BiasLink); not with rope,
        # which rotates dqkv after the kernel
        bl, dsum, ss, lpb = ctx.bias_link, None, None, None
        if bl is not None and bl.pb is not None and not has_rope and \
                C.flash_bwd_one_block(D, S, S, H, Hkv, causal, B):
            lpb = bl.pb
            ss = lpb.store.slot_for_write(lpb)
            dsum = ss.view(lpb.shape) if ss is not None else torch.empty(lpb.shape, device=x.device,
                                                                         dtype=torch.float32)
        C.flash_bwd(do.contiguous(), q, k, v, o, lse, causal, lens if has_lens else None, scale, dqkv, dsum)
        if dsum is not None:
            lpb.store.mark_written(lpb) if ss is not None else lpb.store.deposit(lpb, dsum)
            bl.done = True
        if has_rope:
            C.rope_(dqkv[:, : (H + Hkv) * D], pos, table, True)
        return (dqkv,) + (None,) * 13


def attention_qkv(qkv, B: int, S: int, heads: int, kv_heads: int, head_dim: int, causal: bool = False,
                  kv_lens: Optional[torch.Tensor] = None, rope: Optional[tuple] = None,
                  scale: Optional[float] = None, bias_link=None, rope_in_place: bool = False,
                  rope_applied: bool = False):
    """Self-attention of a packed QKV projection ``qkv`` [B*S, (heads + 2*kv_heads) * head_dim] (q heads, then k,
    then v); ``rope`` = (pos [B*S] int32, table) applies rotary embeddings to q and k. Returns o [B, S, heads, D].
    GPU bf16: one fused path (``_FlashQKV``); otherwise the split + ``attention`` reference composition.
    ``bias_link`` (``nn.BiasLink``, also given to the projection ``linear``): short sequences emit the projection's
    bias gradient from the attention backward, and the linear skips its column-sum pass. ``rope_in_place``: rotate
    q / k inside ``qkv`` itself instead of a copy (the caller's projection output is a temporary: Llama's 201 MB
    per-layer clone at s4096 b4). Contract of ``rope_in_place``: the projection output has no other reader --
    no hook, no saved-for-backward reference (``_Linear`` saves its input, not its output), no ``grad_link`` --
    since those would see the rotated values; ``tests/test_attention_gpu.py`` pins in place == copy bitwise.
    ``rope_applied``: q / k already rotated by the projection's epilogue (``ops.nn.linear_rope``); the backward still
    returns the gradient of the UN-rotated projection output (dqkv rotated back), which is what that linear's backward
    takes."""
    D = head_dim
    scale = scale or 1.0 / math.sqrt(D)
    W = (heads + 2 * kv_heads) * D
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128) and qkv.shape[-1] == W and \
            W % 8 == 0 and qkv.is_contiguous():
        pos, table = rope if rope is not None else (None, None)
        return _FlashQKV.apply(qkv, B, S, heads, kv_heads, D, causal, kv_lens, scale, pos, table, bias_link,
                               rope_in_place, rope_applied)
    if rope_applied:
        raise RuntimeError("attention_qkv: q / k rotated by the projection epilogue need the fused GPU path")
    q, k, v = qkv.split([heads * D, kv_heads * D, kv_heads * D], dim=-1)
    if rope is not None:
        from k8s_amd.ops import nn as _nn

        q, k = _nn.rope(q, rope[0], rope[1]), _nn.rope(k, rope[0], rope[1])
    return attention(q.reshape(B, S, heads, D), k.reshape(B, S, kv_heads, D), v.reshape(B, S, kv_heads, D),
                     causal=causal, kv_lens=kv_lens, scale=scale)
