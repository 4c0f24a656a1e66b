"""Autograd ops of k8s_amd: HIP kernels on GPU, fp32 references on CPU.

Every op that owns parameters takes :class:`~k8s_amd.parallel.flat.Param`
handles plus the store's ``anchor`` and deposits parameter gradients straight
into the flat gradient buffer (see ``parallel/flat.py``); it returns ``None``
for them to autograd.

Layouts: convolution activations are NHWC ``[N, H, W, C]`` bf16 (channels
last, what the MFMA implicit-GEMM and the NHWC BatchNorm kernels want);
conv weights are KRSC ``[K, R, S, C]``; linear weights ``[out, in]``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from k8s_amd.ops import reference as ref
from k8s_amd.ops._ext import load as _load_ext


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _C():
    return _load_ext()


# =========================================================================== convolution
def _conv_impl():
    from k8s_amd.ops import conv as _conv  # lazy: conv module selects HIP implicit-GEMM vs MIOpen oracle

    return _conv


def _zero_scratch(store, device, n):
    from k8s_amd.parallel.flat import ZeroArena

    arena = store.__dict__.get("zero_arena")
    if arena is None or arena.device != torch.device(device):
        arena = store.zero_arena = ZeroArena(device)
    return arena.take(n)


class GradLink:
    """Carries one tensor's gradient from one autograd node to another that runs later in the backward
    pass, so the sum of the two contributions is formed inside a kernel (e.g. a ResNet identity block:
    the residual branch's dres is accumulated in conv1's dgrad epilogue instead of by a separate add).
    With ``shared=True`` the link joins two convolutions that read the same input (a ResNet downsample
    block's conv1 and downsample conv): whichever backward runs first hands its dx over instead of returning
    it, and the second accumulates it in its own dgrad epilogue -- correct in either autograd order."""
    __slots__ = ("grad", "shared")

    def __init__(self, shared: bool = False):
        self.grad = None
        self.shared = shared


class BiasLink:
    """Joins a linear (``linear(..., bias_link=l)``) to the LayerNorm that reads its output (``layer_norm(y, ...,
    bias_link=l)``): the norm's backward also emits the column sums of the gradient it returns for y -- that
    linear's bias gradient -- from its parameter-gradient kernel, so the linear skips its column-sum pass."""
    __slots__ = ("pb", "done")

    def __init__(self):
        self.pb, self.done = None, False


class ActLink:
    """Joins a linear with an activation (the producer, ``linear(x, W1, b1, act="gelu", act_link=l)``) to the linear
    that reads its output (the consumer, ``linear(y, W2, b2, act_in=l)``): the consumer's data gradient is formed as
    (dy . W2) * act'(pre), with the producer's bias gradient as its column sums, in the 4-wave GEMM's epilogue
    (gemm256.hip copy_out_x ACT < 0; ``gemm.dact_ok`` shapes) -- the producer's backward then skips its
    activation-backward pass (read dy and pre, write g) and its bias column sums. BERT's FFN1 -> FFN2."""
    __slots__ = ("saved", "act", "pb", "done")

    def __init__(self):
        self.saved, self.act, self.pb, self.done = None, None, None, False


class SwiGLULink:
    """Joins ``swiglu(gu, link=l)`` to the linear that reads its output (``linear(y, W, swiglu_in=l)``, Llama's down
    projection): that linear's data gradient takes the SwiGLU backward in its epilogue and produces the gradient of gu
    directly (gemm256.hip copy_out_x ACT = -3, ``gemm.swiglu_ok`` shapes), so neither the [T, F] gradient of the
    SwiGLU output nor the separate SwiGLU-backward pass over gu exists. ``blk``: gu's column layout (0 = gate | up
    halves, 64 = blocks of 64 gate then 64 up columns, ``linear_swiglu``)."""
    __slots__ = ("saved", "dgu", "blk")

    def __init__(self, blk: int = 0):
        self.saved, self.dgu, self.blk = None, None, blk


class MaskedGrad:
    """A residual gradient handed over unmaterialised: ``dy`` masked by the packed 1-bit ReLU ``mask`` of the BN
    forward (bit j of byte e = element 8e + j). The 1x1 dgrad that receives it reads the pair in its epilogue
    (GEMM add_src / add_mask), so the BN backward writes no dres tensor (2 B/element) and the dgrad reads 1/8 B
    of mask more than it would have read of dres."""
    __slots__ = ("dy", "mask")

    def __init__(self, dy, mask):
        self.dy, self.mask = dy, mask

    def materialize(self):
        return _C().mask_apply(self.dy, self.mask)


class BnStatLink:
    """Joins a residual BatchNorm (``y = relu(BN(x) + r)``, packed ReLU mask; or the two-BatchNorm form of a ResNet
    downsample block) to the 1x1 convolution that reads y with a masked residual addend (a ResNet identity block's
    conv1): that convolution's data gradient -- the whole gradient of y -- also accumulates the BatchNorm-backward
    sums (sum g, sum g (x - mean) for g = mask ? dy : 0) in its epilogue (gemm_short.hip EPI 3 / 4), so the
    BatchNorm's backward skips its reduction sweep over dy and x. The same for a non-residual BatchNorm + ReLU
    (``relu``: ResNet's bn1) read by a stride-1 3x3 convolution on the staged-window kernel (conv3x3.hip epilogue,
    g = relu_on(x) ? dy : 0 from the BatchNorm's affine). The BatchNorm's forward fills (x, mask, mean[, x2,
    mean2]) and tags y with the link (``y._k8s_bnstat``); the convolution's backward deposits the sums and the
    identity of the dy they were taken over; the BatchNorm's backward uses them only when it receives exactly that dy
    (so a second consumer of y, whose gradient autograd would add, falls back to the reduction)."""
    __slots__ = ("x", "mask", "mean", "x2", "mean2", "invstd", "gamma", "beta", "relu", "sums", "sums2", "dy_key",
                 "store", "pending", "last_full")

    def __init__(self, store=None):
        self.store = store  # the BatchNorm's ParamStore: its per-step zeroed scratch holds the sums
        self.x = self.mask = self.mean = self.x2 = self.mean2 = None
        self.invstd = self.gamma = self.beta = None
        self.relu = False  # a non-residual BatchNorm + ReLU (mask None: g = relu_on(x) ? dy : 0, from the affine)
        self.sums = self.sums2 = self.dy_key = None
        # sums over the first of two data gradients into y (a stage-entry block's conv1), awaiting the second's
        # correction (its downsample convolution, ops.conv._dgrad_strided_hip); dy_key is set only once complete
        self.pending = False
        # two stride-1 data gradients into y (the stem pool's output, read by layer 1's conv1 and downsample): the
        # first takes no sums, the second -- accumulating onto the first -- takes them over the final tensor
        self.last_full = False

    def take(self, dy):
        """(sums, sums2) if they were taken over ``dy``, else None; clears the deposit either way."""
        sums, sums2, key = self.sums, self.sums2, self.dy_key
        self.sums = self.sums2 = self.dy_key = None
        self.x = self.mask = self.mean = self.x2 = self.mean2 = None  # the BatchNorm's backward is the last reader
        self.invstd = self.gamma = self.beta = None
        if sums is None or key != (dy.data_ptr(), tuple(dy.shape)):
            return None
        return sums, sums2


# BatchNorm-backward sums in the masked-addend 1x1 dgrad epilogue (BnStatLink); K8S_AMD_BN_BSTATS=0 for the A/B
BN_BSTATS = os.environ.get("K8S_AMD_BN_BSTATS", "1") != "0"
# ... and for the stem's BatchNorm + ReLU + max pool (its sums in layer 1's downsample dgrad)
BSTATS_POOL = os.environ.get("K8S_AMD_BN_BSTATS_POOL", "1") != "0"


class MaskLink:
    """Joins a residual BN (ReLU, packed mask) to the plain BN that produced its residual input (a ResNet
    downsample branch): the residual BN's backward passes its incoming dy through unchanged as the residual's
    gradient and leaves its ReLU mask here; the plain BN's backward applies the mask while it reads dy (its
    reduce and apply kernels' mask path), so the masked gradient is never written out."""
    __slots__ = ("mask",)

    def __init__(self):
        self.mask = None


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, p, stride, padding, with_stats, link=None, bn_link=None):
        impl = _conv_impl()
        w = p.weight if x.dtype == p.weight.dtype else p.master.to(x.dtype)
        sums = None
        if with_stats and impl.fwd_uses_hip(x, w, stride, padding):
            sums = _zero_scratch(p.store, x.device, _C().conv_stat_replicas * 2 * w.shape[0]).view(
                _C().conv_stat_replicas, 2, w.shape[0])
        xs = None
        if impl.subsample_ok(x, w, stride, padding):  # 1x1 / stride 2: a stride-1 GEMM on the subsampled input
            xs = getattr(x, "_k8s_sub2", None) if stride == 2 else None  # written by x's BatchNorm (SubLink)
            if xs is None or xs.shape[:3] != ((x.shape[0], (x.shape[1] + 1) // 2, (x.shape[2] + 1) // 2)):
                xs = _C().subsample_nhwc(x, stride)
            y = impl.conv_fwd(xs, w, 1, 0, sums)
        else:
            y = impl.conv_fwd(x, w, stride, padding, sums)
        ctx.save_for_backward(x, xs)
        ctx.p, ctx.stride, ctx.padding, ctx.link, ctx.bn_link = p, stride, padding, link, bn_link
        ctx.x_requires_grad = x.requires_grad
        if sums is not None:
            ctx.mark_non_differentiable(sums)
        # the statistics output never gets a gradient: without this autograd materialises a zeros_like(sums) for
        # it on every backward (one fill kernel per conv, 56 per ResNet-50 step)
        ctx.set_materialize_grads(False)
        return y, sums

    @staticmethod
    def backward(ctx, gy, _gsums=None):
        x, xs = ctx.saved_tensors
        p = ctx.p
        impl = _conv_impl()
        w = p.weight if x.dtype == p.weight.dtype else p.master.to(x.dtype)
        gy = gy.contiguous()
        addend = None
        if ctx.link is not None:
            addend, ctx.link.grad = ctx.link.grad, None
            if addend is None and ctx.link.shared and ctx.x_requires_grad:  # first of the two readers of x
                ctx.link.grad = impl.conv_bwd(gy, x, w, ctx.stride, ctx.padding, True, p, x_sub=xs,
                                              bn_link=ctx.bn_link)
                return None, None, None, None, None, None, None, None
        dx = impl.conv_bwd(gy, x, w, ctx.stride, ctx.padding, ctx.x_requires_grad, p, addend=addend, x_sub=xs,
                           bn_link=ctx.bn_link)
        return dx, None, None, None, None, None, None, None


def conv2d_nhwc(x: torch.Tensor, p, stride: int = 1, padding: int = 0, with_stats: bool = False,
                grad_link: "GradLink" = None):
    """NHWC convolution with KRSC weight ``p`` (no bias).

    With ``with_stats`` returns ``(y, sums)``: ``sums`` = fp32 [2, K] per-channel sum / sum of squares of y
    accumulated in the conv epilogue (None when the layer runs on the fallback path) -- the following
    ``batch_norm_act(..., sums=sums)`` then needs no statistics pass. ``grad_link``: a gradient for x
    deposited there by a later-backward node (``batch_norm_act(res_link=...)``) is added to dx in the dgrad."""
    bn_link = getattr(x, "_k8s_bnstat", None)
    y, sums = _Conv2dNHWC.apply(x, p.store.anchor, p, stride, padding, with_stats, grad_link, bn_link)
    return (y, sums) if with_stats else y


class _StemS2D(torch.autograd.Function):
    """The 7x7 / stride-2 / pad-3 stem as a 4x4 / stride-1 conv over the 2x2 space-to-depth image
    (csrc/kernels/stem.hip): the master weight stays [K, 7, 7, C]; forward maps it to [K, 4, 4, 16], backward maps
    the 4x4 weight gradient back into the parameter's flat fp32 slot. The image needs no gradient."""

    @staticmethod
    def forward(ctx, xs, anchor, p):
        C_ = _C()
        w7 = p.weight if p.weight.dtype == xs.dtype else p.master.to(xs.dtype)
        w4 = C_.stem_w_s2d(w7.contiguous())
        sums = _zero_scratch(p.store, xs.device, C_.conv_stat_replicas * 2 * w4.shape[0]).view(
            C_.conv_stat_replicas, 2, w4.shape[0])
        if tuple(w4.shape) == (64, 4, 4, 16) and (xs.shape[2] - 3) % 16 == 0 and xs.shape[2] - 3 <= 112:
            y = C_.stem_conv_fwd(xs.contiguous(), w4, sums)  # LDS-tiled input window (stem.hip)
        else:
            y = C_.conv_fwd(xs, w4, 1, 0, 1, False, None, 0, sums)
        _conv_impl().STATS["hip_fwd"] += 1
        ctx.save_for_backward(xs)
        ctx.p, ctx.kshape = p, tuple(w4.shape)
        ctx.mark_non_differentiable(sums)
        ctx.set_materialize_grads(False)
        return y, sums

    @staticmethod
    def backward(ctx, gy, _gsums=None):
        (xs,) = ctx.saved_tensors
        p, C_ = ctx.p, _C()
        dw4 = torch.empty(ctx.kshape, device=xs.device, dtype=torch.float32)
        if ctx.kshape == (64, 4, 4, 16) and (xs.shape[2] - 3) % 16 == 0 and xs.shape[2] - 3 <= 112:
            C_.stem_wgrad(xs.contiguous(), gy.contiguous(), dw4)  # LDS-tiled persistent kernel (stem.hip)
        else:
            _conv_impl()._wgrad_hip(C_, gy.contiguous(), xs, dw4, 1, 0, False)
        _conv_impl().STATS["hip_wgrad"] += 1
        store = p.store
        slot = store.slot_for_write(p)
        if slot is not None:
            C_.stem_dw_s2d(dw4, slot.view(p.shape))
            store.mark_written(p)
        else:
            tmp = torch.empty(p.shape, device=xs.device, dtype=torch.float32)
            C_.stem_dw_s2d(dw4, tmp)
            store.deposit(p, tmp)
        return None, None, None


def stem_conv_s2d(xs, p):
    """(y, BN statistics) of the 7x7/s2 stem weight ``p`` applied to a space-to-depth image ``xs`` [N, H/2+3,
    W/2+3, 16] (``stem_s2d_input``); GPU only."""
    return _StemS2D.apply(xs, p.store.anchor, p)


def stem_s2d_input(images, pad: int = 3):
    """[N, H, W, <= 8] bf16 image -> [N, (H+2*pad)/2, (W+2*pad)/2, 16] space-to-depth input of ``stem_conv_s2d``."""
    return _C().stem_s2d_input(images.contiguous(), pad)


# =========================================================================== batchnorm + act
class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, anchor, pg, pb, run_mean, run_var, training, momentum, eps, relu, sums=None,
                res_link=None, dy_link=None, stat_link=None, sub2=None):
        x = x.contiguous()
        if res is not None:
            res = res.contiguous()
        # residual + ReLU on the GPU: the forward also writes the packed ReLU mask (1 bit per element) that the
        # backward's reduce and apply passes read instead of the bf16 output (saves ~2 B/elem per pass)
        want_mask = relu and res is not None and _gpu(x)
        mask = None
        want_sub = sub2 is not None and x.dim() == 4
        if _gpu(x) and sums is not None and training:
            out = _C().bn_fwd_from_sums(x, res, pg.master, pb.master, sums, run_mean, run_var, momentum, eps, relu,
                                        want_mask, want_sub)
            if want_sub:  # y[:, ::2, ::2] for the next block's downsample convolution (SubLink)
                sub2.y = out[-1]
        elif _gpu(x):
            out = _C().bn_fwd(x, res, pg.master, pb.master, run_mean, run_var, training, momentum, eps, relu,
                              want_mask)
        else:
            out = ref.bn_fwd(x, res, pg.master, pb.master, run_mean, run_var, training, momentum, eps, relu)
        y, mean, invstd = out[0], out[1], out[2]
        if want_mask:
            mask = out[3]
        # without a residual the ReLU mask is recomputed from x in the backward kernels (no need to keep y)
        keep_y = relu and (res is not None or not _gpu(x)) and mask is None
        ctx.save_for_backward(x, y if keep_y else None, mean, invstd, mask)
        ctx.pg, ctx.pb, ctx.has_res, ctx.res_link = pg, pb, res is not None, res_link
        ctx.relu_x = relu and not keep_y and mask is None
        ctx.dy_link = dy_link if (dy_link is not None and not relu and res is None) else None
        ctx.stat_link = None
        if stat_link is not None and training and (mask is not None or ctx.relu_x):
            stat_link.x, stat_link.mask, stat_link.mean, stat_link.store = x, mask, mean, pg.store
            if mask is None:
                stat_link.relu, stat_link.invstd, stat_link.gamma, stat_link.beta = True, invstd, pg.master, pb.master
            ctx.stat_link = stat_link
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, invstd, mask = ctx.saved_tensors
        pg, pb = ctx.pg, ctx.pb
        store = pg.store
        dy = dy.contiguous()
        if ctx.dy_link is not None and ctx.dy_link.mask is not None:  # dy arrives unmasked: apply the mask here
            mask, ctx.dy_link.mask = ctx.dy_link.mask, None
        mask_out = isinstance(ctx.res_link, MaskLink) and mask is not None and ctx.has_res
        if _gpu(x):
            sg, sb = store.slot_for_write(pg), store.slot_for_write(pb)
            dg = sg if sg is not None else torch.empty(pg.shape, device=x.device, dtype=torch.float32)
            db = sb if sb is not None else torch.empty(pb.shape, device=x.device, dtype=torch.float32)
            # residual gradient for a linked consumer: (dy, mask) instead of a written dres tensor
            handoff = isinstance(ctx.res_link, GradLink) and ctx.has_res and mask is not None
            want_dres = ctx.has_res and not (handoff or mask_out)
            pre = ctx.stat_link.take(dy) if ctx.stat_link is not None else None
            if pre is not None and mask is None:  # relu_x: the reduction came with dy (BnStatLink)
                dx, dres = _C().bn_bwd_relu_from_sums(dy, x, pre[0], mean, invstd, pg.master, pb.master, dg, db)[0], None
            elif pre is not None:  # the reduction came with dy from its producer's epilogue (BnStatLink)
                dx, dres = _C().bn_bwd_from_sums(dy, x, mask, pre[0], mean, invstd, pg.master, pb.master, dg, db,
                                                 want_dres)
            else:
                dx, dres = _C().bn_bwd(dy, x, y, mean, invstd, pg.master, pb.master, ctx.relu_x, dg, db, want_dres,
                                       mask)
            if handoff:
                dres = MaskedGrad(dy, mask)
            elif mask_out:  # the producing plain BN masks dy itself (MaskLink)
                dres = dy
                ctx.res_link.mask = mask
            if sg is not None:
                store.mark_written(pg)
            else:
                store.deposit(pg, dg)
            if sb is not None:
                store.mark_written(pb)
            else:
                store.deposit(pb, db)
        else:
            dx, dres, dg, db = ref.bn_bwd(dy, x, y, mean, invstd, pg.master)
            store.deposit(pg, dg)
            store.deposit(pb, db)
        if ctx.has_res and isinstance(ctx.res_link, GradLink):  # hand dres to the node that adds it in a kernel
            ctx.res_link.grad, dres = dres, None
        return (dx, (dres if ctx.has_res else None), None, None, None, None, None, None, None, None, None, None, None,
                None, None, None)


# Which BatchNorm + ReLU outputs of a ResNet bottleneck are normalised on load by the convolution that consumes them
# (``bn_relu_conv``) instead of being written by an apply pass. Default "1x1": bn2 -> the 1x1 conv3 everywhere.
# "3x3" also normalises bn1 in the 3x3 conv2 wherever the staged-window kernels take the layer (stride 1:
# conv3x3.hip forward, wgrad_tile.hip weight gradient, each transforming a staged element once, not once per tap as
# the round-3 implicit-GEMM path did). Measured round 4 (ResNet-50 b1024, one box, rocprofv3 per-kernel diff,
# profiles/r04_bn1_onload_diff.txt): it removes 11 of 32 apply passes (-0.78 ms / step) but the in-LDS transform pass
# costs the staged forward +0.36 ms and the tiled weight gradient +0.71 ms (a VALU / LDS phase between the window
# DMA and the MFMAs): 13.78-13.84k vs 13.85-13.87k img/s, so it stays opt-in.
BN_ONLOAD = os.environ.get("K8S_AMD_BN_ONLOAD", "1x1")
if BN_ONLOAD not in ("0", "1x1", "3x3"):  # an unknown value must not quietly mean "1x1"
    raise ValueError("K8S_AMD_BN_ONLOAD must be 0 (BN applied by its own pass), 1x1 or 3x3, not %r" % BN_ONLOAD)


def _bn_param_grads(store, pg, pb, device):
    sg, sb = store.slot_for_write(pg), store.slot_for_write(pb)
    dg = sg if sg is not None else torch.empty(pg.shape, device=device, dtype=torch.float32)
    db = sb if sb is not None else torch.empty(pb.shape, device=device, dtype=torch.float32)

    def finish():
        store.mark_written(pg) if sg is not None else store.deposit(pg, dg)
        store.mark_written(pb) if sb is not None else store.deposit(pb, db)

    return dg, db, finish


class _BnReluConv(torch.autograd.Function):
    """conv(relu(BN(x)), w) for a training-mode BatchNorm whose statistics came from x's producing conv epilogue
    (``sums``): the BN is finalised to per-channel (scale, shift) and APPLIED INSIDE THE CONVOLUTION'S OPERAND LOAD
    (gemm.hip XForm) -- the z = relu(BN(x)) tensor is never written, saving the apply pass (read x, write z) and
    z's memory. Backward: the weight gradient normalises x on load the same way; the data gradient gives dz, and
    the BN backward (reduce + apply, ReLU mask recomputed from x bit-exactly) turns it into dx.
    Returns (y, y's BN statistics sums) like ``conv2d_nhwc(..., with_stats=True)``."""

    @staticmethod
    def forward(ctx, x, sums, anchor, pg, pb, run_mean, run_var, momentum, eps, pw, stride, padding):
        C_ = _C()
        x = x.contiguous()
        M = x.numel() // x.shape[-1]
        mean, invstd, params = C_.bn_finalize(sums, pg.master, pb.master, run_mean, run_var, M, momentum, eps)
        w = pw.weight
        ysums = _zero_scratch(pw.store, x.device, C_.conv_stat_replicas * 2 * w.shape[0]).view(
            C_.conv_stat_replicas, 2, w.shape[0])
        y = C_.conv_fwd(x, w, stride, padding, 1, False, None, 0, ysums, xform=params)
        _conv_impl().STATS["hip_fwd"] += 1
        ctx.save_for_backward(x, mean, invstd, params)
        ctx.pg, ctx.pb, ctx.pw, ctx.stride, ctx.padding = pg, pb, pw, stride, padding
        ctx.x_requires_grad = x.requires_grad
        ctx.mark_non_differentiable(ysums)
        ctx.set_materialize_grads(False)
        return y, ysums

    @staticmethod
    def backward(ctx, gy, _gsums=None):
        x, mean, invstd, params = ctx.saved_tensors
        pg, pb, pw = ctx.pg, ctx.pb, ctx.pw
        impl = _conv_impl()
        gy = gy.contiguous()
        # the BatchNorm-backward sums in the data gradient's epilogue where a kernel takes them (BnStatLink)
        link = None
        if BN_BSTATS:
            link = BnStatLink(pg.store)
            link.x, link.mean, link.invstd, link.gamma, link.beta, link.relu = (x, mean, invstd, pg.master, pb.master,
                                                                                True)
        dz = impl.conv_bwd(gy, x, pw.weight, ctx.stride, ctx.padding, True, pw, xform=params, bn_link=link)
        dg, db, finish = _bn_param_grads(pg.store, pg, pb, x.device)
        pre = link.take(dz) if link is not None else None
        if pre is not None:
            dx = _C().bn_bwd_relu_from_sums(dz, x, pre[0], mean, invstd, pg.master, pb.master, dg, db)[0]
        else:
            dx, _ = _C().bn_bwd(dz, x, None, mean, invstd, pg.master, pb.master, True, dg, db, False)
        finish()
        return (dx if ctx.x_requires_grad else None,) + (None,) * 11


# Largest BatchNorm channel count normalised on load (K8S_AMD_ONLOAD_MAXC). The on-load operand path feeds the MFMAs
# through VGPRs instead of the LDS-DMA path: in the compute-bound stage-3/4 1x1 products (bn2 of 256 / 512 channels)
# it ran the conv3 forward and weight gradient at 0.19-0.33 of their floor against 0.41-0.52 for the same layers'
# plain data gradient (profiles/r05_resnet50_roofline.jsonl), more than the [M, C/4] apply pass it saves. Round 6,
# same box alternating (profiles/r06_notes.md): limit 128 +1.0-1.3 %, 256 +0.4-0.8 %, none = the round-5 default.
ONLOAD_MAXC = int(os.environ.get("K8S_AMD_ONLOAD_MAXC", "128"))
# bn1 normalised on load by the staged-window 3x3 kernels up to this many channels (K8S_AMD_ONLOAD3_MAXC; 0 = only
# with BN_ONLOAD == "3x3")
ONLOAD3_MAXC = int(os.environ.get("K8S_AMD_ONLOAD3_MAXC", "0"))


def onload_ok(x, conv) -> bool:
    """Whether ``conv`` can consume relu(BN(x)) normalised on load in all three of its products: a 1x1 stride-1
    convolution (the GEMM operand paths), or a 3x3 one the staged-window kernels take (``BN_ONLOAD == "3x3"``)."""
    if BN_ONLOAD == "0" or x.shape[-1] > ONLOAD_MAXC:
        return False
    K_, R, S, C = conv.w.shape
    if R == 1 and S == 1:
        return conv.stride == 1 and conv.pad == 0
    return ((BN_ONLOAD == "3x3" or x.shape[-1] <= ONLOAD3_MAXC) and x.dim() == 4 and
            bool(_C().conv3x3_staged_ok(x.shape[1], x.shape[2], C, K_, R, S, conv.stride, conv.pad)))


def bn_relu_conv(t, bn, conv):
    """``conv(bn(t))`` for ``t = (x, sums)`` from ``conv2d_nhwc(..., with_stats=True)``, a training-mode ReLU
    BatchNorm ``bn`` (models/resnet.BN) and a convolution ``conv`` (models/resnet.Conv): normalised on load
    (``_BnReluConv``) where the kernels take it (``onload_ok``), else the separate BN apply + conv. Returns (y, y's
    sums)."""
    x, sums = t if isinstance(t, tuple) else (t, None)
    w = conv.w
    if (sums is not None and bn.training and _gpu(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 64 == 0
            and w.weight.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and w.grad.dtype == torch.float32
            and onload_ok(x, conv)):
        return _BnReluConv.apply(x, sums, w.store.anchor, bn.gamma, bn.beta, bn.running_mean, bn.running_var,
                                 bn.momentum, bn.eps, w, conv.stride, conv.pad)
    return conv(bn(t))


# BatchNorm apply passes write the stride-2 subsample for a following downsample block (SubLink);
# K8S_AMD_SUB2_FUSED=0: the separate subsample pass (A/B)
SUB2_FUSED = os.environ.get("K8S_AMD_SUB2_FUSED", "1") != "0"


class SubLink:
    """The stride-2 subsample of a BatchNorm output, written by the BatchNorm's own apply pass (bn_apply_kernel) when
    the next ResNet block is a downsample block: its 1x1 / stride-2 downsample convolution (run as a stride-1 GEMM on
    the subsampled input, ops.conv.SUB1X1) then takes it instead of a separate subsample pass over the tensor."""
    __slots__ = ("y",)

    def __init__(self):
        self.y = None


def batch_norm_act(x, pg, pb, run_mean, run_var, residual=None, relu=True, training=True, momentum=0.1,
                   eps=1e-5, sums=None, res_link=None, dy_link=None, sub2=False):
    """y = act(BN(x) + residual) over the last (channel) dim of an NHWC tensor.

    ``sums`` (fp32 [2, C] from ``conv2d_nhwc(..., with_stats=True)``) skips the statistics pass.
    ``res_link``: the residual's gradient is handed to that GradLink (and NOT returned to autograd); the
    node consuming the link must add it (``conv2d_nhwc(..., grad_link=link)`` on the same tensor).
    ``res_link`` may also be a MaskLink whose ``dy_link`` end is the plain BN that produced ``residual``."""
    link = BnStatLink() if (BN_BSTATS and relu and training and _gpu(x)) else None
    sub = SubLink() if (sub2 and SUB2_FUSED and sums is not None and _gpu(x)) else None
    y = _BnAct.apply(x, residual, pg.store.anchor, pg, pb, run_mean, run_var, training, momentum, eps, relu,
                     sums, res_link, dy_link, link, sub)
    if link is not None and link.x is not None:
        y._k8s_bnstat = link
    if sub is not None and sub.y is not None:
        y._k8s_sub2 = sub.y
    return y


# =========================================================================== layernorm / rmsnorm
class _Norm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, anchor, pg, pb, eps, rms, res_link=None, bias_link=None):
        # an unused second output (x + res) must not get a materialised zero gradient (one [T, D] fill per norm)
        ctx.set_materialize_grads(False)
        x = x.contiguous()
        if res is not None:
            res = res.contiguous()
        beta = pb.master if pb is not None else None
        if _gpu(x):
            y, mean, rstd, xsum = _C().norm_fwd(x, res, pg.master, beta, eps, rms)
        else:
            y, mean, rstd, xsum = ref.norm_fwd(x, res, pg.master, beta, eps, rms)
        xin = xsum if res is not None else x
        ctx.save_for_backward(xin, mean, rstd)
        ctx.pg, ctx.pb, ctx.rms, ctx.has_res = pg, pb, rms, res is not None
        ctx.res_link = res_link if res is not None else None
        ctx.bias_link = bias_link
        if res is not None:
            return y, xsum
        return y, None

    @staticmethod
    def backward(ctx, dy, dxsum):
        xin, mean, rstd = ctx.saved_tensors
        pg, pb = ctx.pg, ctx.pb
        store = pg.store
        if dy is None:
            dy = torch.zeros(xin.shape, device=xin.device, dtype=xin.dtype)
        dy = dy.contiguous()
        dres = dxsum.contiguous() if (dxsum is not None and ctx.has_res) else None
        if _gpu(xin):
            # gamma / beta gradients straight into their flat fp32 slots on first use (no temporary + copy)
            sg = store.slot_for_write(pg)
            sb = store.slot_for_write(pb) if pb is not None else None
            dg = sg.view(pg.shape) if sg is not None else torch.empty(pg.shape, device=xin.device,
                                                                       dtype=torch.float32)
            db = None
            if pb is not None:
                db = sb.view(pb.shape) if sb is not None else torch.empty(pb.shape, device=xin.device,
                                                                           dtype=torch.float32)
            bl = ctx.bias_link
            lpb = bl.pb if (bl is not None and dres is None) else None
            dsum = None
            if lpb is not None:  # the producing linear's bias gradient (column sums of dx) from the same pass
                ss = store.slot_for_write(lpb) if lpb.store is store else None
                dsum = ss.view(lpb.shape) if ss is not None else torch.empty(lpb.shape, device=xin.device,
                                                                             dtype=torch.float32)
            dx = _C().norm_bwd(dy, xin, pg.master, mean, rstd, dres, dg, db, ctx.rms, dsum=dsum)
            store.mark_written(pg) if sg is not None else store.deposit(pg, dg)
            if pb is not None:
                store.mark_written(pb) if sb is not None else store.deposit(pb, db)
            if lpb is not None:
                lpb.store.mark_written(lpb) if ss is not None else lpb.store.deposit(lpb, dsum)
                bl.done = True
        else:
            dx, dg, db = ref.norm_bwd(dy, xin, pg.master, mean, rstd, dres, ctx.rms)
            store.deposit(pg, dg)
            if pb is not None:
                store.deposit(pb, db)
        dres_out = None
        if ctx.has_res:
            dres_out = dx
            link = ctx.res_link
            if link is not None:
                if link.grad is None:  # the residual's other consumer (a linear) runs later: it adds dx in its
                    link.grad = dx     # dgrad epilogue and returns the sum, so nothing is returned here
                    dres_out = None
                else:  # that linear already ran and handed its dgrad over: form the sum here
                    dres_out = dx + link.grad
                    link.grad = None
        return dx, dres_out, None, None, None, None, None, None, None


def layer_norm(x, pg, pb, eps=1e-12, residual=None, res_link=None, bias_link=None):
    """LayerNorm over the last dim; with ``residual`` returns (norm(x+res), x+res). ``res_link`` (a GradLink
    shared with the linear that also reads ``residual``): the two gradient contributions of ``residual`` are
    summed in that linear's dgrad epilogue instead of by a separate add. ``bias_link``: see ``BiasLink``."""
    y, xsum = _Norm.apply(x, residual, pg.store.anchor, pg, pb, eps, False, res_link, bias_link)
    return (y, xsum) if residual is not None else y


def rms_norm(x, pg, eps=1e-5, residual=None, res_link=None):
    y, xsum = _Norm.apply(x, residual, pg.store.anchor, pg, None, eps, True, res_link)
    return (y, xsum) if residual is not None else y


# =========================================================================== linear
def _gemm():
    from k8s_amd.ops import gemm as _g

    return _g


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, anchor, pw, pb, act, grad_link=None, bias_link=None, act_link=None, act_in=None,
                swiglu_in=None):
        g = _gemm()
        w = pw.weight if x.dtype == pw.weight.dtype else pw.master.to(x.dtype)
        x2 = x.reshape(-1, x.shape[-1])
        b = pb.master if pb is not None else None
        y, pre = g.linear_fwd(x2, w, b, act)
        ctx.save_for_backward(x2, pre)
        ctx.pw, ctx.pb, ctx.act, ctx.xshape, ctx.grad_link = pw, pb, act, x.shape, grad_link
        ctx.bias_link = bias_link
        if bias_link is not None and act is None:
            bias_link.pb = pb
        # producer end of an ActLink: what the consumer's fused data gradient needs (saved: the GELU pre-activation /
        # the ReLU output, as this node's own backward would read)
        ctx.act_link = act_link if (act_link is not None and act is not None and pb is not None and
                                    pre is not None and pre.dtype == torch.bfloat16) else None
        if ctx.act_link is not None:
            act_link.saved, act_link.act, act_link.pb, act_link.done = pre, act, pb, False
        ctx.act_in = act_in
        ctx.swiglu_in = swiglu_in
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, pre = ctx.saved_tensors
        pw, pb = ctx.pw, ctx.pb
        g = _gemm()
        w = pw.weight if x2.dtype == pw.weight.dtype else pw.master.to(x2.dtype)
        gy2 = gy.reshape(-1, gy.shape[-1]).contiguous()
        link = ctx.grad_link
        addend = None
        if link is not None and link.grad is not None:  # x's other gradient contribution, handed over (GradLink)
            addend = link.grad.reshape(x2.shape)
            link.grad = None
        db_done = ctx.bias_link is not None and ctx.bias_link.done  # the reading norm produced it
        act = ctx.act
        if ctx.act_link is not None and ctx.act_link.done:  # the consumer's data gradient applied act' and took db
            ctx.act_link.done, ctx.act_link.saved = False, None
            act, db_done = None, True
        dx_act = None
        li = ctx.act_in
        if li is not None and li.saved is not None and g.dact_ok(x2, w, addend, gy):
            dx_act = (li.saved, li.act, li.pb, li.pb.store)
        sl, dx_swiglu = ctx.swiglu_in, None
        if dx_act is None and sl is not None and sl.saved is not None and g.swiglu_ok(x2, w, addend, gy):
            dx_swiglu = sl.saved
        dx, dw, db = g.linear_bwd(gy2, x2, w, pre, act, pw=pw, store=pw.store,
                                  need_db=pb is not None and not db_done, dx_addend=addend, pb=pb, dx_act=dx_act,
                                  dx_swiglu=dx_swiglu, swiglu_blk=sl.blk if dx_swiglu is not None else 0)
        if dx_act is not None:
            li.done, li.saved = True, None
        if dx_swiglu is not None:  # the SwiGLU's backward returns dgu; x's own gradient is never formed
            sl.dgu, sl.saved = dx, None
            dx = dx.new_zeros(()).expand(ctx.xshape)  # (stride 0: never materialised, ignored by the SwiGLU node)
        if dw is not None:
            pw.store.deposit(pw, dw)
        if pb is not None and db is not None:  # None: written straight into its slot
            pb.store.deposit(pb, db)
        if link is not None and addend is None:  # ran first: hand dx to the norm backward, which forms the sum
            link.grad = dx.reshape(ctx.xshape)
            return (None,) * 10
        return (dx.reshape(ctx.xshape),) + (None,) * 9


# BERT's FFN1 -> FFN2 activation backward fused into FFN2's data gradient (ActLink); tests switch it off to compare
ACT_FUSE = True
# Llama's SwiGLU backward fused into the down projection's data gradient (SwiGLULink); likewise (and
# K8S_AMD_SWIGLU_FUSE=0 for whole-run A/Bs)
SWIGLU_FUSE = os.environ.get("K8S_AMD_SWIGLU_FUSE", "1") != "0"


def linear(x, pw, pb=None, act: Optional[str] = None, grad_link=None, bias_link=None, act_link=None, act_in=None,
           swiglu_in=None):
    """y = act(x @ W^T + b); W [out, in] bf16 from the flat store. ``grad_link``: see ``layer_norm``;
    ``bias_link``: see ``BiasLink``; ``act_link`` (on the producer, with ``act``) / ``act_in`` (on the consumer):
    see ``ActLink``."""
    if not ACT_FUSE:
        act_link = act_in = None
    if not SWIGLU_FUSE:
        swiglu_in = None
    return _Linear.apply(x, pw.store.anchor, pw, pb, act, grad_link, bias_link, act_link, act_in, swiglu_in)


# =========================================================================== embedding
class _EmbeddingSum(torch.autograd.Function):
    """sum_i W_i[row_i(t)] over 1-3 tables on the GPU (csrc/kernels/embedding.hip): gather + sum in one pass, the
    backward scatter-adds (fp32 atomics) straight into each table's flat fp32 gradient slot. ``ids`` None = a
    position table (row = token % S)."""

    @staticmethod
    def forward(ctx, anchor, S, dtype, *flat):
        ids = list(flat[0::2])
        pws = list(flat[1::2])
        T = next(i.numel() for i in ids if i is not None) if any(i is not None for i in ids) else None
        ws = [pw.weight if pw.weight.dtype == dtype else pw.master.to(dtype) for pw in pws]
        ids_c = [i.reshape(-1).contiguous() if i is not None else None for i in ids]
        out = _C().embed_fwd(ws, ids_c, T, S)
        ctx.save_for_backward(*[i if i is not None else torch.empty(0) for i in ids_c])
        ctx.has_ids = [i is not None for i in ids_c]
        ctx.pws, ctx.S = pws, S
        return out

    @staticmethod
    def backward(ctx, g):
        saved = ctx.saved_tensors
        ids = [t if h else None for t, h in zip(saved, ctx.has_ids)]
        g = g.contiguous()
        grads, finish = [], []
        for pw in ctx.pws:
            store = pw.store
            slot = store.slot_for_write(pw)
            if slot is not None:  # first writer: zero the slot, scatter-add into it
                slot.zero_()
                grads.append(slot.view(pw.shape))
                finish.append(lambda pw=pw: pw.store.mark_written(pw))
            elif pw.grad.dtype == torch.float32:  # tied weight already holds the other use's gradient
                grads.append(pw.grad.view(pw.shape))
                finish.append(lambda pw=pw: pw.store._notify(pw))
            else:
                tmp = torch.zeros(pw.shape, device=g.device, dtype=torch.float32)
                grads.append(tmp)
                finish.append(lambda pw=pw, tmp=tmp: pw.store.deposit(pw, tmp))
        _C().embed_bwd(g, grads, ids, ctx.S)
        for f in finish:
            f()
        return (None, None, None) + (None,) * (2 * len(ctx.pws))


def embedding_sum(tables, S: int = 0, dtype=torch.bfloat16):
    """Sum of embedding lookups: ``tables`` = [(ids [B, S] int64 or None for positions 0..S-1, param), ...] (1-3),
    returns [B*S, D]. One fused HIP gather (and scatter-add backward) on the GPU; aten gathers on the CPU."""
    ids0 = next(i for i, _ in tables if i is not None)
    pw0 = tables[0][1]
    if _gpu(pw0.master) and pw0.shape[1] % 8 == 0 and len(tables) <= 3:
        flat = []
        for i, pw in tables:
            flat += [i, pw]
        return _EmbeddingSum.apply(pw0.store.anchor, S or ids0.shape[-1], dtype, *flat)
    T = ids0.numel()
    out = None
    for i, pw in tables:
        if i is None:
            i = torch.arange(S or ids0.shape[-1], device=ids0.device).repeat(T // (S or ids0.shape[-1]))
        e = embedding(i.reshape(-1), pw, dtype)
        out = e if out is None else out + e
    return out


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, anchor, pw, dtype):
        w = pw.weight if pw.weight.dtype == dtype else pw.master.to(dtype)
        ctx.save_for_backward(ids)
        ctx.pw = pw
        return F.embedding(ids, w)

    @staticmethod
    def backward(ctx, gy):
        (ids,) = ctx.saved_tensors
        pw = ctx.pw
        V, D = pw.shape
        store = pw.store
        slot = store.slot_for_write(pw)
        if slot is not None:  # scatter-add straight into the flat fp32 gradient slot (no [V, D] temporary)
            slot.zero_()
            slot.index_add_(0, ids.reshape(-1), gy.reshape(-1, D).to(slot.dtype))
            store.mark_written(pw)
        elif pw.grad.dtype == torch.float32:  # tied weight already holds the other use's gradient
            pw.grad.index_add_(0, ids.reshape(-1), gy.reshape(-1, D).float())
            store._notify(pw)
        else:
            dw = torch.zeros((V, D), device=gy.device, dtype=torch.float32)
            dw.index_add_(0, ids.reshape(-1), gy.reshape(-1, D).float())
            store.deposit(pw, dw)
        return None, None, None, None


def embedding(ids, pw, dtype=torch.bfloat16):
    return _Embedding.apply(ids, pw.store.anchor, pw, dtype)


# =========================================================================== loss
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, smoothing, valid):
        # logits [R, Vpad]: only the first `valid` columns are classes (MFMA-friendly padded vocabularies)
        logits = logits if logits.stride(-1) == 1 else logits.contiguous()
        ctx.valid = valid
        full = logits
        if valid is not None and valid != logits.shape[1]:
            logits = logits[:, :valid]
        if _gpu(logits):
            loss, lse = _C().xent_fwd(logits, labels, ignore_index, smoothing)
        else:
            loss, lse = ref.xent_fwd(logits, labels, ignore_index, smoothing)
        nvalid = (labels != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(full, labels, lse, nvalid)
        ctx.ignore_index, ctx.smoothing = ignore_index, smoothing
        return loss.sum() / nvalid

    @staticmethod
    def backward(ctx, gl):
        full, labels, lse, nvalid = ctx.saved_tensors
        dscale = (gl.float() / nvalid).reshape(1)
        V = ctx.valid if ctx.valid is not None else full.shape[1]
        if _gpu(full):
            d = _C().xent_bwd(full, labels, lse, dscale, ctx.ignore_index, ctx.smoothing, V)
        else:
            d = torch.zeros_like(full)
            d[:, :V] = ref.xent_bwd(full[:, :V], labels, lse, dscale, ctx.ignore_index, ctx.smoothing)
        return d, None, None, None, None


def cross_entropy(logits, labels, ignore_index: int = -100, smoothing: float = 0.0, valid: int = None):
    """Mean softmax cross-entropy over valid rows of [R, V] logits (classes = first ``valid`` columns)."""
    return _CrossEntropy.apply(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), ignore_index, smoothing,
                               valid)


# =========================================================================== pooling (NHWC)
class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = _C().maxpool_fwd(x.contiguous(), k, s, p)
        ctx.save_for_backward(idx)
        ctx.hw, ctx.ksp = x.shape[1:3], (k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W = ctx.hw
        return _C().maxpool_bwd(dy.contiguous(), idx, H, W, *ctx.ksp), None, None, None


def max_pool_nhwc(x, k=3, s=2, p=1):
    """NHWC max pooling; GPU: gfx950 kernel saving the winning window position as uint8 (gather backward)."""
    if _gpu(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        return _MaxPoolNHWC.apply(x, k, s, p)
    y = F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p)
    return y.permute(0, 2, 3, 1).contiguous()


class _BnReluMaxPool(torch.autograd.Function):
    """max_pool(relu(BN(x)), 3, 2, 1) for the ResNet stem in one pass each way (batchnorm.hip
    bn_relu_maxpool_fwd_kernel / pool_bn_bwd_*): the BN output is never stored; the backward gathers the
    max-pool gradient inside the BatchNorm backward's reduce and apply passes. Statistics from the conv epilogue."""

    @staticmethod
    def forward(ctx, x, sums, anchor, pg, pb, run_mean, run_var, momentum, eps):
        x = x.contiguous()
        # BnStatLink (mask kind): the pooled output's data gradients take the BatchNorm-backward sums in their
        # epilogue -- g = bit ? dpool : 0 lands on the window winner, so (winner's x, its ReLU bit) per pooled
        # element is all they need -- and the backward skips pool_bn_bwd_reduce's sweep over the 112 x 112 x
        want = BN_BSTATS and BSTATS_POOL
        outs = _C().bn_relu_maxpool(x, sums, pg.master, pb.master, run_mean, run_var, momentum, eps, want)
        y, idx, mean, invstd = outs[:4]
        ctx.save_for_backward(x, idx, mean, invstd)
        ctx.pg, ctx.pb = pg, pb
        ctx.link = None
        if want:
            link = BnStatLink(pg.store)
            link.x, link.mask, link.mean, link.last_full = outs[4], outs[5], mean, True
            y._k8s_bnstat = ctx.link = link
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, idx, mean, invstd = ctx.saved_tensors
        pg, pb = ctx.pg, ctx.pb
        dg, db, finish = _bn_param_grads(pg.store, pg, pb, x.device)
        dy = dy.contiguous()
        pre = ctx.link.take(dy) if ctx.link is not None else None
        if pre is not None:
            dx = _C().pool_bn_bwd_from_sums(dy, idx, x, mean, invstd, pg.master, pb.master, dg, db, pre[0])
        else:
            dx = _C().pool_bn_bwd(dy, idx, x, mean, invstd, pg.master, pb.master, dg, db)
        finish()
        return (dx,) + (None,) * 8


def bn_relu_maxpool(t, bn):
    """``max_pool_nhwc(bn(t), 3, 2, 1)`` for ``t = (x, sums)`` from a conv with the statistics epilogue and a
    training-mode ReLU BatchNorm ``bn`` (models/resnet.BN): fused on the GPU where the kernels take the shape, else
    the separate BN + max pool."""
    x, sums = t if isinstance(t, tuple) else (t, None)
    if (sums is not None and bn.training and _gpu(x) and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.shape[-1] % 8 == 0 and 256 % (x.shape[-1] // 8) == 0):
        return _BnReluMaxPool.apply(x, sums, bn.gamma.store.anchor, bn.gamma, bn.beta, bn.running_mean,
                                    bn.running_var, bn.momentum, bn.eps)
    return max_pool_nhwc(bn(t), 3, 2, 1)


# ResNet downsample blocks: bn3 and the downsample BN in one apply pass (bn_act_dual), their backwards in one reduce
# sweep + one apply pass (measured round 3: 13.27k -> 13.41k and 13.40k -> 13.56k img/s). tests/test_resnet_gpu.py
# switches BN_DUAL off to check the fused path against the separate BatchNorms.
BN_DUAL = True


class _BnActDual(torch.autograd.Function):
    """relu(BN(x) + BN_r(xr)) for a ResNet downsample block (bn3 over conv3's output, the downsample BN over the
    downsample conv's output), statistics of both from their convs' epilogue sums (batchnorm.hip
    launch_bn_fwd_from_sums_dual). The downsample BN's output is never written: as a separate pass it was stored
    (2 B / element) and read back once by bn3's apply. Backward: both BatchNorm backwards read the same dy through the
    packed ReLU mask of y (what the MaskLink hand-over of the separate path does)."""

    @staticmethod
    def forward(ctx, x, sums, xr, sums_r, anchor, pg, pb, run_mean, run_var, pgr, pbr, run_mean_r, run_var_r,
                momentum, eps, stat_link=None):
        x, xr = x.contiguous(), xr.contiguous()
        y, mean, invstd, mask, mean_r, invstd_r = _C().bn_fwd_from_sums_dual(
            x, sums, pg.master, pb.master, run_mean, run_var, xr, sums_r, pgr.master, pbr.master, run_mean_r,
            run_var_r, momentum, eps)
        ctx.save_for_backward(x, xr, mean, invstd, mask, mean_r, invstd_r)
        ctx.p = (pg, pb, pgr, pbr)
        ctx.stat_link = stat_link
        if stat_link is not None:
            stat_link.x, stat_link.mask, stat_link.mean, stat_link.x2, stat_link.mean2 = x, mask, mean, xr, mean_r
            stat_link.store = pg.store
        return y

    @staticmethod
    def backward(ctx, dy):
        x, xr, mean, invstd, mask, mean_r, invstd_r = ctx.saved_tensors
        pg, pb, pgr, pbr = ctx.p
        dy = dy.contiguous()
        C_ = _C()
        dg, db, finish = _bn_param_grads(pg.store, pg, pb, x.device)
        dgr, dbr, finish_r = _bn_param_grads(pgr.store, pgr, pbr, x.device)
        pre = ctx.stat_link.take(dy) if ctx.stat_link is not None else None
        if pre is not None and pre[1] is not None:  # both reductions came with dy (BnStatLink)
            dx, dxr = C_.bn_bwd_dual_from_sums(dy, mask, x, mean, invstd, pg.master, pb.master, dg, db, pre[0], xr,
                                               mean_r, invstd_r, pgr.master, pbr.master, dgr, dbr, pre[1])
        else:
            # one reduce sweep and one apply pass for both (dy and the mask read once per pass)
            dx, dxr = C_.bn_bwd_dual(dy, mask, x, mean, invstd, pg.master, pb.master, dg, db, xr, mean_r, invstd_r,
                                     pgr.master, pbr.master, dgr, dbr)
        finish()
        finish_r()
        return (dx, None, dxr) + (None,) * 13


def bn_act_dual(t, bn, tr, bn_r):
    """``relu(bn(t) + bn_r(tr))`` for ``t`` / ``tr`` = (conv output, epilogue sums) pairs and training-mode
    BatchNorms (models/resnet.BN); None when the fused kernel does not apply (caller runs the separate BNs)."""
    if not BN_DUAL or not (isinstance(t, tuple) and isinstance(tr, tuple)):
        return None
    (x, sums), (xr, sums_r) = t, tr
    if (sums is None or sums_r is None or not (bn.training and bn_r.training) or not _gpu(x)
            or x.dtype != torch.bfloat16 or xr.shape != x.shape or x.shape[-1] % 8 != 0):
        return None
    link = BnStatLink() if BN_BSTATS else None
    y = _BnActDual.apply(x, sums, xr, sums_r, bn.gamma.store.anchor, bn.gamma, bn.beta, bn.running_mean,
                         bn.running_var, bn_r.gamma, bn_r.beta, bn_r.running_mean, bn_r.running_var, bn.momentum,
                         bn.eps, link)
    if link is not None:
        y._k8s_bnstat = link
    return y


class _AvgPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = x.shape[1:3]
        return _C().avgpool_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return _C().avgpool_bwd(dy.contiguous(), *ctx.hw)


def global_avg_pool_nhwc(x):
    """[N, H, W, C] -> [N, C] mean; GPU bf16: one HIP pass each way (pool.hip), fp32 accumulation."""
    if _gpu(x) and x.dtype == torch.bfloat16 and x.shape[-1] % 8 == 0:
        return _AvgPoolNHWC.apply(x)
    return x.mean(dim=(1, 2))


# =========================================================================== transformer elementwise (K9)
def _swiglu_split(gu, blk):
    """(gate, up) fp32 views of a [.., 2F] gate|up tensor in either column layout (``SwiGLULink.blk``)."""
    F2 = gu.shape[-1] // 2
    if not blk:
        return gu.float().split(F2, -1)
    v = gu.float().reshape(*gu.shape[:-1], F2 // blk, 2, blk)
    return v[..., 0, :].reshape(*gu.shape[:-1], F2), v[..., 1, :].reshape(*gu.shape[:-1], F2)


def _swiglu_join(dg, du, blk):
    if not blk:
        return torch.cat([dg, du], -1)
    F2 = dg.shape[-1]
    lead = dg.shape[:-1]
    return torch.stack([dg.reshape(*lead, F2 // blk, blk), du.reshape(*lead, F2 // blk, blk)], -2).reshape(
        *lead, 2 * F2)


def _swiglu_bwd_any(gu, dy, blk):
    F2 = gu.shape[-1] // 2
    if _gpu(gu) and gu.dtype == torch.bfloat16 and F2 % 8 == 0:
        return _C().swiglu_bwd(gu, dy.contiguous(), blk)
    g, u = _swiglu_split(gu, blk)
    s_ = torch.sigmoid(g)
    d = dy.float()
    return _swiglu_join(d * u * s_ * (1 + g * (1 - s_)), d * g * s_, blk).to(gu.dtype)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, link=None, blk=0):
        gu = gu.contiguous()
        F2 = gu.shape[-1] // 2
        if _gpu(gu) and gu.dtype == torch.bfloat16 and F2 % 8 == 0:
            y = _C().swiglu_fwd(gu, blk)
        else:
            g, u = _swiglu_split(gu, blk)
            y = (torch.nn.functional.silu(g) * u).to(gu.dtype)
        ctx.save_for_backward(gu)
        ctx.link, ctx.blk = link, blk
        if link is not None:
            link.saved, link.dgu, link.blk = gu.reshape(-1, 2 * F2), None, blk
        return y

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        link = ctx.link
        if link is not None and link.dgu is not None:  # formed by the consuming linear's data gradient
            dgu, link.dgu, link.saved = link.dgu, None, None
            return dgu.reshape(gu.shape), None, None
        if link is not None:
            link.saved = None
        return _swiglu_bwd_any(gu, dy, ctx.blk), None, None


def swiglu(gu, link=None, blk: int = 0):
    """silu(gate) * up over a fused [.., 2F] gate|up projection (``blk``: its column layout, see ``SwiGLULink``).
    ``link``: see ``SwiGLULink``."""
    return _SwiGLU.apply(gu, link if SWIGLU_FUSE else None, blk)


# The gate|up projection's SwiGLU in its GEMM epilogue (gemm256.hip copy_out_swiglu; K8S_AMD_SWIGLU_EPI=0 for A/Bs).
SWIGLU_EPI = os.environ.get("K8S_AMD_SWIGLU_EPI", "1") != "0"


class _LinearSwiGLU(torch.autograd.Function):
    """h = silu(x Wg^T) * (x Wu^T) from ONE 4-wave GEMM whose epilogue writes both gu (what the backward reads) and h:
    the weight's rows are in the 64-blocked gate|up order, so every wave's 128 output columns hold a gate block and its
    up block (``SwiGLULink.blk`` = 64). Backward: dgu from the down projection's fused data gradient (``link``) or
    the SwiGLU-backward kernel, then the projection's data / weight gradients (``gemm.linear_bwd``)."""

    @staticmethod
    def forward(ctx, x, anchor, pw, link=None):
        x2 = x.reshape(-1, x.shape[-1])
        gu, h = _C().gemm_swiglu_fwd(x2, pw.weight)
        ctx.save_for_backward(x2, gu)
        ctx.pw, ctx.link, ctx.xshape = pw, link, x.shape
        if link is not None:
            link.saved, link.dgu, link.blk = gu, None, 64
        return h.reshape(*x.shape[:-1], h.shape[-1])

    @staticmethod
    def backward(ctx, dh):
        x2, gu = ctx.saved_tensors
        link, pw = ctx.link, ctx.pw
        if link is not None and link.dgu is not None:
            dgu, link.dgu, link.saved = link.dgu, None, None
        else:
            if link is not None:
                link.saved = None
            dgu = _swiglu_bwd_any(gu, dh.reshape(gu.shape[0], -1), 64)
        dx, dw, _ = _gemm().linear_bwd(dgu.reshape(gu.shape), x2, pw.weight, None, None, pw=pw, store=pw.store,
                                       need_db=False)
        if dw is not None:
            pw.store.deposit(pw, dw)
        return dx.reshape(ctx.xshape), None, None, None


# The QKV projection's rotary embedding in its GEMM epilogue (gemm256.hip copy_out_rope; K8S_AMD_ROPE_EPI=0 for A/Bs).
ROPE_EPI = os.environ.get("K8S_AMD_ROPE_EPI", "1") != "0"


class _LinearRope(torch.autograd.Function):
    """y = rope(x W^T) on the first ``rot_cols`` columns (the q / k heads, head dim 128) from one 4-wave GEMM with the
    rotation in its copy-out. Backward takes the gradient of the UN-rotated output -- what ``attention_qkv(...,
    rope_applied=True)`` returns (it rotates dqkv back, as for its own in-place rotation) -- so it is a plain linear
    backward."""

    @staticmethod
    def forward(ctx, x, anchor, pw, pos, table, rot_cols):
        x2 = x.reshape(-1, x.shape[-1])
        y = _C().gemm_rope(x2, pw.weight, pos, table, rot_cols)
        ctx.save_for_backward(x2)
        ctx.pw, ctx.xshape = pw, x.shape
        return y.reshape(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        (x2,) = ctx.saved_tensors
        pw = ctx.pw
        gy2 = gy.reshape(-1, gy.shape[-1]).contiguous()
        dx, dw, _ = _gemm().linear_bwd(gy2, x2, pw.weight, None, None, pw=pw, store=pw.store, need_db=False)
        if dw is not None:
            pw.store.deposit(pw, dw)
        return dx.reshape(ctx.xshape), None, None, None, None, None


def linear_rope(x, pw, pos, table, rot_cols: int):
    """(y, rotated): the projection ``x pw^T`` with the rotary embedding of its first ``rot_cols`` columns applied in
    the GEMM epilogue when the kernel takes the shape (``rotated`` True: pass ``rope_applied=True`` to
    ``attention_qkv``), else the plain projection (``rotated`` False: the attention op rotates)."""
    x2 = x.reshape(-1, x.shape[-1])
    if (ROPE_EPI and _gpu(x) and x.dtype == torch.bfloat16 and pw.weight.dtype == torch.bfloat16 and x2.is_contiguous()
            and pw.grad.dtype == torch.float32 and table.dim() == 3 and table.shape[1] == 64
            and bool(_C().gemm_rope_ok(x2.shape[0], pw.shape[0], x2.shape[1], rot_cols))):
        return _LinearRope.apply(x, pw.store.anchor, pw, pos, table, rot_cols), True
    return linear(x, pw), False


def linear_swiglu(x, pw, link=None, blk: int = 64):
    """silu(gate) * up of the fused gate|up projection ``pw`` ([2F, in], rows in ``blk``-blocked gate|up order) of x:
    on the GPU's whole-tile shapes one GEMM with the SwiGLU in its epilogue (``_LinearSwiGLU``), else the projection
    then ``swiglu``. ``link``: the SwiGLULink of the consuming down projection."""
    x2 = x.reshape(-1, x.shape[-1])
    F = pw.shape[0] // 2
    if (SWIGLU_EPI and blk == 64 and _gpu(x) and x.dtype == torch.bfloat16 and pw.weight.dtype == torch.bfloat16
            and x2.is_contiguous() and pw.grad.dtype == torch.float32
            and bool(_C().gemm_swiglu_fwd_ok(x2.shape[0], F, x2.shape[1]))):
        return _LinearSwiGLU.apply(x, pw.store.anchor, pw, link if SWIGLU_FUSE else None)
    return swiglu(linear(x, pw), link=link, blk=blk)


def rope_table(max_pos: int, dim: int, theta: float = 10000.0, device=None) -> torch.Tensor:
    """[max_pos, dim/2, 2] fp32 (cos, sin), built once on the host side of the step."""
    inv = 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], -1).float().to(device)


def _rope_ref(x, pos, table, inverse=False):
    T = x.shape[0]
    D = table.shape[1] * 2
    xs = x.float().reshape(T, -1, D)
    cs = table[pos.long()]  # [T, D/2, 2]
    c, s = cs[..., 0][:, None, :], cs[..., 1][:, None, :]
    if inverse:
        s = -s
    x1, x2 = xs[..., : D // 2], xs[..., D // 2:]
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)
    return out.reshape(x.shape).to(x.dtype)


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos, table):
        ctx.save_for_backward(pos, table)
        if _gpu(x) and x.dtype == torch.bfloat16:
            y = x.contiguous().clone()
            _C().rope_(y, pos, table, False)
            return y
        return _rope_ref(x, pos, table)

    @staticmethod
    def backward(ctx, dy):
        pos, table = ctx.saved_tensors
        if _gpu(dy) and dy.dtype == torch.bfloat16:
            d = dy.contiguous().clone()
            _C().rope_(d, pos, table, True)
            return d, None, None
        return _rope_ref(dy, pos, table, inverse=True), None, None


def rope(x, pos, table):
    """Rotary embedding of x [T, H*D] (token-major, rotate-half), pos [T] int32, table from ``rope_table``."""
    return _Rope.apply(x, pos, table)
