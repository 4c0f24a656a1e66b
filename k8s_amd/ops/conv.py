"""NHWC convolution (K2) on the gfx950 implicit-GEMM MFMA kernel.

Activations NHWC bf16, weights KRSC bf16. Per product:

    fwd    y  = conv(x, w)                  ConvA implicit im2col (C % 64 == 0; per-16-B-unit decode for
                                            other C % 8 == 0, e.g. the 8-channel stem)
    wgrad  dw = dy^T . im2col(x)            fp32, split-K atomics, written straight into the
                                            parameter's flat gradient slot
    dgrad  1x1, stride 1: dx = dy . w       plain GEMM, w read N-major (no transpose)
           RxS, stride 1: dx = conv(dy, w') w' = spatially flipped, in/out-swapped w
                                            (tiny per-step transform), pad' = R-1-pad
           stride s     : split by output parity (a, b): each of the s*s sub-grids of dx is a stride-1
                          conv of dy with the taps r = a + pad - s*d (d = row offset into dy), written
                          through the GEMM epilogue's sub-grid row map; parities with no taps are zero

Every ResNet-50 shape runs on these kernels (plus the streaming tall-K weight gradient of
``csrc/kernels/wgrad_stream.hip`` for the 1x1 / strided layers with few output tiles): there is no vendor
candidate in the dispatch. Round 1 timed MIOpen against our kernels per shape; with the streaming weight
gradient the whole-step difference of forcing our kernels everywhere measured at noise level (ResNet-50 b1024:
8884/8869 vs 8967/8878 img/s, scripts/gpurun/bench_ab.sh) and a cold node no longer builds MIOpen kernels
(~16 s of the job-create -> step 0 latency in round 1, profiles/r01_coldstart.md). Shapes outside the kernels'
contract (C or K not a multiple of 8, dilation, CPU tensors) go through ATen's convolution on a channels-last
view; on the GPU they are counted in ``STATS`` and warned about once.
"""
from __future__ import annotations

import os
import warnings

import torch
import torch.nn.functional as F

from k8s_amd.ops._ext import load as _load


# (Round 2 built a BatchNorm-backward statistics epilogue for the data gradients -- the BN backward's reduction
# pass computed in the dgrad that produces its input; it measured a net loss twice, 10.61k vs 11.00k img/s in round 2
# and 12.02k vs 12.20k with only the long-K dgrads in round 3 (scripts/gpurun/env_ab.sh), and was removed.)

STATS = {"hip_fwd": 0, "aten_fwd": 0, "hip_wgrad": 0, "aten_wgrad": 0, "hip_dgrad": 0, "aten_dgrad": 0,
         "bn_bstats": 0}

# (Round 5 built weight gradients on a second HIP stream -- each conv's dW kernel forked off the compute stream to
# overlap the data gradient and BatchNorm passes after it. The streams co-ran, but the HBM-bound kernels stretched:
# +0.7 % at b1024, noise at the b3072 default (profiles/r05_wgrad_side_ab.md); its serial-vs-side gradient test then
# failed intermittently on the GPU (1 in ~3 runs, one fixed 2e-3 difference: an unordered operand somewhere in the
# fork / join), so it was removed rather than shipped off by default.)


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(y):
    return y.permute(0, 2, 3, 1).contiguous()


def _hip(*ts):
    return all(t.is_cuda and t.dtype == torch.bfloat16 for t in ts)


def fwd_ok(x, w):
    return _hip(x, w) and x.shape[-1] % 8 == 0 and w.shape[0] % 8 == 0


def _key(op, x, w, stride, padding):
    return "%s|%s|%s|%d|%d" % (op, "x".join(map(str, x.shape)), "x".join(map(str, w.shape)), stride, padding)


def fwd_uses_hip(x, w, stride, padding) -> bool:
    """Whether the forward of this shape runs on our kernel (every shape inside its contract does)."""
    return fwd_ok(x, w)


_WARNED = set()


def _vendor(op, x, w, stride, padding):
    """Count and warn once about a GPU product that has to use ATen/MIOpen (CPU tensors always use ATen: the
    plain-PyTorch oracle path, not counted)."""
    if x.is_cuda:
        STATS["aten_" + op] += 1
        key = _key("conv_" + op, x, w, stride, padding)
        if key not in _WARNED:
            _WARNED.add(key)
            warnings.warn("k8s_amd conv: %s is outside the MFMA kernels' shape contract; using ATen" % key)


def conv_fwd(x, w, stride, padding, stats=None):
    """y = conv(x, w); with ``stats`` (zeroed fp32 [R, 2, K]) the epilogue also accumulates the per-channel
    sum / sum-of-squares of y for the following BatchNorm (HIP path only)."""
    if fwd_uses_hip(x, w, stride, padding):
        STATS["hip_fwd"] += 1
        return _load().conv_fwd(x, w, stride, padding, 1, False, None, 0, stats)
    _vendor("fwd", x, w, stride, padding)
    return _nhwc(F.conv2d(_nchw(x), _nchw(w), None, stride, padding))


def _aten_bwd(gy, x, w, stride, padding, need_dx, need_dw):
    dx, dw, _ = torch.ops.aten.convolution_backward(
        _nchw(gy), _nchw(x), _nchw(w), None, [stride, stride], [padding, padding], [1, 1], False, [0, 0], 1,
        [bool(need_dx), bool(need_dw), False])
    return (_nhwc(dx) if dx is not None else None), (dw.permute(0, 2, 3, 1) if dw is not None else None)


def _wgrad_hip(C_, gy, x, out, stride, padding, acc, xform=None):
    """dW (fp32, written or accumulated into ``out``): the streaming tall-K kernel where it applies (1x1 and
    strided layers with few output tiles; decided in the binding), a plain split-K GEMM for other 1x1 / stride 1
    layers (no im2col decode), else the implicit-GEMM split-K kernel. ``xform`` (fp32 [2, C] BatchNorm scale |
    shift): the activation operand is relu(x * scale + shift), normalised as the GEMM loads it (the streaming
    kernel has no such path: those shapes take the GEMMs)."""
    K, R, S, C = out.shape
    N, Ho, Wo = gy.shape[0], gy.shape[1], gy.shape[2]
    if (R == 1 and S == 1 and stride == 1 and padding == 0
            and (xform is not None or not C_.wgrad_stream_eligible(N, Ho, Wo, C, K, R, S))):
        C_.gemm(gy.reshape(-1, K), False, x.reshape(-1, C), False, out.view(K, C), True, None, 0, None, acc, 1.0, 0,
                xform_b=xform, xform_c=C if xform is not None else 0)
    else:
        C_.conv_wgrad(x, gy, out, stride, padding, 1, 0, acc, xform=xform)


# which data-gradient kernels take a non-residual BatchNorm + ReLU's backward sums (nn.BnStatLink, relu): the 3x3
# staged-window kernel and the 1x1 tile kernel (K8S_AMD_BN_BSTATS_3X3 / _GEMM = 0 for the A/B)
BSTATS_3X3 = os.environ.get("K8S_AMD_BN_BSTATS_3X3", "1") != "0"
BSTATS_GEMM = os.environ.get("K8S_AMD_BN_BSTATS_GEMM", "1") != "0"
# a stage-entry block's residual BN: sums over conv1's dgrad completed by the downsample's strided dgrad
BSTATS_ENTRY = os.environ.get("K8S_AMD_BN_BSTATS_ENTRY", "1") != "0"
# a residual BN's sums in a masked-addend 1x1 dgrad too deep for gemm_short (the tile kernel: stage 4, K = 512)
BSTATS_TILE_MASK = os.environ.get("K8S_AMD_BN_BSTATS_TILE_MASK", "1") != "0"
# a BatchNorm + ReLU's sums in the parities of a stride-2 data gradient (ResNet's stage-entry bn1). Off by default:
# the parities' epilogue x reads cost what the reduction saves (b3072: +1.7 ms in the parity kernels for the 1.55 ms of
# the three reductions; same-box A/B within noise, profiles/r06_notes.md)
BSTATS_STRIDED = os.environ.get("K8S_AMD_BN_BSTATS_STRIDED", "0") != "0"
# ... including the two-BatchNorm form at a gemm_short depth (K = 256: that epilogue spills). Off by default: the
# plain product runs on gemm_short at 659 us, the tile kernel with the sums at 1,537 us, for a ~510 us reduction
# (scripts/microbench/bst_shapes.py, profiles/r06_bst_shapes.jsonl)
BSTATS_TILE_SHORT = os.environ.get("K8S_AMD_BN_BSTATS_TILE_SHORT", "0") != "0"


def _bn_sums(C_, bn_link, C, device):
    """Zeroed fp32 [conv_stat_replicas, 2, C] for a BnStatLink's sums: the BatchNorm store's per-step scratch (one fill
    per step) where it has one, else a fresh zeros tensor."""
    R = C_.conv_stat_replicas
    if bn_link.store is not None:
        from k8s_amd.ops.nn import _zero_scratch
        return _zero_scratch(bn_link.store, device, R * 2 * C).view(R, 2, C)
    return torch.zeros(R, 2, C, device=device, dtype=torch.float32)


def _dgrad_hip(C_, gy, w, padding, addend=None, bn_link=None):
    """dx on our kernels; with ``addend`` (bf16, shape of dx) a 1x1 dgrad accumulates onto it in the GEMM
    epilogue and returns it (the fused residual-gradient add). ``bn_link`` (nn.BnStatLink, with a masked addend):
    the epilogue also accumulates the BatchNorm-backward sums of dx for the BatchNorm(s) that produced x."""
    K, R, S, C = w.shape
    masked = addend is not None and not torch.is_tensor(addend)  # nn.MaskedGrad: (dy, packed ReLU mask)
    if (BSTATS_3X3 and bn_link is not None and bn_link.relu and bn_link.x is not None and addend is None and R == 3
            and S == 3
            and padding == 1 and gy.shape[1] == gy.shape[2] and bn_link.x.shape[:3] == gy.shape[:3]
            and C_.conv3x3_staged_ok(gy.shape[1], gy.shape[2], C, K, 3, 3, 1, 1)):
        sums = _bn_sums(C_, bn_link, C, gy.device)
        dx = C_.conv3x3_dgrad_bnstats(gy, C_.conv_dgrad_wtrans(w), bn_link.x, bn_link.gamma, bn_link.beta,
                                      bn_link.mean, bn_link.invstd, sums)
        bn_link.sums, bn_link.sums2, bn_link.dy_key = sums, None, (dx.data_ptr(), tuple(dx.shape))
        STATS["bn_bstats"] += 1
        return dx
    if R == 1 and S == 1 and padding == 0:
        N, H, W_, _ = gy.shape
        if masked and bn_link is not None and not bn_link.relu and bn_link.x is not None and \
                bn_link.x.shape == (N, H, W_, C) and \
                C_.gemm_short_bnstats_ok(N * H * W_, C, K, bn_link.x2 is not None):
            sums = _bn_sums(C_, bn_link, C, gy.device)
            sums2 = _bn_sums(C_, bn_link, C, gy.device) if bn_link.x2 is not None else None
            out = C_.dgrad_short_bnstats(
                gy.reshape(-1, K), w.reshape(K, C), addend.dy.view(-1, C), addend.mask, bn_link.x.view(-1, C),
                bn_link.mask, bn_link.mean, sums, None if sums2 is None else bn_link.x2.view(-1, C), bn_link.mean2,
                sums2).view(N, H, W_, C)
            bn_link.sums, bn_link.sums2, bn_link.dy_key = sums, sums2, (out.data_ptr(), tuple(out.shape))
            STATS["bn_bstats"] += 1
            return out
        if (masked and BSTATS_TILE_MASK and bn_link is not None and not bn_link.relu and bn_link.x is not None
                and bn_link.mask is not None and bn_link.x.shape == (N, H, W_, C) and N * H * W_ < 2 ** 31
                and (BSTATS_TILE_SHORT or bn_link.x2 is None or not C_.gemm_short_bnstats_ok(N * H * W_, C, K, False))):
            # the same on the tile kernel: K = 512 (the stage-4 identity blocks) and the two-BatchNorm form past
            # gemm_short's K = 128 (a downsample block's output read by the next block's conv1 at stages 3-4)
            out = torch.empty(N, H, W_, C, device=gy.device, dtype=gy.dtype)
            sums = _bn_sums(C_, bn_link, C, gy.device)
            dual = bn_link.x2 is not None
            sums2 = _bn_sums(C_, bn_link, C, gy.device) if dual else None
            C_.gemm_dgrad_bnstats_mask(gy.reshape(-1, K), w.reshape(K, C), out.view(-1, C), bn_link.x.view(-1, C),
                                       bn_link.mask, bn_link.mean, sums, addend.dy.view(-1, C), addend.mask,
                                       bn_link.x2.view(-1, C) if dual else None, bn_link.mean2 if dual else None,
                                       sums2)
            bn_link.sums, bn_link.sums2, bn_link.dy_key = sums, sums2, (out.data_ptr(), tuple(out.shape))
            STATS["bn_bstats"] += 1
            return out
        if (BSTATS_GEMM and bn_link is not None and bn_link.relu and bn_link.x is not None and addend is None
                and bn_link.x.shape == (N, H, W_, C) and C_.gemm_dgrad_bnstats_ok(N * H * W_, C, K)):
            sums = _bn_sums(C_, bn_link, C, gy.device)
            out = C_.gemm_dgrad_bnstats(gy.reshape(-1, K), w.reshape(K, C), bn_link.x.view(-1, C), bn_link.gamma,
                                        bn_link.beta, bn_link.mean, bn_link.invstd, sums).view(N, H, W_, C)
            bn_link.sums, bn_link.sums2, bn_link.dy_key = sums, None, (out.data_ptr(), tuple(out.shape))
            STATS["bn_bstats"] += 1
            return out
        if (BSTATS_ENTRY and addend is None and bn_link is not None and not bn_link.relu and not bn_link.last_full and bn_link.mask is not None
                and bn_link.x2 is None and bn_link.x is not None and bn_link.x.shape == (N, H, W_, C)
                and C_.gemm_short_bnstats_ok(N * H * W_, C, K, False)):
            # the first of two data gradients into a residual BN's output (a stage-entry block's conv1): the sums
            # over its values, completed by the downsample's strided dgrad (_dgrad_strided_hip)
            sums = _bn_sums(C_, bn_link, C, gy.device)
            out = C_.dgrad_short_bnstats(gy.reshape(-1, K), w.reshape(K, C), None, None, bn_link.x.view(-1, C),
                                         bn_link.mask, bn_link.mean, sums).view(N, H, W_, C)
            bn_link.sums, bn_link.sums2, bn_link.dy_key, bn_link.pending = sums, None, None, True
            STATS["bn_bstats"] += 1
            return out
        if masked:  # the epilogue reads dy and the mask bits itself: no materialised residual gradient
            out = torch.empty(N, H, W_, C, device=gy.device, dtype=gy.dtype)
            C_.gemm(gy.reshape(-1, K), True, w.reshape(K, C), False, out.view(-1, C), False, None, 0, None, True,
                    1.0, 1, add_src=addend.dy.view(-1, C), add_mask=addend.mask)
            return out
        if (addend is not None and bn_link is not None and bn_link.last_full and bn_link.x is not None
                and bn_link.mask is not None and bn_link.x.shape == (N, H, W_, C) and addend.is_contiguous()
                and C % 8 == 0 and N * H * W_ < 2 ** 31):
            # the second of two data gradients into a BatchNorm's output (nn.BnStatLink.last_full: the stem pool's,
            # 64 channels, the tile kernel): accumulated onto the first's, the sums taken over the final tensor
            sums = _bn_sums(C_, bn_link, C, gy.device)
            C_.gemm_dgrad_bnstats_mask(gy.reshape(-1, K), w.reshape(K, C), addend.view(-1, C), bn_link.x.view(-1, C),
                                       bn_link.mask, bn_link.mean, sums)
            bn_link.sums, bn_link.sums2, bn_link.dy_key = sums, None, (addend.data_ptr(), tuple(addend.shape))
            STATS["bn_bstats"] += 1
            return addend
        if addend is not None:
            C_.gemm(gy.reshape(-1, K), True, w.reshape(K, C), False, addend.view(-1, C), False, None, 0, None, True,
                    1.0, 1)
            return addend
        return C_.gemm(gy.reshape(-1, K), True, w.reshape(K, C), False, None, False, None, 0, None, False, 1.0,
                       1).reshape(N, H, W_, C)
    if masked:
        addend = addend.materialize()
    dx = C_.conv_fwd(gy, C_.conv_dgrad_wtrans(w), 1, R - 1 - padding, 1, False, None, 0, None)
    return dx if addend is None else dx.add_(addend)


def _parity_taps(R, a, pad, stride):
    """[(d, r)] sorted by d: taps r of an R-tap filter that reach output rows h = i*stride + a, read from dy
    row i + d. None if the offsets are not contiguous (cannot be one stride-1 correlation)."""
    taps = sorted(((a + pad - r) // stride, r) for r in range(R) if (a + pad - r) % stride == 0)
    if taps and [d for d, _ in taps] != list(range(taps[0][0], taps[0][0] + len(taps))):
        return None
    return taps


def strided_dgrad_ok(gy, w, stride, padding):
    K, R, S, C = w.shape
    if stride < 2 or K % 8 or C % 8:
        return False
    for a in range(stride):
        for b in range(stride):
            tr, ts = _parity_taps(R, a, padding, stride), _parity_taps(S, b, padding, stride)
            if tr is None or ts is None:
                return False
            if tr and ts and tr[0][0] != ts[0][0]:
                return False  # one pad for both dims
    return True


def _dgrad_strided_hip(C_, gy, w, stride, padding, H, W, addend=None, bn_link=None):
    """dx [N, H, W, C] of a stride-s conv on our implicit-GEMM kernel, one launch per output parity.

    With ``addend`` (bf16 [N, H, W, C], e.g. the gradient the block input already got from the other branch)
    every parity accumulates onto it in the GEMM epilogue and it is returned: no memset for the parities no
    tap reaches (they keep the addend) and no separate add pass."""
    K, R, S, C = w.shape
    N = gy.shape[0]
    # completing a residual BN's backward sums started by the first data gradient into `addend` (nn.BnStatLink
    # pending): the live parity's epilogue adds the changes it makes (gemm.hip BST sub-grid path)
    fix = (bn_link is not None and bn_link.pending and R == 1 and S == 1 and padding == 0 and addend is not None
           and torch.is_tensor(addend) and addend.is_contiguous() and bn_link.x is not None
           and bn_link.x.shape == addend.shape)
    if bn_link is not None and bn_link.pending and not fix:
        bn_link.sums, bn_link.pending = None, False  # cannot complete: the BN takes its own reduction
    # a BatchNorm + ReLU's sums (nn.BnStatLink relu kind: ResNet's bn1 before a stride-2 3x3 conv2): every parity
    # stores its own pixels and adds the sums over them (gemm.hip BST sub-grid path, relu kind)
    relu_sums = (BSTATS_STRIDED and bn_link is not None and bn_link.relu and bn_link.x is not None and addend is None
                 and not bn_link.pending and bn_link.x.shape == (N, H, W, C) and C > 64 and K % 64 == 0)
    rsums = _bn_sums(C_, bn_link, C, gy.device) if relu_sums else None
    parities = [(a, b) for a in range(stride) for b in range(stride)]
    empty = [(a, b) for a, b in parities
             if not _parity_taps(R, a, padding, stride) or not _parity_taps(S, b, padding, stride)]
    if addend is not None:
        dx = addend
    else:
        # parities no tap reaches are zero: one contiguous memset beats strided fills of the sub-grids
        # (1x1 stride-2: 3 of 4 parities; strided fills made that path 1.8x slower than MIOpen)
        dx = (torch.zeros if empty else torch.empty)(N, H, W, C, device=gy.device, dtype=gy.dtype)
    live = [(a, b, _parity_taps(R, a, padding, stride), _parity_taps(S, b, padding, stride))
            for a in range(stride) for b in range(stride)]
    live = [(a, b, tr, ts) for a, b, tr, ts in live if tr and ts]
    # every parity's [C, Tr, Ts, K] sub-weight gathered by one kernel (taps r*S + s, row-major over Tr x Ts)
    packed, offs = C_.conv_dgrad_wsub(w, [[r * S + s_ for _, r in tr for _, s_ in ts] for _, _, tr, ts in live])
    offs = offs.tolist()
    for i, (a, b, tr, ts) in enumerate(live):
        n = C * len(tr) * len(ts) * K
        wsub = packed[offs[i]:offs[i] + n].view(C, len(tr), len(ts), K)
        Hs, Ws = (H - a + stride - 1) // stride, (W - b + stride - 1) // stride
        if fix:
            C_.conv_fwd_subgrid(gy, wsub, -tr[0][0], Hs, Ws, dx, stride, a, b, True, bn_link.x, bn_link.mask,
                                bn_link.mean, bn_link.sums)
        elif relu_sums:
            C_.conv_fwd_subgrid(gy, wsub, -tr[0][0], Hs, Ws, dx, stride, a, b, False, bn_link.x, None, bn_link.mean,
                                rsums, bn_link.gamma, bn_link.beta, bn_link.invstd)
        else:
            C_.conv_fwd_subgrid(gy, wsub, -tr[0][0], Hs, Ws, dx, stride, a, b, addend is not None)
    if fix:
        bn_link.dy_key, bn_link.pending = (dx.data_ptr(), tuple(dx.shape)), False
    if relu_sums:
        bn_link.sums, bn_link.sums2, bn_link.dy_key = rsums, None, (dx.data_ptr(), tuple(dx.shape))
        STATS["bn_bstats"] += 1
    return dx


def conv_bwd(gy, x, w, stride, padding, need_dx, p=None, addend=None, xform=None, x_sub=None, bn_link=None):
    """Returns dx (+ ``addend``, e.g. the residual branch's gradient of the same tensor, fused into the
    dgrad epilogue where our kernel runs) or None; deposits dw into ``p``'s flat gradient slot. ``xform``: the
    convolution's input is relu(bn(x)) normalised on load (see ``_wgrad_hip``); dx is then the gradient w.r.t.
    that normalised input. ``x_sub``: a 1x1 / pad-0 convolution's input already subsampled by its stride
    (``nn._Conv2dNHWC`` with ``subsample_ok``): the weight gradient runs as the stride-1 product on it; ``x`` then only gives dx's shape."""
    K, R, S, C = w.shape
    C_ = _load() if gy.is_cuda else None
    if x_sub is not None:
        _wgrad_hip(C_, gy, x_sub, p.grad.view(p.shape), 1, 0, p.written)
        STATS["hip_wgrad"] += 1
        p.store._notify(p) if p.written else p.store.mark_written(p)
        p = None  # done
    hip = _hip(gy, x, w)
    if xform is not None and not (hip and C % 64 == 0 and K % 8 == 0 and p is not None
                                  and p.grad.dtype == torch.float32):
        raise RuntimeError("normalize-on-load weight gradient outside the kernels' contract")
    if addend is not None and not torch.is_tensor(addend) and not (
            hip and stride == 1 and K % 8 == 0 and C % 8 == 0):
        addend = addend.materialize()  # only the stride-1 dgrad on our kernels takes the (dy, mask) pair
    # ---- weight gradient
    dw_done = False
    if hip and C % 8 == 0 and K % 8 == 0 and p is not None and p.grad.dtype == torch.float32:
        STATS["hip_wgrad"] += 1
        acc = p.written
        _wgrad_hip(C_, gy, x, p.grad.view(p.shape), stride, padding, acc, xform)
        if acc:
            p.store._notify(p)
        else:
            p.store.mark_written(p)
        dw_done = True
    # ---- data gradient
    dx = None
    if need_dx:
        if hip and stride == 1 and K % 8 == 0 and C % 8 == 0:
            STATS["hip_dgrad"] += 1
            dx = _dgrad_hip(C_, gy, w, padding, addend, bn_link)
        elif hip and strided_dgrad_ok(gy, w, stride, padding):
            STATS["hip_dgrad"] += 1
            dx = _dgrad_strided_hip(C_, gy, w, stride, padding, x.shape[1], x.shape[2], addend, bn_link)
        else:
            _vendor("dgrad", x, w, stride, padding)
            dx, _ = _aten_bwd(gy, x, w, stride, padding, True, False)
            if addend is not None:
                dx = dx + addend
    return _finish_dw(dx, dw_done, p, gy, x, w, stride, padding)


# 1x1 / stride-2 / pad-0 convolutions (ResNet's downsample branch) as stride-1 GEMMs on the subsampled input: one
# subsample pass (pool.hip), then the forward (with the BN statistics, the 4-wave / short-K kernels) and the weight
# gradient take the plain-GEMM paths instead of the strided implicit-GEMM gather; the data gradient keeps the
# strided parity path (it accumulates onto the block input's other gradient). K8S_AMD_SUB1X1=0 for the A/B.
SUB1X1 = os.environ.get("K8S_AMD_SUB1X1", "1") != "0"


def subsample_ok(x, w, stride, padding) -> bool:
    K, R, S, C = w.shape
    return (SUB1X1 and stride > 1 and R == 1 and S == 1 and padding == 0 and _hip(x, w) and C % 64 == 0
            and K % 8 == 0 and x.is_contiguous())


def _finish_dw(dx, dw_done, p, gy, x, w, stride, padding):
    if not dw_done and p is not None:
        _vendor("wgrad", x, w, stride, padding)
        _, dw = _aten_bwd(gy, x, w, stride, padding, False, True)
        p.store.deposit(p, dw)
    return dx
