"""NHWC convolution entry points (K2).

``conv_fwd`` / ``conv_bwd`` take NHWC bf16 activations and KRSC weights and
return NHWC / KRSC results. The gfx950 implicit-GEMM kernels
(``csrc/kernels/conv_igemm.hip``) serve every shape they support; the
remaining shapes (and CPU tensors) go through ATen's convolution on a
channels-last view, which on ROCm is MIOpen.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _nhwc(y):
    return y.permute(0, 2, 3, 1).contiguous()


def conv_fwd(x, w, stride, padding):
    y = F.conv2d(_nchw(x), _nchw(w), None, stride, padding)
    return _nhwc(y)


def conv_bwd(gy, x, w, stride, padding, need_dx=True):
    dx, dw, _ = torch.ops.aten.convolution_backward(
        _nchw(gy), _nchw(x), _nchw(w), None, [stride, stride], [padding, padding], [1, 1], False, [0, 0], 1,
        [bool(need_dx), True, False])
    return (_nhwc(dx) if dx is not None else None), dw.permute(0, 2, 3, 1)
