"""ResNet-50 (v1.5) in NHWC bf16 on the k8s_amd op set.

Architecture = torchvision ``resnet50`` (bottleneck blocks [3, 4, 6, 3],
stride on the 3x3 conv, 25.56 M parameters), laid out for MI355X:
activations NHWC bf16, conv weights KRSC bf16 (flat-store copies of fp32
masters), BatchNorm statistics/affine in fp32, BN + residual-add + ReLU fused
into one kernel, loss = fused softmax cross-entropy.

This is the model of BASELINE config 1/2 ("ResNet-50 TfJob ... synthetic
ImageNet"); the reference itself only launches TF containers
(`/root/reference/pkg/spec/tf_job.go:87`), see SURVEY.md §2.6.
"""
from __future__ import annotations

import math
from typing import List

import torch
import torch.nn as nn

from k8s_amd.ops import nn as K
from k8s_amd.parallel.flat import ParamStore, init_const, init_kaiming_normal, init_uniform


class BN(nn.Module):
    def __init__(self, store: ParamStore, name: str, c: int, zero_init: bool = False):
        super().__init__()
        self.gamma = store.new(name + ".weight", (c,), init_const(0.0 if zero_init else 1.0), decay=False, lowp=False)
        self.beta = store.new(name + ".bias", (c,), init_const(0.0), decay=False, lowp=False)
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.momentum, self.eps = 0.1, 1e-5

    def forward(self, x, residual=None, relu=True, res_link=None, dy_link=None, sub2=False):
        sums = None
        if isinstance(x, tuple):  # (conv output, fused statistics)
            x, sums = x
        return K.batch_norm_act(x, self.gamma, self.beta, self.running_mean, self.running_var, residual, relu,
                                self.training, self.momentum, self.eps, sums=sums, res_link=res_link,
                                dy_link=dy_link, sub2=sub2)


class Conv(nn.Module):
    def __init__(self, store: ParamStore, name: str, cin: int, cout: int, k: int, stride: int = 1):
        super().__init__()
        self.w = store.new(name + ".weight", (cout, k, k, cin), init_kaiming_normal(cin * k * k))
        self.stride, self.pad = stride, k // 2

    def forward(self, x, grad_link=None):
        # BN statistics are accumulated in the conv epilogue (returned alongside y)
        return K.conv2d_nhwc(x, self.w, self.stride, self.pad, with_stats=True, grad_link=grad_link)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, store, name, cin, width, stride, downsample):
        super().__init__()
        cout = width * 4
        self.conv1 = Conv(store, name + ".conv1", cin, width, 1)
        self.bn1 = BN(store, name + ".bn1", width)
        self.conv2 = Conv(store, name + ".conv2", width, width, 3, stride)
        self.bn2 = BN(store, name + ".bn2", width)
        self.conv3 = Conv(store, name + ".conv3", width, cout, 1)
        self.bn3 = BN(store, name + ".bn3", cout, zero_init=True)
        self.down = None
        if downsample:
            self.down = Conv(store, name + ".downsample.0", cin, cout, 1, stride)
            self.down_bn = BN(store, name + ".downsample.1", cout)

    def forward(self, x, sub2=False):
        """``sub2``: the next block is a stride-2 downsample block -- bn3's apply pass also writes y[:, ::2, ::2]
        for its downsample convolution (ops.nn.SubLink)."""
        idn = x
        identity = self.down is None and x.requires_grad
        # identity block: x's two gradient contributions (residual via bn3, main path via conv1) are summed
        # inside conv1's dgrad epilogue instead of by a separate elementwise add
        link = K.GradLink() if identity else None
        # downsample block: x feeds conv1 and the downsample conv; their two dgrads are summed in the
        # epilogue of whichever runs second (shared link) instead of by autograd's separate add
        dlink = K.GradLink(shared=True) if (self.down is not None and x.requires_grad) else None
        # downsample block: bn3's ReLU mask is applied by the downsample BN's backward as it reads dy. The branch is
        # built FIRST so autograd (highest sequence number first) runs its backward LAST: the stride-2 1x1 dgrad
        # then accumulates onto conv1's dx (shared GradLink) instead of zero-filling the 3 parities it never writes
        mlink = dn = None
        if self.down is not None:
            mlink = K.MaskLink()
            dn = self.down(x, grad_link=dlink)
            # bn3 + downsample BN in one apply pass where the fused kernel applies (ops.nn.bn_act_dual)
            fuse = K.BN_DUAL and isinstance(dn, tuple) and dn[1] is not None and self.training and dn[0].is_cuda
            if not fuse:
                idn = self.down_bn(dn, relu=False, dy_link=mlink)
        t = self.conv1(x, grad_link=link or dlink)
        # bn1 / bn2 + ReLU: normalised on load by the consuming convolution where ops.nn.BN_ONLOAD and its kernels
        # take it (ops.nn.bn_relu_conv: no apply pass, no z tensor), else applied by the BN kernel
        t = K.bn_relu_conv(t, self.bn1, self.conv2)
        t = K.bn_relu_conv(t, self.bn2, self.conv3)
        if dn is not None and fuse:
            y = K.bn_act_dual(t, self.bn3, dn, self.down_bn)
            if y is not None:
                return y
            idn = self.down_bn(dn, relu=False, dy_link=mlink)
        return self.bn3(t, residual=idn, relu=True, res_link=link or mlink, sub2=sub2)


class ResNet(nn.Module):
    def __init__(self, store: ParamStore, layers: List[int] = (3, 4, 6, 3), num_classes: int = 1000,
                 in_ch: int = 3, width: int = 64, stem_s2d: bool = True):
        super().__init__()
        self.store = store
        # GPU: the 7x7/s2 stem runs as a 4x4 conv over the space-to-depth image (ops.nn.stem_conv_s2d)
        self.stem_s2d = stem_s2d
        # the stem reads a channel-padded image (3 -> 8 channels, zeros) so every NHWC row is 16-B aligned
        self.in_ch = in_ch
        self.stem_ch = (in_ch + 7) // 8 * 8
        self.conv1 = Conv(store, "conv1", self.stem_ch, width, 7, 2)
        self.bn1 = BN(store, "bn1", width)
        blocks = []
        cin = width
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(Bottleneck(store, "layer%d.%d" % (i + 1, j), cin, w, stride, j == 0))
                cin = w * 4
        self.blocks = nn.ModuleList(blocks)
        self.fc_w = store.new("fc.weight", (num_classes, cin), init_uniform(1.0 / math.sqrt(cin)))
        self.fc_b = store.new("fc.bias", (num_classes,), init_uniform(1.0 / math.sqrt(cin)), decay=False,
                              lowp=False)
        self.num_classes = num_classes

    def finalize(self, device, **kw):
        self.store.finalize(device, **kw)
        # zero the padded stem input channels' weights so padding is exact
        if self.stem_ch != self.in_ch:
            with torch.no_grad():
                self.conv1.w.master[..., self.in_ch:].zero_()
            self.store.refresh_lowp()
        return self.to(device)

    def prepare_input(self, images_nhwc: torch.Tensor, s2d: bool = None) -> torch.Tensor:
        """[N, H, W, 3] -> the stem's input: on the GPU (bf16) the [N, H/2+3, W/2+3, 16] space-to-depth image
        of ``stem_conv_s2d``; otherwise (or ``s2d=False``) [N, H, W, 8] (zero channel padding)."""
        use = self.stem_s2d if s2d is None else s2d
        if use and images_nhwc.is_cuda and images_nhwc.dtype == torch.bfloat16 and self.conv1.w.shape[1] == 7:
            return K.stem_s2d_input(images_nhwc, pad=3)
        if images_nhwc.shape[-1] == self.stem_ch:
            return images_nhwc
        pad = self.stem_ch - images_nhwc.shape[-1]
        return torch.nn.functional.pad(images_nhwc, (0, pad))

    def forward(self, x):
        if x.shape[-1] == 16 and self.stem_s2d and x.is_cuda:  # space-to-depth stem (prepare_input)
            t = K.stem_conv_s2d(x, self.conv1.w)
        else:
            t = self.conv1(x)
        # bn1 + ReLU + 3x3/s2 max pool: one fused pass each way on the GPU (the 112x112 BN output is never stored)
        y = K.bn_relu_maxpool(t, self.bn1)
        for i, b in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            y = b(y, sub2=nxt is not None and nxt.down is not None and nxt.down.stride == 2)
        y = K.global_avg_pool_nhwc(y)
        return K.linear(y, self.fc_w, self.fc_b)


def resnet50(store: ParamStore, num_classes: int = 1000) -> ResNet:
    return ResNet(store, (3, 4, 6, 3), num_classes)


def resnet_tiny(store: ParamStore, num_classes: int = 10) -> ResNet:
    """Small ResNet for CPU tests (same block structure, 1 block per stage, width 8)."""
    return ResNet(store, (1, 1, 1, 1), num_classes, width=8)
