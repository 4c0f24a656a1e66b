"""Staged-window 3x3 / stride-1 convolution (csrc/kernels/conv3x3.hip) against fp32 PyTorch references.

Forward (with the BN statistics epilogue), BatchNorm + ReLU normalised on load (including the zero padding, which
must stay zero), and the data gradient (the same kernel on flipped, in/out-swapped weights), at the three ResNet-50
stride-1 3x3 shapes; every case also runs with ``K8S_AMD_CONV3X3=0`` (the implicit GEMM) for the A/B switch.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (H = W, C, K): the stride-1 conv2 of ResNet-50 stages 1-3 (and the shapes of their data gradients)
SHAPES = [(56, 64, 64), (28, 128, 128), (14, 256, 256), (28, 256, 128)]


def _C():
    from k8s_amd.ops._ext import load

    return load()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def _ref_conv(x, w):
    return F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), padding=1).permute(0, 2, 3, 1)


@pytest.mark.parametrize("on", [True, False])
@pytest.mark.parametrize("H,C,K", SHAPES)
def test_conv3x3_forward_and_stats(cuda, monkeypatch, on, H, C, K):
    monkeypatch.setenv("K8S_AMD_CONV3X3", "1" if on else "0")
    torch.manual_seed(0)
    N = 3
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    w = (torch.randn(K, 3, 3, C, device=cuda) / (3 * C ** 0.5)).bfloat16()
    C_ = _C()
    stats = torch.zeros(C_.conv_stat_replicas, 2, K, device=cuda)
    y = C_.conv_fwd(x, w, 1, 1, 1, False, None, 0, stats)
    ref = _ref_conv(x, w)
    assert y.shape == (N, H, H, K)
    assert _rel(y, ref) < 1e-2
    yf = y.float().reshape(-1, K)
    s = stats.sum(0)
    torch.testing.assert_close(s[0], yf.sum(0), rtol=2e-3, atol=2e-2)
    torch.testing.assert_close(s[1], (yf * yf).sum(0), rtol=2e-3, atol=2e-2)


@pytest.mark.parametrize("H,C,K", SHAPES)
def test_conv3x3_bn_relu_on_load(cuda, H, C, K):
    """conv(relu(x * scale + shift)) with the transform applied to the staged window: against the fp32 reference of
    the normalised input -- a positive shift would make padded taps nonzero if the padding were transformed."""
    torch.manual_seed(1)
    N = 2
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    w = (torch.randn(K, 3, 3, C, device=cuda) / (3 * C ** 0.5)).bfloat16()
    scale = torch.rand(C, device=cuda) + 0.5
    shift = torch.rand(C, device=cuda) * 0.5 + 0.1  # > 0: relu(shift) != 0, so padding must not be transformed
    params = torch.stack([scale, shift]).contiguous()
    y = _C().conv_fwd(x, w, 1, 1, 1, False, None, 0, None, xform=params)
    z = torch.relu(x.float() * scale + shift).bfloat16()  # what the apply pass would have written
    assert _rel(y, _ref_conv(z, w)) < 1e-2


@pytest.mark.parametrize("on", [True, False])
@pytest.mark.parametrize("H,C,K", SHAPES)
def test_conv3x3_data_gradient(cuda, monkeypatch, on, H, C, K):
    """dx of a stride-1 3x3 conv through ops/conv.py (the staged-window kernel on the flipped weights)."""
    from k8s_amd.ops import conv

    monkeypatch.setenv("K8S_AMD_CONV3X3", "1" if on else "0")
    torch.manual_seed(2)
    N = 2
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    w = (torch.randn(K, 3, 3, C, device=cuda) / (3 * C ** 0.5)).bfloat16()
    gy = torch.randn(N, H, H, K, device=cuda).bfloat16()
    dx = conv.conv_bwd(gy, x, w, 1, 1, True, None)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), padding=1).backward(gy.float().permute(0, 3, 1, 2))
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("H,C", [(56, 64), (28, 128), (14, 256)])
def test_wgrad_tile_bn_relu_on_load(cuda, H, C):
    """The tiled 3x3 weight gradient with the activation operand normalised on load (wgrad_tile.hip XF): against the
    fp32 weight gradient of the conv of relu(x * scale + shift), padding untransformed (shift > 0)."""
    torch.manual_seed(3)
    N = 2
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    dy = torch.randn(N, H, H, C, device=cuda).bfloat16()
    scale = torch.rand(C, device=cuda) + 0.5
    shift = torch.rand(C, device=cuda) * 0.5 + 0.1
    params = torch.stack([scale, shift]).contiguous()
    dw = torch.empty(C, 3, 3, C, device=cuda)
    _C().conv_wgrad(x, dy, dw, 1, 1, 1, 0, False, xform=params)
    z = torch.relu(x.float() * scale + shift).bfloat16().float().permute(0, 3, 1, 2)
    wr = torch.zeros(C, C, 3, 3, device=cuda, requires_grad=True)
    F.conv2d(z, wr, padding=1).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(dw, wr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_resnet_bottleneck_onload_matches_apply_path(cuda, monkeypatch):
    """A stride-1 bottleneck at stage-1 width on the default (bn1 normalised on load by the staged kernels) against
    the same block with bn1 applied by the BN kernel (``K8S_AMD_BN_ONLOAD=1x1``): outputs, input gradient and every
    parameter gradient agree to bf16 rounding."""
    from k8s_amd.models import resnet
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore

    outs = {}
    for mode in ("3x3", "1x1", "0"):  # "0": every BN applied by its own pass (honoured)
        monkeypatch.setattr(K, "BN_ONLOAD", mode)
        torch.manual_seed(4)
        store = ParamStore()
        blk = resnet.Bottleneck(store, "b", 256, 64, 1, False)
        store.finalize(cuda, seed=11)
        store.by_name["b.bn3.weight"].master.fill_(1.0)  # zero-init gamma would cut the main path off
        blk.to(cuda)
        x = torch.randn(4, 56, 56, 256, device=cuda).bfloat16().requires_grad_(True)
        store.begin_step()
        y = blk(x)
        y.float().square().mean().backward()
        outs[mode] = (y.detach().float(), x.grad.float(), store.grad.clone())
    for other in ("1x1", "0"):
        a, b = outs["3x3"], outs[other]
        assert _rel(a[0], b[0]) < 1e-2
        assert _rel(a[1], b[1]) < 2e-2
        assert _rel(a[2], b[2]) < 2e-2

