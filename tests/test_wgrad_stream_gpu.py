"""Streaming tall-K weight gradient (wgrad_stream.hip) vs a plain PyTorch fp32 reference.

Shapes are ResNet-50 layers (1x1 at 56x56 / 28x28, strided 1x1 downsample, 3x3 stride 1 / 2) at a reduced batch,
with ragged row counts (N*Ho*Wo not a multiple of the 64-row step) and accumulation. The trainer sends only the
narrow (K or R*S*C = 64) layers here (128 x 64 tiles at K % 128 == 0, else 64 x 64); the cases it does not take
are skipped.""" 
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [  # N, H, C, K, R, stride, pad
    (8, 56, 64, 256, 1, 1, 0), (8, 56, 256, 64, 1, 1, 0), (8, 56, 64, 64, 1, 1, 0), (8, 56, 256, 128, 1, 1, 0),
    (8, 56, 256, 512, 1, 2, 0), (6, 28, 512, 128, 1, 1, 0), (6, 28, 128, 512, 1, 1, 0),
    (16, 56, 128, 128, 3, 2, 1), (7, 57, 64, 64, 3, 1, 1), (4, 14, 256, 256, 3, 1, 1),
]


def _ref_dw(x, gy, K, C, R, stride, pad):
    xf = x.float().permute(0, 3, 1, 2).contiguous()
    gf = gy.float().permute(0, 3, 1, 2).contiguous()
    dw = torch.nn.grad.conv2d_weight(xf, (K, C, R, R), gf, stride=stride, padding=pad)
    return dw.permute(0, 2, 3, 1).contiguous()  # KRSC


CASES += [(8, 56, 64, 128, 1, 1, 0), (6, 28, 64, 512, 1, 1, 0)]  # K % 128 == 0 with C = 64: the 128 x 64 tile


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", CASES)
def test_wgrad_stream_matches_fp32(cuda, N, H, C, K, R, stride, pad):
    from k8s_amd.ops._ext import load

    C_ = load()
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    Ho = (H + 2 * pad - R) // stride + 1
    gy = torch.randn(N, Ho, Ho, K, device=cuda).bfloat16()
    if not C_.wgrad_stream_eligible(N, Ho, Ho, C, K, R, R):
        pytest.skip("not a shape the streaming kernel takes")
    ref = _ref_dw(x, gy, K, C, R, stride, pad)
    dw = torch.full((K, R, R, C), float("nan"), device=cuda)  # must be fully overwritten
    C_.conv_wgrad(x, gy, dw, stride, pad, 1, 0, False)
    rel = ((dw - ref).norm() / ref.norm()).item()
    assert rel < 3e-3, rel
    dw2 = torch.ones_like(dw)
    C_.conv_wgrad(x, gy, dw2, stride, pad, 1, 0, True)  # accumulate
    assert ((dw2 - 1.0 - ref).norm() / ref.norm()).item() < 3e-3


def test_trainer_routing_narrow_only(cuda):
    """Without the override only the 64-wide layers stream (the generic kernel wins elsewhere)."""
    from k8s_amd.ops._ext import load

    C_ = load()
    assert C_.wgrad_stream_eligible(1024, 56, 56, 64, 256, 1, 1)
    assert C_.wgrad_stream_eligible(1024, 56, 56, 256, 64, 1, 1)
    assert not C_.wgrad_stream_eligible(1024, 14, 14, 256, 256, 3, 3)
    assert not C_.wgrad_stream_eligible(1024, 28, 28, 512, 128, 1, 1)
