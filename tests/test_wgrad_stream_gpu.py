"""Streaming tall-K weight gradient (wgrad_stream.hip) vs a plain PyTorch fp32 reference.

Shapes are ResNet-50 layers (1x1 at 56x56 / 28x28, strided 1x1 downsample, 3x3 stride 1 / 2) at a reduced batch,
with ragged row counts (N*Ho*Wo not a multiple of the 64-row step) and accumulation. The trainer sends only the
narrow (K or R*S*C = 64) layers here; K8S_AMD_WGS_ANY=1 opens the kernel to every case, and every tile variant
($K8S_AMD_WGS_TILE) the shape divides into is checked."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [  # N, H, C, K, R, stride, pad
    (8, 56, 64, 256, 1, 1, 0), (8, 56, 256, 64, 1, 1, 0), (8, 56, 64, 64, 1, 1, 0), (8, 56, 256, 128, 1, 1, 0),
    (8, 56, 256, 512, 1, 2, 0), (6, 28, 512, 128, 1, 1, 0), (6, 28, 128, 512, 1, 1, 0),
    (16, 56, 128, 128, 3, 2, 1), (7, 57, 64, 64, 3, 1, 1), (4, 14, 256, 256, 3, 1, 1),
]
TILES = ["128x64", "128x128", "256x128", "64x64"]


def _ref_dw(x, gy, K, C, R, stride, pad):
    xf = x.float().permute(0, 3, 1, 2).contiguous()
    gf = gy.float().permute(0, 3, 1, 2).contiguous()
    dw = torch.nn.grad.conv2d_weight(xf, (K, C, R, R), gf, stride=stride, padding=pad)
    return dw.permute(0, 2, 3, 1).contiguous()  # KRSC


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("N,H,C,K,R,stride,pad", CASES)
def test_wgrad_stream_matches_fp32(cuda, monkeypatch, N, H, C, K, R, stride, pad, tile):
    from k8s_amd.ops._ext import load

    kt, ct = map(int, tile.split("x"))
    if K % kt or (R * R * C) % ct:
        pytest.skip("tile does not divide the shape")
    monkeypatch.setenv("K8S_AMD_WGS_ANY", "1")
    monkeypatch.setenv("K8S_AMD_WGS_TILE", tile)
    C_ = load()
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    Ho = (H + 2 * pad - R) // stride + 1
    gy = torch.randn(N, Ho, Ho, K, device=cuda).bfloat16()
    if not C_.wgrad_stream_eligible(N, Ho, Ho, C, K, R, R):
        pytest.skip("more output tiles than the streaming kernel takes")
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
