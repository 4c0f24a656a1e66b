"""Short-K streaming GEMM (gemm_short.hip) vs plain PyTorch fp32 references.

The kernel takes the 1x1 convolutions with a reduction of 64 / 128 / 256 channels and N % 128 == 0 output
channels: the forward (K-major weights, optional BatchNorm statistics and normalize-on-load of the input) and the
data gradient (weights read transposed; plain, accumulating, or onto a masked addend). Row counts with tails
(M % 32 != 0) exercise the buffer-descriptor range checks, and the large case runs many tiles per wave so the
counted-wait steady state of the prefetch ring is covered, not only its first round.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _C():
    from k8s_amd.ops._ext import load

    return load()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def _unpack_bits(mask, shape):
    bits = mask.reshape(-1, 1).int()
    return ((bits >> torch.arange(8, device=mask.device).int()) & 1).reshape(shape).bool()


def _bn_params(C, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    scale = (torch.rand(C, generator=g) * 1.5 + 0.25) * torch.where(torch.rand(C, generator=g) < 0.2, -1.0, 1.0)
    shift = torch.randn(C, generator=g) * 0.5
    return torch.cat([scale, shift]).float().to(device).contiguous()


# (rows M, reduction K, output columns N)
FWD = [(147, 64, 256), (6272, 128, 512), (1000, 256, 1024), (4096, 64, 128), (3136, 256, 256),
       (600017, 128, 128), (300007, 64, 256)]


@pytest.mark.parametrize("M,K,N", FWD)
@pytest.mark.parametrize("stats", [True, False])
@pytest.mark.parametrize("xform", [False, True])
def test_short_conv1x1_fwd(cuda, M, K, N, stats, xform):
    C_ = _C()
    assert C_.gemm_short_ok(M, N, K)
    torch.manual_seed(1)
    x = (torch.randn(1, 1, M, K, device=cuda) * 2 + 0.3).bfloat16()
    w = (torch.randn(N, 1, 1, K, device=cuda) * K ** -0.5).bfloat16()
    p = _bn_params(K, cuda, 2) if xform else None
    st = torch.zeros(C_.conv_stat_replicas, 2, N, device=cuda) if stats else None
    y = C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, st, xform=p)
    a = x.reshape(M, K).float()
    if xform:  # the kernel rounds relu(x * scale + shift) to bf16 before the MFMA, as the BN apply pass would
        a = (a.double() * p[:K].double() + p[K:].double()).float().clamp_min(0.0).bfloat16().float()
    ref = a @ w.reshape(N, K).float().t()
    yy = y.reshape(M, N)
    assert _rel(yy, ref) < 1e-2
    if stats:  # sum / sum of squares of the stored bf16 values
        yf = yy.float()
        torch.testing.assert_close(st.sum(0)[0], yf.sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(st.sum(0)[1], (yf * yf).sum(0), rtol=1e-4, atol=1e-2)


DGRAD = [(147, 64, 256), (6272, 128, 512), (1000, 256, 384), (4104, 128, 128), (600017, 256, 128),
         (300007, 64, 256)]


@pytest.mark.parametrize("M,K,N", DGRAD)
@pytest.mark.parametrize("mode", ["store", "accumulate", "masked", "addend"])
def test_short_dgrad(cuda, M, K, N, mode):
    """dx[M, N] = dy[M, K] . w[K, N] (w read transposed), stored, accumulated onto dx, or added to a second tensor
    under packed ReLU bits (the identity block's residual gradient)."""
    C_ = _C()
    assert C_.gemm_short_ok(M, N, K)
    torch.manual_seed(3)
    gy = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(K, N, device=cuda) * K ** -0.5).bfloat16()
    ref = gy.float() @ w.float()
    if mode == "store":
        out = C_.gemm(gy, True, w, False, None, False, None, 0, None, False, 1.0, 1)
    elif mode == "accumulate":
        base = torch.randn(M, N, device=cuda).bfloat16()
        ref = ref + base.float()
        out = base.clone()
        C_.gemm(gy, True, w, False, out, False, None, 0, None, True, 1.0, 1)
    else:
        dy = torch.randn(M, N, device=cuda).bfloat16()
        mask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)
        if mode == "addend":
            mask.fill_(255)
        on = _unpack_bits(mask, (M, N))
        ref = ref + torch.where(on, dy.float(), torch.zeros_like(dy.float()))
        out = torch.full((M, N), 7.0, device=cuda, dtype=torch.bfloat16)  # overwritten, never read
        C_.gemm(gy, True, w, False, out, False, None, 0, None, True, 1.0, 1, dy, mask)
        # bit-identical to materialising (bit ? dy : 0) and accumulating onto it (the two-step form)
        dres = C_.mask_apply(dy, mask)
        C_.gemm(gy, True, w, False, dres, False, None, 0, None, True, 1.0, 1)
        assert torch.equal(dres, out)
    assert _rel(out, ref) < 1e-2


@pytest.mark.parametrize("M,K,N", [(6272, 128, 512), (1000, 256, 384)])
def test_short_matches_tile_kernel(cuda, M, K, N, monkeypatch):
    """The streaming kernel and gemm.hip's tile kernel (K8S_AMD_GEMM_SHORT=0) agree to bf16 rounding."""
    C_ = _C()
    torch.manual_seed(4)
    gy = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(K, N, device=cuda) * K ** -0.5).bfloat16()
    a = C_.gemm(gy, True, w, False, None, False, None, 0, None, False, 1.0, 1)
    monkeypatch.setenv("K8S_AMD_GEMM_SHORT", "0")
    assert not C_.gemm_short_ok(M, N, K)
    b = C_.gemm(gy, True, w, False, None, False, None, 0, None, False, 1.0, 1)
    assert _rel(a, b) < 4e-3


def test_short_contract(cuda):
    C_ = _C()
    assert C_.gemm_short_ok(1024, 256, 128)
    assert not C_.gemm_short_ok(1024, 192, 128)   # N % 128
    assert not C_.gemm_short_ok(1024, 256, 512)   # long reduction: the tile kernels
    assert not C_.gemm_short_ok(1024, 256, 96)
    # > 2 GiB operands run as row-chunked launches (each under the 32-bit buffer-offset range)
    assert C_.gemm_short_ok(1 << 24, 256, 128)


@pytest.mark.parametrize("M,K,N", [(6272, 128, 256), (10007, 64, 256)])
def test_short_row_chunked_launches_match_one_launch(cuda, M, K, N, monkeypatch):
    """Products above 2 GiB run as consecutive row ranges (gemm_short_rows_per_launch); K8S_AMD_GEMM_SHORT_ROWS
    forces that path at a small size. Outputs are bit-identical to one launch (rows are independent); the BN
    statistics accumulate across the launches; the masked dgrad reads its mask bytes from each range's offset."""
    C_ = _C()
    torch.manual_seed(5)
    x = (torch.randn(1, 1, M, K, device=cuda) + 0.2).bfloat16()
    w = (torch.randn(N, 1, 1, K, device=cuda) * K ** -0.5).bfloat16()
    p = _bn_params(K, cuda, 6)
    gy = torch.randn(M, K, device=cuda).bfloat16()
    wd = (torch.randn(K, N, device=cuda) * K ** -0.5).bfloat16()
    dy = torch.randn(M, N, device=cuda).bfloat16()
    mask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)

    def run():
        st = torch.zeros(C_.conv_stat_replicas, 2, N, device=cuda)
        y = C_.conv_fwd(x, w, 1, 0, 1, False, None, 0, st, xform=p)
        out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        C_.gemm(gy, True, wd, False, out, False, None, 0, None, True, 1.0, 1, dy, mask)
        torch.cuda.synchronize()
        return y, st.sum(0), out

    y1, s1, d1 = run()
    monkeypatch.setenv("K8S_AMD_GEMM_SHORT_ROWS", "1024")  # 7-10 launches, the last one ragged
    y2, s2, d2 = run()
    assert torch.equal(y1, y2)
    assert torch.equal(d1, d2)
    torch.testing.assert_close(s2, s1, rtol=1e-5, atol=1e-2)
