"""256 x 256-tile phased MFMA GEMM (gemm256.hip) vs plain PyTorch fp32 references.

Shapes are chosen so ``gemm256_eligible`` routes them to the large-tile kernel (>= 192 output tiles), with ragged
M / N edges, every operand layout (K-major / MN-major for A and B) and every epilogue.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from k8s_amd.ops._ext import load

    return load()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 512), (3000, 4104, 320), (2056, 6144, 64), (4096, 3080, 1024)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm256_layouts(cuda, M, N, K, ak, bk):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    A = a if ak else a.t().contiguous()
    B = b if bk else b.t().contiguous()
    c = _C().gemm(A, ak, B, bk, None, False, None, 0, None, False, 1.0, 1)
    assert c.shape == (M, N)
    assert _rel(c, ref) < 1e-2
    cf = _C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)
    assert _rel(cf, ref) < 1e-3


def test_gemm256_identity_asymmetric(cuda):
    """A = I with an asymmetric B at a size the 256 kernel takes: catches a transposed or permuted C write."""
    n = 4096
    eye = torch.eye(n, device=cuda).bfloat16()
    b = (torch.arange(n * 256, device=cuda).reshape(n, 256) % 251).float().bfloat16()  # exact in bf16
    b = b.repeat(1, 16)[:, :n].contiguous()
    for ak in (True, False):
        c = _C().gemm(eye, ak, b, True, None, True, None, 0, None, False, 1.0, 1)
        assert torch.equal(c, b.float().t())


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm256_epilogue(cuda, act, bias):
    torch.manual_seed(1)
    M, N, K = 4096, 3072, 768
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16() * 0.05
    bvec = torch.randn(N, device=cuda) if bias else None
    pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    y = _C().gemm(a, True, w, True, None, False, bvec, act, pre, False, 1.0, 1)
    p_ref = a.float() @ w.float().t() + (bvec if bias else 0.0)
    y_ref = [p_ref, torch.relu(p_ref), F.gelu(p_ref, approximate="tanh")][act]
    assert _rel(pre, p_ref) < 1e-2
    assert _rel(y, y_ref) < 1e-2
    # the plain bf16 store goes through the LDS-staged epilogue
    y2 = _C().gemm(a, True, w, True, None, False, bvec, act, None, False, 1.0, 1)
    assert _rel(y2, y_ref) < 1e-2


def test_gemm256_accumulate_alpha(cuda):
    """fp32 accumulate into an existing slot (the flat-gradient weight-gradient path) and alpha scaling."""
    torch.manual_seed(2)
    M, N, K = 4096, 4096, 2048
    g = torch.randn(K, M, device=cuda).bfloat16()  # wgrad: both operands MN-major
    x = torch.randn(K, N, device=cuda).bfloat16()
    ref = g.float().t() @ x.float()
    out = torch.full((M, N), 3.0, device=cuda)
    _C().gemm(g, False, x, False, out, True, None, 0, None, True, 1.0, 0)
    assert _rel(out - 3.0, ref) < 2e-3
    y = _C().gemm(g, False, x, False, None, True, None, 0, None, False, 0.25, 1)
    assert _rel(y, 0.25 * ref) < 2e-3
    yb = torch.full((M, N), 1.0, device=cuda, dtype=torch.bfloat16)
    _C().gemm(g, False, x, False, yb, False, None, 0, None, True, 1.0, 1)
    assert _rel(yb.float() - 1.0, ref) < 2e-2


def test_gemm256_long_k(cuda):
    """A long reduction (Llama down-projection / LM-head dgrad depth) stays accurate."""
    torch.manual_seed(3)
    M, N, K = 4096, 4096, 14336
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    c = _C().gemm(a, True, b, True, None, True, None, 0, None, False, 1.0, 1)
    assert _rel(c, ref) < 1e-3
