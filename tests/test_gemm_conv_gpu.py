"""MFMA GEMM / implicit-GEMM conv kernels vs plain PyTorch fp32 references."""
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


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (1000, 520, 192), (4096, 4096, 1024), (129, 136, 128),
                                   (8, 1000, 2048),
                                   # ragged K (K % 64 != 0, read as zeros): the 1000-class head's data gradient
                                   (1024, 2048, 1000), (136, 264, 104)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_layouts(cuda, M, N, K, ak, bk):
    if (not ak and M % 8) or (not bk and N % 8):
        pytest.skip("MN-major operands need a multiple of 8")
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


def test_gemm_identity_asymmetric(cuda):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 128
    eye = torch.eye(n, device=cuda).bfloat16()
    b = (torch.arange(n * n, device=cuda).reshape(n, n) % 251).float().bfloat16()  # asymmetric, exact in bf16
    c = _C().gemm(eye, True, b, True, None, True, None, 0, None, False, 1.0, 1)
    assert torch.equal(c, b.float().t())


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (1000, 776, 192), (300, 132, 128), (40, 64, 64)])
@pytest.mark.parametrize("with_pre", [True, False])
def test_gemm_epilogue(cuda, act, M, N, K, with_pre):
    """bias / ReLU / GELU / pre-activation epilogue: the LDS-staged lean path (N % 8 == 0) and the general one."""
    torch.manual_seed(1)
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.randn(N, K, device=cuda).bfloat16() * 0.05
    bias = torch.randn(N, device=cuda)
    pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16) if with_pre else None
    y = _C().gemm(a, True, w, True, None, False, bias, act, pre, False, 1.0, 1)
    p_ref = a.float() @ w.float().t() + bias
    y_ref = [p_ref, torch.relu(p_ref), F.gelu(p_ref, approximate="tanh")][act]
    if with_pre:
        assert _rel(pre, p_ref) < 1e-2
    assert _rel(y, y_ref) < 1e-2


def test_gemm_splitk_accumulate(cuda):
    torch.manual_seed(2)
    M, N, K = 64, 128, 50000  # tall-K weight-gradient shape
    a = torch.randn(K, M, device=cuda).bfloat16()
    b = torch.randn(K, N, device=cuda).bfloat16()
    ref = a.float().t() @ b.float()
    out = torch.full((M, N), 3.0, device=cuda)
    _C().gemm(a, False, b, False, out, True, None, 0, None, True, 1.0, 0)  # accumulate onto 3.0
    assert _rel(out - 3.0, ref) < 2e-3
    out2 = _C().gemm(a, False, b, False, None, True, None, 0, None, False, 1.0, 0)
    assert _rel(out2, ref) < 2e-3


CONV_CASES = [
    # N, H, W, C, K, R, stride, pad
    (4, 14, 14, 64, 64, 3, 1, 1),
    (2, 28, 28, 128, 128, 3, 2, 1),
    (3, 7, 7, 512, 2048, 1, 1, 0),
    (2, 16, 16, 256, 128, 1, 2, 0),
    (2, 9, 11, 64, 72, 3, 1, 1),
]


SMALL_C_CASES = [(2, 32, 32, 8, 64, 7, 2, 3), (2, 15, 13, 24, 40, 3, 1, 1), (1, 9, 9, 8, 16, 1, 1, 0)]


@pytest.mark.parametrize("case", CONV_CASES + SMALL_C_CASES)
def test_conv_fwd(cuda, case):
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(3)
    x = torch.randn(N, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(K, R, R, C, device=cuda) * 0.05).bfloat16()
    y = _C().conv_fwd(x, w, st, pad, 1, False, None, 0, None)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, st, pad).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES + [(2, 32, 32, 8, 64, 7, 2, 3)])
def test_conv_wgrad(cuda, case):
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(4)
    x = torch.randn(N, H, W, C, device=cuda).bfloat16()
    Ho = (H + 2 * pad - R) // st + 1
    Wo = (W + 2 * pad - R) // st + 1
    dy = torch.randn(N, Ho, Wo, K, device=cuda).bfloat16()
    dw = torch.empty(K, R, R, C, device=cuda)
    _C().conv_wgrad(x, dy, dw, st, pad, 1, 0, False)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(False)
    wr = torch.zeros(K, C, R, R, device=cuda, requires_grad=True)
    F.conv2d(xr, wr, None, st, pad).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(dw, wr.grad.permute(0, 2, 3, 1)) < 5e-3


# + reductions (the dgrad's K) that are not a multiple of 64 (K % 8 is the contract)
@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[6] == 1] + [(2, 15, 13, 24, 40, 3, 1, 1),
                                                                         (1, 9, 9, 8, 16, 1, 1, 0),
                                                                         (2, 8, 8, 8, 8, 1, 1, 0),
                                                                         (2, 6, 6, 32, 32, 3, 1, 1)])
def test_conv_dgrad_stride1(cuda, case):
    from k8s_amd.ops import conv as kc

    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(5)
    x = torch.randn(N, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(K, R, R, C, device=cuda) * 0.05).bfloat16()
    dy = torch.randn(N, H, W, K, device=cuda).bfloat16()
    dx = kc.conv_bwd(dy, x, w, st, pad, True, None)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), None, st, pad).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES + SMALL_C_CASES[:1])
def test_conv_fwd_bn_stats_epilogue(cuda, case):
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(6)
    x = torch.randn(N, H, W, C, device=cuda).bfloat16()
    w = (torch.randn(K, R, R, C, device=cuda) * 0.05).bfloat16()
    stats = torch.zeros(_C().conv_stat_replicas, 2, K, device=cuda)
    y = _C().conv_fwd(x, w, st, pad, 1, False, None, 0, stats)
    yf = y.float().reshape(-1, K)
    tot = stats.sum(0)
    assert _rel(tot[0], yf.sum(0)) < 1e-3
    assert _rel(tot[1], (yf * yf).sum(0)) < 1e-3


@pytest.mark.parametrize("F2", [2 * 256, 2 * 2056])
def test_elementwise_kernels(cuda, F2):
    from k8s_amd.ops import nn as K

    torch.manual_seed(8)
    T = 96
    gu = torch.randn(T, F2, device=cuda).bfloat16()
    y = _C().swiglu_fwd(gu)
    g, u = gu.float().split(F2 // 2, -1)
    assert _rel(y, F.silu(g) * u) < 1e-2
    dy = torch.randn(T, F2 // 2, device=cuda).bfloat16()
    gg = gu.float().requires_grad_(True)
    a, b = gg.split(F2 // 2, -1)
    (F.silu(a) * b).backward(dy.float())
    assert _rel(_C().swiglu_bwd(gu, dy), gg.grad) < 1e-2
    if (F2 // 2) % 64 == 0:  # the 64-blocked gate|up layout (Llama's fused gate|up epilogue) against the CPU op
        gcpu = gu.cpu()
        assert _rel(_C().swiglu_fwd(gu, 64).cpu(), K.swiglu(gcpu.float(), blk=64)) < 1e-2
        gq = gcpu.float().requires_grad_(True)
        K.swiglu(gq, blk=64).backward(dy.cpu().float())
        assert _rel(_C().swiglu_bwd(gu, dy, 64).cpu(), gq.grad) < 1e-2
    # rope forward then inverse = identity; matches the reference
    H, D = 4, 128
    x = torch.randn(T, H * D, device=cuda).bfloat16()
    pos = torch.arange(T, device=cuda, dtype=torch.int32)
    table = K.rope_table(512, D, 500000.0, cuda)
    xr = x.clone()
    _C().rope_(xr, pos, table, False)
    assert _rel(xr, K._rope_ref(x, pos, table)) < 1e-2
    _C().rope_(xr, pos, table, True)
    assert _rel(xr, x) < 2e-2
    # gelu / relu backward and column sums
    pre = torch.randn(T, 512, device=cuda).bfloat16()
    d = torch.randn(T, 512, device=cuda).bfloat16()
    pp = pre.float().requires_grad_(True)
    F.gelu(pp, approximate="tanh").backward(d.float())
    assert _rel(_C().gelu_bwd(d, pre), pp.grad) < 1e-2
    assert _rel(_C().relu_bwd(d, torch.relu(pre)), d.float() * (pre.float() > 0)) < 1e-3
    assert _rel(_C().colsum(d), d.float().sum(0)) < 1e-3


@pytest.mark.parametrize("shape,ksp", [((2, 112, 112, 64), (3, 2, 1)), ((3, 9, 7, 16), (3, 2, 1)),
                                       ((2, 8, 8, 8), (2, 2, 0)), ((2, 10, 10, 8), (3, 1, 1))])
def test_maxpool_nhwc(cuda, shape, ksp):
    from k8s_amd.ops import nn as K

    torch.manual_seed(9)
    k, s, p = ksp
    x = torch.randn(*shape, device=cuda).bfloat16().requires_grad_(True)
    y = K.max_pool_nhwc(x, k, s, p)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p)
    assert torch.equal(y.float(), yr.permute(0, 2, 3, 1))
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(x.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2


# stride-2 data gradients (ResNet-50 v1.5 strided 3x3 and 1x1 downsample, the 7x7 stem; odd sizes) on the
# parity-decomposed implicit GEMM with the sub-grid epilogue
@pytest.mark.parametrize("N,H,C,K,R,st,pad", [(4, 56, 128, 128, 3, 2, 1), (4, 28, 256, 512, 1, 2, 0),
                                              (2, 15, 64, 128, 3, 2, 1), (2, 32, 8, 64, 7, 2, 3),
                                              (3, 14, 512, 1024, 1, 2, 0),
                                              # K (and C) % 64 != 0: the per-unit implicit-GEMM decode
                                              (8, 8, 32, 32, 3, 2, 1), (2, 9, 24, 40, 3, 2, 1),
                                              (3, 8, 16, 24, 1, 2, 0)])
def test_conv_dgrad_strided(cuda, N, H, C, K, R, st, pad):
    from k8s_amd.ops import conv as kc

    torch.manual_seed(7)
    Ho = (H + 2 * pad - R) // st + 1
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    w = (torch.randn(K, R, R, C, device=cuda) * 0.05).bfloat16()
    dy = torch.randn(N, Ho, Ho, K, device=cuda).bfloat16()
    assert kc.strided_dgrad_ok(dy, w, st, pad)
    dx = kc._dgrad_strided_hip(_C(), dy, w, st, pad, H, H)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), None, st, pad).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


# the residual-gradient add fused into the strided dgrad: every parity accumulates onto the addend in the
# GEMM epilogue; parities no tap reaches keep the addend unchanged
@pytest.mark.parametrize("N,H,C,K,R,st,pad", [(4, 28, 256, 512, 1, 2, 0), (2, 15, 64, 128, 3, 2, 1),
                                              (3, 14, 512, 1024, 1, 2, 0), (8, 8, 32, 32, 3, 2, 1)])
def test_conv_dgrad_strided_accumulate(cuda, N, H, C, K, R, st, pad):
    from k8s_amd.ops import conv as kc

    torch.manual_seed(11)
    Ho = (H + 2 * pad - R) // st + 1
    x = torch.randn(N, H, H, C, device=cuda).bfloat16()
    w = (torch.randn(K, R, R, C, device=cuda) * 0.05).bfloat16()
    dy = torch.randn(N, Ho, Ho, K, device=cuda).bfloat16()
    addend = torch.randn(N, H, H, C, device=cuda).bfloat16()
    ref_add = addend.float().clone()
    out = kc._dgrad_strided_hip(_C(), dy, w, st, pad, H, H, addend)
    assert out.data_ptr() == addend.data_ptr()
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, w.float().permute(0, 3, 1, 2), None, st, pad).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(out, xr.grad.permute(0, 2, 3, 1) + ref_add) < 1e-2


def test_linear_head_1000_classes_no_fallback(cuda):
    """The ResNet-50 fc (N = 1000, not a multiple of the 64-deep k-step of the dgrad product) stays on our
    kernels: dgrad zero-pads N, fwd / wgrad need only N % 8."""
    from k8s_amd.ops import gemm

    torch.manual_seed(3)
    M, N, K = 256, 1000, 2048
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.02).bfloat16()
    gy = torch.randn(M, N, device=cuda).bfloat16()
    before = dict(gemm.FALLBACKS)
    y, saved = gemm.linear_fwd(x, w, None)
    dx, dw, db = gemm.linear_bwd(gy, x, w, saved, None)
    assert gemm.FALLBACKS == before
    assert _rel(y, x.float() @ w.float().t()) < 1e-2
    assert _rel(dx, gy.float() @ w.float()) < 1e-2
    assert _rel(dw, gy.float().t() @ x.float()) < 1e-2
    assert _rel(db, gy.float().sum(0)) < 1e-2


@pytest.mark.parametrize("N", [10, 6, 13])
@pytest.mark.parametrize("act", [None, "relu"])
def test_linear_ragged_n_no_fallback(cuda, N, act):
    """A 10-class head (N % 4 != 0) runs forward and backward on our kernels over zero-padded weight rows."""
    from k8s_amd.ops import gemm

    torch.manual_seed(5)
    M, K = 64, 256
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    b = torch.randn(N, device=cuda)
    gy = torch.randn(M, N, device=cuda).bfloat16()
    before = dict(gemm.FALLBACKS)
    y, saved = gemm.linear_fwd(x, w, b, act)
    dx, dw, db = gemm.linear_bwd(gy, x, w, saved, act)
    assert gemm.FALLBACKS == before
    pre = x.float() @ w.float().t() + b
    ref = torch.relu(pre) if act == "relu" else pre
    assert y.shape == (M, N) and y.is_contiguous()
    assert _rel(y, ref) < 1e-2
    g = gy.float() * (pre > 0) if act == "relu" else gy.float()
    assert _rel(dx, g @ w.float()) < 2e-2
    assert _rel(dw, g.t() @ x.float()) < 2e-2
    assert _rel(db, g.sum(0)) < 2e-2


def _unpack_bits(mask, shape):
    bits = mask.reshape(-1, 1).int()
    return ((bits >> torch.arange(8, device=mask.device).int()) & 1).reshape(shape).bool()


@pytest.mark.parametrize("with_mask", [True, False])
def test_gemm_masked_addend_epilogue(cuda, with_mask):
    """1x1 dgrad accumulating onto a separate addend masked by packed ReLU bits (identity-block residual
    gradient read as (dy, mask) instead of a materialised dres): out = gy.w + (bit ? dy : 0)."""
    torch.manual_seed(7)
    C_ = _C()
    M, K, C = 3000, 128, 192
    gy = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(K, C, device=cuda) * 0.1).bfloat16()
    dy = torch.randn(M, C, device=cuda).bfloat16()
    mask = torch.randint(0, 256, (M * C // 8,), device=cuda, dtype=torch.uint8)
    out = torch.full((M, C), 7.0, device=cuda, dtype=torch.bfloat16)  # overwritten, never read
    C_.gemm(gy, True, w, False, out, False, None, 0, None, True, 1.0, 1, dy, mask if with_mask else None)
    on = _unpack_bits(mask, (M, C)) if with_mask else torch.ones(M, C, dtype=torch.bool, device=cuda)
    ref = gy.float() @ w.float() + torch.where(on, dy.float(), torch.zeros_like(dy.float()))
    assert _rel(out, ref) < 1e-2
    # the same as the two-step form: materialise bit ? dy : 0, then accumulate onto it in place
    if with_mask:
        dres = C_.mask_apply(dy, mask)
        assert torch.equal(dres.float(), torch.where(on, dy.float(), torch.zeros_like(dy.float())))
        C_.gemm(gy, True, w, False, dres, False, None, 0, None, True, 1.0, 1)
        assert torch.equal(dres, out)


@pytest.mark.parametrize("act", [1, 2])
@pytest.mark.parametrize("R,C", [(8192, 3072), (1000, 776), (37, 64)])
def test_act_bwd_colsum(cuda, act, R, C):
    """activation backward fused with its column sums (a linear's bias gradient) vs the separate kernels."""
    torch.manual_seed(4)
    dy = torch.randn(R, C, device=cuda).bfloat16()
    pre = torch.randn(R, C, device=cuda).bfloat16()
    y = torch.relu(pre) if act == 1 else pre
    g, db = _C().act_bwd_colsum(dy, y, act)
    ref = _C().relu_bwd(dy, y) if act == 1 else _C().gelu_bwd(dy, pre)
    assert torch.equal(g, ref)
    assert _rel(db, ref.float().sum(0)) < 1e-4
    out = torch.empty(C, device=cuda)
    g2, db2 = _C().act_bwd_colsum(dy, y, act, out)
    assert db2.data_ptr() == out.data_ptr() and torch.equal(db2, db)


# ----------------------------------------------------------------------------- normalize on load (gemm.hip XForm)
def _bn_params(C, device, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    scale = (torch.rand(C, generator=g) * 1.5 + 0.25) * torch.where(torch.rand(C, generator=g) < 0.2, -1.0, 1.0)
    shift = torch.randn(C, generator=g) * 0.5
    return torch.cat([scale, shift]).float().to(device).contiguous()


def _bn_relu_ref(x, params):
    """z as batchnorm.hip's apply writes it, bf16(relu(fma(x, scale, shift))): the fma through float64 (the product
    of two floats is exact there; the sum's double rounding can differ from a true fma in rare last bits)"""
    C = x.shape[-1]
    z = (x.double() * params[:C].double() + params[C:].double()).float().clamp_min(0.0)
    return z.bfloat16()


XF_CASES = [
    # N, H, W, C, K, R, stride, pad
    (4, 14, 14, 64, 64, 3, 1, 1),       # 3x3, padded taps stay zero
    (2, 28, 28, 128, 128, 3, 2, 1),     # strided 3x3 (ResNet stage-entry conv2)
    (8, 14, 14, 64, 256, 1, 1, 0),      # 1x1, K = 64: the single-buffer kernel (ResNet conv3 at stage 1)
    (3, 7, 7, 512, 2048, 1, 1, 0),      # 1x1, long K: the double-buffered kernel
    (2, 9, 11, 64, 72, 3, 1, 1),        # ragged M / N tails
    (16, 8, 8, 128, 64, 1, 1, 0),       # N = 64: the 256 x 64 tile
]


@pytest.mark.parametrize("case", XF_CASES)
def test_conv_fwd_normalize_on_load(cuda, case):
    """conv(relu(bn(x))) with the BN applied in the A-operand load equals conv of the materialised z (what the BN
    apply pass would have written), statistics epilogue included."""
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(5)
    x = (torch.randn(N, H, W, C, device=cuda) * 2 + 0.3).bfloat16()
    w = (torch.randn(K, R, R, C, device=cuda) * 0.05).bfloat16()
    p = _bn_params(C, cuda, 1)
    reps = _C().conv_stat_replicas
    s1 = torch.zeros(reps, 2, K, device=cuda)
    y = _C().conv_fwd(x, w, st, pad, 1, False, None, 0, s1, xform=p)
    z = _bn_relu_ref(x, p)
    s2 = torch.zeros(reps, 2, K, device=cuda)
    y2 = _C().conv_fwd(z, w, st, pad, 1, False, None, 0, s2)
    # same kernel arithmetic on (almost always) the same operand bits: a rare 1-ulp z difference (see _bn_relu_ref)
    # moves a few outputs by ~1 bf16 ulp at most
    d = (y.float() - y2.float()).abs()
    assert (d > 0).float().mean().item() < 1e-3 and d.max().item() <= 0.02 * y2.float().abs().max().item(), d.max()
    ref = F.conv2d(z.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, st, pad).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2
    torch.testing.assert_close(s1.sum(0), s2.sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("case", XF_CASES + [(2, 56, 56, 64, 64, 3, 1, 1)])
def test_conv_wgrad_normalize_on_load(cuda, case):
    """dW with the activation operand normalised on load (implicit-GEMM B, or the plain 1x1 GEMM with split-K
    slabs) vs an fp32 reference on the materialised z."""
    N, H, W, C, K, R, st, pad = case
    torch.manual_seed(6)
    x = (torch.randn(N, H, W, C, device=cuda) * 2 + 0.3).bfloat16()
    Ho = (H + 2 * pad - R) // st + 1
    Wo = (W + 2 * pad - R) // st + 1
    dy = torch.randn(N, Ho, Wo, K, device=cuda).bfloat16()
    p = _bn_params(C, cuda, 2)
    z = _bn_relu_ref(x, p)
    zr = z.float().permute(0, 3, 1, 2)
    wr = torch.zeros(K, C, R, R, device=cuda, requires_grad=True)
    F.conv2d(zr, wr, None, st, pad).backward(dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(0, 2, 3, 1)
    dw = torch.empty(K, R, R, C, device=cuda)
    _C().conv_wgrad(x, dy, dw, st, pad, 1, 0, False, xform=p)
    assert _rel(dw, ref) < 5e-3
    if R == 1 and st == 1:
        dw2 = torch.full((K, C), 7.0, device=cuda)
        _C().gemm(dy.reshape(-1, K), False, x.reshape(-1, C), False, dw2, True, None, 0, None, False, 1.0, 0,
                  xform_b=p, xform_c=C)
        assert _rel(dw2, ref.reshape(K, C)) < 5e-3
        base = torch.randn(K, C, device=cuda)
        dw3 = base.clone()
        _C().gemm(dy.reshape(-1, K), False, x.reshape(-1, C), False, dw3, True, None, 0, None, True, 1.0, 1,
                  xform_b=p, xform_c=C)
        assert _rel(dw3 - base, ref.reshape(K, C)) < 5e-3


def test_bn_relu_conv_matches_separate_ops(cuda):
    """ops.nn.bn_relu_conv (BN applied in the conv's loads) vs batch_norm_act + conv2d_nhwc on the same inputs:
    outputs, statistics, input gradient, conv weight / BN parameter gradients and running statistics."""
    from k8s_amd.models.resnet import BN, Conv
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore

    def build():
        store = ParamStore()
        pre = Conv(store, "pre", 64, 128, 1)
        bn = BN(store, "bn", 128)
        conv = Conv(store, "conv", 128, 128, 3, 2)
        store.finalize(cuda, seed=11)
        gen = torch.Generator(device=cuda).manual_seed(12)  # the same BN affine in both builds
        with torch.no_grad():
            bn.gamma.master.uniform_(0.5, 1.5, generator=gen)
            bn.beta.master.normal_(0.0, 0.3, generator=gen)
        return store, pre, bn.to(cuda), conv

    torch.manual_seed(7)
    x0 = torch.randn(4, 16, 16, 64, device=cuda).bfloat16().requires_grad_(True)
    g = torch.randn(4, 8, 8, 128, device=cuda).bfloat16()
    outs = []
    for fused in (True, False):
        store, pre, bn, conv = build()
        store.begin_step()
        x = x0.detach().clone().requires_grad_(True)
        t = pre(x)
        y, s = K.bn_relu_conv(t, bn, conv) if fused else conv(bn(t))
        y.backward(g)
        store.zero_unwritten()
        outs.append((y.detach(), s.detach().sum(0), x.grad, store.grad.clone(), bn.running_mean.clone(),
                     bn.running_var.clone()))
    (y1, s1, dx1, g1, rm1, rv1), (y2, s2, dx2, g2, rm2, rv2) = outs
    assert torch.equal(y1, y2)
    torch.testing.assert_close(s1, s2, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(rm1, rm2)
    torch.testing.assert_close(rv1, rv2)
    assert _rel(dx1, dx2) < 1e-2
    assert _rel(g1, g2) < 1e-2


@pytest.mark.parametrize("N,H,W,C", [(2, 56, 56, 64), (3, 13, 16, 64), (2, 28, 28, 128), (3, 14, 14, 256)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad3x3_tiled_vs_fp32(cuda, N, H, W, C, accumulate):
    """LDS-tiled 3x3 weight gradient (wgrad_tile.hip; C = K in 64-channel pieces, stride 1, pad 1) against the fp32
    weight gradient of the same convolution (H = 13 / 14: tiles running past the image)."""
    torch.manual_seed(5)
    x = torch.randn(N, H, W, C, device=cuda).bfloat16()
    dy = torch.randn(N, H, W, C, device=cuda).bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (C, C, 3, 3), dy.float().permute(0, 3, 1, 2),
                                      1, 1).permute(0, 2, 3, 1)
    base = torch.randn(C, 3, 3, C, device=cuda) if accumulate else torch.zeros(C, 3, 3, C, device=cuda)
    dw = base.clone()
    _C().conv_wgrad(x, dy, dw, 1, 1, 1, 0, accumulate, None)
    assert _rel(dw, ref + (base if accumulate else 0)) < 1e-3


@pytest.mark.parametrize("M,N,K,ak,bk", [(256, 1024, 200704, False, False), (512, 128, 65536, False, False),
                                         (256, 512, 32768, True, False)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm256_splitk(cuda, M, N, K, ak, bk, accumulate):
    """Tall-K fp32 products on the 256 x 256 kernel with split-K (the ResNet 1x1 weight-gradient shapes)."""
    torch.manual_seed(6)
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    A = a if ak else a.t().contiguous()
    B = b if bk else b.t().contiguous()
    base = torch.randn(M, N, device=cuda) if accumulate else None
    out = base.clone() if accumulate else None
    c = _C().gemm(A, ak, B, bk, out, True, None, 0, None, accumulate, 1.0, 0)
    assert _rel(c, ref + (base if accumulate else 0)) < 2e-3


@pytest.mark.parametrize("shape", [(1024, 16, 16, 1024, 256), (256, 14, 14, 512, 2048)])
def test_conv1x1_deep_w4_stats_epilogue(cuda, shape, monkeypatch):
    """ResNet's deep-reduction 1x1 forwards on the 4-wave GEMM with the BatchNorm-statistics epilogue (gemm256.hip
    copy_out_stats; whole 256 x 256 tiles filling the chip): y against an fp32 reference, the statistics against the
    stored values, and both against the 128 x 128 tile kernel (K8S_AMD_W4_STATS=0)."""
    N, H, W, C, K = shape
    assert _C().gemm_rope_ok is not None  # (the extension is the in-tree one)
    torch.manual_seed(9)
    x = (torch.randn(N, H, W, C, device=cuda) * 0.5).bfloat16()
    w = (torch.randn(K, 1, 1, C, device=cuda) * 0.03).bfloat16()
    out = {}
    for arm in ("1", "0"):
        monkeypatch.setenv("K8S_AMD_W4_STATS", arm)
        stats = torch.zeros(_C().conv_stat_replicas, 2, K, device=cuda)
        y = _C().conv_fwd(x, w, 1, 0, 1, False, None, 0, stats)
        out[arm] = (y, stats.sum(0))
    ref = x.float().reshape(-1, C) @ w.float().reshape(K, C).t()
    for arm, (y, tot) in out.items():
        yf = y.float().reshape(-1, K)
        assert _rel(yf, ref) < 1e-2, arm
        assert _rel(tot[0], yf.sum(0)) < 1e-3, arm
        assert _rel(tot[1], (yf * yf).sum(0)) < 1e-3, arm
    assert _rel(out["1"][0], out["0"][0]) < 5e-3


@pytest.mark.parametrize("arm", ["1", "0"])
def test_downsample_1x1_stride2_subsampled(cuda, arm, monkeypatch):
    """The 1x1 / stride-2 downsample convolution as a stride-1 GEMM on the subsampled input (pool.hip
    subsample_nhwc; ops.conv.SUB1X1) and on the strided implicit-GEMM path: y, BN statistics, dx and dW against
    fp32 PyTorch."""
    from k8s_amd.ops import conv as kc
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore, init_normal

    monkeypatch.setattr(kc, "SUB1X1", arm == "1")
    torch.manual_seed(10)
    N, H, C, Ko = 8, 28, 256, 512
    store = ParamStore()
    p = store.new("down", (Ko, 1, 1, C), init_normal(0.05))
    store.finalize(cuda)
    x = torch.randn(N, H, H, C, device=cuda).bfloat16().requires_grad_(True)
    store.begin_step()
    y, sums = K.conv2d_nhwc(x, p, 2, 0, with_stats=True)
    gy = torch.randn_like(y)
    y.backward(gy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = p.master.detach().clone().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.conv2d(xr, wr.bfloat16().float(), None, 2, 0)
    yr.backward(gy.float().permute(0, 3, 1, 2))
    yrf = yr.detach().permute(0, 2, 3, 1)
    assert _rel(y, yrf) < 1e-2
    yf = y.float().reshape(-1, Ko)
    assert _rel(sums.sum(0)[0], yf.sum(0)) < 1e-3
    assert _rel(x.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert _rel(p.grad, wr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("M,K,N,dual,rows", [(3000, 64, 256, False, 0), (3000, 64, 256, True, 0),
                                             (2056, 128, 512, True, 0),
                                             (2056, 128, 512, False, 0), (1000, 256, 1024, False, 0),
                                             # row-chunked launches (the stage-1 form at batch >= 2048)
                                             (3000, 64, 256, True, 1024), (2056, 128, 512, False, 512)])
def test_dgrad_short_bnstats_epilogue(cuda, M, K, N, dual, rows, monkeypatch):
    """The identity-block 1x1 data gradient with a masked addend that also accumulates the BatchNorm-backward sums of
    its result (gemm_short.hip EPI 3 / 4): dx bitwise equal to the plain masked-addend dgrad, the sums against fp32
    sums over the stored dx: sum g and sum g (x - mean), g = bit ? dx : 0 with the BatchNorm's own ReLU bits."""
    C_ = _C()
    if rows:
        monkeypatch.setenv("K8S_AMD_GEMM_SHORT_ROWS", str(rows))
    assert C_.gemm_short_bnstats_ok(M, N, K, dual)
    torch.manual_seed(11)
    gy = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(K, N, device=cuda) * 0.1).bfloat16()
    dy = torch.randn(M, N, device=cuda).bfloat16()
    amask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)
    x = (torch.randn(M, N, device=cuda) * 2 + 0.5).bfloat16()
    bmask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)
    mean = torch.randn(N, device=cuda) * 0.3
    R = C_.conv_stat_replicas
    sums = torch.zeros(R, 2, N, device=cuda)
    x2 = mean2 = sums2 = None
    if dual:
        x2 = (torch.randn(M, N, device=cuda) - 0.25).bfloat16()
        mean2 = torch.randn(N, device=cuda) * 0.2
        sums2 = torch.zeros(R, 2, N, device=cuda)
    out = C_.dgrad_short_bnstats(gy, w, dy, amask, x, bmask, mean, sums, x2, mean2, sums2)
    plain = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    C_.gemm(gy, True, w, False, plain, False, None, 0, None, True, 1.0, 1, dy, amask)
    assert torch.equal(out, plain)
    g = torch.where(_unpack_bits(bmask, (M, N)), out.float(), torch.zeros(M, N, device=cuda))
    tot = sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-4
    assert _rel(tot[1], (g * (x.float() - mean)).sum(0)) < 1e-4
    if dual:
        assert _rel(sums2.sum(0)[1], (g * (x2.float() - mean2)).sum(0)) < 1e-4


def test_bn_bwd_from_sums_matches_reduce(cuda):
    """bn_bwd_from_sums (final + apply from a producer's sums) against bn_bwd (its own reduction sweep) on the same
    masked dy: dx, dgamma, dbeta."""
    C_ = _C()
    torch.manual_seed(12)
    M, C = 4096, 256
    x = (torch.randn(M, C, device=cuda) * 1.5 + 0.3).bfloat16()
    dy = torch.randn(M, C, device=cuda).bfloat16()
    mask = torch.randint(0, 256, (M * C // 8,), device=cuda, dtype=torch.uint8)
    mean = x.float().mean(0)
    invstd = torch.rsqrt(x.float().var(0, unbiased=False) + 1e-5)
    gamma, beta = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda) * 0.1
    g = torch.where(_unpack_bits(mask, (M, C)), dy.float(), torch.zeros(M, C, device=cuda))
    sums = torch.zeros(C_.conv_stat_replicas, 2, C, device=cuda)
    sums[0, 0] = g.sum(0)
    sums[0, 1] = (g * (x.float() - mean)).sum(0)
    dg1, db1, dg2, db2 = (torch.empty(C, device=cuda) for _ in range(4))
    dx1, _ = C_.bn_bwd(dy, x, None, mean, invstd, gamma, beta, False, dg1, db1, False, mask)
    dx2, _ = C_.bn_bwd_from_sums(dy, x, mask, sums, mean, invstd, gamma, beta, dg2, db2, False)
    assert _rel(db2, db1) < 1e-5 and _rel(dg2, dg1) < 1e-4
    assert _rel(dx2, dx1) < 5e-3


@pytest.mark.parametrize("N,H,C,K", [(3, 56, 64, 64), (2, 28, 128, 128), (3, 14, 256, 256)])
def test_conv3x3_dgrad_bnstats_epilogue(cuda, N, H, C, K):
    """The stride-1 3x3 data gradient on the staged-window kernel with the BatchNorm-backward sums of the
    relu(BN(x)) that fed the convolution (conv3x3.hip epilogue): dx bitwise equal to the plain dgrad, the sums
    against fp32 sums over the stored dx with the forward's ReLU decision relu_on(x) recomputed from the affine."""
    C_ = _C()
    torch.manual_seed(13)
    gy = torch.randn(N, H, H, K, device=cuda).bfloat16()
    w = (torch.randn(K, 3, 3, C, device=cuda) * 0.05).bfloat16()
    x = (torch.randn(N, H, H, C, device=cuda) * 1.5 + 0.2).bfloat16()
    mean = x.float().reshape(-1, C).mean(0)
    invstd = torch.rsqrt(x.float().reshape(-1, C).var(0, unbiased=False) + 1e-5)
    gamma, beta = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda) * 0.2
    sums = torch.zeros(C_.conv_stat_replicas, 2, C, device=cuda)
    wt = C_.conv_dgrad_wtrans(w)
    dx = C_.conv3x3_dgrad_bnstats(gy, wt, x, gamma, beta, mean, invstd, sums)
    plain = C_.conv_fwd(gy, wt, 1, 1, 1, False, None, 0, None)
    assert torch.equal(dx, plain)
    scale = gamma * invstd
    shift = torch.addcmul(beta, -mean, scale)  # fma(-mean, scale, beta) up to rounding: compare the decision loosely
    z = (x.float() * scale + shift).bfloat16().float()
    g = torch.where(z > 0, dx.float(), torch.zeros_like(dx.float())).reshape(-1, C)
    tot = sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-3
    assert _rel(tot[1], (g * (x.float().reshape(-1, C) - mean)).sum(0)) < 1e-3


@pytest.mark.parametrize("M,K,N", [(9000, 256, 64), (4100, 512, 128), (1000, 384, 72),
                                   # the 4-wave kernel's copy_out_bnbwd: whole waves, and a stream-K tail
                                   (65536, 1024, 256), (150528, 2048, 512)])
def test_gemm_dgrad_bnstats_epilogue(cuda, M, K, N):
    """The 1x1 data gradient on its regular kernel (the tile kernel's BST epilogue, or the 4-wave kernel's ACT 6
    copy-out) with the BatchNorm-backward sums of the relu(BN(x)) that fed the convolution: dx bitwise equal to the
    plain dgrad, the sums against fp32 sums over the stored dx with the forward's ReLU decision."""
    C_ = _C()
    assert C_.gemm_dgrad_bnstats_ok(M, N, K)
    torch.manual_seed(14)
    gy = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(K, N, device=cuda) * 0.05).bfloat16()
    x = (torch.randn(M, N, device=cuda) * 1.5 + 0.2).bfloat16()
    mean = x.float().mean(0)
    invstd = torch.rsqrt(x.float().var(0, unbiased=False) + 1e-5)
    gamma, beta = torch.rand(N, device=cuda) + 0.5, torch.randn(N, device=cuda) * 0.2
    sums = torch.zeros(C_.conv_stat_replicas, 2, N, device=cuda)
    dx = C_.gemm_dgrad_bnstats(gy, w, x, gamma, beta, mean, invstd, sums)
    plain = C_.gemm(gy, True, w, False, None, False, None, 0, None, False, 1.0, 1)
    assert torch.equal(dx, plain)
    scale = gamma * invstd
    shift = torch.addcmul(beta, -mean, scale)
    z = (x.float() * scale + shift).bfloat16().float()
    g = torch.where(z > 0, dx.float(), torch.zeros_like(dx.float()))
    tot = sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-3
    assert _rel(tot[1], (g * (x.float() - mean)).sum(0)) < 1e-3


@pytest.mark.parametrize("N,H,K1,C,K2", [(4, 16, 128, 256, 512), (2, 14, 256, 512, 1024)])
def test_stage_entry_bn_sums_two_dgrads(cuda, N, H, K1, C, K2):
    """A residual BN's backward sums over the sum of two data gradients into its output (a ResNet stage-entry block:
    conv1's 1x1 dgrad, then the downsample's 1x1 / stride-2 dgrad accumulated onto it): the first takes the sums over
    its values (gemm_short EPI 5), the second adds the changes it makes at its parity (gemm.hip BST sub-grid path).
    Against fp32 sums over the final tensor with the BN's packed ReLU bits."""
    from k8s_amd.ops import conv as kc
    from k8s_amd.ops import nn as K

    C_ = _C()
    torch.manual_seed(15)
    M = N * H * H
    gy = torch.randn(M, K1, device=cuda).bfloat16()
    w1 = (torch.randn(K1, C, device=cuda) * 0.05).bfloat16()
    x = (torch.randn(N, H, H, C, device=cuda) * 1.5 + 0.2).bfloat16()
    mask = torch.randint(0, 256, (M * C // 8,), device=cuda, dtype=torch.uint8)
    mean = torch.randn(C, device=cuda) * 0.2
    link = K.BnStatLink()
    link.x, link.mask, link.mean = x, mask, mean
    sums = torch.zeros(C_.conv_stat_replicas, 2, C, device=cuda)
    out = C_.dgrad_short_bnstats(gy, w1, None, None, x.view(-1, C), mask, mean, sums).view(N, H, H, C)
    plain = C_.gemm(gy, True, w1, False, None, False, None, 0, None, False, 1.0, 1)
    assert torch.equal(out.view(-1, C), plain)
    link.sums, link.pending = sums, True
    dy2 = torch.randn(N, H // 2, H // 2, K2, device=cuda).bfloat16()
    w2 = (torch.randn(K2, 1, 1, C, device=cuda) * 0.05).bfloat16()
    dx = kc._dgrad_strided_hip(C_, dy2, w2, 2, 0, H, H, out, link)
    assert dx.data_ptr() == out.data_ptr() and not link.pending and link.dy_key == (dx.data_ptr(), tuple(dx.shape))
    ref_dx = plain.float().view(N, H, H, C).clone()
    ref_dx[:, ::2, ::2, :] += (dy2.float().reshape(-1, K2) @ w2.float().reshape(K2, C)).view(N, H // 2, H // 2, C)
    assert _rel(dx, ref_dx) < 1e-2
    g = torch.where(_unpack_bits(mask, (M, C)), dx.float().view(-1, C), torch.zeros(M, C, device=cuda))
    tot = sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-3
    assert _rel(tot[1], (g * (x.float().view(-1, C) - mean)).sum(0)) < 1e-3


def test_gemm_dgrad_bnstats_mask_accumulate(cuda):
    """The second of two stride-1 data gradients into the stem pool's output (layer 1's downsample after its conv1):
    the tile kernel accumulates onto the first's gradient and takes the BatchNorm-backward sums (mask kind) over the
    final tensor in its epilogue (gemm.hip BST fast path; ops.conv._dgrad_hip, BnStatLink.last_full) -- against fp32
    sums. Ragged M (not a multiple of the 128-row tile)."""
    from k8s_amd.ops import conv as kc
    from k8s_amd.ops import nn as K

    C_ = _C()
    torch.manual_seed(21)
    N, H, C, K1, K2 = 4, 27, 64, 64, 256
    M = N * H * H
    x = (torch.randn(N, H, H, C, device=cuda) * 1.5 + 0.2).bfloat16()
    mask = torch.randint(0, 256, (M * C // 8,), device=cuda, dtype=torch.uint8)
    mean = torch.randn(C, device=cuda) * 0.2
    gy1 = torch.randn(N, H, H, K1, device=cuda).bfloat16()
    w1 = (torch.randn(K1, 1, 1, C, device=cuda) * 0.05).bfloat16()
    gy2 = torch.randn(N, H, H, K2, device=cuda).bfloat16()
    w2 = (torch.randn(K2, 1, 1, C, device=cuda) * 0.05).bfloat16()
    link = K.BnStatLink()
    link.x, link.mask, link.mean, link.last_full = x, mask, mean, True
    dx1 = kc._dgrad_hip(C_, gy1, w1, 0, None, link)
    assert link.sums is None and not link.pending
    dx = kc._dgrad_hip(C_, gy2, w2, 0, dx1, link)
    assert dx.data_ptr() == dx1.data_ptr()
    assert link.dy_key == (dx.data_ptr(), tuple(dx.shape)) and link.sums is not None
    ref = gy1.float().reshape(-1, K1) @ w1.float().reshape(K1, C) + gy2.float().reshape(-1, K2) @ w2.float().reshape(K2, C)
    assert _rel(dx.view(-1, C), ref) < 1e-2
    g = torch.where(_unpack_bits(mask, (M, C)), dx.float().view(-1, C), torch.zeros(M, C, device=cuda))
    tot = link.sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-3
    assert _rel(tot[1], (g * (x.float().view(-1, C) - mean)).sum(0)) < 1e-3


@pytest.mark.parametrize("M,N,K,dual", [(1000, 256, 512, False), (3 * 49 * 4, 2048, 512, False),
                                        (1000, 256, 256, True), (3 * 49 * 4, 2048, 512, True)])
def test_gemm_dgrad_bnstats_masked_addend(cuda, M, N, K, dual):
    """A stage-4 identity block's conv1 data gradient (K = 512: not a gemm_short depth) on the tile kernel: out =
    dgrad + (addend bit ? addend : 0) with the residual BatchNorm's backward sums of out in the same epilogue
    (gemm.hip BST fast path, masked addend), against fp32."""
    C_ = _C()
    torch.manual_seed(23)
    gy = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(K, N, device=cuda) * 0.05).bfloat16()
    add = torch.randn(M, N, device=cuda).bfloat16()
    amask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)
    x = (torch.randn(M, N, device=cuda) * 1.5 + 0.2).bfloat16()
    mask = torch.randint(0, 256, (M * N // 8,), device=cuda, dtype=torch.uint8)
    mean = torch.randn(N, device=cuda) * 0.2
    sums = torch.zeros(C_.conv_stat_replicas, 2, N, device=cuda)
    out = torch.full((M, N), float("nan"), device=cuda).bfloat16()
    x2 = (torch.randn(M, N, device=cuda) - 0.3).bfloat16() if dual else None
    mean2 = torch.randn(N, device=cuda) * 0.1 if dual else None
    sums2 = torch.zeros(C_.conv_stat_replicas, 2, N, device=cuda) if dual else None
    C_.gemm_dgrad_bnstats_mask(gy, w, out, x, mask, mean, sums, add, amask, x2, mean2, sums2)
    ref = gy.float() @ w.float() + torch.where(_unpack_bits(amask, (M, N)), add.float(), torch.zeros(M, N, device=cuda))
    assert _rel(out, ref) < 1e-2
    g = torch.where(_unpack_bits(mask, (M, N)), out.float(), torch.zeros(M, N, device=cuda))
    tot = sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-3
    assert _rel(tot[1], (g * (x.float() - mean)).sum(0)) < 1e-3
    if dual:
        assert _rel(sums2.sum(0)[1], (g * (x2.float() - mean2)).sum(0)) < 1e-3


@pytest.mark.parametrize("N,H,C,K", [(4, 28, 128, 128), (2, 14, 256, 256), (3, 13, 128, 192)])
def test_strided_dgrad_bn_relu_sums(cuda, monkeypatch, N, H, C, K):
    """A stride-2 3x3 data gradient (ResNet's stage-entry conv2) as its four parities, each storing its own pixels and
    adding the BatchNorm + ReLU backward sums of the bn1 that fed the convolution (gemm.hip BST sub-grid path, relu
    kind; the 1x1 parity on the K-major source, the others on the implicit GEMM): dx equal to the parity path without
    the sums, the sums against fp32 sums over the stored dx with the forward's ReLU decision. Odd H: ragged parities."""
    from k8s_amd.ops import conv as kc
    from k8s_amd.ops import nn as K_

    C_ = _C()
    torch.manual_seed(16)
    Ho = (H + 1) // 2
    gy = torch.randn(N, Ho, Ho, K, device=cuda).bfloat16()
    w = (torch.randn(K, 3, 3, C, device=cuda) * 0.05).bfloat16()
    x = (torch.randn(N, H, H, C, device=cuda) * 1.5 + 0.2).bfloat16()
    mean = x.float().reshape(-1, C).mean(0)
    invstd = torch.rsqrt(x.float().reshape(-1, C).var(0, unbiased=False) + 1e-5)
    gamma, beta = torch.rand(C, device=cuda) + 0.5, torch.randn(C, device=cuda) * 0.2
    link = K_.BnStatLink()
    link.x, link.mean, link.invstd, link.gamma, link.beta, link.relu = x, mean, invstd, gamma, beta, True
    monkeypatch.setattr(kc, "BSTATS_STRIDED", True)  # (off by default: neutral at the step level)
    dx = kc._dgrad_strided_hip(C_, gy, w, 2, 1, H, H, None, link)
    assert link.sums is not None and link.dy_key == (dx.data_ptr(), tuple(dx.shape))
    plain = kc._dgrad_strided_hip(C_, gy, w, 2, 1, H, H, None, None)
    assert torch.equal(dx, plain)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float().permute(0, 3, 1, 2), gy.float().permute(0, 3, 1, 2),
                                     stride=2, padding=1).permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 1e-2
    scale = gamma * invstd
    shift = torch.addcmul(beta, -mean, scale)
    z = (x.float() * scale + shift).bfloat16().float()
    g = torch.where(z > 0, dx.float(), torch.zeros_like(dx.float())).reshape(-1, C)
    tot = link.sums.sum(0)
    assert _rel(tot[0], g.sum(0)) < 1e-3
    assert _rel(tot[1], (g * (x.float().reshape(-1, C) - mean)).sum(0)) < 1e-3
