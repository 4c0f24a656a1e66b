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


# stream-K tail (gemm256_plan): T = w * 256 + r tiles with r <= 128 run the last r tiles split sk ways along K with
# the in-kernel fixed-order fix-up. (M, N, K) -> tiles, sk: 16x24 = 384 -> 2 (Llama QKV); 16x18 = 288 -> 4 at
# K = 2048; 16x21 = 336 -> 3; 16x20 = 320 -> 4; ragged edges on a 2-split tail. Sub-wave grids take no tail.
SK_SHAPES = [(4096, 6144, 4096), (4096, 4608, 2048), (4096, 5376, 3072), (4096, 5120, 4096), (4000, 6136, 2048)]


def _sk_env(monkeypatch, on):
    monkeypatch.setenv("K8S_AMD_GEMM256_SK", "1" if on else "0")


@pytest.mark.parametrize("M,N,K", SK_SHAPES)
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False)])
def test_gemm256_stream_k_tail_matches_fp32(cuda, monkeypatch, M, N, K, ak, bk):
    """the stream-K tail against an fp32 PyTorch product, bf16 and fp32 outputs; the
    result is deterministic (bit-identical over repeated launches, whichever split arrives last)."""
    torch.manual_seed(3)
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    A = a if ak else a.t().contiguous()
    B = b if bk else b.t().contiguous()
    _sk_env(monkeypatch, True)
    c = _C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)
    assert _rel(c, ref) < 1e-4
    for _ in range(3):
        assert torch.equal(_C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1), c)
    cb = _C().gemm(A, ak, B, bk, None, False, None, 0, None, False, 1.0, 1)  # bf16: the 4-wave kernel's tail (NT)
    assert _rel(cb, ref) < 1e-2
    for _ in range(3):
        assert torch.equal(_C().gemm(A, ak, B, bk, None, False, None, 0, None, False, 1.0, 1), cb)
    _sk_env(monkeypatch, False)  # the whole-tile path agrees to fp32 rounding
    c0 = _C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)
    assert _rel(c0, c) < 1e-5


@pytest.mark.parametrize("act", [0, 2])
def test_gemm256_stream_k_tail_epilogues(cuda, monkeypatch, act):
    """The fix-up hands the summed tile to the normal epilogue: bias + GELU + pre-activation copy, and an fp32
    accumulate into an existing buffer with alpha, on a 2-split tail."""
    torch.manual_seed(4)
    M, N, K = 4096, 6144, 4096
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.02).bfloat16()
    bvec = torch.randn(N, device=cuda)
    _sk_env(monkeypatch, True)
    pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    y = _C().gemm(a, True, w, True, None, False, bvec, act, pre, False, 1.0, 1)
    p_ref = a.float() @ w.float().t() + bvec
    y_ref = F.gelu(p_ref, approximate="tanh") if act == 2 else p_ref
    assert _rel(pre, p_ref) < 1e-2 and _rel(y, y_ref) < 1e-2
    out = torch.full((M, N), -1.5, device=cuda)
    _C().gemm(a, True, w, True, out, True, None, 0, None, True, 0.5, 1)
    assert _rel(out + 1.5, 0.5 * (a.float() @ w.float().t())) < 1e-4


def test_gemm256_stream_k_sync_words_reset(cuda, monkeypatch):
    """Back-to-back launches of different stream-K plans reuse the ticket / flag words: every launch must leave
    them zero (a stale ticket would make a split skip its fix-up and write a partial tile)."""
    torch.manual_seed(5)
    _sk_env(monkeypatch, True)
    for M, N, K in SK_SHAPES[:4] * 2:
        a = torch.randn(M, K, device=cuda).bfloat16()
        b = torch.randn(N, K, device=cuda).bfloat16()
        c = _C().gemm(a, True, b, True, None, True, None, 0, None, False, 1.0, 1)
        assert _rel(c, a.float() @ b.float().t()) < 1e-4, (M, N, K)
        cb = _C().gemm(a, True, b, True, None, False, None, 0, None, False, 1.0, 1)  # 4-wave kernel's sync words
        assert _rel(cb, a.float() @ b.float().t()) < 1e-2, (M, N, K)


@pytest.mark.parametrize("M", [4, 12, 1000])
@pytest.mark.parametrize("N", [4, 12, 1000])
def test_linear_ragged_rows_and_columns_on_our_kernels(cuda, M, N):
    """ragged M / N (a batch-4 classifier head, 12 classes) run on our GEMM kernels -- the row
    tails masked in-kernel, a ragged N zero-padded to 16-B units in the backward -- with no PyTorch fallback, against
    fp32 PyTorch: forward with bias, data gradient, and the weight gradient written into the flat fp32 slot."""
    from k8s_amd.ops import gemm

    torch.manual_seed(6)
    Kd = 2048
    x = torch.randn(M, Kd, device=cuda).bfloat16()
    w = (torch.randn(N, Kd, device=cuda) * 0.02).bfloat16()
    b = torch.randn(N, device=cuda)
    before = dict(gemm.FALLBACKS)
    y, saved = gemm.linear_fwd(x, w, b)
    ref = x.float() @ w.float().t() + b
    assert _rel(y, ref) < 1e-2
    gy = torch.randn(M, N, device=cuda).bfloat16()
    dx, dw, db = gemm.linear_bwd(gy, x, w, saved, None)
    assert _rel(dx, gy.float() @ w.float()) < 1e-2
    assert _rel(dw, gy.float().t() @ x.float()) < 1e-2
    assert _rel(db, gy.float().sum(0)) < 1e-2
    assert gemm.FALLBACKS == before, gemm.FALLBACKS


@pytest.mark.parametrize("mode", ["0", "2"])
def test_gemm256_mode_switch_sides(cuda, monkeypatch, mode):
    """$K8S_AMD_GEMM256: 0 routes every product to the 128 x 128 kernel, 2 every product the 256 x 256 kernel can
    take -- both non-default sides against fp32, all three operand forms."""
    monkeypatch.setenv("K8S_AMD_GEMM256", mode)
    torch.manual_seed(7)
    M, N, K = 2048, 1536, 1024
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    for ak, bk in [(True, True), (True, False), (False, False)]:
        A = a if ak else a.t().contiguous()
        B = b if bk else b.t().contiguous()
        c = _C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)
        assert _rel(c, ref) < 1e-4, (ak, bk)


# 4-wave kernel (gemm256.hip g4): A K-major, B K-major or MN-major, whole 256 tiles, plain bf16 output, >= 256 tiles.
# K = 64 / 128 / 192 run the one-, two- and three-stage paths of its peeled K loop.
W4_SHAPES = [(4096, 4096, 64), (4096, 4096, 128), (4096, 4096, 192), (2048, 8192, 4096), (8192, 4096, 640)]


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])  # fwd, dgrad, wgrad
@pytest.mark.parametrize("M,N,K", W4_SHAPES)
def test_gemm_w4_matches_fp32(cuda, monkeypatch, M, N, K, ak, bk):
    torch.manual_seed(6)
    a = torch.randn(M, K, device=cuda).bfloat16()
    b = torch.randn(N, K, device=cuda).bfloat16()
    ref = a.float() @ b.float().t()
    A = a if ak else a.t().contiguous()
    B = b if bk else b.t().contiguous()
    monkeypatch.setenv("K8S_AMD_GEMM_W4", "1")
    y = _C().gemm(A, ak, B, bk, None, False, None, 0, None, False, 1.0, 1)
    assert _rel(y, ref) < 1e-2
    y2 = _C().gemm(A, ak, B, bk, None, False, None, 0, None, False, 0.5, 1)  # alpha
    assert _rel(y2, 0.5 * ref) < 1e-2
    c = _C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)  # fp32 output (weight gradients)
    assert _rel(c, ref) < 1e-4
    out = torch.full((M, N), -1.5, device=cuda)
    _C().gemm(A, ak, B, bk, out, True, None, 0, None, True, 0.5, 1)  # accumulate into an existing fp32 buffer
    assert _rel(out + 1.5, 0.5 * ref) < 1e-4
    monkeypatch.setenv("K8S_AMD_GEMM_W4", "0")  # the ring kernel: the same product to bf16 / fp32 rounding
    y0 = _C().gemm(A, ak, B, bk, None, False, None, 0, None, False, 1.0, 1)
    assert _rel(y, y0) < 1e-2
    c0 = _C().gemm(A, ak, B, bk, None, True, None, 0, None, False, 1.0, 1)
    assert _rel(c, c0) < 1e-5


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_w4_epilogue_extras(cuda, monkeypatch, act, bias):
    """The 4-wave kernel's X epilogue (the transformer linears at a batch that fills the chip: BERT-base at 131k
    tokens): bias + ReLU / GELU + the pre-activation copy for the forward form, and the bf16 accumulate of the data
    gradient, against fp32 PyTorch and against the ring kernel ($K8S_AMD_GEMM_W4=0)."""
    torch.manual_seed(8)
    M, N, K = 8192, 3072, 768  # 32 x 12 = 384 tiles: whole waves + a stream-K tail
    a = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) * 0.05).bfloat16()
    bvec = torch.randn(N, device=cuda) if bias else None
    p_ref = a.float() @ w.float().t() + (bvec if bias else 0.0)
    y_ref = [p_ref, torch.relu(p_ref), F.gelu(p_ref, approximate="tanh")][act]
    out = {}
    for side in ("1", "0"):
        monkeypatch.setenv("K8S_AMD_GEMM_W4", side)
        pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        y = _C().gemm(a, True, w, True, None, False, bvec, act, pre, False, 1.0, 1)
        assert _rel(pre, p_ref) < 1e-2 and _rel(y, y_ref) < 1e-2, side
        y2 = _C().gemm(a, True, w, True, None, False, bvec, act, None, False, 1.0, 1)  # no pre-activation copy
        assert _rel(y2, y_ref) < 1e-2, side
        out[side] = y
    assert _rel(out["1"], out["0"]) < 1e-2
    # data-gradient form with a bf16 accumulate (a residual's other gradient contribution added in the epilogue)
    g = torch.randn(M, N, device=cuda).bfloat16()
    old = torch.randn(M, K, device=cuda).bfloat16()
    monkeypatch.setenv("K8S_AMD_GEMM_W4", "1")
    dx = old.clone()
    _C().gemm(g, True, w, False, dx, False, None, 0, None, True, 1.0, 1)
    assert _rel(dx, old.float() + g.float() @ w.float()) < 1e-2


W4_SPLIT_SHAPES = [(768, 768, 65536), (2304, 768, 32768), (768, 3072, 16384), (256, 1024, 65536)]


@pytest.mark.parametrize("M,N,K", W4_SPLIT_SHAPES)
def test_gemm_w4_tall_k_split(cuda, monkeypatch, M, N, K):
    """Weight gradients of few output tiles on the 4-wave kernel: the K range split unevenly over gridDim.y (the last
    split shorter) into fp32 slabs, combined by splitk_reduce -- stored and accumulated into an existing slot, against
    fp32 PyTorch and the ring kernel's even split; deterministic over repeated launches."""
    torch.manual_seed(9)
    g = torch.randn(K, M, device=cuda).bfloat16()  # both operands MN-major, as linear_bwd's dW = g^T x
    x = torch.randn(K, N, device=cuda).bfloat16()
    ref = g.float().t() @ x.float()
    monkeypatch.setenv("K8S_AMD_GEMM_W4", "1")
    c = _C().gemm(g, False, x, False, None, True, None, 0, None, False, 1.0, 0)
    assert _rel(c, ref) < 1e-4
    for _ in range(2):
        assert torch.equal(_C().gemm(g, False, x, False, None, True, None, 0, None, False, 1.0, 0), c)
    out = torch.full((M, N), 2.0, device=cuda)
    _C().gemm(g, False, x, False, out, True, None, 0, None, True, 1.0, 0)
    assert _rel(out - 2.0, ref) < 1e-4
    monkeypatch.setenv("K8S_AMD_GEMM_W4", "0")
    c0 = _C().gemm(g, False, x, False, None, True, None, 0, None, False, 1.0, 0)
    assert _rel(c, c0) < 1e-5


def _gelu_grad(x):
    k0, k1 = 0.7978845608028654, 0.044715
    t = torch.tanh(k0 * (x + k1 * x ** 3))
    return 0.5 * (1 + t) + 0.5 * x * (1 - t * t) * k0 * (1 + 3 * k1 * x * x)


@pytest.mark.parametrize("act", [1, 2])
def test_gemm_dact_matches_fp32(cuda, act):
    """Data gradient fused with the input activation's backward and the producer's bias gradient (gemm256.hip
    copy_out_x ACT < 0, `gemm_dact`): dx = (g . W) * act'(pre), db = column sums of dx, against fp32 PyTorch; db
    written, then accumulated onto an existing value."""
    torch.manual_seed(10)
    M, Nout, Kin = 16384, 768, 3072  # BERT-base FFN2's data gradient: 64 x 12 = 768 tiles
    g = torch.randn(M, Nout, device=cuda).bfloat16()
    w = (torch.randn(Nout, Kin, device=cuda) * 0.05).bfloat16()
    pre = torch.randn(M, Kin, device=cuda).bfloat16()
    if act == 1:
        pre = torch.relu(pre)  # the ReLU path reads the ReLU output
    assert _C().gemm_dact_ok(M, Kin, Nout)
    db = torch.empty(Kin, device=cuda)
    dx = _C().gemm_dact(g, w, pre, act, db, False)
    d = g.float() @ w.float()
    deriv = (pre.float() > 0).float() if act == 1 else _gelu_grad(pre.float())
    ref = d * deriv
    assert _rel(dx, ref) < 1e-2
    assert _rel(db, dx.float().sum(0)) < 1e-4  # the sums of the stored bf16 values
    assert _rel(db, ref.sum(0)) < 1e-2
    db2 = torch.full((Kin,), 0.5, device=cuda)
    dx2 = _C().gemm_dact(g, w, pre, act, db2, True)
    assert torch.equal(dx2, dx)
    assert _rel(db2 - 0.5, db) < 1e-5


def test_linear_act_link_matches_unfused(cuda):
    """BERT's FFN (linear + GELU -> linear) with FFN1's GELU backward and bias gradient fused into FFN2's data
    gradient (nn.ActLink) against the unfused path (nn.ACT_FUSE = False): x, W1, b1, W2, b2 gradients."""
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore, init_normal

    torch.manual_seed(11)
    T, H, F4 = 16384, 768, 3072
    grads = {}
    for fuse in (True, False):
        K.ACT_FUSE = fuse
        try:
            store = ParamStore()
            w1 = store.new("w1", (F4, H), init_normal(0.02))
            b1 = store.new("b1", (F4,), init_normal(0.02), decay=False, lowp=False)
            w2 = store.new("w2", (H, F4), init_normal(0.02))
            b2 = store.new("b2", (H,), init_normal(0.02), decay=False, lowp=False)
            store.finalize(cuda, seed=5)
            g = torch.Generator(device=cuda).manual_seed(12)
            x = torch.randn(T, H, device=cuda, generator=g).bfloat16().requires_grad_(True)
            gy = torch.randn(T, H, device=cuda, generator=g).bfloat16()
            store.begin_step()
            al = K.ActLink()
            f = K.linear(x, w1, b1, act="gelu", act_link=al)
            y = K.linear(f, w2, b2, act_in=al)
            y.backward(gy)
            grads[fuse] = (x.grad.float(), w1.grad.clone(), b1.grad.clone(), w2.grad.clone(), b2.grad.clone())
        finally:
            K.ACT_FUSE = True
    for a, b, name in zip(grads[True], grads[False], ("x", "w1", "b1", "w2", "b2")):
        assert _rel(a, b) < 1e-3, name


def test_gemm_swiglu_bwd_matches_two_pass():
    """The down projection's data gradient with the SwiGLU backward in its epilogue (dgu [M, 2F] from g . w and gu)
    against the two-pass form on the same kernels (bit-identical: same accumulators, same bf16 rounding, the SwiGLU
    kernel's formula) and against an fp32 reference."""
    torch.manual_seed(4)
    C = _C()
    M, F, K = 4096, 4096, 512
    assert C.gemm_swiglu_bwd_ok(M, F, K)
    g = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(K, F, device="cuda") * 0.05).bfloat16()
    gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
    dgu = C.gemm_swiglu_bwd(g, w, gu)
    dy = C.gemm(g, True, w, False, None, False, None, 0, None, False, 1.0, 1)
    two = C.swiglu_bwd(gu, dy)
    assert torch.equal(dgu, two)
    gg, uu = gu.float().split(F, -1)
    s = torch.sigmoid(gg)
    d = g.float() @ w.float()
    ref = torch.cat([d * uu * s * (1 + gg * (1 - s)), d * gg * s], -1)
    assert _rel(dgu, ref) < 2e-2


def _blocked_split(gu, blk=64):
    F2 = gu.shape[-1] // 2
    v = gu.float().reshape(gu.shape[0], F2 // blk, 2, blk)
    return v[:, :, 0].reshape(gu.shape[0], F2), v[:, :, 1].reshape(gu.shape[0], F2)


def test_gemm_swiglu_fwd_matches_two_pass():
    """The gate|up projection with the SwiGLU in its epilogue (gemm256.hip copy_out_swiglu: gu and h = silu(g) u
    from one 4-wave GEMM, gate / up in 64-column blocks) against the plain GEMM + the blocked SwiGLU kernel
    (bit-identical: same accumulation, same bf16 rounding, the SwiGLU kernel's formula) and an fp32 reference."""
    torch.manual_seed(5)
    C = _C()
    M, F, K = 4096, 4096, 512
    assert C.gemm_swiglu_fwd_ok(M, F, K)
    x = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(2 * F, K, device="cuda") * 0.05).bfloat16()
    gu, h = C.gemm_swiglu_fwd(x, w)
    gu2 = C.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1)
    assert torch.equal(gu, gu2)
    assert torch.equal(h, C.swiglu_fwd(gu2, 64))
    g, u = _blocked_split((x.float() @ w.float().t()))
    assert _rel(h, torch.nn.functional.silu(g) * u) < 2e-2


def test_gemm_swiglu_bwd_blocked_matches_two_pass():
    """The SwiGLU backward in the down projection's data gradient on the 64-blocked gate|up layout (act -4) against
    the two-pass form (blocked SwiGLU-backward kernel), bit-identical, and an fp32 reference."""
    torch.manual_seed(6)
    C = _C()
    M, F, K = 4096, 4096, 512
    g = (torch.randn(M, K, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(K, F, device="cuda") * 0.05).bfloat16()
    gu = torch.randn(M, 2 * F, device="cuda").bfloat16()
    dgu = C.gemm_swiglu_bwd(g, w, gu, 64)
    dy = C.gemm(g, True, w, False, None, False, None, 0, None, False, 1.0, 1)
    assert torch.equal(dgu, C.swiglu_bwd(gu, dy, 64))
    gg, uu = _blocked_split(gu)
    s = torch.sigmoid(gg)
    d = g.float() @ w.float()
    dg, du = d * uu * s * (1 + gg * (1 - s)), d * gg * s
    ref = torch.stack([dg.reshape(M, -1, 64), du.reshape(M, -1, 64)], 2).reshape(M, 2 * F)
    assert _rel(dgu, ref) < 2e-2


def test_gemm_rope_matches_two_pass():
    """The QKV projection with the q / k rotary embedding in the 4-wave GEMM's copy-out (gemm256.hip copy_out_rope)
    against the plain GEMM + the in-place rope kernel (bit-identical: same staged bf16 values, the same explicit-fma
    formula) and against an fp32 reference; the v heads pass through unrotated."""
    from k8s_amd.ops import nn as K

    torch.manual_seed(7)
    C = _C()
    B, S, H, Hkv, D = 8, 2048, 8, 2, 128  # 64 x 6 = 384 output tiles: a full wave of the 4-wave kernel
    M, N, Kd, rot = B * S, (H + 2 * Hkv) * D, 512, (H + Hkv) * D
    assert C.gemm_rope_ok(M, N, Kd, rot)
    x = (torch.randn(M, Kd, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(N, Kd, device="cuda") * 0.05).bfloat16()
    pos = torch.arange(S, device="cuda", dtype=torch.int32).repeat(B)
    table = K.rope_table(4096, D, 500000.0, "cuda")
    y = C.gemm_rope(x, w, pos, table, rot)
    y2 = C.gemm(x, True, w, True, None, False, None, 0, None, False, 1.0, 1)
    C.rope_(y2[:, :rot], pos, table, False)
    assert torch.equal(y, y2)
    ref = x.float() @ w.float().t()
    ref = torch.cat([K._rope_ref(ref[:, :rot], pos, table), ref[:, rot:]], -1)
    assert _rel(y, ref) < 2e-2
