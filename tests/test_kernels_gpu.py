"""Numerics of the gfx950 HIP kernels vs the plain-PyTorch fp32 references."""
import pytest
import torch

from k8s_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _C():
    from k8s_amd.ops._ext import load

    return load()


def _close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * max(1.0, scale), "max err %g (scale %g)" % (err, scale)


@pytest.mark.parametrize("C,M", [(64, 4096), (256, 1000), (2048, 98), (24, 333)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_fwd_bwd(cuda, C, M, relu, res):
    torch.manual_seed(0)
    x = (torch.randn(M, C, device=cuda) * 3 + 1).bfloat16()
    r = torch.randn(M, C, device=cuda).bfloat16() if res else None
    g = torch.rand(C, device=cuda) + 0.5
    b = torch.randn(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    rm2, rv2 = rm.clone(), rv.clone()
    y, mean, invstd = _C().bn_fwd(x, r, g, b, rm, rv, True, 0.1, 1e-5, relu)
    yr, meanr, invr = ref.bn_fwd(x, r, g, b, rm2, rv2, True, 0.1, 1e-5, relu)
    _close(mean, meanr, 1e-4)
    _close(invstd, invr, 1e-3)
    _close(y, yr, 2e-2)
    _close(rm, rm2, 1e-4)
    _close(rv, rv2, 1e-3)
    dy = torch.randn(M, C, device=cuda).bfloat16()
    dg, db = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    dx, dres = _C().bn_bwd(dy, x, y if relu else None, mean, invstd, g, b, False, dg, db, res)
    dxr, dresr, dgr, dbr = ref.bn_bwd(dy, x, yr if relu else None, meanr, invr, g)
    _close(dg, dgr, 2e-2)
    _close(db, dbr, 2e-2)
    _close(dx, dxr, 3e-2)
    if res:
        _close(dres, dresr, 1e-2)


@pytest.mark.parametrize("C,M", [(64, 4096), (256, 1000), (2048, 98)])
def test_bn_from_conv_sums_and_relu_from_x(cuda, C, M):
    """BN fed by conv-epilogue statistics (replicated partial sums) and backward with the ReLU mask
    recomputed from x must match the two-pass kernels."""
    torch.manual_seed(7)
    x = (torch.randn(M, C, device=cuda) * 2 + 0.5).bfloat16()
    g = torch.rand(C, device=cuda) + 0.5
    b = torch.randn(C, device=cuda)
    R = _C().conv_stat_replicas
    sums = torch.zeros(R, 2, C, device=cuda)
    xf = x.float()
    for r in range(R):  # spread the row sums over the replicas like the conv epilogue does
        part = xf[r::R]
        sums[r, 0] = part.sum(0)
        sums[r, 1] = (part * part).sum(0)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, mean, invstd = _C().bn_fwd_from_sums(x, None, g, b, sums, rm, rv, 0.1, 1e-5, True)
    yr, meanr, invr = ref.bn_fwd(x, None, g, b, torch.zeros(C, device=cuda), torch.ones(C, device=cuda), True, 0.1,
                                 1e-5, True)
    _close(mean, meanr, 1e-4)
    _close(invstd, invr, 1e-3)
    _close(y, yr, 2e-2)
    dy = torch.randn(M, C, device=cuda).bfloat16()
    dg, db = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    dx, _ = _C().bn_bwd(dy, x, None, mean, invstd, g, b, True, dg, db, False)
    dxr, _, dgr, dbr = ref.bn_bwd(dy, x, y, mean, invstd, g)
    _close(dx, dxr, 3e-2)
    _close(dg, dgr, 2e-2)
    _close(db, dbr, 2e-2)


@pytest.mark.parametrize("D", [768, 4096, 1024, 136])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("res", [False, True])
# one partial block / many, ragged tails; 16411 rows: the fused one-pass backward of short rows (D <= 1024), its last
# block partial and an odd row count (the two-row trips' early exit)
@pytest.mark.parametrize("R", [257, 2100, 16411])
def test_norm_fwd_bwd(cuda, D, rms, res, R):
    torch.manual_seed(1)
    x = torch.randn(R, D, device=cuda).bfloat16()
    r = torch.randn(R, D, device=cuda).bfloat16() if res else None
    g = torch.rand(D, device=cuda) + 0.5
    b = None if rms else torch.randn(D, device=cuda)
    y, mean, rstd, xs = _C().norm_fwd(x, r, g, b, 1e-5, rms)
    yr, meanr, rstdr, xsr = ref.norm_fwd(x, r, g, b, 1e-5, rms)
    _close(y, yr, 2e-2)
    _close(rstd, rstdr, 1e-3)
    xin = xs if res else x
    dy = torch.randn(R, D, device=cuda).bfloat16()
    dres = torch.randn(R, D, device=cuda).bfloat16() if res else None
    dg = torch.empty(D, device=cuda)
    db = None if rms else torch.empty(D, device=cuda)
    dx = _C().norm_bwd(dy, xin, g, mean, rstd, dres, dg, db, rms)
    dxr, dgr, dbr = ref.norm_bwd(dy, xin, g, meanr, rstdr, dres, rms)
    _close(dx, dxr, 3e-2)
    _close(dg, dgr, 2e-2)
    if not rms:
        _close(db, dbr, 2e-2)
    if not res:  # the dx column sums (the producing linear's bias gradient) from the parameter kernel
        dsum = torch.empty(D, device=cuda)
        dx2 = _C().norm_bwd(dy, xin, g, mean, rstd, None, dg, db, rms, dsum=dsum)
        assert torch.equal(dx2, dx)
        _close(dsum, dxr.float().sum(0), 2e-2)


@pytest.mark.parametrize("R,V,dt", [(64, 1000, torch.bfloat16), (8, 30522, torch.bfloat16), (16, 1003, torch.float32),
                                    (4, 128256, torch.bfloat16)])
@pytest.mark.parametrize("smooth", [0.0, 0.1])
def test_xent(cuda, R, V, dt, smooth):
    torch.manual_seed(2)
    x = (torch.randn(R, V, device=cuda) * 4).to(dt)
    lab = torch.randint(0, V, (R,), device=cuda)
    lab[1] = -100
    loss, lse = _C().xent_fwd(x, lab, -100, smooth)
    lr, lser = ref.xent_fwd(x, lab, -100, smooth)
    _close(lse, lser, 1e-4)
    _close(loss, lr, 1e-3)
    ds = torch.tensor([0.37], device=cuda)
    d = _C().xent_bwd(x, lab, lse, ds, -100, smooth, V)
    dr = ref.xent_bwd(x, lab, lser, ds, -100, smooth)
    _close(d, dr, 2e-2 if dt == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("Vpad", [30528, 30720])  # BERT's word table at 64- / 256-column padding
def test_xent_padded_vocab(cuda, Vpad):
    """logits [R, Vpad] with the classes in the first V columns: the gradient's pad columns come back zero even when
    the output buffer starts as garbage (the binding allocates it uninitialised)."""
    torch.manual_seed(5)
    R, V = 32, 30522
    full = (torch.randn(R, Vpad, device=cuda) * 4).bfloat16()
    lab = torch.randint(0, V, (R,), device=cuda)
    loss, lse = _C().xent_fwd(full[:, :V], lab, -100, 0.0)
    _, lser = ref.xent_fwd(full[:, :V].contiguous(), lab, -100, 0.0)
    _close(lse, lser, 1e-4)
    ds = torch.tensor([1.0], device=cuda)
    torch.full((R * Vpad * 4,), float("nan"), device=cuda)  # dirty the caching allocator's free blocks
    d = _C().xent_bwd(full, lab, lse, ds, -100, 0.0, V)
    assert d.shape == (R, Vpad)
    assert torch.equal(d[:, V:], torch.zeros_like(d[:, V:]))
    _close(d[:, :V], ref.xent_bwd(full[:, :V].contiguous(), lab, lser, ds, -100, 0.0), 2e-2)


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nesterov", [False, True])
def test_fused_sgd(cuda, gdt, nesterov):
    torch.manual_seed(3)
    n = 64 * 1000
    p = torch.randn(n, device=cuda)
    mom = torch.randn(n, device=cuda)
    g = torch.randn(n, device=cuda).to(gdt)
    mask = (torch.rand(n // 64, device=cuda) > 0.5).to(torch.uint8)
    pbf = torch.empty(n, device=cuda, dtype=torch.bfloat16)
    p2, m2, pbf2 = p.clone(), mom.clone(), pbf.clone()
    st = torch.tensor([0.5], device=cuda)
    _C().fused_sgd(p, mom, g, pbf, mask, 0.1, 0.9, 1e-2, 0.25, st, nesterov, False)
    ref.sgd(p2, m2, g, pbf2, mask, 0.1, 0.9, 1e-2, 0.25, st, nesterov, False)
    _close(p, p2, 1e-6)
    _close(mom, m2, 1e-6)
    _close(pbf, pbf2, 1e-2)


@pytest.mark.parametrize("decoupled", [True, False])
def test_fused_adam(cuda, decoupled):
    torch.manual_seed(4)
    n = 64 * 777
    p = torch.randn(n, device=cuda)
    m1 = torch.randn(n, device=cuda) * 0.1
    m2 = torch.rand(n, device=cuda) * 0.1
    g = torch.randn(n, device=cuda).bfloat16()
    mask = (torch.rand(n // 64, device=cuda) > 0.3).to(torch.uint8)
    P, A, B = p.clone(), m1.clone(), m2.clone()
    _C().fused_adam(p, m1, m2, g, None, mask, 1e-3, 0.9, 0.999, 1e-8, 0.01, 0.5, None, 7, decoupled)
    ref.adam(P, A, B, g, None, mask, 1e-3, 0.9, 0.999, 1e-8, 0.01, 0.5, None, 7, decoupled)
    _close(p, P, 1e-5)
    _close(m1, A, 1e-6)
    _close(m2, B, 1e-6)


@pytest.mark.parametrize("n", [64 * 100, 64 * (1 << 18) + 192])  # tail-only; 4-vector trips + tail
def test_grad_clip(cuda, n):
    g = torch.randn(n, device=cuda)
    st = _C().grad_sumsq(g)
    _close(st, ref.grad_sumsq(g), 1e-4)
    f = _C().clip_factor(st, 1.0)
    norm = g.norm().item()
    assert abs(f.item() - min(1.0, 1.0 / (norm + 1e-6))) < 1e-5
    g[n // 3] = float("inf")
    st = _C().grad_sumsq(g)
    assert _C().clip_factor(st, 1.0).item() == 0.0
    g[n // 3] = 0.0
    g[5] = float("nan")
    st = _C().grad_sumsq(g)
    assert _C().clip_factor(st, 1.0).item() == 0.0


@pytest.mark.parametrize("C,M", [(64, 4096), (256, 1000), (2048, 98), (24, 333)])
@pytest.mark.parametrize("from_sums", [False, True])
def test_bn_packed_relu_mask(cuda, C, M, from_sums):
    """Residual BN + ReLU: the forward's packed mask (bit j of byte e = y[8e+j] > 0) gives the backward the same
    dx / dres / dgamma / dbeta as reading the bf16 output y."""
    torch.manual_seed(1)
    x = (torch.randn(M, C, device=cuda) * 2).bfloat16()
    r = torch.randn(M, C, device=cuda).bfloat16()
    g = torch.rand(C, device=cuda) + 0.5
    b = torch.randn(C, device=cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    if from_sums:
        xf = x.float()
        sums = torch.zeros(_C().conv_stat_replicas, 2, C, device=cuda)
        sums[0, 0], sums[0, 1] = xf.sum(0), (xf * xf).sum(0)
        y, mean, invstd, mask = _C().bn_fwd_from_sums(x, r, g, b, sums, rm, rv, 0.1, 1e-5, True, True)
    else:
        y, mean, invstd, mask = _C().bn_fwd(x, r, g, b, rm, rv, True, 0.1, 1e-5, True, True)
    assert mask.dtype == torch.uint8 and mask.numel() == M * C // 8
    bits = ((mask.long().unsqueeze(-1) >> torch.arange(8, device=cuda)) & 1).reshape(M, C).bool()
    assert torch.equal(bits, y.float() > 0)
    dy = torch.randn(M, C, device=cuda).bfloat16()
    dg1, db1, dg2, db2 = (torch.empty(C, device=cuda) for _ in range(4))
    dx1, dres1 = _C().bn_bwd(dy, x, y, mean, invstd, g, b, False, dg1, db1, True)
    dx2, dres2 = _C().bn_bwd(dy, x, None, mean, invstd, g, b, False, dg2, db2, True, mask)
    assert torch.equal(dres1, dres2)
    _close(dx2, dx1, 1e-2)
    _close(dg2, dg1, 1e-4)
    _close(db2, db1, 1e-4)


# position rows summed in the tail loop only / in 8-token trips too; 150 tokens: a partial token run
@pytest.mark.parametrize("B,S", [(4, 96), (40, 96), (3, 50)])
@pytest.mark.parametrize("D", [256, 776])
def test_embedding_sum_gather_and_scatter(cuda, B, S, D):
    """BERT-style word + position + token-type lookup (embedding.hip) vs torch gathers; the backward's fp32
    scatter-adds (incl. the 2-row token-type table's register-reduced path and the position table's
    owner-per-row path) vs index_add_. D = 776: the large-table kernel's wave walks 256-column chunks, the last one
    partial."""
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore, init_normal

    torch.manual_seed(3)
    V = 1000
    store = ParamStore()
    word = store.new("word", (V, D), init_normal(0.5))
    pos = store.new("pos", (128, D), init_normal(0.5))
    typ = store.new("typ", (2, D), init_normal(0.5))
    store.finalize(cuda)
    ids = torch.randint(0, V, (B, S), device=cuda)
    tt = torch.randint(0, 2, (B, S), device=cuda)
    out = K.embedding_sum([(ids, word), (None, pos), (tt, typ)], S)
    pids = torch.arange(S, device=cuda).repeat(B)
    ref = (word.master[ids.reshape(-1)].bfloat16().float() + pos.master[pids].bfloat16().float()
           + typ.master[tt.reshape(-1)].bfloat16().float())
    assert ((out.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    g = torch.randn_like(out)
    out.backward(g)
    gf = g.float()
    for p, rows in ((word, ids.reshape(-1)), (pos, pids), (typ, tt.reshape(-1))):
        want = torch.zeros(p.shape, device=cuda).index_add_(0, rows, gf)
        got = p.grad.view(p.shape)
        assert ((got - want).norm() / want.norm()).item() < 1e-5, p.name


def test_global_avg_pool_nhwc(cuda):
    from k8s_amd.ops import nn as K

    torch.manual_seed(4)
    x = torch.randn(8, 7, 7, 2048, device=cuda).bfloat16().requires_grad_(True)
    y = K.global_avg_pool_nhwc(x)
    ref = x.float().mean(dim=(1, 2))
    assert ((y.float() - ref).abs().max()).item() < 1e-2
    g = torch.randn_like(y)
    (dx,) = torch.autograd.grad(y, x, g)
    assert ((dx.float() - (g.float() / 49)[:, None, None, :]).abs().max()).item() < 1e-3


@pytest.mark.parametrize("world,n", [(2, 64 * 1000), (8, 64 * 4097), (8, 999), (3, 8 * 77)])
def test_slice_sum_and_cast_bf16(cuda, world, n):
    """bf16 gradient transport kernels (parallel/ddp.py, ps.py): the fp32->bf16 pack matches torch's rounding and
    the owner's sum of the world received chunks is the fp32 rank-order sum (bitwise), both outputs."""
    torch.manual_seed(world)
    g = torch.randn(world * n, device=cuda) * 3
    send = _C().cast_bf16(g)
    assert torch.equal(send, g.to(torch.bfloat16))
    out = torch.empty(n, device=cuda)
    out_bf = torch.empty(n, device=cuda, dtype=torch.bfloat16)
    _C().slice_sum(send, world, out, out_bf)
    chunks = send.view(world, n).float()
    want = torch.zeros(n, device=cuda)
    for r in range(world):
        want = want + chunks[r]
    assert torch.equal(out, want)
    assert torch.equal(out_bf, want.to(torch.bfloat16))


@pytest.mark.parametrize("N,H,W,C", [(4, 32, 30, 64), (2, 31, 17, 64), (3, 12, 12, 32)])
def test_bn_relu_maxpool_fused_vs_fp32(cuda, N, H, W, C):
    """Stem BN + ReLU + 3x3/s2/p1 max pool in one pass (and its backward gathering the pool gradient inside the BN
    backward) against an fp32 reference: batch statistics, z = bf16(relu(BN(x))) (the stored activation the
    separate kernels would write, so max-pool ties resolve alike), max_pool2d autograd for the pool gradient, then
    the training-mode BatchNorm backward formula."""
    torch.manual_seed(11)
    x = (torch.randn(N, H, W, C, device=cuda) * 2 + 0.3).bfloat16()
    g = torch.rand(C, device=cuda) + 0.5
    b = torch.randn(C, device=cuda) * 0.5
    xf = x.float().reshape(-1, C)
    M = xf.shape[0]
    sums = torch.stack([xf.sum(0), (xf * xf).sum(0)]).reshape(1, 2, C).contiguous()
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y, idx, mean, invstd = _C().bn_relu_maxpool(x, sums, g, b, rm, rv, 0.1, 1e-5)
    assert y.shape == (N, (H + 1) // 2, (W + 1) // 2, C)
    var = xf.var(0, unbiased=False)
    _close(mean, xf.mean(0), 1e-4)
    _close(invstd, torch.rsqrt(var + 1e-5), 1e-3)
    sc = g * invstd
    sh = b - mean * sc
    pre = (x.float() * sc + sh).bfloat16().float()
    z = torch.relu(pre)
    zr = z.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(zr, 3, 2, 1)
    assert torch.equal(y.float().permute(0, 3, 1, 2), yr.detach().bfloat16().float())
    dy = torch.randn_like(y)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    dz = zr.grad.permute(0, 2, 3, 1).bfloat16().float() * (pre > 0)
    dz = dz.reshape(-1, C)
    xhat = (xf - mean) * invstd
    dbr, dgr = dz.sum(0), (dz * xhat).sum(0)
    dxr = (g * invstd) * (dz - dbr / M - xhat * dgr / M)
    dg, db = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    dx = _C().pool_bn_bwd(dy, idx, x, mean, invstd, g, b, dg, db)
    _close(db, dbr, 1e-3)
    _close(dg, dgr, 1e-3)
    rel = ((dx.float().reshape(-1, C) - dxr).norm() / dxr.norm()).item()
    assert rel < 1e-2, rel
    # the BnStatLink outputs (each pooled element's winner x and ReLU bit) and the backward from sums taken over them
    # (what the consumers' dgrad epilogues accumulate: g = bit ? dy : 0, sum g, sum g (x_winner - mean))
    rm2, rv2 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    y2, idx2, mean2, invstd2, xarg, ybits = _C().bn_relu_maxpool(x, sums, g, b, rm2, rv2, 0.1, 1e-5, True)
    assert torch.equal(y2, y) and torch.equal(idx2, idx)
    bits = ((ybits.view(-1, 1) >> torch.arange(8, device=cuda, dtype=torch.uint8)) & 1).bool().view(y.shape)
    assert torch.equal(bits, y > 0)
    # winner x from the saved window position: tap (dh, dw) of window (ho, wo) is pixel (2 ho - 1 + dh, 2 wo - 1 + dw)
    Ho, Wo = y.shape[1], y.shape[2]
    pos = idx.long()
    hh = (2 * torch.arange(Ho, device=cuda).view(1, Ho, 1, 1) - 1 + pos // 3).clamp(0, H - 1)
    ww = (2 * torch.arange(Wo, device=cuda).view(1, 1, Wo, 1) - 1 + pos % 3).clamp(0, W - 1)
    nn_ = torch.arange(N, device=cuda).view(N, 1, 1, 1).expand_as(pos)
    cc = torch.arange(C, device=cuda).view(1, 1, 1, C).expand_as(pos)
    xw = x[nn_, hh, ww, cc]
    valid = y > 0
    assert torch.equal(xarg[valid], xw[valid])
    R = _C().conv_stat_replicas
    gsel = torch.where(bits, dy.float(), torch.zeros_like(dy.float())).reshape(-1, C)
    bsums = torch.zeros(R, 2, C, device=cuda)
    bsums[0, 0] = gsel.sum(0)
    bsums[1, 1] = (gsel * (xarg.float().reshape(-1, C) - mean2)).sum(0)
    dg2, db2 = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    dx2 = _C().pool_bn_bwd_from_sums(dy, idx2, x, mean2, invstd2, g, b, dg2, db2, bsums)
    # sums over the pooled gradient itself: a pixel that wins several windows adds their dy unrounded (the reference
    # and the reduce pass sum the bf16-rounded dz of that pixel), so ~1 bf16 ulp of such pixels apart
    _close(db2, dbr, 5e-3)
    _close(dg2, dgr, 5e-3)
    rel = ((dx2.float().reshape(-1, C) - dxr).norm() / dxr.norm()).item()
    assert rel < 1e-2, rel
