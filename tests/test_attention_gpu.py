"""Flash attention (K5) fwd/bwd vs the fp32 matmul/softmax reference: strided QKV views, GQA, causal,
key-padding lengths, sequence tails."""
import math

import pytest
import torch

from k8s_amd.ops.attention import _Flash, attention_reference

pytestmark = pytest.mark.gpu


def _close(a, b, tol, what):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= tol * max(1.0, scale), "%s: max err %g (scale %g)" % (what, err, scale)


CASES = [
    # B, S, Hq, Hkv, D, causal, lens
    (2, 128, 12, 12, 64, False, None),
    (2, 200, 4, 4, 64, False, [200, 77]),
    (1, 256, 8, 2, 128, True, None),
    (2, 333, 4, 1, 128, True, None),
    (2, 192, 4, 4, 128, False, [1, 150]),
    (1, 64, 2, 2, 64, True, None),
    (1, 1100, 4, 2, 64, True, None),        # D = 64 long sequence: 128-wide key / query tiles
    (2, 1024, 2, 2, 64, False, [1024, 900]),
    (1, 4096, 32, 8, 128, True, None),      # Llama-3-8B attention at the benchmarked sequence length
    (1, 2048, 12, 12, 64, False, None),     # BERT-style heads at a long sequence
    # causal dK/dV split into chunks (fp32 partials + reduce): GQA group of 3 (chunks straddle query heads), key
    # lengths (key blocks past kv_len have empty chunks), ragged last query tile
    (2, 700, 6, 2, 128, True, [700, 333]),
    (1, 600, 2, 2, 64, True, [450]),
    # one-block backward of short sequences (S <= 128, D = 64, no GQA): one query half, ragged key chunk, key
    # lengths incl. an empty row, causal with lengths, and a GQA short case that keeps the three-kernel form
    (3, 77, 4, 4, 64, False, [77, 30, 0]),
    (2, 128, 3, 3, 64, True, [128, 65]),
    (2, 100, 4, 4, 64, True, None),
    (2, 128, 4, 2, 64, False, None),
]


@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal,lens", CASES)
def test_flash_fwd_bwd(cuda, B, S, Hq, Hkv, D, causal, lens):
    torch.manual_seed(0)
    # q, k, v as column slices of one fused projection output (the models' layout)
    qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=cuda).bfloat16()
    q = qkv[..., :Hq * D].view(B, S, Hq, D)
    k = qkv[..., Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D)
    v = qkv[..., (Hq + Hkv) * D:].view(B, S, Hkv, D)
    kv_lens = torch.tensor(lens, device=cuda, dtype=torch.int32) if lens else None
    scale = 1.0 / math.sqrt(D)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref = attention_reference(qr, kr, vr, causal, kv_lens, scale)
    qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    out = _Flash.apply(qq, kk, vv, causal, kv_lens, scale)
    valid = torch.ones(B, S, 1, 1, device=cuda)
    if lens:  # rows whose keys are all masked: the reference gives NaN, the kernel 0
        for bi, n in enumerate(lens):
            if n == 0:
                valid[bi] = 0
    _close(out * valid, torch.nan_to_num(ref) * valid, 2e-2, "O")
    do = torch.randn_like(out)
    ref.backward(do.float())
    out.backward(do)
    _close(qq.grad, torch.nan_to_num(qr.grad), 3e-2, "dQ")
    _close(kk.grad, torch.nan_to_num(kr.grad), 3e-2, "dK")
    _close(vv.grad, torch.nan_to_num(vr.grad), 3e-2, "dV")


def test_flash_lse(cuda):
    from k8s_amd.ops._ext import load

    torch.manual_seed(1)
    B, S, H, D = 1, 130, 2, 128
    q, k, v = (torch.randn(B, S, H, D, device=cuda).bfloat16() for _ in range(3))
    o, lse = load().flash_fwd(q, k, v, False, None, 0.1)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * 0.1
    ref = torch.logsumexp(s, -1) / math.log(2.0)  # the kernel stores log2-domain lse
    _close(lse[..., :S], ref, 1e-3, "lse")


@pytest.mark.parametrize("B,S,H,Hkv,D,causal,rope,lens", [
    (2, 128, 12, 12, 64, False, False, True),    # BERT-style, key padding
    (1, 512, 32, 8, 128, True, True, False),     # Llama-style GQA + rotary
])
def test_attention_qkv_packed_matches_split(cuda, B, S, H, Hkv, D, causal, rope, lens):
    """attention_qkv (strided q/k/v views of the fused projection, in-place rotary, packed dqkv written in place)
    against the fp32 split + rope + reference-attention composition, forward and the packed gradient."""
    from k8s_amd.ops import nn as K
    from k8s_amd.ops.attention import attention_qkv, attention_reference

    torch.manual_seed(7)
    W = (H + 2 * Hkv) * D
    qkv = (torch.randn(B * S, W, device=cuda) * 0.5).bfloat16().requires_grad_(True)
    pos = torch.arange(S, device=cuda, dtype=torch.int32).repeat(B)
    table = K.rope_table(S, D, device=cuda)
    kv_lens = torch.tensor([S - 17 * (i + 1) for i in range(B)], device=cuda, dtype=torch.int32) if lens else None
    o = attention_qkv(qkv, B, S, H, Hkv, D, causal=causal, kv_lens=kv_lens,
                      rope=(pos, table) if rope else None)
    go = torch.randn_like(o)
    (g,) = torch.autograd.grad(o, qkv, go)

    xr = qkv.detach().float().requires_grad_(True)
    q, k, v = xr.split([H * D, Hkv * D, Hkv * D], dim=-1)
    if rope:
        q, k = K._rope_ref(q, pos, table), K._rope_ref(k, pos, table)
    ref = attention_reference(q.reshape(B, S, H, D), k.reshape(B, S, Hkv, D), v.reshape(B, S, Hkv, D), causal,
                              kv_lens)
    (gr,) = torch.autograd.grad(ref, xr, go.float())
    rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
    assert rel(o, ref) < 2e-2
    assert rel(g, gr) < 3e-2


@pytest.mark.parametrize("B,S,H,causal,lens", [(3, 128, 4, False, [128, 60, 0]), (2, 77, 3, True, None),
                                                (300, 16, 2, False, None)])  # > 256 partial rows: two-level fold
def test_flash_bwd_packed_bias_grad(cuda, B, S, H, causal, lens):
    """One-block backward's column partials of the packed gradient (the QKV projection's bias gradient, folded over
    the batch) against the column sums of the dqkv it wrote."""
    from k8s_amd.ops._ext import load

    C = load()
    D = 64
    assert C.flash_bwd_one_block(D, S, S, H, H, causal, B)
    torch.manual_seed(3)
    x = torch.randn(B * S, 3 * H * D, device=cuda).bfloat16()
    g = x.view(B, S, 3 * H, D)
    q, k, v = g.narrow(2, 0, H), g.narrow(2, H, H), g.narrow(2, 2 * H, H)
    lens_t = torch.tensor(lens, device=cuda, dtype=torch.int32) if lens else None
    o, lse = C.flash_fwd(q, k, v, causal, lens_t, 0.125)
    do = torch.randn_like(o)
    dqkv = torch.empty_like(x)
    db = torch.full((3 * H * D,), float("nan"), device=cuda)
    C.flash_bwd(do, q, k, v, o, lse, causal, lens_t, 0.125, dqkv, db)
    ref = dqkv.float().sum(0)
    _close(db, ref, 2e-2, "db")


def test_attention_qkv_rope_in_place_matches_copy(cuda):
    """rope_in_place=True (the q / k columns of the projection output rotated where they are) gives the same output
    and the same gradient at the projection's input as the copying form."""
    from k8s_amd.ops import nn as K
    from k8s_amd.ops.attention import attention_qkv

    torch.manual_seed(9)
    B, S, H, Hkv, D = 2, 256, 8, 2, 128
    W = (H + 2 * Hkv) * D
    base = (torch.randn(B * S, W, device=cuda) * 0.5).bfloat16()
    pos = torch.arange(S, device=cuda, dtype=torch.int32).repeat(B)
    table = K.rope_table(S, D, device=cuda)
    outs = []
    for in_place in (False, True):
        leaf = base.clone().requires_grad_(True)
        qkv = leaf * 1.0  # a non-leaf temporary, as a projection output is
        o = attention_qkv(qkv, B, S, H, Hkv, D, causal=True, rope=(pos, table), rope_in_place=in_place)
        go = torch.ones_like(o) * 0.01
        (g,) = torch.autograd.grad(o, leaf, go)
        outs.append((o.float(), g.float()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
