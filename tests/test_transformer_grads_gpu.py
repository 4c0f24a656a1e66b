"""BERT and Llama training steps on the GPU kernels (bf16 MFMA GEMMs, flash attention, fused norms, RoPE,
SwiGLU, fused cross-entropy) vs plain torch.nn.functional fp32 twins on the same weights: loss and every
parameter gradient. The tolerance is the ResNet test's noise-floor rule (tests/test_resnet_gpu.py): a gradient
may differ from fp32 by at most 2x what stock PyTorch bf16 autocast differs by, + 0.03."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _gelu(x):
    return F.gelu(x, approximate="tanh")


def _rms(x, g, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * g.float()).to(x.dtype)


def _rope(x, pos, table):
    T, D = x.shape[0], table.shape[1] * 2
    xs = x.reshape(T, -1, D)
    cs = table[pos.long()]
    c, s = cs[..., 0][:, None, :].to(x.dtype), cs[..., 1][:, None, :].to(x.dtype)
    x1, x2 = xs[..., : D // 2], xs[..., D // 2:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).reshape(x.shape)


def _attn(q, k, v, causal, kv_lens=None):
    """q [B, S, Hq, D], k/v [B, S, Hkv, D] -> [B, S, Hq, D]; GQA by repeating each kv head over its group."""
    B, S, Hq, D = q.shape
    rep = Hq // k.shape[2]
    qh, kh, vh = (t.permute(0, 2, 1, 3) for t in (q, k, v))
    kh, vh = kh.repeat_interleave(rep, 1), vh.repeat_interleave(rep, 1)
    mask = None
    if kv_lens is not None:
        mask = (torch.arange(S, device=q.device)[None, :] < kv_lens[:, None])[:, None, None, :]
    o = F.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask, is_causal=causal, scale=1.0 / math.sqrt(D))
    return o.permute(0, 2, 1, 3)


def _check(store, loss, ref_loss, ref, stock):
    assert abs(loss - ref_loss) < 3e-2 * max(1.0, abs(ref_loss)), (loss, ref_loss)
    bad = []
    for p in store.params:
        if p.name not in ref or ref[p.name] is None:
            continue
        r = ref[p.name].float()
        if r.norm().item() == 0:
            continue
        err = (p.grad.float() - r).norm().item() / r.norm().item()
        floor = (stock[p.name].float() - r).norm().item() / r.norm().item()
        if err > 2.0 * floor + 0.03:
            bad.append((p.name, round(err, 4), round(floor, 4)))
    assert not bad, bad


# ---------------------------------------------------------------------------------------------------- Llama
def _llama_twin(m, store, ids, labels, autocast):
    c = m.c
    P = {p.name: p.master.detach().clone().reshape(p.shape).requires_grad_(True) for p in store.params}
    B, S = ids.shape
    d = c.head_dim
    pos = torch.arange(S, device=ids.device, dtype=torch.int32).repeat(B)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        x = F.embedding(ids, P["model.embed_tokens.weight"]).reshape(B * S, c.hidden)
        for i in range(c.layers):
            n = "model.layers.%d." % i
            h = _rms(x, P[n + "input_layernorm.weight"], c.eps)
            qkv = h @ P[n + "self_attn.qkv_proj.weight"].t()
            q, k, v = qkv.split([c.heads * d, c.kv_heads * d, c.kv_heads * d], -1)
            q, k = _rope(q, pos, m.table), _rope(k, pos, m.table)
            o = _attn(q.reshape(B, S, c.heads, d), k.reshape(B, S, c.kv_heads, d), v.reshape(B, S, c.kv_heads, d),
                      True)
            x = x + o.reshape(B * S, -1) @ P[n + "self_attn.o_proj.weight"].t()
            h = _rms(x, P[n + "post_attention_layernorm.weight"], c.eps)
            gu = h @ P[n + "mlp.gate_up_proj.weight"].t()  # rows in 64-blocked gate|up order (models/llama.py)
            gu = gu.reshape(gu.shape[0], -1, 2, 64)
            g, u = gu[:, :, 0].reshape(gu.shape[0], -1), gu[:, :, 1].reshape(gu.shape[0], -1)
            x = x + (F.silu(g) * u) @ P[n + "mlp.down_proj.weight"].t()
        h = _rms(x, P["model.norm.weight"], c.eps)
        logits = h @ P["lm_head.weight"].t()
    loss = F.cross_entropy(logits.float(), labels.reshape(-1))
    loss.backward()
    return loss.item(), {k: v.grad for k, v in P.items()}


def test_llama_tiny_gradients_match_fp32_twin(cuda):
    from k8s_amd.models.llama import LLAMA_TINY, LlamaForCausalLM, synthetic_batch
    from k8s_amd.parallel.flat import ParamStore

    torch.manual_seed(0)
    store = ParamStore()
    m = LlamaForCausalLM(store, LLAMA_TINY).finalize(cuda, seed=7)
    g = torch.Generator(device=cuda).manual_seed(3)
    ids, labels = synthetic_batch(LLAMA_TINY, 2, 128, cuda, generator=g)
    store.begin_step()
    loss = m(ids, labels)
    loss.backward()
    store.zero_unwritten()
    ref_loss, ref = _llama_twin(m, store, ids, labels, autocast=False)
    _, stock = _llama_twin(m, store, ids, labels, autocast=True)
    _check(store, loss.float().item(), ref_loss, ref, stock)


# ---------------------------------------------------------------------------------------------------- BERT
def _bert_twin(m, store, ids, tt, mlm_labels, nsp_labels, kv_lens, autocast):
    c = m.c
    P = {p.name: p.master.detach().clone().reshape(p.shape).requires_grad_(True) for p in store.params}
    B, S = ids.shape
    h, nh = c.hidden, c.heads
    d = h // nh
    pos_ids = torch.arange(S, device=ids.device).expand(B, S)

    def ln(x, g, b):
        return F.layer_norm(x, (h,), P[g], P[b], c.eps)

    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        e = (F.embedding(ids, P["bert.embeddings.word_embeddings.weight"])
             + F.embedding(pos_ids, P["bert.embeddings.position_embeddings.weight"])
             + F.embedding(tt, P["bert.embeddings.token_type_embeddings.weight"]))
        x = ln(e.reshape(B * S, h), "bert.embeddings.LayerNorm.weight", "bert.embeddings.LayerNorm.bias")
        for i in range(c.layers):
            n = "bert.encoder.layer.%d." % i
            qkv = x @ P[n + "attention.qkv.weight"].t() + P[n + "attention.qkv.bias"]
            q, k, v = qkv.split([h, h, h], -1)
            o = _attn(q.reshape(B, S, nh, d), k.reshape(B, S, nh, d), v.reshape(B, S, nh, d), False, kv_lens)
            a = o.reshape(B * S, h) @ P[n + "attention.output.dense.weight"].t() + P[n + "attention.output.dense.bias"]
            x = ln(a + x, n + "attention.output.LayerNorm.weight", n + "attention.output.LayerNorm.bias")
            f = _gelu(x @ P[n + "intermediate.dense.weight"].t() + P[n + "intermediate.dense.bias"])
            f = f @ P[n + "output.dense.weight"].t() + P[n + "output.dense.bias"]
            x = ln(f + x, n + "output.LayerNorm.weight", n + "output.LayerNorm.bias")
        t = _gelu(x @ P["cls.predictions.transform.dense.weight"].t() + P["cls.predictions.transform.dense.bias"])
        t = ln(t, "cls.predictions.transform.LayerNorm.weight", "cls.predictions.transform.LayerNorm.bias")
        logits = t @ P["bert.embeddings.word_embeddings.weight"].t() + P["cls.predictions.bias"]
        cls = x.reshape(B, S, h)[:, 0]
        pooled = torch.tanh(cls @ P["bert.pooler.dense.weight"].t() + P["bert.pooler.dense.bias"])
        nsp_logits = pooled @ P["cls.seq_relationship.weight"].t() + P["cls.seq_relationship.bias"]
    mlm = F.cross_entropy(logits.float()[:, :c.vocab_size], mlm_labels.reshape(-1), ignore_index=-100)
    nsp = F.cross_entropy(nsp_logits.float()[:, :2], nsp_labels)
    loss = mlm + nsp
    loss.backward()
    return loss.item(), {k: v.grad for k, v in P.items()}


@pytest.mark.parametrize("gathered", [True, False])
def test_bert_tiny_gradients_match_fp32_twin(cuda, gathered):
    """gathered: MLM head on the masked-position slots (pretraining data format); the twin runs the head on every
    token with the equivalent dense labels, so the two must agree on loss and every gradient."""
    import dataclasses

    from k8s_amd.models.bert import BERT_TINY, BertForPreTraining, dense_mlm_labels, synthetic_batch
    from k8s_amd.parallel.flat import ParamStore

    torch.manual_seed(0)
    cfg = BERT_TINY if gathered else dataclasses.replace(BERT_TINY, max_predictions=0)
    store = ParamStore()
    m = BertForPreTraining(store, cfg).finalize(cuda, seed=11)
    g = torch.Generator(device=cuda).manual_seed(4)
    batch = synthetic_batch(cfg, 4, 128, cuda, generator=g, mask_prob=0.3 if not gathered else 0.08)
    ids, tt, labels, nsp = batch[:4]
    pos = batch[4] if gathered else None
    dense = dense_mlm_labels(labels, pos, 128) if gathered else labels
    kv_lens = torch.tensor([128, 100, 64, 128], device=cuda, dtype=torch.int32)
    store.begin_step()
    loss, _, _ = m(ids, tt, labels, nsp, pos, kv_lens=kv_lens)
    loss.backward()
    store.zero_unwritten()
    ref_loss, ref = _bert_twin(m, store, ids, tt, dense, nsp, kv_lens, autocast=False)
    _, stock = _bert_twin(m, store, ids, tt, dense, nsp, kv_lens, autocast=True)
    # padded key rows of the [CLS]-only NSP head see no gradient in either path; pad decoder columns neither
    _check(store, loss.float().item(), ref_loss, ref, stock)


def test_llama_swiglu_fused_backward_matches_unfused(cuda):
    """Llama with the SwiGLU backward inside the down projection's data gradient (nn.SwiGLULink) gives the same
    loss and parameter gradients as the separate SwiGLU-backward pass (a shape the 4-wave kernel takes:
    4,096 tokens x 4,096 intermediate)."""
    import dataclasses

    from k8s_amd.models import llama as M
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore

    cfg = dataclasses.replace(M.LLAMA_TINY, layers=1, intermediate=4096, max_position=1024)
    out = []
    for fuse in (False, True):
        K.SWIGLU_FUSE = fuse
        try:
            store = ParamStore()
            model = M.LlamaForCausalLM(store, cfg).finalize(cuda, seed=2)
            gen = torch.Generator(device=cuda)
            gen.manual_seed(3)
            batch = M.synthetic_batch(cfg, 4, 1024, cuda, generator=gen)
            store.begin_step()
            loss = model(*batch, dtype=torch.bfloat16)
            loss.backward()
            store.zero_unwritten()
            out.append((loss.float().item(), store.grad.clone()))
        finally:
            K.SWIGLU_FUSE = True
    (l0, g0), (l1, g1) = out
    assert l0 == l1
    assert torch.equal(g0, g1), (g0 - g1).abs().max().item()


def test_llama_swiglu_epilogue_matches_separate_pass(cuda):
    """Llama with the SwiGLU in the gate|up GEMM's epilogue (ops.nn.linear_swiglu) gives the same loss and parameter
    gradients, bitwise, as the projection followed by the separate SwiGLU kernel (a shape the 4-wave kernel takes)."""
    import dataclasses

    from k8s_amd.models import llama as M
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore

    cfg = dataclasses.replace(M.LLAMA_TINY, layers=1, intermediate=4096, max_position=1024)
    assert K._C().gemm_swiglu_fwd_ok(4 * 1024, cfg.intermediate, cfg.hidden)  # the epilogue path is the one taken
    out = []
    for epi in (False, True):
        K.SWIGLU_EPI = epi
        try:
            store = ParamStore()
            model = M.LlamaForCausalLM(store, cfg).finalize(cuda, seed=2)
            gen = torch.Generator(device=cuda)
            gen.manual_seed(3)
            batch = M.synthetic_batch(cfg, 4, 1024, cuda, generator=gen)
            store.begin_step()
            loss = model(*batch, dtype=torch.bfloat16)
            loss.backward()
            store.zero_unwritten()
            out.append((loss.float().item(), store.grad.clone()))
        finally:
            K.SWIGLU_EPI = True
    (l0, g0), (l1, g1) = out
    assert l0 == l1
    assert torch.equal(g0, g1), (g0 - g1).abs().max().item()


def test_llama_rope_epilogue_matches_in_place_rope(cuda):
    """Llama with the q / k rotary embedding in the QKV GEMM's epilogue (ops.nn.linear_rope + attention_qkv
    rope_applied) gives the same loss and parameter gradients, bitwise, as the in-place rope pass (a shape the 4-wave
    kernel takes)."""
    import dataclasses

    from k8s_amd.models import llama as M
    from k8s_amd.ops import nn as K
    from k8s_amd.parallel.flat import ParamStore

    cfg = dataclasses.replace(M.LLAMA_TINY, layers=1, hidden=2048, heads=16, kv_heads=4, intermediate=4096,
                              max_position=1024)
    # 8 x 1024 tokens x 24 heads of 128: 32 x 12 tiles of the 4-wave kernel, so the epilogue path is the one taken
    assert K._C().gemm_rope_ok(8 * 1024, (cfg.heads + 2 * cfg.kv_heads) * 128, cfg.hidden,
                               (cfg.heads + cfg.kv_heads) * 128)
    out = []
    for epi in (False, True):
        K.ROPE_EPI = epi
        try:
            store = ParamStore()
            model = M.LlamaForCausalLM(store, cfg).finalize(cuda, seed=2)
            gen = torch.Generator(device=cuda)
            gen.manual_seed(3)
            batch = M.synthetic_batch(cfg, 8, 1024, cuda, generator=gen)
            store.begin_step()
            loss = model(*batch, dtype=torch.bfloat16)
            loss.backward()
            store.zero_unwritten()
            out.append((loss.float().item(), store.grad.clone()))
        finally:
            K.ROPE_EPI = True
    (l0, g0), (l1, g1) = out
    assert l0 == l1
    assert torch.equal(g0, g1), (g0 - g1).abs().max().item()
