"""BERT-base pretraining model (MLM + NSP) on the k8s_amd op set.

BASELINE config 3: "BERT-base TfJob 8 WORKER data-parallel, fused Adam HIP
kernel". Architecture = bert-base-uncased: vocab 30522 (padded to 30528 so
every GEMM is MFMA-tile friendly; the 6 pad logits are excluded from the loss
by the cross-entropy kernel's row stride), hidden 768, 12 layers, 12 heads,
FFN 3072, GELU, post-LN, LayerNorm eps 1e-12, max 512 positions, 2 token
types. MLM decoder weights are tied to the word embeddings (the flat store
counts the two uses, ``Param.uses = 2``).

Per layer the hot path is: fused QKV GEMM -> flash attention (key-padding
mask) -> O GEMM (+bias) -> add & LayerNorm fused kernel -> FFN1 GEMM with
bias+GELU epilogue -> FFN2 GEMM (+bias) -> add & LayerNorm.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from k8s_amd.ops import nn as K
from k8s_amd.ops.attention import attention_qkv
from k8s_amd.parallel.flat import ParamStore, init_const, init_normal


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    init_std: float = 0.02
    # masked-LM slots per sequence (``max_predictions_per_seq`` of the original pretraining data): the MLM head runs
    # on the gathered masked positions only; 0 = head on every token with dense [B, S] labels
    max_predictions: int = 20

    # the word table / tied decoder padded to whole 256-column tiles: the MLM decoder's three products (logits, their
    # data and weight gradients) then run on the 4-wave 256 x 256 GEMM instead of the ring kernel's ragged-N path
    # (the loss masks the padded logits: cross_entropy(valid=vocab_size))
    vocab_pad: int = 256

    @property
    def padded_vocab(self) -> int:
        return (self.vocab_size + self.vocab_pad - 1) // self.vocab_pad * self.vocab_pad


BERT_BASE = BertConfig()
BERT_TINY = BertConfig(vocab_size=1000, hidden=128, layers=2, heads=2, intermediate=512, max_position=128,
                       max_predictions=12)


class BertLayer(nn.Module):
    def __init__(self, store: ParamStore, name: str, c: BertConfig):
        super().__init__()
        h, f = c.hidden, c.intermediate
        std = init_normal(c.init_std)
        self.c = c
        self.qkv_w = store.new(name + ".attention.qkv.weight", (3 * h, h), std)
        self.qkv_b = store.new(name + ".attention.qkv.bias", (3 * h,), init_const(0), decay=False, lowp=False)
        self.o_w = store.new(name + ".attention.output.dense.weight", (h, h), std)
        self.o_b = store.new(name + ".attention.output.dense.bias", (h,), init_const(0), decay=False, lowp=False)
        self.ln1_g = store.new(name + ".attention.output.LayerNorm.weight", (h,), init_const(1), decay=False,
                               lowp=False)
        self.ln1_b = store.new(name + ".attention.output.LayerNorm.bias", (h,), init_const(0), decay=False,
                               lowp=False)
        self.f1_w = store.new(name + ".intermediate.dense.weight", (f, h), std)
        self.f1_b = store.new(name + ".intermediate.dense.bias", (f,), init_const(0), decay=False, lowp=False)
        self.f2_w = store.new(name + ".output.dense.weight", (h, f), std)
        self.f2_b = store.new(name + ".output.dense.bias", (h,), init_const(0), decay=False, lowp=False)
        self.ln2_g = store.new(name + ".output.LayerNorm.weight", (h,), init_const(1), decay=False, lowp=False)
        self.ln2_b = store.new(name + ".output.LayerNorm.bias", (h,), init_const(0), decay=False, lowp=False)

    def forward(self, x, B, S, kv_lens):
        c = self.c
        h, nh = c.hidden, c.heads
        d = h // nh
        # x is read by the QKV GEMM and, as the residual, by LN1 (likewise LN1's output by FFN1 and LN2): each
        # GradLink sums the two gradient contributions in the GEMM's dgrad epilogue instead of a separate add
        l1, l2 = K.GradLink(), K.GradLink()
        # and the O / FFN2 bias gradients come from the LayerNorm backward that reads their outputs (BiasLink)
        # (and short sequences take the QKV bias gradient from the attention backward's column partials)
        b0, b1, b2 = K.BiasLink(), K.BiasLink(), K.BiasLink()
        qkv = K.linear(x, self.qkv_w, self.qkv_b, grad_link=l1, bias_link=b0)  # [T, 3h]
        o = attention_qkv(qkv, B, S, nh, nh, d, causal=False, kv_lens=kv_lens,
                          bias_link=b0)  # packed QKV gradient in place
        a = K.linear(o.reshape(B * S, h), self.o_w, self.o_b, bias_link=b1)
        x, _ = K.layer_norm(a, self.ln1_g, self.ln1_b, c.eps, residual=x, res_link=l1, bias_link=b1)
        # FFN1's GELU backward and bias gradient inside FFN2's data-gradient epilogue (ActLink)
        al = K.ActLink()
        f = K.linear(x, self.f1_w, self.f1_b, act="gelu", grad_link=l2, act_link=al)
        f = K.linear(f, self.f2_w, self.f2_b, bias_link=b2, act_in=al)
        x, _ = K.layer_norm(f, self.ln2_g, self.ln2_b, c.eps, residual=x, res_link=l2, bias_link=b2)
        return x


class BertForPreTraining(nn.Module):
    def __init__(self, store: ParamStore, c: BertConfig = BERT_BASE):
        super().__init__()
        self.store, self.c = store, c
        h = c.hidden
        std = init_normal(c.init_std)
        self.word = store.new("bert.embeddings.word_embeddings.weight", (c.padded_vocab, h), std)
        self.word.uses = 2  # embedding gather + tied MLM decoder
        self.pos = store.new("bert.embeddings.position_embeddings.weight", (c.max_position, h), std)
        self.typ = store.new("bert.embeddings.token_type_embeddings.weight", (c.type_vocab, h), std)
        self.emb_ln_g = store.new("bert.embeddings.LayerNorm.weight", (h,), init_const(1), decay=False, lowp=False)
        self.emb_ln_b = store.new("bert.embeddings.LayerNorm.bias", (h,), init_const(0), decay=False, lowp=False)
        self.layers = nn.ModuleList([BertLayer(store, "bert.encoder.layer.%d" % i, c) for i in range(c.layers)])
        self.pool_w = store.new("bert.pooler.dense.weight", (h, h), std)
        self.pool_b = store.new("bert.pooler.dense.bias", (h,), init_const(0), decay=False, lowp=False)
        self.mlm_w = store.new("cls.predictions.transform.dense.weight", (h, h), std)
        self.mlm_b = store.new("cls.predictions.transform.dense.bias", (h,), init_const(0), decay=False, lowp=False)
        self.mlm_ln_g = store.new("cls.predictions.transform.LayerNorm.weight", (h,), init_const(1), decay=False,
                                  lowp=False)
        self.mlm_ln_b = store.new("cls.predictions.transform.LayerNorm.bias", (h,), init_const(0), decay=False,
                                  lowp=False)
        self.dec_b = store.new("cls.predictions.bias", (c.padded_vocab,), init_const(0), decay=False, lowp=False)
        self.nsp_w = store.new("cls.seq_relationship.weight", (64, h), std)  # 2 classes, padded to 64 rows
        self.nsp_b = store.new("cls.seq_relationship.bias", (64,), init_const(0), decay=False, lowp=False)

    def finalize(self, device, **kw):
        self.store.finalize(device, **kw)
        return self.to(device)

    def forward(self, input_ids, token_type_ids, mlm_labels, nsp_labels, mlm_positions=None, kv_lens=None,
                dtype=torch.bfloat16):
        """``mlm_positions`` [B, P] (with ``mlm_labels`` [B, P], -100 on unused slots) runs the MLM head on those rows
        only, as BERT pretraining does (the head's gradient is zero on every unlabelled row, so loss and gradients
        equal the every-token head's); without it ``mlm_labels`` is dense [B, S]."""
        B, S = input_ids.shape
        c = self.c
        h = c.hidden
        # word + position + token-type lookups summed in one gather pass (scatter-add backward)
        e = K.embedding_sum([(input_ids, self.word), (None, self.pos), (token_type_ids, self.typ)], S, dtype)
        x = K.layer_norm(e.reshape(B * S, h), self.emb_ln_g, self.emb_ln_b, c.eps)
        for layer in self.layers:
            x = layer(x, B, S, kv_lens)
        if mlm_positions is not None:
            rows = (mlm_positions + torch.arange(B, device=x.device).unsqueeze(1) * S).reshape(-1)
            xm = x.index_select(0, rows)  # [B * P, h]; backward scatters into the encoder output gradient
        else:
            xm = x  # MLM head on every token (labels -100 are ignored by the loss kernel)
        t = K.linear(xm, self.mlm_w, self.mlm_b, act="gelu")
        t = K.layer_norm(t, self.mlm_ln_g, self.mlm_ln_b, c.eps)
        logits = K.linear(t, self.word, self.dec_b)  # tied decoder, [T, padded_vocab]
        mlm = K.cross_entropy(logits, mlm_labels.reshape(-1), valid=c.vocab_size)
        # NSP head on [CLS]
        cls = x.reshape(B, S, h)[:, 0].contiguous()
        pooled = torch.tanh(K.linear(cls, self.pool_w, self.pool_b).float()).to(dtype)
        nsp_logits = K.linear(pooled, self.nsp_w, self.nsp_b)
        nsp = K.cross_entropy(nsp_logits, nsp_labels, valid=2)
        return mlm + nsp, mlm, nsp


def synthetic_batch(c: BertConfig, batch: int, seq: int, device, generator=None, mask_prob=0.15):
    """Random pretraining batch. With ``c.max_predictions`` it has the original data format: per sequence
    min(max_predictions, max(1, round(seq * mask_prob))) masked positions (sorted, never [CLS] at 0), padded to
    max_predictions slots with position 0 / label -100; returns (ids, token_types, labels [B, P], nsp, positions).
    Otherwise a Bernoulli mask with dense labels [B, S]; returns (ids, token_types, labels, nsp)."""
    g = generator
    ids = torch.randint(0, c.vocab_size, (batch, seq), device=device, generator=g)
    tt = torch.zeros(batch, seq, dtype=torch.long, device=device)
    tt[:, seq // 2:] = 1
    nsp = torch.randint(0, 2, (batch,), device=device, generator=g)
    if c.max_predictions:
        P = c.max_predictions
        n = min(P, max(1, int(round(seq * mask_prob))), seq - 1)
        pick = torch.rand(batch, seq - 1, device=device, generator=g).argsort(dim=1)[:, :n] + 1
        pos = torch.zeros(batch, P, dtype=torch.long, device=device)
        pos[:, :n] = pick.sort(dim=1).values
        labels = torch.full((batch, P), -100, dtype=torch.long, device=device)
        labels[:, :n] = ids.gather(1, pos[:, :n])
        return ids, tt, labels, nsp, pos
    sel = torch.rand(batch, seq, device=device, generator=g) < mask_prob
    labels = torch.where(sel, ids, torch.full_like(ids, -100))
    return ids, tt, labels, nsp


def dense_mlm_labels(labels, positions, seq: int):
    """[B, P] slot labels at ``positions`` -> dense [B, S] labels (-100 elsewhere), for every-token references."""
    B = labels.shape[0]
    out = torch.full((B, seq), -100, dtype=labels.dtype, device=labels.device)
    keep = labels != -100
    out[torch.arange(B, device=labels.device).unsqueeze(1).expand_as(labels)[keep], positions[keep]] = labels[keep]
    return out
