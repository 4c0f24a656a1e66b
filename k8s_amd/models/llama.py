"""Llama-3 decoder (8B and small test configs) on the k8s_amd op set.

BASELINE config 4: "Llama-3 8B TfJob 8 WORKER ring all-reduce (no PS), bf16,
CDNA4 MFMA GEMM path". Architecture = Llama-3-8B: vocab 128256, hidden 4096,
32 layers, 32 query heads / 8 KV heads (GQA), head dim 128, SwiGLU FFN 14336,
RMSNorm eps 1e-5, RoPE theta 500000, untied embeddings (8.03 B parameters).

MI355X sizing: bf16 weights 16 GB + fp32 master 32 GB + fp32
grads 32 GB + Adam 64 GB fit one 288 GB GPU with room for activations, so the
8-GPU config is pure data parallel with a ring all-reduce of the flat gradient
buffer (``parallel/ddp.py``) -- no tensor/pipeline parallelism needed.

Per layer: RMSNorm (fused residual add) -> fused QKV GEMM [T, 6144] with RoPE on
q/k in its epilogue -> causal GQA flash attention -> O GEMM -> RMSNorm (+residual) -> fused
gate|up GEMM [T, 28672] -> SwiGLU -> down GEMM.
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
class LlamaConfig:
    vocab_size: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    intermediate: int = 14336
    max_position: int = 8192
    rope_theta: float = 500000.0
    eps: float = 1e-5
    init_std: float = 0.02

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


LLAMA3_8B = LlamaConfig()
LLAMA_TINY = LlamaConfig(vocab_size=512, hidden=256, layers=2, heads=4, kv_heads=2, intermediate=512,
                         max_position=256)
# a ~1B-parameter shape for quick single-GPU checks of the same kernels
LLAMA_1B = LlamaConfig(vocab_size=128256, hidden=2048, layers=16, heads=32, kv_heads=8, intermediate=8192)


class LlamaLayer(nn.Module):
    def __init__(self, store: ParamStore, name: str, c: LlamaConfig):
        super().__init__()
        self.c = c
        h, d = c.hidden, c.head_dim
        std = init_normal(c.init_std)
        out_std = init_normal(c.init_std / math.sqrt(2 * c.layers))
        self.attn_norm = store.new(name + ".input_layernorm.weight", (h,), init_const(1), decay=False, lowp=False)
        self.qkv = store.new(name + ".self_attn.qkv_proj.weight", ((c.heads + 2 * c.kv_heads) * d, h), std)
        self.o = store.new(name + ".self_attn.o_proj.weight", (h, c.heads * d), out_std)
        self.mlp_norm = store.new(name + ".post_attention_layernorm.weight", (h,), init_const(1), decay=False,
                                  lowp=False)
        # rows: blocks of 64 gate rows then the matching 64 up rows (ops.nn.linear_swiglu), so every wave tile of the
        # gate|up GEMM holds matching gate / up columns and its epilogue applies the SwiGLU; halves if F % 64 != 0
        self.gate_up = store.new(name + ".mlp.gate_up_proj.weight", (2 * c.intermediate, h), std)
        self.swiglu_blk = 64 if c.intermediate % 64 == 0 else 0
        self.down = store.new(name + ".mlp.down_proj.weight", (h, c.intermediate), out_std)

    def forward(self, x, res, B, S, pos, table):
        """x: this layer's input stream delta, res: running residual (None for the first layer).
        Returns (delta, residual) so every residual add is fused into the next RMSNorm."""
        c = self.c
        d = c.head_dim
        if res is None:
            res = x
            hn = K.rms_norm(x, self.attn_norm, c.eps)
        else:
            hn, res = K.rms_norm(x, self.attn_norm, c.eps, residual=res)
        # the q / k rotary embedding in the QKV GEMM's epilogue where the kernel takes the shape (else in place below)
        qkv, rotated = K.linear_rope(hn, self.qkv, pos, table, (c.heads + c.kv_heads) * d)
        # causal GQA flash attention and the packed QKV gradient in one op (no split/cat/copies)
        o = attention_qkv(qkv, B, S, c.heads, c.kv_heads, d, causal=True, rope=(pos, table),
                          rope_in_place=True,  # qkv: this linear's output, read by nothing else
                          rope_applied=rotated)
        a = K.linear(o.reshape(B * S, c.heads * d), self.o)
        hn, res = K.rms_norm(a, self.mlp_norm, c.eps, residual=res)
        sl = K.SwiGLULink(self.swiglu_blk)  # the SwiGLU backward inside the down projection's data gradient
        # gate|up projection + SwiGLU: one GEMM with the SwiGLU in its epilogue where the kernel takes the shape
        f = K.linear(K.linear_swiglu(hn, self.gate_up, link=sl, blk=self.swiglu_blk), self.down, swiglu_in=sl)
        return f, res


class LlamaForCausalLM(nn.Module):
    def __init__(self, store: ParamStore, c: LlamaConfig = LLAMA3_8B):
        super().__init__()
        self.store, self.c = store, c
        std = init_normal(c.init_std)
        self.embed = store.new("model.embed_tokens.weight", (c.vocab_size, c.hidden), std)
        self.layers = nn.ModuleList([LlamaLayer(store, "model.layers.%d" % i, c) for i in range(c.layers)])
        self.norm = store.new("model.norm.weight", (c.hidden,), init_const(1), decay=False, lowp=False)
        self.lm_head = store.new("lm_head.weight", (c.vocab_size, c.hidden), std)
        self.table = None

    def finalize(self, device, **kw):
        self.store.finalize(device, **kw)
        self.table = K.rope_table(self.c.max_position, self.c.head_dim, self.c.rope_theta, device)
        return self.to(device)

    def forward(self, input_ids, labels, dtype=torch.bfloat16):
        B, S = input_ids.shape
        c = self.c
        pos = torch.arange(S, device=input_ids.device, dtype=torch.int32).repeat(B)
        x = K.embedding_sum([(input_ids, self.embed)], S, dtype).reshape(B * S, c.hidden)
        res = None
        for layer in self.layers:
            x, res = layer(x, res, B, S, pos, self.table)
        hn, _ = K.rms_norm(x, self.norm, c.eps, residual=res)
        logits = K.linear(hn, self.lm_head)
        return K.cross_entropy(logits, labels.reshape(-1))


def synthetic_batch(c: LlamaConfig, batch: int, seq: int, device, generator=None):
    ids = torch.randint(0, c.vocab_size, (batch, seq + 1), device=device, generator=generator)
    return ids[:, :-1].contiguous(), ids[:, 1:].contiguous()
