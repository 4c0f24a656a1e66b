#!/usr/bin/env python3
"""Stock PyTorch-ROCm baselines on the same MI355X (the reference publishes no numbers, so
each row is compared against the stock stack measured with the same harness).

* resnet50  -- torch.nn ResNet-50 v1.5 (no torchvision in the image: a plain definition of the standard
               architecture), channels_last, bf16 autocast, MIOpen convs / BN, torch.optim.SGD(fused)
* bert_base -- transformers BertForPreTraining (random init, SDPA attention), bf16 autocast, AdamW(fused)
* llama_1b / llama3_8b -- transformers LlamaForCausalLM (random init, SDPA), bf16 weights, AdamW(fused)

    python benchmarks/stock_baselines.py --model resnet50 --steps 20 --warmup 5

Prints one JSON line with the same fields as bench.py (value = samples or tokens per second, 1 GPU).
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, w, stride, down):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, w, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(w)
        self.conv2 = nn.Conv2d(w, w, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(w)
        self.conv3 = nn.Conv2d(w, w * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(w * 4)
        self.relu = nn.ReLU(inplace=True)
        self.down = nn.Sequential(nn.Conv2d(cin, w * 4, 1, stride, bias=False), nn.BatchNorm2d(w * 4)) if down else None

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + idt)


class ResNet50(nn.Module):
    def __init__(self, ncls=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for i, n in enumerate((3, 4, 6, 3)):
            w = 64 * 2 ** i
            for j in range(n):
                blocks.append(Bottleneck(cin, w, 2 if (j == 0 and i > 0) else 1, j == 0))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(cin, ncls)

    def forward(self, x):
        y = self.blocks(self.stem(x))
        return self.fc(torch.flatten(nn.functional.adaptive_avg_pool2d(y, 1), 1))


def build(name, batch, seq):
    dev = torch.device("cuda")
    if name == "resnet50":
        m = ResNet50().to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (batch,), device=dev)
        opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5, fused=True)

        def loss():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return nn.functional.cross_entropy(m(x), y)
        return m, opt, loss, batch, "images"
    from transformers import BertConfig, BertForPreTraining, LlamaConfig, LlamaForCausalLM

    if name == "bert_base":
        cfg = BertConfig(attn_implementation="sdpa")
        m = BertForPreTraining(cfg).to(dev)
        ids = torch.randint(0, cfg.vocab_size, (batch, seq), device=dev)
        tt = torch.zeros_like(ids)
        lab = torch.where(torch.rand(batch, seq, device=dev) < 0.15, ids, torch.full_like(ids, -100))
        nsp = torch.randint(0, 2, (batch,), device=dev)
        opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.01, fused=True)

        def loss():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return m(input_ids=ids, token_type_ids=tt, labels=lab, next_sentence_label=nsp).loss
        return m, opt, loss, batch * seq, "tokens"
    if name in ("llama_1b", "llama3_8b"):
        kw = dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                  num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192, rope_theta=500000.0)
        if name == "llama_1b":
            kw.update(hidden_size=2048, intermediate_size=8192, num_hidden_layers=16)
        cfg = LlamaConfig(attn_implementation="sdpa", **kw)
        m = LlamaForCausalLM(cfg).to(dev)
        ids = torch.randint(0, cfg.vocab_size, (batch, seq + 1), device=dev)
        opt = torch.optim.AdamW(m.parameters(), lr=3e-4, weight_decay=0.01, fused=True)

        def loss():
            with torch.autocast("cuda", dtype=torch.bfloat16):
                return m(input_ids=ids[:, :-1], labels=ids[:, 1:]).loss
        return m, opt, loss, batch * seq, "tokens"
    raise ValueError(name)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--seq", type=int, default=None)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--miopen-find-mode", default=None,
                    help="MIOPEN_FIND_MODE for the run (e.g. FAST: heuristic-ranked short Find; NORMAL: full Find)")
    ap.add_argument("--no-find", action="store_true",
                    help="cudnn.benchmark off: MIOpen immediate mode (heuristic solution per shape, no Find search) "
                         "-- the only way a cold box compiles the batch-1024 kernels inside a GPU-call limit")
    a = ap.parse_args(argv)
    if a.miopen_find_mode:
        import os

        os.environ["MIOPEN_FIND_MODE"] = a.miopen_find_mode  # read by MIOpen at its first convolution
    batch = a.batch or {"resnet50": 256, "bert_base": 64, "llama_1b": 2, "llama3_8b": 1}[a.model]
    seq = a.seq or {"bert_base": 128}.get(a.model, 2048)
    torch.backends.cudnn.benchmark = not a.no_find
    m, opt, loss_fn, units, unit = build(a.model, batch, seq)

    def step():
        opt.zero_grad(set_to_none=True)
        loss = loss_fn()
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        step()
        torch.cuda.synchronize()
        print("warmup step %d/%d done" % (i + 1, a.warmup), file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "stock PyTorch-ROCm %s train throughput" % a.model, "value": round(units * a.steps / dt, 2),
                      "unit": "%s/s" % unit, "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
                      "ms_per_step": round(1000 * dt / a.steps, 3), "batch": batch,
                      "seq": seq if unit == "tokens" else None, "final_loss": round(float(loss), 4),
                      "stack": "torch %s (MIOpen / hipBLASLt / SDPA / fused optim)" % torch.__version__,
                      "miopen_find": not a.no_find, "miopen_find_mode": a.miopen_find_mode}), flush=True)


if __name__ == "__main__":
    main()
