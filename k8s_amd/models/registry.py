"""Model registry: name -> (model on a flat ParamStore, synthetic batch, loss).

Every workload the trainer (``python -m k8s_amd.trainer``) and the benches
can run, at the exact BASELINE.json shapes plus small variants for CPU tests.
Data is synthetic (random images / token ids of the named shape): the
reference's workloads are external TF programs and there is no dataset access.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, Optional, Tuple

import torch

from k8s_amd.ops import nn as K
from k8s_amd.parallel.flat import ParamStore


@dataclass
class Workload:
    name: str
    model: torch.nn.Module
    store: ParamStore
    batch: Callable[[int], Tuple]          # step -> inputs tuple (on device)
    loss: Callable[[Tuple], torch.Tensor]  # inputs -> scalar loss
    units_per_step: int                    # images or tokens per step per rank
    unit: str                              # "images" | "tokens"
    optimizer: str = "sgd"                 # default optimizer family
    lr: float = 0.1
    meta: Dict = field(default_factory=dict)


MODELS = ("resnet50", "resnet_tiny", "bert_base", "bert_tiny", "llama3_8b", "llama_1b", "llama_tiny")
# each model's default optimizer family (Workload.optimizer), known before the model is built
MODEL_OPTIMIZER = {"resnet50": "sgd", "resnet_tiny": "sgd", "bert_base": "adam", "bert_tiny": "adam",
                   "llama3_8b": "adam", "llama_1b": "adam", "llama_tiny": "adam"}


def build(name: str, device, batch: int, seq: Optional[int] = None, image: Optional[int] = None,
          seed: int = 0, grad_dtype=torch.float32, fixed_batch: bool = True, pad_to: int = 64,
          data_seed: Optional[int] = None, mlm_every_token: bool = False) -> Workload:
    """Construct ``name`` on ``device`` with per-rank ``batch``. ``fixed_batch`` reuses one synthetic batch
    (what a throughput benchmark wants); otherwise every step draws a new one."""
    device = torch.device(device)
    dtype = torch.bfloat16 if device.type == "cuda" else torch.float32
    store = ParamStore()
    gen = torch.Generator(device=device)
    gen.manual_seed(1000 + (seed if data_seed is None else data_seed))

    def cached(make):
        box = {}

        def get(step):
            if fixed_batch:
                if "b" not in box:
                    box["b"] = make()
                return box["b"]
            return make()

        return get

    if name in ("resnet50", "resnet_tiny"):
        from k8s_amd.models.resnet import resnet50, resnet_tiny

        ncls = 1000 if name == "resnet50" else 10
        image = image or (224 if name == "resnet50" else 32)
        model = (resnet50(store, ncls) if name == "resnet50" else resnet_tiny(store, ncls))
        model = model.finalize(device, grad_dtype=grad_dtype, seed=seed, pad_to=pad_to)

        def make():
            x = torch.randn(batch, image, image, 3, device=device, generator=gen).to(dtype)
            return model.prepare_input(x).contiguous(), torch.randint(0, ncls, (batch,), device=device,
                                                                      generator=gen)

        return Workload(name, model, store, cached(make), lambda b: K.cross_entropy(model(b[0]), b[1]), batch,
                        "images", "sgd", 0.1, {"image": image, "classes": ncls})

    if name in ("bert_base", "bert_tiny"):
        from k8s_amd.models import bert as M

        cfg = M.BERT_BASE if name == "bert_base" else M.BERT_TINY
        if mlm_every_token:  # the MLM head on every token (dense labels), like HF BertForPreTraining
            import dataclasses

            cfg = dataclasses.replace(cfg, max_predictions=0)
        seq = seq or (128 if name == "bert_base" else 32)
        model = M.BertForPreTraining(store, cfg).finalize(device, grad_dtype=grad_dtype, seed=seed, pad_to=pad_to)

        def make():
            return M.synthetic_batch(cfg, batch, seq, device, generator=gen)

        return Workload(name, model, store, cached(make), lambda b: model(*b, dtype=dtype)[0], batch * seq,
                        "tokens", "adam", 1e-4, {"seq": seq})

    if name in ("llama3_8b", "llama_1b", "llama_tiny"):
        from k8s_amd.models import llama as M

        cfg = {"llama3_8b": M.LLAMA3_8B, "llama_1b": M.LLAMA_1B, "llama_tiny": M.LLAMA_TINY}[name]
        seq = seq or (4096 if name != "llama_tiny" else 64)
        model = M.LlamaForCausalLM(store, cfg).finalize(device, grad_dtype=grad_dtype, seed=seed, pad_to=pad_to)

        def make():
            return M.synthetic_batch(cfg, batch, seq, device, generator=gen)

        return Workload(name, model, store, cached(make), lambda b: model(*b, dtype=dtype), batch * seq, "tokens",
                        "adam", 3e-4, {"seq": seq})

    raise ValueError("unknown model %r (choose from %s)" % (name, ", ".join(MODELS)))
