"""Model definitions on CPU (fp32 oracle path): parameter counts of the BASELINE shapes and a few training
steps of the tiny variants through the trainer's registry."""
import pytest
import torch

from k8s_amd.models import bert, llama
from k8s_amd.models.registry import build
from k8s_amd.ops.optim import FusedAdam
from k8s_amd.parallel.flat import ParamStore


def test_bert_base_parameter_count():
    s = ParamStore()
    bert.BertForPreTraining(s, bert.BERT_BASE)
    # bert-base-uncased pretraining = 110,106,428 (+ 6 padded vocab rows / logits, + 62 padded NSP rows)
    n = s.num_parameters()
    pad = 6 * 768 + 6 + 62 * 768 + 62
    assert n - pad == 110106428


def test_llama3_8b_parameter_count():
    s = ParamStore()
    llama.LlamaForCausalLM(s, llama.LLAMA3_8B)
    assert s.num_parameters() == 8030261248


@pytest.mark.parametrize("name", ["bert_tiny", "llama_tiny"])
def test_tiny_models_train_on_cpu(name):
    torch.manual_seed(0)
    w = build(name, "cpu", batch=4, seed=0)
    opt = FusedAdam(w.store, lr=3e-3, weight_decay=0.0)
    losses = []
    for step in range(6):
        w.store.begin_step()
        loss = w.loss(w.batch(step))
        loss.backward()
        w.store.zero_unwritten()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0] * 0.9, losses
