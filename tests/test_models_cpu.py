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
    # bert-base-uncased pretraining = 110,106,428 (+ the padded vocab rows / logits -- 198 at 256-column padding --
    # + 62 padded NSP rows)
    n = s.num_parameters()
    pv = bert.BERT_BASE.padded_vocab - bert.BERT_BASE.vocab_size
    assert bert.BERT_BASE.padded_vocab % 256 == 0 and 0 <= pv < 256
    pad = pv * 768 + pv + 62 * 768 + 62
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


def test_bert_gathered_mlm_head_matches_every_token_head():
    """The MLM head on the masked-position slots (pretraining data format) gives the loss and flat gradient of the
    head on every token with the equivalent dense labels."""
    import dataclasses

    torch.manual_seed(0)
    res = []
    g = torch.Generator().manual_seed(3)
    batch = bert.synthetic_batch(bert.BERT_TINY, 3, 32, "cpu", generator=g, mask_prob=0.2)
    ids, tt, labels, nsp, pos = batch
    assert labels.shape == (3, 12) and (labels[:, :6] != -100).all() and (labels[:, 6:] == -100).all()
    assert (pos[:, :6] > 0).all() and (pos[:, :6].diff(dim=1) > 0).all()
    dense = bert.dense_mlm_labels(labels, pos, 32)
    assert int((dense != -100).sum()) == 18
    for gathered in (True, False):
        cfg = bert.BERT_TINY if gathered else dataclasses.replace(bert.BERT_TINY, max_predictions=0)
        s = ParamStore()
        m = bert.BertForPreTraining(s, cfg).finalize("cpu", seed=5)
        s.begin_step()
        loss = m(ids, tt, labels if gathered else dense, nsp, pos if gathered else None, dtype=torch.float32)[0]
        loss.backward()
        s.zero_unwritten()
        res.append((loss.item(), s.grad.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-5
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-4, atol=1e-6)
