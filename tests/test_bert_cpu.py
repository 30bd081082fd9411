"""CPU plumbing: tiny BERT fwd/bwd + FusedLAMB reference path + amp O0 (config 1-style)."""
import torch

from apex import amp
from apex.models.bert import BertConfig, BertForPreTraining, param_groups_for_lamb, synthetic_batch
from apex.optimizers import FusedLAMB


def test_tiny_bert_trains_on_cpu():
    torch.manual_seed(0)
    cfg = BertConfig.tiny()
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    model = BertForPreTraining(cfg)
    opt = FusedLAMB(param_groups_for_lamb(model), lr=5e-3)
    model, opt = amp.initialize(model, opt, opt_level="O0", verbosity=0)
    batch = synthetic_batch(cfg, 4, 32)
    losses = []
    for _ in range(6):
        loss = model(**batch)
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0]
