"""End-to-end numerics: a tiny BERT trained on the GPU with the production stack — amp O2
(bf16 model, fp32 masters, dynamic loss scale), FusedLAMB, FusedLayerNorm, the MFMA flash
attention and fused GEMM epilogues — tracks the same model trained in pure fp32 PyTorch on
the CPU (reference formulations of every op, the reference LAMB in
apex.multi_tensor_apply.ops.lamb_reference) from the same initial weights and batches.

Dropout is off (the two sides have different RNGs). Reference style: the output-dtype and
value checks of /root/reference/tests/run_amp/test_basic_casts.py:14-21, extended to a whole
training trajectory.
"""
import copy

import pytest
import torch


@pytest.mark.gpu
def test_tiny_bert_o2_lamb_tracks_fp32_reference():
    from apex import amp
    from apex.amp._amp_state import _amp_state
    from apex.models.bert import BertConfig, BertForPreTraining, param_groups_for_lamb, synthetic_batch
    from apex.optimizers import FusedLAMB

    torch.manual_seed(0)
    cfg = BertConfig.tiny()
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    ref = BertForPreTraining(cfg)  # CPU fp32
    gpu = copy.deepcopy(ref).cuda()
    init = {n: p.detach().clone() for n, p in ref.named_parameters()}
    g = torch.Generator().manual_seed(1)
    batches = [synthetic_batch(cfg, 8, 64, generator=g) for _ in range(3)]

    # fp32 CPU reference (FusedLAMB's reference path on CPU tensors)
    _amp_state.optimizers, _amp_state.loss_scalers = [], []
    ropt = FusedLAMB(param_groups_for_lamb(ref, 0.01), lr=2e-3, max_grad_norm=1.0)
    ref_losses = []
    for i in range(6):
        loss = ref(**batches[i % 3])
        loss.backward()
        ropt.step()
        ropt.zero_grad()
        ref_losses.append(float(loss))

    _amp_state.optimizers, _amp_state.loss_scalers = [], []
    opt = FusedLAMB(param_groups_for_lamb(gpu, 0.01), lr=2e-3, max_grad_norm=1.0)
    gpu, opt = amp.initialize(gpu, opt, opt_level="O2", cast_model_type=torch.bfloat16, verbosity=0)
    assert next(gpu.parameters()).dtype == torch.bfloat16
    losses = []
    for i in range(6):
        b = {k: v.cuda() for k, v in batches[i % 3].items()}
        loss = gpu(**b)
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss.float()))
    # loss trajectory: bf16 activations, fp32 statistics -> within 2 %
    for a, r in zip(losses, ref_losses):
        assert abs(a - r) <= 0.02 * abs(r), (losses, ref_losses)
    assert losses[-1] < losses[0] and ref_losses[-1] < ref_losses[0]
    # parameter deltas (fp32 masters vs fp32 reference): same direction and size per tensor
    masters = [p for grp in opt.param_groups for p in grp["params"]]
    ref_params = [p for grp in ropt.param_groups for p in grp["params"]]
    assert len(masters) == len(ref_params)
    name_of = {id(p): n for n, p in ref.named_parameters()}
    checked = 0
    for m, r in zip(masters, ref_params):
        n = name_of[id(r)]
        d_ref = (r.detach() - init[n]).flatten()
        d_gpu = (m.detach().cpu().float() - init[n]).flatten()
        if d_ref.norm() < 1e-6:
            continue
        cos = torch.nn.functional.cosine_similarity(d_ref, d_gpu, dim=0)
        ratio = d_gpu.norm() / d_ref.norm()
        assert cos > 0.97 and 0.9 < ratio < 1.1, (n, float(cos), float(ratio))
        checked += 1
    assert checked >= len(ref_params) // 2
