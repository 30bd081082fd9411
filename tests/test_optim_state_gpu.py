"""Optimizer step accounting and checkpoints on the GPU:

* FusedAdam keeps its step count on the device and advances it only when the loss scaler did
  not skip the step: an overflow-skipped step must not enter the bias corrections;
* FusedSGD's first-run momentum init (buf = g) is not used up by a skipped first step;
* FusedLAMB state_dict: no scratch buffers, and save -> torch.load(map_location="cpu",
  weights_only=True) -> load -> step continues exactly like the uninterrupted optimizer;
* dropout keys come from the device generator: different under different TP-tracker states,
  identical when the state is replayed.
"""
import io

import pytest
import torch


def _params(seed=0, n=3):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.randn(37 + 11 * i, 5, device="cuda", generator=g) for i in range(n)]


def _grads(step, shapes):
    g = torch.Generator(device="cuda").manual_seed(100 + step)
    return [torch.randn(*s, device="cuda", generator=g) for s in shapes]


@pytest.mark.gpu
def test_fused_adam_skipped_step_not_counted():
    from apex.optimizers import FusedAdam

    init = _params()
    ps = [torch.nn.Parameter(t.clone()) for t in init]
    rs = [torch.nn.Parameter(t.clone()) for t in init]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=0.01, adam_w_mode=True)
    ref = torch.optim.AdamW(rs, lr=1e-2, weight_decay=0.01, eps=1e-8)
    noop = torch.zeros(1, dtype=torch.int32, device="cuda")
    opt._amp_noop = noop
    shapes = [p.shape for p in ps]
    for step, skip in enumerate([False, True, False, False]):
        gs = _grads(step, shapes)
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        noop.fill_(1 if skip else 0)
        opt.step()
        if not skip:
            for r, g in zip(rs, gs):
                r.grad = g.clone()
            ref.step()
    for p, r in zip(ps, rs):
        torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-5, atol=1e-6)
    assert opt.state_dict()["param_groups"][0]["step"] == 3


@pytest.mark.gpu
def test_fused_sgd_skipped_first_step_keeps_first_run():
    from apex.optimizers import FusedSGD

    init = _params(1)
    ps = [torch.nn.Parameter(t.clone()) for t in init]
    rs = [torch.nn.Parameter(t.clone()) for t in init]
    opt = FusedSGD(ps, lr=0.1, momentum=0.9, dampening=0.5)
    ref = torch.optim.SGD(rs, lr=0.1, momentum=0.9, dampening=0.5)
    noop = torch.zeros(1, dtype=torch.int32, device="cuda")
    opt._amp_noop = noop
    shapes = [p.shape for p in ps]
    for step, skip in enumerate([True, False, False]):
        gs = _grads(step, shapes)
        for p, g in zip(ps, gs):
            p.grad = g.clone()
        noop.fill_(1 if skip else 0)
        opt.step()
        if not skip:
            for r, g in zip(rs, gs):
                r.grad = g.clone()
            ref.step()
    for p, r in zip(ps, rs):
        torch.testing.assert_close(p.detach(), r.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_fused_lamb_state_dict_roundtrip_cpu_map_location():
    from apex.optimizers import FusedLAMB

    init = _params(2)
    a = [torch.nn.Parameter(t.clone()) for t in init]
    opt = FusedLAMB(a, lr=1e-2, weight_decay=0.01)
    shapes = [p.shape for p in a]
    for step in range(2):
        for p, g in zip(a, _grads(step, shapes)):
            p.grad = g.clone()
        opt.step()
    sd = opt.state_dict()
    # only per-parameter moments are serialised (no fp32 update scratch, no device step tensors)
    assert all(isinstance(k, int) for k in sd["state"]), list(sd["state"])[:5]
    assert all(set(v) == {"exp_avg", "exp_avg_sq"} for v in sd["state"].values())
    assert sd["param_groups"][0]["step"] == 2
    buf = io.BytesIO()
    torch.save(sd, buf)
    buf.seek(0)
    loaded = torch.load(buf, map_location="cpu", weights_only=True)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    opt2 = FusedLAMB(b, lr=1e-2, weight_decay=0.01)
    opt2.load_state_dict(loaded)
    for step in range(2, 4):
        gs = _grads(step, shapes)
        for p, q, g in zip(a, b, gs):
            p.grad = g.clone()
            q.grad = g.clone()
        opt.step()
        opt2.step()
    for p, q in zip(a, b):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=0, atol=0)
    assert opt2.state_dict()["param_groups"][0]["step"] == 4


@pytest.mark.gpu
def test_dropout_keys_follow_device_generator_and_tp_tracker():
    from apex.transformer.tensor_parallel.random import CudaRNGStatesTracker
    from apex.utils.rng import philox_seed_offset

    dev = torch.device("cuda", 0)
    torch.cuda.manual_seed(7)
    k1 = philox_seed_offset(dev)
    k2 = philox_seed_offset(dev)
    assert k1 != k2  # successive launches never share a Philox stream
    torch.cuda.manual_seed(7)
    assert philox_seed_offset(dev) == k1  # reproducible under manual_seed
    # two "TP ranks": tracker states seeded seed+2718+rank
    keys = []
    for rank in range(2):
        tr = CudaRNGStatesTracker()
        tr.add("model-parallel-rng", 1234 + 2718 + rank)
        with tr.fork():
            keys.append(philox_seed_offset(dev))
    assert keys[0] != keys[1]
    # and the same tracker state replays the same key (activation-checkpoint recompute)
    tr = CudaRNGStatesTracker()
    tr.add("model-parallel-rng", 1234 + 2718)
    with tr.fork():
        assert philox_seed_offset(dev) == keys[0]


@pytest.mark.gpu
def test_attention_dropout_masks_differ_across_tp_states():
    from apex.contrib.multihead_attn.flash import flash_attention_packed
    from apex.transformer.tensor_parallel.random import CudaRNGStatesTracker

    torch.manual_seed(0)
    qkv = torch.randn(2, 128, 3, 4, 64, device="cuda", dtype=torch.bfloat16)
    outs = []
    for rank in (0, 1, 0):
        tr = CudaRNGStatesTracker()
        tr.add("model-parallel-rng", 99 + rank)
        with tr.fork():
            outs.append(flash_attention_packed(qkv, 0.3, causal=True))
    assert not torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])
