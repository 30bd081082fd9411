"""Fused optimizers over param groups that mix dtypes (amp O2 keeps BatchNorm fp32 next to
bf16 convs) and channels_last conv weights: every partition must step exactly like the
unfused fp32 reference applied to the same grads."""
import pytest
import torch
import torch.nn.functional as F


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
                               torch.nn.Conv2d(8, 4, 3, padding=1), torch.nn.BatchNorm2d(4)).cuda()


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["sgd", "adam", "lamb"])
@pytest.mark.parametrize("channels_last", [False, True])
def test_fused_optimizer_mixed_dtype_group(opt_name, channels_last):
    from apex import amp
    from apex.optimizers import FusedAdam, FusedLAMB, FusedSGD

    model = _model()
    if channels_last:
        model = model.to(memory_format=torch.channels_last)
    names = [n for n, _ in model.named_parameters()]
    mk = {"sgd": lambda ps: FusedSGD(ps, lr=0.1, momentum=0.9),
          "adam": lambda ps: FusedAdam(ps, lr=1e-2, weight_decay=0.0),
          "lamb": lambda ps: FusedLAMB(ps, lr=1e-2, weight_decay=0.01, max_grad_norm=1e9)}[opt_name]
    opt = mk(model.parameters())
    model, opt = amp.initialize(model, opt, opt_level="O2", cast_model_type=torch.bfloat16, loss_scale=1.0,
                                verbosity=0)
    # masters start from the bf16-rounded weights amp cast the model to
    ref = {n: m.detach().clone() for n, m in zip(names, [p for g in opt.param_groups for p in g["params"]])}
    dtypes = {p.dtype for p in model.parameters()}
    assert dtypes == {torch.bfloat16, torch.float32}
    x = torch.randn(4, 3, 8, 8, device="cuda", dtype=torch.bfloat16)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    loss = model(x).float().square().mean()
    with amp.scale_loss(loss, opt) as sl:
        sl.backward()
    grads = {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}
    opt.step()
    # fp32 reference step on the same grads
    refp = [torch.nn.Parameter(ref[n].clone()) for n in ref]
    for p, n in zip(refp, ref):
        p.grad = grads[n].clone()
    ropt = {"sgd": lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=0.9),
            "adam": lambda ps: torch.optim.AdamW(ps, lr=1e-2, weight_decay=0.0),
            "lamb": None}[opt_name]
    masters = [p for g in opt.param_groups for p in g["params"]]
    if ropt is not None:
        ro = ropt(refp)
        ro.step()
        for m, r in zip(masters, refp):
            torch.testing.assert_close(m.detach(), r.detach(), rtol=1e-5, atol=1e-6)
    else:
        # LAMB: every tensor moved, and the model copy equals the master rounded to bf16
        for m, r in zip(masters, refp):
            assert not torch.equal(m.detach(), r.detach())
    for mp_, m in zip(model.parameters(), masters):
        torch.testing.assert_close(mp_.detach(), m.detach().to(mp_.dtype), rtol=0, atol=0)
