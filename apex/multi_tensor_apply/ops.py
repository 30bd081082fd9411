"""amp_C-compatible multi-tensor ops.

Each op has the signature ``op(chunk_size, noop_flag, tensor_lists, *args)`` used
by ``multi_tensor_applier``. Device tensors run the fused HIP kernels
(csrc/multi_tensor.hip) through a cached MTPlan; CPU tensors run the PyTorch
reference below, which is also the fp32 numerics reference for the tests.
``noop_flag`` is an int32 device tensor: kernels set it to 1 on inf/nan
(scale/axpby/l2norm) and optimizers skip the update while it is non-zero.
"""
from __future__ import annotations

import math

import torch

from .. import _ext
from . import get_plan


def _noop_set(noop, bad: bool):
    if noop is not None and bad:
        noop.fill_(1)


def _nonfinite(t: torch.Tensor) -> bool:
    return not bool(torch.isfinite(t).all())


# ----------------------------------------------------------------------------
def multi_tensor_scale(chunk_size, noop, tensor_lists, scale):
    """out = in * scale ; noop |= any non-finite input."""
    ins, outs = tensor_lists[0], tensor_lists[1]
    if not ins:
        return
    if _ext.use_native(ins[0]):
        plan = get_plan([ins, outs], chunk_size)
        if isinstance(scale, torch.Tensor):
            plan.scale(scale, 1.0, noop)
        else:
            plan.scale(None, float(scale), noop)
        return
    s = float(scale) if not isinstance(scale, torch.Tensor) else float(scale.item())
    bad = False
    for i, o in zip(ins, outs):
        bad |= _nonfinite(i)
        o.copy_(i.float() * s)
    _noop_set(noop, bad)


def multi_tensor_axpby(chunk_size, noop, tensor_lists, a, b, arg_to_check):
    xs, ys, outs = tensor_lists
    if not xs:
        return
    if _ext.use_native(xs[0]):
        get_plan([xs, ys, outs], chunk_size).axpby(float(a), float(b), int(arg_to_check), noop)
        return
    bad = False
    for x, y, o in zip(xs, ys, outs):
        if arg_to_check in (-1, 0):
            bad |= _nonfinite(x)
        if arg_to_check in (-1, 1):
            bad |= _nonfinite(y)
        o.copy_(a * x.float() + b * y.float())
    _noop_set(noop, bad)


def multi_tensor_l2norm(chunk_size, noop, tensor_lists, per_tensor=False):
    """Returns (global_norm[1], per_tensor_norms[T] or empty)."""
    xs = tensor_lists[0]
    if not xs:
        z = torch.zeros(1)
        return z, torch.zeros(0)
    if _ext.use_native(xs[0]):
        g, p = get_plan([xs], chunk_size).l2norm(0, bool(per_tensor), None, 1.0, noop)
        return g, p
    norms = torch.stack([x.float().norm() for x in xs])
    bad = any(_nonfinite(x) for x in xs)
    _noop_set(noop, bad)
    tot = norms.pow(2).sum().sqrt().reshape(1)
    return tot, (norms if per_tensor else torch.zeros(0))


def multi_tensor_sgd(chunk_size, noop, tensor_lists, wd, momentum, dampening, lr, nesterov,
                     first_run, wd_after_momentum, scale=1.0):
    gs, ps, moms = tensor_lists[0], tensor_lists[1], tensor_lists[2]
    copies = tensor_lists[3] if len(tensor_lists) > 3 else None
    if not gs:
        return
    if _ext.use_native(gs[0]):
        lists = [gs, ps, moms] + ([copies] if copies is not None else [])
        st = scale if isinstance(scale, torch.Tensor) else None
        get_plan(lists, chunk_size).sgd(float(lr), float(momentum), float(dampening), float(wd),
                                        bool(nesterov), bool(first_run), bool(wd_after_momentum),
                                        1.0 if st is not None else float(scale), st, noop, None)
        return
    if noop is not None and int(noop.item()) != 0:
        return
    s = float(scale.item()) if isinstance(scale, torch.Tensor) else float(scale)
    for i, (g, p, m) in enumerate(zip(gs, ps, moms)):
        gg = g.float() * s
        pf = p.float()
        if wd != 0 and not wd_after_momentum:
            gg = gg + wd * pf
        if momentum != 0:
            if first_run:
                m.copy_(gg)
            else:
                m.mul_(momentum).add_(gg, alpha=1 - dampening)
            gg = gg + momentum * m if nesterov else m.clone()
        if wd != 0 and wd_after_momentum:
            gg = gg + wd * pf
        pf = pf - lr * gg
        p.copy_(pf)
        if copies is not None:
            copies[i].copy_(pf)


ADAM_MODE_L2 = 0
ADAM_MODE_ADAMW = 1


def multi_tensor_adam(chunk_size, noop, tensor_lists, lr, beta1, beta2, eps, step, mode,
                      bias_correction, weight_decay, grad_scale=1.0):
    gs, ps, ms, vs = tensor_lists[:4]
    copies = tensor_lists[4] if len(tensor_lists) > 4 else None
    if not gs:
        return
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    if _ext.use_native(gs[0]):
        lists = [gs, ps, ms, vs] + ([copies] if copies is not None else [])
        st = grad_scale if isinstance(grad_scale, torch.Tensor) else None
        get_plan(lists, chunk_size).adam(float(lr), float(beta1), float(beta2), float(eps),
                                         float(weight_decay), bc1, bc2, int(mode) == ADAM_MODE_ADAMW,
                                         1.0 if st is not None else float(grad_scale), st, noop, None,
                                         bool(bias_correction))
        return
    if noop is not None and int(noop.item()) != 0:
        return
    s = float(grad_scale.item()) if isinstance(grad_scale, torch.Tensor) else float(grad_scale)
    for i, (g, p, m, v) in enumerate(zip(gs, ps, ms, vs)):
        gg = g.float() * s
        pf = p.float()
        if mode == ADAM_MODE_L2 and weight_decay != 0:
            gg = gg + weight_decay * pf
        m.mul_(beta1).add_(gg, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
        upd = (m / bc1) / ((v / bc2).sqrt() + eps)
        if mode == ADAM_MODE_ADAMW and weight_decay != 0:
            upd = upd + weight_decay * pf
        pf = pf - lr * upd
        p.copy_(pf)
        if copies is not None:
            copies[i].copy_(pf)


def lamb_reference(gs, ps, ms, vs, lr, beta1, beta2, eps, step, bias_correction, weight_decay,
                   grad_averaging, mode, global_grad_norm, max_grad_norm, use_nvlamb=False,
                   grad_scale=1.0, copies=None):
    """PyTorch fp32 reference of the fused LAMB update (apex FusedLAMB semantics)."""
    gn = float(global_grad_norm)
    clip = gn / max_grad_norm if (max_grad_norm > 0 and gn > max_grad_norm) else 1.0
    bc1 = 1 - beta1 ** step if bias_correction else 1.0
    bc2 = 1 - beta2 ** step if bias_correction else 1.0
    b3 = 1 - beta1 if grad_averaging else 1.0
    for i, (g, p, m, v) in enumerate(zip(gs, ps, ms, vs)):
        gg = g.float() * grad_scale / clip
        pf = p.float()
        if mode == ADAM_MODE_L2 and weight_decay != 0:
            gg = gg + weight_decay * pf
        m.mul_(beta1).add_(gg, alpha=b3)
        v.mul_(beta2).addcmul_(gg, gg, value=1 - beta2)
        u = (m / bc1) / ((v / bc2).sqrt() + eps)
        if mode == ADAM_MODE_ADAMW and weight_decay != 0:
            u = u + weight_decay * pf
        ratio = lr
        if use_nvlamb or weight_decay != 0:
            pn, un = float(pf.norm()), float(u.norm())
            if pn != 0 and un != 0:
                ratio = lr * pn / un
        pf = pf - ratio * u
        p.copy_(pf)
        if copies is not None:
            copies[i].copy_(pf)


def multi_tensor_lamb(chunk_size, noop, tensor_lists, lr, beta1, beta2, eps, step,
                      bias_correction, weight_decay, grad_averaging, mode, global_grad_norm,
                      max_grad_norm, use_nvlamb=False):
    """amp_C.multi_tensor_lamb-compatible entry (host-side ``step``).

    The fused kernel keeps its own device step counter; for this compat entry it is
    seeded with ``step - 1`` so bias correction matches the caller's step.
    """
    gs, ps, ms, vs = tensor_lists[:4]
    if not gs:
        return
    if _ext.use_native(gs[0]):
        lists = [gs, ps, ms, vs] + ([tensor_lists[4]] if len(tensor_lists) > 4 else [])
        stp = torch.full((1,), int(step) - 1, dtype=torch.int32, device=gs[0].device)
        gn = global_grad_norm if isinstance(global_grad_norm, torch.Tensor) else \
            torch.full((1,), float(global_grad_norm), device=gs[0].device)
        get_plan(lists, chunk_size).lamb(float(lr), float(beta1), float(beta2), float(eps),
                                         float(weight_decay), float(max_grad_norm),
                                         int(mode) == ADAM_MODE_ADAMW, bool(bias_correction),
                                         bool(grad_averaging), bool(use_nvlamb), 1.0, None, noop,
                                         None, stp, gn.float().reshape(1))
        return
    if noop is not None and int(noop.item()) != 0:
        return
    gn = float(global_grad_norm.item()) if isinstance(global_grad_norm, torch.Tensor) else \
        float(global_grad_norm)
    lamb_reference(gs, ps, ms, vs, lr, beta1, beta2, eps, step, bias_correction, weight_decay,
                   grad_averaging, mode, gn, max_grad_norm, use_nvlamb,
                   copies=tensor_lists[4] if len(tensor_lists) > 4 else None)


def update_scale_(scale, growth_tracker, found_inf, growth_factor, backoff_factor,
                  growth_interval, min_scale=0.0, max_scale=float("inf")):
    """Device-side dynamic loss-scale update (no host sync)."""
    if _ext.use_native(scale):
        _ext.require().update_scale(scale, growth_tracker, found_inf, float(growth_factor),
                                    float(backoff_factor), int(growth_interval), float(min_scale),
                                    float(max_scale) if math.isfinite(max_scale) else 3.4e38)
        return
    if int(found_inf.item()):
        scale.mul_(backoff_factor).clamp_(min=min_scale)
        growth_tracker.zero_()
    else:
        growth_tracker.add_(1)
        if int(growth_tracker.item()) >= growth_interval:
            scale.mul_(growth_factor).clamp_(max=max_scale)
            growth_tracker.zero_()
