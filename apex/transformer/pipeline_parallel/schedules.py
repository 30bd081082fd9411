"""Pipeline schedules (NS-08): no pipelining, 1F1B, and interleaved 1F1B.

``forward_step_func(batch, model) -> (output_tensor, loss_func)`` where
``loss_func(output_tensor) -> (loss, logs)`` is applied on the last stage. Models expose
``set_input_tensor(tensor)`` for the activation received from the previous stage.
``batch`` is either a list of microbatches or a tensor / dict / tuple that is split along
dim 0 into ``get_num_microbatches()`` microbatches.

1F1B (PipeDream-flush): stage s runs (pp - s - 1) warm-up forwards, then alternates one
forward / one backward, then drains; at most (pp - s) microbatches of activations are alive
on stage s, which is what lets PP=2 of a large GPT fit alongside TP=4 in 288 GB/GPU with
big microbatches.
"""
from __future__ import annotations

import torch

from .. import parallel_state as ps
from . import p2p_communication as p2p
from .utils import get_num_microbatches


def _split_microbatches(batch, n):
    if isinstance(batch, list):
        assert len(batch) == n, "got {} microbatches, expected {}".format(len(batch), n)
        return batch
    if isinstance(batch, torch.Tensor):
        return list(batch.chunk(n, dim=0))
    if isinstance(batch, dict):
        parts = {k: (v.chunk(n, 0) if isinstance(v, torch.Tensor) else [v] * n) for k, v in batch.items()}
        return [{k: parts[k][i] for k in batch} for i in range(n)]
    if isinstance(batch, tuple):
        parts = [x.chunk(n, 0) if isinstance(x, torch.Tensor) else [x] * n for x in batch]
        return [tuple(p[i] for p in parts) for i in range(n)]
    raise TypeError("unsupported batch type {}".format(type(batch)))


def _unwrap(model):
    return model[0] if isinstance(model, (list, tuple)) else model


def _set_input(model, t):
    m = model
    while not hasattr(m, "set_input_tensor") and hasattr(m, "module"):
        m = m.module
    if hasattr(m, "set_input_tensor"):
        m.set_input_tensor(t)


def forward_step(forward_step_func, batch, model, input_tensor, losses_reduced, num_microbatches,
                 grad_scaler=None):
    _set_input(model, input_tensor)
    output_tensor, loss_func = forward_step_func(batch, model)
    if ps.is_pipeline_last_stage():
        out = loss_func(output_tensor)
        loss, logs = out if isinstance(out, tuple) else (out, {})
        output_tensor = loss / num_microbatches
        losses_reduced.append(logs if logs else {"loss": loss.detach()})
    return output_tensor


def _sync_ctx(model, sync):
    """Gradient all-reduce only in the LAST backward pass of a model chunk: a data-parallel
    wrapper with ``no_sync`` (apex / torch DDP) keeps its hooks off for the earlier microbatches,
    whose gradients just accumulate, and overlaps its bucket all-reduces with the final one."""
    ns = getattr(model, "no_sync", None)
    return ns() if (ns is not None and not sync) else _null()


def backward_step(input_tensor, output_tensor, output_tensor_grad, grad_scaler=None):
    if input_tensor is not None:
        input_tensor.retain_grad()
    if output_tensor_grad is None and grad_scaler is not None:
        output_tensor = grad_scaler(output_tensor)
    if output_tensor_grad is not None and output_tensor_grad.dtype != output_tensor.dtype:
        output_tensor_grad = output_tensor_grad.to(output_tensor.dtype)  # wire dtype -> output dtype
    torch.autograd.backward(output_tensor, grad_tensors=output_tensor_grad)
    return input_tensor.grad if input_tensor is not None else None


def forward_backward_no_pipelining(forward_step_func, batch, model, *, forward_only=False, tensor_shape=None,
                                   dtype=None, grad_scaler=None, disable_autocast=False, **kwargs):
    model = _unwrap(model)
    n = get_num_microbatches()
    mbs = _split_microbatches(batch, n)
    losses = []
    ctx = getattr(model, "no_sync", None)
    for i, mb in enumerate(mbs):
        sync_ctx = ctx() if (ctx is not None and i < n - 1 and not forward_only) else _null()
        with sync_ctx:
            out = forward_step(forward_step_func, mb, model, None, losses, n, grad_scaler)
            if not forward_only:
                backward_step(None, out, None, grad_scaler)
    return losses


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def forward_backward_pipelining_without_interleaving(forward_step_func, batch, model, *, forward_only=False,
                                                     tensor_shape=None, dtype=torch.float32,
                                                     grad_scaler=None, disable_autocast=False, **kwargs):
    """1F1B schedule (non-interleaved)."""
    assert tensor_shape is not None, "tensor_shape is required for pipeline parallelism"
    model = _unwrap(model)
    n = get_num_microbatches()
    mbs = _split_microbatches(batch, n)
    pp = ps.get_pipeline_model_parallel_world_size()
    rank = ps.get_pipeline_model_parallel_rank()
    warmup = min(pp - rank - 1, n) if not forward_only else n
    remaining = n - warmup
    inputs, outputs, losses = [], [], []
    it = iter(mbs)
    done = [0]

    def bwd(i_t, o_t, og):
        done[0] += 1
        with _sync_ctx(model, done[0] == n):
            return backward_step(i_t, o_t, og, grad_scaler)

    for _ in range(warmup):
        inp = p2p.recv_forward(tensor_shape, dtype)
        out = forward_step(forward_step_func, next(it), model, inp, losses, n, grad_scaler)
        p2p.send_forward(out, tensor_shape, dtype)
        if not forward_only:
            inputs.append(inp)
            outputs.append(out)

    inp = p2p.recv_forward(tensor_shape, dtype) if remaining > 0 else None
    for i in range(remaining):
        last = i == remaining - 1
        out = forward_step(forward_step_func, next(it), model, inp, losses, n, grad_scaler)
        if forward_only:
            p2p.send_forward(out, tensor_shape, dtype)
            if not last:
                inp = p2p.recv_forward(tensor_shape, dtype)
            continue
        out_grad = p2p.send_forward_recv_backward(out, tensor_shape, dtype)
        inputs.append(inp)
        outputs.append(out)
        i_t, o_t = inputs.pop(0), outputs.pop(0)
        in_grad = bwd(i_t, o_t, out_grad)
        if last:
            inp = None
            p2p.send_backward(in_grad, tensor_shape, dtype)
        else:
            inp = p2p.send_backward_recv_forward(in_grad, tensor_shape, dtype)

    if not forward_only:
        for _ in range(warmup):
            i_t, o_t = inputs.pop(0), outputs.pop(0)
            out_grad = p2p.recv_backward(tensor_shape, dtype)
            in_grad = bwd(i_t, o_t, out_grad)
            p2p.send_backward(in_grad, tensor_shape, dtype)
    return losses


def _forward_backward_pipelining_with_interleaving(forward_step_func, batch, model, *, forward_only=False,
                                                   tensor_shape=None, dtype=torch.float32, grad_scaler=None,
                                                   disable_autocast=False, **kwargs):
    """Interleaved 1F1B over V = ``len(model)`` model chunks per rank (virtual pipeline stages).

    The model is cut into P*V virtual stages; rank r holds chunks c = 0..V-1, i.e. virtual stages
    c*P + r, so activations flow rank r -> r+1 inside a chunk and from the last rank back to rank
    0 between chunks (the p2p ring). Work on a rank is a sequence of n*V forward units and n*V
    backward units, visited in groups of P microbatches per chunk:

      unit k -> chunk (k mod P*V) // P (backward: mirrored, V-1-that), microbatch (k // (P*V))*P + k mod P

    Rank r runs W = 2(P-r-1) + (V-1)P warm-up forward units (all of them when n == P or
    forward_only), then alternates one forward and one backward unit, then drains the remaining
    backward units. Every step exchanges activations and gradients in ONE grouped p2p call
    (send fwd / send bwd / recv fwd / recv bwd), whose send/recv pairs match on neighbouring
    ranks by construction. Peak live activations per rank are about W + 1 units instead of the
    n*V of an all-forward-then-all-backward (GPipe) order, and the pipeline bubble shrinks by V
    against plain 1F1B. n must be a multiple of P.
    """
    assert isinstance(model, (list, tuple)) and len(model) > 1
    assert tensor_shape is not None
    V = len(model)
    P = ps.get_pipeline_model_parallel_world_size()
    rank = ps.get_pipeline_model_parallel_rank()
    n = get_num_microbatches()
    if n % P != 0:
        raise RuntimeError("interleaved schedule needs the number of microbatches ({}) to be a multiple of "
                           "the pipeline size ({})".format(n, P))
    mbs = _split_microbatches(batch, n)
    total = n * V
    all_warmup = forward_only or n == P
    warmup = total if all_warmup else min((P - rank - 1) * 2 + (V - 1) * P, total)
    remaining = total - warmup
    inputs = [[] for _ in range(V)]
    outputs = [[] for _ in range(V)]
    out_grads = [[] for _ in range(V)]
    losses = []
    stats = {"max_live": 0}

    def chunk_of(k, forward=True):
        c = (k % (P * V)) // P
        return c if forward else V - 1 - c

    def mb_of(k):
        return (k // (P * V)) * P + k % P

    def live():
        return sum(len(o) for o in outputs)

    def fwd_unit(k):
        c = chunk_of(k)
        ps.set_virtual_pipeline_model_parallel_rank(c)
        if ps.is_pipeline_first_stage() and len(inputs[c]) == len(outputs[c]):
            inputs[c].append(None)
        out = forward_step(forward_step_func, mbs[mb_of(k)], model[c], inputs[c][-1], losses, n, grad_scaler)
        outputs[c].append(out)
        stats["max_live"] = max(stats["max_live"], live())
        if forward_only:  # nothing to keep for a backward
            inputs[c].pop()
            outputs[c].pop()
        return out

    bwd_done = [0] * V

    def bwd_unit(k):
        c = chunk_of(k, forward=False)
        ps.set_virtual_pipeline_model_parallel_rank(c)
        if ps.is_pipeline_last_stage() and len(out_grads[c]) == 0:
            out_grads[c].append(None)
        bwd_done[c] += 1
        with _sync_ctx(model[c], bwd_done[c] == n):
            return backward_step(inputs[c].pop(0), outputs[c].pop(0), out_grads[c].pop(0), grad_scaler)

    ps.set_virtual_pipeline_model_parallel_rank(0)
    inputs[0].append(p2p.recv_forward(tensor_shape, dtype))
    for k in range(warmup):
        out = fwd_unit(k)
        nxt = chunk_of(k + 1)
        recv_prev = not (ps.is_pipeline_first_stage(ignore_virtual=True) and nxt == 0) and k != total - 1
        if ps.is_pipeline_last_stage():  # the loss stays here
            out = None
        if k == warmup - 1 and not all_warmup:
            recv_next = not ps.is_pipeline_last_stage(ignore_virtual=True)
            inp, og = p2p.send_forward_backward_recv_forward_backward(out, None, recv_prev, recv_next,
                                                                      tensor_shape, dtype)
            if recv_next:
                out_grads[V - 1].append(og)
        else:
            inp = p2p.send_forward_recv_forward(out, recv_prev, tensor_shape, dtype)
        if recv_prev:
            inputs[nxt].append(inp)

    for i in range(remaining):
        kf, kb = warmup + i, i
        out = fwd_unit(kf)
        ig = bwd_unit(kb)
        ps.set_virtual_pipeline_model_parallel_rank(chunk_of(kf))
        if ps.is_pipeline_last_stage():
            out = None
        ps.set_virtual_pipeline_model_parallel_rank(chunk_of(kb, forward=False))
        if ps.is_pipeline_first_stage():
            ig = None
        # which chunk the next received activation / gradient belongs to
        if ps.is_pipeline_first_stage(ignore_virtual=True):
            nf = chunk_of(kf - (P - 1))
            recv_prev = nf != V - 1
            nf += 1
        else:
            nf, recv_prev = chunk_of(kf + 1), True
        if ps.is_pipeline_last_stage(ignore_virtual=True):
            nb = chunk_of(kb - (P - 1), forward=False)
            recv_next = nb != 0
            nb -= 1
        else:
            nb, recv_next = chunk_of(kb + 1, forward=False), True
        if i == remaining - 1:
            recv_prev = False
        inp, og = p2p.send_forward_backward_recv_forward_backward(out, ig, recv_prev, recv_next, tensor_shape,
                                                                  dtype)
        if recv_prev:
            inputs[nf].append(inp)
        if recv_next:
            out_grads[nb].append(og)

    if not forward_only:
        if all_warmup:
            ps.set_virtual_pipeline_model_parallel_rank(V - 1)
            out_grads[V - 1].append(p2p.recv_backward(tensor_shape, dtype))
        for kb in range(remaining, total):
            ig = bwd_unit(kb)
            nb = chunk_of(kb + 1, forward=False)
            recv_next = not (ps.is_pipeline_last_stage(ignore_virtual=True) and nb == V - 1) and kb != total - 1
            og = p2p.send_backward_recv_backward(ig, recv_next, tensor_shape, dtype)
            if recv_next:
                out_grads[nb].append(og)
    ps.set_virtual_pipeline_model_parallel_rank(0)
    _LAST_SCHEDULE_STATS.clear()
    _LAST_SCHEDULE_STATS.update(stats, warmup=warmup, units=total)
    return losses


_LAST_SCHEDULE_STATS = {}


def last_schedule_stats():
    """{'max_live': peak stored forward units, 'warmup': warm-up units, 'units': n*V} of the most
    recent interleaved schedule on this rank (tests / memory planning)."""
    return dict(_LAST_SCHEDULE_STATS)


def get_forward_backward_func(virtual_pipeline_model_parallel_size=None, pipeline_model_parallel_size=None):
    pp = pipeline_model_parallel_size or ps.get_pipeline_model_parallel_world_size()
    if pp > 1:
        if virtual_pipeline_model_parallel_size is not None:
            return _forward_backward_pipelining_with_interleaving
        return forward_backward_pipelining_without_interleaving
    return forward_backward_no_pipelining
