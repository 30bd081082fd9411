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
        in_grad = backward_step(i_t, o_t, out_grad, grad_scaler)
        if last:
            inp = None
            p2p.send_backward(in_grad, tensor_shape, dtype)
        else:
            inp = p2p.send_backward_recv_forward(in_grad, tensor_shape, dtype)

    if not forward_only:
        for _ in range(warmup):
            i_t, o_t = inputs.pop(0), outputs.pop(0)
            out_grad = p2p.recv_backward(tensor_shape, dtype)
            in_grad = backward_step(i_t, o_t, out_grad, grad_scaler)
            p2p.send_backward(in_grad, tensor_shape, dtype)
    return losses


def _forward_backward_pipelining_with_interleaving(forward_step_func, batch, model, *, forward_only=False,
                                                   tensor_shape=None, dtype=torch.float32, grad_scaler=None,
                                                   disable_autocast=False, **kwargs):
    """Interleaved 1F1B over ``len(model)`` virtual stages per rank (depth-first order of model
    chunks). Implemented as the reference-equivalent sequence of chunk-wise forward passes
    followed by backward passes in reverse chunk order per microbatch group, which keeps
    every send matched with a receive on the neighbouring rank."""
    assert isinstance(model, (list, tuple)) and len(model) > 1
    assert tensor_shape is not None
    n = get_num_microbatches()
    mbs = _split_microbatches(batch, n)
    nchunks = len(model)
    losses = []
    saved = [[] for _ in range(nchunks)]
    for mb in mbs:
        for c in range(nchunks):
            ps.set_virtual_pipeline_model_parallel_rank(c)
            inp = p2p.recv_forward(tensor_shape, dtype)
            out = forward_step(forward_step_func, mb, model[c], inp, losses, n, grad_scaler)
            p2p.send_forward(out, tensor_shape, dtype)
            saved[c].append((inp, out))
    if not forward_only:
        for _ in mbs:
            for c in reversed(range(nchunks)):
                ps.set_virtual_pipeline_model_parallel_rank(c)
                inp, out = saved[c].pop(0)
                og = p2p.recv_backward(tensor_shape, dtype)
                ig = backward_step(inp, out, og, grad_scaler)
                p2p.send_backward(ig, tensor_shape, dtype)
    ps.set_virtual_pipeline_model_parallel_rank(0)
    return losses


def get_forward_backward_func(virtual_pipeline_model_parallel_size=None, pipeline_model_parallel_size=None):
    pp = pipeline_model_parallel_size or ps.get_pipeline_model_parallel_world_size()
    if pp > 1:
        if virtual_pipeline_model_parallel_size is not None:
            return _forward_backward_pipelining_with_interleaving
        return forward_backward_pipelining_without_interleaving
    return forward_backward_no_pipelining
