"""Point-to-point activation exchange between pipeline stages (NS-08).

Each call batches its sends/receives into one ``batch_isend_irecv`` (RCCL group call), so
a 1F1B steady-state step "send activation forward + receive gradient backward" is a single
grouped launch on the direct xGMI link between the two stage peers. Shapes/dtypes are
agreed up front (``tensor_shape``), so no metadata exchange is needed per message.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import parallel_state as ps


def _devices(sent):
    """(wire device, compute device). RCCL moves device buffers; gloo only host buffers, so a
    gloo run with GPU activations stages through the host (rehearsals, CPU tests)."""
    if sent is not None:
        compute = sent.device
    elif torch.cuda.is_available() and torch.cuda.is_initialized():
        compute = torch.device("cuda", torch.cuda.current_device())
    else:
        compute = torch.device("cpu")
    wire = compute if dist.get_backend() == "nccl" else torch.device("cpu")
    return wire, compute


def _communicate(tensor_send_next, tensor_send_prev, recv_prev, recv_next, tensor_shape, dtype):
    sent = tensor_send_next if tensor_send_next is not None else tensor_send_prev
    dev, compute = _devices(sent)
    t_prev = torch.empty(tensor_shape, dtype=dtype, device=dev) if recv_prev else None
    t_next = torch.empty(tensor_shape, dtype=dtype, device=dev) if recv_next else None
    group = ps.get_pipeline_model_parallel_group()
    # the wire format is the agreed (shape, dtype): a stage whose output is wider (amp O2 casts
    # model outputs to fp32) sends it in the agreed dtype, or the peer's receive size mismatches
    if tensor_send_prev is not None:
        tensor_send_prev = tensor_send_prev.detach().to(device=dev, dtype=dtype)
    if tensor_send_next is not None:
        tensor_send_next = tensor_send_next.detach().to(device=dev, dtype=dtype)
    prev, nxt = ps.get_pipeline_model_parallel_prev_rank(), ps.get_pipeline_model_parallel_next_rank()
    send_prev = dist.P2POp(dist.isend, tensor_send_prev.contiguous(), prev, group) if tensor_send_prev is not None else None
    recv_prev_op = dist.P2POp(dist.irecv, t_prev, prev, group) if t_prev is not None else None
    send_next = dist.P2POp(dist.isend, tensor_send_next.contiguous(), nxt, group) if tensor_send_next is not None else None
    recv_next_op = dist.P2POp(dist.irecv, t_next, nxt, group) if t_next is not None else None
    # Messages between one pair of ranks are matched in issue order (RCCL p2p has no tags). With
    # two stages the previous and the next rank are the SAME peer, so an activation and a gradient
    # travel between the pair in one grouped call: even ranks issue (send next, recv prev,
    # send prev, recv next) and odd ranks (recv prev, send next, recv next, send prev), so each
    # direction carries the activation first and the gradient second on both ends.
    if ps.get_pipeline_model_parallel_rank() % 2 == 0:
        order = (send_next, recv_prev_op, send_prev, recv_next_op)
    else:
        order = (recv_prev_op, send_next, recv_next_op, send_prev)
    ops = [op for op in order if op is not None]
    if ops:
        # wait() orders the compute stream after RCCL's stream (no host synchronisation)
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    if t_prev is not None:
        t_prev = t_prev.to(compute).requires_grad_(True)
    if t_next is not None:
        t_next = t_next.to(compute)
    return t_prev, t_next


def recv_forward(tensor_shape, dtype=torch.float32):
    if ps.is_pipeline_first_stage():
        return None
    return _communicate(None, None, True, False, tensor_shape, dtype)[0]


def recv_backward(tensor_shape, dtype=torch.float32):
    if ps.is_pipeline_last_stage():
        return None
    return _communicate(None, None, False, True, tensor_shape, dtype)[1]


def send_forward(output_tensor, tensor_shape=None, dtype=torch.float32):
    if not ps.is_pipeline_last_stage():
        _communicate(output_tensor, None, False, False, tensor_shape, dtype)


def send_backward(input_tensor_grad, tensor_shape=None, dtype=torch.float32):
    if not ps.is_pipeline_first_stage():
        _communicate(None, input_tensor_grad, False, False, tensor_shape, dtype)


def send_forward_recv_backward(output_tensor, tensor_shape, dtype=torch.float32):
    if ps.is_pipeline_last_stage():
        return None
    return _communicate(output_tensor, None, False, True, tensor_shape, dtype)[1]


def send_backward_recv_forward(input_tensor_grad, tensor_shape, dtype=torch.float32):
    if ps.is_pipeline_first_stage():
        return None
    return _communicate(None, input_tensor_grad, True, False, tensor_shape, dtype)[0]


def send_forward_recv_forward(output_tensor, recv_prev, tensor_shape, dtype=torch.float32):
    return _communicate(output_tensor, None, recv_prev, False, tensor_shape, dtype)[0]


def send_backward_recv_backward(input_tensor_grad, recv_next, tensor_shape, dtype=torch.float32):
    return _communicate(None, input_tensor_grad, False, recv_next, tensor_shape, dtype)[1]


def send_forward_backward_recv_forward_backward(output_tensor, input_tensor_grad, recv_prev, recv_next,
                                                tensor_shape, dtype=torch.float32):
    return _communicate(output_tensor, input_tensor_grad, recv_prev, recv_next, tensor_shape, dtype)
