"""Manual master-parameter utilities (R-13, K-02).

Reference: apex/fp16_utils/fp16util.py:6-144. The copies between model and master
params are single multi-tensor launches on the GPU (one chunk table for all
params) instead of a Python loop of ``copy_``; the flat-master variant packs into
one contiguous fp32 buffer. The "half" dtype may be fp16 or bf16.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

from .. import _ext

_LOW = (torch.float16, torch.bfloat16)


class tofp16(nn.Module):
    """Model wrapper that casts the input to half (or ``dtype``)."""

    def __init__(self, dtype=torch.float16):
        super().__init__()
        self.dtype = dtype

    def forward(self, input):
        return input.to(self.dtype)


class tobf16(tofp16):
    def __init__(self):
        super().__init__(torch.bfloat16)


def BN_convert_float(module):
    """Keep BatchNorm layers in fp32 after ``module.half()`` (reference :21-34)."""
    if isinstance(module, torch.nn.modules.batchnorm._BatchNorm) and module.affine is True:
        module.float()
    for child in module.children():
        BN_convert_float(child)
    return module


def network_to_half(network, dtype=torch.float16):
    """``Sequential(tofp16(), BN_convert_float(network.half()))`` (reference :37-41)."""
    return nn.Sequential(tofp16(dtype), BN_convert_float(network.to(dtype)))


def network_to_bf16(network):
    return network_to_half(network, torch.bfloat16)


def convert_module(module, dtype):
    for param in module.parameters(recurse=False):
        if param is not None:
            if param.data.dtype.is_floating_point:
                param.data = param.data.to(dtype=dtype)
            if param._grad is not None and param._grad.data.dtype.is_floating_point:
                param._grad.data = param._grad.data.to(dtype=dtype)
    for buf in module.buffers(recurse=False):
        if buf is not None and buf.data.dtype.is_floating_point:
            buf.data = buf.data.to(dtype=dtype)


def convert_network(network, dtype):
    for module in network.modules():
        if isinstance(module, torch.nn.modules.batchnorm._BatchNorm) and module.affine is True:
            continue
        convert_module(module, dtype)
    return network


def prep_param_lists(model, flat_master=False):
    """Returns (model_params, master_params); master is fp32 (optionally one flat tensor)."""
    model_params = [param for param in model.parameters() if param.requires_grad]
    if flat_master:
        try:
            master_params = _flatten_dense_tensors([param.data for param in model_params]).float()
        except Exception:
            print("Error in prep_param_lists:  model may contain a mixture of parameters "
                  "of different types.  Use flat_master=False, or use FP16_Optimizer.")
            raise
        master_params = torch.nn.Parameter(master_params)
        master_params.requires_grad = True
        if master_params.grad is None:
            master_params.grad = master_params.new(*master_params.size())
        return model_params, [master_params]
    master_params = [param.clone().float().detach() for param in model_params]
    for param in master_params:
        param.requires_grad = True
    return model_params, master_params


def _mt_copy(src, dst, scale=1.0):
    """dst[i] = src[i] * scale for lists of device tensors (one launch per dtype pair)."""
    if not src:
        return
    if _ext.use_native(src[0]):
        from ..multi_tensor_apply import get_plan

        groups = {}
        for s, d in zip(src, dst):
            groups.setdefault((s.dtype, d.dtype), ([], []))
            groups[(s.dtype, d.dtype)][0].append(s)
            groups[(s.dtype, d.dtype)][1].append(d)
        for ss, dd in groups.values():
            get_plan([ss, dd]).scale(None, float(scale), None)
        return
    for s, d in zip(src, dst):
        if scale == 1.0:
            d.copy_(s)
        else:
            d.copy_(s.float() * scale)


def model_grads_to_master_grads(model_params, master_params, flat_master=False):
    """Copy model grads into the fp32 master grads (reference :93-112)."""
    if flat_master:
        master_params[0].grad.data.copy_(_flatten_dense_tensors([p.grad.data for p in model_params]))
        return
    src, dst = [], []
    for model, master in zip(model_params, master_params):
        if model.grad is not None:
            if master.grad is None:
                master.grad = torch.empty_like(master.data)
            src.append(model.grad.data)
            dst.append(master.grad.data)
        else:
            master.grad = None
    _mt_copy(src, dst)


def master_params_to_model_params(model_params, master_params, flat_master=False):
    """Copy fp32 masters back into the model params (reference :115-129)."""
    if flat_master:
        for model, master in zip(model_params, _unflatten_dense_tensors(master_params[0].data, model_params)):
            model.data.copy_(master)
        return
    _mt_copy([m.data for m in master_params], [p.data for p in model_params])


def to_python_float(t):
    if hasattr(t, "item"):
        return t.item()
    return t[0]


def clip_grad_norm(parameters, max_norm, norm_type=2):
    """``torch.nn.utils.clip_grad_norm_``; the 2-norm of device grads is one fused
    multi-tensor reduction (K-07) and the rescale one multi-tensor scale."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    params = [p for p in parameters if p.grad is not None]
    if not params:
        return torch.tensor(0.0)
    if norm_type == 2 and _ext.use_native(params[0].grad):
        from ..multi_tensor_apply import get_plan

        by_dt = {}
        for p in params:
            by_dt.setdefault(p.grad.dtype, []).append(p.grad)
        sq = None
        for gl in by_dt.values():
            gn, _ = get_plan([gl]).l2norm(0, False, None, 1.0, None)
            sq = gn * gn if sq is None else sq + gn * gn
        total = sq.sqrt()
        coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
        for gl in by_dt.values():
            get_plan([gl, gl]).scale(coef.reshape(()), 1.0, None)
        return total.reshape(())
    return torch.nn.utils.clip_grad_norm_(params, max_norm, norm_type)
