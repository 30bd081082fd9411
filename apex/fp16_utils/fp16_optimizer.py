"""FP16_Optimizer (R-11): fp32 master weights + static/dynamic loss scaling around any
torch optimizer. Reference: apex/fp16_utils/fp16_optimizer.py:11-551.

Behaviour kept: overflow is checked only with dynamic scaling, on the
MODEL grads, before the master copy; the scale is updated inside ``step()`` before
deciding to skip ("OVERFLOW!"); the closure path retries while overflowing;
``clip_master_grads`` returns -1 on overflow. Fixed: the reference tested
``torch.cuda.is_available`` without calling it (always truthy).

MI355X: model->master grad copy + 1/scale (K-02) is one multi-tensor launch per dtype
pair, master->model copy another, the overflow check one fused reduction (K-01).
Low-precision params may be fp16 or bf16.
"""
from __future__ import annotations

import torch

from .fp16util import _mt_copy, clip_grad_norm
from .loss_scaler import DynamicLossScaler, LossScaler

_LOW = (torch.float16, torch.bfloat16)


class FP16_Optimizer:
    def __init__(self, init_optimizer, static_loss_scale=1.0, dynamic_loss_scale=False,
                 dynamic_loss_args=None, verbose=True):
        self.verbose = verbose
        self.optimizer = init_optimizer
        self.fp16_groups = []
        self.fp32_from_fp16_groups = []
        self.fp32_from_fp32_groups = []
        for i, param_group in enumerate(self.optimizer.param_groups):
            self.maybe_print("FP16_Optimizer processing param group {}:".format(i))
            fp16_this, fp32_this, master_this = [], [], []
            for j, param in enumerate(param_group["params"]):
                if not param.requires_grad:
                    continue
                if param.dtype in _LOW:
                    self.maybe_print("FP16_Optimizer received {} with {}".format(param.dtype, param.size()))
                    fp16_this.append(param)
                    master = param.detach().clone().float()
                    master.requires_grad = True
                    param_group["params"][j] = master
                    master_this.append(master)
                    if param in self.optimizer.state:
                        self.optimizer.state[master] = self.optimizer.state.pop(param)
                elif param.dtype == torch.float32:
                    self.maybe_print("FP16_Optimizer received torch.float32 with {}".format(param.size()))
                    fp32_this.append(param)
                    param_group["params"][j] = param
                else:
                    raise TypeError("Wrapped parameters must be either float32, float16 or bfloat16. "
                                    "Received {}".format(param.dtype))
            self.fp16_groups.append(fp16_this)
            self.fp32_from_fp16_groups.append(master_this)
            self.fp32_from_fp32_groups.append(fp32_this)
        # re-cast any existing per-param optimizer state to the master dtype
        self.optimizer.load_state_dict(self.optimizer.state_dict())
        if dynamic_loss_scale:
            self.dynamic_loss_scale = True
            self.loss_scaler = DynamicLossScaler(**(dynamic_loss_args or {}))
        else:
            self.dynamic_loss_scale = False
            self.loss_scaler = LossScaler(static_loss_scale)
        self.overflow = False
        self.first_closure_call_this_step = True
        self.clip_grad_norm = clip_grad_norm

    def maybe_print(self, msg):
        if self.verbose:
            print(msg)

    def __getstate__(self):
        raise RuntimeError("FP16_Optimizer should be serialized using state_dict().")

    def __setstate__(self, state):
        raise RuntimeError("FP16_Optimizer should be deserialized using load_state_dict().")

    def zero_grad(self, set_grads_to_None=False):
        for group in self.optimizer.param_groups:
            for p in group["params"]:
                if set_grads_to_None:
                    p.grad = None
                elif p.grad is not None:
                    if p.grad._base is None:
                        p.grad.detach_()
                    p.grad.zero_()
        for fp16_group in self.fp16_groups:
            for param in fp16_group:
                if set_grads_to_None:
                    param.grad = None
                elif param.grad is not None:
                    if param.grad._base is None:  # DDP bucket views cannot detach_ in place
                        param.grad.detach_()
                    param.grad.zero_()

    def _check_overflow(self):
        params = [p for g in self.fp16_groups for p in g] + [p for g in self.fp32_from_fp32_groups for p in g]
        self.overflow = self.loss_scaler.has_overflow(params)

    def _update_scale(self, has_overflow=False):
        self.loss_scaler.update_scale(has_overflow)

    def _master_params_to_model_params(self):
        src = [m.data for g in self.fp32_from_fp16_groups for m in g]
        dst = [p.data for g in self.fp16_groups for p in g]
        _mt_copy(src, dst)

    def _model_grads_to_master_grads(self, scale=1.0):
        src, dst = [], []
        for fp16_group, master_group in zip(self.fp16_groups, self.fp32_from_fp16_groups):
            for model, master in zip(fp16_group, master_group):
                if model.grad is not None:
                    if master.grad is None:
                        master.grad = torch.empty_like(master.data)
                    src.append(model.grad.data)
                    dst.append(master.grad.data)
                else:
                    master.grad = None
        _mt_copy(src, dst, scale)

    def _downscale_master(self):
        if self.loss_scale != 1.0:
            grads = [p.grad.data for g in self.fp32_from_fp32_groups for p in g if p.grad is not None]
            _mt_copy(grads, grads, 1.0 / self.loss_scale)

    def clip_master_grads(self, max_norm, norm_type=2):
        if not self.overflow:
            fp32_params = [p for g in self.optimizer.param_groups for p in g["params"]]
            return self.clip_grad_norm(fp32_params, max_norm, norm_type)
        return -1

    def state_dict(self):
        """Plain containers + tensors only (the reference pickled the scaler object), so a
        checkpoint loads with ``torch.load(..., weights_only=True)``."""
        sd = {}
        sd["loss_scaler"] = self.loss_scaler.state_dict()
        sd["dynamic_loss_scale"] = self.dynamic_loss_scale
        sd["overflow"] = self.overflow
        sd["first_closure_call_this_step"] = self.first_closure_call_this_step
        sd["optimizer_state_dict"] = self.optimizer.state_dict()
        sd["fp32_from_fp16"] = [[m.detach() for m in g] for g in self.fp32_from_fp16_groups]
        return sd

    def load_state_dict(self, state_dict):
        scaler = state_dict["loss_scaler"]
        if isinstance(scaler, dict):
            self.loss_scaler = DynamicLossScaler() if state_dict["dynamic_loss_scale"] else LossScaler()
            self.loss_scaler.load_state_dict(scaler)
        else:  # a scaler object (in-process round trip)
            self.loss_scaler = scaler
        self.dynamic_loss_scale = state_dict["dynamic_loss_scale"]
        self.overflow = state_dict["overflow"]
        self.first_closure_call_this_step = state_dict["first_closure_call_this_step"]
        self.optimizer.load_state_dict(state_dict["optimizer_state_dict"])
        for current_group, saved_group in zip(self.fp32_from_fp16_groups, state_dict["fp32_from_fp16"]):
            for current, saved in zip(current_group, saved_group):
                current.data.copy_(saved.data)

    def step(self, closure=None):
        scale = self.loss_scaler.loss_scale
        self._update_scale(self.overflow)
        if self.overflow:
            print("OVERFLOW! Skipping step. Attempted loss scale: {}, reducing to {}"
                  .format(scale, self.loss_scale))
            return
        if closure is not None:
            retval = self._step_with_closure(closure)
        else:
            retval = self.optimizer.step()
        self._master_params_to_model_params()
        return retval

    def _step_with_closure(self, closure):
        def wrapped_closure():
            if self.first_closure_call_this_step:
                self.first_closure_call_this_step = False
            else:
                self._master_params_to_model_params()
            temp_loss = closure()
            while self.overflow:
                scale = self.loss_scaler.loss_scale
                self._update_scale(self.overflow)
                print("OVERFLOW within closure! Skipping step. Attempted loss scale: {}, "
                      "reducing to {}".format(scale, self.loss_scale))
                temp_loss = closure()
            return temp_loss

        retval = self.optimizer.step(wrapped_closure)
        self.first_closure_call_this_step = True
        return retval

    def backward(self, loss, update_master_grads=True):
        self.loss_scaler.backward(loss.float())
        if update_master_grads:
            self.update_master_grads()

    def update_master_grads(self):
        if self.dynamic_loss_scale:
            self._check_overflow()
            if self.overflow:
                return
        # fused copy + downscale (K-02): master.grad = model.grad / scale
        self._model_grads_to_master_grads(1.0 / self.loss_scale)
        self._downscale_master()

    def inspect_master_grad_data(self):
        if self.overflow:
            print("Warning:  calling FP16_Optimizer.inspect_master_grad_data while in an overflow "
                  "state.  Gradients are currently invalid (may be inf, nan, or stale).  "
                  "Returning None.")
            return None
        master_grads_data = []
        for param_group in self.optimizer.param_groups:
            master_grads_this_group = []
            for param in param_group["params"]:
                master_grads_this_group.append(param.grad.data if param.grad is not None else None)
            master_grads_data.append(master_grads_this_group)
        return master_grads_data

    def _get_loss_scale(self):
        return self.loss_scaler.loss_scale

    def _set_loss_scale(self, value):
        self.loss_scaler.cur_scale = value

    loss_scale = property(_get_loss_scale, _set_loss_scale)

    def _get_state(self):
        return self.optimizer.state

    def _set_state(self, value):
        self.optimizer.state = value

    state = property(_get_state, _set_state)

    def _get_param_groups(self):
        return self.optimizer.param_groups

    def _set_param_groups(self, value):
        self.optimizer.param_groups = value

    param_groups = property(_get_param_groups, _set_param_groups)
