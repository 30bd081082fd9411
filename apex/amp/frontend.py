"""``amp.initialize`` with opt levels O0-O3 (NS-01).

Opt levels (same contract as apex's later frontend; not in the v0.1 reference):
  O0  fp32 passthrough                         (cast none, no patching, scale 1)
  O1  cast-policy engine over torch functions  (apex.amp lists, dynamic scale)
  O2  model cast to low precision, BN fp32, fp32 master weights, dynamic scale
  O3  pure low precision                       (no masters, scale 1)
The low-precision dtype is fp16 by default (apex parity) and bf16 when requested
(``cast_model_type=torch.bfloat16`` or ``half_dtype=torch.bfloat16``); with bf16 the
default loss scale is 1.0 (bf16 has fp32's exponent range).
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from ._amp_state import _amp_state, maybe_print, warn_or_err


class Properties:
    def __init__(self):
        self.options = {
            "enabled": False,
            "opt_level": None,
            "cast_model_type": None,
            "patch_torch_functions": False,
            "keep_batchnorm_fp32": None,
            "master_weights": None,
            "loss_scale": 1.0,
            "half_dtype": torch.float16,
            "cast_model_outputs": None,
        }

    def _update_options_dict(self, new_options):
        for k, v in new_options.items():
            if k in self.options:
                self.options[k] = v
            else:
                raise ValueError("Tried to set unexpected option {}".format(k))

    def __getattr__(self, name):
        if "options" in self.__dict__:
            options = self.__dict__["options"]
            if name in options:
                return options[name]
        raise AttributeError("'{}' object has no attribute '{}'".format(type(self).__name__, name))

    def __setattr__(self, name, value):
        if "options" in self.__dict__ and name in self.options:
            if name == "cast_model_type":
                if self.opt_level == "O1" and value is not None and value is not torch.float32:
                    warn_or_err("O1 inserts casts around Torch functions rather than model weights, "
                                "so with O1 the model weights themselves should remain FP32.")
                self.options[name] = value
            elif name == "patch_torch_functions":
                if self.opt_level != "O1" and value:
                    warn_or_err("Currently, patch_torch_functions=True should only be set by "
                                "selecting opt_level='O1'.")
                self.options[name] = value
            elif name == "keep_batchnorm_fp32":
                if self.opt_level == "O1" and value is not None:
                    warn_or_err("With opt_level O1, batchnorm functions are automatically patched "
                                "to run in FP32, so keep_batchnorm_fp32 should be None.")
                if value == "False":
                    self.options[name] = False
                elif value == "True":
                    self.options[name] = True
                else:
                    assert value in (True, False, None)
                    self.options[name] = value
            elif name == "master_weights":
                if self.opt_level == "O1" and value is not None:
                    warn_or_err("It doesn't make sense to use master_weights with O1.")
                self.options[name] = value
            elif name == "loss_scale":
                self.options[name] = value if value == "dynamic" else float(value)
            else:
                self.options[name] = value
        else:
            super().__setattr__(name, value)


class O3:
    brief = "O3:  Pure low-precision training."
    more = "Calls .half()/.bfloat16() on the model; no master weights; loss scale 1."

    def __call__(self, p):
        p.enabled = True
        p.opt_level = "O3"
        p.cast_model_type = p.half_dtype
        p.patch_torch_functions = False
        p.keep_batchnorm_fp32 = False
        p.master_weights = False
        p.loss_scale = 1.0
        return p


class O2:
    brief = "O2:  Low-precision training with FP32 batchnorm and FP32 master weights."
    more = "Model cast to low precision (BN kept fp32), fp32 master weights in the optimizer."

    def __call__(self, p):
        p.enabled = True
        p.opt_level = "O2"
        p.cast_model_type = p.half_dtype
        p.patch_torch_functions = False
        p.keep_batchnorm_fp32 = True
        p.master_weights = True
        p.loss_scale = "dynamic" if p.half_dtype == torch.float16 else 1.0
        return p


class O1:
    brief = "O1:  Insert automatic casts around torch functions and Tensor methods."
    more = "Whitelist ops (GEMM/conv) run in low precision, blacklist ops in fp32."

    def __call__(self, p):
        p.enabled = True
        p.opt_level = "O1"
        p.cast_model_type = None
        p.patch_torch_functions = True
        p.keep_batchnorm_fp32 = None
        p.master_weights = None
        p.loss_scale = "dynamic" if p.half_dtype == torch.float16 else 1.0
        return p


class O0:
    brief = "O0:  Pure FP32 training."
    more = "No casts, no loss scaling: an fp32 baseline through the same code path."

    def __call__(self, p):
        p.enabled = True
        p.opt_level = "O0"
        p.cast_model_type = torch.float32
        p.patch_torch_functions = False
        p.keep_batchnorm_fp32 = None
        p.master_weights = False
        p.loss_scale = 1.0
        return p


opt_levels = {"O3": O3(), "O2": O2(), "O1": O1(), "O0": O0()}


def initialize(models, optimizers=None, enabled=True, opt_level="O1", cast_model_type=None,
               patch_torch_functions=None, keep_batchnorm_fp32=None, master_weights=None,
               loss_scale=None, cast_model_outputs=None, num_losses=1, verbosity=1,
               min_loss_scale=None, max_loss_scale=2.0 ** 24, half_dtype=None, fp8=False):
    """Configure models/optimizers for mixed precision. Returns (models, optimizers)
    with the same structure that was passed in (single object or list).

    ``fp8`` (MI355X extension, not in the reference): True or an ``apex.fp8.Fp8Recipe`` runs the
    fused ops' forward / input-gradient GEMMs in per-tensor scaled fp8 on top of ``opt_level``
    (O2 / O3 recommended: the weights are then bf16/fp16 model params); each patched
    ``optimizer.step()`` then updates the fp8 scales (apex.fp8.step)."""
    from ._initialize import _initialize

    _amp_state.opt_properties = Properties()
    _amp_state.verbosity = verbosity
    if not enabled:
        if optimizers is None:
            return models
        return models, optimizers
    if opt_level not in opt_levels:
        raise RuntimeError("Unexpected optimization level {}. Options are 'O0', 'O1', 'O2', 'O3'. "
                           "Note that in `O0`, `O1`, etc., the prefix O is the letter O, not the "
                           "number zero.".format(opt_level))
    if half_dtype is None and cast_model_type in (torch.bfloat16, torch.float16):
        half_dtype = cast_model_type
    _amp_state.opt_properties.options["half_dtype"] = half_dtype or torch.float16
    _amp_state.opt_properties = opt_levels[opt_level](_amp_state.opt_properties)
    maybe_print("Selected optimization level {}".format(opt_levels[opt_level].brief), True)
    overrides = OrderedDict(cast_model_type=cast_model_type,
                            patch_torch_functions=patch_torch_functions,
                            keep_batchnorm_fp32=keep_batchnorm_fp32, master_weights=master_weights,
                            loss_scale=loss_scale, cast_model_outputs=cast_model_outputs)
    for k, v in overrides.items():
        if v is not None:
            setattr(_amp_state.opt_properties, k, v)
    for k, v in _amp_state.opt_properties.options.items():
        maybe_print("{:22} : {}".format(k, v), True)
    _amp_state.min_loss_scale = min_loss_scale
    _amp_state.max_loss_scale = max_loss_scale
    _amp_state.fp8 = bool(fp8)
    if fp8:
        from .. import fp8 as _fp8

        _fp8.enable(fp8 if isinstance(fp8, _fp8.Fp8Recipe) else None)
        maybe_print("fp8                    : {}".format(_fp8.state().recipe), True)
    else:
        from .. import fp8 as _fp8

        if _fp8._GLOBAL:
            _fp8.disable()
    return _initialize(models, optimizers, _amp_state.opt_properties, num_losses, cast_model_outputs)


def state_dict(destination=None):
    if destination is None:
        destination = OrderedDict()
    for idx, scaler in enumerate(_amp_state.loss_scalers):
        destination["loss_scaler%d" % idx] = scaler.state_dict()
    return destination


def load_state_dict(state_dict):
    if len(state_dict) != len(_amp_state.loss_scalers):
        print("Warning: state_dict contains {} entries, while {} loss_scalers are used".format(
            len(state_dict), len(_amp_state.loss_scalers)))
    state_dict = state_dict.copy()
    nb = len(_amp_state.loss_scalers)
    unexpected, missing = [], []
    for key in list(state_dict.keys()):
        if "loss_scaler" not in key:
            unexpected.append(key)
            continue
        idx = int(key[len("loss_scaler"):])
        if idx >= nb:
            unexpected.append(key)
            continue
        _amp_state.loss_scalers[idx].load_state_dict(state_dict[key])
    if unexpected:
        raise RuntimeError("Error(s) in loading state_dict. Unexpected key(s): {}".format(
            ", ".join(unexpected)))
