"""apex.fp16_utils — manual and automatic fp32-master-weight utilities (R-11..R-14).

Reference exports: apex/fp16_utils/__init__.py:1-19.
"""
from .fp16util import (BN_convert_float, clip_grad_norm, convert_module, convert_network,
                       master_params_to_model_params, model_grads_to_master_grads,
                       network_to_bf16, network_to_half, prep_param_lists, to_python_float,
                       tobf16, tofp16)
from .fused_weight_norm import Fused_Weight_Norm
from .fp16_optimizer import FP16_Optimizer
from .loss_scaler import DynamicLossScaler, LossScaler
