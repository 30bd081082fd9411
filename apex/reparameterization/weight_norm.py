"""WeightNorm reparameterization (R-21): ``w = g * v / ||v||`` (norm over all dims but ``dim``).

Reference: apex/reparameterization/weight_norm.py:22-78. ``compute_weight`` goes through
the HIP weight-norm kernels (apex.fp16_utils.Fused_Weight_Norm, K-03), which the
reference could not do (its fused function was a stub).
"""
from __future__ import annotations

import torch
from torch.nn.parameter import Parameter

from ..fp16_utils import Fused_Weight_Norm
from ..fp16_utils.fused_weight_norm import _norm_except_dim
from .reparameterization import Reparameterization


def _norm(p, dim):
    """Norm over all dims except ``dim`` (keepdim shape), computed in fp32."""
    return _norm_except_dim(p, dim).to(p.dtype)


class WeightNorm(Reparameterization):
    def compute_weight(self, module=None, name=None):
        if module is None:
            module = self.module
        if name is None:
            name = self.name
        module, name = Reparameterization.get_module_and_name(module, name)
        g = getattr(module, name + "_g")
        v = getattr(module, name + "_v")
        return Fused_Weight_Norm.apply(v, g, self.dim)

    def reparameterize(self, name, weight, dim):
        names = [name + "_g", name + "_v"]
        params = [Parameter(_norm(weight, dim).data), Parameter(weight.data)]
        return names, params
