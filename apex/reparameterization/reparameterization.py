"""Weight reparameterization hooks (R-20).

API of the reference (apex/reparameterization/reparameterization.py:4-151): a hook object
that replaces ``module.<name>`` by reparameterization parameters and recomputes the weight
in a forward pre-hook. Staleness is tracked with the parameters' autograd version
counters (the weight is recomputed after any in-place update such as an optimizer step,
and on every forward while autograd is recording) instead of the reference's module
backward hook, which torch 2 deprecates.
"""
from __future__ import annotations

import torch
from torch.nn.parameter import Parameter


class Reparameterization:
    def __init__(self, name, dim, module, retain_forward=True):
        self.name = name
        self.dim = dim
        self.evaluated = False
        self.retain_forward = retain_forward
        self.reparameterization_names = []
        self.backward_hook_key = None
        self.module = module
        self._versions = None
        self._pre_handle = None

    def compute_weight(self, module=None, name=None):
        raise NotImplementedError

    def reparameterize(self, name, weight, dim):
        raise NotImplementedError

    @staticmethod
    def apply(module, name, dim, reparameterization=None, hook_child=True):
        if reparameterization is None:
            reparameterization = Reparameterization
        module2use, name2use = Reparameterization.get_module_and_name(module, name)
        if name2use is None or isinstance(module2use, (torch.nn.Embedding, torch.nn.EmbeddingBag)):
            return None
        weight = getattr(module2use, name2use, None)
        if not isinstance(weight, torch.Tensor) or weight.dim() <= 1:
            return None
        if name2use not in module2use._parameters:
            return None  # buffers (e.g. running stats) are not reparameterized
        fn = reparameterization(name2use, dim, module2use) if hook_child else \
            reparameterization(name, dim, module)
        del module2use._parameters[name2use]
        names, params = fn.reparameterize(name2use, weight, dim)
        for n, p in zip(names, params):
            module2use.register_parameter(n, p)
        fn.reparameterization_names = names
        setattr(module2use, name2use, None)
        hook_module = module2use if hook_child else module
        fn._pre_handle = hook_module.register_forward_pre_hook(fn)
        fn.backward_hook_key = fn._pre_handle.id
        return fn

    @staticmethod
    def get_module_and_name(module, name):
        names = name.split(".")
        if len(names) == 1 and names[0] != "":
            return module, names[0]
        if len(names) > 1:
            m = module
            for n in names[:-1]:
                m = getattr(m, n)
            return m, names[-1]
        return None, None

    def get_params(self, module):
        return [getattr(module, n) for n in self.reparameterization_names]

    def remove(self, module):
        module2use, name2use = Reparameterization.get_module_and_name(module, self.name)
        for p in self.get_params(module2use):
            p.requires_grad = False
        weight = self.compute_weight(module2use, name2use)
        if hasattr(module2use, name2use):
            delattr(module2use, name2use)
        for n in self.reparameterization_names:
            del module2use._parameters[n]
        module2use.register_parameter(name2use, Parameter(weight.data))
        if self._pre_handle is not None:
            self._pre_handle.remove()

    def _stale(self, module2use):
        vers = tuple(p._version for p in self.get_params(module2use))
        stale = (not self.evaluated) or vers != self._versions or torch.is_grad_enabled()
        self._versions = vers
        return stale

    def __call__(self, module, inputs):
        module2use, name2use = Reparameterization.get_module_and_name(module, self.name)
        _w = getattr(module2use, name2use)
        if _w is None or self._stale(module2use):
            setattr(module2use, name2use, self.compute_weight(module2use, name2use))
            self.evaluated = True

    def backward_hook(self, module, grad_input, grad_output):
        """Kept for API compatibility: marks the weight stale."""
        self.evaluated = False
