"""apex.reparameterization — weight normalisation and generic reparameterizations (R-22).

Functional API of the reference (apex/reparameterization/__init__.py:4-127):
``apply_weight_norm``, ``remove_weight_norm``, ``apply_reparameterization``,
``remove_reparameterization``.
"""
from .reparameterization import Reparameterization
from .weight_norm import WeightNorm


def apply_weight_norm(module, name="", dim=0, hook_child=True):
    """Replace ``name`` (all >1-d params when empty) by magnitude ``<name>_g`` and
    direction ``<name>_v``; the weight is recomputed before every forward."""
    return apply_reparameterization(module, reparameterization=WeightNorm, hook_child=hook_child,
                                    name=name, dim=dim)


def remove_weight_norm(module, name="", remove_all=False):
    return remove_reparameterization(module, reparameterization=WeightNorm, name=name,
                                     remove_all=remove_all)


def apply_reparameterization(module, reparameterization=None, name="", dim=0, hook_child=True):
    assert reparameterization is not None
    if name != "":
        Reparameterization.apply(module, name, dim, reparameterization, hook_child)
    else:
        for n in list(module.state_dict().keys()):
            apply_reparameterization(module, reparameterization, n, dim, hook_child)
    return module


def _hooks_of(module):
    return [(k, h) for k, h in module._forward_pre_hooks.items() if isinstance(h, Reparameterization)]


def remove_reparameterization(module, reparameterization=Reparameterization, name="", remove_all=False):
    if name != "" or remove_all:
        to_remove = []
        for m in module.modules():
            for k, hook in _hooks_of(m):
                if isinstance(hook, reparameterization) and (remove_all or hook.name == name):
                    to_remove.append((m, k, hook))
        for m, k, hook in to_remove:
            hook.remove(m)
            m._forward_pre_hooks.pop(k, None)
        if remove_all or to_remove:
            return module
        raise ValueError("reparameterization of '{}' not found in {}".format(name, module))
    modules = [module] + [x for x in module.modules()]
    for m in modules:
        remove_reparameterization(m, reparameterization=reparameterization, remove_all=True)
    return module


__all__ = ["Reparameterization", "WeightNorm", "apply_weight_norm", "remove_weight_norm",
           "apply_reparameterization", "remove_reparameterization"]
