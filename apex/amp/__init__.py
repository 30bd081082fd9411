"""apex.amp — automatic mixed precision for MI355X.

New-style API (NS-01): ``initialize``, ``scale_loss``, ``state_dict``,
``load_state_dict``, ``master_params``.
Reference API (R-01..R-10, apex/amp/__init__.py:1-2): ``init``, ``half_function``,
``float_function``, ``promote_function``, ``register_half_function``,
``register_float_function``, ``register_promote_function``.
"""
from ._amp_state import _amp_state, master_params
from .frontend import initialize, load_state_dict, state_dict
from .handle import AmpHandle, NoOpHandle, scale_loss
from .amp import (bfloat16_function, float_function, half_function, init, promote_function,
                  register_bfloat16_function, register_float_function, register_half_function,
                  register_promote_function)

__all__ = ["initialize", "scale_loss", "state_dict", "load_state_dict", "master_params", "init",
           "half_function", "float_function", "promote_function", "register_half_function",
           "register_float_function", "register_promote_function", "bfloat16_function",
           "register_bfloat16_function", "AmpHandle", "NoOpHandle"]
