"""apex for AMD Instinct MI355X (gfx950 / CDNA4).

A from-scratch, MI355X-native framework with the capabilities and public API of
NVIDIA Apex (reference: mbrukman/apex-1 v0.1). Hot paths are
hand-written HIP kernels in ``apex._C`` (csrc/); collectives use RCCL through
torch.distributed.

Reference package root imports fp16_utils, parallel and amp (apex/__init__.py:3-5);
RNN and reparameterization are opt-in imports, as in the reference.
"""
__version__ = "0.1.0+mi355x"

from . import _ext  # noqa: F401
from . import amp  # noqa: F401
from . import fp16_utils  # noqa: F401
from . import parallel  # noqa: F401
from . import optimizers  # noqa: F401
from . import normalization  # noqa: F401
