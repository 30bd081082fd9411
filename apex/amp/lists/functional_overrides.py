"""View of apex.amp.policy.FUNCTIONAL in the apex.amp.lists layout."""
from ..policy import FUNCTIONAL as _T

MODULE = _T["module"]
FP16_FUNCS = list(_T["low"])
FP32_FUNCS = list(_T["fp32"])
CASTS = list(_T["promote"])
SEQUENCE_CASTS = list(_T["sequence"])
BANNED_FUNCS = list(_T["banned"])
