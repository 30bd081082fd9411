"""apex.transformer.functional — fused scale / mask / softmax."""
from .fused_softmax import FusedScaleMaskSoftmax, ScaledMaskedSoftmax, ScaledSoftmax, ScaledUpperTriangMaskedSoftmax
