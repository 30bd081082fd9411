"""apex.contrib — fused attention (multihead_attn) and softmax cross-entropy (xentropy)."""
