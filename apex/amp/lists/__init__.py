"""Per-namespace views of apex.amp.policy (API compatibility with apex.amp.lists)."""
