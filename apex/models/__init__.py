"""apex.models — workloads of BASELINE.json written from scratch (random init)."""
