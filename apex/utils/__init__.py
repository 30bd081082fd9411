"""Runtime utilities: benchmark harness, metrics (reduce_tensor / meters / JSONL logging),
profiler ranges, input prefetcher with the fused normalize kernel."""
from .metrics import AverageMeter, JsonlLogger, reduce_tensor  # noqa: F401
