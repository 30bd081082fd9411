"""Pre-tuned library GEMM selection (PyTorch TunableOp over hipBLASLt / rocBLAS).

Plain library GEMMs (the dense projections of the transformer layers) go to hipBLASLt. Its
default heuristic picks a kernel per shape that is not always the fastest on MI355X — the
long-K weight-gradient GEMMs in particular. TunableOp benchmarks every hipBLASLt and rocBLAS
solution for a shape once and records the winner; the results for the benchmark shapes are
committed under ``tuning/`` (one file per device ordinal, identical content) and loaded
read-only at start-up, so no tuning happens inside a timed run. Shapes missing from the file
use the library default.

Regenerate (on an MI355X):  APEX_TUNABLEOP_TUNE=1 python bench.py --steps 3 --warmup 2
then copy ``tuning/tunableop_results0.csv`` to ordinals 1..7. The file also holds the GPT-2 1.5B
and Megatron GPT (micro-batch 4 x 2048) shapes, tuned over hipBLASLt by tools/gpu_tune_one.sh
and merged (profiles/r2_tunableop_models_ab.jsonl: GPT-2 72.3k -> 77.2k tokens/s, Megatron
45.5k -> 46.7k, same box).
"""
from __future__ import annotations

import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEFAULT_DIR = os.path.join(ROOT, "tuning")


def enable_tuned_gemms(directory: str | None = None) -> bool:
    """Point TunableOp at the committed results. Must run before the first GEMM.

    Returns False (library defaults) when disabled with APEX_TUNABLEOP=0 or no file exists.
    """
    if os.environ.get("APEX_TUNABLEOP", "1") == "0":
        return False
    directory = directory or DEFAULT_DIR
    tune = os.environ.get("APEX_TUNABLEOP_TUNE", "0") == "1"
    if not tune and not os.path.exists(os.path.join(directory, "tunableop_results0.csv")):
        return False
    os.makedirs(directory, exist_ok=True)
    os.environ.setdefault("PYTORCH_TUNABLEOP_ENABLED", "1")
    os.environ.setdefault("PYTORCH_TUNABLEOP_TUNING", "1" if tune else "0")
    os.environ.setdefault("PYTORCH_TUNABLEOP_FILENAME", os.path.join(directory, "tunableop_results%d.csv"))
    if tune:
        os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS", "8")
        os.environ.setdefault("PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS", "2")
    return True
