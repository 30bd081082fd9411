"""Test runner (reference tests/run_test.py ran unittest discovery over run_amp and
run_fp16_optimizer). Runs the CPU tier, then the GPU tier when a GPU is visible.

  python tests/run_tests.py [extra pytest args]
"""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def main(argv):
    rc = pytest.main([HERE, "-q", "-m", "not gpu"] + argv)
    if rc != 0:
        return rc
    import torch

    if torch.cuda.is_available():
        rc = pytest.main([HERE, "-q", "-m", "gpu"] + argv)
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
