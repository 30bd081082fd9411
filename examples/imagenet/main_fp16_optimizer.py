"""ImageNet-style training with FP16_Optimizer (reference examples/imagenet/main_fp16_optimizer.py):
``main.py --precision fp16_opt``; extra flags pass through."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from main import main  # noqa: E402

if __name__ == "__main__":
    main(["--precision", "fp16_opt"] + sys.argv[1:])
