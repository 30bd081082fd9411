"""ImageNet-style training with apex.parallel.Reducer — grads all-reduced once after backward,
at a point the user picks (reference examples/imagenet/main_reducer.py): ``main.py --reducer``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from main import main  # noqa: E402

if __name__ == "__main__":
    main(["--reducer", "--precision", "manual"] + sys.argv[1:])
