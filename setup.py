"""Build / install apex for MI355X (gfx950).

  python setup.py build_ext --inplace     # compile csrc/*.hip + bindings into apex/_C*.so
  python setup.py develop                  # same, then put the checkout on sys.path

The HIP translation units are compiled with ``hipcc --offload-arch=gfx950`` by
tools/build_ext.py (parallel, incremental); setuptools only drives it. There is no CUDA
build and no hipify step.
"""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_ext import build_ext

ROOT = os.path.dirname(os.path.abspath(__file__))


class HipBuild(build_ext):
    def run(self):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import build_ext as hip_build

        out = hip_build.build(jobs=int(os.environ.get("MAX_JOBS", os.cpu_count() or 8)), force=self.force,
                              verbose=bool(self.verbose))
        if not self.inplace:  # copy next to the built package as well
            dst = os.path.join(self.build_lib, "apex", os.path.basename(out))
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            self.copy_file(out, dst)


setup(
    name="apex",
    version="0.1.0+mi355x",
    description="MI355X-native mixed precision and distributed training utilities for PyTorch-ROCm",
    packages=find_packages(include=["apex", "apex.*"]),
    package_data={"apex": ["_C*.so"]},
    cmdclass={"build_ext": HipBuild},
    ext_modules=[],
    python_requires=">=3.9",
)
