"""In-tree builder for ``apex._C`` (gfx950 only).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into an
object that contains only HIP code (no torch headers -> seconds per file);
``csrc/bindings.cpp`` is compiled once by the host compiler against torch's
headers; everything is linked into ``apex/_C<EXT_SUFFIX>`` next to the package so
that the shared object travels with the repository snapshot to the GPU box.

No hipify, no CUDA path, no JIT cache under ~/.cache.

Usage:  python tools/build_ext.py [-j N] [--force] [--verbose]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("APEX_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch

    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir, inc, os.path.join(tdir, "lib"), abi


def output_path() -> str:
    return os.path.join(ROOT, "apex", "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build step failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    if r.stdout.strip() and verbose:
        print(r.stdout)


def build(jobs: int | None = None, force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    tdir, tinc, tlib, abi = _torch_paths()
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-DNDEBUG"]
    steps = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            cmd = [hipcc, f"--offload-arch={ARCH}", "-c", src, "-o", obj, "-munsafe-fp-atomics"] + common
            steps.append(cmd)
    bind = os.path.join(CSRC, "bindings.cpp")
    bobj = os.path.join(BUILD, "bindings.cpp.o")
    objs.append(bobj)
    if force or _newer(bobj, [bind] + headers):
        py_inc = sysconfig.get_paths()["include"]
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-c", bind, "-o", bobj] + common + [
            f"-I{i}" for i in tinc] + [
            f"-I{py_inc}", f"-I{ROCM}/include", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
            f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            "-Wno-deprecated-declarations"]
        steps.append(cmd)
    jobs = jobs or min(8, os.cpu_count() or 4)
    if steps:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_run, c, verbose) for c in steps]
            for f in futs:
                f.result()
    out = output_path()
    if force or steps or _newer(out, objs):
        cxx = os.environ.get("CXX", "g++")
        cmd = [cxx, "-shared", "-o", out] + objs + [
            f"-L{tlib}", f"-Wl,-rpath,{tlib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            "-lc10_hip", "-ltorch_hip", "-lamdhip64"]
        _run(cmd, verbose)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args()
    out = build(a.j, a.force, a.verbose)
    print(out)


if __name__ == "__main__":
    sys.exit(main())
