"""Single-node multi-process launcher (R-19).

    python -m apex.parallel.multiproc [--nproc N] script.py [script args...]

Reference (apex/parallel/multiproc.py:12-35): one child per GPU, ``--world-size`` and
``--rank i`` appended to (or overwritten in) each child's argv, rank 0 on stdout, others
logged to ``GPU_<i>.log``, then wait. Added for MI355X clusters: the torchrun-style
environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT,
HSA_ENABLE_IPC_MODE_LEGACY=0 for RCCL's dmabuf IPC) is exported to every child, and a
child that fails terminates the others so a job never hangs half-dead.
The GPU count is read without initialising HIP in the launcher (children own the GPUs).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def _gpu_count():
    try:
        import torch

        return max(torch.cuda.device_count(), 1)
    except Exception:
        return 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _set_arg(argv, flag, value):
    argv = list(argv)
    if flag in argv:
        argv[argv.index(flag) + 1] = str(value)
    else:
        argv += [flag, str(value)]
    return argv


def launch(argv, nproc=None, log_dir=".", inject_args=True, poll=0.2):
    world = nproc or _gpu_count()
    if "--world-size" in argv:
        world = int(argv[argv.index("--world-size") + 1])
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs, logs = [], []
    for i in range(world):
        child = list(argv)
        if inject_args:
            child = _set_arg(child, "--world-size", world)
            child = _set_arg(child, "--rank", i)
        env = dict(os.environ, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port, HSA_ENABLE_IPC_MODE_LEGACY="0")
        out = None
        if i > 0:
            out = open(os.path.join(log_dir, "GPU_{}.log".format(i)), "w")
            logs.append(out)
        print(" ".join([sys.executable] + child), flush=True)
        procs.append(subprocess.Popen([sys.executable] + child, stdout=out, stderr=subprocess.STDOUT if out else None,
                                      env=env))
    rc = 0
    try:
        alive = set(range(world))
        while alive:
            for i in list(alive):
                r = procs[i].poll()
                if r is None:
                    continue
                alive.discard(i)
                if r != 0 and rc == 0:  # first failure decides the exit code
                    rc = r if r > 0 else 128 - r
                    print("multiproc: rank {} exited with {}; terminating the others".format(i, r),
                          file=sys.stderr, flush=True)
                    for j in alive:
                        procs[j].send_signal(signal.SIGTERM)
            time.sleep(poll)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        rc = 130
    finally:
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        for f in logs:
            f.close()
    return rc


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    nproc = None
    if argv[:1] == ["--nproc"]:
        nproc = int(argv[1])
        argv = argv[2:]
    if not argv:
        print(__doc__)
        return 2
    return launch(argv, nproc)


if __name__ == "__main__":
    sys.exit(main())
