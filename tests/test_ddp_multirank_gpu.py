"""Multi-rank DDP race test on the GPU (SURVEY R-43; reference tests/distributed/ddp_race_condition_test.py
and run_race_test.sh): 2 and 4 processes, every rank on cuda:0, gloo collectives over the real
bucket buffers, closed-form gradient checks every iteration (tests/ddp_multirank_worker.py).

The ranks are separate processes started by torch.distributed.run in a child process (this test
process never forks a GPU context); each is bounded by a timeout. RCCL's own multi-rank path needs
one GPU per rank (it refuses duplicates), so the reduction-stream ordering of the RCCL path is
screened at one rank with several communicators in tests/test_ddp_race_gpu.py."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, mode, iters=10, n=1 << 20, timeout=150):
    env = dict(os.environ)
    # one hardware queue per process: 4 HIP processes x 4 queues oversubscribe one GPU's queue slots and
    # get time-sliced (profiles/r5_rehearsal_hw_queues.txt)
    env.update(PYTHONUNBUFFERED="1", OMP_NUM_THREADS="2", APEX_DIST_SHARE_GPU="1", GPU_MAX_HW_QUEUES="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "ddp_multirank_worker.py"), "--mode", mode, "--iters", str(iters),
           "--numel", str(n)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines, dec, i = [], json.JSONDecoder(), 0  # rank lines may interleave on one stdout line
    while True:
        i = r.stdout.find('{"rank"', i)
        if i < 0:
            break
        obj, i = dec.raw_decode(r.stdout, i)
        lines.append(obj)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    return lines


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("mode", ["default", "delay", "main_grad", "fp32_reduce"])
def test_multirank_closed_form(world, mode):
    lines = _launch(world, mode)
    assert sorted(l["rank"] for l in lines) == list(range(world)), lines
    for l in lines:
        assert l["ok"], l
