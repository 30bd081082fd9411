"""CPU/gloo rehearsal of bench.py's N-rank path (the driver's 2/4/8-GPU scaling runs).

``bench.py --cpu-rehearsal`` runs the SAME sequence the multi-GPU bench runs — pre-flight
known-value all-reduces, in-job bucket-size probe and selection, apex DDP with the chosen buckets,
warmup + timed steps bracketed by barriers, MAX over ranks, the fp32 pass, the all-reduce probe,
one JSON line from rank 0 — on CPU over gloo with a tiny BERT, launched exactly as the driver
launches it (``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1``)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [2, 4])
def test_bench_n_rank_path_on_gloo(n):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("APEX_DDP_MESSAGE_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--cpu-rehearsal", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE JSON line, nothing else on stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["parallelism"] == f"dp{n}" and out["config"]["global_batch"] == 8 * n
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    d = out["dist"]
    assert d["preflight"]["ok"] is True and d["preflight"]["nranks"] == n
    assert d["bucket_choice"].startswith("probe") and len(d["bucket_probe"]) == 3
    assert d["message_size"] in [p["numel"] for p in d["bucket_probe"]]
    assert out["allreduce_probe"]["bytes"] > 0 and out["allreduce_probe"]["us"] > 0
    assert out["ddp"]["world_size"] == n and out["ddp"]["num_buckets"] >= 2
    assert out["fp32_ms_per_step"] > 0 and out["speedup_vs_fp32"] > 0
    assert "rehearsal" in out and "NOT a measurement" in out["rehearsal"]
