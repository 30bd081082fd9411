"""Multi-GPU readiness checks on CPU/gloo (world 2): the known-value pre-flight all-reduce
passes, a rank that receives corrupted results makes EVERY rank raise (none hangs), and the
bucket-size selection picks the smallest size near the best bus bandwidth (pure function)."""
import os
import socket
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from apex.parallel import preflight


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, sabotage):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        if sabotage and rank == 1:
            real = dist.all_reduce

            def bad(t, *a, **k):
                r = real(t, *a, **k)
                if t.numel() == 1 << 12:  # corrupt the data check only
                    t.add_(1)
                return r

            dist.all_reduce = bad
        try:
            out = preflight.preflight_allreduce(None, "cpu", numel=1 << 12)
            res = "ok" if (not sabotage and out["nranks"] == world and out["small_allreduce_us"] > 0) else f"no error {out}"
        except preflight.PreflightError as e:
            res = "ok" if (sabotage and "[1]" in str(e)) else str(e)
        if not sabotage:
            probe = preflight.probe_bucket_sizes(None, "cpu", sizes=(1000, 4000), dtype=torch.float32, iters=2)
            msg, first = preflight.select_bucket_sizes(probe, min_first=10)
            assert msg in (1000, 4000) and first <= msg
        q.put((rank, res))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sabotage", [False, True])
def test_preflight_allreduce(sabotage):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, sabotage)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] == "ok" for r in res), res


def test_select_bucket_sizes():
    probe = [{"numel": 8_000_000, "us": 150.0, "busbw_gbs": 180.0},
             {"numel": 25_000_000, "us": 400.0, "busbw_gbs": 215.0},
             {"numel": 50_000_000, "us": 790.0, "busbw_gbs": 220.0}]
    assert preflight.select_bucket_sizes(probe) == (25_000_000, 6_250_000)
    # bandwidth already flat at the smallest size: pick it
    flat = [dict(p, busbw_gbs=200.0) for p in probe]
    assert preflight.select_bucket_sizes(flat)[0] == 8_000_000
    assert preflight.select_bucket_sizes(probe, tolerance=1.0)[0] == 50_000_000


def test_channel_cap(monkeypatch):
    monkeypatch.delenv("NCCL_MAX_NCHANNELS", raising=False)
    monkeypatch.setenv("APEX_DDP_CHANNELS", "16")
    preflight.apply_channel_cap()
    assert os.environ["NCCL_MAX_NCHANNELS"] == "16"
    assert preflight.rccl_env()["APEX_DDP_CHANNELS"] == "16"
