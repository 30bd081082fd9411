"""apex DDP over RCCL on the GPU with a one-rank process group: the bucket collectives really
run (``single_rank_collectives``), on the reduction streams, through ncclAvg / fp32 staging /
several communicators, and the gradients equal the plain single-GPU gradients. This exercises
the RCCL code path of the 8-GPU scaling run on a one-GPU box."""
import socket

import pytest
import torch
import torch.distributed as dist


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl_one_rank():
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [{}, {"allreduce_always_fp32": True}, {"num_allreduce_streams": 2},
                                  {"delay_allreduce": True}, {"gradient_predivide_factor": 4.0}])
def test_ddp_rccl_single_rank_matches_plain(rccl_one_rank, opts):
    from apex.parallel import DistributedDataParallel as DDP

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64)).cuda().bfloat16()
    ref = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64)).cuda().bfloat16()
    ref.load_state_dict(net.state_dict())
    model = DDP(net, message_size=4096, comm_timing=True, **opts)
    model.single_rank_collectives = True
    assert dist.get_backend() == "nccl" and model.reduction_stream is not None
    for it in range(3):
        x = torch.randn(32, 64, device="cuda", dtype=torch.bfloat16)
        model.zero_grad()
        model(x).float().square().mean().backward()
        ref.zero_grad()
        ref(x).float().square().mean().backward()
        for p, q in zip(net.parameters(), ref.parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-2, atol=1e-3)
    st = model.comm_stats()
    assert st["backend"] == "nccl" and st["num_buckets"] >= 2
    if not opts.get("delay_allreduce"):
        assert len(st["bucket_ready_to_reduced_ms"]) == st["num_buckets"]
        assert st["exposed_comm_samples"] == 2
