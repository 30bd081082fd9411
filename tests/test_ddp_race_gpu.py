"""Race screen for apex DDP on GPU streams (reference
tests/distributed/ddp_race_condition_test.py): the bucket all-reduces run on the reduction
streams of several RCCL communicators (one-rank group with ``single_rank_collectives``), while
the producers of the gradients are delayed by random device sleeps injected into the backward.
Every iteration the gradients read on the default stream right after ``backward()`` (no host
sync in between) must equal their closed form — a collective that started before its bucket was
complete, or a consumer that did not wait for the reduction stream, shows up as a stale value.
Both gradient paths are covered: autograd-produced (copied into the buckets) and fused producers
writing straight into the bucket slots (apex.parallel.grad_target)."""
import random
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


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


class _Delay(torch.autograd.Function):
    """Identity whose backward first spins the GPU for a random time (perturbs the order in which
    gradients and their buckets become ready relative to the reduction streams)."""

    @staticmethod
    def forward(ctx, x, cycles):
        ctx.cycles = cycles
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        torch.cuda._sleep(ctx.cycles)
        return g, None


class _Closed(torch.nn.Module):
    """loss = sum_i <w_i, x_i> * c_i  ->  dL/dw_i = c_i x_i exactly (fp32)."""

    def __init__(self, n, dim):
        super().__init__()
        self.ws = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(dim)) for _ in range(n)])

    def forward(self, xs, cs, rng):
        out = 0.0
        for w, x, c in zip(self.ws, xs, cs):
            out = out + _Delay.apply(w, rng.randint(0, 200000)).mul(x).sum() * c
        return out


@pytest.mark.parametrize("opts", [dict(num_allreduce_streams=3), dict(num_allreduce_streams=2,
                                                                     allreduce_always_fp32=True),
                                  dict(delay_allreduce=True)])
def test_closed_form_gradients_under_random_producer_delays(rccl_one_rank, opts):
    from apex.parallel import DistributedDataParallel as DDP

    n, dim = 24, 4099  # odd sizes: buckets straddle parameters
    net = _Closed(n, dim).cuda()
    model = DDP(net, message_size=3 * dim, **opts)
    model.single_rank_collectives = True
    rng = random.Random(0)
    for it in range(8):
        xs = [torch.full((dim,), float(i + 1 + it), device="cuda") for i in range(n)]
        cs = [float(rng.choice([1, 2, 3])) for _ in range(n)]
        for p in net.parameters():
            p.grad = None
        model(xs, cs, rng).backward()
        got = [p.grad.clone() for p in net.parameters()]  # default stream, no host sync first
        for i, g in enumerate(got):
            assert torch.equal(g, torch.full_like(g, cs[i] * (i + 1 + it))), (it, i)


def test_fused_slot_writes_under_random_delays(rccl_one_rank):
    """Fused dense layers (bf16) write their weight gradients straight into the bucket slots while
    other layers' producers are delayed; every step's gradients equal a DDP-free twin's."""
    from apex.ops import fused as fops
    from apex.optimizers import FusedSGD
    from apex.parallel import DistributedDataParallel as DDP

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.l = torch.nn.ModuleList([torch.nn.Linear(256, 256) for _ in range(6)])

        def forward(self, x, rng=None):
            for m in self.l:
                if rng is not None:
                    x = _Delay.apply(x, rng.randint(0, 300000))
                x = fops.fused_dense(x, m.weight, m.bias).relu()
            return x.float().square().mean()

    torch.manual_seed(0)
    net = Net().cuda().bfloat16()
    twin = Net().cuda().bfloat16()
    twin.load_state_dict(net.state_dict())
    model = DDP(net, message_size=70000, num_allreduce_streams=3)
    model.single_rank_collectives = True
    opt = FusedSGD(net.parameters(), lr=0.0)
    rng = random.Random(1)
    for it in range(6):
        x = torch.randn(512, 256, device="cuda").bfloat16()
        opt.zero_grad()
        model(x, rng).backward()
        got = [p.grad.clone() for p in net.parameters()]
        twin.zero_grad(set_to_none=True)
        twin(x).backward()
        for g, q in zip(got, twin.parameters()):
            torch.testing.assert_close(g.float(), q.grad.float(), rtol=1e-2, atol=1e-3)
        opt.step()
