"""DDP fp32_main_grad on the GPU (one-rank RCCL group): 8 micro-batches through the fused dense
op, whose weight-gradient GEMM accumulates its fp32 result straight into ``main_grad``
(split-K fp32 slabs summed into the buffer by splitk_reduce(accumulate=True)). main_grad must
match the fp32 sum of the per-micro-batch products dY^T X to fp32 tolerance; the bf16 ``.grad``
accumulation of the same gradients (the pre-r3 Megatron path) must not."""
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


class _Dense(torch.nn.Module):
    def __init__(self, n, k):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.05)

    def forward(self, x):
        from apex.ops.fused import fused_dense

        return fused_dense(x, self.weight, None)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["lib", "tt"])  # hipBLASLt / split-K slabs vs gemm_tt_acc's epilogue
@pytest.mark.parametrize("M", [2048, 16384])  # 16384 tokens: the split-K (several slabs) path
def test_main_grad_accumulates_in_fp32(rccl_one_rank, M, path, monkeypatch):
    from apex.ops import fused
    from apex.parallel import DistributedDataParallel as DDP

    monkeypatch.setattr(fused, "_MAIN_GRAD_GEMM", path)
    torch.manual_seed(0)
    N, K, mbs = 256, 512, 8
    net = _Dense(N, K)
    model = DDP(net, message_size=1 << 20, fp32_main_grad=True)
    model.single_rank_collectives = True
    xs = [torch.randn(M, K, device="cuda", dtype=torch.bfloat16) for _ in range(mbs)]
    cs = [torch.randn(M, N, device="cuda", dtype=torch.bfloat16) for _ in range(mbs)]
    for i, (x, c) in enumerate(zip(xs, cs)):
        ctx = model.no_sync() if i < mbs - 1 else torch.enable_grad()
        with ctx:
            (model(x) * c).float().sum().backward()  # dY = c exactly
        assert net.weight.grad is None
    torch.cuda.synchronize()
    ref = sum(c.float().t() @ x.float() for x, c in zip(xs, cs))
    got = net.weight.main_grad
    scale = float(ref.abs().max())
    err32 = float((got - ref).abs().max()) / scale
    # the bf16 path: each micro-batch's dW rounded to bf16 and summed in bf16
    acc16 = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    for x, c in zip(xs, cs):
        acc16 += (c.float().t() @ x.float()).to(torch.bfloat16)
    err16 = float((acc16.float() - ref).abs().max()) / scale
    assert err32 < 1e-5, err32
    assert err16 > 20 * err32, (err16, err32)


@pytest.mark.gpu
@pytest.mark.parametrize("R,P,Q", [(2048, 256, 512), (8192, 768, 1024), (1024, 2560, 512)])
def test_gemm_tt_acc_matches_fp32(R, P, Q):
    """out[P, Q] += a^T b by the transposed-read MFMA kernel's fp32 read-modify-write epilogue."""
    from apex import _ext

    C = _ext.require()
    torch.manual_seed(1)
    a = torch.randn(R, P, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(R, Q, device="cuda", dtype=torch.bfloat16)
    out = torch.randn(P, Q, device="cuda", dtype=torch.float32) * 10
    ref = out + a.float().t() @ b.float()
    C.gemm_tt_acc(a, b, out)
    err = float((out - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err
