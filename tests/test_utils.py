"""apex.utils: metrics (K-10 reduce_tensor / reduce_scalars over gloo), JSONL logger, profiler
ranges, the prefetcher (CPU path) and the K-09 fused normalize kernel + SyncBN on torch
channels_last tensors (GPU)."""
import json

import pytest
import torch
import torch.distributed as dist

from test_transformer import _spawn


def _reduce(rank, world):
    from apex.utils.metrics import reduce_scalars, reduce_tensor

    t = torch.tensor([float(rank + 1)])
    torch.testing.assert_close(reduce_tensor(t), torch.tensor([(world + 1) / 2]))
    a, b, c = reduce_scalars(rank, torch.tensor(2.0 * rank), 5)
    assert a == pytest.approx((world - 1) / 2) and b == pytest.approx(world - 1) and c == 5


def test_reduce_tensor_gloo():
    _spawn(_reduce, 3)


def test_meter_logger_ranges(tmp_path):
    from apex.utils import AverageMeter, JsonlLogger
    from apex.utils import prof

    m = AverageMeter()
    for v, n in [(1.0, 2), (4.0, 1)]:
        m.update(v, n)
    assert m.avg == pytest.approx(2.0) and m.val == 4.0
    p = tmp_path / "m" / "log.jsonl"
    with JsonlLogger(str(p), rank=0) as lg:
        lg.log(step=1, loss=torch.tensor(0.5))
        lg.log(step=2, loss=0.25)
    rows = [json.loads(l) for l in p.read_text().splitlines()]
    assert [r["step"] for r in rows] == [1, 2] and rows[0]["loss"] == 0.5
    prof.enable(True)

    @prof.annotate("f")
    def f(x):
        with prof.range("inner"):
            return x + 1

    assert f(1) == 2
    prof.enable(False)


def test_prefetcher_cpu():
    from apex.utils.prefetch import DataPrefetcher, normalize_images

    x = torch.randint(0, 256, (2, 4, 4, 3), dtype=torch.uint8)
    y = normalize_images(x)
    ref = (x.float().permute(0, 3, 1, 2) - torch.tensor([123.675, 116.28, 103.53]).view(1, 3, 1, 1)) / \
        torch.tensor([58.395, 57.12, 57.375]).view(1, 3, 1, 1)
    torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5)
    loader = [(x, torch.tensor([0, 1])), (x, torch.tensor([1, 0]))]
    out = list(DataPrefetcher(loader, device="cpu"))
    assert len(out) == 2 and out[1][1].tolist() == [1, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("mode", ["nhwc_nchw", "nhwc_cl", "nchw"])
@pytest.mark.parametrize("shape", [(3, 224, 224, 3), (2, 7, 9, 3), (2, 8, 8, 1)])
def test_input_normalize_kernel(dtype, mode, shape):
    import apex
    from apex.utils.prefetch import normalize_images

    apex._ext.require()
    torch.manual_seed(0)
    B, H, W, C = shape
    if mode == "nhwc_nchw" and (H * W) % 8:
        pytest.skip("transposing kernel needs H*W % 8 == 0")
    mean, std = [100.0, 110.0, 120.0][:C], [50.0, 60.0, 70.0][:C]
    if mode == "nchw":
        x = torch.randint(0, 256, (B, C, H, W), dtype=torch.uint8, device="cuda")
        ref = (x.float() - torch.tensor(mean, device="cuda").view(1, -1, 1, 1)) / \
            torch.tensor(std, device="cuda").view(1, -1, 1, 1)
        y = normalize_images(x, mean, std, nhwc=False, dtype=dtype)
    else:
        x = torch.randint(0, 256, (B, H, W, C), dtype=torch.uint8, device="cuda")
        ref = (x.float().permute(0, 3, 1, 2) - torch.tensor(mean, device="cuda").view(1, -1, 1, 1)) / \
            torch.tensor(std, device="cuda").view(1, -1, 1, 1)
        y = normalize_images(x, mean, std, nhwc=True, channels_last=(mode == "nhwc_cl"), dtype=dtype)
        if mode == "nhwc_cl":
            assert y.is_contiguous(memory_format=torch.channels_last)
    assert y.dtype == dtype and y.shape == (B, C, H, W)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)


@pytest.mark.gpu
def test_syncbn_channels_last_memory_format():
    from apex.parallel import SyncBatchNorm

    torch.manual_seed(0)
    C = 64
    ref = torch.nn.BatchNorm2d(C).cuda()
    sbn = SyncBatchNorm(C).cuda()
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.uniform_(-0.5, 0.5)
    sbn.load_state_dict(ref.state_dict())
    x = (torch.randn(8, C, 14, 14, device="cuda") * 2 + 1).contiguous(memory_format=torch.channels_last)
    xr = x.detach().clone().requires_grad_(True)
    x.requires_grad_(True)
    y, yr = sbn(x), ref(xr)
    assert y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y, yr, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(sbn.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(sbn.running_var, ref.running_var, rtol=1e-4, atol=1e-5)
