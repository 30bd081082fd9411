"""vocab_parallel_cross_entropy at TP = 1 on the GPU runs the fused HIP softmax cross-entropy on the
16-bit logits (no fp32 logits copy, no saved softmax); checked against the fp32 torch composition
(the TP > 1 path) for losses, label smoothing and logits gradients. Megatron's LM-head shapes:
vocab 50304 (and an odd vocab for the scalar tail)."""
import socket

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def tp1():
    from apex.transformer import parallel_state as ps

    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1)
    ps.initialize_model_parallel(1, 1)
    yield
    ps.destroy_model_parallel()
    if own:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("V", [50304, 1001])
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_vocab_parallel_xent_tp1_native(tp1, V, smoothing):
    import apex
    from apex.transformer import tensor_parallel as tp
    from apex.transformer.tensor_parallel.cross_entropy import _VocabParallelCrossEntropy

    apex._ext.require()
    torch.manual_seed(V)
    logits = (torch.randn(2, 512, V, device="cuda") * 3).to(torch.bfloat16)
    target = torch.randint(0, V, (2, 512), device="cuda")
    a = logits.clone().requires_grad_(True)
    loss = tp.vocab_parallel_cross_entropy(a, target, smoothing)
    assert loss.shape == target.shape and loss.dtype == torch.float32
    b = logits.float().requires_grad_(True)
    ref = _VocabParallelCrossEntropy.apply(b, target, smoothing)
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    if smoothing == 0.0:
        plain = F.cross_entropy(logits.float().view(-1, V), target.view(-1), reduction="none").view_as(loss)
        torch.testing.assert_close(loss, plain, rtol=1e-4, atol=1e-4)
    g = torch.rand_like(loss)
    loss.backward(g)
    ref.backward(g)
    assert a.grad.dtype == torch.bfloat16
    torch.testing.assert_close(a.grad.float(), b.grad, rtol=2e-2, atol=2e-4)
