"""amp cast-engine expectations (port of the reference's tests/run_amp/* semantics).

Reference: tests/run_amp/test_basic_casts.py:14-158, test_promotion.py:12-72,
test_rnn.py:10-113 (GPU-only there). Here every expectation runs on CPU with the
engine's cast-device set widened to 'cpu' and the low-precision dtype bf16, and on
the GPU (marker ``gpu``) for both fp16 and bf16.
"""
import functools as ft
import itertools as it

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from apex import amp
from apex.amp import utils as amp_utils

H, B, C, K, T = 32, 8, 8, 3, 6

CASES = [("cpu", torch.bfloat16)]
if torch.cuda.is_available():
    CASES += [pytest.param(("cuda", torch.float16), marks=pytest.mark.gpu, id="cuda-float16"),
              pytest.param(("cuda", torch.bfloat16), marks=pytest.mark.gpu, id="cuda-bfloat16")]


@pytest.fixture(params=CASES, ids=lambda c: f"{c[0]}-{str(c[1])[6:]}" if isinstance(c, tuple) else None)
def env(request):
    dev, low = request.param
    amp_utils.set_cast_devices({dev})
    handle = amp.init(enabled=True, half_dtype=low)
    yield dev, low, handle
    handle._deactivate()
    amp_utils.set_cast_devices({"cuda"})


def _expect(kind, low, typ):
    return {"half": low, "float": torch.float32, "match": typ}[kind]


def run_layer_test(dev, low, fns, kind, shape, test_backward=True):
    for fn, typ in it.product(fns, [low, torch.float32]):
        x = torch.randn(shape, dtype=typ, device=dev).requires_grad_()
        y = fn(x)
        assert y.dtype == _expect(kind, low, typ), (fn, typ, y.dtype)
        if test_backward:
            y.float().sum().backward()
            assert x.grad.dtype == typ


def test_linear_is_half(env):
    dev, low, _ = env
    m = nn.Linear(H, H).to(dev)
    f = ft.partial(F.linear, weight=m.weight, bias=m.bias)
    run_layer_test(dev, low, [m, f], "half", (B, H))


def test_conv2d_is_half(env):
    dev, low, _ = env
    m = nn.Conv2d(C, C, K).to(dev)
    f = ft.partial(F.conv2d, weight=m.weight, bias=m.bias)
    run_layer_test(dev, low, [m, f], "half", (B, C, H, H))


def test_softmax_is_float(env):
    dev, low, _ = env
    run_layer_test(dev, low, [nn.Softmax(dim=1), ft.partial(F.softmax, dim=1)], "float", (B, H))


def test_group_norm_is_float(env):
    dev, low, _ = env
    m = nn.GroupNorm(num_groups=4, num_channels=C).to(dev)
    run_layer_test(dev, low, [m], "float", (B, C, H, H))


def test_mse_loss_is_float(env):
    dev, low, _ = env
    target = torch.randn(B, H, device=dev)
    mod = nn.MSELoss()
    run_layer_test(dev, low, [lambda x: mod(x, target)], "float", (B, H))


def test_relu_is_match(env):
    dev, low, _ = env
    run_layer_test(dev, low, [nn.ReLU(), F.relu], "match", (B, H))


def test_batch_norm_is_match(env):
    dev, low, _ = env
    m = nn.BatchNorm2d(num_features=C).to(dev)
    run_layer_test(dev, low, [m], "match", (B, C, H, H))
    m.eval()
    f = ft.partial(F.batch_norm, running_mean=m.running_mean, running_var=m.running_var,
                   weight=m.weight, bias=m.bias, training=False)
    run_layer_test(dev, low, [m, f], "match", (B, C, H, H), test_backward=False)


def test_bce_banned_then_allowed(env):
    dev, low, handle = env
    x = torch.rand(B, H, device=dev).to(low)
    y = torch.rand(B, H, device=dev).to(low)
    with pytest.raises(NotImplementedError):
        F.binary_cross_entropy(x, y)
    handle._deactivate()
    h2 = amp.init(enabled=True, allow_banned=True, half_dtype=low)
    try:
        out = F.binary_cross_entropy(torch.rand(B, H, device=dev).to(low), y)
        assert out.dtype == torch.float32
    finally:
        h2._deactivate()


def test_tensor_methods(env):
    dev, low, _ = env
    a = torch.randn(B, H, device=dev)
    b = torch.randn(H, H, device=dev)
    assert a.matmul(b).dtype == low
    assert (a @ b).dtype == low
    assert a.pow(2).dtype == torch.float32
    assert (a.to(low) ** 2).dtype == torch.float32
    assert a.to(low).sum().dtype == torch.float32
    assert a.to(low).cpu().dtype == torch.float32


def test_promotion(env):
    dev, low, _ = env
    x = torch.randn(B, H, device=dev)
    y = torch.randn(B, H, device=dev).to(low)
    for fn in (torch.add, torch.mul, torch.div, lambda a, b: a + b, lambda a, b: a * b,
               lambda a, b: a - b, lambda a, b: a / b):
        assert fn(x, y).dtype == torch.float32
        assert fn(y, y).dtype == low
        assert fn(x, x).dtype == torch.float32
    assert torch.cat([x, y]).dtype == torch.float32
    assert torch.stack([y, y]).dtype == low


def test_inplace_exp_is_error_for_low(env):
    dev, low, _ = env
    x = torch.randn(B, H, device=dev).to(low)
    with pytest.raises(NotImplementedError):
        x.exp_()
    xf = torch.randn(B, H, device=dev)
    xf.exp_()


def test_inplace_add_matches_self(env):
    dev, low, _ = env
    x = torch.zeros(B, H, device=dev).to(low)
    y = torch.ones(B, H, device=dev)
    x.add_(y)
    assert x.dtype == low
    assert float(x[0, 0]) == 1.0


@pytest.mark.parametrize("cell", [nn.LSTMCell, nn.GRUCell, nn.RNNCell])
def test_rnn_cells_are_half(env, cell):
    dev, low, _ = env
    m = cell(H, H).to(dev)
    for typ in (low, torch.float32):
        x = torch.randn(B, H, device=dev, dtype=typ).requires_grad_()
        out = m(x)
        y = out[0] if isinstance(out, tuple) else out
        assert y.dtype == low
        y.float().sum().backward()
        assert x.grad.dtype == typ


@pytest.mark.parametrize("rnn", [nn.LSTM, nn.GRU, nn.RNN])
@pytest.mark.parametrize("layers,bidir", [(1, False), (2, True)])
def test_rnns_are_half(env, rnn, layers, bidir):
    dev, low, _ = env
    m = rnn(H, H, num_layers=layers, bidirectional=bidir).to(dev)
    for typ in (low, torch.float32):
        x = torch.randn(T, B, H, device=dev, dtype=typ).requires_grad_()
        y, _ = m(x)
        assert y.dtype == low
        y.float().sum().backward()
        assert x.grad.dtype == typ
        assert m.weight_ih_l0.grad is not None and m.weight_ih_l0.grad.dtype == torch.float32


def test_disabled_is_noop():
    h = amp.init(enabled=False)
    assert not h.is_active()
    x = torch.randn(B, H)
    assert F.linear(x, torch.randn(H, H)).dtype == torch.float32


def test_user_registry_and_decorators():
    amp_utils.set_cast_devices({"cpu"})
    import types

    mod = types.SimpleNamespace(f=lambda a: a, g=lambda a: a)
    amp.register_half_function(mod, "f")
    amp.register_float_function(mod, "g")
    h = amp.init(enabled=True, half_dtype=torch.bfloat16)
    try:
        assert mod.f(torch.randn(3)).dtype == torch.bfloat16
        assert mod.g(torch.randn(3).bfloat16()).dtype == torch.float32

        @amp.half_function
        def hf(a):
            return a

        @amp.float_function
        def ff(a):
            return a

        assert hf(torch.randn(3)).dtype == torch.bfloat16
        assert ff(torch.randn(3).bfloat16()).dtype == torch.float32
    finally:
        h._deactivate()
        amp_utils.set_cast_devices({"cuda"})
    with pytest.raises(ValueError):
        amp.register_half_function(mod, "nope")


def test_handle_scale_loss_skips_on_overflow():
    amp_utils.set_cast_devices({"cpu"})
    h = amp.init(enabled=True, half_dtype=torch.bfloat16)
    try:
        p = nn.Parameter(torch.ones(4))
        opt = torch.optim.SGD([p], lr=1.0)
        loss = (p * float("inf")).sum()
        with h.scale_loss(loss, opt) as sl:
            sl.backward()
        before = h._default_scaler.loss_scale()
        opt.step()  # must be skipped
        assert torch.equal(p.detach(), torch.ones(4))
        assert before == 2.0 ** 15
        loss = (p * 2).sum()
        opt.zero_grad()
        with h.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        assert torch.allclose(p.detach(), torch.full((4,), -1.0))
    finally:
        h._deactivate()
        amp_utils.set_cast_devices({"cuda"})
