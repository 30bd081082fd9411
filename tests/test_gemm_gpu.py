"""Hand-written MFMA GEMM (csrc/gemm.hip) and its fused epilogues vs fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _C():
    import apex._ext as e

    return e.require()


def _ref_mm(a, b):
    return a.float().reshape(-1, a.shape[-1]) @ b.float().t()


def _close(x, ref, tol):
    err = float((x.float() - ref).abs().max())
    scale = float(ref.abs().max()) + 1e-6
    assert err <= tol * scale, (err, scale)


SHAPES = [(512, 256, 64), (256, 512, 128), (300, 200, 128), (1000, 1600, 1600), (4096, 1024, 1024),
          (77, 8, 64), (2048, 3072, 1024)]


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", SHAPES + [(512, 512, 64), (512, 512, 128), (768, 256, 192), (512, 384, 32 * 3 * 64)])
def test_gemm_plain(dt, M, N, K):
    C = _C()
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV).to(dt)
    b = torch.randn(N, K, device=DEV).to(dt)
    c, _ = C.gemm(a, b, C.EPI_NONE)
    _close(c, _ref_mm(a, b), 1e-2)


def test_gemm_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C-write (cdna guide §3)."""
    C = _C()
    n = 256
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    b = (torch.arange(n * n, device=DEV).reshape(n, n) % 97).to(torch.bfloat16)
    c, _ = C.gemm(a, b, C.EPI_NONE)
    torch.testing.assert_close(c.float(), b.float().t(), rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (4096, 1024, 1024), (300, 200, 128)])
def test_gemm_bias(M, N, K):
    C = _C()
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    c, _ = C.gemm(a, b, C.EPI_BIAS, bias)
    _close(c, _ref_mm(a, b) + bias.float(), 1e-2)


@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (4096, 4096, 1024), (300, 200, 128)])
def test_gemm_bias_gelu(M, N, K):
    C = _C()
    a = (torch.randn(M, K, device=DEV) / K ** 0.5).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    y, h = C.gemm(a, b, C.EPI_BIAS_GELU, bias)
    href = _ref_mm(a, b) + bias.float()
    _close(h, href, 1e-2)
    _close(y, F.gelu(href), 1.5e-2)


@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (4096, 4096, 1024), (300, 200, 128)])
def test_gemm_dgelu_bias_grad(M, N, K):
    C = _C()
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    h = torch.randn(M, N, device=DEV).bfloat16()
    dh, db = C.gemm(a, b, C.EPI_DGELU, None, h, torch.float32)
    hr = h.float().requires_grad_(True)
    F.gelu(hr).backward(_ref_mm(a, b))
    _close(dh, hr.grad, 1.5e-2)
    torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-4, atol=1e-3)


def _gelu_grad_ref(h, tanh):
    hr = h.float().requires_grad_(True)
    F.gelu(hr, approximate="tanh" if tanh else "none").backward(torch.ones_like(hr))
    return hr.grad


@pytest.mark.parametrize("tanh", [False, True])
@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (4096, 4096, 1024), (300, 200, 128)])
def test_gemm_bias_gelu_stores_derivative(M, N, K, tanh):
    """EPI_BIAS_GELU_D: y = gelu(h), aux = gelu'(h) (fp32 reference). h = the GEMM output rounded
    to 16 bits (the epilogue's LDS transposition) + bias, NOT rounded again: no pre-activation is
    stored, so the kernel evaluates gelu / gelu' on the fp32 sum."""
    C = _C()
    a = (torch.randn(M, K, device=DEV) / K ** 0.5).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    y, gd = C.gemm(a, b, C.EPI_BIAS_GELU_TANH_D if tanh else C.EPI_BIAS_GELU_D, bias)
    href = _ref_mm(a, b).bfloat16().float() + bias.float()
    _close(y, F.gelu(href, approximate="tanh" if tanh else "none"), 1.5e-2)
    _close(gd, _gelu_grad_ref(href, tanh), 1.5e-2)


@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (4096, 4096, 1024), (300, 200, 128)])
def test_gemm_mul_bias_grad(M, N, K):
    """EPI_MUL: dh = (A B^T) * G and the bias gradient from the stored dh."""
    C = _C()
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    g = torch.rand(M, N, device=DEV).bfloat16()
    dh, db = C.gemm(a, b, C.EPI_MUL, None, g, torch.float32)
    _close(dh, _ref_mm(a, b) * g.float(), 1.5e-2)
    torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-4, atol=1e-3)


def test_mlp_stored_derivative_matches_reference():
    """apex.ops.blocks.mlp (GELU-derivative-storing forward + multiply backward) vs fp32 autograd."""
    from apex.ops import blocks

    torch.manual_seed(0)
    x = (torch.randn(512, 256, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    w1 = (torch.randn(1024, 256, device=DEV) / 16).bfloat16().requires_grad_(True)
    b1 = (torch.randn(1024, device=DEV) * 0.1).bfloat16().requires_grad_(True)
    w2 = (torch.randn(256, 1024, device=DEV) / 32).bfloat16().requires_grad_(True)
    for act in (0, 1):
        out = blocks.mlp(x, w1, b1, w2, act)
        go = torch.randn_like(out)
        grads = torch.autograd.grad(out, (x, w1, b1, w2), go)
        xs = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2)]
        ref = F.linear(F.gelu(F.linear(xs[0], xs[1], xs[2]), approximate="tanh" if act else "none"), xs[3])
        rgrads = torch.autograd.grad(ref, xs, go.float())
        _close(out, ref.detach(), 2e-2)
        for g_, r_ in zip(grads, rgrads):
            _close(g_, r_, 3e-2)


@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (4096, 1024, 4096)])
def test_gemm_resid(M, N, K):
    C = _C()
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    c, _ = C.gemm(a, b, C.EPI_RESID, None, r)
    _close(c, _ref_mm(a, b) + r.float(), 1e-2)


def test_gemm_strided_and_3d():
    C = _C()
    base = torch.randn(512, 3 * 1024, device=DEV).bfloat16()
    a = base[:, 1024:2048]  # row stride 3072
    b = torch.randn(256, 1024, device=DEV).bfloat16()
    c, _ = C.gemm(a, b, C.EPI_NONE)
    _close(c, _ref_mm(a, b), 1e-2)
    a3 = torch.randn(4, 128, 1024, device=DEV).bfloat16()
    c3, _ = C.gemm(a3, b, C.EPI_NONE)
    assert c3.shape == (4, 128, 256)
    _close(c3.reshape(-1, 256), _ref_mm(a3, b), 1e-2)


def test_transpose():
    C = _C()
    for r, c in [(1024, 4096), (1000, 33), (1, 64)]:
        x = torch.randn(r, c, device=DEV).bfloat16()
        torch.testing.assert_close(C.transpose(x), x.t().contiguous(), rtol=0, atol=0)


def test_gemm_supported_rejects():
    C = _C()
    a = torch.randn(64, 128, device=DEV).bfloat16()
    assert not C.gemm_supported(a, torch.randn(12, 128, device=DEV).bfloat16())  # N % 8
    assert not C.gemm_supported(torch.randn(64, 96, device=DEV).bfloat16(),
                                torch.randn(16, 96, device=DEV).bfloat16())  # K % 64
    assert not C.gemm_supported(a.float(), torch.randn(16, 128, device=DEV))  # fp32
    assert C.gemm_supported(a, torch.randn(16, 128, device=DEV).bfloat16())


@pytest.mark.parametrize("R,P,Q,splits", [(256, 256, 256, 1), (1024, 256, 512, 2), (2048, 512, 256, 4),
                                          (8192, 1024, 1024, 8), (64, 256, 256, 1), (576, 256, 512, 3),
                                          # partial 256-tiles (GPT-2's 1600 / 4800): clamped staging
                                          (1024, 1600, 480, 2), (512, 200, 264, 1), (2048, 4800, 1600, 4),
                                          (128, 8, 1608, 1),
                                          # slice counts that do not divide the K-tiles (slices of 2-3,
                                          # 6-7, 9-10 K-tiles; one K-tile each)
                                          (448, 256, 256, 3), (1280, 512, 256, 3), (3072, 768, 1024, 5),
                                          (320, 256, 256, 5)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gemm_tt_weight_grad(R, P, Q, splits, dt):
    """dW = dY^T X through the transposed-read (ds_read_b64_tr_b16) main loop, split-K slabs (the
    slices: whole K-tiles, [s T / S, (s + 1) T / S) of the T K-tiles)."""
    C = _C()
    torch.manual_seed(R + P + Q)
    dy = torch.randn(R, P, device=DEV).to(dt)
    x = torch.randn(R, Q, device=DEV).to(dt)
    assert C.gemm_tt_supported(dy, x, splits)
    ref = dy.float().t() @ x.float()
    out = C.gemm_tt(dy, x, splits, dt)
    assert out.shape == (P, Q) and out.dtype == dt
    _close(out, ref, 1e-2)
    out32 = C.gemm_tt(dy, x, splits, torch.float32)
    _close(out32, ref, 1e-4)


@pytest.mark.parametrize("N,K", [(1024, 4096), (4096, 1024)])
def test_wgrad_tt_policy_writes_slot(N, K, monkeypatch):
    """apex.ops.fused._wgrad on the FFN weight shapes (>= 64 output tiles, >= 16k tokens): the
    transposed-read kernel in 4 slices, the split-K reduction writing straight into a gradient
    slot (a view inside a larger bucket), equal to the library path and the fp32 reference."""
    from apex.ops import fused

    torch.manual_seed(N)
    M = 16384
    dy = torch.randn(M, N, device=DEV).bfloat16()
    x = torch.randn(M, K, device=DEV).bfloat16()
    monkeypatch.setattr(fused, "_WGRAD_TT", "auto")
    assert fused._wgrad_tt_splits(M, N, K) == 4
    bucket = torch.full((N * K + 64,), 7.0, device=DEV, dtype=torch.bfloat16)
    slot = bucket[32:32 + N * K].view(N, K)
    r = fused._wgrad(dy, x, out=slot)
    assert r.data_ptr() == slot.data_ptr()
    assert (bucket[:32] == 7).all() and (bucket[32 + N * K:] == 7).all()
    ref = dy.float().t() @ x.float()
    _close(slot, ref, 1e-2)
    monkeypatch.setattr(fused, "_WGRAD_TT", "0")
    lib = fused._wgrad(dy, x)
    _close(slot, lib.float(), 1e-2)


def test_gemm_tt_acc_partial_tiles():
    """main_grad accumulation (EPI_F32_ACC read-modify-write) on a partial-tile shape: only [P, Q] is
    touched (a guard band after the accumulator stays), the sum adds onto the previous contents."""
    C = _C()
    torch.manual_seed(3)
    R, P, Q = 1024, 1600, 488
    dy = torch.randn(R, P, device=DEV).bfloat16()
    x = torch.randn(R, Q, device=DEV).bfloat16()
    buf = torch.full((P * Q + 256,), 5.0, device=DEV)
    mg = buf[:P * Q].view(P, Q)
    mg.copy_(torch.randn(P, Q, device=DEV))
    before = mg.clone()
    C.gemm_tt_acc(dy, x, mg)
    ref = before + dy.float().t() @ x.float()
    _close(mg, ref, 1e-4)
    assert (buf[P * Q:] == 5.0).all()


def test_gemm_tt_asymmetric_identity():
    C = _C()
    n = 256
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)  # [R=n, P=n]
    b = (torch.arange(n * n, device=DEV).reshape(n, n) % 89).to(torch.bfloat16)  # [R, Q]
    torch.testing.assert_close(C.gemm_tt(a, b, 1, torch.bfloat16).float(), b.float(), rtol=0, atol=0)


@pytest.mark.parametrize("M,N,K", [(1000, 1600, 1600), (2048, 4096, 1024)])
def test_gemm_tanh_gelu_epilogues(M, N, K):
    C = _C()
    a = (torch.randn(M, K, device=DEV) / K ** 0.5).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    y, h = C.gemm(a, b, C.EPI_BIAS_GELU_TANH, bias)
    href = _ref_mm(a, b) + bias.float()
    _close(h, href, 1e-2)
    _close(y, F.gelu(href, approximate="tanh"), 1.5e-2)
    hh = torch.randn(M, N, device=DEV).bfloat16()
    bt = (torch.randn(N, K, device=DEV) / K ** 0.5).bfloat16()
    dh, db = C.gemm(a, bt, C.EPI_DGELU_TANH, None, hh, torch.float32)
    hr = hh.float().requires_grad_(True)
    F.gelu(hr, approximate="tanh").backward(_ref_mm(a, bt))
    _close(dh, hr.grad, 1.5e-2)
    torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("act", [0, 1])
def test_mlp_block_matches_composition(act):
    """apex.ops.blocks.mlp (fused epilogues) vs F.linear / F.gelu in fp32 on the same bf16 inputs."""
    from apex.ops import blocks

    torch.manual_seed(act)
    x = torch.randn(4, 256, 512, device=DEV).bfloat16().requires_grad_(True)
    w1 = (torch.randn(2048, 512, device=DEV) * 0.03).bfloat16().requires_grad_(True)
    b1 = (torch.randn(2048, device=DEV) * 0.1).bfloat16().requires_grad_(True)
    w2 = (torch.randn(512, 2048, device=DEV) * 0.03).bfloat16().requires_grad_(True)
    y = blocks.mlp(x, w1, b1, w2, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    ref = [t.detach().float().requires_grad_(True) for t in (x, w1, b1, w2)]
    yr = F.linear(F.gelu(F.linear(ref[0], ref[1], ref[2]), approximate="tanh" if act else "none"), ref[3])
    yr.backward(dy.float())
    _close(y, yr, 2e-2)
    for got, r in zip((x, w1, b1, w2), ref):
        _close(got.grad, r.grad, 3e-2)


def _f8_codes(x, dt):
    s = (torch.finfo(dt).max / x.abs().max().float()).reshape(1)
    return (x.float() * s).to(dt).view(torch.uint8), (1.0 / s).float()


@pytest.mark.parametrize("R,P,Q,splits", [(128, 256, 256, 1), (1024, 256, 512, 2), (2048, 512, 768, 4),
                                          (8192, 1024, 1024, 8), (384, 256, 256, 3),
                                          # partial 256-tiles: clamped staging, bounds-checked slab stores
                                          (1024, 1600, 480, 2), (256, 16, 272, 1), (512, 4800, 1600, 2),
                                          # uneven slices (1 and 2; 2 and 3 128-row K-tiles)
                                          (384, 256, 256, 2), (640, 512, 256, 2)])
@pytest.mark.parametrize("fmt_a", [1, 0])
def test_gemm_tt_f8_weight_grad(R, P, Q, splits, fmt_a):
    """fp8 dW = alpha dY8^T X8 through the ds_read_b64_tr_b8 transposed-read main loop: against the
    fp32 product of the dequantised codes (the kernel's exact inputs), asymmetric random data."""
    C = _C()
    torch.manual_seed(R + P + Q + fmt_a)
    dta = torch.float8_e5m2 if fmt_a == 1 else torch.float8_e4m3fn
    dy = torch.randn(R, P, device=DEV) * torch.linspace(0.5, 2.0, P, device=DEV)
    x = torch.randn(R, Q, device=DEV) + torch.linspace(-1.0, 1.0, R, device=DEV)[:, None]
    a8, sa = _f8_codes(dy, dta)
    b8, sb = _f8_codes(x, torch.float8_e4m3fn)
    assert C.gemm_tt_f8_supported(a8, b8, splits)
    ref = (a8.view(dta).float() * sa).t() @ (b8.view(torch.float8_e4m3fn).float() * sb)
    out32 = C.gemm_tt_f8(a8, b8, sa, sb, fmt_a, 0, splits, torch.float32)
    assert out32.shape == (P, Q)
    _close(out32, ref, 1e-4)
    out = C.gemm_tt_f8(a8, b8, sa, sb, fmt_a, 0, splits, torch.bfloat16)
    assert out.dtype == torch.bfloat16
    _close(out, ref, 1e-2)


def test_gemm_tt_f8_identity_rows():
    """A = one-hot K-rows (dY8[r, p] = 1 iff p == r % P): dW[p, :] is the sum of X8's rows r = p mod P,
    which pins the transposed-read byte gather (a wrong K-row / column pairing shows up as a
    permutation, which a symmetric check could miss)."""
    C = _C()
    R, P, Q = 512, 256, 272
    a = torch.zeros(R, P, device=DEV)
    a[torch.arange(R), torch.arange(R) % P] = 1.0
    x = torch.arange(R * Q, device=DEV, dtype=torch.float32).view(R, Q) % 13 - 6
    a8 = a.to(torch.float8_e4m3fn).view(torch.uint8)
    b8 = x.to(torch.float8_e4m3fn).view(torch.uint8)
    one = torch.ones(1, device=DEV)
    out = C.gemm_tt_f8(a8, b8, one, one, 0, 0, 1, torch.float32)
    ref = x.view(R // P, P, Q).sum(0)
    assert torch.equal(out, ref)


def test_gemm_tt_f8_supported_rejects():
    C = _C()
    a = torch.zeros(256, 256, device=DEV, dtype=torch.uint8)
    assert C.gemm_tt_f8_supported(a, a, 2)
    assert not C.gemm_tt_f8_supported(a, a, 3)  # 256 rows = two 128-row K-tiles: at most 2 slices
    assert not C.gemm_tt_f8_supported(a[:, :248].contiguous(), a, 1)  # P % 16
    assert not C.gemm_tt_f8_supported(a.bfloat16(), a.bfloat16(), 1)
