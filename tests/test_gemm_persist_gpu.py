"""The persistent MFMA GEMM (csrc/gemm.hip gemm_persist_kernel) under kernel-level test.

The launcher takes the persistent kernel for every full-tile 16-bit NT product with more 256x256
tiles than CUs (BERT-Large b768: every own-kernel GEMM of the step). Its epilogue runs in two
64-row halves with the next tile's first K-tile in flight and counted vmcnt waits, so it gets its
own shapes here (>256 full tiles, several tiles per workgroup) for EVERY epilogue it instantiates,
in bf16 and fp16:

* against the fp32 PyTorch reference of the same op (the tolerances of tests/test_gemm_gpu.py);
* bitwise against the one-tile-per-workgroup kernel (C.set_gemm_persist(0, 0) forces it, in the
  same process): the two kernels share the main loop and the epilogue math, so any difference is
  a staging / wait / tile-walk bug of the persistent path;
* a kernel-trace check that the persistent kernel is really the one that ran.

The fp8 persistent kernel (off by default, APEX_GEMM_PERSIST_F8) is covered by the same bitwise
comparison through C.set_gemm_persist(1, 1).
"""
import contextlib

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _C():
    import apex._ext as e

    return e.require()


@contextlib.contextmanager
def _persist(which, v):
    C = _C()
    prev = C.set_gemm_persist(which, v)
    try:
        yield
    finally:
        C.set_gemm_persist(which, prev)


def _ref_mm(a, b):
    return a.float() @ b.float().t()


def _close(x, ref, tol):
    err = float((x.float() - ref).abs().max())
    scale = float(ref.abs().max()) + 1e-6
    assert err <= tol * scale, (err, scale)


def _cus():
    return torch.cuda.get_device_properties(0).multi_processor_count


# (M, N, K): tiles = M/256 * N/256, all > 256 (the CU count) so the launcher takes the persistent
# kernel; the first is 288 tiles (just over one round), the second 768 (three tiles per workgroup,
# BERT's attention-out / residual width and K), the third 297 tiles with K = one K-tile (the
# prologue's nt == 1 branch and the stores-only counted wait); K = 128 and 192 (two and three K-tiles)
# cover the later tiles' K-tile 0/1 pair whose A(1) / B(1) the previous epilogue issued between its
# halves' stores (the nt == 2 waits, and an odd tail after that pair)
SHAPES = [(4608, 4096, 256), (49152, 1024, 1024), (8448, 2304, 64), (4608, 4096, 128), (8448, 2304, 192)]


def _tiles(M, N):
    return (M // 256) * (N // 256)


EPIS = ["NONE", "BIAS", "BIAS_GELU", "BIAS_GELU_TANH", "BIAS_GELU_D", "BIAS_GELU_TANH_D", "RESID", "MUL", "DGELU",
        "DGELU_TANH"]


def _inputs(M, N, K, dt, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    a = (torch.randn(M, K, device=DEV, generator=g) / K ** 0.5).to(dt)
    b = torch.randn(N, K, device=DEV, generator=g).to(dt)
    bias = (torch.randn(N, device=DEV, generator=g) * 0.5).to(dt)
    aux = torch.randn(M, N, device=DEV, generator=g).to(dt)
    return a, b, bias, aux


def _run(C, epi, a, b, bias, aux):
    e = getattr(C, "EPI_" + epi)
    if epi in ("NONE",):
        return C.gemm(a, b, e)
    if epi in ("BIAS", "BIAS_GELU", "BIAS_GELU_TANH", "BIAS_GELU_D", "BIAS_GELU_TANH_D"):
        return C.gemm(a, b, e, bias)
    if epi == "RESID":
        return C.gemm(a, b, e, None, aux)
    return C.gemm(a, b, e, None, aux, torch.float32)  # MUL / DGELU(_TANH): + bias-grad column sums


def _check_ref(epi, out, a, b, bias, aux):
    acc = _ref_mm(a, b)
    c, d = out
    if epi == "NONE":
        _close(c, acc, 1e-2)
    elif epi == "BIAS":
        _close(c, acc + bias.float(), 1e-2)
    elif epi in ("BIAS_GELU", "BIAS_GELU_TANH"):
        h = acc + bias.float()
        _close(d, h, 1e-2)
        _close(c, F.gelu(d.float(), approximate="tanh" if epi.endswith("TANH") else "none"), 1.5e-2)
    elif epi in ("BIAS_GELU_D", "BIAS_GELU_TANH_D"):
        tanh = "TANH" in epi
        h = (acc.to(a.dtype).float() + bias.float()).requires_grad_(True)
        y = F.gelu(h, approximate="tanh" if tanh else "none")
        (g,) = torch.autograd.grad(y.sum(), h)
        _close(c, y.detach(), 1.5e-2)
        _close(d, g, 1.5e-2)
    elif epi == "RESID":
        _close(c, acc + aux.float(), 1e-2)
    elif epi == "MUL":
        _close(c, acc * aux.float(), 1.5e-2)
        torch.testing.assert_close(d, c.float().sum(0), rtol=1e-3, atol=1e-2)
    else:  # DGELU(_TANH): dh = acc * gelu'(aux)
        hr = aux.float().requires_grad_(True)
        F.gelu(hr, approximate="tanh" if epi.endswith("TANH") else "none").backward(acc)
        _close(c, hr.grad, 1.5e-2)
        torch.testing.assert_close(d, c.float().sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("epi", EPIS)
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_persistent_gemm_matches_fp32_and_one_tile_kernel(M, N, K, epi, dt):
    C = _C()
    assert _tiles(M, N) > _cus(), "shape must exceed one tile per CU to reach the persistent kernel"
    a, b, bias, aux = _inputs(M, N, K, dt, seed=M + N + K + len(epi))
    with _persist(0, 1):
        got = _run(C, epi, a, b, bias, aux)
    _check_ref(epi, got, a, b, bias, aux)
    with _persist(0, 0):
        ref = _run(C, epi, a, b, bias, aux)
    torch.cuda.synchronize()
    for x, y in zip(got, ref):
        if x is None:
            assert y is None
            continue
        # the bias-grad partials are summed over (tile, wave-row) rows by the same kernel either way
        assert torch.equal(x, y), (epi, float((x.float() - y.float()).abs().max()))


def test_persistent_gemm_output_repeatable():
    """Two launches on the same inputs (a different next-tile prefetch interleaving each time):
    bitwise equal, so no output depends on LDS-DMA timing."""
    C = _C()
    a, b, bias, aux = _inputs(8192, 2304, 512, torch.bfloat16, seed=5)
    with _persist(0, 1):
        r1 = C.gemm(a, b, C.EPI_MUL, None, aux, torch.float32)
        r2 = C.gemm(a, b, C.EPI_MUL, None, aux, torch.float32)
    assert torch.equal(r1[0], r2[0]) and torch.equal(r1[1], r2[1])


def test_persistent_kernel_is_the_one_that_runs():
    """The launcher's switch reaches the persistent kernel (kernel names from the torch profiler's
    device trace) and set_gemm_persist(0, 0) turns it off."""
    from torch.profiler import ProfilerActivity, profile

    C = _C()
    a, b, bias, _ = _inputs(4608, 4096, 256, torch.bfloat16, seed=7)

    def names(v):
        with _persist(0, v):
            C.gemm(a, b, C.EPI_BIAS, bias)
            torch.cuda.synchronize()
            with profile(activities=[ProfilerActivity.CUDA]) as p:
                C.gemm(a, b, C.EPI_BIAS, bias)
                torch.cuda.synchronize()
        return [e.name for e in p.events() if "gemm" in e.name]

    on = names(1)
    if not on:
        pytest.skip("profiler recorded no device kernels on this build")
    assert any("gemm_persist_kernel" in n for n in on), on
    off = names(0)
    assert off and not any("gemm_persist_kernel" in n for n in off), off


@pytest.mark.parametrize("epi", ["NONE", "BIAS", "RESID", "BIAS_GELU_D", "MUL", "DGELU"])
def test_fp8_persistent_gemm_bitwise_vs_one_tile(epi):
    """The fp8 persistent kernel (mainloop_bk64 body with fresh staging addresses, halved epilogue,
    one deferred amax atomic per workgroup) against the one-tile fp8 kernel: identical outputs, and
    identical fp8 side codes + amax where the epilogue writes them."""
    C = _C()
    M, N, K = 4608, 4096, 256
    torch.manual_seed(21)
    one = torch.ones(1, device=DEV)
    fa = 1 if epi in ("RESID", "MUL", "DGELU") else 0
    a8 = C.fp8_quantize(torch.randn(M, K, device=DEV).bfloat16(), fa, one)
    w8 = C.fp8_quantize((torch.randn(N, K, device=DEV) * 0.1).bfloat16(), 0, one)
    bias = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    aux = torch.randn(M, N, device=DEV).bfloat16()
    e = getattr(C, "EPI_" + epi)
    q8 = epi in ("BIAS_GELU_D", "MUL", "DGELU")

    def run():
        kw = {}
        codes = amax = None
        if q8:
            codes = torch.full((M, N), 7, device=DEV, dtype=torch.uint8)
            amax = torch.zeros(1, device=DEV)
            kw = dict(q8_out=codes, q8_scale=torch.tensor([3.0], device=DEV), q8_amax=amax, q8_fmt=fa)
        if epi in ("NONE",):
            out = C.gemm_f8(a8, w8, one, one, fa, e, None, None, None, torch.bfloat16, **kw)
        elif epi in ("BIAS", "BIAS_GELU_D"):
            out = C.gemm_f8(a8, w8, one, one, fa, e, bias, None, None, torch.bfloat16, **kw)
        elif epi == "RESID":
            out = C.gemm_f8(a8, w8, one, one, fa, e, None, aux, None, torch.bfloat16, **kw)
        else:
            out = C.gemm_f8(a8, w8, one, one, fa, e, None, aux, torch.float32, torch.bfloat16, **kw)
        torch.cuda.synchronize()
        return out, codes, amax

    with _persist(1, 1):
        (o1, d1), c1, m1 = run()
    with _persist(1, 0):
        (o0, d0), c0, m0 = run()
    assert torch.equal(o1, o0)
    if d0 is not None:
        assert torch.equal(d1, d0)
    if q8:
        assert torch.equal(c1, c0)
        assert float(m1) == float(m0)
