"""Fused transformer elementwise kernels vs PyTorch fp32 references (GPU only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = {torch.float32: 2e-5, torch.bfloat16: 2e-2, torch.float16: 3e-3}


def _C():
    import apex._ext as e

    return e.require()


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("rows,cols", [(333, 4096), (64, 1000), (1, 8)])
def test_bias_act(dt, act, rows, cols):
    from apex.ops import fused

    torch.manual_seed(rows + cols)
    h = torch.randn(rows, cols, device=DEV).to(dt).requires_grad_(True)
    b = torch.randn(cols, device=DEV).to(dt).requires_grad_(True)
    y = fused._BiasAct.apply(h, b, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    hr, br = h.detach().float().requires_grad_(True), b.detach().float().requires_grad_(True)
    yr = fused._act_ref(hr + br, act)
    yr.backward(dy.float())
    t = TOL[dt]
    torch.testing.assert_close(y.float(), yr, rtol=t, atol=t)
    torch.testing.assert_close(h.grad.float(), hr.grad, rtol=t * 2, atol=t * 2)
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=t * 4, atol=t * rows ** 0.5 * 4)


def test_colsum():
    C = _C()
    x = torch.randn(5000, 1032, device=DEV).bfloat16()
    out = C.colsum(x, torch.float32)
    torch.testing.assert_close(out, x.float().sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("p", [0.0, 0.1, 0.5])
def test_bias_dropout_add(p):
    from apex.ops import fused

    torch.manual_seed(1)
    rows, cols = 300, 1024
    x = torch.randn(rows, cols, device=DEV).bfloat16().requires_grad_(True)
    b = torch.randn(cols, device=DEV).bfloat16().requires_grad_(True)
    r = torch.randn(rows, cols, device=DEV).bfloat16().requires_grad_(True)
    torch.manual_seed(7)
    y = fused.bias_dropout_add(x, b, r, p)
    # recover the mask: same seed, res = 0, x + b = 1 -> kept entries are exactly `scale`
    torch.manual_seed(7)
    ones = fused.bias_dropout_add(torch.ones_like(x), torch.zeros_like(b), torch.zeros_like(r), p)
    keep = ones.detach().float() != 0
    t = (x + b).detach().float()
    delta = (y - r).detach().float()
    if p > 0:
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 0.02
        scale = 1.0 / (1 - round(p * 65536) / 65536)
        torch.testing.assert_close(delta[keep], (t * scale)[keep], rtol=3e-2, atol=3e-2)
    else:
        torch.testing.assert_close(delta, t, rtol=2e-2, atol=2e-2)
    dy = torch.randn_like(y)
    y.backward(dy)
    torch.testing.assert_close(r.grad, dy)
    m = keep.float() * (1.0 / (1 - round(p * 65536) / 65536) if p > 0 else 1.0)
    torch.testing.assert_close(x.grad.float(), dy.float() * m, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(b.grad.float(), (dy.float() * m).sum(0), rtol=2e-2, atol=0.5)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cols", [1024, 768, 1600, 2048])
def test_dense_bdaln_no_dropout(dt, cols):
    from apex.ops import fused

    torch.manual_seed(cols)
    rows, k = 257, 512
    x = (torch.randn(rows, k, device=DEV) * 0.5).to(dt).requires_grad_(True)
    w = (torch.randn(cols, k, device=DEV) * 0.05).to(dt).requires_grad_(True)
    b = torch.randn(cols, device=DEV).to(dt).requires_grad_(True)
    res = torch.randn(rows, cols, device=DEV).to(dt).requires_grad_(True)
    g = (1 + 0.1 * torch.randn(cols, device=DEV)).to(dt).requires_grad_(True)
    be = (0.1 * torch.randn(cols, device=DEV)).to(dt).requires_grad_(True)
    y = fused.dense_bias_dropout_add_ln(x, w, b, res, g, be, 0.0, 1e-12)
    dy = torch.randn_like(y)
    y.backward(dy)
    leaves = [t.detach().float().requires_grad_(True) for t in (x, w, b, res, g, be)]
    xr, wr, br, rr, gr, ber = leaves
    yr = F.layer_norm(rr + F.linear(xr, wr, br), (cols,), gr, ber, 1e-12)
    yr.backward(dy.float())
    t = 3e-2 if dt == torch.bfloat16 else 5e-3
    torch.testing.assert_close(y.float(), yr, rtol=t, atol=t * 2)
    for got, ref, name in zip((x, w, b, res, g, be), leaves, "x w b res g be".split()):
        scale = ref.grad.abs().max().item() + 1e-6
        err = (got.grad.float() - ref.grad).abs().max().item() / scale
        assert err < 4 * t, (name, err)


def test_dense_bdaln_dropout_statistics():
    from apex.ops import fused

    torch.manual_seed(0)
    rows, k, cols, p = 512, 256, 1024, 0.1
    x = torch.randn(rows, k, device=DEV).bfloat16()
    w = (torch.randn(cols, k, device=DEV) * 0.05).bfloat16()
    b = torch.zeros(cols, device=DEV).bfloat16()
    res = torch.zeros(rows, cols, device=DEV).bfloat16()
    g = torch.ones(cols, device=DEV).bfloat16()
    be = torch.zeros(cols, device=DEV).bfloat16()
    # identical seeds -> identical outputs (mask regenerated deterministically)
    torch.manual_seed(5)
    y1 = fused.dense_bias_dropout_add_ln(x, w, b, res, g, be, p, 1e-5)
    torch.manual_seed(5)
    y2 = fused.dense_bias_dropout_add_ln(x, w, b, res, g, be, p, 1e-5)
    assert torch.equal(y1, y2)
    y3 = fused.dense_bias_dropout_add_ln(x, w, b, res, g, be, p, 1e-5)
    assert not torch.equal(y1, y3)


def test_fused_dense_bias_grad():
    from apex.ops import fused

    torch.manual_seed(2)
    x = torch.randn(4, 33, 64, device=DEV).bfloat16().requires_grad_(True)
    w = torch.randn(96, 64, device=DEV).bfloat16().requires_grad_(True)
    b = torch.randn(96, device=DEV).bfloat16().requires_grad_(True)
    y = fused.fused_dense(x, w, b)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    F.linear(xr, wr, br).backward(dy.float())
    torch.testing.assert_close(b.grad.float(), br.grad, rtol=2e-2, atol=0.3)
    torch.testing.assert_close(w.grad.float(), wr.grad, rtol=3e-2, atol=0.3)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("M,N,K", [(32768, 1024, 1024), (16384, 3072, 1024), (8192, 1024, 4096), (4096, 256, 512)])
def test_wgrad_splitk(dt, M, N, K):
    from apex.ops import fused

    torch.manual_seed(3)
    dy = torch.randn(M, N, device=DEV).to(dt)
    x = torch.randn(M, K, device=DEV).to(dt)
    s = fused._wgrad_splits(M, N, K)
    dw = fused._wgrad(dy, x)
    assert dw.dtype == dt and dw.shape == (N, K)
    ref = dy.float().t() @ x.float()
    # fp32 split-K accumulation: only the final rounding to the grad dtype differs from fp32
    tol = 2 ** -7 if dt == torch.bfloat16 else 2 ** -10
    torch.testing.assert_close(dw.float(), ref, rtol=tol, atol=tol * float(ref.abs().max()))
    if M >= 8192:
        assert s > 1


def test_splitk_reduce_tail():
    import apex

    C = apex._ext.require()
    slabs = torch.randn(3, 5, 12, device=DEV)  # 60 elements: vector path + no tail; and odd sizes below
    torch.testing.assert_close(C.splitk_reduce(slabs, torch.float32), slabs.sum(0))
    slabs = torch.randn(4, 20, device=DEV)
    torch.testing.assert_close(C.splitk_reduce(slabs, torch.bfloat16).float(), slabs.sum(0).bfloat16().float())


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_bert_sublayer_fusion_matches_op_by_op(p):
    """Whole-sublayer Functions (residual grads in the GEMM epilogues) vs the op-by-op path."""
    from apex.models.bert import BertConfig, BertLayer

    torch.manual_seed(0)
    c = BertConfig(hidden_size=256, num_attention_heads=4, intermediate_size=1024, num_hidden_layers=1,
                   hidden_dropout_prob=p, attention_probs_dropout_prob=p)
    layer = BertLayer(c).to(DEV).bfloat16()
    x = torch.randn(4, 64, 256, device=DEV).bfloat16()
    k_lens = torch.tensor([64, 40, 64, 17], device=DEV, dtype=torch.int32)
    outs = []
    for fused in (True, False):
        layer.use_sublayer_fusion = fused
        layer.zero_grad()
        xi = x.clone().requires_grad_(True)
        torch.manual_seed(123)
        y = layer(xi, k_lens)
        torch.manual_seed(7)
        dy = torch.randn_like(y)
        y.backward(dy)
        outs.append((y.float(), xi.grad.float(), {n: q.grad.float() for n, q in layer.named_parameters()}))
    (y1, dx1, g1), (y2, dx2, g2) = outs
    torch.testing.assert_close(y1, y2, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dx1, dx2, rtol=3e-2, atol=3e-2)
    for n in g1:  # bias grads are 256-row sums of bf16 values: tolerance relative to their scale
        torch.testing.assert_close(g1[n], g2[n], rtol=5e-2, atol=5e-2 * max(1.0, float(g2[n].abs().max())), msg=n)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("cols,p", [(1024, 0.0), (1024, 0.1), (768, 0.1), (512, 0.0)])
def test_bdaln_bwd_from_output_matches_stored_input(dt, cols, p):
    """Memory-efficient post-LN (store_s=False forward, backward from y and beta) vs the stored-s
    backward of the same forward: identical outputs, gradients within the 16-bit storage error, and
    both against the fp32 autograd reference."""
    C = _C()
    torch.manual_seed(cols)
    rows = 999
    t = torch.randn(rows, cols, device=DEV).to(dt)
    b = torch.randn(cols, device=DEV).to(dt)
    res = torch.randn(rows, cols, device=DEV).to(dt)
    g = (1 + 0.2 * torch.randn(cols, device=DEV)).to(dt)
    be = (0.3 * torch.randn(cols, device=DEV)).to(dt)
    dy = torch.randn(rows, cols, device=DEV).to(dt)
    y, s, mean, rstd = C.bdaln_fwd(t, b, res, g, be, 1e-12, p, 11, 3)
    y2, s2, mean2, rstd2 = C.bdaln_fwd(t, b, res, g, be, 1e-12, p, 11, 3, store_s=False)
    assert s2.numel() == 0 and torch.equal(y, y2) and torch.equal(rstd, rstd2)
    ref = C.bdaln_bwd(dy, s, g, mean, rstd, p, 11, 3, True)
    got = C.bdaln_bwd(dy, y2, g, mean2, rstd2, p, 11, 3, True, beta=be)
    for a, r, name in zip(got, ref, ("dres", "dx", "dgamma", "dbeta", "dbias")):
        scale = r.float().abs().max().item() + 1e-6
        err = (a.float() - r.float()).abs().max().item() / scale
        assert err < (2e-2 if dt == torch.bfloat16 else 4e-3), (name, err)
    if p == 0.0:  # against fp32 autograd of LN(res + t + b)
        leaves = [x.float().requires_grad_(True) for x in (t, b, res, g, be)]
        tr, br, rr, gr, ber = leaves
        F.layer_norm(rr + tr + br, (cols,), gr, ber, 1e-12).backward(dy.float())
        tol = 3e-2 if dt == torch.bfloat16 else 5e-3
        for a, r, name in ((got[0], rr.grad, "dres"), (got[2], gr.grad, "dgamma"), (got[3], ber.grad, "dbeta")):
            err = (a.float() - r).abs().max().item() / (r.abs().max().item() + 1e-6)
            assert err < 4 * tol, (name, err)


@pytest.mark.parametrize("zero", [False, True])
@pytest.mark.parametrize("cols,p", [(1024, 0.1), (512, 0.0)])
def test_bdaln_conditional_s_zero_gamma(zero, cols, p):
    """s_cond forward / s_alt backward (the memory-efficient post-LN default): with a gamma entry of
    exactly 0 the forward stores s and the backward reads it (no 0 * inf NaNs, gradients equal to the
    stored-input backward); without one, s stays unwritten and the backward rebuilds x-hat from y."""
    C = _C()
    dt = torch.bfloat16
    torch.manual_seed(cols + int(zero))
    rows = 777
    t = torch.randn(rows, cols, device=DEV).to(dt)
    b = torch.randn(cols, device=DEV).to(dt)
    res = torch.randn(rows, cols, device=DEV).to(dt)
    g = (1 + 0.2 * torch.randn(cols, device=DEV)).to(dt)
    if zero:
        g[5] = 0
        g[cols - 3] = 0
    be = (0.3 * torch.randn(cols, device=DEV)).to(dt)
    dy = torch.randn(rows, cols, device=DEV).to(dt)
    y, s, mean, rstd = C.bdaln_fwd(t, b, res, g, be, 1e-12, p, 11, 3)
    sentinel = torch.full((rows, cols), 7.0, device=DEV, dtype=dt)
    y2, s2, mean2, rstd2 = C.bdaln_fwd(t, b, res, g, be, 1e-12, p, 11, 3, s_cond=True)
    assert torch.equal(y, y2) and torch.equal(rstd, rstd2) and s2.shape == s.shape
    if zero:
        assert torch.equal(s2, s)  # written because gamma has a zero
    ref = C.bdaln_bwd(dy, s, g, mean, rstd, p, 11, 3, True)
    got = C.bdaln_bwd(dy, y2, g, mean2, rstd2, p, 11, 3, True, beta=be, s_alt=s2 if zero else sentinel)
    for a, r, name in zip(got, ref, ("dres", "dx", "dgamma", "dbeta", "dbias")):
        assert torch.isfinite(a.float()).all(), name
        if zero:
            assert torch.equal(a, r), name  # the same stored-input body on the same s
        else:
            err = (a.float() - r.float()).abs().max().item() / (r.float().abs().max().item() + 1e-6)
            assert err < 2e-2, (name, err)  # rebuilt from y (the sentinel s_alt is never read)
