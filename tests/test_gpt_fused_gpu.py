"""GPT-2 pre-LN residual stream with each LayerNorm fused into the residual update before it
(fops.bias_dropout_add_ln: bdaln kernel each way, the stream's second gradient added inside the
LayerNorm backward) against the per-block path (bias_dropout_add, then a separate LayerNorm; autograd
sums the two gradients of the stream): logits and every parameter gradient, bf16 on the GPU."""
import pytest
import torch


def _per_block(m, ids):
    x = m.wte(ids) + m.wpe(torch.arange(ids.shape[1], device=ids.device))[None]
    for blk in m.blocks:
        x = blk(x)
    from apex.ops import fused as fops

    return fops.fused_dense(m.ln_f(x), m.wte.weight, None)


@pytest.mark.gpu
def test_gpt_fused_prenorm_matches_per_block():
    from apex.models import GPTConfig, GPTModel

    torch.manual_seed(0)
    c = GPTConfig.tiny()
    c.dropout = 0.0
    m = GPTModel(c).cuda().to(torch.bfloat16)
    ids = torch.randint(0, c.vocab_size, (2, 64), device="cuda")
    out = m(ids)
    g = torch.randn_like(out)
    out.backward(g)
    fused = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    ref = _per_block(m, ids)
    ref.backward(g)
    torch.testing.assert_close(out.float(), ref.float(), rtol=2e-2, atol=2e-2)
    # relative Frobenius error per parameter (bf16 kernels with different fusion points; the tied
    # embedding accumulates two large gradients, so elementwise tolerances do not fit it)
    errs = {n: float((fused[n] - p.grad.float()).norm() / p.grad.float().norm().clamp_min(1e-12))
            for n, p in m.named_parameters()}
    print({n: round(e, 5) for n, e in errs.items()})
    assert max(errs.values()) < 2e-2, errs


@pytest.mark.gpu
def test_gpt_fused_prenorm_dropout_runs():
    from apex.models import GPTConfig, GPTModel
    from apex.models.gpt import synthetic_batch

    torch.manual_seed(0)
    c = GPTConfig.tiny()
    m = GPTModel(c).cuda().to(torch.bfloat16)
    b = synthetic_batch(c, 2, 64, device="cuda")
    loss = m(**b)
    loss.backward()
    assert torch.isfinite(loss)
    assert all(p.grad is not None and torch.isfinite(p.grad.float()).all() for p in m.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("cols", [1024, 1600, 2560, 4096])
def test_bias_dropout_add_ln_vs_fp32(cols):
    """s = res + (x + b), y = LN(s); both outputs used (the pre-LN residual stream), p = 0: values and
    the gradients of x, b, res, gamma, beta against fp32 autograd; 2560 / 4096 run the wide kernels."""
    import torch.nn.functional as F

    from apex.ops import fused as fops

    torch.manual_seed(cols)
    rows = 3000
    dt = torch.bfloat16
    x = torch.randn(rows, cols, device="cuda").to(dt).requires_grad_(True)
    res = torch.randn(rows, cols, device="cuda").to(dt).requires_grad_(True)
    b = (torch.randn(cols, device="cuda") * 0.1).to(dt).requires_grad_(True)
    g = (1 + 0.1 * torch.randn(cols, device="cuda")).to(dt).requires_grad_(True)
    be = (0.1 * torch.randn(cols, device="cuda")).to(dt).requires_grad_(True)
    s, y = fops.bias_dropout_add_ln(x, b, res, g, be, 0.0, 1e-5)
    ds, dy = torch.randn_like(s), torch.randn_like(y)
    torch.autograd.backward([s, y], [ds, dy])
    ref = [t.detach().float().requires_grad_(True) for t in (x, b, res, g, be)]
    sr = ref[2] + ref[0] + ref[1]
    yr = F.layer_norm(sr, (cols,), ref[3], ref[4], 1e-5)
    torch.autograd.backward([sr, yr], [ds.float(), dy.float()])
    torch.testing.assert_close(s.float(), sr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=5e-2)
    for t, r in zip((x, b, res, g, be), ref):
        err = float((t.grad.float() - r.grad).norm() / r.grad.norm())
        assert err < 1e-2, err
