"""Memory-efficient post-LN sublayers (apex.ops.blocks, APEX_LN_MEM=1 default): no saved LN input in
the common case, exact gradients when a gamma entry is exactly 0 (the saved input comes back), checked
against an fp32 PyTorch composition of the same sublayer."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _attn_ref(x, wqkv, bqkv, wo, bo, g, be, heads, eps):
    B, S, E = x.shape
    d = E // heads
    qkv = F.linear(x, wqkv, bqkv).view(B, S, 3, heads, d)
    q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
    p = torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(d), -1)
    o = (p @ v).transpose(1, 2).reshape(B, S, E)
    return F.layer_norm(x + F.linear(o, wo, bo), (E,), g, be, eps)


def _ffn_ref(x, w1, b1, w2, b2, g, be, eps):
    return F.layer_norm(x + F.linear(F.gelu(F.linear(x, w1, b1)), w2, b2), (x.shape[-1],), g, be, eps)


def _params(kind, E, dt, zero):
    torch.manual_seed(17 + E + int(zero))
    mk = lambda *s, sc=0.05: (sc * torch.randn(*s, device=DEV)).to(dt).requires_grad_(True)
    g = (1 + 0.2 * torch.randn(E, device=DEV)).to(dt)
    if zero:
        g[3] = 0
        g[E - 5] = 0
    g.requires_grad_(True)
    be = mk(E, sc=0.3)
    if kind == "attn":
        return [mk(3 * E, E), mk(3 * E), mk(E, E), mk(E), g, be]
    return [mk(4 * E, E), mk(4 * E), mk(E, 4 * E), mk(E), g, be]


def _run(kind, x, ps, heads=16):
    from apex.ops import blocks

    if kind == "attn":
        return blocks.attention_sublayer(x, *ps, heads, 0.0, 0.0, 1e-12)
    return blocks.ffn_sublayer(x, *ps, 0.0, 1e-12)


@pytest.mark.parametrize("kind", ["attn", "ffn"])
@pytest.mark.parametrize("zero", [False, True])
def test_sublayer_mem_mode_saves_no_input_and_matches_fp32(kind, zero):
    from apex.ops import blocks

    if not blocks._LN_MEM:
        pytest.skip("APEX_LN_MEM=0")
    dt, E = torch.bfloat16, 1024
    ps = _params(kind, E, dt, zero)
    x = torch.randn(4, 128, E, device=DEV).to(dt).requires_grad_(True)
    y = _run(kind, x, ps)
    assert y is not None
    s_alt = y.grad_fn.saved_tensors[-1]
    if zero:
        assert s_alt is not None and s_alt.numel() == x.numel()  # the zero-gamma fallback input
    else:
        assert s_alt is None  # nothing [tokens, hidden] beyond the LN output itself
    dy = torch.randn_like(y)
    y.backward(dy)
    leaves = [t.detach().float().requires_grad_(True) for t in [x] + ps]
    ref = _attn_ref(*leaves, 16, 1e-12) if kind == "attn" else _ffn_ref(*leaves, 1e-12)
    ref.backward(dy.float())
    for got, r, name in zip([x] + ps, leaves, ["x", "w_in", "b_in", "w_out", "b_out", "gamma", "beta"]):
        gg = got.grad.float()
        assert torch.isfinite(gg).all(), name
        err = (gg - r.grad).abs().max().item() / (r.grad.abs().max().item() + 1e-6)
        assert err < 4e-2, (name, err)
    err = (y.float() - ref).abs().max().item()
    assert err < 5e-2, err


def test_gamma_zero_written_between_steps_is_seen():
    """A gamma zeroed in place by a raw write (no version bump) as part of an optimizer step turns the
    fallback on at the next forward; restoring it turns it off again. The check is re-armed by the
    global optimizer-step hook (apex.ops.blocks._GammaZeroCheck), so the write is followed by a step
    here — earlier tests in the process have run optimizer steps, after which a backward alone no
    longer re-arms it (one host read per step under gradient accumulation)."""
    from apex.ops import blocks

    if not blocks._LN_MEM:
        pytest.skip("APEX_LN_MEM=0")
    dt, E = torch.bfloat16, 1024
    ps = _params("ffn", E, dt, False)
    x = torch.randn(2, 128, E, device=DEV).to(dt).requires_grad_(True)
    y = _run("ffn", x, ps)
    assert y.grad_fn.saved_tensors[-1] is None
    y.sum().backward()
    with torch.no_grad():
        ps[4].data[7] = 0  # raw write (no version bump), as an optimizer kernel writes through its pointer
    torch.optim.SGD([ps[4]], lr=0.0).step()  # the step post-hook re-arms the check
    y = _run("ffn", x, ps)
    assert y.grad_fn.saved_tensors[-1] is not None
    y.sum().backward()
    assert torch.isfinite(x.grad.float()).all() and torch.isfinite(ps[4].grad.float()).all()
    with torch.no_grad():
        ps[4][7] = 1.0
    y = _run("ffn", x, ps)
    assert y.grad_fn.saved_tensors[-1] is None


def test_gamma_check_one_host_read_per_step_with_accumulation():
    """4 accumulated micro-batches per FusedLAMB step through both sublayer kinds: the gamma-zero
    check reads the device once per optimizer step (the step hook marks it dirty, backward does not
    once an optimizer step has been seen), and a zero the optimizer writes into a gamma (raw-pointer
    kernel, no version bump) is seen at the next step's first forward, which then keeps the LN input."""
    from apex.ops import blocks
    from apex.optimizers import FusedLAMB

    if not blocks._LN_MEM:
        pytest.skip("APEX_LN_MEM=0")
    dt, E = torch.bfloat16, 1024
    pa, pf = _params("attn", E, dt, False), _params("ffn", E, dt, False)
    opt = FusedLAMB(pa + pf, lr=1e-4)
    x = torch.randn(2, 128, E, device=DEV).to(dt)
    gz = blocks._GZ
    reads = []
    for step in range(3):
        r0 = gz.host_reads
        for micro in range(4):
            y = _run("ffn", _run("attn", x, pa), pf)
            y.float().square().mean().backward()
        reads.append(gz.host_reads - r0)
        opt.step()
        opt.zero_grad()
    assert reads[1:] == [1, 1], reads  # (step 0 may re-check before the first step hook fires)
    # a zero written by the optimizer's kernel: seen by the next forward
    pf[4].data[7] = 0  # .data write: no version bump, like a fused-kernel write
    dummy = torch.nn.Parameter(torch.zeros(1, device=DEV))
    torch.optim.SGD([dummy], lr=0.0).step()  # any optimizer's step fires the global hook
    y = _run("ffn", x, pf)
    assert y.grad_fn.saved_tensors[-1] is not None  # the zero-gamma fallback input is kept
