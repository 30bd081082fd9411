"""Ring-attention block contract on the flash kernels (apex.transformer.context_parallel).

The ring's communication is covered on CPU/gloo (tests/test_context_parallel.py); here the device
block math is checked in one process: the key sequence is cut into chunks, each (query chunk, key
chunk) block runs flash_attn_fwd, the blocks are merged through their log-sum-exp, and the block
backward (flash_attn_bwd fed the MERGED output and lse) is summed per chunk — exactly what each ring
step does — against one full-sequence flash attention and the fp32 reference, causal (diagonal
blocks causal, lower blocks full, upper skipped) and not.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal, scale):
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), k.float()) * scale
    if causal:
        S = s.shape[-1]
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s.device).triu(1), float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", s.softmax(-1), v.float())


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("D", [64, 128])
def test_ring_blocks_match_full(causal, D):
    from apex.transformer import context_parallel as cp

    torch.manual_seed(0)
    B, S, H, n = 2, 1024, 4, 4
    dev = "cuda"
    q, k, v, do = (torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16) for _ in range(4))
    scale = D ** -0.5
    qs, ks, vs, dos = (t.chunk(n, dim=1) for t in (q, k, v, do))
    outs, lses = [], []
    aux = {}
    for a in range(n):
        acc = [None, None]
        for b in range(n):
            if causal and b > a:
                continue
            o, lse, x = cp._blk_fwd(qs[a], ks[b], vs[b], causal and a == b, scale, 0.0)
            acc = list(cp._merge(acc[0], acc[1], o, lse))
            aux[(a, b)] = x
        outs.append(acc[0].to(q.dtype))
        lses.append(acc[1])
    out = torch.cat(outs, dim=1)
    ref = _ref(q, k, v, causal, scale)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)

    dq = torch.zeros(q.shape, device=dev)
    dk = torch.zeros(k.shape, device=dev)
    dv = torch.zeros(v.shape, device=dev)
    for (a, b), x in aux.items():
        g = cp._blk_bwd(dos[a], qs[a], ks[b], vs[b], outs[a], lses[a], causal and a == b, scale, 0.0, x)
        dq.chunk(n, dim=1)[a].add_(g[0].float())
        dk.chunk(n, dim=1)[b].add_(g[1].float())
        dv.chunk(n, dim=1)[b].add_(g[2].float())
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    _ref(qr, kr, vr, causal, scale).backward(do.float())
    for got, want in ((dq, qr.grad), (dk, kr.grad), (dv, vr.grad)):
        err = (got - want).abs().max().item() / want.abs().max().item()
        assert err < 2e-2, err


def test_ring_attention_single_rank_is_flash():
    """CP size 1 (no group): ring_attention is one flash call."""
    from apex.contrib.multihead_attn.flash import flash_attention
    from apex.transformer import context_parallel as cp

    torch.manual_seed(1)
    q, k, v = (torch.randn(2, 256, 4, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    out = cp._RingAttention.apply(q, k, v, None, [0], 0, True, 0.125, 0.0, "contiguous")
    torch.testing.assert_close(out, flash_attention(q, k, v, causal=True, scale=0.125), atol=0, rtol=0)
    # backward at CP size 1 (no process group, torch.distributed not initialised): no ring send to
    # itself; equal to the flash backward up to the fp32 accumulation of the single block
    qa, ka, va = (t.clone().requires_grad_() for t in (q, k, v))
    qb, kb, vb = (t.clone().requires_grad_() for t in (q, k, v))
    do = torch.randn_like(q)
    cp.ring_attention(qa, ka, va, causal=True, scale=0.125).backward(do)
    flash_attention(qb, kb, vb, causal=True, scale=0.125).backward(do)
    for a, b in ((qa, qb), (ka, kb), (va, vb)):
        torch.testing.assert_close(a.grad.float(), b.grad.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_lse_merge_kernel_matches_torch_merge(dt):
    """The fused HIP log-sum-exp merge (csrc/context_parallel.hip) against the torch composition,
    including rows with no visible key (+inf lse) on either side and the first-block initialisation."""
    import apex._ext as e
    from apex.transformer import context_parallel as cp

    C = e.require()
    torch.manual_seed(2)
    B, S, H, D = 2, 96, 3, 64
    blocks = []
    for j in range(3):
        o = torch.randn(B, S, H, D, device="cuda").to(dt)
        lse = torch.randn(B, H, S, device="cuda") * 3
        lse[0, 1, j * 7:(j * 7) + 5] = float("inf")  # empty rows in this block
        lse[1, 2, 40:45] = float("inf")  # empty in every block
        blocks.append((o, lse))
    acc_o = acc_l = None
    ref_o = ref_l = None
    for o, lse in blocks:
        acc_o, acc_l = cp._merge(acc_o, acc_l, o, lse)  # native path on the GPU
        # torch reference path
        l2 = torch.where(torch.isposinf(lse), torch.full_like(lse, float("-inf")), lse)
        if ref_o is None:
            ref_o, ref_l = o.float(), l2.clone()
        else:
            new = torch.logaddexp(ref_l, l2)
            safe = torch.where(torch.isneginf(new), torch.zeros_like(new), new)
            ref_o = ref_o * torch.exp(ref_l - safe).transpose(1, 2).unsqueeze(-1) + \
                o.float() * torch.exp(l2 - safe).transpose(1, 2).unsqueeze(-1)
            ref_l = new
    assert cp._native_merge(blocks[0][0], blocks[0][1])
    torch.testing.assert_close(acc_l, ref_l, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(acc_o, ref_o, rtol=1e-5, atol=1e-5)
    assert torch.isneginf(acc_l[1, 2, 40:45]).all() and (acc_o[1, 40:45, 2] == 0).all()


@pytest.mark.gpu
def test_lse_merge_kernel_row_range_matches_cpu_merge():
    """The HIP merge into a row range of a larger accumulator (s0 > 0, first block not covering all
    rows) against the torch composition on the CPU."""
    from apex.transformer import context_parallel as cp

    torch.manual_seed(3)
    B, S, H, D = 2, 64, 3, 64
    o0 = torch.randn(B, S // 2, H, D)
    l0 = torch.randn(B, H, S // 2) * 2
    o1 = torch.randn(B, S, H, D)
    l1 = torch.randn(B, H, S) * 2
    l1[1, 0, 3:6] = float("inf")
    steps = [(o0, l0, S // 2), (o1, l1, 0), (o0 * 0.5, l0 - 1.0, 0)]
    g_o = g_l = c_o = c_l = None
    for o, l, s0 in steps:
        g_o, g_l = cp._merge(g_o, g_l, o.cuda().bfloat16(), l.cuda(), s0, S)
        c_o, c_l = cp._merge(c_o, c_l, o.bfloat16().float(), l, s0, S)
    torch.testing.assert_close(g_l.cpu(), c_l, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(g_o.cpu(), c_o, rtol=1e-5, atol=1e-5)


def test_ring_step_key_split_on_two_streams_matches_flash(monkeypatch):
    """A small non-causal step block runs as two key halves on two streams (_step_fwd / _step_bwd):
    forward merged through the log-sum-exp, dQ summed, dK / dV per half — equal to one flash call."""
    from apex.contrib.multihead_attn.flash import flash_attention
    from apex.transformer import context_parallel as cp

    torch.manual_seed(4)
    q, k, v = (torch.randn(1, 512, 4, 64, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    monkeypatch.setenv("APEX_CP_KV_SPLIT", "1")  # opt-in (measured slower in the emulation)
    assert cp._kv_parts(q, k, False) == 2
    do = torch.randn_like(q)
    res = {}
    for split in ("1", "0"):
        monkeypatch.setenv("APEX_CP_KV_SPLIT", split)
        qa, ka, va = (t.clone().requires_grad_() for t in (q, k, v))
        out = cp._RingAttention.apply(qa, ka, va, None, [0], 0, False, 0.125, 0.0, "contiguous")
        out.backward(do)
        torch.cuda.synchronize()
        res[split] = (out.float(), qa.grad.float(), ka.grad.float(), va.grad.float())
    qb, kb, vb = (t.clone().requires_grad_() for t in (q, k, v))
    ref = flash_attention(qb, kb, vb, causal=False, scale=0.125)
    ref.backward(do)
    for got in res.values():
        torch.testing.assert_close(got[0], ref.float(), atol=2e-2, rtol=2e-2)
        for g, b in zip(got[1:], (qb, kb, vb)):
            torch.testing.assert_close(g, b.grad.float(), atol=2e-2, rtol=2e-2)
