"""Fused BERT embedding block (apex.ops.fused.bert_embeddings: csrc/fused_ops.hip embed_ln_*) on the
GPU against a plain PyTorch fp32 reference of the same op — gathers, sum, LayerNorm, dropout — in
forward and for every gradient (word / position / type tables, gamma, beta); duplicate-heavy id
sets exercise the word-table segment sum."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tables(V, NP, TV, H, dt, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    mk = lambda *s: (torch.randn(*s, device=DEV, generator=g) * 0.5).to(dt).requires_grad_(True)
    gamma = (1 + 0.1 * torch.randn(H, device=DEV, generator=g)).to(dt).requires_grad_(True)
    beta = (0.1 * torch.randn(H, device=DEV, generator=g)).to(dt).requires_grad_(True)
    return mk(V, H), mk(NP, H), mk(TV, H), gamma, beta


def _ref(ids, tids, Ww, Wp, Wt, gamma, beta, eps, mask=None, p=0.0):
    S = ids.shape[1]
    x = Ww.float()[ids] + Wp.float()[:S][None] + (Wt.float()[tids] if tids is not None else Wt.float()[0])
    y = F.layer_norm(x, (x.shape[-1],), gamma.float(), beta.float(), eps)
    if mask is not None:
        y = y * mask / (1 - p)
    return y


@pytest.mark.parametrize("B,S,H,V,dup", [(4, 128, 1024, 30528, False), (8, 64, 768, 1000, True),
                                         (3, 40, 256, 50, True), (2, 16, 512, 7, True)])
@pytest.mark.parametrize("types", [True, False])
def test_embeddings_match_fp32_reference(B, S, H, V, dup, types):
    from apex.ops.fused import bert_embeddings

    dt = torch.bfloat16
    Ww, Wp, Wt, gamma, beta = _tables(V, 512, 2, H, dt, seed=B + S)
    g = torch.Generator(device=DEV).manual_seed(3)
    ids = torch.randint(0, min(V, 5) if dup else V, (B, S), device=DEV, generator=g)
    tids = torch.randint(0, 2, (B, S), device=DEV, generator=g) if types else None
    y = bert_embeddings(ids, tids, Ww, Wp, Wt, gamma, beta, 0.0, 1e-12)
    dy = torch.randn(y.shape, device=DEV, generator=g).to(dt)
    grads = torch.autograd.grad(y, [Ww, Wp, Wt, gamma, beta], dy)
    ref_in = [t.detach().float().requires_grad_(True) for t in (Ww, Wp, Wt, gamma, beta)]
    yr = _ref(ids, tids, *ref_in, 1e-12)
    rgrads = torch.autograd.grad(yr, ref_in, dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    for name, a, b in zip(("word", "pos", "type", "gamma", "beta"), grads, rgrads):
        tol = 2e-2 * max(1.0, float(b.abs().max()))
        torch.testing.assert_close(a.float(), b, rtol=3e-2, atol=tol, msg=lambda m: f"{name}: {m}")
    assert float(grads[1][S:].abs().max()) == 0.0  # positions past S get no gradient


def test_embeddings_dropout_mask_consistent():
    """p > 0: the kept elements are the LN output scaled by 1/(1-p), about p of them are zero, and
    the backward regenerates the same mask (the reference gradient built from y's zero pattern
    matches)."""
    from apex.ops.fused import bert_embeddings

    dt, p = torch.bfloat16, 0.25
    B, S, H, V = 8, 128, 1024, 30528
    Ww, Wp, Wt, gamma, beta = _tables(V, 512, 2, H, dt, seed=5)
    g = torch.Generator(device=DEV).manual_seed(7)
    ids = torch.randint(0, V, (B, S), device=DEV, generator=g)
    tids = torch.randint(0, 2, (B, S), device=DEV, generator=g)
    torch.manual_seed(11)
    y = bert_embeddings(ids, tids, Ww, Wp, Wt, gamma, beta, p, 1e-12)
    mask = (y != 0).float()
    assert abs(1 - float(mask.mean()) - p) < 0.01
    dy = torch.randn(y.shape, device=DEV, generator=g).to(dt)
    grads = torch.autograd.grad(y, [Ww, Wp, Wt, gamma, beta], dy)
    ref_in = [t.detach().float().requires_grad_(True) for t in (Ww, Wp, Wt, gamma, beta)]
    pq = round(p * 65536) / 65536  # the kernels' 16-bit keep threshold
    yr = _ref(ids, tids, *ref_in, 1e-12, mask=mask, p=pq)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    rgrads = torch.autograd.grad(yr, ref_in, dy.float())
    for name, a, b in zip(("word", "pos", "type", "gamma", "beta"), grads, rgrads):
        tol = 2e-2 * max(1.0, float(b.abs().max()))
        torch.testing.assert_close(a.float(), b, rtol=3e-2, atol=tol, msg=lambda m: f"{name}: {m}")


def test_bert_model_uses_fused_embeddings_and_matches_unfused():
    from apex.models.bert import BertConfig, BertEmbeddings

    c = BertConfig(vocab_size=1000, hidden_size=256, num_hidden_layers=1, num_attention_heads=4,
                   intermediate_size=1024, hidden_dropout_prob=0.0)
    torch.manual_seed(0)
    emb = BertEmbeddings(c).to(DEV).bfloat16()
    ids = torch.randint(0, 1000, (4, 64), device=DEV)
    tids = torch.randint(0, 2, (4, 64), device=DEV)
    y = emb(ids, tids)
    BertEmbeddings.use_fused = False
    try:
        yr = emb(ids, tids)
    finally:
        BertEmbeddings.use_fused = True
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=2e-2)
