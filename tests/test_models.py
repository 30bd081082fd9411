"""Model zoo on CPU: GPT-2 / ResNet / MLP forward+backward, and the Megatron GPT under
TP=2 (vs a serial functional reference built from the gathered shards) and PP=2 (1F1B
schedule vs the serial model, tied-embedding grad sync)."""
import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from test_transformer import _spawn


def test_gpt_tiny_loss_matches_reference():
    from apex.models import GPTConfig, GPTModel
    from apex.models.gpt import synthetic_batch

    torch.manual_seed(0)
    c = GPTConfig.tiny()
    c.dropout = 0.0
    m = GPTModel(c)
    b = synthetic_batch(c, 2, 16, generator=torch.Generator().manual_seed(1))
    loss = m(**b)
    logits = m(b["input_ids"])
    ref = F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), b["labels"][:, 1:].reshape(-1))
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
    assert GPTConfig().padded_vocab == 50304


def test_gpt_fused_prenorm_path_matches_per_block_cpu():
    """GPTModel.forward's fused residual-stream path (forward_fused) against the per-block forward."""
    from apex.models import GPTConfig, GPTModel

    torch.manual_seed(0)
    c = GPTConfig.tiny()
    c.dropout = 0.0
    m = GPTModel(c)
    ids = torch.randint(0, c.vocab_size, (2, 16))
    logits = m(ids)
    x = m.wte(ids) + m.wpe(torch.arange(16))[None]
    for blk in m.blocks:
        x = blk(x)
    ref = m.ln_f(x) @ m.wte.weight.t()
    torch.testing.assert_close(logits, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("cl", [False, True])
def test_resnet_forward_backward(cl):
    from apex.models import resnet18, resnet50
    from apex.models.resnet import synthetic_batch

    torch.manual_seed(0)
    for fn in (resnet18, resnet50):
        m = fn(num_classes=10)
        if cl:
            m = m.to(memory_format=torch.channels_last)
        x, y = synthetic_batch(2, 64, 10, channels_last=cl)
        loss = F.cross_entropy(m(x), y)
        loss.backward()
        assert torch.isfinite(loss)
        assert m.conv1.weight.grad is not None
    assert sum(p.numel() for p in resnet50().parameters()) == 25557032


def test_mlp_o0_sgd_step():
    from apex import amp
    from apex.models import MLP
    from apex.models.mlp import synthetic_batch

    torch.manual_seed(0)
    m = MLP()
    opt = torch.optim.SGD(m.parameters(), lr=1e-3)
    m, opt = amp.initialize(m, opt, opt_level="O0", verbosity=0)
    x, y = synthetic_batch()
    losses = []
    for _ in range(5):
        opt.zero_grad()
        loss = F.mse_loss(m(x), y)
        with amp.scale_loss(loss, opt) as sl:
            sl.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0]


def _full_weights(model, tpws, c):
    """Gather the TP shards of every layer into the serial layout."""

    def gather(t, dim):
        parts = [torch.empty_like(t) for _ in range(tpws)]
        dist.all_gather(parts, t.detach().contiguous())
        return torch.cat(parts, dim)

    H, nh = c.hidden_size, c.num_attention_heads
    d = H // nh
    W = {"E": gather(model.word_embeddings.weight, 0), "P": model.position_embeddings.weight.detach(),
         "layers": []}
    for L in model.layers:
        wq = gather(L.query_key_value.weight, 0).view(tpws, 3, nh // tpws, d, H).transpose(0, 1).reshape(3 * H, H)
        bq = gather(L.query_key_value.bias, 0).view(tpws, 3, nh // tpws, d).transpose(0, 1).reshape(3 * H)
        W["layers"].append(dict(
            ln1=(L.input_layernorm.weight.detach(), L.input_layernorm.bias.detach()), wq=wq, bq=bq,
            wd=gather(L.dense.weight, 1), bd=L.dense.bias.detach(),
            ln2=(L.post_attention_layernorm.weight.detach(), L.post_attention_layernorm.bias.detach()),
            w1=gather(L.dense_h_to_4h.weight, 0), b1=gather(L.dense_h_to_4h.bias, 0),
            w2=gather(L.dense_4h_to_h.weight, 1), b2=L.dense_4h_to_h.bias.detach()))
    W["lnf"] = (model.final_layernorm.weight.detach(), model.final_layernorm.bias.detach())
    return W


def _serial_loss(W, ids, c):
    B, S = ids.shape
    H, nh = c.hidden_size, c.num_attention_heads
    x = W["E"][ids] + W["P"][:S][None]
    for L in W["layers"]:
        h = F.layer_norm(x, (H,), *L["ln1"], eps=c.layernorm_epsilon)
        qkv = F.linear(h, L["wq"], L["bq"]).view(B, S, 3, nh, H // nh)
        q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
        ctx = F.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, S, H)
        x = x + F.linear(ctx, L["wd"], L["bd"])
        h = F.layer_norm(x, (H,), *L["ln2"], eps=c.layernorm_epsilon)
        x = x + F.linear(F.gelu(F.linear(h, L["w1"], L["b1"])), L["w2"], L["b2"])
    x = F.layer_norm(x, (H,), *W["lnf"], eps=c.layernorm_epsilon)
    logits = x @ W["E"].t()
    return F.cross_entropy(logits[:, :-1].reshape(-1, logits.shape[-1]), ids[:, 1:].reshape(-1))


def _megatron_tp(rank, world):
    from apex.models.megatron_gpt import MegatronGPTConfig, build_stage
    from apex.transformer import parallel_state as ps

    ps.initialize_model_parallel(world, 1)
    c = MegatronGPTConfig.tiny()
    c.hidden_dropout = c.attention_dropout = 0.0
    torch.manual_seed(0)
    model = build_stage(c)
    with torch.no_grad():  # non-trivial biases / LN params
        for n, p in model.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn(p.shape, generator=torch.Generator().manual_seed(len(n) + rank)) * 0.05)
    for n, p in model.named_parameters():  # replicated params must agree across TP ranks
        if "layernorm" in n or n.endswith("dense.bias") or n.endswith("4h_to_h.bias") or "position" in n:
            dist.broadcast(p.data, 0)
    ids = torch.randint(0, c.vocab_size, (2, 32), generator=torch.Generator().manual_seed(7))
    loss = model(ids, ids)
    W = _full_weights(model, world, c)
    ref = _serial_loss(W, ids, c)
    torch.testing.assert_close(loss, ref, rtol=1e-4, atol=1e-4)
    loss.backward()
    # replicated LN grads: identical on every TP rank
    g = model.layers[0].input_layernorm.weight.grad.clone()
    g0 = g.clone()
    dist.broadcast(g0, 0)
    torch.testing.assert_close(g, g0)


def test_megatron_gpt_tensor_parallel():
    _spawn(_megatron_tp, 2)


def _megatron_pp(rank, world):
    from apex.models.megatron_gpt import (MegatronGPT, MegatronGPTConfig, build_stage, sync_embedding_grads,
                                          sync_initial_embeddings)
    from apex.transformer import parallel_state as ps
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator

    ps.initialize_model_parallel(1, world)
    n_micro, mb = 2, 2
    setup_microbatch_calculator(rank, None, n_micro * mb, mb, 1)
    c = MegatronGPTConfig.tiny()
    c.hidden_dropout = c.attention_dropout = 0.0
    torch.manual_seed(0)
    full = MegatronGPT(c)
    stage = build_stage(c)
    per = c.num_layers // world
    r = ps.get_pipeline_model_parallel_rank()
    with torch.no_grad():
        for i, L in enumerate(stage.layers):
            L.load_state_dict(full.layers[r * per + i].state_dict())
        if stage.pre_process:
            stage.word_embeddings.weight.copy_(full.word_embeddings.weight)
            stage.position_embeddings.weight.copy_(full.position_embeddings.weight)
        if stage.post_process:
            stage.final_layernorm.load_state_dict(full.final_layernorm.state_dict())
    sync_initial_embeddings(stage)
    torch.testing.assert_close(stage.word_embeddings.weight, full.word_embeddings.weight)
    ids = torch.randint(0, c.vocab_size, (n_micro * mb, 16), generator=torch.Generator().manual_seed(3))

    def fwd_step(batch, m):
        out = m(batch, batch if ps.is_pipeline_last_stage() else None)

        def loss_fn(o):
            return o, {"loss": o.detach()}

        return out, loss_fn

    fb = get_forward_backward_func(None, world)
    losses = fb(fwd_step, ids, stage, forward_only=False, tensor_shape=(mb, 16, c.hidden_size),
                dtype=torch.float32)
    sync_embedding_grads(stage)
    total = 0.0
    for chunk in ids.chunk(n_micro):
        loss = full(chunk, chunk) / n_micro
        loss.backward()
        total += float(loss)
    for i, L in enumerate(stage.layers):
        ref = full.layers[r * per + i]
        for (n, p), (_, q) in zip(L.named_parameters(), ref.named_parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-5, msg=n)
    torch.testing.assert_close(stage.word_embeddings.weight.grad, full.word_embeddings.weight.grad,
                               rtol=1e-4, atol=1e-6)
    if ps.is_pipeline_last_stage():
        assert abs(sum(float(l["loss"]) for l in losses) / n_micro - total) < 1e-5


def test_megatron_gpt_pipeline_parallel():
    _spawn(_megatron_pp, 2)
