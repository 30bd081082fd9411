"""BASELINE config 5's layout — Megatron GPT at tensor-parallel 4 x pipeline-parallel 2 — as 8
gloo ranks on the CPU, against the same network run serially: the pipelined, sharded loss and
every parameter gradient (gathered back from the TP shards) must equal the serial ones.

This is the multi-rank code path of the 8-GPU run (TP mappings, vocab-parallel embedding and
cross entropy, 1F1B p2p exchange, tied-embedding gradient sync over the embedding group,
DP all-reduce on apex DDP buckets) rehearsed without GPUs.
"""
import os
import socket
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

TP, PP = 4, 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_wrap, args=(fn, r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] == "ok" for r in res), res


def _wrap(fn, rank, world, port, q, *args):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.set_num_threads(1)
        fn(rank, world, *args)
        q.put((rank, "ok"))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        from apex.transformer import parallel_state as ps

        ps.destroy_model_parallel()
        dist.destroy_process_group()


def _tp_gather(t, dim):
    from apex.transformer import parallel_state as ps

    g = ps.get_tensor_model_parallel_group()
    parts = [torch.empty_like(t) for _ in range(TP)]
    dist.all_gather(parts, t.detach().contiguous(), group=g)
    return torch.cat(parts, dim)


def _layer_full(L, c, attr):
    """One decoder layer's tensors (weights or grads) in the serial layout."""
    H, nh = c.hidden_size, c.num_attention_heads
    d = H // nh
    get = (lambda p: p.detach()) if attr == "data" else (lambda p: p.grad.detach())
    wq = _tp_gather(get(L.query_key_value.weight), 0).view(TP, 3, nh // TP, d, H).transpose(0, 1).reshape(3 * H, H)
    bq = _tp_gather(get(L.query_key_value.bias), 0).view(TP, 3, nh // TP, d).transpose(0, 1).reshape(3 * H)
    return dict(ln1=(get(L.input_layernorm.weight), get(L.input_layernorm.bias)), wq=wq, bq=bq,
                wd=_tp_gather(get(L.dense.weight), 1), bd=get(L.dense.bias),
                ln2=(get(L.post_attention_layernorm.weight), get(L.post_attention_layernorm.bias)),
                w1=_tp_gather(get(L.dense_h_to_4h.weight), 0), b1=_tp_gather(get(L.dense_h_to_4h.bias), 0),
                w2=_tp_gather(get(L.dense_4h_to_h.weight), 1), b2=get(L.dense_4h_to_h.bias))


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


def _tp4_pp2(rank, world):
    from apex.models.megatron_gpt import MegatronGPTConfig, build_stage, sync_embedding_grads, sync_initial_embeddings
    from apex.transformer import parallel_state as ps
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator

    ps.initialize_model_parallel(TP, PP)
    assert ps.get_data_parallel_world_size() == world // (TP * PP)
    n_micro, mb, S = 4, 2, 16
    setup_microbatch_calculator(rank, None, n_micro * mb, mb, 1)
    c = MegatronGPTConfig.tiny()  # 4 layers, hidden 128, 4 heads
    c.hidden_dropout = c.attention_dropout = 0.0
    torch.manual_seed(100 + rank)  # every shard different; replicated params synced below
    stage = build_stage(c)
    with torch.no_grad():
        for n, p in stage.named_parameters():
            if p.ndim == 1:
                p.add_(torch.randn(p.shape) * 0.05)
    tp_src, tp_group = ps.get_tensor_model_parallel_src_rank(), ps.get_tensor_model_parallel_group()
    for n, p in stage.named_parameters():  # params replicated across the TP group
        if not getattr(p, "tensor_model_parallel", False):
            dist.broadcast(p.data, tp_src, group=tp_group)
    sync_initial_embeddings(stage)
    ids = torch.randint(0, c.vocab_size, (n_micro * mb, S), generator=torch.Generator().manual_seed(3))

    def fwd_step(batch, m):
        out = m(batch, batch if ps.is_pipeline_last_stage() else None)
        return out, (lambda o: (o, {"loss": o.detach()}))

    fb = get_forward_backward_func(None, PP)
    losses = fb(fwd_step, ids, stage, forward_only=False, tensor_shape=(mb, S, c.hidden_size), dtype=torch.float32)
    sync_embedding_grads(stage)

    # ---- serial reference from the gathered weights of both stages
    mine = {"layers": [_layer_full(L, c, "data") for L in stage.layers]}
    if stage.pre_process:
        mine["E"] = _tp_gather(stage.word_embeddings.weight.detach(), 0)
        mine["P"] = stage.position_embeddings.weight.detach()
    if stage.post_process:
        mine["lnf"] = (stage.final_layernorm.weight.detach(), stage.final_layernorm.bias.detach())
    allw = [None] * world
    dist.all_gather_object(allw, (ps.get_pipeline_model_parallel_rank(), ps.get_tensor_model_parallel_rank(), mine))
    st = {s: w for s, t, w in allw if t == 0}
    W = {"E": st[0]["E"], "P": st[0]["P"], "lnf": st[PP - 1]["lnf"],
         "layers": [L for s in range(PP) for L in st[s]["layers"]]}
    leaves = []

    def req(t):
        t = t.clone().requires_grad_(True)
        leaves.append(t)
        return t

    W = {"E": req(W["E"]), "P": req(W["P"]), "lnf": tuple(req(t) for t in W["lnf"]),
         "layers": [{k: (tuple(req(t) for t in v) if isinstance(v, tuple) else req(v)) for k, v in L.items()}
                    for L in W["layers"]]}
    total = 0.0
    for chunk in ids.chunk(n_micro):
        loss = _serial_loss(W, chunk, c) / n_micro
        loss.backward()
        total += float(loss.detach())
    if ps.is_pipeline_last_stage():
        got = sum(float(l["loss"]) for l in losses) / n_micro
        assert abs(got - total) < 1e-4, (got, total)
    # ---- gradients: this stage's shards, gathered to the serial layout
    per = c.num_layers // PP
    r = ps.get_pipeline_model_parallel_rank()
    for i, L in enumerate(stage.layers):
        g = _layer_full(L, c, "grad")
        ref = W["layers"][r * per + i]
        for k, v in g.items():
            rv = ref[k]
            if isinstance(v, tuple):
                for a, b in zip(v, rv):
                    torch.testing.assert_close(a, b.grad, rtol=2e-4, atol=2e-5, msg=f"layer {i} {k}")
            else:
                torch.testing.assert_close(v, rv.grad, rtol=2e-4, atol=2e-5, msg=f"layer {i} {k}")
    # tied word embedding: both stages hold the sum of the embedding and LM-head gradients
    ge = _tp_gather(stage.word_embeddings.weight.grad.detach(), 0)
    torch.testing.assert_close(ge, W["E"].grad, rtol=2e-4, atol=2e-5)
    if stage.pre_process:
        torch.testing.assert_close(stage.position_embeddings.weight.grad, W["P"].grad, rtol=2e-4, atol=2e-5)


def test_megatron_gpt_tp4_pp2_matches_serial():
    _spawn(_tp4_pp2, TP * PP)
