"""apex.transformer (NS-08) on CPU/gloo: TP layers, vocab-parallel embedding + CE, 1F1B pipeline
schedule vs single-process references; fused scale-mask softmax kernels on GPU."""
import os
import socket
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F


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
    ps = [ctx.Process(target=_wrap, args=(fn, r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
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


def _tp_layers(rank, world):
    from apex.transformer import parallel_state as ps
    from apex.transformer import tensor_parallel as tp

    ps.initialize_model_parallel(world, 1)
    assert ps.get_tensor_model_parallel_world_size() == world
    torch.manual_seed(0)
    col = tp.ColumnParallelLinear(8, 16, gather_output=False, keep_master_weight_for_test=True)
    torch.manual_seed(1)
    row = tp.RowParallelLinear(16, 6, input_is_parallel=True, keep_master_weight_for_test=True)
    with torch.no_grad():
        col.bias.uniform_(-1, 1)
        row.bias.uniform_(-1, 1)
    cb = [torch.empty_like(col.bias) for _ in range(world)]
    dist.all_gather(cb, col.bias.detach().contiguous())
    cb = torch.cat(cb)
    torch.manual_seed(5)
    x = torch.randn(4, 8, requires_grad=True)
    h, _ = col(x)
    y, _ = row(torch.relu(h))
    xr = x.detach().clone().requires_grad_(True)
    yr = F.linear(torch.relu(F.linear(xr, col.master_weight, cb)), row.master_weight, row.bias.detach())
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    y.sum().backward()
    yr.sum().backward()
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-5, atol=1e-5)

    # vocab-parallel embedding and cross entropy
    torch.manual_seed(2)
    emb = tp.VocabParallelEmbedding(12, 5)
    parts = [torch.empty_like(emb.weight) for _ in range(world)]
    dist.all_gather(parts, emb.weight.detach().contiguous())
    W = torch.cat(parts)
    ids = torch.tensor([[0, 3, 11], [7, 6, 1]])
    torch.testing.assert_close(emb(ids), F.embedding(ids, W))
    torch.manual_seed(3)
    logits = torch.randn(2, 3, 12)
    target = torch.randint(0, 12, (2, 3))
    per = 12 // world
    local = logits[..., rank * per:(rank + 1) * per].clone().requires_grad_(True)
    loss = tp.vocab_parallel_cross_entropy(local, target)
    ref = F.cross_entropy(logits.view(-1, 12), target.view(-1), reduction="none").view(2, 3)
    torch.testing.assert_close(loss, ref, rtol=1e-5, atol=1e-5)
    loss.sum().backward()
    lr = logits.clone().requires_grad_(True)
    F.cross_entropy(lr.view(-1, 12), target.view(-1), reduction="sum").backward()
    torch.testing.assert_close(local.grad, lr.grad[..., rank * per:(rank + 1) * per], rtol=1e-5, atol=1e-5)
    # label smoothing
    ls = tp.vocab_parallel_cross_entropy(logits[..., rank * per:(rank + 1) * per], target, 0.1)
    refs = F.cross_entropy(logits.view(-1, 12), target.view(-1), reduction="none",
                           label_smoothing=0.1 * 12 / 11).view(2, 3)
    torch.testing.assert_close(ls, refs, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("world", [2, 4])
def test_tensor_parallel_layers(world):
    _spawn(_tp_layers, world)


class _Stage(torch.nn.Module):
    wide = False  # emit fp64 (wider than the fp32 wire dtype), as amp O2 does with fp32 outputs

    def __init__(self, w):
        super().__init__()
        self.lin = torch.nn.Linear(6, 6)
        with torch.no_grad():
            self.lin.weight.copy_(w[0])
            self.lin.bias.copy_(w[1])
        self.input_tensor = None

    def set_input_tensor(self, t):
        self.input_tensor = t

    def forward(self, x):
        inp = x if self.input_tensor is None else self.input_tensor
        out = torch.tanh(self.lin(inp))
        return out.double() if self.wide else out


def _pipeline(rank, world, n_micro, wide=False):
    from apex.transformer import parallel_state as ps
    from apex.transformer.pipeline_parallel import get_forward_backward_func, setup_microbatch_calculator

    ps.initialize_model_parallel(1, world)
    setup_microbatch_calculator(rank, None, n_micro * 2, 2, 1)
    torch.manual_seed(0)
    weights = [(torch.randn(6, 6) * 0.5, torch.randn(6) * 0.1) for _ in range(world)]
    data = torch.randn(n_micro * 2, 6)
    target = torch.randn(n_micro * 2, 6)
    stage = ps.get_pipeline_model_parallel_rank()
    model = _Stage(weights[stage])
    model.wide = wide
    tgt_chunks = list(target.chunk(n_micro))
    state = {"i": 0}

    def fwd_step(batch, m):
        out = m(batch)
        t = tgt_chunks[state["i"] % n_micro]
        if ps.is_pipeline_last_stage():
            state["i"] += 1

        def loss_fn(o):
            o = o.float()
            return F.mse_loss(o, t), {"loss": F.mse_loss(o, t).detach()}

        return out, loss_fn

    fb = get_forward_backward_func(None, world)
    losses = fb(fwd_step, data, model, forward_only=False, tensor_shape=(2, 6), dtype=torch.float32)
    # single-process reference
    ref = [_Stage(w) for w in weights]
    total = 0.0
    for xb, tb in zip(data.chunk(n_micro), target.chunk(n_micro)):
        h = xb
        for s in ref:
            h = s(h)
        loss = F.mse_loss(h, tb) / n_micro
        loss.backward()
        total += float(loss)
    torch.testing.assert_close(model.lin.weight.grad, ref[stage].lin.weight.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(model.lin.bias.grad, ref[stage].lin.bias.grad, rtol=1e-5, atol=1e-6)
    if ps.is_pipeline_last_stage():
        assert len(losses) == n_micro
        assert abs(sum(float(l["loss"]) for l in losses) / n_micro - total) < 1e-5


@pytest.mark.parametrize("world,n_micro", [(2, 4), (4, 6), (4, 2)])
def test_pipeline_1f1b_matches_serial(world, n_micro):
    _spawn(_pipeline, world, n_micro)


def test_pipeline_stage_output_wider_than_wire_dtype():
    """A stage whose output dtype differs from the agreed p2p dtype still exchanges correctly."""
    _spawn(_pipeline, 2, 4, True)


def _groups(rank, world):
    from apex.transformer import parallel_state as ps

    ps.initialize_model_parallel(2, 2)
    assert ps.get_tensor_model_parallel_world_size() == 2
    assert ps.get_pipeline_model_parallel_world_size() == 2
    assert ps.get_data_parallel_world_size() == world // 4
    assert ps.get_tensor_model_parallel_src_rank() == (rank // 2) * 2
    assert ps.is_pipeline_first_stage() == (rank < world // 2)


def test_parallel_state_groups():
    _spawn(_groups, 8)


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("sk", [128, 1024, 2048])
@pytest.mark.parametrize("kind", ["causal", "padding", "none"])
def test_fused_scale_mask_softmax(dt, sk, kind):
    from apex.transformer.enums import AttnMaskType
    from apex.transformer.functional import FusedScaleMaskSoftmax

    torch.manual_seed(sk)
    b, h = 2, 3
    sq = sk
    x = torch.randn(b, h, sq, sk, device="cuda").to(dt).requires_grad_(True)
    mask = None
    if kind == "padding":
        mask = torch.rand(b, 1, sq, sk, device="cuda") > 0.8

    def mask_func(s, m):
        return s.masked_fill(m, -10000.0)

    mt = AttnMaskType.causal if kind == "causal" else AttnMaskType.padding
    m = FusedScaleMaskSoftmax(dt == torch.float16, dt == torch.bfloat16, mt, True, mask_func, True, 0.125)
    y = m(x, mask)
    ref = FusedScaleMaskSoftmax(dt == torch.float16, dt == torch.bfloat16, mt, False, mask_func, True, 0.125)
    xr = x.detach().clone().requires_grad_(True)
    yr = ref(xr, mask)
    tol = 2e-2 if dt == torch.bfloat16 else 3e-3
    torch.testing.assert_close(y.float(), yr.float(), rtol=tol, atol=tol)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    torch.testing.assert_close(x.grad.float(), xr.grad.float(), rtol=tol * 2, atol=tol * 2)
