"""apex DDP over RCCL on the GPU with a one-rank process group: the bucket collectives really
run (``single_rank_collectives``), on the reduction streams, through ncclAvg / fp32 staging /
several communicators, and the gradients equal the plain single-GPU gradients. This exercises
the RCCL code path of the 8-GPU scaling run on a one-GPU box."""
import socket

import pytest
import torch
import torch.distributed as dist


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def rccl_one_rank():
    if not dist.is_initialized():
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [{}, {"allreduce_always_fp32": True}, {"num_allreduce_streams": 2},
                                  {"delay_allreduce": True}, {"gradient_predivide_factor": 4.0}])
def test_ddp_rccl_single_rank_matches_plain(rccl_one_rank, opts):
    from apex.parallel import DistributedDataParallel as DDP

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64)).cuda().bfloat16()
    ref = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 64)).cuda().bfloat16()
    ref.load_state_dict(net.state_dict())
    model = DDP(net, message_size=4096, comm_timing=True, **opts)
    model.single_rank_collectives = True
    assert dist.get_backend() == "nccl" and model.reduction_stream is not None
    for it in range(3):
        x = torch.randn(32, 64, device="cuda", dtype=torch.bfloat16)
        model.zero_grad()
        model(x).float().square().mean().backward()
        ref.zero_grad()
        ref(x).float().square().mean().backward()
        for p, q in zip(net.parameters(), ref.parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-2, atol=1e-3)
    st = model.comm_stats()
    assert st["backend"] == "nccl" and st["num_buckets"] >= 2
    if not opts.get("delay_allreduce"):
        assert len(st["bucket_ready_to_reduced_ms"]) == st["num_buckets"]
        assert st["exposed_comm_samples"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("delay", [False, True])
def test_fused_producers_write_into_bucket_slots(rccl_one_rank, delay):
    """A small BERT under apex DDP + FusedAdam (zero_grad releases the bucket views): the fused
    blocks write every weight / bias / LayerNorm / embedding gradient straight into its bucket
    slot (grad_target), autograd adopts the slot as p.grad without a copy, and the gradients over
    three steps (plus a no_sync accumulation step) equal the same model's without DDP."""
    from apex.models.bert import BertConfig, BertForPreTraining, synthetic_batch
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    cfg = BertConfig(vocab_size=1000, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=1024, max_position_embeddings=128, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    net = BertForPreTraining(cfg).cuda().bfloat16()
    ref = BertForPreTraining(cfg).cuda().bfloat16()
    ref.load_state_dict(net.state_dict())
    model = DDP(net, message_size=1 << 20, delay_allreduce=delay)
    opt = FusedAdam(net.parameters(), lr=0.0)  # lr 0: the weights stay equal to ref's
    g = torch.Generator(device="cuda").manual_seed(1)
    batches = [synthetic_batch(cfg, 8, 64, device="cuda", generator=g) for _ in range(4)]
    names = [n for n, _ in net.named_parameters()]
    for it, b in enumerate(batches[:3]):
        opt.zero_grad()
        model(**b).backward()
        ref.zero_grad(set_to_none=True)
        ref(**b).backward()
        for n, p, q in zip(names, net.parameters(), ref.parameters()):
            assert p.grad is not None, n
            if it > 0:  # from the second step the layout exists: every grad lives in its slot
                assert getattr(p, "_apex_grad_is_bucket_view", False)
                flat = p._apex_bucket_flat
                lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * flat.element_size()
                assert lo <= p.grad.data_ptr() < hi, n
            torch.testing.assert_close(p.grad.float(), q.grad.float(), rtol=2e-2, atol=2e-3, msg=n)
        opt.step()
    # gradient accumulation: micro-batch 1 under no_sync, micro-batch 2 reduces
    opt.zero_grad()
    with model.no_sync():
        model(**batches[0]).backward()
    model(**batches[3]).backward()
    ref.zero_grad(set_to_none=True)
    ref(**batches[0]).backward()
    ref(**batches[3]).backward()
    for n, p, q in zip(names, net.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad.float(), q.grad.float(), rtol=2e-2, atol=4e-3, msg=n)


@pytest.mark.gpu
def test_gpt_layernorm_and_bias_grads_written_into_slots(rccl_one_rank):
    """The GPT-2 block's FusedLayerNorm weight/bias, fused-dense bias and bias-dropout-add bias
    gradients are written by their HIP backward kernels straight into the DDP bucket slots
    (ln_bwd / colsum / bias_dropout_add_bwd outputs), and every gradient over two steps equals
    the same model's without DDP (tied embedding / LM-head weight included)."""
    from apex.models.gpt import GPTConfig, GPTModel, synthetic_batch
    from apex.optimizers import FusedAdam
    from apex.parallel import DistributedDataParallel as DDP

    cfg = GPTConfig.tiny()
    cfg.dropout = 0.0
    torch.manual_seed(0)
    net = GPTModel(cfg).cuda().bfloat16()
    ref = GPTModel(cfg).cuda().bfloat16()
    ref.load_state_dict(net.state_dict())
    model = DDP(net, message_size=1 << 20)
    opt = FusedAdam(net.parameters(), lr=0.0)
    g = torch.Generator(device="cuda").manual_seed(2)
    batches = [synthetic_batch(cfg, 4, 64, device="cuda", generator=g) for _ in range(2)]
    names = [n for n, _ in net.named_parameters()]
    for it, b in enumerate(batches):
        opt.zero_grad()
        model(**b).backward()
        ref.zero_grad(set_to_none=True)
        ref(**b).backward()
        for n, p, q in zip(names, net.parameters(), ref.parameters()):
            assert p.grad is not None, n
            if it > 0:
                flat = p._apex_bucket_flat
                lo, hi = flat.data_ptr(), flat.data_ptr() + flat.numel() * flat.element_size()
                assert lo <= p.grad.data_ptr() < hi, n
            torch.testing.assert_close(p.grad.float(), q.grad.float(), rtol=2e-2, atol=3e-3, msg=n)
        opt.step()
