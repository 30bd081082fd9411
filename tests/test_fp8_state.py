"""apex.fp8 bookkeeping on the CPU (no kernels): recipe validation, slot allocation and growth,
the autocast / global switches, amp.initialize(fp8=...) wiring and the checkpoint format.
The kernels and the training path are covered on the GPU by tests/test_fp8_gpu.py."""
import pytest
import torch

from apex import fp8


@pytest.fixture(autouse=True)
def _reset():
    fp8.disable()
    yield
    fp8.disable()


def test_recipe_formats():
    r = fp8.Fp8Recipe()
    assert (r.fmt("fwd"), r.fmt("bwd")) == (fp8.E4M3, fp8.E5M2)
    with pytest.raises(ValueError):
        fp8.Fp8Recipe(fwd_format="e3m4").fmt("fwd")


def test_slots_grow_and_keep_values():
    st = fp8.Fp8State(fp8.Fp8Recipe(amax_history_len=4), device="cpu")
    keys = [(i, "x") for i in range(300)]
    for i, k in enumerate(keys):
        s = st.slot(k, fp8.E4M3 if i % 2 == 0 else fp8.E5M2)
        st.scale[s] = float(i + 1)
    assert st.n == 300 and st._cap >= 300 and st.hist.shape == (st._cap, 4)
    for i, k in enumerate(keys):
        s = st.slots[k]
        assert float(st.scale[s]) == i + 1
        assert float(st.fmax[s]) == (448.0 if i % 2 == 0 else 57344.0)
    assert st.slot(keys[5], fp8.E4M3) == st.slots[keys[5]]  # stable


def test_autocast_and_global_switch():
    assert fp8.active() is None
    with fp8.fp8_autocast(device="cpu") as st:
        assert fp8.active() is st
        with fp8.fp8_autocast(device="cpu"):
            assert fp8.active() is st  # same recipe: same state
        assert fp8.active() is st
    assert fp8.active() is None
    with fp8.fp8_autocast(enabled=False):
        assert fp8.active() is None
    st = fp8.enable(device="cpu")
    assert fp8.active() is st
    fp8.disable()
    assert fp8.active() is None


def test_new_recipe_resets_state():
    a = fp8.state(fp8.Fp8Recipe(), device="cpu")
    assert fp8.state(fp8.Fp8Recipe(), device="cpu") is a  # equal recipe
    b = fp8.state(fp8.Fp8Recipe(margin=1), device="cpu")
    assert b is not a and b.smax_scale == 0.5


def test_amp_initialize_fp8_flag_and_step_hook():
    from apex import amp
    from apex.amp._amp_state import _amp_state

    _amp_state.optimizers, _amp_state.loss_scalers = [], []
    model = torch.nn.Linear(8, 8)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model, opt = amp.initialize(model, opt, opt_level="O0", verbosity=0, fp8=True)
    st = fp8.active()
    assert st is not None and _amp_state.fp8
    model(torch.randn(2, 8)).sum().backward()
    opt.step()
    assert st.steps == 1 and st.gen == 1  # the patched step ran apex.fp8.step()
    _amp_state.optimizers, _amp_state.loss_scalers = [], []
    model2 = torch.nn.Linear(8, 8)
    opt2 = torch.optim.SGD(model2.parameters(), lr=0.1)
    amp.initialize(model2, opt2, opt_level="O0", verbosity=0)
    assert fp8.active() is None  # re-initialising without fp8 turns it off


def test_state_dict_by_parameter_name():
    lin = torch.nn.Linear(4, 4)
    st = fp8.Fp8State(device="cpu")
    kw = st.key_of(lin.weight)
    sw = st.slot((kw, "w"), fp8.E4M3)
    sx = st.slot((kw, "x"), fp8.E4M3)
    st.slot((12345, "x"), fp8.E4M3)  # not a parameter of lin: dropped from the named dict
    st.scale[sx] = 3.0
    st.hist[sx, 0] = 7.0
    st._fresh.discard(sx)
    sd = st.state_dict(lin)
    assert set(sd["slots"]) == {"weight:w", "weight:x"}
    st2 = fp8.Fp8State(device="cpu")
    st2.load_state_dict(sd, lin)
    k2 = st2.key_of(lin.weight)
    s2 = st2.slots[(k2, "x")]
    assert float(st2.scale[s2]) == 3.0 and float(st2.hist[s2, 0]) == 7.0
    assert s2 not in st2._fresh and st2.slots[(k2, "w")] in st2._fresh
    del sw


def test_slot_keys_survive_id_reuse_and_recycle():
    """Slots are keyed by a counter stored on the tensor, not id(): a tensor re-created every
    step (an O1 cast) reuses the freed slot instead of growing the buffers, and a new tensor never
    inherits a dead one's scale history. A freed slot is reusable only after the next step()
    boundary (_recycle_slots), in sorted order, so every rank of the amax reduction group reuses
    slots in the same order (the timing still depends on when each rank frees the tensor: see
    Fp8State._release)."""
    st = fp8.Fp8State(device="cpu")
    for step in range(50):
        w = torch.randn(4, 4)  # a fresh per-step weight copy
        s = st.slot((st.key_of(w), "x"), fp8.E4M3)
        assert s in st._fresh  # new tensor: fresh (current scaling), no inherited history
        st.scale[s] = 5.0
        del w
        w2 = torch.randn(4, 4)  # created after w died, same step: must not get w's slot yet
        assert st.slot((st.key_of(w2), "x"), fp8.E4M3) != s
        del w2
        st._recycle_slots()  # the step boundary
    assert st.n == 2  # two slots, recycled 50 times
    keep = torch.randn(4, 4)
    sk = st.slot((st.key_of(keep), "x"), fp8.E4M3)
    assert float(st.scale[sk]) == 1.0  # the recycled slot was reset


def test_amax_reduction_defaults_to_data_parallel_group(monkeypatch):
    from apex.transformer import parallel_state as ps

    st = fp8.Fp8State(device="cpu")
    sentinel = object()
    monkeypatch.setattr(ps, "model_parallel_is_initialized", lambda: True)
    monkeypatch.setattr(ps, "get_data_parallel_group", lambda: sentinel)
    assert st.reduction_group() is sentinel
    explicit = object()
    st2 = fp8.Fp8State(fp8.Fp8Recipe(amax_reduction_group=explicit), device="cpu")
    assert st2.reduction_group() is explicit


def _mismatch_worker(rank, world, port, q):
    import os
    import traceback

    import torch.distributed as dist

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        st = fp8.Fp8State(device="cpu")
        ws = [torch.randn(2, 2) for _ in range(2 + rank)]  # rank 1 quantises one tensor more
        for w in ws:
            st.slot((st.key_of(w), "x"), fp8.E4M3)
        st.amax[: st.n] = torch.arange(st.n, dtype=torch.float32) + rank
        try:
            st._reduce_amax(None)
            q.put((rank, "no error"))
        except RuntimeError as e:
            q.put((rank, "ok" if "slot counts differ" in str(e) else str(e)))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_amax_reduction_detects_slot_mismatch():
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_mismatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=30)
    assert all(r[1] == "ok" for r in res), res


def test_wgrad_split_policy():
    """fp8 weight-gradient slices: fewest workgroup rounds per token (ceil(tiles x slices / 256) / slices), each slice a
    whole number of 128-token K-tiles and at least 1024 tokens (BERT-Large at 98304 tokens)."""
    sp = fp8._f8_wgrad_splits
    assert sp(98304, 4096, 1024) == 4  # 64 tiles
    assert sp(98304, 1024, 4096) == 4
    assert sp(98304, 3072, 1024) == 16  # 48 tiles: 3 full rounds beat 1.5 (8) and 0.75 (4)
    assert sp(98304, 1024, 1024) == 16  # 16 tiles
    assert sp(2048, 1024, 1024) == 2  # slices stay >= 1024 tokens
    assert sp(384, 256, 256) == 1


def test_operand_codes_match_the_consumed_tensor():
    """operand_codes hands back the last fp8 GEMM's codes only for the tensor that GEMM consumed
    (same bytes: address + shape of the held operand, unmodified since), once; a mismatch, an
    in-place write in between, a declined GEMM or a second call gets None."""
    st = fp8.Fp8State(device="cpu")
    a = torch.zeros(4, 8)
    codes, inv = torch.zeros(4, 8, dtype=torch.uint8), torch.ones(1)
    st._last = st._remember(a, codes, inv)
    assert st.operand_codes(torch.zeros(4, 8)) is None  # another tensor
    st._last = st._remember(a, codes, inv)
    assert st.operand_codes(a.view(8, 4)) is None  # same storage, other shape
    st._last = st._remember(a, codes, inv)
    got = st.operand_codes(a.view(4, 8))  # a fresh view of the same bytes (what the blocks pass)
    assert got[0] is codes and got[1] is inv
    assert st.operand_codes(a) is None  # taken
    st._last = st._remember(a, codes, inv)
    a.add_(1)  # written in place after its codes were taken: stale codes
    assert st.operand_codes(a) is None
    st._last = st._remember(a, codes, inv)
    st.step()
    assert st.operand_codes(a) is None  # a step boundary drops it
    # a GEMM the fp8 path declines clears the claim (a later tensor reusing the address gets nothing)
    st._last = st._remember(a, codes, inv)
    assert st.forward_gemm(torch.zeros(4, 100), torch.zeros(8, 100), 0) is None
    assert st._last is None


def test_wgrad_declines_without_recipe_or_codes():
    st = fp8.Fp8State(fp8.Fp8Recipe(fp8_wgrad=False), device="cpu")
    c = (torch.zeros(256, 256, dtype=torch.uint8), torch.ones(1))
    assert st.wgrad(c, c, torch.bfloat16) is None
    st2 = fp8.Fp8State(device="cpu")
    assert st2.wgrad(None, c, torch.bfloat16) is None
