"""Model-parallel process groups (NS-08): tensor (TP), pipeline (PP) and data (DP) parallel.

Rank layout (Megatron convention, chosen for 8x MI355X on a fully connected xGMI mesh):
TP groups are runs of ``tp`` consecutive ranks, PP groups stride by ``world / pp``, DP
groups take the ranks with equal (tp rank, pp stage). With TP=4, PP=2 on 8 GPUs the two
TP groups {0..3} and {4..7} each own 6 direct xGMI links, so the per-layer TP all-reduces
never share a link with the other group, and the PP send/recv between stage peers
(i, i+4) is a single direct link.
All collectives go through torch.distributed (RCCL on ROCm; gloo on CPU for tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_TENSOR_MODEL_PARALLEL_GROUP = None
_PIPELINE_MODEL_PARALLEL_GROUP = None
_MODEL_PARALLEL_GROUP = None
_EMBEDDING_GROUP = None
_POSITION_EMBEDDING_GROUP = None
_DATA_PARALLEL_GROUP = None
_EMBEDDING_GLOBAL_RANKS = None
_PIPELINE_GLOBAL_RANKS = None
_DATA_PARALLEL_GLOBAL_RANKS = None
_TENSOR_GLOBAL_RANKS = None
_CONTEXT_PARALLEL_GROUP = None
_CONTEXT_PARALLEL_GLOBAL_RANKS = None

_VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = None
_VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
_PIPELINE_MODEL_PARALLEL_SPLIT_RANK = None

_MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = None
_MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
_MPU_TENSOR_MODEL_PARALLEL_RANK = None
_MPU_PIPELINE_MODEL_PARALLEL_RANK = None


def is_unitialized():
    return _DATA_PARALLEL_GROUP is None


def initialize_model_parallel(tensor_model_parallel_size_=1, pipeline_model_parallel_size_=1,
                              virtual_pipeline_model_parallel_size_=None,
                              pipeline_model_parallel_split_rank_=None, *, default_backend=None,
                              p2p_backend=None, context_parallel_size_=1):
    """Create TP / PP / DP / embedding groups over the already-initialised default group.

    ``context_parallel_size_`` (cp > 1): each DP group is further cut into runs of ``cp``
    consecutive DP ranks that shard the SEQUENCE of one sample (apex.transformer.context_parallel:
    ring / Ulysses attention over these groups). The DP group keeps every CP rank, so the gradient
    all-reduce over it sums the sequence shards' contributions (Megatron's dp x cp reduction); the
    number of distinct data replicas is dp / cp. With TP = 4 the DP peers of a rank are 4 ranks
    apart, each pair on its own direct xGMI link, so the CP ring's p2p hops never share a link
    with the TP all-reduces."""
    assert dist.is_initialized()
    world_size = dist.get_world_size()
    tp = min(tensor_model_parallel_size_, world_size)
    pp = min(pipeline_model_parallel_size_, world_size)
    if world_size % (tp * pp) != 0:
        raise RuntimeError("world_size ({}) is not divisible by tensor_model_parallel_size ({}) x "
                           "pipeline_model_parallel_size ({})".format(world_size, tp, pp))
    dp = world_size // (tp * pp)
    num_tp_groups = world_size // tp
    num_pp_groups = world_size // pp
    rank = dist.get_rank()

    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK, _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    if virtual_pipeline_model_parallel_size_ is not None:
        assert pp > 1, "interleaved schedule needs pipeline_model_parallel_size > 1"
        _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = 0
        _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = virtual_pipeline_model_parallel_size_
    global _PIPELINE_MODEL_PARALLEL_SPLIT_RANK
    _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = pipeline_model_parallel_split_rank_

    kw = {} if default_backend is None else {"backend": default_backend}

    global _DATA_PARALLEL_GROUP, _DATA_PARALLEL_GLOBAL_RANKS
    assert _DATA_PARALLEL_GROUP is None, "data parallel group is already initialized"
    for i in range(pp):
        start, end = i * num_pp_groups, (i + 1) * num_pp_groups
        for j in range(tp):
            ranks = list(range(start + j, end, tp))
            g = dist.new_group(ranks, **kw)
            if rank in ranks:
                _DATA_PARALLEL_GROUP = g
                _DATA_PARALLEL_GLOBAL_RANKS = ranks

    global _CONTEXT_PARALLEL_GROUP, _CONTEXT_PARALLEL_GLOBAL_RANKS
    cp = int(context_parallel_size_ or 1)
    if dp % cp != 0:
        raise RuntimeError("data-parallel size ({}) is not divisible by context_parallel_size ({})".format(dp, cp))
    assert _CONTEXT_PARALLEL_GROUP is None, "context parallel group is already initialized"
    for dp_ranks in _dp_rank_table(world_size, tp, pp):
        for c in range(0, dp, cp):
            ranks = dp_ranks[c:c + cp]
            g = dist.new_group(ranks, **kw) if cp > 1 else None
            if rank in ranks:
                _CONTEXT_PARALLEL_GROUP = g if cp > 1 else _SINGLETON
                _CONTEXT_PARALLEL_GLOBAL_RANKS = ranks

    global _MODEL_PARALLEL_GROUP
    for i in range(dp):
        ranks = [dp_ranks[i] for dp_ranks in _dp_rank_table(world_size, tp, pp)]
        g = dist.new_group(ranks, **kw)
        if rank in ranks:
            _MODEL_PARALLEL_GROUP = g

    global _TENSOR_MODEL_PARALLEL_GROUP, _TENSOR_GLOBAL_RANKS
    for i in range(num_tp_groups):
        ranks = list(range(i * tp, (i + 1) * tp))
        g = dist.new_group(ranks, **kw)
        if rank in ranks:
            _TENSOR_MODEL_PARALLEL_GROUP = g
            _TENSOR_GLOBAL_RANKS = ranks

    global _PIPELINE_MODEL_PARALLEL_GROUP, _PIPELINE_GLOBAL_RANKS, _EMBEDDING_GROUP
    global _EMBEDDING_GLOBAL_RANKS, _POSITION_EMBEDDING_GROUP
    pkw = kw if p2p_backend is None else {"backend": p2p_backend}
    for i in range(num_pp_groups):
        ranks = list(range(i, world_size, num_pp_groups))
        g = dist.new_group(ranks, **pkw)
        if rank in ranks:
            _PIPELINE_MODEL_PARALLEL_GROUP = g
            _PIPELINE_GLOBAL_RANKS = ranks
        if len(ranks) > 1:
            emb = [ranks[0], ranks[-1]]
            pos = [ranks[0]]
            if pipeline_model_parallel_split_rank_ is not None and \
                    ranks[pipeline_model_parallel_split_rank_] not in emb:
                emb = [ranks[0], ranks[pipeline_model_parallel_split_rank_], ranks[-1]]
                pos = [ranks[0], ranks[pipeline_model_parallel_split_rank_]]
        else:
            emb, pos = ranks, ranks
        eg = dist.new_group(emb, **kw)
        pg = dist.new_group(pos, **kw)
        if rank in emb:
            _EMBEDDING_GROUP = eg
        if rank in ranks:
            _EMBEDDING_GLOBAL_RANKS = emb
        if rank in pos:
            _POSITION_EMBEDDING_GROUP = pg


_SINGLETON = object()  # cp = 1: no group is created (every rank holds its whole sequence)


def _dp_rank_table(world_size, tp, pp):
    num_pp_groups = world_size // pp
    table = []
    for i in range(pp):
        start, end = i * num_pp_groups, (i + 1) * num_pp_groups
        for j in range(tp):
            table.append(list(range(start + j, end, tp)))
    return table


def model_parallel_is_initialized():
    return not (_TENSOR_MODEL_PARALLEL_GROUP is None or _PIPELINE_MODEL_PARALLEL_GROUP is None
                or _DATA_PARALLEL_GROUP is None)


def get_model_parallel_group():
    assert _MODEL_PARALLEL_GROUP is not None, "model parallel group is not initialized"
    return _MODEL_PARALLEL_GROUP


def get_tensor_model_parallel_group():
    assert _TENSOR_MODEL_PARALLEL_GROUP is not None, "tensor model parallel group is not initialized"
    return _TENSOR_MODEL_PARALLEL_GROUP


def get_pipeline_model_parallel_group():
    assert _PIPELINE_MODEL_PARALLEL_GROUP is not None, "pipeline model parallel group is not initialized"
    return _PIPELINE_MODEL_PARALLEL_GROUP


def get_data_parallel_group():
    assert _DATA_PARALLEL_GROUP is not None, "data parallel group is not initialized"
    return _DATA_PARALLEL_GROUP


def get_embedding_group():
    assert _EMBEDDING_GROUP is not None, "embedding group is not initialized"
    return _EMBEDDING_GROUP


def get_position_embedding_group():
    assert _POSITION_EMBEDDING_GROUP is not None, "position embedding group is not initialized"
    return _POSITION_EMBEDDING_GROUP


def is_rank_in_embedding_group(ignore_virtual=False):
    rank = dist.get_rank()
    if ignore_virtual:
        return rank in (_EMBEDDING_GLOBAL_RANKS or [])
    if rank in (_EMBEDDING_GLOBAL_RANKS or []):
        if rank == _EMBEDDING_GLOBAL_RANKS[0]:
            return is_pipeline_first_stage(ignore_virtual=False)
        if rank == _EMBEDDING_GLOBAL_RANKS[-1]:
            return is_pipeline_last_stage(ignore_virtual=False)
        return True
    return False


def set_tensor_model_parallel_world_size(world_size):
    global _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE
    _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = world_size


def set_pipeline_model_parallel_world_size(world_size):
    global _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = world_size


def get_tensor_model_parallel_world_size():
    if _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE is not None:
        return _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE
    return dist.get_world_size(group=get_tensor_model_parallel_group())


def get_pipeline_model_parallel_world_size():
    if _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE is not None:
        return _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    return dist.get_world_size(group=get_pipeline_model_parallel_group())


def set_tensor_model_parallel_rank(rank):
    global _MPU_TENSOR_MODEL_PARALLEL_RANK
    _MPU_TENSOR_MODEL_PARALLEL_RANK = rank


def set_pipeline_model_parallel_rank(rank):
    global _MPU_PIPELINE_MODEL_PARALLEL_RANK
    _MPU_PIPELINE_MODEL_PARALLEL_RANK = rank


def get_tensor_model_parallel_rank():
    if _MPU_TENSOR_MODEL_PARALLEL_RANK is not None:
        return _MPU_TENSOR_MODEL_PARALLEL_RANK
    return dist.get_rank(group=get_tensor_model_parallel_group())


def get_pipeline_model_parallel_rank():
    if _MPU_PIPELINE_MODEL_PARALLEL_RANK is not None:
        return _MPU_PIPELINE_MODEL_PARALLEL_RANK
    return dist.get_rank(group=get_pipeline_model_parallel_group())


def get_pipeline_model_parallel_split_rank():
    return _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def is_pipeline_first_stage(ignore_virtual=False):
    if not ignore_virtual and get_virtual_pipeline_model_parallel_world_size() is not None and \
            get_virtual_pipeline_model_parallel_rank() != 0:
        return False
    return get_pipeline_model_parallel_rank() == 0


def is_pipeline_last_stage(ignore_virtual=False):
    if not ignore_virtual:
        vws = get_virtual_pipeline_model_parallel_world_size()
        if vws is not None and get_virtual_pipeline_model_parallel_rank() != vws - 1:
            return False
    return get_pipeline_model_parallel_rank() == get_pipeline_model_parallel_world_size() - 1


def is_pipeline_stage_before_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    rank = get_pipeline_model_parallel_rank() if rank is None else rank
    return _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is None or rank < _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def is_pipeline_stage_after_split(rank=None):
    if get_pipeline_model_parallel_world_size() == 1:
        return True
    rank = get_pipeline_model_parallel_rank() if rank is None else rank
    return _PIPELINE_MODEL_PARALLEL_SPLIT_RANK is None or rank >= _PIPELINE_MODEL_PARALLEL_SPLIT_RANK


def get_virtual_pipeline_model_parallel_rank():
    return _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK


def set_virtual_pipeline_model_parallel_rank(rank):
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = rank


def get_virtual_pipeline_model_parallel_world_size():
    return _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE


def get_tensor_model_parallel_src_rank():
    """Global rank of the first rank in this rank's TP group."""
    return _TENSOR_GLOBAL_RANKS[0]


def get_data_parallel_src_rank():
    return _DATA_PARALLEL_GLOBAL_RANKS[0]


def get_pipeline_model_parallel_first_rank():
    return _PIPELINE_GLOBAL_RANKS[0]


def get_pipeline_model_parallel_last_rank():
    return _PIPELINE_GLOBAL_RANKS[get_pipeline_model_parallel_world_size() - 1]


def get_pipeline_model_parallel_next_rank():
    r = get_pipeline_model_parallel_rank()
    ws = get_pipeline_model_parallel_world_size()
    return _PIPELINE_GLOBAL_RANKS[(r + 1) % ws]


def get_pipeline_model_parallel_prev_rank():
    r = get_pipeline_model_parallel_rank()
    ws = get_pipeline_model_parallel_world_size()
    return _PIPELINE_GLOBAL_RANKS[(r - 1) % ws]


def get_context_parallel_group():
    """The CP group (None when cp = 1: the sequence is not sharded)."""
    assert _CONTEXT_PARALLEL_GROUP is not None, "context parallel group is not initialized"
    return None if _CONTEXT_PARALLEL_GROUP is _SINGLETON else _CONTEXT_PARALLEL_GROUP


def get_context_parallel_global_ranks():
    assert _CONTEXT_PARALLEL_GLOBAL_RANKS is not None, "context parallel group is not initialized"
    return list(_CONTEXT_PARALLEL_GLOBAL_RANKS)


def get_context_parallel_world_size():
    g = get_context_parallel_group()
    return 1 if g is None else dist.get_world_size(group=g)


def get_context_parallel_rank():
    g = get_context_parallel_group()
    return 0 if g is None else dist.get_rank(group=g)


def get_data_parallel_world_size():
    return dist.get_world_size(group=get_data_parallel_group())


def get_data_parallel_rank():
    return dist.get_rank(group=get_data_parallel_group())


def destroy_model_parallel():
    global _MODEL_PARALLEL_GROUP, _TENSOR_MODEL_PARALLEL_GROUP, _PIPELINE_MODEL_PARALLEL_GROUP
    global _DATA_PARALLEL_GROUP, _EMBEDDING_GROUP, _POSITION_EMBEDDING_GROUP
    global _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK, _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    global _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE, _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE
    global _MPU_TENSOR_MODEL_PARALLEL_RANK, _MPU_PIPELINE_MODEL_PARALLEL_RANK
    global _EMBEDDING_GLOBAL_RANKS, _PIPELINE_GLOBAL_RANKS, _DATA_PARALLEL_GLOBAL_RANKS, _TENSOR_GLOBAL_RANKS
    global _PIPELINE_MODEL_PARALLEL_SPLIT_RANK, _CONTEXT_PARALLEL_GROUP, _CONTEXT_PARALLEL_GLOBAL_RANKS
    _CONTEXT_PARALLEL_GROUP = _CONTEXT_PARALLEL_GLOBAL_RANKS = None
    _MODEL_PARALLEL_GROUP = _TENSOR_MODEL_PARALLEL_GROUP = _PIPELINE_MODEL_PARALLEL_GROUP = None
    _DATA_PARALLEL_GROUP = _EMBEDDING_GROUP = _POSITION_EMBEDDING_GROUP = None
    _VIRTUAL_PIPELINE_MODEL_PARALLEL_RANK = _VIRTUAL_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
    _MPU_TENSOR_MODEL_PARALLEL_WORLD_SIZE = _MPU_PIPELINE_MODEL_PARALLEL_WORLD_SIZE = None
    _MPU_TENSOR_MODEL_PARALLEL_RANK = _MPU_PIPELINE_MODEL_PARALLEL_RANK = None
    _EMBEDDING_GLOBAL_RANKS = _PIPELINE_GLOBAL_RANKS = _DATA_PARALLEL_GLOBAL_RANKS = None
    _TENSOR_GLOBAL_RANKS = None
    _PIPELINE_MODEL_PARALLEL_SPLIT_RANK = None
