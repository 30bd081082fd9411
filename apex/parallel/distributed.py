"""apex.parallel.DistributedDataParallel and Reducer over RCCL (R-15, R-16, R-17, NS-07).

Reference algorithm (apex/parallel/distributed.py:96-351):
  * params broadcast from rank 0 at construction (:160);
  * first iteration: record grad-ready order, cut buckets at ``message_size``
    elements per dtype, all-reduce everything at the end of backward and broadcast
    rank 0's bucket layout (:176-221);
  * steady state: a hook per param drops the grad into its bucket; a full bucket that
    is next in order is all-reduced on a side stream, out-of-order buckets are queued
    and drained in order (:279-315); the epilogue makes the compute stream wait and
    checks every bucket fired (:223-233).

MI355X-first redesign (same observable behaviour):
  * ZERO-COPY buckets: after the first iteration every grad is a VIEW into one
    persistent flat buffer per dtype laid out in grad-ready order, so a bucket is a
    contiguous slice (no flatten/unflatten copies, K-04 disappears) and the
    ``delay_allreduce`` path is ONE all-reduce per dtype;
  * averaging uses RCCL's native ncclAvg (``ReduceOp.AVG``) when the backend is
    RCCL ("nccl" on ROCm), so no separate divide kernel;
  * each full, in-order bucket is handed to a reduction stream (the reference's
    ``reduction_stream``) that first waits on the compute stream; the collective (plus the
    fp32 cast and copy-back under ``allreduce_always_fp32``) runs from there, so backward
    never blocks on communication; the end-of-backward callback waits on every bucket and
    joins the compute stream to the reduction streams (``_join_streams``);
  * ``num_allreduce_streams`` > 1 spreads buckets round-robin over several communicators,
    each with its own stream, so more than one RCCL collective is in flight over xGMI;
  * bucket size defaults to the reference's 1e7 elements but is tunable
    (``message_size`` / ``APEX_DDP_MESSAGE_SIZE``): on 8x MI355X each RCCL channel
    rides one of 7 xGMI links (~153 GB/s), so buckets of tens of MB keep all
    channels busy while still starting communication early in backward
    (``first_bucket_size`` makes the first bucket smaller to start even sooner).
"""
from __future__ import annotations

import contextlib
import os
import warnings
from collections import OrderedDict

import torch
import torch.distributed as dist
from torch.nn.modules import Module

from .. import _ext
from ..utils import prof

_ALIGN_SLOTS = os.environ.get("APEX_DDP_ALIGN", "1") != "0"  # 16-byte gradient slots (A/B knob)

# ----------------------------------------------------------------------------
# flat collective helpers (R-17)
# ----------------------------------------------------------------------------


def _is_rccl(group=None) -> bool:
    try:
        return dist.get_backend(group) == "nccl"
    except Exception:
        return False


def _dense_non_overlapping(t) -> bool:
    """True when t's elements exactly fill numel() slots in some dimension order (e.g. a
    channels_last conv weight), so a bucket slice can carry t's own strides."""
    expected = 1
    for stride, size in sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1):
        if stride != expected:
            return False
        expected *= size
    return True


def _flatten(tensors):
    return torch.cat([t.contiguous().view(-1) for t in tensors]) if len(tensors) > 1 else \
        tensors[0].contiguous().view(-1).clone()


def _unflatten_copy(flat, tensors):
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n


def _all_reduce_avg(flat, group=None, async_op=False, predivide=1.0):
    world = dist.get_world_size(group)
    if _is_rccl(group) and predivide == 1.0:
        return dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=group, async_op=async_op)
    if predivide != 1.0:
        flat.mul_(1.0 / predivide)
    w = dist.all_reduce(flat, group=group, async_op=async_op)
    post = predivide / world
    if async_op:
        return _PostScaleWork(w, flat, post)
    if post != 1.0:
        flat.mul_(post)
    return None


class _PostScaleWork:
    def __init__(self, work, flat, post):
        self.work, self.flat, self.post = work, flat, post

    def wait(self):
        self.work.wait()
        if self.post != 1.0:
            self.flat.mul_(self.post)


_MAIN_GRAD_GUARD = None


def _install_main_grad_guard():
    """A global optimizer step pre-hook (installed once, by the first fp32_main_grad DDP): an
    optimizer that reads ``p.grad`` (torch.optim, or any non-apex optimizer) stepping parameters
    whose gradients live in ``main_grad`` would silently never update them — raise instead. apex's
    fused optimizers read main_grad; under amp O2 the optimizer holds fp32 masters (no main_grad),
    whose grads amp fills from main_grad."""
    global _MAIN_GRAD_GUARD
    if _MAIN_GRAD_GUARD is not None:
        return

    def guard(opt, args, kwargs):
        from ..optimizers._base import FusedOptimizerBase

        if isinstance(opt, FusedOptimizerBase):
            return
        for g in opt.param_groups:
            for p in g["params"]:
                if p.grad is None and getattr(p, "main_grad", None) is not None:
                    raise RuntimeError(
                        "{} steps parameters whose gradients are in p.main_grad (apex DDP fp32_main_grad=True) "
                        "and reads p.grad, which DDP leaves None: use an apex.optimizers fused optimizer (they "
                        "read main_grad) or amp.initialize (O2 masters get their grads from main_grad), or "
                        "construct DDP with fp32_main_grad=False".format(type(opt).__name__))

    from torch.optim.optimizer import register_optimizer_step_pre_hook

    _MAIN_GRAD_GUARD = register_optimizer_step_pre_hook(guard)


def _group_root(group):
    """Global rank of a group's rank 0 (collective src/dst arguments are global ranks)."""
    return dist.get_global_rank(group, 0) if group is not None else 0


def apply_flat_dist_call(bucket, call, extra_args=None, group=None):
    """Flatten a same-dtype bucket, run ``call`` on it, average after all_reduce,
    and copy the result back (reference semantics, apex/parallel/distributed.py:11-23).
    For broadcast, ``extra_args[0]`` is the source as a rank WITHIN ``group``."""
    coalesced = _flatten(bucket)
    if call is dist.all_reduce:
        _all_reduce_avg(coalesced, group)
    elif call is dist.broadcast and group is not None:
        src = dist.get_global_rank(group, extra_args[0] if extra_args else 0)
        dist.broadcast(coalesced, src, group=group)
    elif extra_args is not None:
        call(coalesced, *extra_args, group=group) if group is not None else call(coalesced, *extra_args)
    else:
        call(coalesced)
    _unflatten_copy(coalesced, bucket)


def flat_dist_call(tensors, call, extra_args=None, group=None):
    """Group ``tensors`` by dtype/device and apply ``call`` once per group (C1/C2/C4/C7)."""
    buckets = OrderedDict()
    for t in tensors:
        buckets.setdefault((t.dtype, t.device), []).append(t)
    for bucket in buckets.values():
        apply_flat_dist_call(bucket, call, extra_args, group)


def extract_tensors(maybe_tensor, tensor_list):
    if torch.is_tensor(maybe_tensor):
        tensor_list.append(maybe_tensor)
    else:
        try:
            for item in maybe_tensor:
                extract_tensors(item, tensor_list)
        except TypeError:
            return


class Reducer:
    """Manual all-reduce helper (R-16, apex/parallel/distributed.py:52-93).

    ``Reducer(module)`` broadcasts the module's params from rank 0; ``reduce()``
    averages all present grads across ranks (one collective per dtype). Passing a
    list of grads instead reduces exactly those tensors.
    """

    def __init__(self, module_or_grads_list, process_group=None):
        self.group = process_group
        if isinstance(module_or_grads_list, Module):
            self.module = module_or_grads_list
            flat_dist_call([p.data for p in self.module.parameters()], dist.broadcast, (0,), self.group)
        else:
            self.module = None
            self.grads = []
            extract_tensors(module_or_grads_list, self.grads)

    def reduce(self):
        if self.module:
            grads = [p.grad.data for p in self.module.parameters() if p.grad is not None]
        else:
            grads = self.grads
        if grads:
            flat_dist_call(grads, dist.all_reduce, group=self.group)


# ----------------------------------------------------------------------------
# DistributedDataParallel
# ----------------------------------------------------------------------------
class _Bucket:
    __slots__ = ("dtype", "flat", "start", "numel", "params", "ready", "work", "tmp", "lane", "ev_ready",
                 "ev_done")

    def __init__(self, dtype, flat, start, numel, params):
        self.dtype, self.flat, self.start, self.numel, self.params = dtype, flat, start, numel, params
        self.ready = 0
        self.work = None
        self.tmp = None       # fp32 staging copy (allreduce_always_fp32)
        self.lane = 0         # which communicator / reduction stream carried it
        self.ev_ready = None  # comm_timing events (reduction stream): bucket handed to comm ...
        self.ev_done = None   # ... and reduced (after the collective's wait)

    @property
    def buf(self):
        return self.flat[self.start:self.start + self.numel]


_TARGETS_GIVEN = set()  # ids of params whose bucket slot was handed out in the current backward


def grad_target(p):
    """Where a fused backward may write ``p``'s gradient directly: a FRESH view of p's slot in
    its apex DDP gradient bucket, when p has no gradient yet in this backward (the fused
    optimizers' ``zero_grad`` releases the views instead of zero-filling the buckets). The
    producer writes the whole gradient there and returns the view; autograd then adopts it as
    ``p.grad`` without a copy (a fresh, unshared view is what lets AccumulateGrad steal it) and
    the bucket needs no accumulate kernel. ``None``: allocate as usual (no DDP, not contiguous,
    or a gradient is already accumulating, e.g. inside ``no_sync()`` micro-batches)."""
    slot = getattr(p, "_apex_grad_slot", None)
    if slot is None or p.grad is not None or id(p) in _TARGETS_GIVEN:
        # (a second producer of the same parameter in one backward — tied weights — must not
        # write the slot too: autograd sums both results before p.grad is set)
        return None
    _TARGETS_GIVEN.add(id(p))
    flat, off, n = slot
    return flat.narrow(0, off, n).view(p.shape)


def _lane_groups(process_group, k, backend):
    """k communicators ("lanes") over the ranks of ``process_group``.

    ``dist.new_group`` is collective over the DEFAULT group: every process must call it for every
    group, with the same rank lists in the same order, or group names / store keys collide (a hang,
    or communicators wired across the wrong ranks). With a subgroup (e.g. the data-parallel group
    under TP/PP) each rank knows only its own group, so the rank lists of all groups are first
    exchanged over the default group (every rank constructs its DDP at the same point, as with any
    collective setup) and every rank then creates the k lanes of EVERY group, in sorted order,
    keeping its own.
    """
    world = dist.get_world_size()
    if process_group is None:
        return [dist.new_group(ranks=list(range(world)), backend=backend) for _ in range(k)]
    mine = tuple(dist.get_process_group_ranks(process_group))
    allg = [None] * world
    dist.all_gather_object(allg, mine)
    groups = sorted(set(tuple(g) for g in allg))
    covered = sorted(r for g in groups for r in g)
    if covered != list(range(world)):
        raise ValueError("num_allreduce_streams > 1 with a process_group needs disjoint groups covering "
                         "every rank; pass allreduce_communicators instead")
    lanes = None
    for g in groups:
        made = [dist.new_group(ranks=list(g), backend=backend) for _ in range(k)]
        if g == mine:
            lanes = made
    return lanes


class DistributedDataParallel(Module):
    """Bucketed, backward-overlapped data parallelism over RCCL.

    Args mirror the reference (apex/parallel/distributed.py:96-124) plus later apex options:

    * ``message_size``: elements per bucket (default 1e7; env ``APEX_DDP_MESSAGE_SIZE``).
    * ``first_bucket_size``: smaller first bucket so communication starts sooner.
    * ``delay_allreduce``: one all-reduce per dtype at the end of backward.
    * ``allreduce_trigger_params``: params whose gradients, once all have arrived, trigger the
      all-reduce of every bucket (manual control of when communication starts).
    * ``allreduce_always_fp32``: reduce a bucket through an fp32 copy (cast, collective and
      copy-back all on the reduction stream, so backward is never blocked).
    * ``num_allreduce_streams`` / ``allreduce_communicators``: buckets round-robin over k
      communicators, each with its own reduction stream, so several RCCL collectives are in
      flight at once (each communicator drives its own channels over the xGMI links).
      ``allreduce_communicators`` passes the process groups explicitly.
    * ``gradient_average`` / ``gradient_predivide_factor``: average = divide by predivide before
      the sum and by world/predivide after it (RCCL's native ncclAvg when predivide == 1).
      ``gradient_average_split_factor`` is the deprecated name of the predivide factor.
    * ``retain_allreduce_buffers``: the reduced buckets are always kept — every grad is a view of
      a persistent flat buffer per dtype (``allreduce_buffers``), so the flag needs no copy.
    * ``prof``: emit a roctx range per bucket collective.
    * ``comm_timing``: record HIP events per bucket and per backward so ``comm_stats()`` reports
      bucket sizes, ready->reduced latency and the communication time the compute stream waited
      for at the end of backward (exposed comm).
    * ``fp32_main_grad``: every parameter's gradient accumulates in an fp32 ``p.main_grad`` (views
      of fp32 bucket buffers laid out in reverse registration order at construction) instead of
      ``p.grad`` — Megatron's main_grad, for gradient accumulation over micro-batches of a 16-bit
      model without bf16 rounding at every add (the reference's fp32 master-grad semantics,
      ``/root/reference/apex/fp16_utils/fp16util.py:93-112``). The fused weight-gradient GEMMs
      accumulate straight into main_grad (fp32 output, beta = 1; ``apex.ops.fused._wgrad``) and
      hand autograd a placeholder; any other gradient is added into main_grad by the hook and
      ``p.grad`` released. The buckets are reduced in fp32; the fused optimizers and amp read
      ``main_grad``; ``zero_grad`` zero-fills the buffers.
    """

    def __init__(self, module, message_size=10000000, delay_allreduce=False, shared_param=None,
                 allreduce_trigger_params=None, retain_allreduce_buffers=False,
                 allreduce_always_fp32=False, num_allreduce_streams=1,
                 allreduce_communicators=None, gradient_average=True,
                 gradient_predivide_factor=1.0, gradient_average_split_factor=None, prof=False,
                 first_bucket_size=None, process_group=None, broadcast_buffers=True,
                 comm_timing=False, fp32_main_grad=False):
        super().__init__()
        if shared_param is not None:
            raise ValueError("shared_param is no longer supported as an option. It was misleadingly "
                             "named from the start. It turns out overlapping communication with "
                             "computation should work fine with shared parameters. If you still "
                             "wish to delay communication to the end of the backward pass, use "
                             "delay_allreduce=True|False instead.")
        if gradient_average_split_factor is not None:
            warnings.warn("gradient_average_split_factor is deprecated; use gradient_predivide_factor",
                          DeprecationWarning)
            gradient_predivide_factor = gradient_average_split_factor
        self.module = module
        self.group = process_group
        self.world_size = dist.get_world_size(process_group)
        self.message_size = int(os.environ.get("APEX_DDP_MESSAGE_SIZE", message_size))
        self.first_bucket_size = first_bucket_size
        self.delay_allreduce = delay_allreduce or bool(int(os.environ.get("APEX_DDP_DELAY", "0")))
        self.allreduce_always_fp32 = allreduce_always_fp32
        self.retain_allreduce_buffers = True  # always: grads are views of the persistent buckets
        self.gradient_average = gradient_average
        self.gradient_predivide_factor = float(gradient_predivide_factor)
        self.broadcast_buffers = broadcast_buffers
        self.prof = prof
        self.comm_timing = comm_timing
        self.single_rank_collectives = False
        backend = dist.get_backend(process_group)
        self._rccl = backend == "nccl"
        if self._rccl:
            for p in module.parameters():
                if not p.is_cuda:
                    raise ValueError("RCCL backend requires every parameter on the GPU")
        # communicators (lanes): bucket i rides lane i % k
        if allreduce_communicators is not None:
            self._groups = list(allreduce_communicators)
        elif num_allreduce_streams > 1:
            self._groups = _lane_groups(process_group, num_allreduce_streams, backend)
        else:
            self._groups = [process_group]
        self.num_allreduce_streams = len(self._groups)
        self._cuda = self._rccl and torch.cuda.is_available()
        self._make_streams()
        self._params = [p for p in module.parameters() if p.requires_grad]
        self._param_index = {id(p): i for i, p in enumerate(self._params)}
        self._trigger = None
        if allreduce_trigger_params is not None:
            self._trigger = {self._param_index[id(p)] for p in allreduce_trigger_params}
        self._trigger_seen = 0
        self._layout_ready = False
        self._buckets = []
        self._flat = {}            # dtype -> flat buffer
        self._param_bucket = {}    # param idx -> bucket idx
        self._ready_order = []
        self._callback_queued = False
        # fp32_main_grad: 16-bit gradients of unfused producers (biases, norms, embeddings) awaiting
        # ONE multi-tensor add into main_grad (torch's mixed-dtype add is a ~50 us launch per
        # tensor: 2080 launches, 105 ms of a Megatron GPT step)
        self._pending_mg = []
        self._mg_flush_queued = False
        self._next_bucket = 0
        self._allreduce_enabled = True
        self._hooks = []
        self._iter_events = []     # (end-of-backward, comm-done) event pairs, comm_timing only
        self.fp32_main_grad = fp32_main_grad
        self._sync_params()
        if fp32_main_grad:
            # main_grad must exist before the first backward so the producers can accumulate into
            # it: a provisional layout in reverse registration order. The first backward records the
            # order the gradients actually become ready in (as the 16-bit path does) and
            # _end_of_backward re-lays the buffers out in that order (rank 0's order wins), so that
            # in steady state a bucket never waits on a parameter that arrives late
            self._layout_from_order(list(reversed(range(len(self._params)))), dtype=torch.float32)
            _install_main_grad_guard()
        self._create_hooks()

    # ------------------------------------------------------------ setup
    def _make_streams(self):
        # the reference's reduction_stream (distributed.py:144): one per communicator lane
        self._streams = [torch.cuda.Stream() for _ in self._groups] if self._cuda else [None] * len(self._groups)
        self.reduction_stream = self._streams[0]

    def _sync_params(self):
        if self.world_size == 1:
            return
        tensors = [p.data for p in self.module.parameters()]
        if self.broadcast_buffers:
            tensors += [b.data for b in self.module.buffers()]
        if tensors:
            flat_dist_call(tensors, dist.broadcast, (0,), self.group)

    def _create_hooks(self):
        for p in self._params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._grad_hook))

    def __getstate__(self):
        attrs = dict(self.__dict__)
        for k in ("reduction_stream", "_streams", "_hooks", "_iter_events"):
            attrs.pop(k, None)  # reference bug fix (distributed.py:168-172)
        return attrs

    def __setstate__(self, state):
        super().__setstate__(state)
        self._make_streams()
        self._iter_events = []
        self._hooks = []
        self._create_hooks()

    # ------------------------------------------------------------ control
    def enable_allreduce(self):
        self._allreduce_enabled = True

    def disable_allreduce(self):
        self._allreduce_enabled = False

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate grads locally (no communication) inside this context."""
        old = self._allreduce_enabled
        self._allreduce_enabled = False
        try:
            yield
        finally:
            self._allreduce_enabled = old

    def zero_grad_buffer(self):
        """Zero-fill the fp32 main_grad buffers (fp32_main_grad mode; one fill per buffer)."""
        if self.fp32_main_grad:
            for flat in self._flat.values():
                flat.zero_()

    def zero_grad(self, set_to_none: bool = True):
        """Module.zero_grad, plus the fp32 main_grad buffers in fp32_main_grad mode (where p.grad is
        never used: without this, Module.zero_grad / torch.optim's zero_grad would leave main_grad
        accumulating across steps)."""
        super().zero_grad(set_to_none)
        self.zero_grad_buffer()

    @property
    def allreduce_buffers(self):
        """The persistent flat gradient buffers (one per dtype), reduced in place."""
        return list(self._flat.values())

    def reduce_gradients(self):
        """All-reduce every gradient now (one collective per dtype), outside any backward pass:
        for callers that ran all their backward passes under ``no_sync()`` (e.g. a pipeline
        schedule). Builds the bucket layout on first use."""
        if not self._layout_ready:
            self._build_layout()
            self._layout_ready = True
        self._flush_main_grad()
        for i, p in enumerate(self._params):
            if self.fp32_main_grad:
                if p.grad is not None:  # a gradient produced outside the hooks
                    if not p.grad._is_zerotensor():
                        p.main_grad.add_(p.grad)
                    p.grad = None
            else:
                self._ensure_view(i, p)
        for flat in self._flat.values():
            self._reduce_now(flat)

    def forward(self, *inputs, **kwargs):
        _TARGETS_GIVEN.clear()
        self._callback_queued = False
        self._next_bucket = 0
        self._trigger_seen = 0
        self._ready_order = []
        for b in self._buckets:
            b.ready = 0
            b.work = None
            b.tmp = None
        return self.module(*inputs, **kwargs)

    # ------------------------------------------------------------ hooks
    def _grad_hook(self, p):
        if self.fp32_main_grad:
            # a bare ZeroTensor placeholder: a fused producer accumulated into main_grad already;
            # anything else (an unfused producer, or a tied weight's other uses summed with the
            # placeholder by autograd) is added here
            g = p.grad
            if g is not None and not g._is_zerotensor():
                if g.is_cuda and g.dtype != p.main_grad.dtype and g.is_contiguous() and _ext.use_native(g):
                    self._pending_mg.append((p.main_grad, g))
                    if not self._mg_flush_queued:
                        torch.autograd.Variable._execution_engine.queue_callback(self._flush_main_grad)
                        self._mg_flush_queued = True
                else:
                    p.main_grad.add_(g)
            p.grad_added_to_main_grad = False
            p.grad = None
        if not self._allreduce_enabled:
            return
        if not self._callback_queued:
            torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
            self._callback_queued = True
        idx = self._param_index[id(p)]
        if not self._layout_ready or self.delay_allreduce:
            if not self._layout_ready:
                self._ready_order.append(idx)
            else:
                self._ensure_view(idx, p)
            return
        if self._trigger is not None and self._trigger_seen == len(self._trigger):
            # every bucket is already on the wire: writing this gradient into its slot would race
            # with the collective and the value would never be reduced (replicas diverge)
            raise RuntimeError("allreduce_trigger_params: a gradient arrived after the trigger params fired "
                               "the all-reduce; the trigger params must be the LAST to receive gradients in "
                               "backward (e.g. the first layer's weight)")
        if not self.fp32_main_grad:
            self._ensure_view(idx, p)
        if self._trigger is not None:
            if idx in self._trigger:
                self._trigger_seen += 1
                if self._trigger_seen == len(self._trigger):
                    for b in self._buckets:
                        b.ready = len(b.params)
                    self._launch_ready_in_order()
            return
        bi = self._param_bucket[idx]
        b = self._buckets[bi]
        b.ready += 1
        if b.ready > len(b.params):
            raise RuntimeError("The same param received more than one gradient in one backward "
                               "pass; shared params must be registered once.")
        if b.ready == len(b.params) and bi == self._next_bucket:
            self._launch_ready_in_order()

    def _flush_main_grad(self):
        """main_grad += g for every deferred 16-bit gradient: one fused multi-tensor axpby launch
        (csrc/multi_tensor.hip, fp32 x + bf16/fp16 y -> fp32). Runs before any bucket holding one
        of them is reduced and at the end of every backward pass."""
        self._mg_flush_queued = False
        if not self._pending_mg:
            return
        pend, self._pending_mg = self._pending_mg, []
        from ..multi_tensor_apply import get_plan

        by_dtype = {}
        for mg, g in pend:
            by_dtype.setdefault(g.dtype, []).append((mg, g))
        for items in by_dtype.values():
            mgs = [mg for mg, _ in items]
            gs = [g for _, g in items]
            get_plan([mgs, gs, mgs]).axpby(1.0, 1.0, -1, None)

    def _ensure_view(self, idx, p):
        if self.fp32_main_grad:
            return  # main_grad is the bucket view; p.grad is never used
        v = self._views[idx]
        g = p.grad
        if g is None or g.data_ptr() != v.data_ptr():
            if g is not None:
                v.copy_(g)
            else:
                v.zero_()
            p.grad = v

    def _launch_ready_in_order(self):
        while self._next_bucket < len(self._buckets):
            b = self._buckets[self._next_bucket]
            if b.ready != len(b.params):
                break
            self._start_bucket(b, self._next_bucket % len(self._groups))
            self._next_bucket += 1

    # ------------------------------------------------------------ collectives
    def _start_bucket(self, b, lane):
        """Hand bucket b to communicator `lane`. On the GPU its reduction stream waits for the
        compute stream (grads written), issues the collective (after an fp32 cast under
        allreduce_always_fp32), waits for it — a stream-side wait: the host returns at once —
        and copies an fp32 staging buffer back, so every step of the bucket is ordered on the
        reduction stream and the compute stream only joins it at the end of backward. On the
        CPU (gloo) the wait is a host wait, so it is deferred to the end of backward."""
        self._flush_main_grad()
        b.lane = lane
        stream = self._streams[lane]
        if stream is None:
            b.work, b.tmp = self._issue(b.buf, self._groups[lane], async_op=True)
            return
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            if self.comm_timing:
                b.ev_ready = torch.cuda.Event(enable_timing=True)
                b.ev_ready.record()
            b.work, b.tmp = self._issue(b.buf, self._groups[lane], async_op=True)
            self._complete(b)
            if self.comm_timing:
                b.ev_done = torch.cuda.Event(enable_timing=True)
                b.ev_done.record()

    def _complete(self, b):
        if b.work is not None:
            b.work.wait()
        if b.tmp is not None:
            b.buf.copy_(b.tmp)
        b.work = None
        b.tmp = None

    def _finish_bucket(self, b):
        """CPU path: wait for bucket b's collective (the GPU path completed it on its stream)."""
        if self._streams[b.lane] is None:
            self._complete(b)

    def _issue(self, buf, group, async_op):
        """Returns (work, fp32 staging buffer or None). A one-rank group's average is the identity,
        so nothing is launched (RCCL would still run a full copy kernel over the bucket,
        ~0.66 ms per 50 MB bucket on MI355X) unless ``single_rank_collectives`` is set (tests)."""
        if self.world_size == 1 and not self.single_rank_collectives:
            return None, None
        tmp = None
        target = buf
        if self.allreduce_always_fp32 and buf.dtype != torch.float32:
            tmp = target = buf.float()
        rng = prof.range("apex.ddp.allreduce[{}]".format(buf.numel())) if self.prof else contextlib.nullcontext()
        with rng:
            if not self.gradient_average:
                w = dist.all_reduce(target, group=group, async_op=async_op)
            else:
                w = _all_reduce_avg(target, group, async_op=async_op,
                                    predivide=self.gradient_predivide_factor)
        return w, tmp

    def _reduce_now(self, buf):
        """Synchronous (w.r.t. the compute stream) all-reduce of a whole flat buffer."""
        b = _Bucket(buf.dtype, buf, 0, buf.numel(), [])
        self._start_bucket(b, 0)
        self._finish_bucket(b)
        self._join_streams()

    def _join_streams(self):
        if self._cuda:
            cur = torch.cuda.current_stream()
            for s in self._streams:
                cur.wait_stream(s)

    def _end_of_backward(self):
        _TARGETS_GIVEN.clear()
        self._flush_main_grad()
        ev0 = None
        if self.comm_timing and self._cuda:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        if not self._layout_ready:
            self._build_layout()
            for flat in self._flat.values():
                self._reduce_now(flat)
            self._layout_ready = True
            return
        if self.delay_allreduce:
            for idx, p in enumerate(self._params):
                if p.grad is None and not self.fp32_main_grad:  # no grad this step (view released)
                    self._views[idx].zero_()
                    p.grad = self._views[idx]
            for flat in self._flat.values():
                self._reduce_now(flat)
        else:
            # params that did not receive a grad this iteration: treat as ready (zero grads; in
            # main_grad mode the buffer already holds what was accumulated, zeros if nothing)
            for b in self._buckets:
                if b.ready != len(b.params):
                    if not self.fp32_main_grad:
                        for idx in b.params:
                            p = self._params[idx]
                            if p.grad is None:
                                self._views[idx].zero_()
                                p.grad = self._views[idx]
                    b.ready = len(b.params)
            self._launch_ready_in_order()
            for b in self._buckets:
                self._finish_bucket(b)
            self._join_streams()
            if self._next_bucket != len(self._buckets):
                raise RuntimeError("In epilogue, next_bucket ({}) != num_buckets ({}). This probably "
                                   "indicates some buckets were not allreduced."
                                   .format(self._next_bucket, len(self._buckets)))
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._iter_events.append((ev0, ev1))
            del self._iter_events[:-64]

    def comm_stats(self):
        """Bucket layout and (with comm_timing) timings of the most recent backward passes.
        Synchronises the device: call it outside timed regions."""
        out = {"world_size": self.world_size,
               "backend": dist.get_backend(self.group),
               "num_buckets": len(self._buckets),
               "num_communicators": len(self._groups),
               "message_size": self.message_size,
               "bucket_bytes": [b.numel * b.flat.element_size() for b in self._buckets],
               "allreduce_always_fp32": self.allreduce_always_fp32,
               "fp32_main_grad": self.fp32_main_grad,
               "delay_allreduce": self.delay_allreduce}
        if self.comm_timing and self._cuda:
            torch.cuda.synchronize()
            lat = [b.ev_ready.elapsed_time(b.ev_done) for b in self._buckets
                   if b.ev_ready is not None and b.ev_done is not None]
            exposed = [max(0.0, a.elapsed_time(c)) for a, c in self._iter_events]
            out["bucket_ready_to_reduced_ms"] = [round(x, 3) for x in lat]
            if exposed:
                out["exposed_comm_ms_mean"] = round(sum(exposed) / len(exposed), 3)
                out["exposed_comm_ms_max"] = round(max(exposed), 3)
                out["exposed_comm_samples"] = len(exposed)
        return out

    def reset_comm_stats(self):
        self._iter_events = []

    # ------------------------------------------------------------ layout
    def _build_layout(self):
        """Bucket layout in the recorded grad-ready order (the reference's first-iteration
        recording, /root/reference/apex/parallel/distributed.py:176-203), rank 0's order broadcast
        to every rank. In fp32_main_grad mode it replaces the provisional reverse-registration
        layout, carrying the accumulated main_grad values over."""
        order = list(self._ready_order)
        seen = set(order)
        order += [i for i in range(len(self._params)) if i not in seen]  # never-ready params last
        if self.world_size > 1:
            dev = self._params[0].device
            t = torch.tensor(order, dtype=torch.int64, device=dev if self._rccl else "cpu")
            dist.broadcast(t, _group_root(self.group), group=self.group)  # C3: rank 0's layout wins
            order = [int(x) for x in t.tolist()]
        self._layout_from_order(order, dtype=torch.float32 if self.fp32_main_grad else None)

    def _layout_from_order(self, order, dtype=None):
        by_dtype = OrderedDict()
        for idx in order:
            p = self._params[idx]
            by_dtype.setdefault(dtype or p.dtype, []).append(idx)
        self._views = [None] * len(self._params)
        self._buckets = []
        self._param_bucket = {}
        for dt, idxs in by_dtype.items():
            # every slot starts on a 16-byte boundary: one odd-sized parameter (BERT's 30522-entry
            # MLM bias) otherwise shifts every later gradient view off alignment, and the fused
            # multi-tensor kernels (grad norm, LAMB / Adam) drop to their scalar path for the
            # whole parameter list (the plan's `aligned` flag is all-or-nothing)
            al = max(1, 16 // torch.empty((), dtype=dt).element_size()) if _ALIGN_SLOTS else 1
            total = 0
            for i in idxs:
                total = -(-total // al) * al + self._params[i].numel()
            dev = self._params[idxs[0]].device
            flat = torch.zeros(total, dtype=dt, device=dev)
            flat._apex_nparams = len(idxs)  # lets fused optimizers zero the grads with one fill
            self._flat[dt] = flat
            off, start, cur = 0, 0, []
            limit = self.first_bucket_size or self.message_size
            for i in idxs:
                p = self._params[i]
                n = p.numel()
                off = -(-off // al) * al
                if p.is_contiguous() or not _dense_non_overlapping(p):
                    v = flat[off:off + n].view(p.shape)
                else:  # e.g. channels_last conv weight: the grad view keeps the param's strides
                    v = flat[off:off + n].as_strided(p.shape, p.stride())
                if dtype is not None:  # fp32 main_grad mode
                    old_mg = getattr(p, "main_grad", None)
                    if old_mg is not None:  # re-layout after the first backward: keep what accumulated
                        v.copy_(old_mg)
                    if p.grad is not None:
                        if not p.grad._is_zerotensor():
                            v.add_(p.grad)
                        p.grad = None
                    p.main_grad = v
                    p._apex_main_flat = flat
                    self._views[i] = v
                    cur.append(i)
                    off += n
                    if off - start >= limit:
                        self._buckets.append(_Bucket(dt, flat, start, off - start, cur))
                        start, cur, limit = off, [], self.message_size
                    continue
                if p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v
                p._apex_grad_is_bucket_view = True
                if p.is_contiguous():
                    # lets a fused producer write this param's gradient straight into the bucket
                    # (apex.parallel.grad_target)
                    p._apex_grad_slot = (flat, off, n)
                p._apex_bucket_flat = flat
                self._views[i] = v
                cur.append(i)
                off += n
                if off - start >= limit:
                    self._buckets.append(_Bucket(dt, flat, start, off - start, cur))
                    start, cur, limit = off, [], self.message_size
            if cur:
                self._buckets.append(_Bucket(dt, flat, start, off - start, cur))
        for bi, b in enumerate(self._buckets):
            for i in b.params:
                self._param_bucket[i] = bi
