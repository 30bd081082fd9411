"""apex.ops.blocks._GammaZeroCheck: the host-side "does an LN gamma hold an exact 0" decision of the
memory-efficient post-LN mode costs one device -> host read per OPTIMIZER STEP, not one per
micro-batch forward after a backward (gradient accumulation, 1F1B schedules). CPU-only: the check
is plain torch."""
import torch

from apex.ops.blocks import _GammaZeroCheck, _gz_after_step


def _fresh():
    gz = _GammaZeroCheck()
    return gz


def test_one_host_read_per_optimizer_step_with_accumulation():
    import apex.ops.blocks as B

    gz = _fresh()
    old = B._GZ
    B._GZ = gz  # the global step hook marks the module's instance
    try:
        gammas = [torch.nn.Parameter(torch.ones(16)) for _ in range(4)]
        opt = torch.optim.SGD(gammas, lr=0.1)
        for step in range(3):
            for micro in range(4):  # 4 accumulated micro-batches: forward (checks) + backward
                for g in gammas:
                    assert gz.has_zero(g) is False
                gz.after_backward()
            for g in gammas:
                g.grad = torch.zeros(16)
            opt.step()  # the global post-hook marks the check dirty
            # step 0: the first read (initially dirty) plus the backward-driven re-checks until the
            # first optimizer step was seen; from then on exactly one read per step
        assert gz._steps_seen
        reads_before = gz.host_reads
        for micro in range(4):
            for g in gammas:
                gz.has_zero(g)
            gz.after_backward()
        assert gz.host_reads == reads_before + 1  # one read for the whole accumulation window
    finally:
        B._GZ = old


def test_reads_count_exactly_once_per_step_after_first():
    gz = _fresh()
    gz.after_optimizer_step()  # optimizers in use
    g = torch.nn.Parameter(torch.ones(8))
    counts = []
    for step in range(5):
        for micro in range(4):
            gz.has_zero(g)
            gz.after_backward()
        counts.append(gz.host_reads)
        gz.after_optimizer_step()
    assert counts == [1, 2, 3, 4, 5]


def test_zero_written_by_optimizer_step_is_seen():
    """A fused optimizer writes through raw pointers (no version bump): the step hook is what makes
    the next forward see a new exact zero."""
    gz = _fresh()
    g = torch.nn.Parameter(torch.ones(8))
    assert gz.has_zero(g) is False
    gz.after_optimizer_step()
    assert gz.has_zero(g) is False
    g.data[3] = 0.0  # what a raw-pointer kernel write looks like to autograd: no version change
    assert gz.has_zero(g) is False  # not seen until the next step (documented)
    gz.after_optimizer_step()
    assert gz.has_zero(g) is True


def test_version_counter_write_is_seen_without_step():
    gz = _fresh()
    gz.after_optimizer_step()
    g = torch.nn.Parameter(torch.ones(8))
    assert gz.has_zero(g) is False
    with torch.no_grad():
        g[5] = 0.0  # autograd-visible in-place write bumps _version
    assert gz.has_zero(g) is True


def test_backward_marks_dirty_until_first_step():
    """A hand-written `.data` update loop (no optimizer): every backward re-checks, as before."""
    gz = _fresh()
    g = torch.nn.Parameter(torch.ones(8))
    assert gz.has_zero(g) is False
    g.data[0] = 0.0
    gz.after_backward()
    assert gz.has_zero(g) is True


def test_global_hook_is_registered():
    import apex.ops.blocks as B

    gz = _fresh()
    old = B._GZ
    B._GZ = gz
    try:
        p = torch.nn.Parameter(torch.ones(2))
        p.grad = torch.ones(2)
        gz._dirty = False
        torch.optim.SGD([p], lr=1.0).step()
        assert gz._dirty and gz._steps_seen
        _gz_after_step(None, (), {})
    finally:
        B._GZ = old
