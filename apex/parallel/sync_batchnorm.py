"""SyncBatchNorm (NS-04): BatchNorm whose batch statistics span a process group.

Forward: per-channel local Welford statistics (one HIP reduction, csrc/norm_misc.hip) ->
ONE all_gather of the [C, 3] (mean, M2, count) triples over RCCL -> parallel-Welford
combine on device -> fused normalise (+ optional ReLU). Backward: local (sum dy,
sum dy*(x-mean)) in one HIP reduction -> ONE all_reduce of the [2, C] buffer -> fused
elementwise dx. Exact for uneven per-rank batch sizes (counts travel with the stats).
NCHW by default; ``channel_last=True`` for NHWC tensors.
API follows apex.parallel.SyncBatchNorm / convert_syncbn_model /
create_syncbn_process_group.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch.nn.modules.batchnorm import _BatchNorm

from .. import _ext


def _world(group):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _local_stats_ref(x, channel_last):
    C = x.shape[-1] if channel_last else x.shape[1]
    xf = x.float()
    xf = xf.reshape(-1, C) if channel_last else xf.transpose(0, 1).reshape(C, -1).t()
    n = torch.full((C,), float(xf.shape[0]), dtype=torch.float32, device=x.device)
    mean = xf.mean(0)
    m2 = ((xf - mean) ** 2).sum(0)
    return torch.stack([mean, m2, n], 1)


def _combine_ref(g):  # g [G, C, 3]
    mean, m2, n = g[0, :, 0], g[0, :, 1], g[0, :, 2]
    for k in range(1, g.shape[0]):
        mb, m2b, nb = g[k, :, 0], g[k, :, 1], g[k, :, 2]
        tot = n + nb
        d = mb - mean
        wb = torch.where(tot > 0, nb / tot.clamp(min=1), torch.zeros_like(tot))
        mean = mean + d * wb
        m2 = m2 + m2b + d * d * n * wb
        n = tot
    var = torch.where(n > 0, m2 / n.clamp(min=1), torch.zeros_like(n))
    return mean, var, n


def _bshape(x, channel_last):
    return (1,) * (x.dim() - 1) + (-1,) if channel_last else (1, -1) + (1,) * (x.dim() - 2)


class SyncBatchnormFunction(torch.autograd.Function):
    """y = BN(input) (+ z) (+ ReLU). The residual ``z`` and the ReLU are fused into the HIP
    elementwise kernel; backward masks the gradient with the saved output inside the reduce /
    elementwise kernels (no separate mask pass) and returns the residual's gradient from the same
    pass (the ResNet bottleneck tail relu(bn3(conv3) + identity) as one kernel each way)."""

    @staticmethod
    def forward(ctx, input, weight, bias, running_mean, running_var, eps, momentum, group, channel_last,
                fuse_relu, z=None, num_batches_tracked=None):
        native = _ext.use_native(input)
        x = input.contiguous()  # channel_last: logical [N, ..., C] layout (apex convention)
        C = _ext.require() if native else None
        world = _world(group)
        # the combine kernel also writes invstd and updates fp32 running statistics in place (and,
        # single-process, bumps num_batches_tracked): one launch instead of ~10 small torch ops
        fused_running = native and (running_mean is None or (
            running_mean.dtype == torch.float32 and running_var.dtype == torch.float32
            and running_mean.is_contiguous() and running_var.is_contiguous()))
        rm, rv = (running_mean, running_var) if fused_running else (None, None)
        if fused_running and world == 1:
            mean, var, count, invstd = C.bn_stats(x, channel_last, eps, rm, rv, momentum, num_batches_tracked)
            num_batches_tracked = None
        else:
            local = C.bn_local_stats(x, channel_last) if native else _local_stats_ref(x, channel_last)
            if world > 1:
                gathered = torch.empty((world * local.shape[0], 3), dtype=local.dtype, device=local.device)
                dist.all_gather_into_tensor(gathered, local, group=group)
                gathered = gathered.view(world, -1, 3)
            else:
                gathered = local.unsqueeze(0)
            if native:
                mean, var, count, invstd = C.bn_combine(gathered, eps, rm, rv, momentum)
            else:
                mean, var, count = _combine_ref(gathered)
                invstd = torch.rsqrt(var + eps)
            if running_mean is not None and not fused_running:
                with torch.no_grad():
                    n = count[0] if count.numel() else torch.tensor(1.0)
                    unbiased = var * n / (n - 1).clamp(min=1)
                    running_mean.mul_(1 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
                    running_var.mul_(1 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
        if num_batches_tracked is not None:
            with torch.no_grad():
                num_batches_tracked.add_(1)
        has_z = z is not None
        if native:
            y = C.bn_elemt(x, mean, invstd, weight, bias, channel_last, fuse_relu,
                           z=z.contiguous() if has_z else None)
        else:
            sh = _bshape(x, channel_last)
            y = (x.float() - mean.view(sh)) * invstd.view(sh)
            if weight is not None:
                y = y * weight.float().view(sh)
            if bias is not None:
                y = y + bias.float().view(sh)
            if has_z:
                y = y + z.float()
            if fuse_relu:
                y = torch.relu(y)
            y = y.to(x.dtype)
        # the global count stays on the device (a float(count) here was one host round trip per
        # BatchNorm layer per forward)
        ctx.save_for_backward(x, weight, mean, invstd, y if fuse_relu else None, count)
        ctx.cfg = (group, channel_last, fuse_relu, native, bias is not None, has_z)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, invstd, y, count = ctx.saved_tensors
        group, channel_last, fuse_relu, native, has_bias, has_z = ctx.cfg
        dy = dy.contiguous()
        if fuse_relu and not native:
            dy = dy * (y > 0).to(dy.dtype)
        ym = y if (fuse_relu and native) else None  # the kernels mask with the saved output
        if native:
            C = _ext.require()
            sums = C.bn_bwd_reduce(dy, x, mean, channel_last, ym=ym)
        else:
            sh = _bshape(x, channel_last)
            dims = [d for d in range(x.dim()) if d != (x.dim() - 1 if channel_last else 1)]
            dyf = dy.float()
            sums = torch.stack([dyf.sum(dims), (dyf * (x.float() - mean.view(sh))).sum(dims)])
        if _world(group) > 1:
            dist.all_reduce(sums, group=group)
        dw = (sums[1] * invstd).to(weight.dtype) if weight is not None and ctx.needs_input_grad[1] else None
        db = sums[0].to(weight.dtype) if has_bias and ctx.needs_input_grad[2] else None
        dz = None
        if native:
            dx, dz = C.bn_bwd_elemt(dy, x, mean, invstd, weight, sums, count.contiguous(), channel_last, ym=ym,
                                    with_dz=has_z and ym is not None)
            if has_z and ym is None:
                dz = dy  # no ReLU: the residual's gradient is dy itself
        else:
            sh = _bshape(x, channel_last)
            total = count.clamp(min=1)
            mdy = (sums[0] / total).view(sh)
            mdx = (sums[1] / total).view(sh)
            xm = x.float() - mean.view(sh)
            dx = (dy.float() - mdy - xm * (invstd ** 2).view(sh) * mdx) * invstd.view(sh)
            if weight is not None:
                dx = dx * weight.float().view(sh)
            dx = dx.to(x.dtype)
            dz = dy if has_z else None
        return dx, dw, db, None, None, None, None, None, None, None, (dz if has_z else None), None


class SyncBatchNorm(_BatchNorm):
    """Batch normalisation with statistics synchronised across ``process_group``."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None, channel_last=False, fuse_relu=False):
        super().__init__(num_features, eps=eps, momentum=momentum, affine=affine,
                         track_running_stats=track_running_stats)
        self.process_group = process_group
        self.channel_last = channel_last
        self.fuse_relu = fuse_relu

    def _check_input_dim(self, input):
        if input.dim() < 2:
            raise ValueError("expected at least 2D input (got {}D input)".format(input.dim()))

    def _specify_process_group(self, process_group):
        self.process_group = process_group

    def _specify_channel_last(self, channel_last):
        self.channel_last = channel_last

    def forward(self, input, z=None):
        """BN(input), plus ``z`` (a residual of input's shape, added after the affine transform) and
        the ReLU when ``fuse_relu`` — relu(BN(input) + z), NVIDIA Apex's fused SyncBatchNorm
        semantics — in one HIP kernel each way."""
        self._check_input_dim(input)
        if (not self.channel_last and input.dim() == 4 and input.shape[1] > 1
                and input.is_contiguous(memory_format=torch.channels_last) and not input.is_contiguous()):
            # torch channels_last (NCHW shape, NHWC storage): run the NHWC kernels on the
            # zero-copy [N, H, W, C] view instead of transposing to NCHW and back
            self.channel_last = True
            try:
                zz = z.permute(0, 2, 3, 1) if z is not None else None
                return self.forward(input.permute(0, 2, 3, 1), zz).permute(0, 3, 1, 2)
            finally:
                self.channel_last = False
        use_batch_stats = self.training or not self.track_running_stats
        if not use_batch_stats:
            mean = self.running_mean.float()
            invstd = torch.rsqrt(self.running_var.float() + self.eps)
            if _ext.use_native(input):
                y = _ext.require().bn_elemt(input.contiguous(), mean, invstd, self.weight, self.bias,
                                            self.channel_last, self.fuse_relu,
                                            z=z.contiguous() if z is not None else None)
                return y
            sh = _bshape(input, self.channel_last)
            y = (input.float() - mean.view(sh)) * invstd.view(sh)
            if self.weight is not None:
                y = y * self.weight.float().view(sh) + self.bias.float().view(sh)
            if z is not None:
                y = y + z.float()
            y = torch.relu(y) if self.fuse_relu else y
            return y.to(input.dtype)
        track = self.training and self.track_running_stats
        if self.momentum is not None:
            momentum = self.momentum
        elif track:  # cumulative moving average (torch semantics); one host read, this mode only
            momentum = 1.0 / float(self.num_batches_tracked + 1)
        else:
            momentum = 0.0
        # num_batches_tracked is incremented by the function (inside the combine kernel when it can)
        return SyncBatchnormFunction.apply(input, self.weight, self.bias,
                                           self.running_mean if self.track_running_stats else None,
                                           self.running_var if self.track_running_stats else None,
                                           self.eps, momentum, self.process_group, self.channel_last,
                                           self.fuse_relu, z, self.num_batches_tracked if track else None)


def convert_syncbn_model(module, process_group=None, channel_last=False):
    """Recursively replace every ``torch.nn.modules.batchnorm._BatchNorm`` with SyncBatchNorm."""
    mod = module
    if isinstance(module, _BatchNorm) and not isinstance(module, SyncBatchNorm):
        mod = SyncBatchNorm(module.num_features, module.eps, module.momentum, module.affine,
                            module.track_running_stats, process_group, channel_last=channel_last)
        mod.running_mean = module.running_mean
        mod.running_var = module.running_var
        mod.num_batches_tracked = module.num_batches_tracked
        if module.affine:
            mod.weight.data = module.weight.data.clone().detach()
            mod.bias.data = module.bias.data.clone().detach()
    for name, child in module.named_children():
        mod.add_module(name, convert_syncbn_model(child, process_group=process_group,
                                                  channel_last=channel_last))
    del module
    return mod


def create_syncbn_process_group(group_size):
    """Split the world into groups of ``group_size`` consecutive ranks; returns this rank's
    group (0 -> None, i.e. the whole world)."""
    if group_size == 0:
        return None
    world_size = dist.get_world_size()
    assert world_size >= group_size
    assert world_size % group_size == 0
    group = None
    for group_num in range(world_size // group_size):
        ranks = list(range(group_num * group_size, (group_num + 1) * group_size))
        cur = dist.new_group(ranks=ranks)
        if dist.get_rank() // group_size == group_num:
            group = cur
    assert group is not None
    return group
