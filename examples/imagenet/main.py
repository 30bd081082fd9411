"""ImageNet-style ResNet training on MI355X with apex — one process per GPU.

Covers the three reference scripts (examples/imagenet/main.py, main_fp16_optimizer.py,
main_reducer.py) behind one CLI:
  --precision manual     network_to_half/bf16 + prep_param_lists + model_grads_to_master_grads
                         + master_params_to_model_params with a static loss scale (R-32)
  --precision fp16_opt   FP16_Optimizer wrapping SGD, static or dynamic loss scale (R-33)
  --precision amp        amp.initialize(opt_level O2 by default) + FusedSGD
  --precision fp32       no mixed precision
  --reducer              apex.parallel.Reducer instead of DDP: grads all-reduced once, by the
                         user, after backward (R-34); default is apex DDP (overlapped buckets)
  --sync-bn              convert BatchNorm to apex SyncBatchNorm

Data: no dataset is downloadable here, so the loader synthesises uint8 HWC images with a
class-dependent colour bias (learnable) — the same shape and dtype a JPEG decoder would hand
over. The prefetcher moves each batch to the GPU on a side stream and normalises it with
the fused K-09 kernel (uint8 NHWC -> bf16/fp16 channels_last in one pass). Throughput is
reported as world x batch / batch_time (reference main.py:348,354).

  torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 8 examples/imagenet/main.py -a resnet50 -b 256
"""
from __future__ import annotations

import argparse
import os
import shutil
import time

import torch
import torch.distributed as dist
import torch.nn as nn

import apex
from apex import amp
from apex.fp16_utils import (FP16_Optimizer, master_params_to_model_params, model_grads_to_master_grads,
                             network_to_bf16, network_to_half, prep_param_lists)
from apex.models import resnet
from apex.parallel import DistributedDataParallel as DDP
from apex.parallel import Reducer, convert_syncbn_model
from apex.utils.metrics import AverageMeter, reduce_scalars
from apex.utils.prefetch import DataPrefetcher

ARCHS = ["resnet18", "resnet34", "resnet50", "resnet101", "resnet152"]


def parse(argv=None):
    p = argparse.ArgumentParser(description="apex ImageNet-style training (synthetic data)")
    p.add_argument("--arch", "-a", default="resnet18", choices=ARCHS)
    p.add_argument("-j", "--workers", default=4, type=int)
    p.add_argument("--epochs", default=1, type=int)
    p.add_argument("--start-epoch", default=0, type=int)
    p.add_argument("-b", "--batch-size", default=256, type=int, help="per-process batch")
    p.add_argument("--lr", default=0.1, type=float, help="lr for a global batch of 256")
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("--weight-decay", "--wd", default=1e-4, type=float)
    p.add_argument("--print-freq", "-p", default=10, type=int)
    p.add_argument("--resume", default="", type=str)
    p.add_argument("--checkpoint", default="checkpoint.pt", type=str)
    p.add_argument("-e", "--evaluate", action="store_true")
    p.add_argument("--precision", default="amp", choices=["manual", "fp16_opt", "amp", "fp32"])
    p.add_argument("--half-dtype", default="bf16", choices=["bf16", "fp16"])
    p.add_argument("--opt-level", default="O2")
    p.add_argument("--static-loss-scale", type=float, default=1.0)
    p.add_argument("--dynamic-loss-scale", action="store_true")
    p.add_argument("--reducer", action="store_true")
    p.add_argument("--sync-bn", action="store_true")
    p.add_argument("--image-size", default=224, type=int)
    p.add_argument("--num-classes", default=1000, type=int)
    p.add_argument("--train-size", default=2560, type=int, help="synthetic images per epoch")
    p.add_argument("--val-size", default=512, type=int)
    p.add_argument("--prof", action="store_true", help="stop after a few iterations (profiling)")
    p.add_argument("--local_rank", "--local-rank", default=int(os.environ.get("LOCAL_RANK", 0)), type=int)
    return p.parse_args(argv)


class SyntheticImages(torch.utils.data.Dataset):
    """Deterministic uint8 HWC images; class c adds a per-channel bias so the task is learnable."""

    def __init__(self, n, size, num_classes, seed):
        self.n, self.size, self.nc, self.seed = n, size, num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        y = int(torch.randint(0, self.nc, (1,), generator=g))
        img = torch.randint(0, 160, (self.size, self.size, 3), dtype=torch.uint8, generator=g)
        bias = torch.tensor([(y * 37) % 96, (y * 61) % 96, (y * 89) % 96], dtype=torch.uint8)
        return img + bias, y


def collate(batch):
    return torch.stack([b[0] for b in batch]), torch.tensor([b[1] for b in batch], dtype=torch.int64)


def accuracy(output, target, topk=(1,)):
    maxk = max(topk)
    _, pred = output.topk(maxk, 1, True, True)
    correct = pred.t().eq(target.view(1, -1))
    return [correct[:k].reshape(-1).float().sum() * (100.0 / target.size(0)) for k in topk]


def adjust_learning_rate(args, optimizer, epoch, step, len_epoch):
    """Step decay (x0.1 every 30 epochs, extra at 80) with a 5-epoch linear warmup."""
    factor = epoch // 30 + (1 if epoch >= 80 else 0)
    lr = args.lr_scaled * (0.1 ** factor)
    if epoch < 5:
        lr = lr * float(1 + step + epoch * len_epoch) / (5.0 * len_epoch)
    for g in optimizer.param_groups:
        g["lr"] = lr


class Trainer:
    def __init__(self, args):
        self.args = args
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.cuda = torch.cuda.is_available()
        if self.cuda:
            torch.cuda.set_device(args.local_rank)
        if self.world > 1:
            dist.init_process_group("nccl" if self.cuda else "gloo", init_method="env://")
        self.rank = dist.get_rank() if self.world > 1 else 0
        self.device = torch.device("cuda", args.local_rank) if self.cuda else torch.device("cpu")
        self.half = torch.bfloat16 if args.half_dtype == "bf16" else torch.float16
        args.lr_scaled = args.lr * args.batch_size * self.world / 256.0
        self.best_prec1 = 0.0
        self._build()

    def log(self, *a):
        if self.rank == 0:
            print(*a, flush=True)

    def _build(self):
        a = self.args
        model = getattr(resnet, a.arch)(num_classes=a.num_classes)
        if a.sync_bn:
            model = convert_syncbn_model(model)
        cl = self.cuda
        model = model.to(self.device, memory_format=torch.channels_last if cl else torch.contiguous_format)
        self.input_dtype = torch.float32
        self.master_params = None
        if a.precision == "manual":
            model = network_to_bf16(model) if self.half == torch.bfloat16 else network_to_half(model)
            self.model_params, self.master_params = prep_param_lists(model)
            opt = torch.optim.SGD(self.master_params, a.lr_scaled, momentum=a.momentum,
                                  weight_decay=a.weight_decay)
            self.input_dtype = self.half
        elif a.precision == "fp16_opt":
            model = network_to_bf16(model) if self.half == torch.bfloat16 else network_to_half(model)
            opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), a.lr_scaled, momentum=a.momentum,
                                                 weight_decay=a.weight_decay),
                                 static_loss_scale=a.static_loss_scale, dynamic_loss_scale=a.dynamic_loss_scale,
                                 verbose=False)
            self.input_dtype = self.half
        elif a.precision == "amp":
            from apex.optimizers import FusedSGD

            opt = FusedSGD(model.parameters(), a.lr_scaled, momentum=a.momentum, weight_decay=a.weight_decay)
            model, opt = amp.initialize(model, opt, opt_level=a.opt_level, cast_model_type=self.half
                                        if a.opt_level in ("O2", "O3") else None,
                                        loss_scale="dynamic" if a.dynamic_loss_scale else a.static_loss_scale,
                                        verbosity=0)
            self.input_dtype = self.half if a.opt_level in ("O2", "O3") else torch.float32
        else:
            opt = torch.optim.SGD(model.parameters(), a.lr_scaled, momentum=a.momentum, weight_decay=a.weight_decay)
        self.reducer = None
        if self.world > 1:
            if a.reducer:  # Reducer is not a Module: the model stays as is, grads reduced by hand
                self.reducer = Reducer(model)
            else:
                model = DDP(model)
        self.model, self.optimizer = model, opt
        self.criterion = nn.CrossEntropyLoss()
        if a.resume:
            self.resume(a.resume)
        kw = dict(batch_size=a.batch_size, num_workers=a.workers, collate_fn=collate, pin_memory=self.cuda,
                  drop_last=True)
        tr = SyntheticImages(a.train_size, a.image_size, a.num_classes, seed=1)
        va = SyntheticImages(a.val_size, a.image_size, a.num_classes, seed=2)
        samp = torch.utils.data.distributed.DistributedSampler(tr) if self.world > 1 else None
        self.train_sampler = samp
        self.train_loader = torch.utils.data.DataLoader(tr, shuffle=samp is None, sampler=samp, **kw)
        vsamp = torch.utils.data.distributed.DistributedSampler(va, shuffle=False) if self.world > 1 else None
        self.val_loader = torch.utils.data.DataLoader(va, sampler=vsamp, **kw)

    # ----------------------------------------------------------- checkpoints
    def _inner(self):
        m = self.model
        return m.module if isinstance(m, DDP) else m

    def save(self, epoch, is_best):
        if self.rank != 0:
            return
        state = {"epoch": epoch + 1, "arch": self.args.arch, "state_dict": self._inner().state_dict(),
                 "best_prec1": self.best_prec1, "optimizer": self.optimizer.state_dict()}
        if self.master_params is not None:
            state["master_params"] = [p.detach() for p in self.master_params]
        torch.save(state, self.args.checkpoint)
        if is_best:
            shutil.copyfile(self.args.checkpoint, os.path.splitext(self.args.checkpoint)[0] + "_best.pt")

    def resume(self, path):
        ck = torch.load(path, map_location=self.device, weights_only=True)
        self.args.start_epoch = ck["epoch"]
        self.best_prec1 = ck["best_prec1"]
        self._inner().load_state_dict(ck["state_dict"])
        self.optimizer.load_state_dict(ck["optimizer"])
        if self.master_params is not None and "master_params" in ck:
            for m, s in zip(self.master_params, ck["master_params"]):
                m.data.copy_(s)
        self.log("=> resumed '{}' (epoch {})".format(path, ck["epoch"]))

    # ----------------------------------------------------------- loops
    def _prefetcher(self, loader):
        return DataPrefetcher(loader, device=self.device, nhwc=True, channels_last=self.cuda,
                              dtype=self.input_dtype)

    def _backward_step(self, loss):
        a = self.args
        if a.precision == "manual":
            (loss * a.static_loss_scale).backward()
            if a.reducer and self.world > 1:
                self.reducer.reduce()
            model_grads_to_master_grads(self.model_params, self.master_params)
            if a.static_loss_scale != 1.0:
                for p in self.master_params:
                    p.grad.data.mul_(1.0 / a.static_loss_scale)
            self.optimizer.step()
            master_params_to_model_params(self.model_params, self.master_params)
        elif a.precision == "fp16_opt":
            self.optimizer.backward(loss, update_master_grads=not (a.reducer and self.world > 1))
            if a.reducer and self.world > 1:
                self.reducer.reduce()
                self.optimizer.update_master_grads()
            self.optimizer.step()
        elif a.precision == "amp":
            with amp.scale_loss(loss, self.optimizer) as scaled:
                scaled.backward()
            if a.reducer and self.world > 1:
                self.reducer.reduce()
            self.optimizer.step()
        else:
            loss.backward()
            if a.reducer and self.world > 1:
                self.reducer.reduce()
            self.optimizer.step()

    def _zero_grad(self):
        if self.args.precision == "manual":
            self.model.zero_grad()
            for p in self.master_params:
                p.grad = None
        else:
            self.optimizer.zero_grad()

    def train(self, epoch):
        a = self.args
        bt, losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter(), AverageMeter()
        self.model.train()
        n = len(self.train_loader)
        end = time.time()
        for i, (x, y) in enumerate(self._prefetcher(self.train_loader)):
            adjust_learning_rate(a, self.optimizer, epoch, i, n)
            out = self.model(x)
            loss = self.criterion(out.float(), y)
            self._zero_grad()
            self._backward_step(loss)
            if i % a.print_freq == 0 or i == n - 1:
                p1, p5 = accuracy(out.float().detach(), y, (1, 5))
                # one collective for the three metrics (reference main.py:485-489 issues one each)
                rl, r1, r5 = reduce_scalars(loss, p1, p5)
                if self.cuda:
                    torch.cuda.synchronize()
                losses.update(float(rl), x.size(0))
                top1.update(float(r1), x.size(0))
                top5.update(float(r5), x.size(0))
                bt.update((time.time() - end) / (a.print_freq if i else 1))
                end = time.time()
                self.log("Epoch [{}][{}/{}]  Time {:.3f} ({:.3f})  Speed {:.1f} img/s  Loss {:.4f}  "
                         "Prec@1 {:.2f}  Prec@5 {:.2f}".format(epoch, i, n, bt.val, bt.avg,
                                                               self.world * a.batch_size / max(bt.val, 1e-9),
                                                               losses.val, top1.val, top5.val))
            if a.prof and i >= 10:
                break
        return losses.avg

    @torch.no_grad()
    def validate(self):
        losses, top1, top5 = AverageMeter(), AverageMeter(), AverageMeter()
        self.model.eval()
        for x, y in self._prefetcher(self.val_loader):
            out = self.model(x).float()
            loss = self.criterion(out, y)
            p1, p5 = accuracy(out, y, (1, 5))
            rl, r1, r5 = reduce_scalars(loss, p1, p5)
            losses.update(float(rl), x.size(0))
            top1.update(float(r1), x.size(0))
            top5.update(float(r5), x.size(0))
        self.log(" * Prec@1 {:.3f} Prec@5 {:.3f}".format(top1.avg, top5.avg))
        return top1.avg

    def run(self):
        a = self.args
        if a.evaluate:
            return self.validate()
        prec1 = 0.0
        for epoch in range(a.start_epoch, a.epochs):
            if self.train_sampler is not None:
                self.train_sampler.set_epoch(epoch)
            self.train(epoch)
            if a.prof:
                break
            prec1 = self.validate()
            is_best = prec1 > self.best_prec1
            self.best_prec1 = max(prec1, self.best_prec1)
            self.save(epoch, is_best)
        return prec1


def main(argv=None):
    args = parse(argv)
    if torch.cuda.is_available():
        apex._ext.require()
    t = Trainer(args)
    out = t.run()
    if t.world > 1:
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
