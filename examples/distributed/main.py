"""MNIST-style CNN trained with apex.parallel.DistributedDataParallel, one process per GPU
(RCCL) or per CPU rank (gloo). Capability of reference examples/distributed/main.py; the
dataset is synthesised (28x28 class-dependent blobs) because nothing can be downloaded here.

  python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 2 examples/distributed/main.py
  python -m apex.parallel.multiproc examples/distributed/main.py
"""
from __future__ import annotations

import argparse
import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from apex.parallel import DistributedDataParallel as DDP
from apex.utils.metrics import reduce_tensor


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 10, kernel_size=5)
        self.conv2 = nn.Conv2d(10, 20, kernel_size=5)
        self.conv2_drop = nn.Dropout2d()
        self.fc1 = nn.Linear(320, 50)
        self.fc2 = nn.Linear(50, 10)

    def forward(self, x):
        x = F.relu(F.max_pool2d(self.conv1(x), 2))
        x = F.relu(F.max_pool2d(self.conv2_drop(self.conv2(x)), 2))
        x = F.dropout(F.relu(self.fc1(x.flatten(1))), training=self.training)
        return F.log_softmax(self.fc2(x), dim=1)


def synthetic_digits(n, seed):
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g)
    yy, xx = torch.meshgrid(torch.arange(28.0), torch.arange(28.0), indexing="ij")
    cy, cx = 6 + 2 * (y // 5 * 7).float(), 4 + 4 * (y % 5).float()
    blob = torch.exp(-((yy[None] - cy[:, None, None]) ** 2 + (xx[None] - cx[:, None, None]) ** 2) / 8.0)
    x = blob + 0.3 * torch.randn(n, 28, 28, generator=g)
    return torch.utils.data.TensorDataset(((x - 0.1307) / 0.3081).unsqueeze(1), y)


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--test-batch-size", type=int, default=1000)
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--no-cuda", action="store_true")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--log-interval", type=int, default=10)
    p.add_argument("--train-size", type=int, default=6000)
    p.add_argument("--local_rank", "--local-rank", default=int(os.environ.get("LOCAL_RANK", 0)), type=int)
    args = p.parse_args(argv)
    cuda = not args.no_cuda and torch.cuda.is_available()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if cuda:
        torch.cuda.set_device(args.local_rank)
    if world > 1:
        dist.init_process_group("nccl" if cuda else "gloo", init_method="env://")
    rank = dist.get_rank() if world > 1 else 0
    dev = torch.device("cuda", args.local_rank) if cuda else torch.device("cpu")
    torch.manual_seed(args.seed)
    train_set, test_set = synthetic_digits(args.train_size, 1), synthetic_digits(1000, 2)
    sampler = torch.utils.data.distributed.DistributedSampler(train_set) if world > 1 else None
    loader = torch.utils.data.DataLoader(train_set, batch_size=args.batch_size, shuffle=sampler is None,
                                         sampler=sampler)
    test_loader = torch.utils.data.DataLoader(test_set, batch_size=args.test_batch_size)
    model = Net().to(dev)
    if world > 1:
        model = DDP(model)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum)
    acc = 0.0
    for epoch in range(1, args.epochs + 1):
        if sampler is not None:
            sampler.set_epoch(epoch)
        model.train()
        for i, (x, y) in enumerate(loader):
            x, y = x.to(dev), y.to(dev)
            opt.zero_grad()
            loss = F.nll_loss(model(x), y)
            loss.backward()
            opt.step()
            if i % args.log_interval == 0:
                rl = reduce_tensor(loss.detach().reshape(1))
                if rank == 0:
                    print("Train Epoch: {} [{}/{}]\tLoss: {:.6f}".format(epoch, i * len(x), len(loader.dataset) //
                                                                         world, float(rl)), flush=True)
        model.eval()
        correct, total = 0, 0
        with torch.no_grad():
            for x, y in test_loader:
                x, y = x.to(dev), y.to(dev)
                correct += int((model(x).argmax(1) == y).sum())
                total += len(y)
        acc = 100.0 * correct / total
        if rank == 0:
            print("Test set: Accuracy: {}/{} ({:.0f}%)".format(correct, total, acc), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return acc


if __name__ == "__main__":
    main()
