"""FP16_Optimizer + apex DistributedDataParallel, one process per GPU (RCCL), or per CPU rank
(gloo) without a GPU. Launch:

  python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node 2 \\
      examples/FP16_Optimizer_simple/distributed/distributed_data_parallel.py
  (or: python -m apex.parallel.multiproc examples/.../distributed_data_parallel.py)
(Capability of reference examples/FP16_Optimizer_simple/distributed_apex*/.)
"""
import argparse
import os

import torch
import torch.distributed as dist

from apex.fp16_utils import FP16_Optimizer
from apex.parallel import DistributedDataParallel as DDP

ap = argparse.ArgumentParser()
ap.add_argument("--local_rank", "--local-rank", default=int(os.environ.get("LOCAL_RANK", 0)), type=int)
ap.add_argument("--steps", type=int, default=500)
ap.add_argument("--torch-ddp", action="store_true",
                help="wrap with torch.nn.parallel.DistributedDataParallel instead of apex's (interop check)")
args = ap.parse_args()

cuda = torch.cuda.is_available()
if cuda:
    torch.cuda.set_device(args.local_rank)
dist.init_process_group("nccl" if cuda else "gloo", init_method="env://")
dev = torch.device("cuda", args.local_rank) if cuda else torch.device("cpu")
low = torch.float16 if cuda else torch.bfloat16
N, D_in, D_out = 64, 1024, 16
torch.manual_seed(dist.get_rank())
x = torch.randn(N, D_in, device=dev).to(low)
y = torch.randn(N, D_out, device=dev).to(low)
net = torch.nn.Linear(D_in, D_out).to(dev, low)
if args.torch_ddp:
    model = torch.nn.parallel.DistributedDataParallel(net, device_ids=[args.local_rank] if cuda else None)
else:
    model = DDP(net)
optimizer = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=1e-3), verbose=False)
loss_fn = torch.nn.MSELoss()
for t in range(args.steps):
    optimizer.zero_grad()
    loss = loss_fn(model(x).float(), y.float())
    optimizer.backward(loss)
    optimizer.step()
print("rank {} final loss = {:.5f}".format(dist.get_rank(), float(loss.detach())))
dist.destroy_process_group()
