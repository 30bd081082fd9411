"""FP16_Optimizer in its smallest form: a half-precision Linear(1024 -> 16) trained with SGD,
fp32 master weights and a static (or --dynamic) loss scale. On MI355X the master-grad copy +
unscale and the master -> model copy are single multi-tensor HIP launches.
(Capability of reference examples/FP16_Optimizer_simple/minimal.py.)

  python examples/FP16_Optimizer_simple/minimal.py [--dynamic] [--bf16] [--steps 200]
"""
import argparse

import torch

from apex.fp16_utils import FP16_Optimizer

ap = argparse.ArgumentParser()
ap.add_argument("--dynamic", action="store_true")
ap.add_argument("--bf16", action="store_true")
ap.add_argument("--steps", type=int, default=200)
args = ap.parse_args()

dev = "cuda" if torch.cuda.is_available() else "cpu"
low = torch.bfloat16 if (args.bf16 or dev == "cpu") else torch.float16
N, D_in, D_out = 64, 1024, 16
x = torch.randn(N, D_in, device=dev).to(low)
y = torch.randn(N, D_out, device=dev).to(low)
model = torch.nn.Linear(D_in, D_out).to(dev, low)
sgd = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9)
if args.dynamic:
    optimizer = FP16_Optimizer(sgd, dynamic_loss_scale=True, dynamic_loss_args={"scale_factor": 2}, verbose=False)
else:
    optimizer = FP16_Optimizer(sgd, static_loss_scale=128.0, verbose=False)
loss_fn = torch.nn.MSELoss()
for t in range(args.steps):
    optimizer.zero_grad()
    loss = loss_fn(model(x).float(), y.float())
    optimizer.backward(loss)  # instead of loss.backward(): scales, then copies grads to masters
    optimizer.step()
print("final loss = {:.5f} (loss scale {})".format(float(loss.detach()), optimizer.loss_scale))
