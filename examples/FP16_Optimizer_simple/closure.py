"""FP16_Optimizer with a closure-driven optimizer step (LBFGS-style API): the closure zeroes
grads, computes the loss and calls ``optimizer.backward``; with dynamic loss scaling an
overflowing closure evaluation is retried at a lower scale before the step proceeds.
(Capability of reference examples/FP16_Optimizer_simple/closure.py.)
"""
import argparse

import torch

from apex.fp16_utils import FP16_Optimizer

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
args = ap.parse_args()

dev = "cuda" if torch.cuda.is_available() else "cpu"
low = torch.float16 if dev == "cuda" else torch.bfloat16
N, D_in, D_out = 64, 1024, 16
x = torch.randn(N, D_in, device=dev).to(low)
y = torch.randn(N, D_out, device=dev).to(low)
model = torch.nn.Linear(D_in, D_out).to(dev, low)
optimizer = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=1e-3), dynamic_loss_scale=True, verbose=False)
loss_fn = torch.nn.MSELoss()


def closure():
    optimizer.zero_grad()
    loss = loss_fn(model(x).float(), y.float())
    optimizer.backward(loss)
    return loss


for t in range(args.steps):
    loss = optimizer.step(closure)
print("final loss = {:.5f}".format(float(loss.detach())))
