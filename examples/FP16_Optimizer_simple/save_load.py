"""Checkpointing with FP16_Optimizer: ``state_dict()`` holds the fp32 masters, the wrapped
optimizer's state and the loss-scaler state as plain containers, so the checkpoint reloads with
``torch.load(..., weights_only=True)``; training resumes bit-identically.
(Capability of reference examples/FP16_Optimizer_simple/save_load.py.)
"""
import argparse
import os
import tempfile

import torch

from apex.fp16_utils import FP16_Optimizer

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--ckpt", default=os.path.join(tempfile.gettempdir(), "fp16_opt_ckpt.pt"))
args = ap.parse_args()

dev = "cuda" if torch.cuda.is_available() else "cpu"
low = torch.float16 if dev == "cuda" else torch.bfloat16
N, D_in, D_out = 64, 1024, 16
torch.manual_seed(0)
x = torch.randn(N, D_in, device=dev).to(low)
y = torch.randn(N, D_out, device=dev).to(low)
loss_fn = torch.nn.MSELoss()


def build():
    torch.manual_seed(1)
    model = torch.nn.Linear(D_in, D_out).to(dev, low)
    opt = FP16_Optimizer(torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9), dynamic_loss_scale=True,
                         verbose=False)
    return model, opt


def train(model, opt, n):
    for _ in range(n):
        opt.zero_grad()
        loss = loss_fn(model(x).float(), y.float())
        opt.backward(loss)
        opt.step()
    return loss


model, optimizer = build()
train(model, optimizer, args.steps)
torch.save({"model": model.state_dict(), "optimizer": optimizer.state_dict()}, args.ckpt)
ref = train(model, optimizer, args.steps)

model2, optimizer2 = build()
ck = torch.load(args.ckpt, weights_only=True)
model2.load_state_dict(ck["model"])
optimizer2.load_state_dict(ck["optimizer"])
resumed = train(model2, optimizer2, args.steps)
same = all(torch.equal(a, b) for a, b in zip(model.parameters(), model2.parameters()))
print("final loss = {:.5f}, resumed = {:.5f}, identical params: {}".format(float(ref.detach()),
                                                                          float(resumed.detach()), same))
