"""2-layer MLP — BASELINE.json config 1 ("2-layer MLP amp O0 (fp32 passthrough) + SGD on CPU,
world_size=1"): the plumbing configuration that exercises amp, the optimizers and the
scaler end to end without a GPU. Also the model of the reference's FP16_Optimizer_simple
examples (examples/FP16_Optimizer_simple/minimal.py: Linear(1024 -> 16), N = 64)."""
from __future__ import annotations

import torch
from torch import nn


class MLP(nn.Module):
    def __init__(self, d_in=1024, d_hidden=1024, d_out=16):
        super().__init__()
        self.fc1 = nn.Linear(d_in, d_hidden)
        self.act = nn.ReLU()
        self.fc2 = nn.Linear(d_hidden, d_out)

    def forward(self, x):
        return self.fc2(self.act(self.fc1(x)))


def synthetic_batch(n=64, d_in=1024, d_out=16, device="cpu", generator=None):
    return (torch.randn(n, d_in, device=device, generator=generator),
            torch.randn(n, d_out, device=device, generator=generator))
