#!/usr/bin/env python
"""Single-process sanity example: one optimizer step of a ``Linear(10, 10)``.

Behavioural counterpart of reference src/example/example_single.py:1-27 (one
SGD step on random data, prints the loss).  Runs on the GPU through the
framework's fused Adam when one is present, else on the CPU.

    python src/example/example_single.py
"""
import _bootstrap  # noqa: F401

import torch
from torch import nn

from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
from pytorch_distributed_rnn_amd.utils.flat import flatten_module


def run(device: torch.device, use_adam: bool = False) -> float:
    torch.manual_seed(0)
    model = nn.Linear(10, 10).to(device)
    if use_adam:
        flatten_module(model)
        opt = FusedAdam(model.parameters(), lr=1e-3)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=0.01)
    x = torch.randn(20, 10, device=device)
    y = torch.randn(20, 10, device=device)
    opt.zero_grad()
    loss = nn.functional.mse_loss(model(x), y)
    loss.backward()
    opt.step()
    print(f"loss {loss.item():.6f} on {device}")
    return loss.item()


if __name__ == "__main__":
    run(torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
