"""Run the fp32 H=128 motion model for a few SGD steps several times with the
stacked-layer pipeline on and off and print every loss (bitwise
reproducibility check of both schedules)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_rnn_amd.models.motion import MotionModel  # noqa: E402


def run(cell, pipe, steps=3, B=64, T=32):
    os.environ["PDRNN_TUNE"] = "large_pipe=" + ("1" if pipe else "0")
    torch.manual_seed(3)
    model = MotionModel(9, 128, 2, 6, cell=cell).cuda()
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    x = torch.randn(B, T, 9, device="cuda")
    y = torch.randint(0, 6, (B,), device="cuda")
    out = []
    for _ in range(steps):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        g = torch.cat([p.grad.flatten() for p in model.parameters()])
        out.append((float(loss), float(g.double().norm())))
        opt.step()
    return out


cells = sys.argv[1].split(",") if len(sys.argv) > 1 else ["lstm", "gru"]
extra = sys.argv[2:]  # "ENV=V[,ENV2=V2]" configurations of the layer-by-layer path
for cell in cells:
    for pipe in (1, 1, 0, 0, 0):
        print(cell, "pipe" if pipe else "whole", " ".join(f"{l:.9f}/{g:.9f}" for l, g in run(cell, pipe)), flush=True)
    for cfg in extra:
        kv = dict(e.split("=", 1) for e in cfg.split(","))
        os.environ.update(kv)
        for _ in range(3):
            print(cell, "whole", cfg, " ".join(f"{l:.9f}/{g:.9f}" for l, g in run(cell, 0)), flush=True)
        for k in kv:
            del os.environ[k]
