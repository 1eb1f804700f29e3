#!/usr/bin/env python
"""Toy data-parallel example: DDP over the framework's bucketed reducer.

Behavioural counterpart of reference src/example/example_ddp.py:1-99: the same
seeded ``Linear(10,10)-ReLU-Linear(10,5)`` MLP, a 24-sample random dataset,
SGD lr 1e-3, per-rank batch ``12 // world`` and the same diagnostic prints
(parameter sums before/after the initial broadcast, batch sums, loss,
post-step parameter and gradient sums).  The pass criterion is the
reference README's: the final parameters are identical on every rank.

Differences by design: the backend is gloo (CPU) or RCCL (GPU) instead of MPI
(torch-ROCm has no MPI backend), and ``--shard`` optionally enables the
sampler the reference left commented out (example_ddp.py:57-63).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        src/example/example_ddp.py --backend gloo
"""
import argparse
import json

import _bootstrap  # noqa: F401

import torch
from torch import nn
from torch.utils.data import DataLoader, Dataset

from pytorch_distributed_rnn_amd.data.loader import ShardedSampler
from pytorch_distributed_rnn_amd.parallel import env
from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel


class ToyModel(nn.Module):
    def __init__(self):
        super().__init__()
        self.net1 = nn.Linear(10, 10)
        self.relu = nn.ReLU()
        self.net2 = nn.Linear(10, 5)

    def forward(self, x):
        return self.net2(self.relu(self.net1(x)))


class ToyDataset(Dataset):
    def __init__(self, size: int, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(size, 10, generator=g)
        self.y = torch.randn(size, 5, generator=g)

    def __len__(self):
        return self.x.shape[0]

    def __getitem__(self, i):
        return self.x[i], self.y[i]


def _psum(module) -> float:
    return float(sum(p.detach().double().sum() for p in module.parameters()))


def run(rank: int, world: int, device: torch.device, shard: bool = False, seed: int = 0,
        global_batch: int = 12, quiet: bool = False) -> dict:
    torch.manual_seed(seed + rank)  # deliberately different init per rank: DDP must broadcast rank 0's
    model = ToyModel().to(device)
    before = _psum(model)
    ddp = DistributedDataParallel(model)
    after = _psum(model)
    opt = torch.optim.SGD(ddp.parameters(), lr=1e-3)
    data = ToyDataset(24, seed)
    sampler = ShardedSampler(len(data), num_replicas=world, rank=rank, shuffle=False) if shard else None
    loader = DataLoader(data, batch_size=global_batch // world, sampler=sampler)
    losses = []

    def say(msg):
        if not quiet:
            print(f"[rank {rank}] {msg}", flush=True)

    say(f"param sum before broadcast {before:.6f}, after {after:.6f}")
    for x, y in loader:
        x, y = x.to(device), y.to(device)
        say(f"batch sum {float(x.sum()):.6f}")
        opt.zero_grad()
        loss = nn.functional.mse_loss(ddp(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
        say(f"loss {float(loss):.6f} param sum {_psum(model):.6f} "
            f"grad sum {float(sum(p.grad.double().sum() for p in model.parameters())):.6f}")
    flat = torch.cat([p.detach().flatten().cpu() for p in model.parameters()])
    return {"rank": rank, "losses": losses, "final_param_sum": _psum(model), "params": flat.tolist()}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default=None)
    ap.add_argument("--shard", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="write each rank's result as JSON (rank-suffixed)")
    args = ap.parse_args(argv)
    info = env.init_distributed(args.backend)
    device = env.setup_device(info) if torch.distributed.get_backend() == "nccl" else torch.device("cpu")
    res = run(env.get_rank(), env.get_world_size(), device, shard=args.shard, seed=args.seed)
    print(f"[rank {res['rank']}] final param sum {res['final_param_sum']:.8f}", flush=True)
    if args.out:
        with open(f"{args.out}.{res['rank']}", "w") as f:
            json.dump(res, f)
    env.shutdown()


if __name__ == "__main__":
    main()
