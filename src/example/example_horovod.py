#!/usr/bin/env python
"""Toy Horovod-mode example: optimizer-wrapping data parallelism.

Counterpart of reference src/example/example_horovod.py:1-83: the toy MLP,
``broadcast_parameters`` from rank 0, ``DistributedOptimizer(SGD)`` with
per-tensor gradient hooks fused into one all-reduce buffer, and a sharded
sampler -- on the framework's horovod-compatible API
(``pytorch_distributed_rnn_amd.parallel.horovod``) over RCCL or gloo.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        src/example/example_horovod.py --backend gloo
"""
import argparse
import json

import _bootstrap  # noqa: F401

import torch
from torch import nn
from torch.utils.data import DataLoader

from example_ddp import ToyDataset, ToyModel, _psum
from pytorch_distributed_rnn_amd.data.loader import ShardedSampler
from pytorch_distributed_rnn_amd.parallel import horovod as hvd


def run(device: torch.device, seed: int = 0, global_batch: int = 12) -> dict:
    rank, world = hvd.rank(), hvd.size()
    torch.manual_seed(seed + rank)
    model = ToyModel().to(device)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    opt = hvd.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=1e-3),
                                   named_parameters=model.named_parameters())
    data = ToyDataset(24, seed)
    loader = DataLoader(data, batch_size=global_batch // world,
                        sampler=ShardedSampler(len(data), num_replicas=world, rank=rank))
    losses = []
    for x, y in loader:
        x, y = x.to(device), y.to(device)
        opt.zero_grad()
        loss = nn.functional.mse_loss(model(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
        print(f"[rank {rank}] loss {float(loss):.6f} param sum {_psum(model):.6f}", flush=True)
    flat = torch.cat([p.detach().flatten().cpu() for p in model.parameters()])
    return {"rank": rank, "losses": losses, "final_param_sum": _psum(model), "params": flat.tolist()}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args(argv)
    hvd.init(args.backend)
    device = (torch.device("cuda", hvd.local_rank()) if torch.distributed.get_backend() == "nccl"
              else torch.device("cpu"))
    res = run(device, seed=args.seed)
    print(f"[rank {res['rank']}] final param sum {res['final_param_sum']:.8f}", flush=True)
    if args.out:
        with open(f"{args.out}.{res['rank']}", "w") as f:
            json.dump(res, f)
    from pytorch_distributed_rnn_amd.parallel import env
    env.shutdown()


if __name__ == "__main__":
    main()
