#!/usr/bin/env python
"""Point-to-point example: rank 0 sends one tensor to every other rank.

Counterpart of reference src/example/example_distributed.py:1-24 (which used
the MPI backend).  Here the payload moves with the framework's communicator:
RCCL ``send``/``recv`` over xGMI when ranks own GPUs, gloo on the CPU.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        src/example/example_distributed.py [--backend gloo]
    mpirun -np 2 python src/example/example_distributed.py   (rank from OMPI_* env)
"""
import argparse

import _bootstrap  # noqa: F401

import torch

from pytorch_distributed_rnn_amd.parallel import env
from pytorch_distributed_rnn_amd.parallel.comm import get_comm


def run(rank: int, world: int, device: torch.device) -> float:
    comm = get_comm()
    tensor = torch.zeros(1, device=device)
    if rank == 0:
        tensor += 1
        for dst in range(1, world):
            comm.send(tensor, dst)
    else:
        comm.recv(tensor, 0)
    comm.wait()
    value = float(tensor.item())
    print(f"Rank {rank} has data {value}")
    return value


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default=None)
    args = ap.parse_args(argv)
    info = env.init_distributed(args.backend)
    device = env.setup_device(info) if torch.distributed.get_backend() == "nccl" else torch.device("cpu")
    run(env.get_rank(), env.get_world_size(), device)
    env.shutdown()


if __name__ == "__main__":
    main()
