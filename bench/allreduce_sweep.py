#!/usr/bin/env python
"""All-reduce message-size sweep on the framework's communicator -- the
measurement behind the DDP bucket cap (SURVEY §5 "Distributed communication
backend": buckets sized for RCCL rings over 7 point-to-point xGMI links).

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        bench/allreduce_sweep.py [--min-kb 64] [--max-mb 256] [--iters 20]

One rank per GPU over the native RCCL communicator (``parallel.comm.get_comm``);
on a CPU host it runs the same sweep over gloo (plumbing only).  Rank 0 prints
one JSON line per size: latency, algorithm bandwidth (bytes / time) and bus
bandwidth (2 (W-1)/W x algbw, the ring's per-link figure), timed between
barriers and device synchronisations, MAX over ranks.  Pick the bucket cap at
the knee: the smallest size whose bus bandwidth is within ~10 % of the plateau
(larger buckets only delay the first all-reduce behind the backward)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.parallel.comm import get_comm  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--min-kb", type=float, default=64)
    ap.add_argument("--max-mb", type=float, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args(argv)
    gpu = torch.cuda.is_available()
    env.init_distributed("nccl" if gpu else "gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if gpu else torch.device("cpu")
    comm = get_comm()

    def sync():
        comm.wait()
        if gpu:
            torch.cuda.synchronize(dev)

    nbytes = int(a.min_kb * 1024)
    top = int(a.max_mb * 1024 * 1024)
    while nbytes <= top:
        t = torch.ones(nbytes // 4, device=dev)
        for _ in range(a.warmup):
            comm.all_reduce(t, "sum")
        sync()
        comm.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            comm.all_reduce(t, "sum")
        sync()
        el = torch.tensor([(time.perf_counter() - t0) / a.iters], device=dev)
        comm.all_reduce(el, "max")
        sync()
        sec = float(el.item())
        algbw = nbytes / sec / 1e9
        if rank == 0:
            print(json.dumps({"bytes": nbytes, "world": world, "backend": "rccl" if gpu else "gloo",
                              "us": round(sec * 1e6, 2), "algbw_GBs": round(algbw, 3),
                              "busbw_GBs": round(algbw * 2 * (world - 1) / max(world, 1), 3)}), flush=True)
        nbytes *= 2
    env.shutdown()


if __name__ == "__main__":
    main()
