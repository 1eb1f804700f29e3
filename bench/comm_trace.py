#!/usr/bin/env python
"""Trace target: the autograd DDP path with hook-driven bucket all-reduces on
the native communicator's comm stream (PDRNN_FORCE_COLLECTIVE=1 keeps the
one-rank collective real).  Run under
``rocprofv3 --kernel-trace --output-format csv -- python bench/comm_trace.py``
and summarise with ``tools/prof_streams.py``: the RCCL all-reduce kernels must
sit on a different stream (queue) from the LSTM/xent kernels and start while
the backward of the lower layers is still running."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("PDRNN_FORCE_COLLECTIVE", "1")

import torch  # noqa: E402

from pytorch_distributed_rnn_amd.models.charlm import CharLM  # noqa: E402,F401
from pytorch_distributed_rnn_amd.models.motion import MotionModel  # noqa: E402
from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel  # noqa: E402


def main():
    env.init_distributed("nccl")
    torch.manual_seed(0)
    m = MotionModel(9, 32, 2, 6).cuda()
    ddp = DistributedDataParallel(m, bucket_cap_mb=0.02, first_bucket_cap_mb=0.02)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    x = torch.randn(1440, 128, 9, device="cuda")
    y = torch.randint(0, 6, (1440,), device="cuda")
    for _ in range(6):
        opt.zero_grad(set_to_none=False)
        torch.nn.functional.cross_entropy(ddp(x), y).backward()
        opt.step()
    torch.cuda.synchronize()
    print(f"buckets={len(ddp.bucket_layout())} tracked_collectives={ddp.comm.tracked}", flush=True)
    env.shutdown()


if __name__ == "__main__":
    main()
