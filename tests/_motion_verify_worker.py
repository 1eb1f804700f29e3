"""Worker of tests/test_gpu_multirank.py::test_two_rank_motion_persist_verification:
one rank of a 2-rank motion DDP job (gloo, shared GPU) at --hidden-units 256,
whose fp32 backward recurrence is the grid-synced persistent kernel.  With
PDRNN_TEST_INJECT_RANK=r, rank r flags its first persistent launch as timed
out: in the motion trainers' verification mode (1, per launch) that layer is
re-run on the per-step kernels before its gradient is reduced, so the run
must end where a PDRNN_LSTM_PERSIST=0 run ends.  Writes one JSON file."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pytorch_distributed_rnn_amd import _ext  # noqa: E402
from pytorch_distributed_rnn_amd.models.motion import MotionModel  # noqa: E402
from pytorch_distributed_rnn_amd.ops.adam import FusedAdam  # noqa: E402
from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel  # noqa: E402
from pytorch_distributed_rnn_amd.utils.flat import flatten_module  # noqa: E402


def main():
    env.init_distributed("gloo")
    rank, world = env.get_rank(), env.get_world_size()
    torch.manual_seed(0)
    model = MotionModel(9, 256, 2, 6).cuda()
    flatten_module(model)
    ddp = DistributedDataParallel(model)
    opt = FusedAdam(model.parameters(), lr=2.5e-3)
    mod = _ext.require()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(3, 2 * 48, 32, 9, generator=g)
    y = torch.randint(0, 6, (3, 2 * 48), generator=g)
    if int(os.environ.get("PDRNN_TEST_INJECT_RANK", "-1")) == rank:
        mod.persist_inject_timeouts(1)
    losses = []
    for s in range(3):
        xb = x[s, rank::world].cuda()
        yb = y[s, rank::world].cuda()
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(ddp(xb), yb)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().double().reshape(-1) for p in model.parameters()])
    rec = json.dumps({"rank": rank, "verify": mod.persist_verify_mode(), "fallbacks": mod.persist_fallbacks(),
                      "checksum": float(flat.sum()), "abs": float(flat.abs().sum()), "losses": losses})
    with open(f"mverify_rank{rank}.json", "w") as f:
        f.write(rec + "\n")
    env.shutdown()


if __name__ == "__main__":
    main()
