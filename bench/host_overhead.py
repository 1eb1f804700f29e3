#!/usr/bin/env python
"""Host-enqueue vs device time of the motion DDP training step.

Runs ``Trainer.train_batch`` K times WITHOUT synchronising (host enqueue wall
time per step), then synchronises (device-bound wall time per step).  If the
two are close the step is host-bound and the GPU idles between launches.

    python bench/host_overhead.py --global-batch 180
    PDRNN_FORCE_GRAD_SYNC=1 python bench/host_overhead.py --global-batch 180
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--global-batch", type=int, default=180)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--cprofile", action="store_true", help="print the host-side hot spots (cProfile, tottime)")
    args = ap.parse_args()
    import torch

    from pytorch_distributed_rnn_amd.data.motion import MotionDataset, synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.parallel import env
    from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer

    torch.manual_seed(0)
    env.init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    train_set, _, _ = synthetic_motion(n_train=6912, n_validation=1, n_test=1, seq_length=128, seed=1)
    model = MotionModel(9, 32, 2, len(MotionDataset.LABELS))
    tr = DDPTrainer(model=model, training_set=train_set, batch_size=args.global_batch, learning_rate=0.0025,
                    device=dev)
    loader = tr.train_loader
    idx = [b for b in loader.batch_indices() if b.shape[0] == loader.batch_size]
    batches = [idx[i % len(idx)] for i in range(args.steps)]
    for b in batches[:20]:
        tr.train_batch(loader.make_batch(b))
    torch.cuda.synchronize()
    prof = None
    if args.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for b in batches:
        tr.train_batch(loader.make_batch(b))
    t1 = time.perf_counter()
    if prof is not None:
        prof.disable()
        import pstats
        pstats.Stats(prof).sort_stats("tottime").print_stats(25)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out = {"global_batch": args.global_batch,
           "force_grad_sync": os.environ.get("PDRNN_FORCE_GRAD_SYNC", "0"),
           "host_enqueue_us_per_step": round((t1 - t0) / args.steps * 1e6, 2),
           "wall_us_per_step": round((t2 - t0) / args.steps * 1e6, 2)}
    print(json.dumps(out), flush=True)
    env.shutdown()


if __name__ == "__main__":
    main()
