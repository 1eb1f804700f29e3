#!/usr/bin/env python
"""Per-step wall time of the flagship step (diagnostic for warm-up effects):
times every one of --steps steps with a host timer around a device sync."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--global-batch", type=int, default=1440)
    a = ap.parse_args()
    import torch
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.parallel import env
    from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer
    torch.manual_seed(0)
    env.init_distributed()
    train, _, _ = synthetic_motion(n_train=6912, n_validation=1, n_test=1, seed=0)
    t = DDPTrainer(model=MotionModel(9, 32, 2, 6), training_set=train, batch_size=a.global_batch,
                   learning_rate=0.0025, device=torch.device("cuda", 0))
    loader = t.train_loader
    idx = [b for b in loader.batch_indices() if b.shape[0] == loader.batch_size]
    times = []
    for s in range(a.steps):
        b = loader.make_batch(idx[s % len(idx)])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t.train_batch(b)
        torch.cuda.synchronize()
        times.append((time.perf_counter() - t0) * 1e3)
    print(" ".join(f"{x:.3f}" for x in times))
    env.shutdown()


if __name__ == "__main__":
    main()
