"""Where the reference metric's 1-epoch `Training Duration` goes: cProfile of
the CLI's timed region (local trainer, synthetic data, 1 GPU).

    python bench/epoch_profile.py [--batch-size 1440]
"""
import argparse
import cProfile
import io
import logging
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=1440)
    a = ap.parse_args()
    logging.basicConfig(level=logging.INFO, stream=open(os.devnull, "w"))
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    torch.manual_seed(123456789)
    train, _, _ = synthetic_motion(n_train=6912, n_validation=1, n_test=1, seed=1)
    t = Trainer(MotionModel(9, 32, 2, 6), train, batch_size=a.batch_size, learning_rate=2.5e-3,
                device=torch.device("cuda"))
    pr = cProfile.Profile()
    pr.enable()
    t.train(1)  # first run: what a 1-epoch CLI run measures
    pr.disable()
    print(f"first run Training Duration: {t.last_duration * 1e3:.2f} ms", flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(20)
    print(s.getvalue())
    for _ in range(3):
        t.train(1)
        print(f"Training Duration: {t.last_duration * 1e3:.2f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    t.train(1)
    pr.disable()
    print(f"profiled run: {t.last_duration * 1e3:.2f} ms")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(28)
    print(s.getvalue())


if __name__ == "__main__":
    main()
