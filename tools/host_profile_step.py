"""Host-side cost of one epoch's enqueue through Trainer.train_batches (cProfile),
for the local / DDP / Horovod trainers at world 1 -- where the CLI's epoch loses
time before the GPU is fed.  python tools/host_profile_step.py TRAINER"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer, HorovodTrainer
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    which = sys.argv[1] if len(sys.argv) > 1 else "local"
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29611")
    torch.manual_seed(0)
    train, _, _ = synthetic_motion(n_train=6912, n_validation=1, n_test=1, seed=0)
    model = MotionModel(9, 32, 2, 6)
    cls = {"local": Trainer, "distributed": DDPTrainer, "horovod": HorovodTrainer}[which]
    kw = {} if which != "local" else {"device": torch.device("cuda")}
    t = cls(model=model, training_set=train, batch_size=1440, learning_rate=2.5e-3, **kw)
    t.prepare()
    loader = t.train_loader
    for e in range(3):
        t.sampler.set_epoch(e)
        t.train_batches(list(loader))
    torch.cuda.synchronize()
    t.sampler.set_epoch(10)
    batches = list(loader)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    t.train_batches(batches)
    pr.disable()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"[{which}] enqueue {1e6 * (t1 - t0):.0f} us for {len(batches)} steps", flush=True)
    pstats.Stats(pr).sort_stats("cumulative").print_stats(18)


if __name__ == "__main__":
    main()
