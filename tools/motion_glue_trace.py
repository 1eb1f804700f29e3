#!/usr/bin/env python
"""ATen glue dispatches (fills, copies, casts, adds, gathers) of one motion
training step at bench.py's configuration (e.g. --hidden 128), by op and
input shapes, with the Python frames that issued them when the profiler
records any.  Companion of tools/charlm_glue_trace.py.

    python tools/motion_glue_trace.py --hidden 128 > gpurun_out/motion_glue.txt
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from pytorch_distributed_rnn_amd.data.motion import MotionDataset, synthetic_motion  # noqa: E402
from pytorch_distributed_rnn_amd.models.motion import MotionModel  # noqa: E402
from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer  # noqa: E402

SKIP = ("aten::empty", "aten::view", "aten::as_strided", "aten::slice", "aten::select", "aten::t",
        "aten::transpose", "aten::reshape", "aten::_reshape_alias", "aten::unsqueeze", "aten::permute",
        "aten::empty_strided", "aten::detach", "aten::alias", "aten::expand", "aten::lift_fresh",
        "aten::record_stream", "aten::resolve_conj", "aten::resolve_neg", "aten::result_type")


def main():
    args = bench.parse(sys.argv[1:])
    torch.manual_seed(args.seed)
    env.init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    train_set, _, _ = synthetic_motion(n_train=max(args.epoch_sequences, args.global_batch), n_validation=1,
                                       n_test=1, seq_length=args.seq_len, seed=args.seed)
    model = MotionModel(train_set.num_features, args.hidden, args.layers, len(MotionDataset.LABELS), cell=args.cell,
                        compute_dtype=torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    tr = DDPTrainer(model=model, training_set=train_set, batch_size=args.global_batch, learning_rate=0.0025,
                    weak_scaling=True, device=dev)
    loader = tr.train_loader
    idx = list(loader.batch_indices())
    tr.model.train()
    tr.prepare()
    for b in idx[:3]:
        tr.train_batch(loader.make_batch(b))
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        tr.train_batch(loader.make_batch(idx[3 % len(idx)]))
        torch.cuda.synchronize()
    by = collections.Counter()
    for e in prof.events():
        if not e.name.startswith("aten::") or e.name in SKIP:
            continue
        if getattr(e, "device_time_total", 0.0) <= 0:
            continue
        frames = [f for f in (e.stack or []) if "pytorch_distributed_rnn_amd" in f]
        site = " <- ".join(f.split(ROOT + "/")[-1] for f in frames[:3]) or "-"
        by[(e.name, str(e.input_shapes)[:90], site)] += 1
    print("count  op  shapes  site")
    for k, n in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"{n:4d}  {k[0]}  {k[1]}  {k[2]}")
    print()
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=40, max_name_column_width=70))
    env.shutdown()


if __name__ == "__main__":
    main()
