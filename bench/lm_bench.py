#!/usr/bin/env python
"""Secondary benchmarks (BASELINE.json configs 4 and 5), same JSON-line contract
as bench.py (rank 0 prints one line; value = whole-job tokens/s; timed region
bracketed by barrier + device sync; max over ranks).

  charlm : 2-layer LSTM char-LM, hidden 1024, seq_len 512, bf16 compute, DDP
           (weak scaling: --batch per GPU), TBPTT state carried across steps.
  bilstm : stacked bidirectional LSTM, hidden 4096, fp16 compute, per-timestep
           32-way classification head, batch sized for HBM (--batch per GPU).

    python bench/lm_bench.py --config charlm --steps 10 --warmup 2
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        bench/lm_bench.py --config charlm --gpus 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pytorch_distributed_rnn_amd import _ext  # noqa: E402
from pytorch_distributed_rnn_amd.data.charlm import CharCorpus  # noqa: E402
from pytorch_distributed_rnn_amd.models.charlm import BiLSTMEncoder, CharLM  # noqa: E402
from pytorch_distributed_rnn_amd.ops.adam import FusedAdam  # noqa: E402
from pytorch_distributed_rnn_amd.ops.xent import cross_entropy  # noqa: E402
from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel, format_bucket_layout  # noqa: E402
from pytorch_distributed_rnn_amd.train.lm import LMTrainer  # noqa: E402
from pytorch_distributed_rnn_amd.utils.flat import flatten_module  # noqa: E402
from pytorch_distributed_rnn_amd.utils.memory import device_peak_mib  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("charlm", "bilstm"), default="charlm")
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", 1)))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch")
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--hidden", type=int, default=None)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--input-dim", type=int, default=1024, help="bilstm input features")
    ap.add_argument("--ddp", action="store_true",
                    help="bucketed DDP reducer even at one rank (overlap traces with "
                         "PDRNN_FORCE_COLLECTIVE=1)")
    ap.add_argument("--bucket-mb", type=float, default=None)
    return ap.parse_args(argv)


def main(argv=None):
    a = parse(argv)
    info = env.init_distributed()
    world, rank = env.get_world_size(), env.get_rank()
    dev = env.setup_device(info) if torch.cuda.is_available() else torch.device("cpu")
    torch.manual_seed(0)
    if a.config == "charlm":
        B, T, H = a.batch or 128, a.seq_len or 512, a.hidden or 1024
        corpus = CharCorpus.synthetic(B * world * T * (a.steps + a.warmup + 2) + 1, 256, seed=0)
        tr = LMTrainer(CharLM(256, 256, H, a.layers, 0.0, torch.bfloat16), corpus, B, T, 2e-3, device=dev,
                       distributed=world > 1 or a.ddp, weak_scaling=True, force_ddp=a.ddp,
                       bucket_cap_mb=a.bucket_mb)
        segs = list(CharCorpus.segments(tr.streams, T, a.steps + a.warmup))
        tr.inner.reset_hidden_state()
        step = lambda i: tr.train_step(*segs[i])  # noqa: E731
        dtype, model_name = "bf16", f"char-LM LSTM {a.layers}x{H} (vocab 256, embed 256)"
        metric = "tokens/sec (whole node) char-LM 2-layer LSTM h1024 seq512 bf16 DDP"
    else:
        # batch sized for HBM: B=4096 x T=64 holds ~115 GB of activations on one
        # 288 GB MI355X (B sweep 256/512/1024/2048/4096: 239k/265k/307k/313k/323k tok/s)
        B, T, H = a.batch or 4096, a.seq_len or 64, a.hidden or 4096
        model = BiLSTMEncoder(a.input_dim, H, a.layers, 32, torch.float16).to(dev)
        flatten_module(model)
        net = DistributedDataParallel(model, bucket_cap_mb=a.bucket_mb) if world > 1 or a.ddp else model
        if isinstance(net, DistributedDataParallel) and rank == 0:
            print("bucket layout (launch order): " + format_bucket_layout(net.bucket_layout()), file=sys.stderr,
                  flush=True)
        opt = FusedAdam(model.parameters(), lr=1e-4)
        g = torch.Generator(device=dev).manual_seed(rank)
        xs = torch.randn(T, B, a.input_dim, device=dev, generator=g).half()
        ys = torch.randint(0, 32, (T * B,), device=dev, generator=g)

        def step(i):
            opt.zero_grad()
            loss = cross_entropy(net(xs).reshape(T * B, 32), ys)
            loss.backward()
            opt.step()
            return loss.detach()
        dtype, model_name = "fp16", f"stacked bi-LSTM {a.layers}x{H} (input {a.input_dim}, 32 classes)"
        metric = "tokens/sec (whole node) stacked bidirectional LSTM h4096 fp16"
    for i in range(a.warmup):
        step(i)
    if a.config == "charlm":
        tr.settle()
    env.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = step(a.warmup + i if a.config == "charlm" else i)
    if a.config == "charlm":
        tr.settle()  # deferred verification: any re-run step counts in the timed region
    if dev.type == "cuda":
        torch.cuda.synchronize()
    env.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    toks = B * T * world * a.steps
    if rank == 0:
        print(json.dumps({
            "metric": metric, "value": round(toks / el, 1), "unit": "tokens/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
            "data": "synthetic", "config": {"model": model_name, "global_batch": B * world, "seq_len": T,
                                            "parallelism": f"dp{world}"},
            "final_loss": round(float(loss), 5), "device_peak_mib": round(device_peak_mib(dev), 1),
            "ddp_reducer": isinstance(tr.model if a.config == "charlm" else net, DistributedDataParallel),
            "force_collective": os.environ.get("PDRNN_FORCE_COLLECTIVE", "0") == "1",
            **_ext.persist_stats()}), flush=True)
    env.shutdown()


if __name__ == "__main__":
    main()
