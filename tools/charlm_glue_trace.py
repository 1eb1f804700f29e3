#!/usr/bin/env python
"""Which Python lines issue the char-LM step's non-HIP dispatches (fills,
D2D copies, ATen elementwise kernels)?  Profiles one `LMTrainer.train_step`
of the config-4 shape (bench/lm_bench.py --config charlm) with torch.profiler
(CPU + device activity, Python stacks) after two warmup steps and prints the
ATen ops that launch device work, grouped by their innermost repo frames.

    python tools/charlm_glue_trace.py > gpurun_out/charlm_glue.txt
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from pytorch_distributed_rnn_amd.data.charlm import CharCorpus  # noqa: E402
from pytorch_distributed_rnn_amd.models.charlm import CharLM  # noqa: E402
from pytorch_distributed_rnn_amd.parallel import env  # noqa: E402
from pytorch_distributed_rnn_amd.train.lm import LMTrainer  # noqa: E402

GLUE = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add_", "aten::add", "aten::to", "aten::_to_copy",
        "aten::zeros", "aten::clone", "aten::mul", "aten::mul_", "aten::cat", "aten::stack", "aten::sub",
        "aten::div", "aten::index_select", "aten::sum", "aten::contiguous", "aten::masked_fill_", "aten::where")


def main():
    info = env.init_distributed()
    dev = env.setup_device(info)
    torch.manual_seed(0)
    B, T, H, steps = 128, 512, 1024, 4
    corpus = CharCorpus.synthetic(B * T * (steps + 2) + 1, 256, seed=0)
    tr = LMTrainer(CharLM(256, 256, H, 2, 0.0, torch.bfloat16), corpus, B, T, 2e-3, device=dev,
                   distributed=False, weak_scaling=True)
    segs = list(CharCorpus.segments(tr.streams, T, steps))
    tr.inner.reset_hidden_state()
    for i in range(2):
        tr.train_step(*segs[i])
    tr.settle()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        tr.train_step(*segs[2])
        tr.settle()
        torch.cuda.synchronize()
    evs = prof.events()
    by_site = collections.Counter()
    dev_us = collections.Counter()
    for e in evs:
        if e.name not in GLUE:
            continue
        kids = [k for k in e.cpu_children]
        stack = [f for f in (e.stack or []) if "pytorch_distributed_rnn_amd" in f or "tools/" in f]
        site = " <- ".join(s.split(ROOT + "/")[-1] for s in stack[:3]) or "(no repo frame)"
        by_site[(e.name, site, str(e.input_shapes)[:80])] += 1
        dev_us[(e.name, site, str(e.input_shapes)[:80])] += getattr(e, "device_time_total", 0.0)
        del kids
    print("count  device_us  op  site  shapes")
    for k, n in sorted(by_site.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d} {dev_us[k]:9.1f}  {k[0]}  {k[1]}  {k[2]}")
    print()
    print(prof.key_averages().table(sort_by="device_time_total", row_limit=45, max_name_column_width=70))
    env.shutdown()


if __name__ == "__main__":
    main()
