"""Char-LM training entry point (BASELINE config 4).

    python -m pytorch_distributed_rnn_amd.lm_cli --hidden 1024 --layers 2 --seq-len 512 \\
        --batch-size 64 --max-steps 100 local
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m pytorch_distributed_rnn_amd.lm_cli ... distributed

Data: ``--text FILE`` (bytes) or a synthetic corpus (default).  ``--batch-size``
is global (strong scaling) unless ``--weak-scaling``.
"""
from __future__ import annotations

import argparse
import json
import logging
import sys

import torch

from .data.charlm import CharCorpus
from .models.charlm import CharLM
from .train.lm import LMTrainer

DTYPES = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="char-LM LSTM training")
    p.add_argument("--text", default=None)
    p.add_argument("--synthetic-tokens", type=int, default=4_000_000)
    p.add_argument("--vocab", type=int, default=256)
    p.add_argument("--embed", type=int, default=256)
    p.add_argument("--hidden", type=int, default=1024)
    p.add_argument("--layers", type=int, default=2)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--seq-len", type=int, default=512)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--weak-scaling", action="store_true")
    p.add_argument("--learning-rate", type=float, default=2e-3)
    p.add_argument("--grad-clip", type=float, default=1.0)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--dtype", choices=sorted(DTYPES), default="bf16")
    p.add_argument("--backend", default=None)
    p.add_argument("--bucket-mb", type=float, default=None)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--log", default="INFO")
    p.add_argument("--log-interval", type=int, default=50)
    p.add_argument("--device", default=None)
    p.add_argument("--history-file", default=None)
    p.add_argument("--checkpoint-directory", default=None, help="save <dir>/charlm-epoch<k>.pt after every epoch")
    p.add_argument("--resume", default=None, help="checkpoint to continue from")
    p.add_argument("--trace", action="store_true", help="roctx / torch.profiler ranges around step phases")
    p.add_argument("--profile", default=None, help="torch.profiler capture of the run into this directory")
    p.add_argument("mode", choices=("local", "distributed"))
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    logging.basicConfig(level=args.log, format="%(message)s")
    torch.manual_seed(args.seed)
    corpus = (CharCorpus.from_text(args.text) if args.text
              else CharCorpus.synthetic(args.synthetic_tokens, args.vocab, seed=args.seed))
    model = CharLM(corpus.vocab_size, args.embed, args.hidden, args.layers, args.dropout, DTYPES[args.dtype])
    device = torch.device(args.device) if args.device else None
    trainer = LMTrainer(model, corpus, args.batch_size, args.seq_len, args.learning_rate, device=device,
                        distributed=args.mode == "distributed", backend=args.backend,
                        grad_clip=args.grad_clip, log_interval=args.log_interval,
                        bucket_cap_mb=args.bucket_mb, weak_scaling=args.weak_scaling)
    start = trainer.resume(args.resume) if args.resume else 0
    history = []
    from .utils import tracing
    if args.trace:
        tracing.enable(True)
    with tracing.profile(args.profile, trainer.rank):
        for e in range(start, start + args.epochs):
            h = trainer.train_epoch(e, args.max_steps)
            history.append(h)
            if args.checkpoint_directory:
                from pathlib import Path
                trainer.save(Path(args.checkpoint_directory) / f"charlm-epoch{e}.pt", e, h["loss"])
    if trainer.rank == 0 and args.history_file:
        with open(args.history_file, "w") as f:
            json.dump(history, f)
    if args.mode == "distributed":
        from .parallel import env
        env.shutdown()
    return history


if __name__ == "__main__":
    sys.exit(0 if main() else 1)
