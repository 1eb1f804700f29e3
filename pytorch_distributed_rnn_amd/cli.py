"""Command-line interface: ``python src/motion/main.py [global flags] <command> [options]``.

Same global flags, defaults, ordering (global flags before the subcommand) and
subcommands as the reference CLI (reference: src/motion/main.py:15-43,
src/motion/trainer/__init__.py:10-60, src/motion/param_server/__init__.py:11-37),
so fabfile-style command lines keep working:

    main.py --batch-size 1440 --epochs 1 --seed 123456789 --no-validation local
    mpirun -np 8 python main.py ... distributed          (rank from OMPI_* env)
    torchrun --nproc-per-node 8 main.py ... horovod
    main.py ... parameter-server --world-size 3 --rank 0

Additions (all optional): ``--synthetic``, ``--cell {lstm,gru}``, ``--dtype
{fp32,bf16,fp16}``, ``--bidirectional``, ``--trace`` / ``--profile DIR``,
``--backend``, ``--bucket-mb``, ``--cuda-graph``, ``--kernel {hip,torch}``, ``--resume``,
``--checkpoint-every``, ``--log-interval``, ``--weak-scaling``,
``--fault-delay-ms`` / ``--fault-rank`` (network fault injection stand-in for
tc-netem), ``--history-file``.  Deviations from the reference, documented:
``--validation-fraction`` is honoured (the reference never passes it on),
``history.json`` is written by rank 0 only, ``--seed`` also seeds the
train/validation split.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys
from pathlib import Path
from typing import Optional

import torch

DEFAULT_ROOT = Path(os.environ.get("PDRNN_MOTION_DIR", Path(__file__).resolve().parent.parent / "src" / "motion"))


def build_parser(script_dir: Optional[Path] = None) -> argparse.ArgumentParser:
    root = Path(script_dir) if script_dir is not None else DEFAULT_ROOT
    p = argparse.ArgumentParser(description="SusML JKTM")
    p.add_argument("--checkpoint-directory", default=root / "models", type=Path)
    p.add_argument("--dataset-path", default=root / "data", type=Path)
    p.add_argument("--output-path", default=None, type=Path)
    p.add_argument("--stacked-layer", default=2, type=int)
    p.add_argument("--hidden-units", default=32, type=int)
    p.add_argument("--epochs", default=100, type=int)
    p.add_argument("--validation-fraction", default=0.1, type=float)
    p.add_argument("--batch-size", default=1440, type=int)
    p.add_argument("--learning-rate", default=0.0025, type=float)
    p.add_argument("--dropout", default=0.1, type=float,
                   help="accepted for compatibility; the reference model applies no dropout")
    p.add_argument("--log", default="INFO")
    p.add_argument("--num-threads", default=4, type=int)
    p.add_argument("--seed", default=None, type=int)
    p.add_argument("--no-validation", action="store_true")
    # ---- extensions
    p.add_argument("--synthetic", action="store_true",
                   help="train on generated UCI-HAR-shaped data (also used when no data is found)")
    p.add_argument("--synthetic-size", default=6912, type=int)
    p.add_argument("--cell", choices=("lstm", "gru"), default="lstm")
    p.add_argument("--dtype", choices=("fp32", "bf16", "fp16"), default="fp32",
                   help="bf16/fp16: 16-bit inputs and recurrent weights, fp32 accumulation / masters")
    p.add_argument("--bidirectional", action="store_true",
                   help="bidirectional recurrent stack (head reads out[:, -1, :])")
    p.add_argument("--trace", action="store_true",
                   help="roctx / torch.profiler ranges around forward, backward, all-reduce, optimizer")
    p.add_argument("--profile", default=None, type=Path,
                   help="torch.profiler capture of the training run into this directory")
    p.add_argument("--backend", default=None, help="nccl|rccl|gloo|mpi (default: RCCL on GPU, gloo on CPU)")
    p.add_argument("--bucket-mb", default=None, type=float)
    p.add_argument("--cuda-graph", action="store_true",
                   help="replay the synced fused step (fwd/BPTT + RCCL all-reduce + Adam) from a HIP graph")
    p.add_argument("--kernel", choices=("auto", "hip", "torch"), default="auto",
                   help="auto: HIP kernels, ATen fallback warns; hip: strict (uncovered shapes raise); "
                        "torch: ATen reference (tests)")
    p.add_argument("--device", default=None, help="cpu to force the CPU path")
    p.add_argument("--resume", default=None, type=Path)
    p.add_argument("--checkpoint-every", default=0, type=int)
    p.add_argument("--log-interval", default=0, type=int,
                   help="flush Train Batch lines every N steps (0: once per epoch)")
    p.add_argument("--weak-scaling", action="store_true",
                   help="--batch-size is per rank instead of global")
    p.add_argument("--fault-delay-ms", default=0.0, type=float,
                   help="inject a host delay before every gradient sync (netem stand-in)")
    p.add_argument("--fault-loss", default=0.0, type=float,
                   help="percent of gradient syncs hit by a retransmission stall (netem loss stand-in)")
    p.add_argument("--fault-retransmit-ms", default=200.0, type=float,
                   help="stall of one lost sync (Linux TCP's minimum retransmission timeout)")
    p.add_argument("--fault-rank", default=-1, type=int, help="only this rank is delayed / dropped (-1: all)")
    p.add_argument("--fault-drop-step", default=-1, type=int,
                   help="the --fault-rank rank(s) exit abruptly at this training step (failure-detection test)")
    p.add_argument("--history-file", default="history.json", type=Path)
    p.add_argument("--no-warmup", action="store_true",
                   help="charge kernel loading / workspace sizing to the first timed epoch")

    sub = p.add_subparsers(title="Available commands", metavar="command [options ...]")
    sub.required = True
    from .parallel import param_server
    param_server.add_sub_command(sub)
    for name in ("local", "distributed", "horovod"):
        sp = sub.add_parser(name)
        sp.set_defaults(func=lambda args, _n=name: train(args, _n))
    return p


def _load_datasets(args):
    from .data.motion import MotionDataset, synthetic_motion
    if not args.synthetic:
        try:
            return MotionDataset.load(args.dataset_path, output_path=args.output_path,
                                      validation_fraction=args.validation_fraction, seed=args.seed)
        except FileNotFoundError as e:
            logging.warning("%s -- falling back to synthetic data", e)
    return synthetic_motion(n_train=args.synthetic_size, seed=args.seed or 0)


def _trainer_class(name: str):
    from .train.distributed import DDPTrainer, HorovodTrainer
    from .train.trainer import Trainer
    return {"local": Trainer, "distributed": DDPTrainer, "horovod": HorovodTrainer}[name]


def _apply_common(args) -> None:
    if args.kernel == "torch":
        os.environ["PDRNN_KERNELS"] = "torch"
    elif args.kernel == "hip":
        os.environ["PDRNN_KERNELS"] = "hip-strict"
    if args.device == "cpu":
        os.environ["PDRNN_FORCE_CPU"] = "1"
    if args.fault_delay_ms > 0 or args.fault_drop_step >= 0 or args.fault_loss > 0:
        from .utils import faults
        kw = {"rank": args.fault_rank}
        if args.fault_delay_ms > 0:
            kw["delay_ms"] = args.fault_delay_ms
        if args.fault_loss > 0:
            kw["loss_prob"] = args.fault_loss / 100.0
            kw["retransmit_ms"] = args.fault_retransmit_ms
            kw["seed"] = args.seed or 0
        if args.fault_drop_step >= 0:
            kw["drop_step"] = args.fault_drop_step
        faults.configure(**kw)
    if args.trace:
        from .utils import tracing
        tracing.enable(True)


def train(args, name: str):
    logging.getLogger().setLevel(args.log)
    _apply_common(args)
    training_set, validation_set, test_set = _load_datasets(args)
    logging.info(f"Training set of size {len(training_set)}")
    if args.no_validation:
        validation_set = None
        test_set = None
    else:
        logging.info(f"Validation set of size {len(validation_set)}")
        logging.info(f"Test set of size {len(test_set)}")

    from .data.motion import MotionDataset
    from .models.motion import MotionModel
    model = MotionModel(input_dim=training_set.num_features, hidden_dim=args.hidden_units,
                        layer_dim=args.stacked_layer, output_dim=len(MotionDataset.LABELS),
                        cell=args.cell, bidirectional=args.bidirectional,
                        compute_dtype={"bf16": torch.bfloat16, "fp16": torch.float16}.get(args.dtype, torch.float32))
    trainer_cls = _trainer_class(name)
    kw = dict(model=model, training_set=training_set, validation_set=validation_set,
              test_set=test_set, batch_size=args.batch_size, learning_rate=args.learning_rate,
              checkpoint_dir=args.checkpoint_directory, log_interval=args.log_interval,
              checkpoint_every=args.checkpoint_every, cuda_graph=True if args.cuda_graph else None,
              warmup=not args.no_warmup)
    if args.device == "cpu":
        kw["device"] = torch.device("cpu")
    if name != "local":
        kw["backend"] = args.backend
        kw["weak_scaling"] = args.weak_scaling
        if name == "distributed":
            kw["bucket_cap_mb"] = args.bucket_mb
    trainer = trainer_cls(**kw)
    from .utils import faults
    if faults.active():  # flags above or PDRNN_FAULT_* environment
        faults.install(trainer)
    if args.resume is not None:
        nxt = trainer.resume(args.resume)
        logging.info(f"Resumed from {args.resume} (continuing at epoch {nxt})")
    logging.info(f"Training model for {args.epochs} epochs...")
    rank = getattr(trainer, "rank", 0)
    from .utils import tracing
    with tracing.profile(args.profile, rank):
        _, train_history, validation_history = trainer.train(epochs=args.epochs)
    if rank == 0:
        with open(args.history_file, "w") as f:
            json.dump({"train_history": train_history, "validation_history": validation_history}, f)
    if name != "local":
        from .parallel import env
        env.shutdown()
    return trainer


def main(argv=None, script_dir: Optional[Path] = None):
    parser = build_parser(script_dir)
    args = parser.parse_args(argv)
    if args.seed is not None:
        torch.manual_seed(args.seed)
    torch.set_num_threads(max(1, args.num_threads))
    return args.func(args)


if __name__ == "__main__":
    sys.dont_write_bytecode = True
    main()
