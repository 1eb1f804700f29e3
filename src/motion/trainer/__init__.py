"""Trainer registry compatible with reference ``src/motion/trainer/__init__.py``."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _bootstrap  # noqa: E402,F401

from pytorch_distributed_rnn_amd.cli import train as _train  # noqa: E402
from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer, HorovodTrainer  # noqa: E402,F401
from pytorch_distributed_rnn_amd.train.trainer import Trainer  # noqa: E402,F401

TRAINERS = {"local": Trainer, "distributed": DDPTrainer, "horovod": HorovodTrainer}


def add_sub_commands(sub_parser):
    for name in TRAINERS:
        p = sub_parser.add_parser(name)
        p.set_defaults(func=lambda args, _n=name: _train(args, _n))


def train(args, trainer):
    name = {v: k for k, v in TRAINERS.items()}.get(trainer, "local")
    return _train(args, name)
