"""pytorch_distributed_rnn_amd -- MI355X-native distributed RNN training.

A from-scratch re-design of jkhlr/pytorch-distributed-rnn for AMD Instinct
MI355X (gfx950): fused HIP kernels for the recurrent hot path, flat parameter
storage, a native RCCL communicator and bucketed reducer over xGMI, and the
reference's trainer / CLI / log / checkpoint surfaces.
"""
__version__ = "0.1.0"

from . import _ext  # noqa: F401
