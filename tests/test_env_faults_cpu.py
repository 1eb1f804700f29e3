"""Rank discovery and fault-injection configuration."""
import time

import pytest

from pytorch_distributed_rnn_amd.parallel import env
from pytorch_distributed_rnn_amd.utils import faults


def test_discover_torchrun(monkeypatch):
    for k in list(__import__("os").environ):
        if k.startswith(("OMPI_", "PMI_", "SLURM_")):
            monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_RANK", "3")
    info = env.discover()
    assert (info.rank, info.world_size, info.local_rank, info.launcher) == (3, 8, 3, "torchrun")


def test_discover_openmpi(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "1")
    monkeypatch.setenv("OMPI_COMM_WORLD_SIZE", "4")
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_RANK", "1")
    info = env.discover()
    assert (info.rank, info.world_size, info.local_rank, info.launcher) == (1, 4, 1, "mpirun")


@pytest.mark.parametrize("name,gpu,expect", [("mpi", False, "gloo"), ("rccl", True, "nccl"),
                                             (None, False, "gloo"), (None, True, "nccl")])
def test_backend_aliases(name, gpu, expect):
    assert env.normalize_backend(name, gpu) == expect


class _FakeTrainer:
    rank = 0

    def __init__(self):
        self.calls = 0

    def train_batch(self, batch):
        self.calls += 1
        return batch


def test_fault_delay_is_injected():
    old = faults.config().__dict__.copy()
    try:
        faults.configure(delay_ms=30.0, rank=-1, drop_step=-1, loss_prob=0.0)
        t = _FakeTrainer()
        faults.install(t)
        t0 = time.perf_counter()
        assert t.train_batch(5) == 5
        assert time.perf_counter() - t0 >= 0.025
        assert t.calls == 1
    finally:
        faults.configure(**old)
