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


def test_dropped_rank_fails_survivors_fast(tmp_path):
    """A rank that dies mid-epoch must make every survivor exit non-zero within
    the collective timeout instead of hanging (the reference bounds its waits:
    RPC timeout 60 s, src/motion/param_server/master.py:56; horovodrun
    --start-timeout 300, fabfile.py:227).  Ranks are started directly (no
    torchrun agent that would kill the survivors for us)."""
    import os
    import subprocess
    import sys

    from _mp import ROOT, cpu_env, free_port

    world, timeout_s = 3, 45  # generous: under a loaded test runner a rank can take >20 s to start
    main = os.path.join(ROOT, "src", "motion", "main.py")
    port = str(free_port())
    procs = []
    t0 = time.perf_counter()
    for r in range(world):
        e = cpu_env({"RANK": str(r), "WORLD_SIZE": str(world), "LOCAL_RANK": str(r), "MASTER_PORT": port,
                     "PDRNN_DIST_TIMEOUT_S": str(timeout_s)})
        cmd = [sys.executable, main, "--seed", "1", "--epochs", "50", "--batch-size", "96", "--no-validation",
               "--synthetic", "--synthetic-size", "384", "--device", "cpu", "--hidden-units", "8",
               "--fault-rank", "1", "--fault-drop-step", "3", "distributed"]
        procs.append(subprocess.Popen(cmd, cwd=str(tmp_path), env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    codes, outs = [], []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout_s * 4 + 60)
            codes.append(p.returncode)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    elapsed = time.perf_counter() - t0
    assert codes[1] == 17, (codes, outs[1][-2000:])  # the injected drop
    for r in (0, 2):
        assert codes[r] != 0, f"survivor rank {r} exited 0:\n{outs[r][-2000:]}"
    assert elapsed < timeout_s * 4 + 60, elapsed


def test_extension_loads_when_built(monkeypatch):
    """The in-tree extension imports through the loader (both the default
    module path and the PDRNN_EXT_SO alternative-build path): a loader error
    would otherwise silently put every CPU host-runtime test on the Python
    twins and every GPU run on the loud 'failed to load' path."""
    import glob
    import os

    from pytorch_distributed_rnn_amd import _ext
    pkg = os.path.dirname(_ext.__file__)
    built = glob.glob(os.path.join(pkg, "_C*.so"))
    if not built:
        pytest.skip("extension not built in this tree")
    for so in (None, built[0]):
        if so:
            monkeypatch.setenv("PDRNN_EXT_SO", so)
        else:
            monkeypatch.delenv("PDRNN_EXT_SO", raising=False)
        monkeypatch.setattr(_ext, "_TRIED", False)
        monkeypatch.setattr(_ext, "_C", None)
        assert _ext.extension() is not None, repr(_ext._IMPORT_ERROR)
        assert hasattr(_ext.extension(), "GradReducer")
