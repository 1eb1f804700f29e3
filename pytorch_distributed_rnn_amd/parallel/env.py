"""Process discovery and process-group initialisation.

The reference initialises ``torch.distributed`` with the MPI backend under
``mpirun``/``horovodrun`` (reference: src/motion/trainer/ddp.py:18,
src/example/example_ddp.py:98, fabfile.py:217-231).  torch-ROCm has no MPI
backend, so:

* ranks are discovered from torchrun (``RANK``/``WORLD_SIZE``/``LOCAL_RANK``),
  Open MPI (``OMPI_COMM_WORLD_*``), PMI/MPICH (``PMI_RANK``/``PMI_SIZE``) or
  SLURM -- an ``mpirun -np 8 python main.py ... distributed`` launch still works;
* the backend is RCCL (torch name ``"nccl"``) on GPUs and gloo on the CPU;
  ``"mpi"``/``"rccl"`` are accepted as aliases;
* one process drives one GPU: ``LOCAL_RANK`` selects the device.
"""
from __future__ import annotations

import datetime
import logging
import os
import socket
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ProcessInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    launcher: str = "none"


def _int_env(*names: str) -> Optional[int]:
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            try:
                return int(v)
            except ValueError:
                pass
    return None


def discover() -> ProcessInfo:
    if _int_env("WORLD_SIZE") is not None and _int_env("RANK") is not None:
        launcher = "torchrun"
        rank, world = _int_env("RANK"), _int_env("WORLD_SIZE")
        local = _int_env("LOCAL_RANK")
        lws = _int_env("LOCAL_WORLD_SIZE")
    elif _int_env("OMPI_COMM_WORLD_SIZE") is not None:
        launcher = "mpirun"
        rank, world = _int_env("OMPI_COMM_WORLD_RANK"), _int_env("OMPI_COMM_WORLD_SIZE")
        local = _int_env("OMPI_COMM_WORLD_LOCAL_RANK")
        lws = _int_env("OMPI_COMM_WORLD_LOCAL_SIZE")
    elif _int_env("PMI_SIZE") is not None:
        launcher = "pmi"
        rank, world = _int_env("PMI_RANK"), _int_env("PMI_SIZE")
        local = _int_env("MPI_LOCALRANKID", "PMI_LOCAL_RANK")
        lws = _int_env("MPI_LOCALNRANKS", "PMI_LOCAL_SIZE")
    elif _int_env("SLURM_NTASKS") is not None and _int_env("SLURM_PROCID") is not None:
        launcher = "slurm"
        rank, world = _int_env("SLURM_PROCID"), _int_env("SLURM_NTASKS")
        local = _int_env("SLURM_LOCALID")
        lws = _int_env("SLURM_NTASKS_PER_NODE")
    else:
        return ProcessInfo()
    if local is None:
        n_dev = torch.cuda.device_count() or 1
        local = rank % n_dev
    return ProcessInfo(rank=rank, world_size=world, local_rank=local,
                       local_world_size=lws or world, launcher=launcher)


def normalize_backend(backend: Optional[str], use_gpu: bool) -> str:
    b = (backend or os.environ.get("PDRNN_BACKEND") or "").lower()
    if b in ("", "auto"):
        return "nccl" if use_gpu else "gloo"
    if b in ("rccl", "nccl"):
        return "nccl"
    if b == "mpi":
        if dist.is_mpi_available():
            return "mpi"
        logging.getLogger(__name__).warning(
            "MPI backend unavailable in this torch build; using %s", "nccl (RCCL)" if use_gpu else "gloo")
        return "nccl" if use_gpu else "gloo"
    if b == "gloo":
        return "gloo"
    raise ValueError(f"unknown backend {backend!r}")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def setup_device(info: Optional[ProcessInfo] = None) -> torch.device:
    info = info or discover()
    if torch.cuda.is_available():
        dev = info.local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        return torch.device("cuda", dev)
    return torch.device("cpu")


_TIMEOUT_S = 600.0


def collective_timeout_s() -> float:
    """Bound on any single collective: the process group's timeout
    (``PDRNN_DIST_TIMEOUT_S`` / ``init_distributed(timeout_s=...)``), used by
    gloo itself and by the native RCCL communicator's watchdog
    (``PDRNN_COMM_TIMEOUT_S`` overrides the latter)."""
    v = os.environ.get("PDRNN_COMM_TIMEOUT_S")
    return float(v) if v not in (None, "") else _TIMEOUT_S


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None,
                     use_gpu: Optional[bool] = None) -> ProcessInfo:
    """Initialise the default process group (idempotent) and the device.

    Every distributed wait is bounded by ``timeout_s`` (default 600 s or
    ``PDRNN_DIST_TIMEOUT_S``): gloo raises, torch's RCCL group and the native
    communicator's watchdog abort -- a dead peer fails the job instead of
    hanging it (the reference bounds its waits too: RPC timeout 60 s,
    src/motion/param_server/master.py:56; horovodrun --start-timeout 300,
    fabfile.py:227)."""
    global _TIMEOUT_S
    if timeout_s is None:
        timeout_s = float(os.environ.get("PDRNN_DIST_TIMEOUT_S", 600.0) or 600.0)
    info = discover()
    if use_gpu is None:
        use_gpu = torch.cuda.is_available() and os.environ.get("PDRNN_FORCE_CPU", "0") != "1"
    if dist.is_initialized():
        info.rank, info.world_size = dist.get_rank(), dist.get_world_size()
        return info
    if use_gpu:
        setup_device(info)
    be = normalize_backend(backend, use_gpu)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        if info.world_size > 1:
            os.environ["MASTER_PORT"] = "29500"
        else:
            os.environ["MASTER_PORT"] = str(_free_port())
    _TIMEOUT_S = float(timeout_s)
    kwargs = dict(backend=be, rank=info.rank, world_size=info.world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
    # no device_id: it makes torch create its RCCL communicator eagerly.  The
    # gradient path runs on the native communicator (parallel/comm.py, its
    # unique id exchanged through the TCPStore), so torch's stays lazy and is
    # only created if something issues a torch collective on the GPU group.
    try:
        dist.init_process_group(**kwargs)
    except TypeError:
        kwargs.pop("device_id", None)
        dist.init_process_group(**kwargs)
    return info


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if is_distributed() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_distributed() else 1


def barrier() -> None:
    # one rank has nobody to wait for: a world-1 barrier (an RCCL all-reduce
    # plus a host wait, ~0.3 ms on MI355X -- profiles/r6/bench_trace.md) is skipped
    if is_distributed() and dist.get_world_size() > 1:
        from .comm import native_world_comm
        c = native_world_comm()
        if c is not None:  # the gradient communicator (torch's RCCL comm stays unborn)
            c.barrier()
            return
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def shutdown() -> None:
    if is_distributed():
        try:
            barrier()
        finally:
            dist.destroy_process_group()
