"""Native communicator factory.

``get_comm(group)`` returns the framework's C++ communicator for a process
group:

* GPU + RCCL group -> :class:`RcclComm` (csrc/runtime/comm.cpp): its own
  ncclComm created from a unique id that rank 0 draws and every rank receives
  through the already-initialised torch.distributed group (TCPStore
  rendezvous), its own high-priority HIP stream, and a watchdog thread that
  aborts it (and, by default, ends the process with status
  ``WATCHDOG_EXIT``) when a collective outlives ``collective_timeout_s()``;
* otherwise (gloo / CPU plumbing) -> the same interface over torch.distributed.

Communicators are cached per group.
"""
from __future__ import annotations

import atexit
import logging
import os
from typing import Dict, Optional

import torch
import torch.distributed as dist

from .. import _ext

_CACHE: Dict[int, object] = {}
_NATIVE = set()   # cache keys holding an RcclComm
_UID_SEQ: Dict[tuple, int] = {}  # communicators made so far per member-rank tuple


def _exchange_uid(mod, g, rank: int) -> bytes:
    """Rank 0's ncclUniqueId to every rank of ``g`` through the rendezvous
    TCPStore -- a key/value exchange, not a collective, so torch's own RCCL
    communicator for the group is never created just to bootstrap ours (one
    communicator per process on the gradient path instead of two).  Falls
    back to a broadcast when the default store is not reachable."""
    try:
        store = dist.distributed_c10d._get_default_store()
        ranks = tuple(sorted(dist.get_process_group_ranks(g)))
    except Exception:  # pragma: no cover - private-API drift
        store = None
    if store is None:
        uid = [mod.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=dist.get_global_rank(g, 0), group=g)
        return uid[0]
    # the sequence number counts communicators per member set, which only the
    # members themselves advance: ranks outside a subgroup never skew it
    seq = _UID_SEQ[ranks] = _UID_SEQ.get(ranks, 0) + 1
    key = "pdrnn/rccl_uid/%d/%s" % (seq, "-".join(str(r) for r in ranks))
    if rank == 0:
        uid = mod.rccl_unique_id()
        store.set(key, uid)
        return uid
    return bytes(store.get(key))  # blocks until rank 0 has published (store timeout)


def native_world_comm():
    """The native RCCL communicator of the default group, if one was made
    (barriers and the benchmark's timing reductions then use it instead of
    waking torch's own communicator)."""
    if not dist.is_initialized():
        return None
    key = id(dist.group.WORLD)
    return _CACHE.get(key) if key in _NATIVE else None


class _PyComm:
    """Pure-Python fallback with the Comm interface (no native extension)."""

    def __init__(self, group):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.native_avg = dist.get_backend(group) == "nccl"
        self.aborted = False
        self.tracked = 0
        self._works = []

    def all_reduce(self, t, op="sum"):
        o = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX,
             "min": dist.ReduceOp.MIN}[op]
        self._works.append(dist.all_reduce(t, op=o, group=self.group, async_op=True))

    def all_reduce_inline(self, t, op="sum"):
        self.all_reduce(t, op)
        self.wait()

    def track_current(self):
        pass  # gloo / torch process groups bound their own waits

    def broadcast(self, t, root):
        self._works.append(dist.broadcast(t, dist.get_global_rank(self.group, root), group=self.group,
                                          async_op=True))

    def all_gather(self, out, inp):
        self._works.append(dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True))

    def send(self, t, peer):
        self._works.append(dist.isend(t, dist.get_global_rank(self.group, peer), group=self.group))

    def recv(self, t, peer):
        self._works.append(dist.irecv(t, dist.get_global_rank(self.group, peer), group=self.group))

    def wait(self):
        for w in self._works:
            w.wait()
        self._works.clear()

    def barrier(self):
        self.wait()
        dist.barrier(group=self.group)


def get_comm(group=None, prefer_native: bool = True):
    if not dist.is_initialized():
        raise RuntimeError("init_distributed() first")
    g = group if group is not None else dist.group.WORLD
    key = id(g)
    if key in _CACHE:
        return _CACHE[key]
    backend = dist.get_backend(g)
    mod = _ext.extension()
    use_rccl = (prefer_native and backend == "nccl" and torch.cuda.is_available() and mod is not None
                and os.environ.get("PDRNN_COMM", "rccl") == "rccl")
    if use_rccl:
        rank = dist.get_rank(g)
        world = dist.get_world_size(g)
        uid = _exchange_uid(mod, g, rank)
        from .env import collective_timeout_s
        comm = mod.make_rccl_comm(uid, rank, world, torch.cuda.current_device(), True,
                                  collective_timeout_s())
        _NATIVE.add(key)
    elif mod is not None:
        comm = mod.make_pg_comm(g)
    else:
        comm = _PyComm(g)
    _CACHE[key] = comm
    if mod is not None and torch.cuda.is_available() and dist.get_world_size(g) > 1 \
            and hasattr(mod, "set_persist_verify"):
        # collectives now run beside the compute stream: a persistent
        # recurrence can lose co-residency to them, so every persistent launch
        # is verified (host-synchronised) and a timed-out layer re-run on the
        # per-step kernels before anything uses its result (mode 1, bindings.cpp
        # large_persist).  The LM trainer, which also carries the skip word to
        # Adam and re-runs skipped steps (train/lm.py settle), upgrades its
        # process to the sync-free per-step mode 2 (use_step_verification).
        if os.environ.get("PDRNN_LSTM_PERSIST_VERIFY") is None and mod.persist_verify_mode() != 2:
            mod.set_persist_verify(1)
    return comm


def use_step_verification() -> bool:
    """Switch this multi-rank GPU process to per-step persistent-path
    verification (mode 2: no host sync per launch; a timed-out step's
    optimizer update is skipped on the device and the step re-run).  Only a
    trainer that passes the sticky flag to its optimizer as the skip word and
    re-runs skipped steps may call this (``LMTrainer``); every other trainer
    keeps mode 1, where a timed-out layer is re-run inside its own launch
    sequence before the gradient is used.  Returns True when mode 2 is on."""
    mod = _ext.extension()
    if mod is None or not torch.cuda.is_available() or not hasattr(mod, "set_persist_verify"):
        return False
    if os.environ.get("PDRNN_LSTM_PERSIST_VERIFY") is not None:
        return mod.persist_verify_mode() == 2
    mod.set_persist_verify(2)
    return True


def close_comms() -> None:
    """Release every cached communicator now (native: watchdog joined,
    pending collectives drained with a deadline, RCCL communicator destroyed
    or aborted).  Registered with atexit: the interpreter otherwise may never
    drop the last reference, leaving a watchdog thread polling the HIP runtime
    while the process's exit handlers tear it down (seen as a SIGSEGV in
    exit() under rocprofv3)."""
    for c in list(_CACHE.values()):
        close = getattr(c, "close", None)
        if close is not None:
            try:
                close()
            except Exception as e:  # teardown must not mask the run's own outcome
                logging.warning(f"communicator close failed: {e}")
    reset_comms()


atexit.register(close_comms)


def reset_comms() -> None:
    _CACHE.clear()
    _NATIVE.clear()
