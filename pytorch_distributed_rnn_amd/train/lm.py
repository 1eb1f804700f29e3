"""Language-model trainer: truncated BPTT over token streams, local or
data-parallel (the framework's DDP: bucketed RCCL all-reduce overlapped with
the BPTT backward), fused Adam on the flat parameter buffer, flat-buffer
gradient clipping without a host sync.

The hidden state is carried across consecutive segments of a stream and
reset at every epoch start -- the working version of the reference's dead
``_reset_hidden_state`` hook (reference: src/motion/trainer/base.py:161-162,
src/motion/trainer/ddp.py:35-36).
"""
from __future__ import annotations

import logging
import math
import time
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor, nn

from .. import _ext
from ..data.charlm import CharCorpus
from .checkpoint import adapt_state_dict_keys, save_checkpoint
from ..ops.adam import FusedAdam
from ..ops.xent import cross_entropy
from ..parallel import env
from ..parallel.ddp import DistributedDataParallel
from ..utils.flat import flatten_module
from ..utils.memory import device_peak_mib
from ..utils.tracing import trace_range


class LMTrainer:
    def __init__(self, model: nn.Module, corpus: CharCorpus, global_batch: int, seq_len: int,
                 learning_rate: float = 2e-3, device: Optional[torch.device] = None,
                 distributed: bool = False, backend: Optional[str] = None, grad_clip: float = 1.0,
                 log_interval: int = 50, bucket_cap_mb: Optional[float] = None,
                 weak_scaling: bool = False, force_ddp: bool = False):
        self.rank, self.world = 0, 1
        if distributed:
            info = env.init_distributed(backend)
            self.rank, self.world = env.get_rank(), env.get_world_size()
            if device is None:
                device = (env.setup_device(info) if torch.distributed.get_backend() == "nccl"
                          else torch.device("cpu"))
        if device is None:
            device = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        self.inner = model.to(device)
        flatten_module(self.inner)
        # force_ddp: keep the bucketed reducer at world size 1 (with
        # PDRNN_FORCE_COLLECTIVE=1 every bucket is a real RCCL collective on
        # the comm stream -- the overlap trace of profiles/r2_charlm_overlap.md)
        self.model = (DistributedDataParallel(self.inner, bucket_cap_mb=bucket_cap_mb)
                      if distributed and (self.world > 1 or force_ddp) else self.inner)
        self.flat = next(iter(self.inner._pdrnn_flat.values()))
        self.optimizer = FusedAdam(self.inner.parameters(), lr=learning_rate)
        if distributed and self.world > 1 and device.type == "cuda":
            # this trainer carries the sticky persistent-timeout flag to Adam as
            # its skip word and re-runs skipped steps (settle): the sync-free
            # per-step verification mode is safe here, not in the motion trainers
            from ..parallel.comm import use_step_verification
            use_step_verification()
        self.seq_len = seq_len
        self.grad_clip = grad_clip
        self.log_interval = log_interval
        gb = global_batch * self.world if weak_scaling else global_batch
        self.global_batch = gb
        self.streams = corpus.streams(gb, self.rank, self.world).to(device)
        self.vocab = corpus.vocab_size
        self._pending: List[dict] = []  # steps not yet verified (deferred verification)
        self.direct_grads = True  # one process: gradients written into the flat views (see _fwd_bwd)

    def _clip(self) -> None:
        if self.grad_clip and self.grad_clip > 0:
            g = self.flat.grad
            mod = _ext.extension() if g.is_cuda else None
            if mod is not None and hasattr(mod, "clip_flat") and g.dtype == torch.float32 and g.is_contiguous():
                mod.clip_flat(g, float(self.grad_clip), 1e-6)  # deterministic, no host sync (kernels/adam.hip)
                return
            norm = torch.linalg.vector_norm(g)
            g.mul_(torch.clamp(self.grad_clip / (norm + 1e-6), max=1.0))

    @staticmethod
    def _time_major(inp: Tensor, tgt: Tensor) -> Tuple[Tensor, Tensor]:
        """Sequence-major contiguous [T, B] copies of the [B, T] input and
        target windows, which the embedding gather and the loss read.  For the
        overlapping windows of one stream (target = input shifted by one,
        data/charlm.py segments) that is ONE copy of the [B, T + 1] window
        instead of a transpose copy per consumer."""
        B, T = inp.shape
        if (tgt.shape == inp.shape and tgt.dtype == inp.dtype and tgt.device == inp.device and
                tgt.stride() == inp.stride() and inp.untyped_storage().data_ptr() == tgt.untyped_storage().data_ptr()
                and tgt.storage_offset() == inp.storage_offset() + inp.stride(1)):
            win = inp.as_strided((B, T + 1), inp.stride(), inp.storage_offset())
            both = win.t().contiguous()  # [T + 1, B]
            return both[:T], both[1:]
        return inp.t().contiguous(), tgt.t().contiguous()

    def _fwd_bwd(self, inp: Tensor, tgt: Tensor) -> Tensor:
        from ..ops import gradsink
        inp_tb, tgt_tb = self._time_major(inp, tgt)
        self.optimizer.zero_grad()
        # one process: the in-tree Functions add their weight gradients into
        # the flat gradient views themselves (ops/gradsink.py: no per-parameter
        # autograd add launches); the DDP reducer keeps the autograd path
        with gradsink.direct_grads(self.direct_grads and self.model is self.inner and self.device.type == "cuda"):
            with trace_range("pdrnn.forward"):
                logits = self.model(inp_tb.t(), carry=True)                        # [T, B, V]
                loss = cross_entropy(logits.reshape(-1, logits.shape[-1]), tgt_tb.reshape(-1))
            with trace_range("pdrnn.backward"):
                loss.backward()
        return loss

    # ---------------------------------------------- persistent-path verification
    def _deferred_verify(self) -> bool:
        """Per-step verification of the persistent recurrence (multi-rank jobs:
        bindings.cpp large_persist, persist_verify_mode() == 2), without a host
        synchronisation in the step: the device's sticky timeout flag is
        all-reduced (MAX) across ranks on the stream and handed to the Adam
        launch as its skip word, so a step whose persistent launch lost
        co-residency on ANY rank leaves the parameters untouched everywhere;
        the host reads the flag's pinned copy one step later (:meth:`settle`)
        and re-runs the skipped steps on the per-step kernels."""
        if self.device.type != "cuda":
            return False
        mod = _ext.extension()
        return mod is not None and hasattr(mod, "persist_sticky_flag") and mod.persist_verify_mode() == 2

    def _step_flag(self):
        mod = _ext.extension()
        flag = mod.persist_sticky_flag()
        if self.world > 1:
            from ..parallel.comm import get_comm
            comm = get_comm()
            comm.all_reduce(flag, "max")  # in place: every rank's sticky flag agrees
            comm.wait()                   # stream-ordered (no host wait)
        host = torch.empty(1, dtype=torch.int32, pin_memory=True)
        host.copy_(flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return flag, host, ev

    def settle(self, keep: int = 0) -> int:
        """Confirm unverified steps until at most ``keep`` remain; re-runs (in
        order, from the first one's carried state) every unverified step once
        one of them turns out to have been skipped.  Returns the number of
        re-run steps."""
        pend = self._pending
        while len(pend) > keep:
            p = pend[0]
            p["ev"].synchronize()
            if int(p["host"][0]) == 0:
                pend.pop(0)
                continue
            # skipped on the device: this step and every later unverified one
            # (the flag stays set until cleared here) -- the same on every rank
            mod = _ext.extension()
            mod.persist_step_check()  # clear, count, turn the persistent path off
            mod.persist_disable()
            redo = list(pend)
            pend.clear()
            self.optimizer.rewind(len(redo))
            self.inner._state = redo[0]["carry0"]
            for q in redo:
                loss = self._fwd_bwd(q["inp"], q["tgt"])
                with trace_range("pdrnn.optimizer"):
                    self._clip()
                    self.optimizer.step()
                q["out"].copy_(loss.detach())
            return len(redo)
        return 0

    def train_step(self, inp: Tensor, tgt: Tensor) -> Tensor:
        if not self._deferred_verify():
            loss = self._fwd_bwd(inp, tgt)
            with trace_range("pdrnn.optimizer"):
                self._clip()
                self.optimizer.step()
            return loss.detach()
        self.settle(keep=1)  # the step before the previous one is done by now
        carry0 = getattr(self.inner, "_state", None)
        loss = self._fwd_bwd(inp, tgt)
        flag, host, ev = self._step_flag()
        with trace_range("pdrnn.optimizer"):
            self._clip()
            self.optimizer.step(skip=flag)
        out = loss.detach()  # a re-run overwrites it in place
        self._pending.append(dict(inp=inp, tgt=tgt, carry0=carry0, host=host, ev=ev, out=out))
        return out

    def train_epoch(self, epoch: int = 0, max_steps: Optional[int] = None) -> Dict[str, float]:
        self.inner.train()
        self.inner.reset_hidden_state()
        losses: List[Tensor] = []
        tokens = 0
        t0 = time.perf_counter()
        for step, (inp, tgt) in enumerate(CharCorpus.segments(self.streams, self.seq_len, max_steps)):
            losses.append(self.train_step(inp, tgt))
            tokens += inp.numel()
            if self.log_interval and (step + 1) % self.log_interval == 0:
                self.settle()
                cur = float(torch.stack(losses[-self.log_interval:]).mean())
                logging.info(f"Rank: {self.rank:02d}   Epoch {epoch} Step {step + 1}\tLoss: {cur:.6f}"
                             f"\tbpc: {cur / math.log(2):.4f}")
        self.settle()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - t0
        mean = float(torch.stack(losses).mean()) if losses else float("nan")
        out = {"loss": mean, "tokens": tokens, "duration": dt, "tokens_per_sec": tokens / dt if dt else 0.0,
               "steps": len(losses), "device_peak_mib": device_peak_mib(self.device)}
        ps = _ext.persist_stats()
        out.update(ps)
        logging.info(f"{self.rank}: Epoch {epoch} loss {mean:.6f} tokens/s {out['tokens_per_sec']:.1f} "
                     f"(x{self.world} ranks) device_peak_mib={out['device_peak_mib']:.1f} "
                     f"persist_verify={ps['persist_verify']} persist_fallbacks={ps['persist_fallbacks']}")
        return out

    # ------------------------------------------------------------ checkpoints
    def save(self, path, epoch: int, loss: float):
        """Rank 0 writes the reference checkpoint layout (epoch, model_state,
        optimizer_state, loss); returns the path or None on other ranks."""
        self.settle()
        if self.rank != 0:
            return None
        return save_checkpoint(path, epoch, self.model, self.optimizer, loss)

    def resume(self, path) -> int:
        """Load a checkpoint (weights_only); returns the next epoch index."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        self.model.load_state_dict(adapt_state_dict_keys(ck["model_state"], self.model))
        if ck.get("optimizer_state") is not None:
            self.optimizer.load_state_dict(ck["optimizer_state"])
        return int(ck.get("epoch", 0))
