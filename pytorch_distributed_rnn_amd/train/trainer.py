"""Training engine: epoch loop, evaluation, best-model checkpointing, timing and
memory measurement.

Surface-compatible with the reference ``Trainer`` (reference:
src/motion/trainer/base.py:14-177): same constructor arguments, the same
overridable hooks (``_get_optimizer``, ``_get_data_loader``, ``_get_formatter``,
``_train_step``, ``_evaluate``, ``_save_checkpoint``, ``_reset_hidden_state``),
the same ``train(epochs) -> (model.eval(), train_history, validation_history)``
contract, the same log lines and checkpoint dict.

MI355X-first differences (all behaviour-preserving):

* the model, its flat parameter/gradient buffers and the whole training set
  live in HBM; batches are gathered on the device (``DeviceBatchLoader``);
* the loss is the fused cross-entropy kernel, which also yields the correct
  count, so no extra argmax pass;
* per-step statistics stay on the device and the ``Train Batch`` lines are
  emitted from one host transfer every ``log_interval`` steps (default: once
  per epoch) instead of two blocking ``.item()`` calls per step -- the lines
  and their order are unchanged;
* the measured region is GPU-synchronised on both ends; the peak RSS line is
  followed by a ``Throughput`` line (sequences/s, HBM peak).
"""
from __future__ import annotations

import logging
import os
import time
from pathlib import Path
from typing import Callable, List, Optional, Tuple

import torch
from torch import Tensor, nn

from ..ops import gradsink
from ..data.loader import DeviceBatchLoader, ShardedSampler
from ..ops.adam import FusedAdam
from ..ops.xent import CrossEntropyLoss
from ..utils import memory as mem
from ..utils.flat import flatten_module
from ..utils.tracing import trace_range
from . import checkpoint as ckpt
from .formatter import TrainingMessageFormatter

log = logging.getLogger(__name__)


def default_device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def stats_to_host(rows: List[Tensor]) -> Tensor:
    """Per-batch [loss, n, correct] rows -> one host tensor.  Rows that are
    consecutive rows of one device buffer (the fused step's statistics ring)
    come back as a single device->host copy of that slice, with no gather
    kernel; anything else is stacked first."""
    r0 = rows[0]
    base = r0._base
    if base is not None and base.dim() == 2 and base.is_contiguous() and r0.dim() == 1 and \
            r0.numel() == base.shape[1] and all(r._base is base for r in rows):
        o0 = r0.storage_offset() - base.storage_offset()
        if o0 % base.shape[1] == 0 and all(r.storage_offset() == r0.storage_offset() + i * base.shape[1]
                                           for i, r in enumerate(rows)):
            first = o0 // base.shape[1]
            if first + len(rows) <= base.shape[0]:
                return base[first:first + len(rows)].detach().cpu()
    return torch.stack(rows).detach().cpu()




class _Timeline:
    """Host timestamps of the timed epoch's phases (``PDRNN_EPOCH_TIMELINE=1``:
    printed to stderr after the run) -- where the CLI's Training Duration
    goes beyond the GPU step time (diagnostics only)."""

    def __init__(self):
        self.on = os.environ.get("PDRNN_EPOCH_TIMELINE", "0") == "1"
        self.marks: List[Tuple[str, float]] = []

    def mark(self, name: str) -> None:
        if self.on:
            self.marks.append((name, time.perf_counter()))

    def report(self) -> None:
        if not self.on or not self.marks:
            return
        import sys
        t0, prev = self.marks[0][1], self.marks[0][1]
        for name, t in self.marks:
            print(f"[timeline] {name:<24} +{(t - prev) * 1e6:9.1f} us  @ {(t - t0) * 1e6:9.1f} us", file=sys.stderr)
            prev = t
        self.marks.clear()


_TL = _Timeline()

def _persist_check() -> None:
    """A persistent-recurrence launch that timed out without per-launch
    verification (single rank) fails the run here at the latest."""
    if torch.cuda.is_available():
        from .. import _ext
        mod = _ext.extension()
        if mod is not None and hasattr(mod, "persist_check"):
            mod.persist_check()

class Trainer:
    loss_fn = CrossEntropyLoss()

    def __init__(self, model: nn.Module, training_set, batch_size: int, learning_rate: float,
                 validation_set=None, test_set=None, checkpoint_dir: Optional[Path] = None,
                 sampler: Optional[ShardedSampler] = None, *, device: Optional[torch.device] = None,
                 log_interval: int = 0, checkpoint_every: int = 0, flatten: bool = True,
                 cuda_graph: Optional[bool] = None, warmup: bool = True):
        self.device = torch.device(device) if device is not None else default_device()
        self.warmup = warmup
        # replay the synced fused step from a HIP graph (None: PDRNN_CUDA_GRAPH)
        self.cuda_graph = cuda_graph
        self.model = model.to(self.device)
        inner = getattr(self.model, "module", self.model)
        if flatten and not getattr(inner, "_pdrnn_flat", None):
            flatten_module(inner)
        self.checkpoint_dir = Path(checkpoint_dir) if checkpoint_dir is not None else None
        self.checkpoint_every = checkpoint_every
        self.log_interval = log_interval
        self.sampler = sampler or ShardedSampler(len(training_set), num_replicas=1, rank=0)
        self.train_loader = self._get_data_loader(training_set, batch_size, sampler=self.sampler)
        self.validation_loader = self._get_data_loader(validation_set, batch_size=None)
        self.test_loader = self._get_data_loader(test_set, batch_size=None)
        self.optimizer = self._get_optimizer(self.model, learning_rate)
        self.start_epoch = 0
        self.sequences_seen = 0

    # ------------------------------------------------------------------ hooks
    def _get_optimizer(self, model: nn.Module, lr: float):
        return FusedAdam(model.parameters(), lr=lr)

    def _get_data_loader(self, dataset, batch_size: Optional[int] = None,
                         sampler: Optional[ShardedSampler] = None):
        if dataset is None:
            return None
        inner = getattr(self.model, "module", self.model)
        in_kernel = self.device.type == "cuda" and getattr(inner, "supports_index_batches", False)
        cdt = getattr(inner, "compute_dtype", torch.float32)
        return DeviceBatchLoader(dataset, batch_size, sampler=sampler, device=self.device,
                                 gather_in_kernel=in_kernel,
                                 feature_dtype=cdt if self.device.type == "cuda" else None)

    def _get_formatter(self, epochs: int) -> TrainingMessageFormatter:
        return TrainingMessageFormatter(epochs)

    def _reset_hidden_state(self) -> None:
        target = getattr(self.model, "module", self.model)
        if hasattr(target, "reset_hidden_state"):
            target.reset_hidden_state()

    # ------------------------------------------------------------------ loop
    def train(self, epochs: int):
        training_history: List[float] = []
        validation_history: List[float] = []
        formatter = self._get_formatter(epochs)

        def train_inner():
            best_loss = None
            for epoch in range(self.start_epoch, epochs):
                if self.sampler is not None:
                    self.sampler.set_epoch(epoch)
                logging.info(formatter.epoch_start_message(epoch))
                _TL.mark("epoch_begin")
                self._prefetch_epoch = epoch + 1 if epoch + 1 < epochs else None
                train_loss, _train_acc = self._train_step(formatter)
                _TL.mark("train_step_done")
                training_history.append(train_loss)
                if self.validation_loader is not None:
                    validation_loss, _ = self._evaluate(self.validation_loader, formatter, epoch)
                    validation_history.append(validation_loss)
                    if best_loss is None or best_loss > validation_loss:
                        logging.info(f"New best model in epoch {epoch + 1}")
                        best_loss = validation_loss
                        self._save_checkpoint(epoch, validation_loss, best=True)
                if self.checkpoint_every and (epoch + 1) % self.checkpoint_every == 0:
                    self._save_checkpoint(epoch, train_loss, best=False)

        if self.warmup:
            t0 = time.perf_counter()
            self.prepare()
            logging.info(f"Warm-up (kernel load, workspace sizing; no parameter update): "
                         f"{time.perf_counter() - t0:.4f} s")
        mem.reset_device_peak(self.device if self.device.type == "cuda" else None)
        self.sequences_seen = 0
        # the RSS high-water-mark reset (a page-table walk of the whole address
        # space, ~0.15 ms with the GPU mappings) happens before the clock starts
        with mem.peak_rss_monitor() as rss:
            mem.synchronize()
            start = time.perf_counter()
            _TL.mark("start")
            train_inner()
            _TL.mark("inner_done")
            mem.synchronize()
            duration = time.perf_counter() - start
            _TL.mark("synced")
        memory = rss.peak
        _TL.report()
        _persist_check()
        logging.info(formatter.performance_message(memory, duration))
        logging.info(formatter.throughput_message(self.sequences_seen, duration,
                                                  mem.device_peak_mib(), self.world_size()))
        self.last_duration = duration
        self.last_peak_rss = memory
        if self.test_loader is not None:
            self._evaluate(self.test_loader, formatter)
        return self.model.eval(), training_history, validation_history

    def world_size(self) -> int:
        return 1

    def prepare(self) -> None:
        """One-time device setup before the timed epochs: the fused step runs
        a gradient-only pass (no optimizer update, gradients discarded) for
        each batch shape of the epoch -- the full batch and the short last one
        -- so that kernel code-object loading and the caching allocator's
        first allocations are not charged to the first epoch; then repeats
        the full-batch pass until the GPU has been busy for
        ``PDRNN_WARMUP_MS`` (default 40 ms): after host-side setup the GPU
        clocks ramp up under load and kernel times fall by ~12 % over the
        first ~25 ms (profiles/r2_clock_ramp.md).  A no-op on the CPU /
        autograd path.  Disable with ``warmup=False`` (CLI ``--no-warmup``)."""
        fused = self._fused_step()
        if fused is None:
            return
        loader = self.train_loader
        n = loader.num_items
        sizes = sorted({min(loader.batch_size, n), n % loader.batch_size or loader.batch_size})
        self.model.train()

        def one_pass(b):
            batch = loader.make_batch(torch.arange(b, device=loader.device))
            if len(batch) == 3:
                features, labels_all, idx = batch
                fused.warmup(features, labels_all, idx)
            else:
                data, labels = batch
                fused.warmup(data, labels.reshape(-1).contiguous(), None)

        for b in sizes:
            one_pass(b)
        # the per-epoch index path (host permutation, pinned staging buffer,
        # host->device copy): its first use allocates the staging buffer
        if self.sampler is not None:
            loader.batch_indices()
        # optimizer state (Adam moments: zeros either way) exists before the
        # first timed step instead of being allocated and zeroed inside it
        materialize = getattr(self.optimizer, "materialize_state", None)
        if materialize is not None:
            materialize()
        # the epoch-end statistics read-back (first use of the copy / stack
        # kernels costs ~10 ms of code-object loading on a fresh process)
        ring = getattr(fused, "ring", None)
        if ring is not None:
            stats_to_host([ring[0], ring[1]])
            stats_to_host([ring[1], ring[0]])
        mem.synchronize()
        try:
            budget = float(os.environ.get("PDRNN_WARMUP_MS", "40")) / 1e3
        except ValueError:
            budget = 0.04
        t0 = time.perf_counter()
        for _ in range(1000):
            if time.perf_counter() - t0 >= budget:
                break
            one_pass(max(sizes))
            mem.synchronize()
        # the multi-GPU step replays whole epochs from one HIP graph: captured
        # here, for the epoch's batch sizes (the full ones and the short last)
        if hasattr(fused, "prepare_epoch") and loader.gather_in_kernel:
            bs = loader.batch_size
            fused.prepare_epoch(loader.features, loader.labels, [min(bs, n - k) for k in range(0, n, bs)])
        # the first timed epoch's indices (DataLoader-style prefetch)
        if self.sampler is not None and hasattr(loader, "prefetch"):
            self.sampler.set_epoch(self.start_epoch)
            loader.prefetch()

    def _forward(self, batch) -> Tuple[Tensor, Tensor]:
        if len(batch) == 3:
            features, labels_all, idx = batch
            return self.model(features, idx=idx), labels_all.index_select(0, idx)
        data, labels = batch
        return self.model(data), labels

    # ------------------------------------------------------------ fused step
    def _grad_sync(self):
        """Gradient synchronisation used by the fused step (None: local)."""
        return None

    def _grad_comm(self):
        """The communicator ``_grad_sync`` runs on (its watchdog bounds the
        fused step's graph replays); None: local."""
        return None

    def _fused_step(self):
        if getattr(self, "_fused", False) is not False:
            return self._fused
        self._fused = None
        if os.environ.get("PDRNN_FUSED_STEP", "1") != "0":
            from . import fused_step
            if fused_step.supported(self.model, self.optimizer, self.device):
                self._fused = fused_step.MotionTrainStep(self.model, self.optimizer, self._grad_sync(),
                                                         cuda_graph=self.cuda_graph, comm=self._grad_comm())
        return self._fused

    def _direct_grads_ok(self) -> bool:
        """The in-tree Functions may accumulate weight gradients straight into
        the flat .grad views (ops/gradsink.py).  Multi-rank too: the
        framework's reducers (parallel/ddp.py, parallel/horovod.py) mark a
        parameter ready from a post-accumulate-grad hook, which autograd fires
        after the Function has returned -- with ``.grad`` already the finished
        view (AccumulateGrad runs with an undefined incoming gradient and
        leaves it alone).  Proven against the plain path on gloo ranks
        (tests/test_distributed_cpu.py::test_direct_grads_under_ddp_and_horovod_match).
        torch's own DDP reducer is not used with the flat views.
        (``PDRNN_TUNE=direct_grads=0``: the autograd adds, for A/B.)"""
        from ..utils.tune import tune
        return self.device.type == "cuda" and tune("direct_grads", "1") != "0"

    def train_batch(self, batch) -> Tuple[Tensor, int]:
        """One optimizer step on one batch; returns (stats [loss, n, correct], batch size).

        This is the exact step ``bench.py`` times.  On MI355X the motion model
        runs the fused whole-step path (train/fused_step.py); otherwise the
        autograd path below."""
        fused = self._fused_step()
        if fused is not None and self.model.training:
            if len(batch) == 3:
                features, labels_all, idx = batch
                return fused(features, labels_all, idx), idx.numel()
            data, labels = batch
            return fused(data, labels.reshape(-1).contiguous(), None), labels.shape[0]
        self.optimizer.zero_grad()
        with gradsink.direct_grads(self._direct_grads_ok()):
            with trace_range("pdrnn.forward"):
                output, labels = self._forward(batch)
                labels = labels.long().reshape(-1)
                loss = self.loss_fn(output, labels)
                stats = self.loss_fn.last_stats
            with trace_range("pdrnn.backward"):
                loss.backward()
        with trace_range("pdrnn.optimizer"):
            self.optimizer.step()
        return stats, labels.shape[0]

    def train_batches(self, batches) -> List[Tuple[Tensor, int]]:
        """Several optimizer steps on consecutive batches (an epoch); returns
        ``train_batch``'s (stats, batch size) per batch.  The multi-GPU fused
        step replays all of them from ONE HIP graph
        (``MotionTrainStep.run_steps``); otherwise -- or when ``train_batch``
        is wrapped (fault injection) -- one ``train_batch`` per batch."""
        batches = list(batches)
        fused = self._fused_step()
        if fused is not None and self.model.training and "train_batch" not in self.__dict__ and batches and \
                all(len(b) == 3 for b in batches):
            feats, labels = batches[0][0], batches[0][1]
            if all(b[0] is feats and b[1] is labels for b in batches):
                res = fused.run_steps(feats, labels, [b[2] for b in batches])
                if res is not None:
                    return [(st, b[2].numel()) for st, b in zip(res, batches)]
        return [self.train_batch(b) for b in batches]

    def _train_step(self, formatter: TrainingMessageFormatter):
        # (mode switch only when needed: with the DDP wrapper the first
        # Module.train() of the timed epoch cost 0.4-0.55 ms of host time before
        # the first launch -- profiles/r6/cli_epoch_timeline.md)
        if not self.model.training or any(not m.training for m in self.model.children()):
            self.model.train()
        loader = self.train_loader
        batches = len(loader)
        pending: List[Tuple[int, int, Tensor]] = []
        total_loss = 0.0
        total_correct = 0

        def flush():
            nonlocal total_loss, total_correct
            if not pending:
                return
            host = stats_to_host([s for _, _, s in pending])
            _TL.mark("stats_on_host")
            for (bi, n, _), row in zip(pending, host):
                loss_v, _, correct = float(row[0]), int(row[1]), int(row[2])
                total_loss += loss_v
                total_correct += correct
                logging.info(formatter.train_progress_message(
                    batch_idx=bi, batches=batches, training_examples=n, correct=correct, loss=loss_v))
            pending.clear()
            _TL.mark("logged")

        if self.log_interval:
            for batch_idx, batch in enumerate(loader):
                _TL.mark(f"batch{batch_idx}_ready")
                stats, n = self.train_batch(batch)
                _TL.mark(f"batch{batch_idx}_issued")
                self.sequences_seen += n
                pending.append((batch_idx, n, stats))
                if len(pending) >= self.log_interval:
                    flush()
        else:
            # the whole epoch at once (one graph replay on the multi-GPU fused path)
            for batch_idx, (stats, n) in enumerate(self.train_batches(loader)):
                self.sequences_seen += n
                pending.append((batch_idx, n, stats))
            _TL.mark("epoch_issued")
        # next epoch's indices while the GPU drains this one's steps
        nxt = getattr(self, "_prefetch_epoch", None)
        if nxt is not None and self.sampler is not None and hasattr(loader, "prefetch"):
            loader.prefetch(nxt)
        flush()
        n_train = len(loader.dataset)
        return total_loss / n_train, total_correct / n_train

    @torch.no_grad()
    def _evaluate(self, data_loader, formatter: TrainingMessageFormatter, epoch: Optional[int] = None):
        self.model.eval()
        eval_loss = 0.0
        total_correct = 0
        for batch in data_loader:
            output, labels = self._forward(batch)
            labels = labels.long().reshape(-1)
            loss = self.loss_fn(output, labels)
            stats = self.loss_fn.last_stats.cpu()
            eval_loss += float(stats[0])
            total_correct += int(stats[2])
            if log.isEnabledFor(logging.DEBUG) or logging.getLogger().isEnabledFor(logging.DEBUG):
                logging.debug(f"Model predicted {torch.argmax(output, dim=1).data}; "
                              f"Correct was {labels.data}")
        eval_loss /= len(data_loader)
        num_examples = len(data_loader.dataset)
        accuracy = float(total_correct) / num_examples
        logging.info(formatter.evaluation_message(accuracy, num_examples, epoch, eval_loss, total_correct))
        return eval_loss, accuracy

    def _save_checkpoint(self, epoch: int, loss: float, best: bool = False) -> Optional[Path]:
        if self.checkpoint_dir is None:
            return None
        name = "best-model.pt" if best else f"checkpoint-epoch-{epoch + 1}.pt"
        return ckpt.save_checkpoint(self.checkpoint_dir / name, epoch, self.model, self.optimizer, loss)

    def resume(self, path: Path) -> int:
        """Load a checkpoint written by this framework or the reference; returns next epoch."""
        self.start_epoch = ckpt.load_checkpoint(path, self.model, self.optimizer)
        return self.start_epoch
