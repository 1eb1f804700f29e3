"""Fault injection for distributed runs.

The reference injects network faults with ``tc qdisc ... netem delay/loss`` on
every Raspberry Pi's eth0 (reference: fabfile.py:125-191) and measures epoch
time under 0-400 ms delay and 0-15 % loss.  xGMI inside one MI355X node cannot
be netem'd, so the equivalent knobs act at the framework level:

* ``delay_ms``: host-side sleep injected into every training step of the
  selected rank(s) right before gradient synchronisation -- every other rank
  waits for it inside the all-reduce, exactly like a slow link;
* ``drop_rank`` / ``drop_step``: the selected rank exits abruptly at a given
  step, exercising collective timeouts (``init_distributed(timeout_s=...)``)
  and the launcher's failure detection;
* ``loss_prob``: with this probability a step's synchronisation is delayed by
  ``retransmit_ms`` (a TCP-retransmission-like stall), seeded per rank.

Configured from the CLI (``--fault-delay-ms``, ``--fault-rank``) or from
environment variables ``PDRNN_FAULT_DELAY_MS``, ``PDRNN_FAULT_RANK``,
``PDRNN_FAULT_DROP_STEP``, ``PDRNN_FAULT_LOSS``, ``PDRNN_FAULT_RETRANSMIT_MS``.
"""
from __future__ import annotations

import os
import random
import time
from dataclasses import dataclass
from typing import Optional


@dataclass
class FaultConfig:
    delay_ms: float = 0.0
    rank: int = -1              # -1: every rank
    drop_step: int = -1         # -1: never
    loss_prob: float = 0.0
    retransmit_ms: float = 200.0
    seed: int = 0


_CFG = FaultConfig(
    delay_ms=float(os.environ.get("PDRNN_FAULT_DELAY_MS", 0) or 0),
    rank=int(os.environ.get("PDRNN_FAULT_RANK", -1) or -1),
    drop_step=int(os.environ.get("PDRNN_FAULT_DROP_STEP", -1) or -1),
    loss_prob=float(os.environ.get("PDRNN_FAULT_LOSS", 0) or 0),
    retransmit_ms=float(os.environ.get("PDRNN_FAULT_RETRANSMIT_MS", 200) or 200),
)


def configure(**kw) -> FaultConfig:
    for k, v in kw.items():
        setattr(_CFG, k, v)
    return _CFG


def config() -> FaultConfig:
    return _CFG


def active() -> bool:
    return _CFG.delay_ms > 0 or _CFG.drop_step >= 0 or _CFG.loss_prob > 0


class _Injector:
    def __init__(self, rank: int, cfg: FaultConfig):
        self.rank = rank
        self.cfg = cfg
        self.step = 0
        self.rng = random.Random(cfg.seed * 1000 + rank)

    def targeted(self) -> bool:
        return self.cfg.rank < 0 or self.cfg.rank == self.rank

    def before_sync(self) -> float:
        """Apply the configured fault for this step; returns the injected delay (s)."""
        self.step += 1
        if not self.targeted():
            return 0.0
        if self.cfg.drop_step >= 0 and self.step >= self.cfg.drop_step:
            os._exit(17)  # abrupt failure, like a node dropping off the network
        delay = self.cfg.delay_ms / 1e3
        if self.cfg.loss_prob > 0 and self.rng.random() < self.cfg.loss_prob:
            delay += self.cfg.retransmit_ms / 1e3
        if delay > 0:
            time.sleep(delay)
        return delay


def install(trainer, cfg: Optional[FaultConfig] = None) -> _Injector:
    """Wrap ``trainer.train_batch`` so faults hit between forward and sync."""
    inj = _Injector(getattr(trainer, "rank", 0), cfg or _CFG)
    original = trainer.train_batch

    def train_batch(batch):
        inj.before_sync()
        return original(batch)

    trainer.train_batch = train_batch
    trainer._fault_injector = inj
    return inj
