"""Trace ranges and profiler capture (SURVEY.md §5 "Tracing / profiling").

The reference instruments training with a wall clock and a peak-RSS sampler
only (reference: src/motion/trainer/base.py:93-96).  Here the phases of every
training step -- forward, BPTT backward, gradient all-reduce, optimizer -- can
be bracketed, opt-in (``PDRNN_TRACE=1`` or ``--trace`` on the CLIs), by

* roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm), which
  ``rocprofv3 --marker-trace`` shows on the timeline beside the HIP kernels
  and the RCCL all-reduce, and
* ``torch.profiler.record_function`` labels, which a ``--profile DIR`` capture
  (:func:`profile`) writes into a chrome trace plus a per-op summary table.

Off by default: each range is two host calls on the step's critical path.
"""
from __future__ import annotations

import contextlib
import os
from pathlib import Path
from typing import Iterator, Optional, Union

import torch

_ENABLED = os.environ.get("PDRNN_TRACE", "0") == "1"


def enable(on: bool = True) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


@contextlib.contextmanager
def trace_range(name: str) -> Iterator[None]:
    """Named range around a training-step phase (no-op unless enabled)."""
    if not _ENABLED:
        yield
        return
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except (RuntimeError, AttributeError):
            pushed = False
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def profile(out_dir: Optional[Union[str, Path]], rank: int = 0) -> Iterator[Optional[object]]:
    """torch.profiler capture of the enclosed region (CPU + HIP activity) with
    the trace ranges switched on; writes ``trace_rank{r}.json`` (chrome
    trace) and ``summary_rank{r}.txt`` (top ops by device time) to
    ``out_dir``.  ``out_dir=None``: no-op."""
    if out_dir is None:
        yield None
        return
    from torch.profiler import ProfilerActivity
    from torch.profiler import profile as _profile

    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)
    prev = _ENABLED
    enable(True)
    try:
        with _profile(activities=acts) as prof:
            yield prof
    finally:
        enable(prev)
    prof.export_chrome_trace(str(out / f"trace_rank{rank}.json"))
    key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
    (out / f"summary_rank{rank}.txt").write_text(prof.key_averages().table(sort_by=key, row_limit=40))
