"""Peak host-RSS and device-memory measurement.

Replaces ``memory_profiler.memory_usage`` which the reference wraps around its
epoch loop (reference: src/motion/trainer/base.py:5,93-96): a sampler thread
polls the process RSS (MiB, float -- same unit and format as memory_profiler)
while the wrapped function runs.  Device peak comes from the caching
allocator (``torch.cuda.max_memory_allocated`` on ROCm = HBM bytes in use).
"""
from __future__ import annotations

import os
import resource
import threading
import time
from typing import Any, Callable, Tuple

import torch

try:
    import psutil
except ImportError:  # pragma: no cover - psutil is in the image
    psutil = None


def current_rss_mib() -> float:
    if psutil is not None:
        return psutil.Process(os.getpid()).memory_info().rss / 2 ** 20
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0


class PeakRSSMonitor:
    def __init__(self, interval: float = 0.01):
        self.interval = interval
        self.peak = current_rss_mib()
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self._stop.is_set():
            self.peak = max(self.peak, current_rss_mib())
            self._stop.wait(self.interval)

    def __enter__(self):
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        self._t.join()
        self.peak = max(self.peak, current_rss_mib())
        return False


def _read_hwm_mib() -> float:
    with open("/proc/self/status", "rb") as f:
        for line in f:
            if line.startswith(b"VmHWM:"):
                return int(line.split()[1]) / 1024.0
    raise OSError("no VmHWM in /proc/self/status")


class KernelPeakRSS:
    """Peak RSS of a region from the kernel's own high-water mark: writing
    ``5`` to ``/proc/self/clear_refs`` resets ``VmHWM`` to the current RSS, and
    ``VmHWM`` read at the end is the exact peak in between -- no sampler
    thread competing for the GIL with the training loop (a polling thread
    also misses peaks shorter than its interval).  ``available()`` is False
    where procfs does not allow it; ``measure_peak_rss`` then samples."""

    @staticmethod
    def available() -> bool:
        try:
            with open("/proc/self/clear_refs", "wb") as f:
                f.write(b"5")
            _read_hwm_mib()
            return True
        except OSError:
            return False

    def __enter__(self):
        with open("/proc/self/clear_refs", "wb") as f:
            f.write(b"5")
        return self

    def __exit__(self, *exc):
        self.peak = _read_hwm_mib()
        return False


_HWM_OK = None


def peak_rss_monitor(interval: float = 0.01):
    """Context manager whose ``.peak`` (MiB) is the region's peak RSS."""
    global _HWM_OK
    if _HWM_OK is None:
        _HWM_OK = os.environ.get("PDRNN_RSS_SAMPLER", "0") != "1" and KernelPeakRSS.available()
    return KernelPeakRSS() if _HWM_OK else PeakRSSMonitor(interval)


def measure_peak_rss(fn: Callable[[], Any], interval: float = 0.01) -> Tuple[float, Any]:
    """Run ``fn`` and return (peak RSS in MiB during the run, fn's result)."""
    with peak_rss_monitor(interval) as mon:
        result = fn()
    return mon.peak, result


def device_peak_mib(device=None) -> float:
    if torch.cuda.is_available():
        return torch.cuda.max_memory_allocated(device) / 2 ** 20
    return 0.0


def reset_device_peak(device=None) -> None:
    if torch.cuda.is_available():
        torch.cuda.reset_peak_memory_stats(device)


def synchronize(device=None) -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize(device)


class Stopwatch:
    """perf_counter bracketed by device synchronisation."""

    def __init__(self, device=None):
        self.device = device
        self.elapsed = 0.0

    def __enter__(self):
        synchronize(self.device)
        self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        synchronize(self.device)
        self.elapsed = time.perf_counter() - self._t0
        return False
