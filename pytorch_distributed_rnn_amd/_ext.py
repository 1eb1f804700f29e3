"""Loader for the in-tree native extension ``pytorch_distributed_rnn_amd._C``.

Policy (so that GPU runs never silently fall back to eager PyTorch):

* On a machine with a visible GPU the HIP kernels ARE the compute path.  If the
  extension cannot be imported there, :func:`native` raises with the import
  error, unless ``PDRNN_ALLOW_FALLBACK=1`` is set explicitly.
* On a CPU-only machine (this container, CI) the torch reference path is used
  and :func:`native` returns ``None``.
* ``PDRNN_KERNELS=torch`` forces the reference path everywhere (testing aid,
  mirrors the ``--kernel torch`` CLI flag); ``PDRNN_KERNELS=hip-strict``
  (``--kernel hip``) turns every remaining ATen/MIOpen fallback into an error,
  otherwise such a fallback warns once (:func:`fallback`).
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
from typing import Optional

import torch

_C = None
_IMPORT_ERROR: Optional[BaseException] = None
_TRIED = False


def _try_import():
    global _C, _IMPORT_ERROR, _TRIED
    if _TRIED:
        return _C
    _TRIED = True
    try:
        so = os.environ.get("PDRNN_EXT_SO")
        if so:
            # an alternative build of the extension (e.g. the sanitizer build of
            # _build.py, PDRNN_SANITIZE): loaded under the same module name
            spec = importlib.util.spec_from_file_location("pytorch_distributed_rnn_amd._C", so)
            _C = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules["pytorch_distributed_rnn_amd._C"] = _C
            return _C
        _C = importlib.import_module("pytorch_distributed_rnn_amd._C")
    except BaseException as e:  # noqa: BLE001 - report any loader failure verbatim
        _IMPORT_ERROR = e
        _C = None
    return _C


def kernels_mode() -> str:
    return os.environ.get("PDRNN_KERNELS", "hip").lower()


def gpu_available() -> bool:
    return torch.cuda.is_available()


def extension():
    """Return the imported extension module (or None) regardless of device."""
    return _try_import()


def native(device: Optional[torch.device] = None):
    """The native module if HIP kernels should run for ``device``; else None."""
    if kernels_mode() == "torch":
        return None
    if device is not None and torch.device(device).type != "cuda":
        return None
    if not gpu_available():
        return None
    mod = _try_import()
    if mod is None and os.environ.get("PDRNN_ALLOW_FALLBACK", "0") != "1":
        raise RuntimeError(
            "pytorch_distributed_rnn_amd: GPU present but the native extension failed to load "
            f"({_IMPORT_ERROR!r}). Build it with `python -m pytorch_distributed_rnn_amd._build` "
            "or set PDRNN_ALLOW_FALLBACK=1 to run the (slow) torch reference path."
        )
    return mod


_WARNED = set()


def strict_kernels() -> bool:
    """``PDRNN_KERNELS=hip-strict`` (CLI ``--kernel hip``): a shape that no HIP
    kernel covers raises instead of falling back to ATen/MIOpen."""
    return kernels_mode() in ("hip-strict", "strict")


def fallback(what: str, device=None) -> None:
    """Called right before an op runs the ATen/MIOpen reference on a GPU
    because no HIP kernel covers the configuration: warns once per ``what``
    (never silent), raises under :func:`strict_kernels`.  No-op on CPU runs and
    under ``PDRNN_KERNELS=torch`` (the reference path was asked for)."""
    if kernels_mode() == "torch" or not gpu_available():
        return
    if device is not None and torch.device(device).type != "cuda":
        return
    msg = f"pytorch_distributed_rnn_amd: no HIP kernel for {what}; running the ATen/MIOpen reference"
    if strict_kernels():
        raise RuntimeError(msg + " (strict kernel mode: PDRNN_KERNELS=hip-strict / --kernel hip)")
    if what not in _WARNED:
        _WARNED.add(what)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def require():
    """Import the extension or raise (used by build checks and GPU tests)."""
    mod = _try_import()
    if mod is None:
        raise RuntimeError(f"native extension not importable: {_IMPORT_ERROR!r}")
    return mod


def persist_stats() -> dict:
    """Persistent large-H recurrence health of this process: per-launch
    verification on/off, launches re-run on the per-step kernels after a
    grid-sync timeout, and whether the persistent path is off for good
    (bindings.cpp large_persist)."""
    mod = extension()
    if mod is None or not hasattr(mod, "persist_fallbacks"):
        return {"persist_verify": "off", "persist_fallbacks": 0, "persist_disabled": False}
    mode = int(mod.persist_verify_mode())
    return {"persist_verify": ("off", "launch", "step")[mode] if 0 <= mode <= 2 else str(mode),
            "persist_fallbacks": int(mod.persist_fallbacks()), "persist_disabled": bool(mod.persist_disabled())}
