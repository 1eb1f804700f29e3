"""Checkpoint save / resume.

Format (unchanged from the reference, so files load in stock PyTorch and in the
reference code): ``{"epoch": epoch + 1, "model_state": model.state_dict(),
"optimizer_state": optimizer.state_dict(), "loss": loss}`` written with
``torch.save`` (reference: src/motion/trainer/base.py:164-177).  Under DDP the
model is the wrapper, so keys carry the ``module.`` prefix exactly like
``torch.nn.parallel.DistributedDataParallel``; Horovod/local keys have none.

Additions: tensors are moved to host memory before saving (checkpoints written
on an MI355X load on a CPU-only machine without ``map_location``), and a
resume path the reference does not have, accepting prefixed and unprefixed
keys and loading with ``weights_only=True`` (no arbitrary unpickling).
Fused-kernel private layouts never enter a checkpoint: the flat buffers are
views of the very parameters ``state_dict`` returns.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict, Optional

import torch
from torch import nn


def _to_host(obj: Any) -> Any:
    if torch.is_tensor(obj):
        return obj.detach().to("cpu", copy=True)
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_to_host(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_to_host(v) for v in obj)
    return obj


def save_checkpoint(path: Path, epoch: int, model: nn.Module, optimizer, loss) -> Path:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    checkpoint = {
        "epoch": epoch + 1,
        "model_state": _to_host(model.state_dict()),
        "optimizer_state": _to_host(optimizer.state_dict()) if optimizer is not None else None,
        "loss": float(loss) if loss is not None else None,
    }
    tmp = path.with_name(path.name + ".tmp")
    torch.save(checkpoint, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a truncated best-model.pt
    return path


def adapt_state_dict_keys(state: Dict[str, torch.Tensor], model: nn.Module) -> Dict[str, torch.Tensor]:
    """Add or strip the DDP ``module.`` prefix so ``state`` matches ``model``."""
    want = set(model.state_dict().keys())
    have = set(state.keys())
    if have == want:
        return state
    if all(k.startswith("module.") for k in have) and {k[len("module."):] for k in have} == want:
        return {k[len("module."):]: v for k, v in state.items()}
    if {"module." + k for k in have} == want:
        return {"module." + k: v for k, v in state.items()}
    return state


def load_checkpoint(path: Path, model: nn.Module, optimizer=None, map_location=None) -> int:
    """Restore model (and optimizer) in place; returns the epoch to continue from."""
    ck = torch.load(Path(path), map_location=map_location or "cpu", weights_only=True)
    state = adapt_state_dict_keys(ck["model_state"], model)
    with torch.no_grad():
        # copy in place: keeps flat-buffer views (fused optimizer / reducer) valid
        own = model.state_dict()
        missing = [k for k in own if k not in state]
        if missing:
            raise KeyError(f"checkpoint lacks keys {missing[:5]}...")
        for k, v in own.items():
            v.copy_(state[k].to(v.device, v.dtype))
    if optimizer is not None and ck.get("optimizer_state") is not None:
        optimizer.load_state_dict(ck["optimizer_state"])
    return int(ck.get("epoch", 0))


def read_checkpoint(path: Path) -> Dict[str, Any]:
    return torch.load(Path(path), map_location="cpu", weights_only=True)
