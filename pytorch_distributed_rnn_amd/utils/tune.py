"""Tuning overrides: ``PDRNN_TUNE="key=value,key=value"``.

One environment variable carries every kernel-map / tiling override used for
A/B sweeps and by the tests that force a code path (the native side reads the
same string: ``csrc/runtime/tune.cpp``).  Keys (README.md, tuning overrides):

* small-H fused kernels: ``nb_fwd``, ``nb_bwd``, ``split_fwd``, ``split_bwd``,
  ``dwout`` (0 / force), ``dwout_nb``, ``prio``;
* sequence-in-wave kernels: ``sw_mode``, ``sw_bwd_mode``;
* large-H kernels: ``large_tile``, ``large_pp``, ``large_pp_bwd``, ``rows``,
  ``large_pipe``, ``large_chunks``, ``large_overlap``.

Read on every call: tests flip it in-process."""
from __future__ import annotations

import os
from typing import Dict, Optional


def tune_map() -> Dict[str, str]:
    out: Dict[str, str] = {}
    for item in os.environ.get("PDRNN_TUNE", "").split(","):
        k, eq, v = item.strip().partition("=")
        if eq and k:
            out[k.strip()] = v.strip()
    return out


def tune(key: str, default: Optional[str] = None) -> Optional[str]:
    return tune_map().get(key, default)


def tune_int(key: str, default: int) -> int:
    try:
        return int(tune_map().get(key, default))
    except ValueError:
        return default


def tune_string(values: Dict[str, object]) -> str:
    """``PDRNN_TUNE`` value with ``values`` merged over the current one (None
    removes a key)."""
    cur = tune_map()
    for k, v in values.items():
        if v is None:
            cur.pop(k, None)
        else:
            cur[k] = str(v)
    return ",".join(f"{k}={v}" for k, v in cur.items())
