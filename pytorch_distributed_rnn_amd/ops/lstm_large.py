"""Large-hidden LSTM path (placeholder until the MFMA kernels land)."""
from __future__ import annotations


def supported(x, hidden, num_layers) -> bool:  # noqa: D401
    return False


def lstm_large_forward(*args, **kwargs):
    raise NotImplementedError
