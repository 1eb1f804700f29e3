"""Operators: fused HIP kernels with torch reference fallbacks."""
from .lstm import lstm_forward, lstm_reference  # noqa: F401
from .xent import CrossEntropyLoss, cross_entropy, cross_entropy_with_stats  # noqa: F401
