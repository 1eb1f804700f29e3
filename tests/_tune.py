"""Tests force kernel paths through PDRNN_TUNE (pytorch_distributed_rnn_amd/utils/tune.py)."""
from pytorch_distributed_rnn_amd.utils.tune import tune_string


def set_tune(monkeypatch, **values):
    """Merge ``values`` into PDRNN_TUNE for this test (None removes a key)."""
    monkeypatch.setenv("PDRNN_TUNE", tune_string(values))
