"""Trace ranges / profiler capture (utils/tracing.py) and the CLI switches that
drive them, on the CPU path."""
import json
import os
import sys

import torch

from _mp import ROOT, run
from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
from pytorch_distributed_rnn_amd.models.motion import MotionModel
from pytorch_distributed_rnn_amd.train.trainer import Trainer
from pytorch_distributed_rnn_amd.utils import tracing

MAIN = os.path.join(ROOT, "src", "motion", "main.py")


def test_trace_range_is_a_noop_when_disabled():
    assert not tracing.enabled()
    with tracing.trace_range("pdrnn.nothing"):
        x = torch.ones(3).sum()
    assert float(x) == 3.0


def test_profile_captures_step_phases(tmp_path):
    train, _, _ = synthetic_motion(n_train=96, n_validation=1, n_test=1, seed=0)
    tr = Trainer(MotionModel(9, 8, 2, 6), train, 48, 1e-3, device=torch.device("cpu"))
    with tracing.profile(tmp_path / "prof"):
        tr.train(1)
    assert not tracing.enabled()  # restored after the capture
    trace = json.load(open(tmp_path / "prof" / "trace_rank0.json"))
    names = {e.get("name") for e in trace["traceEvents"]}
    assert {"pdrnn.forward", "pdrnn.backward", "pdrnn.optimizer"} <= names
    assert (tmp_path / "prof" / "summary_rank0.txt").read_text().strip()


def test_cli_bidirectional_fp16_trace_profile(tmp_path):
    out = run([sys.executable, MAIN, "--seed", "2", "--epochs", "1", "--batch-size", "96", "--no-validation",
               "--synthetic", "--synthetic-size", "96", "--device", "cpu", "--hidden-units", "8",
               "--bidirectional", "--trace", "--profile", str(tmp_path / "p"), "local"], cwd=str(tmp_path))
    assert "0: Memory Usage:" in out
    assert (tmp_path / "p" / "trace_rank0.json").exists()


def test_bidirectional_motion_model_head_reads_last_position():
    torch.manual_seed(0)
    m = MotionModel(9, 8, 2, 6, bidirectional=True)
    x = torch.randn(4, 10, 9)
    out, _ = torch.nn.LSTM.forward(m.lstm, x)
    torch.testing.assert_close(m(x), m.fc(out[:, -1, :]))
    assert m.fc.in_features == 16
