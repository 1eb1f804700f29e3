"""Log-line contract (reference: src/motion/trainer/formatter.py:6-31,
evaluation/Experiments.ipynb:49 regex)."""
import re

from pytorch_distributed_rnn_amd.train.formatter import TrainingMessageFormatter, percentage


def test_epoch_and_batch_lines():
    f = TrainingMessageFormatter(3, rank=1)
    assert f.epoch_start_message(0) == "Rank: 01   Start Epoch 0"
    assert (f.train_progress_message(0, 5, 288, 144, 1.2345678)
            == "Rank: 01   Train Batch: 1/5 (20%)\tLoss: 1.234568\tAcc: 144/288 (50%)")


def test_evaluation_lines():
    f = TrainingMessageFormatter(4, rank=0)
    assert (f.evaluation_message(0.5, 10, 1, 0.123456, 5)
            == "Evaluation Epoch: 2/4 (50%)\tLoss: 0.1235\t Accuracy: 5/10 (50%)\n")
    assert f.evaluation_message(0.25, 8, None, 1.0, 2).startswith("Test Evaluation:\tLoss: 1.0000")


def test_performance_line_matches_notebook_regex():
    f = TrainingMessageFormatter(1, rank=0)
    line = f.performance_message(123.5, 4.25)
    m = re.search(r"(\d+): Memory Usage: ([\d.]+), Training Duration: ([\d.]+)", line)
    assert m and m.groups() == ("0", "123.5", "4.25")
    # the extra throughput line must not be picked up by that regex
    assert "Memory Usage" not in f.throughput_message(100, 1.0, 0.0)


def test_percentage():
    assert percentage(1, 4) == 25.0
