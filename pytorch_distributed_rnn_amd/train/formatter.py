"""Log-line formats.

These strings are an API contract: the reference's analysis notebooks parse
them with regexes (``"(\\d+): Memory Usage: ([\\d.]+), Training Duration:
([\\d.]+)"``, reference: evaluation/Experiments.ipynb:49) and the per-step
``Train Batch`` lines carry the loss trajectory used as the world-size
invariance oracle.  Byte-for-byte identical to reference
src/motion/trainer/formatter.py:6-31; new metrics (sequences/s, HBM peak) go on
a separate ``Throughput`` line so the old regexes keep matching.
"""
from __future__ import annotations

from typing import Optional

_PREFIX = "Rank: {rank:02d}   "


def percentage(current: float, overall: float) -> float:
    return 100.0 * (current / overall)


class TrainingMessageFormatter:
    def __init__(self, num_epochs: int, rank: int = 0):
        self.num_epochs = num_epochs
        self.rank = rank

    def _prefix(self) -> str:
        return _PREFIX.format(rank=self.rank)

    def epoch_start_message(self, epoch: int) -> str:
        return f"{self._prefix()}Start Epoch {epoch}"

    def train_progress_message(self, batch_idx: int, batches: int, training_examples: int,
                               correct, loss: float) -> str:
        step = batch_idx + 1
        correct = int(correct)
        return (f"{self._prefix()}Train Batch: {step}/{batches} ({percentage(step, batches):.0f}%)"
                f"\tLoss: {loss:.6f}"
                f"\tAcc: {correct}/{training_examples} "
                f"({percentage(float(correct), training_examples):.0f}%)")

    def evaluation_message(self, accuracy: float, examples: int, epoch: Optional[int],
                           eval_loss: float, total_correct) -> str:
        body = (f"Loss: {eval_loss:.4f}\t Accuracy: {int(total_correct)}/{examples} "
                f"({100.0 * accuracy:.0f}%)\n")
        if epoch is None:
            return "Test Evaluation:\t" + body
        e = epoch + 1
        return f"Evaluation Epoch: {e}/{self.num_epochs} ({percentage(e, self.num_epochs):.0f}%)\t" + body

    def performance_message(self, memory, duration) -> str:
        return f"{self.rank}: Memory Usage: {memory}, Training Duration: {duration}"

    def throughput_message(self, sequences: int, duration: float, device_peak_mib: float,
                           world_size: int = 1) -> str:
        rate = sequences / duration if duration > 0 else float("nan")
        return (f"{self.rank}: Throughput: sequences={sequences} sequences_per_sec={rate:.1f} "
                f"world_size={world_size} device_peak_mib={device_peak_mib:.1f}")
