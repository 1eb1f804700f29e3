"""Motion (UCI-HAR inertial signals) dataset: cached tensors, raw-text
preprocessing, and a synthetic generator with identical shapes.

Parity with the reference data layer:

* ``MotionDataset`` -- ``LABELS``, ``features``/``labels``, ``seq_length``,
  ``num_features``, ``__getitem__``/``__len__``, ``random_split`` and
  ``load(base_path, output_path, validation_fraction)`` that reuses cached
  ``X_{train,validation,test}.pt`` / ``y_*.pt`` and otherwise preprocesses the
  raw text files (reference: src/motion/dataset.py:10-73).
* ``MotionDataProcessor`` -- 9 "Inertial Signals" channels per split ->
  ``[N, 128, 9]`` float32, labels ``[N, 1]`` int64 shifted to 0-based, a
  train/validation split, and the training set truncated to a multiple of 96
  so that 1/2/4/8/12-way data parallel runs see identical global batches
  (reference: src/motion/processor.py:16-119).  Deviation (documented): the
  split permutation is seeded (``seed`` argument) instead of unseeded.
* ``synthetic_motion`` -- no network, no dataset download: class-conditional
  multi-channel oscillations with the exact shapes/dtypes of the processed
  UCI-HAR tensors (N_train = 6912 by default = the reference's truncated size).
"""
from __future__ import annotations

import logging
import math
from pathlib import Path
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch.utils import data

PathLike = Union[str, Path]

SIGNALS = (
    "body_acc_x_", "body_acc_y_", "body_acc_z_",
    "body_gyro_x_", "body_gyro_y_", "body_gyro_z_",
    "total_acc_x_", "total_acc_y_", "total_acc_z_",
)
TRAIN_MULTIPLE = 96  # lcm-friendly size for 1, 2, 4, 8, 12, 16, 24, 32, 48, 96 replicas


class MotionDataProcessor:
    """Raw UCI-HAR text -> tensors (see module docstring)."""

    TRAIN = "train"
    TEST = "test"
    INPUT_SIGNAL_TYPES = SIGNALS

    def __init__(self, seed: Optional[int] = None):
        self.seed = seed

    @staticmethod
    def _read_matrix(path: Path, dtype) -> np.ndarray:
        # whitespace separated; np.loadtxt handles the double-space quirk
        return np.loadtxt(path, dtype=dtype, ndmin=2)

    def load_signals(self, base: Path, split: str) -> torch.Tensor:
        chans = [self._read_matrix(base / split / "Inertial Signals" / f"{s}{split}.txt", np.float32)
                 for s in SIGNALS]
        stacked = np.stack(chans, axis=-1)  # [N, 128, 9]
        return torch.from_numpy(np.ascontiguousarray(stacked))

    def load_labels(self, path: Path) -> torch.Tensor:
        y = self._read_matrix(path, np.int64)
        return torch.from_numpy(y - 1)

    def split(self, x: torch.Tensor, y: torch.Tensor, validation_fraction: float):
        n = x.shape[0]
        rng = np.random.default_rng(self.seed) if self.seed is not None else np.random.default_rng()
        perm = torch.from_numpy(rng.permutation(n))
        n_val = int(n * validation_fraction)
        val_idx, train_idx = perm[:n_val], perm[n_val:]
        return (x[train_idx], y[train_idx]), (x[val_idx], y[val_idx])

    def process_data(self, csv_path: PathLike, validation_fraction: float = 0.05):
        base = Path(csv_path)
        x_train = self.load_signals(base, self.TRAIN)
        x_test = self.load_signals(base, self.TEST)
        y_train = self.load_labels(base / self.TRAIN / "y_train.txt")
        y_test = self.load_labels(base / self.TEST / "y_test.txt")
        (xt, yt), valid = self.split(x_train, y_train, validation_fraction)
        keep = (xt.shape[0] // TRAIN_MULTIPLE) * TRAIN_MULTIPLE
        return (xt[:keep], yt[:keep]), valid, (x_test, y_test)


class MotionDataset(data.Dataset):
    LABELS = [
        "WALKING",
        "WALKING_UPSTAIRS",
        "WALKING_DOWNSTAIRS",
        "SITTING",
        "STANDING",
        "LAYING",
    ]
    SPLITS = ("train", "validation", "test")

    def __init__(self, features: torch.Tensor, labels: torch.Tensor):
        self.features = features
        self.labels = labels
        self.seq_length = features.shape[1]
        self.num_features = features.shape[2]

    def __getitem__(self, index):
        return self.features[index], self.labels[index]

    def __len__(self):
        return len(self.features)

    def to(self, device) -> "MotionDataset":
        return MotionDataset(self.features.to(device), self.labels.to(device))

    def random_split(self, validation_fraction: float):
        n_val = int(len(self) * validation_fraction)
        return data.random_split(self, [len(self) - n_val, n_val])

    @staticmethod
    def get_data_path(base_path: PathLike, data_type: str) -> Tuple[Path, Path]:
        base = Path(base_path)
        return base / f"X_{data_type}.pt", base / f"y_{data_type}.pt"

    @staticmethod
    def processed_data_exists(paths: Sequence[Path]) -> bool:
        return all(Path(p).exists() for p in paths)

    @classmethod
    def load(cls, base_path: PathLike, output_path: Optional[PathLike] = None,
             validation_fraction: float = 0.05, seed: Optional[int] = None) -> List["MotionDataset"]:
        """Cached tensors if all three splits exist, else preprocess raw text."""
        base = Path(base_path)
        cached = []
        for split in cls.SPLITS:
            fx, fy = cls.get_data_path(base, split)
            if cls.processed_data_exists([fx, fy]):
                # tensors only: never unpickle arbitrary objects
                cached.append(cls(torch.load(fx, weights_only=True), torch.load(fy, weights_only=True)))
        if len(cached) == 3:
            logging.info("Preprocessed data found. Skip preprocessing.")
            return cached
        if not (base / "train" / "Inertial Signals").exists():
            raise FileNotFoundError(
                f"no processed tensors or raw UCI-HAR data under {base}; "
                "pass --synthetic to train on generated data of the same shape")
        out = Path(output_path) if output_path is not None else base
        out.mkdir(parents=True, exist_ok=True)
        logging.info("No processed data found. Preprocess raw data...")
        splits = MotionDataProcessor(seed).process_data(base, validation_fraction)
        result = []
        for split, (x, y) in zip(cls.SPLITS, splits):
            fx, fy = cls.get_data_path(out, split)
            torch.save(x, fx)
            torch.save(y, fy)
            result.append(cls(x, y))
        return result


def synthetic_motion(n_train: int = 6912, n_validation: int = 384, n_test: int = 2947,
                     seq_length: int = 128, num_features: int = 9, num_classes: int = 6,
                     seed: int = 0) -> List[MotionDataset]:
    """Learnable synthetic stand-in for UCI-HAR (same shapes and dtypes).

    Each class has its own base frequency / phase pattern per channel; samples
    add amplitude jitter and Gaussian noise, so an LSTM can learn to separate
    them but not trivially."""
    g = torch.Generator().manual_seed(seed)
    t = torch.arange(seq_length, dtype=torch.float32) / seq_length
    freq = 1.0 + torch.rand(num_classes, num_features, generator=g) * 6.0
    phase = torch.rand(num_classes, num_features, generator=g) * 2 * math.pi
    offset = torch.randn(num_classes, num_features, generator=g) * 0.3

    def make(n: int) -> MotionDataset:
        y = torch.randint(0, num_classes, (n, 1), generator=g)
        c = y[:, 0]
        amp = 0.5 + torch.rand(n, 1, num_features, generator=g)
        sig = torch.sin(2 * math.pi * freq[c].unsqueeze(1) * t.view(1, -1, 1) + phase[c].unsqueeze(1))
        x = amp * sig + offset[c].unsqueeze(1) + 0.4 * torch.randn(n, seq_length, num_features, generator=g)
        return MotionDataset(x.float().contiguous(), y.long())

    return [make(n_train), make(n_validation), make(n_test)]
