"""``from dataset import MotionDataset`` compatibility (reference src/motion/dataset.py)."""
import _bootstrap  # noqa: F401

from pytorch_distributed_rnn_amd.data.motion import MotionDataset, synthetic_motion  # noqa: F401
