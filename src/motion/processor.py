"""``from processor import MotionDataProcessor`` compatibility (reference src/motion/processor.py)."""
import _bootstrap  # noqa: F401

from pytorch_distributed_rnn_amd.data.motion import MotionDataProcessor  # noqa: F401
