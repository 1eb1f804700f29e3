"""``from model import MotionModel`` compatibility (reference src/motion/model.py)."""
import _bootstrap  # noqa: F401

from pytorch_distributed_rnn_amd.models.motion import MotionModel  # noqa: F401
