"""``trainer.base.Trainer`` compatibility."""
from pytorch_distributed_rnn_amd.train.trainer import Trainer  # noqa: F401
