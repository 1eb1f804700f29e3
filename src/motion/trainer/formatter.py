"""``trainer.formatter`` compatibility."""
from pytorch_distributed_rnn_amd.train.formatter import TrainingMessageFormatter, percentage  # noqa: F401
