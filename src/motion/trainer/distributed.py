"""``trainer.distributed.DistributedTrainer`` compatibility."""
from pytorch_distributed_rnn_amd.train.distributed import DistributedTrainer  # noqa: F401
