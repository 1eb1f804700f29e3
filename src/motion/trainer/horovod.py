"""``trainer.horovod.HorovodTrainer`` compatibility."""
from pytorch_distributed_rnn_amd.train.distributed import HorovodTrainer  # noqa: F401
