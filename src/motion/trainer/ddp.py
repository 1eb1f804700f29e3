"""``trainer.ddp.DDPTrainer`` compatibility."""
from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer  # noqa: F401
