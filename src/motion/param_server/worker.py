"""``param_server.worker`` compatibility."""
from pytorch_distributed_rnn_amd.parallel.param_server import (  # noqa: F401
    RemoteModel as WorkerNetwork, run_worker)
