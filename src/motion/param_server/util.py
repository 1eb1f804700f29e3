"""``param_server.util`` compatibility."""
from pytorch_distributed_rnn_amd.parallel.param_server import call_method, remote_method  # noqa: F401
