"""``param_server.master`` compatibility."""
from pytorch_distributed_rnn_amd.parallel.param_server import (  # noqa: F401
    ServerModel as MasterNetwork, get_parameter_network, run_parameter_server)
