"""``param_server`` subcommand compatibility (reference src/motion/param_server/__init__.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _bootstrap  # noqa: E402,F401

from pytorch_distributed_rnn_amd.parallel.param_server import add_sub_command, execute  # noqa: E402,F401
