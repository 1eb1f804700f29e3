"""Distributed strategies: DDP (native bucketed reducer), Horovod-style
optimizer wrapping (tensor fusion), parameter server (RPC), plus process
discovery and the native RCCL communicator."""
from .env import (ProcessInfo, barrier, discover, get_rank, get_world_size,  # noqa: F401
                  init_distributed, is_distributed, setup_device, shutdown)
