#!/usr/bin/env python
"""Motion-classification training entry point (CLI-compatible with the
reference ``src/motion/main.py``); implementation in
``pytorch_distributed_rnn_amd.cli``."""
import sys
from pathlib import Path

import _bootstrap  # noqa: F401

from pytorch_distributed_rnn_amd.cli import main

SCRIPT_DIR = Path(__file__).absolute().parent

if __name__ == "__main__":
    sys.dont_write_bytecode = True
    main(script_dir=SCRIPT_DIR)
