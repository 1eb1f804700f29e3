#!/usr/bin/env python
"""Shim for the path the reference README cites (``src/example_ddp.py``);
the example lives in ``src/example/example_ddp.py``."""
import os
import runpy
import sys

_HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "example")
sys.path.insert(0, _HERE)
if __name__ == "__main__":
    runpy.run_path(os.path.join(_HERE, "example_ddp.py"), run_name="__main__")
