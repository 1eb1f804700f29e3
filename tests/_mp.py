"""Helpers for multi-process (torchrun, gloo) tests on the CPU."""
from __future__ import annotations

import os
import re
import socket
import subprocess
import sys
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def cpu_env(extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ)
    env.update({"MASTER_ADDR": "127.0.0.1", "PDRNN_FORCE_CPU": "1", "OMP_NUM_THREADS": "1",
                "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", ""),
                "HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    if extra:
        env.update(extra)
    return env


def run(cmd: List[str], cwd: str, timeout: float = 240, env=None) -> str:
    p = subprocess.run(cmd, cwd=cwd, env=env or cpu_env(), capture_output=True, text=True, timeout=timeout)
    out = p.stdout + p.stderr
    if p.returncode != 0:
        raise AssertionError(f"{' '.join(cmd)} failed ({p.returncode}):\n{out[-4000:]}")
    return out


def torchrun(script_and_args: List[str], nproc: int, cwd: str, timeout: float = 240, env=None) -> str:
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}"] + script_and_args
    return run(cmd, cwd, timeout, env)


_BATCH = re.compile(r"Rank: (\d+)\s+Train Batch: (\d+)/(\d+) \(\d+%\)\tLoss: ([\d.]+)\tAcc: (\d+)/(\d+)")


def batch_losses(log: str) -> Dict[int, List[float]]:
    """rank -> per-step losses parsed from the reference-format Train Batch lines."""
    out: Dict[int, List[float]] = {}
    for m in _BATCH.finditer(log):
        out.setdefault(int(m.group(1)), []).append(float(m.group(4)))
    return out
