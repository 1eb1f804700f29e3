#!/usr/bin/env python
"""Benchmark matrix runner -- the MI355X counterpart of the reference's
fabfile.py harness (reference: fabfile.py:48-66 TRAIN_RUNS, 194-235 command
builder, 240-290 resumable runner, 125-191 netem sweep).

* Matrix: batch {480, 960, 1440} x GPUs {1, 2, 4, 8} x trainer {local,
  distributed, horovod}; ``local`` only at 1 GPU; ``--epochs 1 --seed
  123456789 --no-validation`` like the reference.  ``--fault`` adds the
  network-fault sweep (host-side delay per step and retransmission stalls on
  a share of the syncs, the netem delay / loss stand-ins: xGMI cannot be
  netem'd; see pytorch_distributed_rnn_amd/utils/faults.py).
* Launcher: one process per GPU via ``torch.distributed.run`` on 127.0.0.1
  (replaces mpirun/horovodrun over ssh); ``--launcher mpirun`` emits
  ``mpirun -np N`` lines instead (ranks come from OMPI_* variables).
* Results: JSON Lines, one object per run ``{command, stdout, stderr, config,
  returncode, wall_s}`` -- the reference's per-run record plus exit status.
  Runs whose command is already in the file are skipped (resume), the order
  is shuffled with a fixed seed (reference: fabfile.py:258,270-276).

    python bench/runner.py --results results/matrix.jsonl            # real run
    python bench/runner.py --dry-run                                  # print commands
    python bench/runner.py --device cpu --batches 96 --gpus 1 2 ...   # CPU plumbing
"""
from __future__ import annotations

import argparse
import json
import os
import random
import shlex
import socket
import subprocess
import sys
import time
from pathlib import Path
from typing import Dict, Iterable, List

ROOT = Path(__file__).resolve().parent.parent
MAIN = ROOT / "src" / "motion" / "main.py"
TRAINERS = ("local", "distributed", "horovod")


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def matrix(batches: Iterable[int], gpus: Iterable[int], trainers: Iterable[str],
           delays: Iterable[float], losses: Iterable[float] = (0,)) -> List[Dict]:
    """Configurations; the fault sweeps vary one knob at a time like the
    reference's (delay rules with no loss, loss rules with no delay)."""
    faults = [(d, 0) for d in delays] + [(0, l) for l in losses if l]
    out = []
    for b in batches:
        for n in gpus:
            for tr in trainers:
                if tr == "local" and n != 1:
                    continue
                for d, l in faults:
                    if tr == "local" and (d or l):
                        continue
                    cfg = {"trainer": tr, "hosts": 1, "gpus": n, "slots": n, "fault_delay_ms": d,
                           "parameters": {"--batch-size": b, "--epochs": 1, "--seed": 123456789,
                                          "--no-validation": ""}}
                    if l:
                        cfg["fault_loss_pct"] = l
                    out.append(cfg)
    return out


def command(cfg: Dict, launcher: str, extra: List[str]) -> List[str]:
    params: List[str] = []
    for k, v in cfg["parameters"].items():
        params += [k] + ([str(v)] if v != "" else [])
    if cfg.get("fault_delay_ms"):
        params += ["--fault-delay-ms", str(cfg["fault_delay_ms"])]
    if cfg.get("fault_loss_pct"):
        params += ["--fault-loss", str(cfg["fault_loss_pct"])]
    params += extra
    if cfg["trainer"] == "local":
        return [sys.executable, str(MAIN)] + params + ["local"]
    n = cfg["gpus"]
    if launcher == "mpirun":
        pre = ["mpirun", "--bind-to", "none", "--map-by", "slot", "-np", str(n), sys.executable]
    else:
        pre = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr=127.0.0.1", f"--master-port={free_port()}"]
    return pre + [str(MAIN)] + params + [cfg["trainer"]]


def key(cfg: Dict) -> str:
    return json.dumps({k: cfg.get(k) for k in ("trainer", "gpus", "fault_delay_ms", "fault_loss_pct", "parameters")},
                      sort_keys=True)


def done_keys(path: Path) -> set:
    keys = set()
    if path.exists():
        for line in path.read_text().splitlines():
            try:
                keys.add(key(json.loads(line)["config"]))
            except (ValueError, KeyError):
                pass
    return keys


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--results", type=Path, default=ROOT / "results" / "matrix.jsonl")
    ap.add_argument("--batches", type=int, nargs="+", default=[480, 960, 1440])
    ap.add_argument("--gpus", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--trainers", nargs="+", default=list(TRAINERS), choices=TRAINERS)
    ap.add_argument("--fault", action="store_true",
                    help="the reference's network sweep: delay 0/1/2/5/10/25/50/100/200/300/400 ms, "
                         "loss 0.1/0.5/1/2/5/10/15 %% (reference fabfile.py:125-183)")
    ap.add_argument("--delays", type=float, nargs="+", default=None)
    ap.add_argument("--losses", type=float, nargs="+", default=None)
    ap.add_argument("--launcher", choices=("torchrun", "mpirun"), default="torchrun")
    ap.add_argument("--device", default=None, help="cpu: gloo plumbing run")
    ap.add_argument("--synthetic", action="store_true", default=True)
    ap.add_argument("--extra", default="", help="extra global flags for main.py")
    ap.add_argument("--timeout", type=float, default=3600)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    delays = a.delays if a.delays is not None else \
        ([0, 1, 2, 5, 10, 25, 50, 100, 200, 300, 400] if a.fault else [0])
    losses = a.losses if a.losses is not None else ([0.1, 0.5, 1, 2, 5, 10, 15] if a.fault else [])
    cfgs = matrix(a.batches, a.gpus, a.trainers, delays, losses)
    random.Random(a.seed).shuffle(cfgs)
    extra = shlex.split(a.extra)
    if a.synthetic:
        extra.append("--synthetic")
    if a.device:
        extra += ["--device", a.device]
    skip = done_keys(a.results)
    a.results.parent.mkdir(parents=True, exist_ok=True)
    for cfg in cfgs:
        cmd = command(cfg, a.launcher, extra)
        if key(cfg) in skip:
            print(f"[skip] {shlex.join(cmd)}")
            continue
        if a.dry_run:
            print(shlex.join(cmd))
            continue
        print(f"[run] {shlex.join(cmd)}", flush=True)
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        t0 = time.perf_counter()
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=str(ROOT), env=env)
            rc, so, se = p.returncode, p.stdout, p.stderr
        except subprocess.TimeoutExpired as e:
            rc, so, se = 124, (e.stdout or b"").decode() if isinstance(e.stdout, bytes) else (e.stdout or ""), "timeout"
        rec = {"command": shlex.join(cmd), "stdout": so, "stderr": se, "config": cfg, "returncode": rc,
               "wall_s": round(time.perf_counter() - t0, 3)}
        with open(a.results, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
