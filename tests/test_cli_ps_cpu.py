"""CLI entry point (reference: src/motion/main.py:15-43, trainer/__init__.py:44-60)
and parameter-server liveness (reference: src/motion/param_server/*)."""
import json
import os
import re
import subprocess
import sys

from _mp import ROOT, batch_losses, cpu_env, free_port, run

MAIN = os.path.join(ROOT, "src", "motion", "main.py")


def test_local_cli_log_contract_and_history(tmp_path):
    out = run([sys.executable, MAIN, "--seed", "3", "--epochs", "2", "--batch-size", "192", "--synthetic",
               "--synthetic-size", "384", "--device", "cpu", "--hidden-units", "8",
               "--checkpoint-directory", str(tmp_path / "models"), "local"], cwd=str(tmp_path))
    assert re.search(r"0: Memory Usage: [\d.]+, Training Duration: [\d.]+", out)
    assert "Rank: 00   Start Epoch 0" in out and "Rank: 00   Start Epoch 1" in out
    assert "Evaluation Epoch: 1/2 (50%)" in out and "Test Evaluation:" in out
    assert len(batch_losses(out)[0]) == 4
    hist = json.load(open(tmp_path / "history.json"))
    assert len(hist["train_history"]) == 2 and len(hist["validation_history"]) == 2
    assert (tmp_path / "models" / "best-model.pt").exists()


def test_seed_reproducible(tmp_path):
    args = [sys.executable, MAIN, "--seed", "7", "--epochs", "1", "--batch-size", "96", "--no-validation",
            "--synthetic", "--synthetic-size", "192", "--device", "cpu", "--hidden-units", "8",
            "--log-interval", "1", "local"]
    a = batch_losses(run(args, cwd=str(tmp_path)))[0]
    b = batch_losses(run(args, cwd=str(tmp_path)))[0]
    assert a == b and len(a) == 2


def test_mpirun_style_rank_discovery(tmp_path):
    # one process "launched by mpirun": OMPI_* variables only, no torchrun env
    env = cpu_env({"OMPI_COMM_WORLD_RANK": "0", "OMPI_COMM_WORLD_SIZE": "1",
                   "OMPI_COMM_WORLD_LOCAL_RANK": "0", "MASTER_PORT": str(free_port())})
    out = run([sys.executable, MAIN, "--seed", "1", "--epochs", "1", "--batch-size", "96", "--no-validation",
               "--synthetic", "--synthetic-size", "96", "--device", "cpu", "--hidden-units", "8",
               "distributed"], cwd=str(tmp_path), env=env)
    assert "0: Memory Usage:" in out


def test_parameter_server_liveness(tmp_path):
    port = str(free_port())
    common = ["--seed", "1", "--epochs", "1", "--batch-size", "96", "--no-validation", "--synthetic",
              "--synthetic-size", "192", "--device", "cpu", "--hidden-units", "8", "parameter-server",
              "--world-size", "3", "--master-address", "127.0.0.1", "--master-port", port]
    procs = [subprocess.Popen([sys.executable, MAIN] + common + ["--rank", str(r)], cwd=str(tmp_path),
                              env=cpu_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(3)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-2000:] for o in outs)
    log = "\n".join(outs)
    per = batch_losses(log)
    assert set(per) == {1, 2}  # both trainers stepped
    assert all(x == x and x < 10 for v in per.values() for x in v)  # finite losses


def test_parameter_server_collective_payloads(tmp_path):
    """RPC as control plane, batch/logits/logit-gradient over {server, trainer}
    send/recv groups (gloo here; RCCL when every rank owns a GPU): both
    trainers step the server's model and its loss goes down."""
    port = str(free_port())
    common = ["--seed", "1", "--epochs", "4", "--batch-size", "96", "--no-validation", "--synthetic",
              "--synthetic-size", "384", "--device", "cpu", "--hidden-units", "8", "--log-interval", "1",
              "parameter-server", "--world-size", "3", "--master-address", "127.0.0.1", "--master-port", port,
              "--ps-payload", "collective"]
    procs = [subprocess.Popen([sys.executable, MAIN] + common + ["--rank", str(r)], cwd=str(tmp_path),
                              env=cpu_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(3)]
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-2000:] for o in outs)
    assert "Payload groups initialized (gloo)" in outs[0]
    per = batch_losses("\n".join(outs))
    assert set(per) == {1, 2}, per
    for r, losses in per.items():
        assert all(x == x for x in losses)
        k = max(1, len(losses) // 4)
        assert sum(losses[-k:]) / k < sum(losses[:k]) / k, (r, losses)
