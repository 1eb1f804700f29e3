"""GPU: parameter-server mode (reference hot path:
src/motion/param_server/worker.py:46,52,91-94): the server's model runs on
the HIP kernels of the box's GPU, both trainers step it through RPC +
distributed autograd, and the loss goes down."""
import os
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _mp import ROOT, batch_losses, free_port  # noqa: E402

pytestmark = pytest.mark.gpu

MAIN = os.path.join(ROOT, "src", "motion", "main.py")


@pytest.mark.parametrize("payload", ["rpc", "collective"])
def test_parameter_server_gpu_loss_decreases(tmp_path, payload):
    # collective on a one-GPU box: the {server, trainer} groups are gloo
    # (RCCL needs one GPU per rank), the server's model is on the GPU
    port = str(free_port())
    common = ["--seed", "1", "--epochs", "4", "--batch-size", "96", "--no-validation", "--synthetic",
              "--synthetic-size", "384", "--log-interval", "1", "parameter-server", "--world-size", "3",
              "--master-address", "127.0.0.1", "--master-port", port, "--ps-payload", payload]
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    procs = [subprocess.Popen([sys.executable, MAIN] + common + ["--rank", str(r)], cwd=str(tmp_path),
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(3)]
    outs = []
    try:
        for p in procs:
            try:
                outs.append(p.communicate(timeout=90)[0])
            except subprocess.TimeoutExpired:
                for q in procs:
                    if q.poll() is None:
                        q.kill()
                outs = [q.communicate()[0] for q in procs]
                raise AssertionError("PS run timed out:\n" + "\n=====\n".join(
                    "\n".join(ln for ln in o.splitlines() if "frame #" not in ln)[-4000:] for o in outs))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-2500:] for o in outs)
    per = batch_losses("\n".join(outs))
    assert set(per) == {1, 2}, per  # both trainers stepped
    for r, losses in per.items():
        assert all(x == x for x in losses)
        k = max(1, len(losses) // 4)
        assert sum(losses[-k:]) / k < sum(losses[:k]) / k, (r, losses)  # learning on the server
    if payload == "collective":
        # the server stepped every trainer's update on the native flat Adam
        # (adam_flat_kernel over the flattened server model)
        import re
        m = re.search(r"Server optimizer steps on the native flat Adam: (\d+)", outs[0])
        assert m and int(m.group(1)) == sum(len(v) for v in per.values()), outs[0][-2000:]
