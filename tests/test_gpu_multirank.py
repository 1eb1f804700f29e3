"""World > 1 on the GPU path, rehearsed on one MI355X: two ranks share cuda:0
over the gloo backend (RCCL refuses two ranks on one device; the driver's
8-GPU run covers RCCL with distinct devices).  This exercises the fused
multi-rank step the 2/4/8-GPU benchmark runs -- fused LSTM forward + BPTT on
each rank's shard, gradient all-reduce through the native communicator,
flat Adam -- and checks the reference's correctness oracle: the
mean over ranks of the per-step loss equals the single-process loss."""
import os
import sys

import pytest

from _mp import ROOT, batch_losses, free_port, run

pytestmark = pytest.mark.gpu

MAIN = os.path.join(ROOT, "src", "motion", "main.py")
COMMON = ["--seed", "1", "--epochs", "1", "--batch-size", "480", "--no-validation", "--synthetic",
          "--synthetic-size", "960", "--log-interval", "1"]


def _gpu_env(extra=None):
    env = dict(os.environ)
    env.update({"MASTER_ADDR": "127.0.0.1", "OMP_NUM_THREADS": "1",
                "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "PDRNN_FORCE_CPU"):
        env.pop(k, None)
    env.update(extra or {})
    return env


@pytest.mark.parametrize("mode,hidden,cell", [("distributed", 32, "lstm"), ("horovod", 32, "lstm"),
                                              ("distributed", 128, "lstm"), ("distributed", 32, "gru")])
def test_two_ranks_one_gpu_match_single_process(tmp_path, mode, hidden, cell):
    """hidden 128: the fp32 large-H path (row-owning kernels, stacked-layer
    chunk pipeline on per-layer streams) under the DDP gradient hooks, with
    the weight gradients written into the flat views (ops/gradsink.py); gru:
    the GRU on the sequence-in-wave kernels at world 2."""
    common = COMMON + ["--hidden-units", str(hidden), "--cell", cell]
    local = batch_losses(run([sys.executable, MAIN] + common + ["local"], cwd=str(tmp_path), env=_gpu_env(),
                             timeout=110))[0]
    out = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
               "--master-addr=127.0.0.1", f"--master-port={free_port()}", MAIN] + common + [mode],
              cwd=str(tmp_path), env=_gpu_env({"PDRNN_BACKEND": "gloo"}), timeout=110)
    per = batch_losses(out)
    assert sorted(per) == [0, 1] and len(per[0]) == len(local) == 2
    mean = [(a + b) / 2 for a, b in zip(per[0], per[1])]
    for a, b in zip(mean, local):
        assert abs(a - b) < 1e-5, (mean, local)


def test_two_rank_deferred_persist_verification(tmp_path):
    """Multi-rank per-step verification of the persistent recurrence without a
    host sync (train/lm.py settle, bindings.cpp persist_sticky_flag): rank 0's
    first persistent launch is flagged as timed out; the MAX all-reduce of
    the sticky flag makes BOTH ranks skip their Adam launches on the device
    and re-run the skipped steps on the per-step kernels, so both ranks count
    one fallback and end with the parameters of a run that never took the
    persistent path (PDRNN_LSTM_PERSIST=0)."""
    import json
    worker = os.path.join(ROOT, "tests", "_lm_verify_worker.py")

    def job(extra):
        for r in (0, 1):
            (tmp_path / f"verify_rank{r}.json").unlink(missing_ok=True)
        run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
             "--master-addr=127.0.0.1", f"--master-port={free_port()}", worker],
            cwd=str(tmp_path), env=_gpu_env(extra), timeout=150)
        recs = [json.loads((tmp_path / f"verify_rank{r}.json").read_text()) for r in (0, 1)
                if (tmp_path / f"verify_rank{r}.json").exists()]
        return {r["rank"]: r for r in recs}

    got = job({"PDRNN_TEST_INJECT_RANK": "0"})
    ref = job({"PDRNN_LSTM_PERSIST": "0"})
    assert sorted(got) == [0, 1] and sorted(ref) == [0, 1]
    for r in (0, 1):
        assert got[r]["verify"] == 2, got[r]
        assert got[r]["fallbacks"] == 1 and got[r]["disabled"], got[r]
        assert ref[r]["fallbacks"] == 0, ref[r]
    assert got[0]["checksum"] == got[1]["checksum"]
    for r in (0, 1):
        assert abs(got[r]["checksum"] - ref[r]["checksum"]) <= 1e-6 * ref[r]["abs"], (got[r], ref[r])
        for a, b in zip(got[r]["losses"], ref[r]["losses"]):
            assert abs(a - b) < 1e-4, (got[r]["losses"], ref[r]["losses"])



def test_two_rank_motion_persist_verification(tmp_path):
    """the motion DDP trainer does not carry the LM
    trainer's skip word, so multi-rank jobs keep per-launch verification
    (mode 1): a timed-out persistent backward (fp32 H = 256) is re-run on the
    per-step kernels before its gradient is all-reduced.  Rank 0's first
    persistent launch is flagged as timed out; both ranks end with the
    parameters of a run that never took the persistent path."""
    import json
    worker = os.path.join(ROOT, "tests", "_motion_verify_worker.py")

    def job(extra):
        for r in (0, 1):
            (tmp_path / f"mverify_rank{r}.json").unlink(missing_ok=True)
        run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
             "--master-addr=127.0.0.1", f"--master-port={free_port()}", worker],
            cwd=str(tmp_path), env=_gpu_env(extra), timeout=150)
        recs = [json.loads((tmp_path / f"mverify_rank{r}.json").read_text()) for r in (0, 1)
                if (tmp_path / f"mverify_rank{r}.json").exists()]
        return {r["rank"]: r for r in recs}

    got = job({"PDRNN_TEST_INJECT_RANK": "0"})
    ref = job({"PDRNN_LSTM_PERSIST": "0"})
    assert sorted(got) == [0, 1] and sorted(ref) == [0, 1]
    assert got[0]["verify"] == 1 and got[1]["verify"] == 1, got
    assert got[0]["fallbacks"] == 1 and got[1]["fallbacks"] == 0, got
    assert got[0]["checksum"] == got[1]["checksum"]
    for r in (0, 1):
        assert abs(got[r]["checksum"] - ref[r]["checksum"]) <= 1e-5 * ref[r]["abs"], (got[r], ref[r])
        for a, b in zip(got[r]["losses"], ref[r]["losses"]):
            assert abs(a - b) < 1e-4, (got[r]["losses"], ref[r]["losses"])
