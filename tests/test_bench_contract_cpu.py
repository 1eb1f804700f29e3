"""bench.py driver contract at world size 2 (gloo on the CPU): the launch the
driver uses for N>1 (torch.distributed.run, one rank per device) prints ONE
JSON line from rank 0 with the whole-job value and the dp degree."""
import json
import os

from _mp import ROOT, torchrun


def test_bench_two_ranks_json_contract(tmp_path):
    out = torchrun([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1"], 2,
                   str(tmp_path), timeout=300)
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 1440
    assert d["config"]["per_gpu_batch"] == 720 and d["scaling"] == "strong"
    assert d["value"] > 0 and abs(d["value"] - 1440 * 2 / (d["ms_per_step"] * 2e-3)) / d["value"] < 1e-2
    assert d["vs_baseline"] == round(d["value"] / 85.9, 2)
    assert d["final_loss"] == d["final_loss"]
