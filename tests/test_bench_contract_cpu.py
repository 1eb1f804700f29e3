"""bench.py driver contract at world size 2 (gloo on the CPU): the launch the
driver uses for N>1 (torch.distributed.run, one rank per device) prints ONE
JSON line from rank 0 with the whole-job value and the dp degree."""
import json
import os

import pytest

from _mp import ROOT, torchrun


@pytest.mark.parametrize("world,baseline", [(2, 85.9), (8, 213.3)])
def test_bench_multi_rank_json_contract(tmp_path, world, baseline):
    """world 8: the driver's N=8 scaling launch, rehearsed on gloo."""
    out = torchrun([os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "5", "--warmup", "1"], world,
                   str(tmp_path), timeout=600)
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 5 and d["warmup"] == 1
    assert d["config"]["parallelism"] == f"dp{world}" and d["config"]["global_batch"] == 1440
    assert d["config"]["per_gpu_batch"] == 1440 // world and d["scaling"] == "strong"
    # the headline is the reference's metric: whole epochs (the short last
    # batch included) of epoch_sequences each, over the timed wall time
    assert d["steps_per_epoch"] == 5 and d["epochs"] == 1.0 and d["epoch_sequences"] == 6912
    assert d["timed_sequences"] == 6912 * d["epochs"]
    assert d["value"] > 0 and abs(d["value"] - d["epoch_sequences"] * d["epochs"] /
                                  (d["epoch_time_s"] * d["epochs"])) / d["value"] < 1e-3
    assert abs(d["value"] - d["timed_sequences"] / (d["ms_per_step"] * 5e-3)) / d["value"] < 1e-2
    assert d["step_seq_per_s"] > 0
    assert d["vs_baseline"] == round(d["value"] / baseline, 2)
    assert d["final_loss"] == d["final_loss"]
