"""Benchmark harness (fabfile.py counterpart) and report (notebook counterpart)."""
import json
import os
import sys

from _mp import ROOT, run

sys.path.insert(0, os.path.join(ROOT, "bench"))
import report  # noqa: E402
import runner  # noqa: E402


def test_matrix_matches_reference_shape():
    cfgs = runner.matrix([480, 960, 1440], [1, 2, 4, 8], runner.TRAINERS, [0])
    # local only at one GPU: 3 batches x (1 local + 4 distributed + 4 horovod)
    assert len(cfgs) == 27
    assert all(c["parameters"]["--seed"] == 123456789 for c in cfgs)


def test_runner_resume_and_report(tmp_path):
    res = tmp_path / "m.jsonl"
    args = ["python", os.path.join(ROOT, "bench", "runner.py"), "--results", str(res), "--device", "cpu",
            "--batches", "96", "--gpus", "1", "2", "--trainers", "local", "distributed",
            "--extra", "--synthetic-size 192 --hidden-units 8"]
    run(args, cwd=str(tmp_path), timeout=400)
    recs = [json.loads(l) for l in res.read_text().splitlines()]
    assert len(recs) == 3 and all(r["returncode"] == 0 for r in recs)
    out = run(args, cwd=str(tmp_path))  # resume: nothing left to do
    assert out.count("[skip]") == 3
    rows = report.aggregate([res])
    assert set(rows) == {("local", 1, 96), ("distributed", 1, 96), ("distributed", 2, 96)}
    assert all(v["seq_per_s"] > 0 for v in rows.values())


def test_report_reproduces_baseline_table():
    ev = "/root/reference/evaluation"
    files = [os.path.join(ev, f) for f in ("results_202007141530.json", "results_202007141730.json")]
    if not all(os.path.exists(f) for f in files):
        import pytest
        pytest.skip("reference result files not mounted")
    rows = report.aggregate(files)
    # BASELINE.md dedup table: DDP bs1440 44.8 / 85.9 / 128.5 / 213.3 seq/s
    got = [round(rows[("distributed", n, 1440)]["seq_per_s"], 1) for n in (1, 2, 4, 8)]
    assert got == [44.8, 85.9, 128.5, 213.3]


def test_report_reproduces_baseline_network_rows(tmp_path):
    """the network notebook's numbers (BASELINE.md 'Other
    recorded numbers') from the reference's netem result files, and the
    figures written."""
    import pytest
    ev = "/root/reference/evaluation"
    files = [os.path.join(ev, f) for f in ("results_network_202007211500.json", "results_network_202007211630.json")]
    if not all(os.path.exists(f) for f in files):
        pytest.skip("reference result files not mounted")
    rows = report.aggregate_network(files)

    def row(tr, rt, vals):
        return [round(rows[(tr, 12, rt, float(v))]["duration_s"], 1) for v in vals]
    assert row("distributed", "delay", (0, 10, 50, 100, 200, 400)) == [25.7, 26.9, 29.0, 35.7, 47.9, 72.0]
    assert row("horovod", "delay", (0, 10, 50, 100, 200, 400)) == [61.4, 88.4, 102.8, 107.5, 126.5, 175.7]
    assert row("distributed", "loss", (0, 1, 5, 10)) == [24.4, 24.6, 24.1, 30.1]
    assert row("horovod", "loss", (0, 1, 5, 10, 15)) == [50.1, 71.0, 91.6, 99.8, 132.0]
    # a runner --fault record parses into the same keys
    rec = {"config": {"trainer": "distributed", "gpus": 2, "fault_delay_ms": 50, "parameters": {}},
           "stderr": "INFO:root:0: Memory Usage: 12.5, Training Duration: 1.25\n"}
    assert report.parse_network(rec) == ("distributed", 2, "delay", 50.0, 1.25)
    written = report.plot({}, {}, {}, rows, tmp_path / "plots", "x")
    assert {p.name for p in written} >= {"delay_sweep.png", "loss_sweep.svg"}
