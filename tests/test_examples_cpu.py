"""src/example/* on gloo (BASELINE config 1: example_ddp world_size=2 on CPU).

Pass criterion from the reference README: final parameters equal on all ranks
(reference: README.md:9, src/example/example_ddp.py:84-92)."""
import json
import os

import pytest

from _mp import ROOT, run, torchrun

EX = os.path.join(ROOT, "src", "example")


def _results(tmp_path, world):
    return [json.load(open(tmp_path / f"res.json.{r}")) for r in range(world)]


def test_example_single(tmp_path):
    out = run(["python", os.path.join(EX, "example_single.py")], cwd=str(tmp_path))
    assert "loss" in out


def test_example_distributed_p2p(tmp_path):
    out = torchrun([os.path.join(EX, "example_distributed.py"), "--backend", "gloo"], 2, str(tmp_path))
    assert out.count("has data 1.0") == 2


@pytest.mark.parametrize("shard", [False, True])
def test_example_ddp_world2_params_equal(tmp_path, shard):
    args = [os.path.join(ROOT, "src", "example_ddp.py"), "--backend", "gloo", "--out", str(tmp_path / "res.json")]
    out = torchrun(args + (["--shard"] if shard else []), 2, str(tmp_path))
    r0, r1 = _results(tmp_path, 2)
    assert r0["params"] == r1["params"]
    assert len(r0["losses"]) == (2 if shard else 4)  # 24 samples / (12 // 2) per rank
    assert "param sum before broadcast" in out


def test_example_horovod_world2(tmp_path):
    args = [os.path.join(EX, "example_horovod.py"), "--backend", "gloo", "--out", str(tmp_path / "res.json")]
    torchrun(args, 2, str(tmp_path))
    r0, r1 = _results(tmp_path, 2)
    assert r0["params"] == r1["params"]
