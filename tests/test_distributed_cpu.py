"""Multi-process data parallelism on gloo (CPU).

The reference's implicit correctness oracle: at a fixed global
batch with DistributedSampler sharding, the mean over ranks of the per-step
loss equals the single-process loss (reference logs agree to 5 decimals for
world 1/2/4/8/12, DDP and Horovod).  Checked here for DDP and horovod mode at
world sizes 2 and 4, plus replica consistency (all ranks end with identical
weights in their checkpoints).
"""
import json
import os
import re

import pytest
import torch

from _mp import ROOT, batch_losses, run, torchrun

MAIN = os.path.join(ROOT, "src", "motion", "main.py")
COMMON = ["--seed", "1", "--epochs", "1", "--batch-size", "480", "--no-validation", "--synthetic",
          "--synthetic-size", "960", "--device", "cpu", "--log-interval", "1", "--hidden-units", "16"]


@pytest.fixture(scope="module")
def local_losses(tmp_path_factory):
    d = tmp_path_factory.mktemp("local")
    out = run(["python", MAIN] + COMMON + ["local"], cwd=str(d))
    losses = batch_losses(out)[0]
    assert len(losses) == 2
    return losses


def _rank_mean(log, world):
    per = batch_losses(log)
    assert sorted(per) == list(range(world)), per
    steps = len(per[0])
    return [sum(per[r][s] for r in range(world)) / world for s in range(steps)]


@pytest.mark.parametrize("mode", ["distributed", "horovod"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_world_size_invariance(tmp_path, local_losses, mode, world):
    # world 8 = the driver's scaling node: the same torch.distributed.run
    # launch, rendezvous and per-rank batch split (1440 / 8 = 180 there)
    out = torchrun([MAIN] + COMMON + [mode], nproc=world, cwd=str(tmp_path))
    mean = _rank_mean(out, world)
    assert len(mean) == len(local_losses)
    for a, b in zip(mean, local_losses):
        assert abs(a - b) < 2e-5, (mean, local_losses)
    hist = json.load(open(tmp_path / "history.json"))  # rank 0 only
    assert len(hist["train_history"]) == 1


def test_replicas_stay_identical(tmp_path):
    # every rank checkpoints into its own directory; weights must agree exactly
    script = tmp_path / "replica.py"
    script.write_text(f"""
import sys, torch
sys.path.insert(0, {ROOT!r})
from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
from pytorch_distributed_rnn_amd.models.motion import MotionModel
from pytorch_distributed_rnn_amd.train.distributed import DDPTrainer
torch.manual_seed(int(__import__('os').environ['RANK']))  # different init per rank
train, _, _ = synthetic_motion(n_train=384, n_validation=1, n_test=1, seed=0)
t = DDPTrainer(model=MotionModel(9, 8, 2, 6), training_set=train, batch_size=96, learning_rate=2.5e-3,
               device=torch.device('cpu'), backend='gloo')
t.train(epochs=2)
r = t.rank
torch.save({{k: v for k, v in t.model.module.state_dict().items()}}, {str(tmp_path)!r} + f'/w{{r}}.pt')
""")
    torchrun([str(script)], nproc=2, cwd=str(tmp_path))
    a = torch.load(tmp_path / "w0.pt", weights_only=True)
    b = torch.load(tmp_path / "w1.pt", weights_only=True)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_ddp_checkpoint_has_module_prefix(tmp_path):
    ck_dir = tmp_path / "ck"
    # with validation on, rank 0 evaluates and writes the best model
    torchrun([MAIN, "--checkpoint-directory", str(ck_dir), "--seed", "1", "--epochs", "1",
              "--batch-size", "480", "--synthetic", "--synthetic-size", "960", "--device", "cpu",
              "--hidden-units", "8", "distributed"], nproc=2, cwd=str(tmp_path))
    files = list(ck_dir.iterdir())
    assert files, "rank 0 must checkpoint"
    ck = torch.load(files[0], weights_only=True)
    assert all(k.startswith("module.") for k in ck["model_state"])


def test_rccl_uid_exchange_through_store(tmp_path):
    """The native communicator's unique id goes rank 0 -> every rank through
    the rendezvous TCPStore (no torch collective, so torch's own RCCL
    communicator is never created for it): every rank of a 3-rank group ends
    with rank 0's bytes, and a second communicator gets a fresh key."""
    script = tmp_path / "uid.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch.distributed as dist\n"
        "from pytorch_distributed_rnn_amd.parallel import comm\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "class M:\n"
        "    n = 0\n"
        "    @staticmethod\n"
        "    def rccl_unique_id():\n"
        "        M.n += 1\n"
        "        return bytes([M.n, 7, 0, 255]) * 32\n"
        "a = comm._exchange_uid(M, dist.group.WORLD, r)\n"
        "b = comm._exchange_uid(M, dist.group.WORLD, r)\n"
        "assert a == bytes([1, 7, 0, 255]) * 32 and b == bytes([2, 7, 0, 255]) * 32, (r, a[:4], b[:4])\n"
        "print('uid-ok', r, flush=True)\n"
        "dist.destroy_process_group()\n")
    out = torchrun([str(script)], nproc=3, cwd=str(tmp_path))
    # (the ranks' lines can interleave mid-line on the shared stdout)
    assert sorted(int(r) for r in re.findall(r"uid-ok (\d)", out)) == [0, 1, 2], out


def test_parameter_server_payload_mode_is_agreed(tmp_path):
    """each rank used to pick the PS payload mode from its own GPU
    count.  agree_payload exchanges every rank's answer through a TCPStore,
    so a job whose ranks differ (here rank 2 claims a GPU, the others do not)
    still gets ONE mode and backend everywhere: 'auto' -> rpc, an explicit
    'collective' -> gloo payloads."""
    from _mp import free_port
    script = tmp_path / "agree.py"
    script.write_text(
        "import os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "from pytorch_distributed_rnn_amd.parallel import param_server as ps\n"
        "r, w, port = int(os.environ['RANK']), int(os.environ['WORLD_SIZE']), sys.argv[1]\n"
        "ps._local_gpu_ok = lambda rank, world: rank == 2\n"
        "a = ps.agree_payload('auto', r, w, '127.0.0.1', port, timeout_s=60)\n"
        "b = ps.agree_payload('collective', r, w, '127.0.0.1', str(int(port) + 10), timeout_s=60)\n"
        "c = ps.agree_payload('rpc', r, w, '127.0.0.1', port)\n"
        "open(f'agree{r}.txt', 'w').write(' '.join([a[0], a[1], b[0], b[1], c[0]]))\n")
    torchrun([str(script), str(free_port())], nproc=3, cwd=str(tmp_path))
    for r in range(3):  # one file per rank: stdout lines of the ranks interleave
        assert (tmp_path / f"agree{r}.txt").read_text().split() == ["rpc", "gloo", "collective", "gloo", "rpc"]


def test_ddp_buckets_align_to_layer_direction(tmp_path):
    """GradReducer closes a bucket at every (layer,
    direction) boundary and subdivides a group only above the cap -- no bucket
    mixes two groups; the layout is logged (rank 0) and returned by
    bucket_layout().  Stacked bi-LSTM 2 x 16 + head, world 2 (gloo)."""
    script = tmp_path / "buckets.py"
    script.write_text(
        "import json, logging, os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch\n"
        "from pytorch_distributed_rnn_amd.parallel import env\n"
        "from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel\n"
        "from pytorch_distributed_rnn_amd.models.charlm import BiLSTMEncoder\n"
        "from pytorch_distributed_rnn_amd.utils.flat import flatten_module\n"
        "logging.basicConfig(level=logging.INFO)\n"
        "env.init_distributed('gloo')\n"
        "torch.manual_seed(0)\n"
        "out = {}\n"
        "for cap in (64.0, 0.004):\n"
        "    m = BiLSTMEncoder(8, 16, 2, 4, torch.float32)\n"
        "    flatten_module(m)\n"
        "    d = DistributedDataParallel(m, bucket_cap_mb=cap, first_bucket_cap_mb=cap)\n"
        "    out[str(cap)] = [b['names'] for b in d.bucket_layout()]\n"
        "    x = torch.randn(5, 3, 8)\n"
        "    d(x).sum().backward()\n"
        "    d.finalize() if hasattr(d, 'finalize') else None\n"
        "if env.get_rank() == 0:\n"
        "    open('layout.json', 'w').write(json.dumps(out))\n"
        "env.shutdown()\n")
    log = torchrun([str(script)], nproc=2, cwd=str(tmp_path))
    assert "DDP buckets (launch order)" in log
    layout = json.loads((tmp_path / "layout.json").read_text())

    def key(n):
        leaf = n.rsplit(".", 1)[-1]
        if "_l" in leaf:
            return n.rsplit(".", 1)[0] + leaf[leaf.index("_l"):]
        return n.rsplit(".", 1)[0]
    big = layout["64.0"]
    # one bucket per group, launch order = reverse registration: head, l1_reverse, l1, l0_reverse, l0
    assert [sorted({key(n) for n in b}) for b in big] == [["fc"], ["lstm_l1_reverse"], ["lstm_l1"],
                                                          ["lstm_l0_reverse"], ["lstm_l0"]], big
    small = layout["0.004"]  # 4 KiB cap: groups are split, never mixed
    assert len(small) > len(big)
    assert all(len({key(n) for n in b}) == 1 for b in small), small


def test_ddp_splits_oversized_parameter_across_buckets(tmp_path):
    """a parameter larger than the bucket cap is spread
    over several sub-tensor buckets (512 MiB weight at a 32 MiB cap: 16
    slices) and the all-reduced gradient is still the average of the ranks'
    gradients.  World 2, gloo."""
    script = tmp_path / "split.py"
    script.write_text(
        "import json, os, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch\n"
        "from pytorch_distributed_rnn_amd.parallel import env\n"
        "from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel\n"
        "from pytorch_distributed_rnn_amd.utils.flat import flatten_module\n"
        "env.init_distributed('gloo')\n"
        "rank, world = env.get_rank(), env.get_world_size()\n"
        "torch.manual_seed(0)\n"
        "m = torch.nn.Sequential(torch.nn.Linear(8192, 16384), torch.nn.Linear(16384, 4))\n"
        "flatten_module(m)\n"
        "d = DistributedDataParallel(m, bucket_cap_mb=32, first_bucket_cap_mb=32)\n"
        "lay = d.bucket_layout()\n"
        "def batch(r):\n"
        "    g = torch.Generator().manual_seed(100 + r)\n"
        "    return torch.randn(2, 8192, generator=g)\n"
        "d(batch(rank)).square().sum().backward()\n"
        "w = m[0].weight.grad.clone()\n"
        "ref = torch.zeros_like(w)\n"
        "for r in range(world):\n"
        "    m2 = torch.nn.Sequential(torch.nn.Linear(8192, 16384), torch.nn.Linear(16384, 4))\n"
        "    m2.load_state_dict(m.state_dict())\n"
        "    m2(batch(r)).square().sum().backward()\n"
        "    ref += m2[0].weight.grad / world\n"
        "    del m2\n"
        "err = float((w - ref).abs().max() / ref.abs().max())\n"
        "if rank == 0:\n"
        "    open('split.json', 'w').write(json.dumps({'layout': [{k: b[k] for k in ('names', 'mib') if k in b} |"
        " {'slice': b.get('slice')} for b in lay], 'err': err}))\n"
        "env.shutdown()\n")
    torchrun([str(script)], nproc=2, cwd=str(tmp_path), timeout=600)
    out = json.loads((tmp_path / "split.json").read_text())
    w_buckets = [b for b in out["layout"] if b["names"] == ["0.weight"]]
    assert len(w_buckets) == 16, out["layout"]
    assert all(b["slice"] is not None and b["mib"] <= 32.0 for b in w_buckets)
    spans = sorted(tuple(b["slice"]) for b in w_buckets)
    assert spans[0][0] == 0 and spans[-1][1] == 8192 * 16384
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert out["err"] < 1e-6, out["err"]


def test_ddp_split_uses_regular_cap_behind_first_bucket(tmp_path):
    """a large weight right behind the small head parameters (the
    first bucket still open) is split by the regular bucket cap, not by the
    1 MiB first-bucket cap: 16 MiB at a 4 MiB cap = 4 slices, not 16."""
    script = tmp_path / "split1.py"
    script.write_text(
        "import json, sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch\n"
        "from pytorch_distributed_rnn_amd.parallel import env\n"
        "from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel\n"
        "from pytorch_distributed_rnn_amd.utils.flat import flatten_module\n"
        "env.init_distributed('gloo')\n"
        "m = torch.nn.Sequential(torch.nn.Linear(1024, 4096), torch.nn.Linear(4096, 4))\n"
        "flatten_module(m)\n"
        "d = DistributedDataParallel(m, bucket_cap_mb=4, first_bucket_cap_mb=1)\n"
        "lay = d.bucket_layout()\n"
        "if env.get_rank() == 0:\n"
        "    open('split1.json', 'w').write(json.dumps([b['names'] for b in lay]))\n"
        "env.shutdown()\n")
    torchrun([str(script)], nproc=2, cwd=str(tmp_path), timeout=300)
    names = json.loads((tmp_path / "split1.json").read_text())
    assert sum(1 for n in names if n == ["0.weight"]) == 4, names


def test_allreduce_sweep_tool_world2(tmp_path):
    """bench/allreduce_sweep.py (the bucket-cap measurement) at world 2 on gloo:
    one JSON line per message size from rank 0."""
    import json
    out = torchrun([os.path.join(ROOT, "bench", "allreduce_sweep.py"), "--min-kb", "4", "--max-mb", "0.02",
                    "--iters", "2", "--warmup", "1"], nproc=2, cwd=str(tmp_path))
    rows = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
    assert [r["bytes"] for r in rows] == [4096, 8192, 16384]
    assert all(r["world"] == 2 and r["backend"] == "gloo" and r["us"] > 0 and r["busbw_GBs"] > 0 for r in rows)


def test_direct_grads_under_ddp_and_horovod_match(tmp_path):
    """ops/gradsink.py on multi-rank runs: a Function that
    adds its weight gradients into the flat .grad views itself and returns
    None for them (the pattern of the in-tree Functions) under the
    framework's DDP reducer and Horovod optimizer on 2 gloo ranks: the
    post-accumulate-grad hooks still fire after the view is written, every
    bucket is reduced, and the reduced gradients equal the plain autograd
    path's bit for bit on every rank."""
    script = tmp_path / "direct.py"
    script.write_text(
        "import sys\n"
        f"sys.path.insert(0, {ROOT!r})\n"
        "import torch, torch.distributed as dist\n"
        "from torch import nn\n"
        "from pytorch_distributed_rnn_amd.ops import gradsink\n"
        "from pytorch_distributed_rnn_amd.ops.adam import FusedAdam\n"
        "from pytorch_distributed_rnn_amd.parallel import env, horovod as hvd\n"
        "from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel\n"
        "from pytorch_distributed_rnn_amd.utils.flat import flatten_module\n"
        "class SinkLinear(torch.autograd.Function):\n"
        "    @staticmethod\n"
        "    def forward(ctx, x, w, b):\n"
        "        ctx.save_for_backward(x, w)\n"
        "        ctx.params = (w, b)\n"
        "        ctx.direct = gradsink.enabled()\n"
        "        return x @ w.detach().t() + b.detach()\n"
        "    @staticmethod\n"
        "    def backward(ctx, dy):\n"
        "        x, w = ctx.saved_tensors\n"
        "        dx = dy @ w.detach()\n"
        "        sw, sb = gradsink.sink(ctx.params[0], ctx.direct), gradsink.sink(ctx.params[1], ctx.direct)\n"
        "        if sw is not None and sb is not None:\n"
        "            sw.add_(dy.t() @ x)\n"
        "            sb.add_(dy.sum(0))\n"
        "            return dx, None, None\n"
        "        return dx, dy.t() @ x, dy.sum(0)\n"
        "class Net(nn.Module):\n"
        "    def __init__(self):\n"
        "        super().__init__()\n"
        "        self.a, self.b = nn.Linear(12, 32), nn.Linear(32, 5)\n"
        "    def forward(self, x):\n"
        "        h = torch.tanh(SinkLinear.apply(x, self.a.weight, self.a.bias))\n"
        "        return SinkLinear.apply(h, self.b.weight, self.b.bias)\n"
        "env.init_distributed('gloo')\n"
        "r, W = dist.get_rank(), dist.get_world_size()\n"
        "torch.manual_seed(0)\n"
        "base = Net()\n"
        "gx = torch.Generator().manual_seed(100 + r)\n"
        "xs = [torch.randn(16, 12, generator=gx) for _ in range(3)]\n"
        "def run_ddp(direct):\n"
        "    m = Net(); m.load_state_dict(base.state_dict())\n"
        "    d = DistributedDataParallel(m, bucket_cap_mb=0.001)\n"
        "    out = []\n"
        "    for x in xs:\n"
        "        for p in m.parameters(): p.grad.zero_()\n"
        "        with gradsink.direct_grads(direct):\n"
        "            d(x).square().mean().backward()\n"
        "        out.append(torch.cat([p.grad.reshape(-1).clone() for p in m.parameters()]))\n"
        "    return out\n"
        "def run_hvd(direct):\n"
        "    m = Net(); m.load_state_dict(base.state_dict()); flatten_module(m)\n"
        "    # (the trainers' FusedAdam zeroes the flat gradient in place: the views stay)\n"
        "    opt = hvd.DistributedOptimizer(FusedAdam(m.parameters(), lr=0.0), named_parameters=m.named_parameters())\n"
        "    out = []\n"
        "    for x in xs:\n"
        "        opt.zero_grad()\n"
        "        with gradsink.direct_grads(direct):\n"
        "            m(x).square().mean().backward()\n"
        "        opt.synchronize()\n"
        "        out.append(torch.cat([p.grad.reshape(-1).clone() for p in m.parameters()]))\n"
        "    return out\n"
        "hvd.init('gloo')\n"
        "taken = [0]\n"
        "real_sink = gradsink.sink\n"
        "def counting(p, on):\n"
        "    g = real_sink(p, on)\n"
        "    taken[0] += g is not None\n"
        "    return g\n"
        "gradsink.sink = counting\n"
        "for name, fn in (('ddp', run_ddp), ('hvd', run_hvd)):\n"
        "    taken[0] = 0\n"
        "    a = fn(True)\n"
        "    assert taken[0] == 3 * 4, (name, taken[0])  # every parameter's gradient written in place\n"
        "    b = fn(False)\n"
        "    for ga, gb in zip(a, b):\n"
        "        assert torch.equal(ga, gb), (name, (ga - gb).abs().max())\n"
        "        allg = [torch.empty_like(ga) for _ in range(W)]\n"
        "        dist.all_gather(allg, ga)\n"
        "        assert all(torch.equal(allg[0], g) for g in allg), name\n"
        "    open(f'direct-ok-{name}-{r}', 'w').close()  # (the ranks share stdout)\n"
        "dist.destroy_process_group()\n")
    out = torchrun([str(script)], nproc=2, cwd=str(tmp_path))
    got = sorted(p.name for p in tmp_path.glob("direct-ok-*"))
    assert got == ["direct-ok-ddp-0", "direct-ok-ddp-1", "direct-ok-hvd-0", "direct-ok-hvd-1"], out
