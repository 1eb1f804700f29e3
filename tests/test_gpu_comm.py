"""GPU: the native RCCL communicator, the bucketed DDP reducer and the
horovod-mode fusion reducer on a one-rank RCCL group (the driver's 2/4/8-GPU
runs exercise the same code with more ranks; here: that it initialises,
launches on its own stream, orders against the compute stream and computes
the right thing)."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    from pytorch_distributed_rnn_amd.parallel import comm, env
    old = {k: os.environ.get(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    env.init_distributed("nccl")
    assert dist.get_backend() == "nccl"
    yield
    comm.reset_comms()
    dist.destroy_process_group()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_rccl_comm_collectives(rccl_group):
    from pytorch_distributed_rnn_amd.parallel.comm import get_comm
    c = get_comm()
    assert type(c).__name__ != "_PyComm" and c.world == 1 and c.rank == 0
    x = torch.arange(1000, dtype=torch.float32, device="cuda")
    y = x.clone()
    c.all_reduce(y, "sum")
    c.wait()
    torch.testing.assert_close(y, x)
    c.all_reduce(y, "avg")
    c.broadcast(y, 0)
    out = torch.empty_like(x)
    c.all_gather(out, y)
    rs = torch.empty_like(x)
    c.reduce_scatter(rs, out, "sum")
    c.wait()
    torch.testing.assert_close(rs, x)
    c.barrier()
    z = x.clone()
    c.all_reduce(z, "sum")        # queued on the comm stream ...
    c.all_reduce_inline(z, "avg")  # ... joined before the inline one (same communicator)
    torch.testing.assert_close(z, x)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # a real (non-NULL) stream: RCCL runs on it directly
        w = z * 2
        c.all_reduce_inline(w, "sum")
        w += 1
    torch.cuda.current_stream().wait_stream(side)
    torch.testing.assert_close(w, 2 * x + 1)


@pytest.mark.parametrize("mode", ["all_reduce_now", "all_reduce_inline"])
def test_ddp_reducer_rccl_step_matches_local(rccl_group, mode):
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_rnn_amd.train.fused_step import MotionTrainStep
    from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
    from pytorch_distributed_rnn_amd.utils.flat import flatten_module
    torch.manual_seed(0)
    train, _, _ = synthetic_motion(n_train=192, n_validation=1, n_test=1, seed=0)
    feats, labels = train.features.cuda(), train.labels.cuda().reshape(-1)
    m1 = MotionModel(9, 32, 2, 6).cuda()
    m2 = copy.deepcopy(m1)
    ddp = DistributedDataParallel(m1, bucket_cap_mb=0.01)  # several buckets
    assert len(ddp.bucket_layout()) >= 1
    o1 = FusedAdam(m1.parameters(), lr=2.5e-3)
    flatten_module(m2)
    o2 = FusedAdam(m2.parameters(), lr=2.5e-3)
    s1 = MotionTrainStep(ddp, o1, getattr(ddp.reducer, mode))   # RCCL all-reduce in the step
    s2 = MotionTrainStep(m2, o2, None)                           # local, Adam fused into the reduction
    for i in range(3):
        idx = torch.arange(i * 64, (i + 1) * 64, device="cuda")
        a = s1(feats, labels, idx)
        b = s2(feats, labels, idx)
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_graph_replayed_rccl_step_matches_local(rccl_group):
    """The synced step captured into a HIP graph (fwd/BPTT/reductions + inline
    RCCL all-reduce + Adam with a device step count) and replayed with fresh
    batch indices reproduces the eager local step, step for step, including
    after an eager step in between (device step count re-seeded)."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_rnn_amd.train.fused_step import MotionTrainStep
    from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
    from pytorch_distributed_rnn_amd.utils.flat import flatten_module
    torch.manual_seed(3)
    train, _, _ = synthetic_motion(n_train=512, n_validation=1, n_test=1, seed=3)
    feats, labels = train.features.cuda(), train.labels.cuda().reshape(-1)
    m1 = MotionModel(9, 32, 2, 6).cuda()
    m2 = copy.deepcopy(m1)
    ddp = DistributedDataParallel(m1)
    o1 = FusedAdam(m1.parameters(), lr=2.5e-3)
    flatten_module(m2)
    o2 = FusedAdam(m2.parameters(), lr=2.5e-3)
    s1 = MotionTrainStep(ddp, o1, ddp.reducer.all_reduce_inline, cuda_graph=True)
    s2 = MotionTrainStep(m2, o2, None)
    g = torch.Generator().manual_seed(0)
    outs = []
    for i in range(7):
        idx = torch.randperm(512, generator=g)[:64].cuda()
        if i == 5:  # a host-gathered batch in between runs eagerly
            a = s1(feats.index_select(0, idx), labels.index_select(0, idx), None)
        else:
            a = s1(feats, labels, idx)
        b = s2(feats, labels, idx)
        outs.append((a.clone(), b.clone()))
    assert s1._graph is not None, "the synced step was never captured"
    for a, b in outs:
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    assert o1.state_dict()["state"][0]["step"] == o2.state_dict()["state"][0]["step"]


def test_ddp_autograd_hooks_rccl(rccl_group):
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.parallel.ddp import DistributedDataParallel
    torch.manual_seed(1)
    m1 = MotionModel(9, 16, 2, 6).cuda()
    m2 = copy.deepcopy(m1)
    ddp = DistributedDataParallel(m1)
    x = torch.randn(8, 20, 9, device="cuda")
    y = torch.randint(0, 6, (8,), device="cuda")
    torch.nn.functional.cross_entropy(ddp(x), y).backward()
    torch.nn.functional.cross_entropy(m2(x), y).backward()
    torch.cuda.synchronize()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-6)


def test_horovod_mode_rccl(rccl_group):
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.parallel import horovod as hvd
    hvd.init("nccl")
    assert hvd.size() == 1 and hvd.rank() == 0
    torch.manual_seed(2)
    m1 = MotionModel(9, 16, 2, 6).cuda()
    m2 = copy.deepcopy(m1)
    hvd.broadcast_parameters(m1.state_dict(), root_rank=0)
    o1 = hvd.DistributedOptimizer(torch.optim.Adam(m1.parameters(), lr=1e-3), named_parameters=m1.named_parameters())
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    x = torch.randn(8, 20, 9, device="cuda")
    y = torch.randint(0, 6, (8,), device="cuda")
    for m, o in ((m1, o1), (m2, o2)):
        o.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        o.step()
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    t = torch.ones(10, device="cuda")
    hvd.allreduce_(t, average=True)
    torch.testing.assert_close(t, torch.ones(10, device="cuda"))
