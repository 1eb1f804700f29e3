"""Flat parameter storage + FusedAdam reference path == torch.optim.Adam
(reference: base.py:43,117 Adam lr 2.5e-3)."""
import torch
from torch import nn

from pytorch_distributed_rnn_amd.models.motion import MotionModel
from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
from pytorch_distributed_rnn_amd.utils.flat import contiguous_span, flatten_module


def _train(model, opt, steps=4):
    torch.manual_seed(5)
    for _ in range(steps):
        x = torch.randn(8, 10, 9)
        y = torch.randint(0, 6, (8,))
        opt.zero_grad()
        nn.functional.cross_entropy(model(x), y).backward()
        opt.step()


def test_flatten_module_views():
    m = MotionModel(9, 8, 2, 6)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    flat = flatten_module(m)
    (fp,) = flat.values()
    assert contiguous_span([p.data for p in m.parameters()]) is not None
    for k, v in m.state_dict().items():
        torch.testing.assert_close(v, before[k])
    assert fp.data.numel() == sum(p.numel() for p in m.parameters())


def test_fused_adam_matches_torch_adam():
    torch.manual_seed(0)
    a = MotionModel(9, 8, 2, 6)
    b = MotionModel(9, 8, 2, 6)
    b.load_state_dict(a.state_dict())
    flatten_module(a)
    _train(a, FusedAdam(a.parameters(), lr=2.5e-3))
    _train(b, torch.optim.Adam(b.parameters(), lr=2.5e-3))
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6, msg=n)


def test_fused_adam_state_dict_is_torch_compatible():
    m = MotionModel(9, 8, 2, 6)
    flatten_module(m)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    _train(m, opt, steps=2)
    sd = opt.state_dict()
    ref = torch.optim.Adam(MotionModel(9, 8, 2, 6).parameters(), lr=1e-3)
    ref.load_state_dict(sd)  # loads into stock Adam
    st = sd["state"][0]
    assert set(st.keys()) >= {"step", "exp_avg", "exp_avg_sq"}
    assert float(st["step"]) == 2.0


def test_stats_to_host_ring_slice_and_fallback():
    """Epoch statistics read-back: consecutive rows of the fused step's ring
    come back as one slice copy; wrapped or unrelated rows are stacked."""
    from pytorch_distributed_rnn_amd.train.trainer import stats_to_host
    ring = torch.arange(30.).view(10, 3)
    assert torch.equal(stats_to_host([ring[2], ring[3], ring[4]]), ring[2:5])
    assert torch.equal(stats_to_host([ring[9], ring[0]]), torch.stack([ring[9], ring[0]]))
    a, b = torch.ones(3), torch.zeros(3)
    assert torch.equal(stats_to_host([a, b]), torch.stack([a, b]))


def test_fused_adam_skip_word_leaves_state_untouched():
    """A nonzero skip word (the deferred persistent-path verification of
    train/lm.py) leaves parameters and moments untouched; rewind() takes the
    skipped native step back from the count."""
    torch.manual_seed(0)
    m = MotionModel(9, 8, 2, 6)
    flatten_module(m)
    opt = FusedAdam(m.parameters(), lr=2.5e-3)
    _train(m, opt, steps=2)
    before = [p.detach().clone() for p in m.parameters()]
    for p in m.parameters():
        p.grad = torch.randn_like(p)
    opt.step(skip=torch.ones(1, dtype=torch.int32))
    for p, q in zip(m.parameters(), before):
        assert torch.equal(p.detach(), q)
    opt.step(skip=torch.zeros(1, dtype=torch.int32))
    assert any(not torch.equal(p.detach(), q) for p, q in zip(m.parameters(), before))
    opt.rewind(0)  # CPU path: no flat native state to rewind
