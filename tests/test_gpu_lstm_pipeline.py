"""Stacked-layer chunk pipeline of the fp32 H = 128 LSTM (ops/lstm_large.py
_PipelinedLSTMStack on lstm_rows_fwd_range / lstm_rows_bwd_range) against the
whole-sequence per-layer path and an fp64 torch reference."""
import pytest
import torch

from pytorch_distributed_rnn_amd import _ext
from pytorch_distributed_rnn_amd.models.rnn import LSTM
from pytorch_distributed_rnn_amd.ops import lstm_large

from _tune import set_tune

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _run(m, x, h0, c0, g):
    for p in m.parameters():
        p.grad = None
    xa = x.clone().requires_grad_(True)
    h0a = h0.clone().requires_grad_(True) if h0 is not None else None
    c0a = c0.clone().requires_grad_(True) if c0 is not None else None
    out, (hn, cn) = m(xa, (h0a, c0a) if h0 is not None else None)
    loss = (out * g).sum() + 0.7 * hn.sum() + 0.3 * cn.sum()
    loss.backward()
    res = {"out": out, "hn": hn, "cn": cn, "dx": xa.grad}
    if h0 is not None:
        res["dh0"], res["dc0"] = h0a.grad, c0a.grad
    res.update({n: p.grad.clone() for n, p in m.named_parameters()})
    return res


@pytest.mark.parametrize("L,chunks,B,T,I,bias,state", [(2, 4, 40, 16, 9, True, False), (2, 3, 33, 10, 24, True, True),
                                                       (3, 5, 17, 7, 128, False, True), (2, 1, 16, 5, 9, True, True),
                                                       (2, 16, 20, 12, 9, True, False)])
def test_pipeline_matches_whole_sequence_and_fp64(L, chunks, B, T, I, bias, state, monkeypatch):
    mod = _ext.require()
    assert mod.lstm_rows_range_supported(128)
    torch.manual_seed(7)
    H = 128
    m = LSTM(I, H, L, batch_first=True, bias=bias).cuda()
    x = torch.randn(B, T, I, device="cuda")
    h0 = torch.randn(L, B, H, device="cuda") if state else None
    c0 = torch.randn(L, B, H, device="cuda") if state else None
    g = torch.randn(B, T, H, device="cuda")
    set_tune(monkeypatch, large_chunks=str(chunks))
    calls = []
    orig = lstm_large._PipelinedLSTMStack.apply
    monkeypatch.setattr(lstm_large._PipelinedLSTMStack, "apply", lambda *a: calls.append(1) or orig(*a))
    pipe = _run(m, x, h0, c0, g)
    assert calls, "the pipelined stack did not run"
    set_tune(monkeypatch, large_pipe="0")
    whole = _run(m, x, h0, c0, g)
    assert len(calls) == 1
    ref_m = torch.nn.LSTM(I, H, L, batch_first=True, bias=bias).double().cuda()
    with torch.no_grad():
        for (_, p), (_, q) in zip(m.named_parameters(), ref_m.named_parameters()):
            q.copy_(p.double())
    ref = _run(ref_m, x.double(), h0.double() if state else None, c0.double() if state else None, g.double())
    for k in pipe:
        # forward: the same kernels on the same operands, chunk by chunk
        if k in ("out", "hn", "cn"):
            assert torch.equal(pipe[k], whole[k]), k
        assert _rel(pipe[k], whole[k]) < 1e-5, k
        assert _rel(pipe[k], ref[k]) < 1e-4, k


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_pipeline_runs_beside_the_default_stream(cell):
    """Three training steps through the motion model at H = 128: the per-layer
    streams join the caller's stream (no stale reads across steps).  SGD, not
    Adam: Adam's first steps are ~lr * sign(g), so gradients that agree to
    1e-6 can still move a near-zero-gradient weight in opposite directions."""
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    torch.manual_seed(3)
    model = MotionModel(9, 128, 2, 6, cell=cell).cuda()
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    x = torch.randn(64, 32, 9, device="cuda")
    y = torch.randint(0, 6, (64,), device="cuda")
    losses = []
    for _ in range(3):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    torch.manual_seed(3)
    ref = MotionModel(9, 128, 2, 6, cell=cell).cuda()
    import os
    from pytorch_distributed_rnn_amd.utils.tune import tune_string
    saved = os.environ.get("PDRNN_TUNE")
    os.environ["PDRNN_TUNE"] = tune_string({"large_pipe": "0"})
    try:
        opt = torch.optim.SGD(ref.parameters(), lr=0.5)
        ref_losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(ref(x), y)
            loss.backward()
            opt.step()
            ref_losses.append(float(loss))
    finally:
        if saved is None:
            del os.environ["PDRNN_TUNE"]
        else:
            os.environ["PDRNN_TUNE"] = saved
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-5 * max(1.0, abs(b))
    assert losses[-1] < losses[0]


def _run_gru(m, x, h0, g):
    for p in m.parameters():
        p.grad = None
    xa = x.clone().requires_grad_(True)
    h0a = h0.clone().requires_grad_(True) if h0 is not None else None
    out, hn = m(xa, h0a)
    ((out * g).sum() + 0.7 * hn.sum()).backward()
    res = {"out": out, "hn": hn, "dx": xa.grad}
    if h0 is not None:
        res["dh0"] = h0a.grad
    res.update({n: p.grad.clone() for n, p in m.named_parameters()})
    return res


@pytest.mark.parametrize("L,chunks,B,T,I,bias,state", [(2, 3, 40, 16, 9, True, False), (3, 5, 17, 7, 128, False, True),
                                                       (2, 1, 16, 5, 9, True, True), (2, 12, 20, 12, 9, True, True)])
def test_gru_pipeline_matches_whole_sequence_and_fp64(L, chunks, B, T, I, bias, state, monkeypatch):
    from pytorch_distributed_rnn_amd.models.rnn import GRU
    from pytorch_distributed_rnn_amd.ops import gru_large
    torch.manual_seed(8)
    H = 128
    m = GRU(I, H, L, batch_first=True, bias=bias).cuda()
    x = torch.randn(B, T, I, device="cuda")
    h0 = torch.randn(L, B, H, device="cuda") if state else None
    g = torch.randn(B, T, H, device="cuda")
    set_tune(monkeypatch, large_chunks=str(chunks))
    calls = []
    orig = gru_large._PipelinedGRUStack.apply
    monkeypatch.setattr(gru_large._PipelinedGRUStack, "apply", lambda *a: calls.append(1) or orig(*a))
    pipe = _run_gru(m, x, h0, g)
    assert calls, "the pipelined GRU stack did not run"
    set_tune(monkeypatch, large_pipe="0")
    whole = _run_gru(m, x, h0, g)
    assert len(calls) == 1
    ref_m = torch.nn.GRU(I, H, L, batch_first=True, bias=bias).double().cuda()
    with torch.no_grad():
        for (_, p), (_, q) in zip(m.named_parameters(), ref_m.named_parameters()):
            q.copy_(p.double())
    ref = _run_gru(ref_m, x.double(), h0.double() if state else None, g.double())
    for k in pipe:
        if k in ("out", "hn"):
            assert torch.equal(pipe[k], whole[k]), k
        assert _rel(pipe[k], whole[k]) < 1e-5, k
        assert _rel(pipe[k], ref[k]) < 1e-4, k


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_layer_by_layer_overlap_matches_serial(cell, monkeypatch):
    """The layer-by-layer path's cross-layer backward overlap (the layer
    below's BPTT on a side stream after the layer above's dX event) gives the
    serial path's gradients bit for bit, run after run.  The motion model
    leaves the LSTM's cell-state output unused: before its Functions stopped
    materialising zero gradients, that zero fill was queued on the main stream
    after the event and the side stream sometimes read it first."""
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, large_pipe="0")
    torch.manual_seed(5)
    model = MotionModel(9, 128, 2, 6, cell=cell).cuda()
    x = torch.randn(96, 40, 9, device="cuda")
    y = torch.randint(0, 6, (96,), device="cuda")

    def grads():
        model.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        return [p.grad.clone() for p in model.parameters()]

    set_tune(monkeypatch, large_overlap="0")
    ref = grads()
    set_tune(monkeypatch, large_overlap="1")
    for _ in range(4):
        for a, b in zip(grads(), ref):
            assert torch.equal(a, b)
