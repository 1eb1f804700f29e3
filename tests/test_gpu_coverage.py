"""GPU: configurations the reference CLI accepts (any --hidden-units /
--stacked-layer into nn.LSTM, reference src/motion/main.py:20-21,
src/motion/model.py:9) run on the HIP kernels -- zero-padded hidden units,
layer chunks, per-direction bidirectional launches, dropout between layer
chunks, fp32 large hidden sizes on the MFMA step kernels -- under strict kernel mode (PDRNN_KERNELS=hip-strict: an ATen/MIOpen
fallback raises), checked against fp64 torch modules."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def strict(monkeypatch):
    monkeypatch.setenv("PDRNN_KERNELS", "hip-strict")


def _check(mod_ref, mod, x, h0=None, tol=2e-4):
    out_ref, st_ref = mod_ref(x, h0) if h0 is not None else mod_ref(x)
    hn_ref = st_ref[0] if isinstance(st_ref, tuple) else st_ref
    g = torch.randn_like(out_ref)
    ((out_ref * g).sum() + hn_ref.square().sum()).backward()
    dev = torch.device("cuda")
    xg = x.float().to(dev)
    out, st = mod(xg)
    hn = st[0] if isinstance(st, tuple) else st
    err = (out.double().cpu() - out_ref).abs().max().item()
    assert err < tol, err
    assert (hn.double().cpu() - hn_ref).abs().max().item() < tol
    ((out * g.float().to(dev)).sum() + hn.square().sum()).backward()
    for (n, p), q in zip(mod.named_parameters(), mod_ref.parameters()):
        scale = q.grad.abs().max().item() + 1e-6
        e = (p.grad.double().cpu() - q.grad).abs().max().item()
        assert e / scale < 5e-4, (n, e, scale)


@pytest.mark.parametrize("cell,H,L,bidir", [
    ("lstm", 8, 2, False), ("lstm", 48, 2, False), ("lstm", 24, 3, False), ("lstm", 32, 5, False),
    ("lstm", 32, 2, True), ("lstm", 16, 1, True), ("gru", 8, 2, False), ("gru", 48, 3, False),
    # fp32 large-H: MFMA 16x16x4 f32 step kernels (lstm_large.hip, F32 storage);
    # H = 100 is zero-padded to 128
    ("lstm", 128, 2, False), ("lstm", 100, 1, False), ("lstm", 128, 1, True), ("gru", 128, 2, False),
    ("gru", 192, 1, True),
])
def test_uncovered_shapes_run_on_hip(cell, H, L, bidir):
    from pytorch_distributed_rnn_amd.models.rnn import GRU, LSTM
    torch.manual_seed(0)
    I, B, T = 9, 6, 33
    cls_ref = torch.nn.LSTM if cell == "lstm" else torch.nn.GRU
    ref = cls_ref(I, H, L, batch_first=True, bidirectional=bidir).double()
    mod = (LSTM if cell == "lstm" else GRU)(I, H, L, batch_first=True, bidirectional=bidir).cuda()
    mod.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    _check(ref, mod, torch.randn(B, T, I, dtype=torch.float64))


def test_motion_cli_shapes_train_on_hip(tmp_path):
    """main.py-equivalent model builds with the reference's flags train a step
    through the kernels (strict mode), dropout between layer chunks included."""
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    for H, L, bidir in ((48, 2, False), (8, 2, False), (32, 2, True), (128, 2, False), (256, 1, True)):
        torch.manual_seed(1)
        m = MotionModel(9, H, L, 6, bidirectional=bidir).cuda()
        m.lstm.dropout = 0.1
        m.train()
        x = torch.randn(64, 128, 9, device="cuda")
        y = torch.randint(0, 6, (64,), device="cuda")
        loss = torch.nn.functional.cross_entropy(m(x), y)
        loss.backward()
        assert torch.isfinite(loss)
        assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())
