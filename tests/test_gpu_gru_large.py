"""Large-H GRU on the MFMA step kernels (ops/gru_large.py, CELL = GRU in
csrc/kernels/lstm_large.hip) vs the fp32 torch.nn.GRU on the same
16-bit-rounded inputs, initial states and weights."""
import pytest
import torch

from pytorch_distributed_rnn_amd.models.rnn import GRU
from pytorch_distributed_rnn_amd.ops import gru_large

from _tune import set_tune

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _pair(I, H, L, bi, dt, bias=True, seed=1):
    torch.manual_seed(seed)
    m = GRU(I, H, L, bias=bias, batch_first=True, bidirectional=bi).cuda()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(dt).float())
    ref = torch.nn.GRU(I, H, L, bias=bias, batch_first=True, bidirectional=bi).cuda()
    with torch.no_grad():
        for (_, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            q.copy_(p)
    return m, ref


def _check(m, ref, x, h0, tol_f=2e-2, tol_b=4e-2):
    dt = x.dtype
    x16 = x.clone().requires_grad_(True)
    xr = x.float().clone().requires_grad_(True)
    h0a = h0.clone().requires_grad_(True)
    h0b = h0.float().clone().requires_grad_(True)
    out, hn = m(x16, h0a)
    out_r, hn_r = ref(xr, h0b)
    assert out.dtype == dt and out.shape == out_r.shape and hn.shape == hn_r.shape
    assert _rel(out, out_r) < tol_f
    assert _rel(hn, hn_r) < tol_f
    g = torch.randn_like(out_r)
    gh = torch.randn_like(hn_r)
    ((out.float() * g).sum() + (hn.float() * gh).sum()).backward()
    ((out_r * g).sum() + (hn_r * gh).sum()).backward()
    assert _rel(x16.grad, xr.grad) < tol_b
    assert _rel(h0a.grad, h0b.grad) < tol_b
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < tol_b, n


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,L,bi,B,T,I", [(64, 1, False, 5, 7, 24), (128, 2, False, 33, 9, 40),
                                          (1024, 1, False, 16, 3, 32),  # split-K backward
                                          (64, 2, True, 5, 6, 24), (256, 1, True, 70, 4, 64)])
def test_large_gru_matches_torch(dt, H, L, bi, B, T, I):
    m, ref = _pair(I, H, L, bi, dt)
    x = torch.randn(B, T, I, device="cuda").to(dt)
    assert gru_large.supported(x, H)  # the MFMA path, not the ATen fallback
    h0 = (0.5 * torch.randn(L * (2 if bi else 1), B, H, device="cuda")).to(dt)
    _check(m, ref, x, h0)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4])
def test_large_gru_every_tile(tile, monkeypatch):
    set_tune(monkeypatch, large_tile=str(tile))
    m, ref = _pair(64, 128, 1, True, torch.bfloat16, seed=4)
    x = torch.randn(5, 37, 64, device="cuda").to(torch.bfloat16)
    h0 = torch.zeros(2, 5, 128, device="cuda", dtype=torch.bfloat16)
    _check(m, ref, x, h0)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("bwd", ["0", "2"])
def test_large_gru_pingpong_step_matches_torch(dt, bwd, monkeypatch):
    set_tune(monkeypatch, large_pp="2")
    monkeypatch.setenv("PDRNN_TUNE large_pp_BWD", bwd)
    test_large_gru_matches_torch(dt, 256, 1, True, 300, 3, 64)


def test_large_gru_no_bias_no_state():
    m, ref = _pair(32, 128, 2, False, torch.bfloat16, bias=False, seed=6)
    x = torch.randn(6, 5, 32, device="cuda").to(torch.bfloat16)
    out, hn = m(x)
    out_r, hn_r = ref(x.float())
    assert _rel(out, out_r) < 2e-2 and _rel(hn, hn_r) < 2e-2
    out.float().sum().backward()
    out_r.sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < 4e-2, n
