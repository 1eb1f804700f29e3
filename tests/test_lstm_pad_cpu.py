"""Zero-padding of hidden units (how the fused small-H kernels serve hidden
sizes they are not instantiated for, ops/lstm.py:small_plan) is exact: an LSTM /
GRU with zero-padded gate rows, columns and biases reproduces the unpadded
module's outputs, states and weight gradients (checked on the ATen reference,
fp64)."""
import pytest
import torch

from pytorch_distributed_rnn_amd.ops.lstm import _pad_state, pad_gate_rows


@pytest.mark.parametrize("cell,gates", [("lstm", 4), ("gru", 3)])
@pytest.mark.parametrize("H,HP,I,L", [(8, 16, 9, 2), (24, 32, 5, 3), (48, 64, 9, 1)])
def test_padded_units_stay_zero(cell, gates, H, HP, I, L):
    torch.manual_seed(0)
    mod = (torch.nn.LSTM if cell == "lstm" else torch.nn.GRU)(I, H, L, batch_first=True).double()
    x = torch.randn(3, 7, I, dtype=torch.float64)
    h0 = torch.randn(L, 3, H, dtype=torch.float64)
    c0 = torch.randn(L, 3, H, dtype=torch.float64)
    ref_out, ref_st = mod(x, (h0, c0) if cell == "lstm" else h0)
    (ref_out.square().sum() + (ref_st[0] if cell == "lstm" else ref_st).sum()).backward()
    ref_g = [p.grad.clone() for p in mod.parameters()]
    for p in mod.parameters():
        p.grad = None

    ws = []
    for l in range(L):
        w_ih, w_hh, b_ih, b_hh = (getattr(mod, f"{n}_l{l}") for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh"))
        ws += [pad_gate_rows(w_ih, H, HP, gates, None if l == 0 else HP), pad_gate_rows(w_hh, H, HP, gates, HP),
               pad_gate_rows(b_ih, H, HP, gates), pad_gate_rows(b_hh, H, HP, gates)]
    hp0, cp0 = _pad_state(h0, H, HP), _pad_state(c0, H, HP)
    if cell == "lstm":
        out, hn, cn = torch._VF.lstm(x, (hp0, cp0), ws, True, L, 0.0, False, False, True)
        st = hn
    else:
        out, hn = torch._VF.gru(x, hp0, ws, True, L, 0.0, False, False, True)
        st = hn
    assert torch.equal(out[..., H:], torch.zeros_like(out[..., H:]))
    torch.testing.assert_close(out[..., :H], ref_out)
    (out[..., :H].square().sum() + st[..., :H].sum()).backward()
    for p, g in zip(mod.parameters(), ref_g):
        torch.testing.assert_close(p.grad, g)
