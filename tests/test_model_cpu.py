"""Model / op reference semantics on the CPU (reference: src/motion/model.py:4-17)."""
import torch
from torch import nn

from pytorch_distributed_rnn_amd.models.motion import MotionModel
from pytorch_distributed_rnn_amd.ops.xent import CrossEntropyLoss, cross_entropy_with_stats

REF_KEYS = ["lstm.weight_ih_l0", "lstm.weight_hh_l0", "lstm.bias_ih_l0", "lstm.bias_hh_l0",
            "lstm.weight_ih_l1", "lstm.weight_hh_l1", "lstm.bias_ih_l1", "lstm.bias_hh_l1",
            "fc.weight", "fc.bias"]


class RefMotion(nn.Module):
    """The reference architecture written with stock torch modules."""

    def __init__(self, i, h, l, o):
        super().__init__()
        self.lstm = nn.LSTM(i, h, l, batch_first=True)
        self.fc = nn.Linear(h, o)

    def forward(self, x):
        out, _ = self.lstm(x)
        return self.fc(out[:, -1, :])


def test_state_dict_layout_matches_reference():
    m = MotionModel(9, 32, 2, 6)
    sd = m.state_dict()
    assert list(sd.keys()) == REF_KEYS
    assert sd["lstm.weight_ih_l0"].shape == (128, 9)
    assert sd["lstm.weight_hh_l1"].shape == (128, 32)
    assert sd["fc.weight"].shape == (6, 32)
    assert sum(p.numel() for p in m.parameters()) == 14150  # 14,150 fp32


def test_forward_backward_match_stock_torch():
    torch.manual_seed(0)
    m = MotionModel(9, 16, 2, 6).double()
    ref = RefMotion(9, 16, 2, 6).double()
    ref.load_state_dict(m.state_dict())
    x = torch.randn(5, 20, 9, dtype=torch.float64)
    y = torch.randint(0, 6, (5,))
    out, out_ref = m(x), ref(x)
    torch.testing.assert_close(out, out_ref)
    nn.functional.cross_entropy(out, y).backward()
    nn.functional.cross_entropy(out_ref, y).backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad, q.grad, msg=n)


def test_index_batches_equal_gathered_batches():
    torch.manual_seed(1)
    m = MotionModel(9, 8, 2, 6)
    feats = torch.randn(30, 12, 9)
    idx = torch.tensor([3, 7, 7, 0, 29])
    torch.testing.assert_close(m(feats, idx=idx), m(feats[idx]))


def test_gru_cell_variant():
    m = MotionModel(9, 8, 2, 6, cell="gru")
    assert m(torch.randn(4, 10, 9)).shape == (4, 6)


def test_cross_entropy_with_stats_reference():
    torch.manual_seed(2)
    logits = torch.randn(17, 6, requires_grad=True)
    y = torch.randint(0, 6, (17,))
    loss, stats = cross_entropy_with_stats(logits, y)
    torch.testing.assert_close(loss, nn.functional.cross_entropy(logits, y))
    assert int(stats[2]) == int((logits.argmax(1) == y).sum())
    crit = CrossEntropyLoss()
    assert torch.allclose(crit(logits, y), loss)
