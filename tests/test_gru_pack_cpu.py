"""Host-side layout of the fused GRU (ops/gru_fused.py): the batched 4-block
packing and the single-gather gradient unpack match the per-tensor reference
layout [r | z | n_x | n_h] (no GPU needed: pure tensor indexing)."""
import torch

from pytorch_distributed_rnn_amd.ops import gru_fused


def _ref_pack(weights, NL, H):
    out = []
    for l in range(NL):
        w_ih, w_hh, b_ih, b_hh = weights[4 * l:4 * l + 4]
        I = w_ih.shape[1]
        out += [torch.cat([w_ih, torch.zeros(H, I)]), torch.cat([w_hh[:2 * H], torch.zeros(H, H), w_hh[2 * H:]]),
                torch.cat([b_ih, torch.zeros(H)]), torch.cat([b_hh[:2 * H], torch.zeros(H), b_hh[2 * H:]])]
    return out


def test_pack_and_unpack_match_reference_layout():
    torch.manual_seed(0)
    H, NL, I0 = 32, 2, 9
    gru = torch.nn.GRU(I0, H, NL)
    weights = [p.detach() for p in gru.parameters()]
    packed = gru_fused._pack(weights, NL, H, weights[0])
    ref = _ref_pack(weights, NL, H)
    assert len(packed) == len(ref)
    for a, b in zip(packed, ref):
        assert a.shape == b.shape and a.is_contiguous()
        assert torch.equal(a, b)
    # gradient unpack: a packed gradient vector -> nn.GRU parameter layout
    dparams = torch.randn(sum(t.numel() for t in packed))
    idx = gru_fused._unpack_index(H, (I0, H), dparams.device)
    g = dparams.index_select(0, idx)
    off, views = 0, []
    for t in packed:
        views.append(dparams[off:off + t.numel()].view_as(t))
        off += t.numel()
    expect = []
    for l in range(NL):
        dwih4, dwhh4, dbih4, dbhh4 = views[4 * l:4 * l + 4]
        expect += [dwih4[:3 * H], torch.cat([dwhh4[:2 * H], dwhh4[3 * H:]]), dbih4[:3 * H],
                   torch.cat([dbhh4[:2 * H], dbhh4[3 * H:]])]
    flat_expect = torch.cat([e.reshape(-1) for e in expect])
    assert torch.equal(g, flat_expect)
