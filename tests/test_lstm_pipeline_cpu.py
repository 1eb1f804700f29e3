"""CPU checks of the fp32 stacked-layer pipeline's bookkeeping
(ops/lstm_large.py): time chunks and the chunk-by-chunk weight gradients
(the gemm_f32 torch fallback stands in for the HIP GEMM)."""
import pytest
import torch

from pytorch_distributed_rnn_amd.ops.lstm_large import _chunk_weight_grads, pipeline_chunks

from _tune import set_tune


def test_pipeline_chunks_cover_the_sequence(monkeypatch):
    for c, T in [(4, 128), (3, 10), (16, 12), (1, 5)]:
        set_tune(monkeypatch, large_chunks=str(c))
        ch = pipeline_chunks(T)
        assert len(ch) == min(c, T) and ch[0][0] == 0 and ch[-1][1] == T
        assert all(a[1] == b[0] and a[0] < a[1] for a, b in zip(ch, ch[1:]))


@pytest.mark.parametrize("chunks", [1, 2, 3, 7])
@pytest.mark.parametrize("with_h0", [False, True])
def test_chunked_weight_grads_match_whole_sequence(chunks, with_h0, monkeypatch):
    torch.manual_seed(0)
    T, B, H, I = 7, 3, 8, 5
    G = torch.randn(T, B, 4 * H)
    hd = torch.randn(T, B, H)
    x = torch.randn(T, B, I)
    h0 = torch.randn(B, H) if with_h0 else None
    set_tune(monkeypatch, large_chunks=str(chunks))
    dwih, dwhh, db = torch.full((4 * H, I), float("nan")), torch.full((4 * H, H), float("nan")), torch.empty(4 * H)
    for k, (t0, t1) in enumerate(reversed(pipeline_chunks(T))):  # the backward's order: last chunk first
        _chunk_weight_grads(dwih, dwhh, db, G, hd, h0, x, t0, t1, k == 0)
    hprev = torch.cat([(h0 if h0 is not None else torch.zeros(B, H))[None], hd[:-1]], 0)
    G2 = G.reshape(-1, 4 * H)
    torch.testing.assert_close(dwhh, G2.t() @ hprev.reshape(-1, H), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(dwih, G2.t() @ x.reshape(-1, I), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(db, G2.sum(0), rtol=1e-5, atol=1e-5)
