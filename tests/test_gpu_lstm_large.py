"""Large-H LSTM MFMA path vs the fp32 torch reference on the same 16-bit-rounded
inputs and weights (numerics tests for csrc/kernels/lstm_large.hip)."""
import pytest
import torch

from pytorch_distributed_rnn_amd import _ext
from pytorch_distributed_rnn_amd.models.rnn import LSTM

from _tune import set_tune

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("M,N,K", [(70, 128, 192), (128, 256, 64), (5, 128, 1024), (300, 256, 320)])
@pytest.mark.parametrize("tile", [-1, 0, 1, 2, 3, 4])
def test_gemm_nt_core(dt, M, N, K, tile):
    mod = _ext.require()
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").to(dt)
    b = torch.randn(N, K, device="cuda").to(dt)
    c = mod.gemm_nt(a, b, tile)
    ref = (a.double() @ b.double().t()).float()
    tol = 2e-5 if dt == torch.float32 else 2e-3  # fp32: exact products (v_mfma_f32_16x16x4_f32)
    torch.testing.assert_close(c, ref, rtol=tol, atol=tol * 10)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4])
def test_large_lstm_every_tile(tile, monkeypatch):
    set_tune(monkeypatch, large_tile=str(tile))
    torch.manual_seed(4)
    m = LSTM(64, 128, 1, batch_first=True, bidirectional=True).cuda()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    ref = _ref_model(m)
    x = torch.randn(37, 5, 64, device="cuda").to(torch.bfloat16)
    out, _ = m(x)
    out_r, _ = ref(x.float())
    assert _rel(out, out_r) < 2e-2
    g = torch.randn_like(out_r)
    (out.float() * g).sum().backward()
    (out_r * g).sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < 4e-2, n


def _ref_model(m: LSTM):
    ref = torch.nn.LSTM(m.input_size, m.hidden_size, m.num_layers, batch_first=m.batch_first,
                        bidirectional=m.bidirectional).cuda()
    with torch.no_grad():
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            q.copy_(p)
    return ref


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,L,bi,B,T,I", [(128, 1, False, 5, 7, 24), (128, 2, False, 33, 9, 40),
                                          (1024, 1, False, 16, 3, 32),  # split-K backward (8 slices)
                                          (64, 2, True, 5, 6, 24), (256, 1, True, 70, 4, 64)])
def test_large_lstm_matches_torch(dt, H, L, bi, B, T, I):
    torch.manual_seed(1)
    m = LSTM(I, H, L, batch_first=True, bidirectional=bi).cuda()
    # round weights to the compute dtype so both paths see identical values
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(dt).float())
    ref = _ref_model(m)
    x = torch.randn(B, T, I, device="cuda").to(dt)
    x16 = x.clone().requires_grad_(True)
    xr = x.float().clone().requires_grad_(True)
    out, (hn, cn) = m(x16)
    out_r, (hn_r, cn_r) = ref(xr)
    assert out.dtype == dt and out.shape == out_r.shape
    assert _rel(out, out_r) < 2e-2
    assert _rel(hn, hn_r) < 2e-2
    assert _rel(cn, cn_r) < 2e-2
    g = torch.randn_like(out_r)
    (out.float() * g).sum().backward()
    (out_r * g).sum().backward()
    assert _rel(x16.grad, xr.grad) < 4e-2
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) < 4e-2, n


@pytest.mark.parametrize("mode", ["gemmpipe", "gemm+cell"])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,L,bi,B,T,I", [(256, 1, True, 300, 3, 64), (512, 2, False, 520, 4, 128)])
def test_large_lstm_pingpong_step_matches_torch(dt, H, L, bi, B, T, I, mode, monkeypatch):
    """The 256x256 ping-pong step kernels, forced at shapes below their
    occupancy threshold (batch not a multiple of 256): forward with the
    two-pass cell epilogue, backward either on the fused GemmPipe step kernel
    or as the ping-pong GEMM into the dh workspace + the cell kernel."""
    set_tune(monkeypatch, large_pp="2")
    monkeypatch.setenv("PDRNN_TUNE large_pp_BWD", "2" if mode == "gemm+cell" else "0")
    test_large_lstm_matches_torch(dt, H, L, bi, B, T, I)


@pytest.mark.parametrize("H", [64, 128])  # 64: small fused path with bf16 inputs, 128: MFMA path
def test_large_lstm_state_grads(H):
    torch.manual_seed(3)
    dt = torch.bfloat16
    m = LSTM(32, H, 1, batch_first=False).cuda()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(p.to(dt).float())
    ref = _ref_model(m)
    x = torch.randn(5, 3, 32, device="cuda").to(dt)
    h0 = torch.randn(1, 3, H, device="cuda").to(dt)
    c0 = torch.randn(1, 3, H, device="cuda")
    h0a, c0a = h0.clone().requires_grad_(True), c0.clone().requires_grad_(True)
    h0b, c0b = h0.float().clone().requires_grad_(True), c0.clone().requires_grad_(True)
    _, (hn, cn) = m(x, (h0a, c0a))
    _, (hn_r, cn_r) = ref(x.float(), (h0b, c0b))
    (hn.float().sum() + 0.5 * cn.float().sum()).backward()
    (hn_r.sum() + 0.5 * cn_r.sum()).backward()
    assert _rel(h0a.grad, h0b.grad) < 4e-2
    assert _rel(c0a.grad, c0b.grad) < 4e-2


def test_charlm_trains_on_large_path():
    from pytorch_distributed_rnn_amd.data.charlm import CharCorpus
    from pytorch_distributed_rnn_amd.models.charlm import CharLM
    from pytorch_distributed_rnn_amd.train.lm import LMTrainer
    torch.manual_seed(0)
    corpus = CharCorpus.synthetic(200_000, 64, seed=0)
    tr = LMTrainer(CharLM(64, 32, 128, 2, 0.0, torch.bfloat16), corpus, 16, 64, 3e-3,
                   device=torch.device("cuda", 0), log_interval=0)
    first = tr.train_epoch(0, max_steps=5)["loss"]
    hist = [tr.train_epoch(e, max_steps=40)["loss"] for e in range(1, 3)]
    assert hist[-1] < first - 0.5, (first, hist)


def test_charlm_direct_grads_match_autograd(monkeypatch):
    """One process: the char-LM step's in-tree Functions (16-bit LSTM layer,
    16-bit head, embedding) add their weight gradients into the flat gradient
    views themselves (ops/gradsink.py) instead of returning them for
    autograd's per-parameter adds -- the same gradients, bit for bit, as the
    autograd path, and every sink actually taken."""
    from pytorch_distributed_rnn_amd.data.charlm import CharCorpus
    from pytorch_distributed_rnn_amd.models.charlm import CharLM
    from pytorch_distributed_rnn_amd.ops import gradsink
    from pytorch_distributed_rnn_amd.train.lm import LMTrainer
    torch.manual_seed(0)
    corpus = CharCorpus.synthetic(100_000, 256, seed=0)
    tr = LMTrainer(CharLM(256, 64, 256, 2, 0.0, torch.bfloat16), corpus, 32, 64, 3e-3,
                   device=torch.device("cuda", 0), log_interval=0)
    segs = list(CharCorpus.segments(tr.streams, 64, 2))
    taken = []
    real_sink = gradsink.sink

    def counting_sink(p, on):
        g = real_sink(p, on)
        taken.append(g is not None)
        return g
    monkeypatch.setattr(gradsink, "sink", counting_sink)
    grads = []
    for direct in (True, False):
        tr.direct_grads = direct
        tr.inner.reset_hidden_state()
        tr._fwd_bwd(*segs[0])
        tr._fwd_bwd(*segs[1])  # (a carried state)
        torch.cuda.synchronize()
        grads.append(tr.flat.grad.clone())
        if direct:
            n_direct = sum(taken)
    # embedding 1 + head 2 + 2 layers x 4 per step, two steps
    assert n_direct == 2 * (1 + 2 + 8), n_direct
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_embedding_bwd_csr8(dt):
    mod = _ext.require()
    torch.manual_seed(5)
    V, D, N = 300, 200, 5000
    idx = torch.randint(0, V, (N,), device="cuda")
    idx[:7] = 3  # a hot row
    g = torch.randn(N, D, device="cuda").to(dt)
    dw = mod.embedding_bwd(g, idx, V, 5)
    ref = torch.zeros(V, D, device="cuda").index_add_(0, idx, g.float())
    ref[5] = 0
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=1e-4)
    # bitwise deterministic
    assert torch.equal(dw, mod.embedding_bwd(g, idx, V, 5))
    # fused 16-bit gather
    w = torch.randn(V, D, device="cuda")
    out = mod.embedding_fwd(w, idx, torch.bfloat16)
    assert out.dtype == torch.bfloat16 and torch.equal(out, w[idx].to(torch.bfloat16))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V,D,N", [(256, 256, 65536), (100, 200, 30000)])
def test_embedding_bwd_pieces(dt, V, D, N):
    """Small vocabulary, many contributions per row (char-LM): each row's list
    is split into pieces summed in order -- matches index_add, bitwise
    reproducible, padding row zero, heavily skewed rows included."""
    mod = _ext.require()
    torch.manual_seed(6)
    idx = torch.randint(0, V, (N,), device="cuda")
    idx[: N // 3] = 7  # one very hot row
    g = torch.randn(N, D, device="cuda").to(dt)
    dw = mod.embedding_bwd(g, idx, V, 3)
    ref = torch.zeros(V, D, device="cuda", dtype=torch.float64).index_add_(0, idx, g.double()).float()
    ref[3] = 0
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=2e-3)
    assert torch.equal(dw, mod.embedding_bwd(g, idx, V, 3))


def test_shadow_weights_follow_optimizer_steps():
    """16-bit shadow weights (ops/lstm_large.shadow) are rebuilt whenever the
    fp32 master changes -- FusedAdam's native step bumps the version counters
    -- so training with the cache equals training with the cache dropped
    before every step; bidirectional with h0 covers the shifted dW_hh GEMMs."""
    import copy

    from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
    from pytorch_distributed_rnn_amd.utils.flat import flatten_module
    torch.manual_seed(7)
    m1 = LSTM(64, 128, 2, bidirectional=True).cuda()
    m2 = copy.deepcopy(m1)
    flatten_module(m1)
    flatten_module(m2)
    o1, o2 = FusedAdam(m1.parameters(), lr=1e-2), FusedAdam(m2.parameters(), lr=1e-2)
    x = torch.randn(9, 6, 64, device="cuda").to(torch.bfloat16)
    h0 = torch.randn(4, 6, 128, device="cuda").to(torch.bfloat16)
    c0 = torch.randn(4, 6, 128, device="cuda")
    for _ in range(3):
        for m, o, drop in ((m1, o1, False), (m2, o2, True)):
            if drop:
                for p in m.parameters():
                    if hasattr(p, "_pdrnn_shadow"):
                        del p._pdrnn_shadow
            o.zero_grad()
            out, _ = m(x, (h0, c0))
            out.float().square().mean().backward()
            o.step()
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=0, atol=0, msg=k)
    assert any(hasattr(p, "_pdrnn_shadow") for p in m1.parameters())


@pytest.mark.parametrize("V,N", [(256, 65536), (300, 5000), (16384, 70001), (7, 0), (5, 3)])
def test_embedding_sort_matches_stable_sort(V, N):
    """The in-tree counting sort behind the embedding backward (no library
    sort kernels) equals torch's stable sort: same permutation (ties in index
    order) and the same row offsets, negative indices wrapped."""
    mod = _ext.require()
    torch.manual_seed(9)
    idx = torch.randint(-V, V, (N,), device="cuda")
    perm, off = mod.embedding_sort(idx, V)
    flat = torch.where(idx < 0, idx + V, idx)
    vals, ref_perm = torch.sort(flat, stable=True)
    assert torch.equal(perm, ref_perm)
    assert torch.equal(off, torch.searchsorted(vals, torch.arange(V + 1, device="cuda")))


def test_embedding_bwd_large_vocab_uses_library_sort():
    """Above 16384 rows the backward keeps the library sort: still equal to index_add."""
    mod = _ext.require()
    torch.manual_seed(10)
    V, D, N = 20000, 64, 3000
    idx = torch.randint(0, V, (N,), device="cuda")
    g = torch.randn(N, D, device="cuda")
    dw = mod.embedding_bwd(g, idx, V, -1)
    ref = torch.zeros(V, D, device="cuda").index_add_(0, idx, g)
    torch.testing.assert_close(dw, ref, rtol=1e-5, atol=1e-5)
