"""Numerics of the HIP kernels vs plain PyTorch fp64/fp32 references (GPU only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from pytorch_distributed_rnn_amd import _ext
    return _ext.require()


def _make_lstm(I, H, NL, seed=0):
    torch.manual_seed(seed)
    return torch.nn.LSTM(I, H, NL, batch_first=True)


@pytest.mark.parametrize("H,NL,I", [(32, 2, 9), (32, 1, 32), (16, 3, 5), (64, 1, 40), (32, 4, 32)])
@pytest.mark.parametrize("B,T", [(3, 7), (180, 128)])
def test_lstm_small_fwd_bwd_matches_torch(H, NL, I, B, T):
    from pytorch_distributed_rnn_amd.ops.lstm import lstm_forward
    ref = _make_lstm(I, H, NL).double()
    x = torch.randn(B, T, I, dtype=torch.float64)
    out_ref, (hn_ref, cn_ref) = ref(x)
    g_out = torch.randn_like(out_ref)
    g_hn = torch.randn_like(hn_ref)
    (out_ref * g_out).sum().add_((hn_ref * g_hn).sum()).backward()

    dev = torch.device("cuda")
    ws = [p.detach().float().to(dev).requires_grad_() for p in ref.parameters()]
    xg = x.float().to(dev)
    out, hn, cn = lstm_forward(xg, ws, hidden=H, num_layers=NL, batch_first=True)
    assert torch.allclose(out.double().cpu(), out_ref, atol=2e-5, rtol=1e-4)
    assert torch.allclose(hn.double().cpu(), hn_ref, atol=2e-5, rtol=1e-4)
    assert torch.allclose(cn.double().cpu(), cn_ref, atol=2e-5, rtol=1e-4)
    loss = (out * g_out.float().to(dev)).sum() + (hn * g_hn.float().to(dev)).sum()
    loss.backward()
    for w, p in zip(ws, ref.parameters()):
        scale = p.grad.abs().max().item() + 1e-6
        err = (w.grad.double().cpu() - p.grad).abs().max().item()
        assert err / scale < 2e-4, (err, scale)


def test_lstm_small_seq_first_and_states():
    from pytorch_distributed_rnn_amd.ops.lstm import lstm_forward
    H, NL, I, B, T = 32, 2, 9, 5, 11
    ref = torch.nn.LSTM(I, H, NL).double()
    x = torch.randn(T, B, I, dtype=torch.float64, requires_grad=True)
    h0 = torch.randn(NL, B, H, dtype=torch.float64, requires_grad=True)
    c0 = torch.randn(NL, B, H, dtype=torch.float64, requires_grad=True)
    out_ref, (hn_ref, cn_ref) = ref(x, (h0, c0))
    (out_ref.sum() + hn_ref.pow(2).sum() + cn_ref.sum()).backward()
    dev = torch.device("cuda")
    ws = [p.detach().float().to(dev).requires_grad_() for p in ref.parameters()]
    xg = x.detach().float().to(dev).requires_grad_()
    h0g = h0.detach().float().to(dev).requires_grad_()
    c0g = c0.detach().float().to(dev).requires_grad_()
    out, hn, cn = lstm_forward(xg, ws, h0g, c0g, hidden=H, num_layers=NL, batch_first=False)
    assert torch.allclose(out.double().cpu(), out_ref, atol=2e-5)
    (out.sum() + hn.pow(2).sum() + cn.sum()).backward()
    assert torch.allclose(xg.grad.double().cpu(), x.grad, atol=1e-4)
    assert torch.allclose(h0g.grad.double().cpu(), h0.grad, atol=1e-4)
    assert torch.allclose(c0g.grad.double().cpu(), c0.grad, atol=1e-4)


def test_lstm_small_gather_index():
    from pytorch_distributed_rnn_amd.ops.lstm import lstm_forward
    H, NL, I = 32, 2, 9
    ref = torch.nn.LSTM(I, H, NL, batch_first=True)
    data = torch.randn(50, 16, I)
    idx = torch.randperm(50)[:20]
    out_ref, (hn_ref, _) = ref(data[idx])
    dev = torch.device("cuda")
    ws = [p.detach().to(dev) for p in ref.parameters()]
    with torch.no_grad():
        out, hn, cn = lstm_forward(data.to(dev), ws, hidden=H, num_layers=NL, batch_first=True,
                                   idx=idx.to(dev))
    assert torch.allclose(out.cpu(), out_ref.detach(), atol=2e-5)
    assert torch.allclose(hn.cpu(), hn_ref.detach(), atol=2e-5)


@pytest.mark.parametrize("N,C", [(1440, 6), (37, 1000), (4096, 256)])
def test_xent_matches_torch(N, C):
    from pytorch_distributed_rnn_amd.ops.xent import cross_entropy_with_stats
    logits = torch.randn(N, C, dtype=torch.float64) * 3
    labels = torch.randint(0, C, (N,))
    labels[::7] = -100
    lr = logits.clone().requires_grad_()
    ref = F.cross_entropy(lr, labels, ignore_index=-100)
    ref.backward()
    lg = logits.float().cuda().requires_grad_()
    loss, stats = cross_entropy_with_stats(lg, labels.cuda(), -100)
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-5
    valid = labels != -100
    assert stats[1].item() == valid.sum().item()
    assert stats[2].item() == ((logits.argmax(1) == labels) & valid).sum().item()
    assert torch.allclose(lg.grad.double().cpu(), lr.grad, atol=1e-7)


def test_fused_adam_matches_torch():
    from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
    from pytorch_distributed_rnn_amd.utils.flat import FlatParameters
    torch.manual_seed(0)
    m_ref = torch.nn.Sequential(torch.nn.Linear(9, 32), torch.nn.Linear(32, 6))
    m = torch.nn.Sequential(torch.nn.Linear(9, 32), torch.nn.Linear(32, 6)).cuda()
    m.load_state_dict(m_ref.state_dict())
    flat = FlatParameters(list(m.parameters()))
    opt_ref = torch.optim.Adam(m_ref.parameters(), lr=2.5e-3)
    opt = FusedAdam(m.parameters(), lr=2.5e-3)
    for _ in range(5):
        x = torch.randn(16, 9)
        opt_ref.zero_grad()
        m_ref(x).pow(2).mean().backward()
        opt_ref.step()
        opt.zero_grad()
        m(x.cuda()).pow(2).mean().backward()
        assert flat.grads_attached()
        opt.step()
    for p, q in zip(m.parameters(), m_ref.parameters()):
        assert torch.allclose(p.detach().cpu(), q.detach(), atol=1e-6, rtol=1e-5)
    sd = opt.state_dict()
    assert set(sd["state"][0].keys()) >= {"step", "exp_avg", "exp_avg_sq"}


def test_adam_flat_device_step_advance():
    """Advance mode (graph replay): the kernel uses device step + 1 for the bias
    corrections and the last workgroup writes it back -- over many workgroups,
    matching host-step launches, with the ticket re-armed every launch."""
    from pytorch_distributed_rnn_amd import _ext
    mod = _ext.require()
    torch.manual_seed(0)
    n = 1 << 20  # 1024 workgroups
    p0 = torch.randn(n, device="cuda")
    p1, p2 = p0.clone(), p0.clone()
    m1, v1 = torch.zeros_like(p0), torch.zeros_like(p0)
    m2, v2 = torch.zeros_like(p0), torch.zeros_like(p0)
    step_t = torch.zeros(1, device="cuda")
    ticket = torch.zeros(1, dtype=torch.int32, device="cuda")
    for s in range(1, 5):
        g = torch.randn(n, device="cuda")
        mod.adam_flat(p1, g, m1, v1, None, 1e-2, 0.9, 0.999, 1e-8, 0.0, float(s), 1.0, False, False)
        mod.adam_flat(p2, g, m2, v2, None, 1e-2, 0.9, 0.999, 1e-8, 0.0, 0.0, 1.0, False, False,
                      None, step_t, ticket)
        torch.cuda.synchronize()
        assert float(step_t) == float(s) and int(ticket) == 0
    # bias corrections in fp32 on the device vs double on the host
    torch.testing.assert_close(p2, p1, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v2, v1, rtol=0, atol=0)


def test_adam_flat_skip_word():
    """The device skip word (deferred persistent-path verification): nonzero
    -> the launch changes nothing; zero -> an ordinary step."""
    from pytorch_distributed_rnn_amd import _ext
    mod = _ext.require()
    torch.manual_seed(0)
    n = 1 << 18
    p = torch.randn(n, device="cuda")
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    p0 = p.clone()
    g = torch.randn(n, device="cuda")
    skip = torch.ones(1, dtype=torch.int32, device="cuda")
    mod.adam_flat(p, g, m, v, None, 1e-2, 0.9, 0.999, 1e-8, 0.0, 1.0, 1.0, False, False, None, None, None, skip)
    torch.cuda.synchronize()
    assert torch.equal(p, p0) and int(m.abs().sum()) == 0 and int(v.abs().sum()) == 0
    skip.zero_()
    mod.adam_flat(p, g, m, v, None, 1e-2, 0.9, 0.999, 1e-8, 0.0, 1.0, 1.0, False, False, None, None, None, skip)
    ref = p0.clone()
    m2, v2 = torch.zeros_like(p), torch.zeros_like(p)
    mod.adam_flat(ref, g, m2, v2, None, 1e-2, 0.9, 0.999, 1e-8, 0.0, 1.0, 1.0, False, False)
    torch.cuda.synchronize()
    assert torch.equal(p, ref)


@pytest.mark.parametrize("n,scale", [(1000, 1.0), (14150, 50.0), (3 << 20, 0.001)])
def test_clip_flat_matches_torch(n, scale):
    """In-place gradient-norm clipping (kernels/adam.hip, the LM trainer's
    clip) vs the torch formula: norm in fp32, scale = min(1, c / (norm + eps))."""
    from pytorch_distributed_rnn_amd import _ext
    mod = _ext.require()
    torch.manual_seed(n)
    g = torch.randn(n, device="cuda") * scale
    ref = g.double()
    norm = ref.norm()
    ref = ref * torch.clamp(1.0 / (norm + 1e-6), max=1.0)
    out = mod.clip_flat(g, 1.0, 1e-6)
    torch.cuda.synchronize()
    torch.testing.assert_close(out[1].double(), norm, rtol=1e-5, atol=0)
    torch.testing.assert_close(g.double(), ref, rtol=1e-5, atol=1e-9)
    g2 = torch.randn(n, device="cuda") * scale
    a, b = g2.clone(), g2.clone()
    mod.clip_flat(a, 1.0, 1e-6)
    mod.clip_flat(b, 1.0, 1e-6)
    assert torch.equal(a, b)  # deterministic


def test_embedding_matches_torch():
    C = _C()
    V, D, N = 97, 64, 5000
    w = torch.randn(V, D)
    idx = torch.randint(0, V, (N,))
    out = C.embedding_fwd(w.cuda(), idx.cuda())
    assert torch.equal(out.cpu(), w[idx])
    g = torch.randn(N, D)
    dw = C.embedding_bwd(g.cuda(), idx.cuda(), V, -1)
    ref = torch.zeros(V, D, dtype=torch.float64).index_add_(0, idx, g.double())
    assert torch.allclose(dw.double().cpu(), ref, atol=1e-4)


@pytest.mark.parametrize("V", [16129, 16384])
def test_embedding_backward_at_the_in_tree_sort_limit(V):
    """the in-tree counting sort serves V <= 16384; its scatter
    stages V counters plus a key tile in LDS, past 64 KiB from V = 16129 (the
    launch opts into the larger limit)."""
    C = _C()
    D, N = 32, 20000
    torch.manual_seed(V)
    idx = torch.randint(0, V, (N,))
    g = torch.randn(N, D)
    dw = C.embedding_bwd(g.cuda(), idx.cuda(), V, -1)
    ref = torch.zeros(V, D, dtype=torch.float64).index_add_(0, idx, g.double())
    assert torch.allclose(dw.double().cpu(), ref, atol=1e-4)


@pytest.mark.parametrize("H,NL,I,B,T,bf", [(32, 2, 9, 37, 40, True), (16, 1, 5, 8, 33, False),
                                          (64, 2, 64, 6, 12, True), (32, 3, 32, 5, 20, True)])
def test_fused_gru_matches_torch(H, NL, I, B, T, bf):
    from pytorch_distributed_rnn_amd.models.rnn import GRU
    torch.manual_seed(11)
    m = GRU(I, H, NL, batch_first=bf).cuda()
    ref = torch.nn.GRU(I, H, NL, batch_first=bf).cuda().double()
    with torch.no_grad():
        for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
            q.copy_(p.double())
    x = torch.randn(B, T, I, device="cuda") if bf else torch.randn(T, B, I, device="cuda")
    h0 = torch.randn(NL, B, H, device="cuda")
    xa, h0a = x.clone().requires_grad_(True), h0.clone().requires_grad_(True)
    xb, h0b = x.double().clone().requires_grad_(True), h0.double().clone().requires_grad_(True)
    out, hn = m(xa, h0a)
    out_r, hn_r = ref(xb, h0b)
    torch.testing.assert_close(out.double(), out_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(hn.double(), hn_r, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out_r)
    ((out.double() * g).sum() + hn.double().sum()).backward()
    ((out_r * g).sum() + hn_r.sum()).backward()
    torch.testing.assert_close(xa.grad.double(), xb.grad, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(h0a.grad.double(), h0b.grad, rtol=1e-3, atol=1e-4)
    for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        torch.testing.assert_close(p.grad.double(), q.grad, rtol=1e-3, atol=2e-4, msg=n)


def test_fused_gru_really_runs():
    # the HIP path, not the ATen fallback, must serve this shape
    from pytorch_distributed_rnn_amd.ops import gru_fused
    x = torch.randn(4, 10, 9, device="cuda")
    assert gru_fused.supported(x, 32, 2)
