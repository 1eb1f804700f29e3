"""The weight-shadow pack kernel (csrc/kernels/shadow_pack.hip) against the
torch copies it replaces: every layout the large-H LSTM / GRU and the 16-bit
heads read, in bf16 / fp16 / fp32, bit-exact (round-to-nearest-even like
torch's casts); a refresh after an optimizer step is one launch."""
import pytest
import torch

from pytorch_distributed_rnn_amd import _ext
from pytorch_distributed_rnn_amd.ops import shadow as sh
from pytorch_distributed_rnn_amd.ops.gru_large import _gru_shadows
from pytorch_distributed_rnn_amd.ops.lstm_large import _bias_cat, _shadow_cat, shadow

pytestmark = pytest.mark.gpu


def _interleaved(w, H):
    k = w.shape[1]
    return w.view(4, H, k).transpose(0, 1).reshape(4 * H, k)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("H,I", [(1024, 256), (1024, 1024), (128, 6), (100, 37)])
def test_pack_jobs_match_torch(dt, H, I):
    mod = _ext.require()
    torch.manual_seed(H + I)
    dev = "cuda"
    w = torch.randn(4 * H, I, device=dev) * 3
    w2 = torch.randn(4 * H, I, device=dev)
    b1, b2 = torch.randn(4 * H, device=dev), torch.randn(4 * H, device=dev)
    outs = [torch.empty(4 * H, I, device=dev, dtype=dt), torch.empty(I, 4 * H, device=dev, dtype=dt),
            torch.empty(4 * H, I, device=dev, dtype=dt), torch.empty(4 * H, device=dev, dtype=torch.float32)]
    jobs = [sh.job(outs[0].view(H, 4, I), w.view(4, H, I).transpose(0, 1)),
            sh.job(outs[1], w.t()),
            sh.job(outs[2], w, w2),
            sh.job(outs[3].view(H, 4), b1.view(4, H).t(), b2.view(4, H).t())]
    assert mod.shadow_pack(jobs) == 1
    torch.cuda.synchronize()
    assert torch.equal(outs[0], _interleaved(w, H).to(dt))
    assert torch.equal(outs[1], w.t().to(dt))
    assert torch.equal(outs[2], (w + w2).to(dt))
    assert torch.equal(outs[3], _interleaved((b1 + b2).view(-1, 1), H).view(-1))


def test_pack_over_sixteen_jobs_takes_two_launches():
    mod = _ext.require()
    src = torch.randn(40, 70, device="cuda")
    outs = [torch.empty(70, 40, device="cuda", dtype=torch.bfloat16) for _ in range(20)]
    assert mod.shadow_pack([sh.job(o, src.t()) for o in outs]) == 2
    for o in outs:
        assert torch.equal(o, src.t().to(torch.bfloat16))


def test_model_shadows_refresh_in_one_launch():
    """An LSTM layer's five layouts and a GRU's eleven pieces go stale in one
    optimizer step and come back in a single pack launch, equal to torch."""
    _ext.require()
    torch.manual_seed(3)
    H, I = 256, 64
    dev = "cuda"
    lw = [torch.nn.Parameter(torch.randn(4 * H, I, device=dev)), torch.nn.Parameter(torch.randn(4 * H, H, device=dev)),
          torch.nn.Parameter(torch.randn(4 * H, device=dev)), torch.nn.Parameter(torch.randn(4 * H, device=dev))]
    gw = [torch.nn.Parameter(torch.randn(3 * H, I, device=dev)), torch.nn.Parameter(torch.randn(3 * H, H, device=dev)),
          torch.nn.Parameter(torch.randn(3 * H, device=dev)), torch.nn.Parameter(torch.randn(3 * H, device=dev))]
    dt = torch.bfloat16

    def lookup():
        return (shadow(lw[0], "i", dt, H), shadow(lw[1], "i", dt, H), shadow(lw[1], "t", dt, H),
                shadow(lw[0], "p", dt, H), _bias_cat(lw, 1, H, lw[0].device), _gru_shadows(gw, 1, H, I, dt, dev))
    lookup()
    with torch.no_grad():
        for p in lw + gw:
            p.mul_(0.75)
    before = sh.stats()
    wi, whi, wt, wp, b, g = lookup()
    after = sh.stats()
    assert after["refreshes"] - before["refreshes"] == 1
    assert after["launches"] - before["launches"] == 1
    assert after["jobs"] - before["jobs"] == 5 + 11
    torch.cuda.synchronize()
    assert torch.equal(wi, _interleaved(lw[0].detach(), H).to(dt))
    assert torch.equal(whi, _interleaved(lw[1].detach(), H).to(dt))
    assert torch.equal(wt, lw[1].detach().t().to(dt))
    assert torch.equal(wp, lw[0].detach().to(dt))
    assert torch.equal(b, _interleaved((lw[2] + lw[3]).detach().view(-1, 1), H).view(-1))
    w_ih, w_hh, b_ih, b_hh = (w.detach() for w in gw)
    rec = torch.cat([w_hh[:2 * H], torch.zeros(H, H, device=dev), w_hh[2 * H:]])
    assert torch.equal(g[2][0], rec.to(dt)) and torch.equal(g[3][0], _interleaved(rec, H).to(dt))
    assert torch.equal(g[4][0], rec.t().to(dt))
    assert torch.equal(g[1], _interleaved(torch.cat([w_ih, torch.zeros(H, I, device=dev)]), H).to(dt))
    bias = torch.cat([b_ih[:2 * H] + b_hh[:2 * H], b_ih[2 * H:], b_hh[2 * H:]])
    assert torch.equal(g[5], _interleaved(bias.view(-1, 1), H).view(-1))


def test_pack_16bit_sources_and_stacked_states():
    """16-bit sources (the carried LSTM states): bf16 -> bf16 / fp32 exact,
    and a 2-layer large-H LSTM's stacked (hn, cn) equal the per-layer final
    states, with gradients through both reaching the layers."""
    mod = _ext.require()
    src = (torch.randn(2, 128, 1024, device="cuda") * 4).to(torch.bfloat16)
    a = torch.empty(2, 128, 1024, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(128, 2, 1024, device="cuda", dtype=torch.float32)
    assert mod.shadow_pack([sh.job(a, src), sh.job(b, src.transpose(0, 1))]) == 1
    torch.cuda.synchronize()
    assert torch.equal(a, src) and torch.equal(b, src.transpose(0, 1).float())

    from pytorch_distributed_rnn_amd.models.rnn import LSTM
    torch.manual_seed(7)
    m = LSTM(64, 1024, 2).cuda()
    x = torch.randn(6, 128, 64, device="cuda").to(torch.bfloat16).requires_grad_(True)
    out, (hn, cn) = m(x)
    assert hn.shape == (2, 128, 1024) and cn.shape == (2, 128, 1024)
    assert torch.equal(hn[1], out[-1])  # the top layer's last h
    (hn.float().sum() + cn.float().sum()).backward()
    assert x.grad is not None and torch.isfinite(x.grad.float()).all() and x.grad.float().abs().sum() > 0
    for p in m.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all()


def test_pack_vector_path_guards_alignment():
    """The 4-wide path (unit stride along i2 on both sides) and its guards:
    aligned slices take it, odd offsets / extents fall back to the LDS tile;
    both exact."""
    mod = _ext.require()
    src = torch.randn(96, 260, device="cuda")
    cases = [(slice(0, 256), slice(0, 256)),   # aligned: vector path
             (slice(1, 257), slice(3, 259)),   # odd offsets on both sides
             (slice(0, 255), slice(1, 256))]   # extent not a multiple of 4
    for dt in (torch.bfloat16, torch.float32):
        for ds_, ss_ in cases:
            out = torch.zeros(96, 260, device="cuda", dtype=dt)
            assert mod.shadow_pack([sh.job(out[:, ds_], src[:, ss_], src[:, ss_])]) == 1
            torch.cuda.synchronize()
            ref = torch.zeros(96, 260, device="cuda", dtype=dt)
            ref[:, ds_] = (src[:, ss_] + src[:, ss_]).to(dt)
            assert torch.equal(out, ref), (dt, ds_, ss_)
