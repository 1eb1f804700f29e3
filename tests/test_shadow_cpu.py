"""Weight shadows (ops/shadow.py): the registry rebuilds every stale layout of
a device together after an optimizer step, the layouts equal the direct torch
formulas, and the registry keeps no parameter alive.  CPU: the jobs run as
torch copies (the GPU pack kernel is checked in test_gpu_shadow.py)."""
import gc
import weakref

import torch

from pytorch_distributed_rnn_amd.ops import shadow as sh
from pytorch_distributed_rnn_amd.ops.gru_large import _gru_shadows
from pytorch_distributed_rnn_amd.ops.lstm_large import _bias_cat, _shadow_cat, shadow


def _interleaved(w, H):
    k = w.shape[1]
    return w.view(4, H, k).transpose(0, 1).reshape(4 * H, k)


def test_lstm_shadows_match_formulas_and_refresh_together():
    torch.manual_seed(0)
    H, I = 8, 5
    w_ih = torch.nn.Parameter(torch.randn(4 * H, I))
    w_hh = torch.nn.Parameter(torch.randn(4 * H, H))
    b_ih = torch.nn.Parameter(torch.randn(4 * H))
    b_hh = torch.nn.Parameter(torch.randn(4 * H))
    w2 = torch.nn.Parameter(torch.randn(4 * H, I))
    dt = torch.bfloat16
    wi = shadow(w_ih, "i", dt, H)
    wt = shadow(w_hh, "t", dt, H)
    wp = shadow(w_ih, "p", dt, H)
    cat = _shadow_cat([w_ih, w2], dt, H)
    bias = _bias_cat([w_ih, w_hh, b_ih, b_hh], 1, H, w_ih.device)
    assert torch.equal(wi, _interleaved(w_ih.detach(), H).to(dt))
    assert torch.equal(wt, w_hh.detach().t().to(dt))
    assert torch.equal(wp, w_ih.detach().to(dt))
    assert torch.equal(cat, torch.cat([_interleaved(w_ih.detach(), H), _interleaved(w2.detach(), H)]).to(dt))
    assert torch.equal(bias, _interleaved((b_ih + b_hh).detach().view(4 * H, 1), H).view(-1))
    assert shadow(w_ih, "p", torch.float32, H).data_ptr() == w_ih.data_ptr()  # fp32 "p": the master
    # an optimizer-like in-place update of every master: the first lookup
    # rebuilds all stale shadows at once, the others are then fresh
    with torch.no_grad():
        for p in (w_ih, w_hh, b_ih, b_hh, w2):
            p.add_(0.5)
    before = sh.stats()
    wi2 = shadow(w_ih, "i", dt, H)
    mid = sh.stats()
    assert mid["refreshes"] == before["refreshes"] + 1 and mid["jobs"] - before["jobs"] >= 5
    assert wi2.data_ptr() == wi.data_ptr()  # rebuilt in place
    assert torch.equal(shadow(w_hh, "t", dt, H), w_hh.detach().t().to(dt))
    assert torch.equal(_bias_cat([w_ih, w_hh, b_ih, b_hh], 1, H, w_ih.device),
                       _interleaved((b_ih + b_hh).detach().view(4 * H, 1), H).view(-1))
    assert sh.stats()["refreshes"] == mid["refreshes"]  # nothing left stale
    assert torch.equal(sh.cast(w_ih, dt), w_ih.detach().to(dt))  # the same ("p", bf16) entry


def test_gru_shadows_match_formulas():
    torch.manual_seed(1)
    H, I, ndir = 4, 3, 2
    ws = []
    for _ in range(ndir):
        ws += [torch.nn.Parameter(torch.randn(3 * H, I)), torch.nn.Parameter(torch.randn(3 * H, H)),
               torch.nn.Parameter(torch.randn(3 * H)), torch.nn.Parameter(torch.randn(3 * H))]
    for step in range(2):
        if step:
            with torch.no_grad():
                for p in ws:
                    p.mul_(0.5)
        wih, wih4_all, whh4, whh_p, wt, b4_all = _gru_shadows(ws, ndir, H, I, torch.float32, "cpu")
        for d in range(ndir):
            w_ih, w_hh, b_ih, b_hh = (w.detach() for w in ws[4 * d:4 * d + 4])
            assert torch.equal(wih[d], w_ih)
            stack = torch.cat([w_ih, torch.zeros(H, I)])
            assert torch.equal(wih4_all[d * 4 * H:(d + 1) * 4 * H], _interleaved(stack, H))
            rec = torch.cat([w_hh[:2 * H], torch.zeros(H, H), w_hh[2 * H:]])
            assert torch.equal(whh4[d], rec)
            assert torch.equal(whh_p[d], _interleaved(rec, H))
            assert torch.equal(wt[d], rec.t())
            bias = torch.cat([b_ih[:2 * H] + b_hh[:2 * H], b_ih[2 * H:], b_hh[2 * H:]])
            assert torch.equal(b4_all[d * 4 * H:(d + 1) * 4 * H], _interleaved(bias.view(-1, 1), H).view(-1))


def test_registry_keeps_no_parameter_alive():
    w = torch.nn.Parameter(torch.randn(16, 4))
    shadow(w, "t", torch.bfloat16, 4)
    ref = weakref.ref(w)
    del w
    gc.collect()
    assert ref() is None
    assert sh.refresh(torch.device("cpu")) == 0


def test_job_orders_unit_stride_dims_into_the_tile():
    a = torch.empty(6, 4, 64)   # dst [H, 4, k]
    src = torch.empty(4, 6, 64).transpose(0, 1)
    d, s, _ = sh.job(a, src)
    assert d.stride(2) == 1 and s.stride(2) == 1 and d.shape[0] == 4  # the 4 gates outside the tile
    t = torch.empty(64, 32)
    d, s, _ = sh.job(t, torch.empty(32, 64).t())
    assert d.stride(2) == 1 and s.stride(1) == 1  # transpose: read along i1, write along i2
