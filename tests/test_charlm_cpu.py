"""Char-LM stack on the CPU: corpus layout, TBPTT state carry/reset, and the
DDP world-size invariance of the per-step loss (gloo, W=2)."""
import os
import re

import torch

from _mp import ROOT, run, torchrun
from pytorch_distributed_rnn_amd.data.charlm import CharCorpus
from pytorch_distributed_rnn_amd.models.charlm import BiLSTMEncoder, CharLM

from _tune import set_tune

_STEP = re.compile(r"Rank: (\d+)\s+Epoch 0 Step (\d+)\tLoss: ([\d.]+)")


def test_corpus_streams_and_segments():
    c = CharCorpus(torch.arange(1000), vocab_size=1000)
    s = c.streams(4)
    assert s.shape == (4, 250) and int(s[1, 0]) == 250
    r1 = c.streams(4, rank=1, world=2)
    assert torch.equal(r1, s[2:])
    segs = list(CharCorpus.segments(s, 10, limit=3))
    assert len(segs) == 3
    inp, tgt = segs[1]
    assert torch.equal(tgt[:, :-1], inp[:, 1:]) and int(inp[0, 0]) == 10


def test_synthetic_corpus_is_learnable_shape():
    c = CharCorpus.synthetic(5000, 64, seed=1)
    assert len(c) == 5000 and int(c.tokens.max()) < 64 and int(c.tokens.min()) >= 0
    assert (c.tokens == 0).float().mean() > 0.05  # separators present


def test_tbptt_carry_and_reset():
    torch.manual_seed(0)
    m = CharLM(32, 8, 16, 2)
    tok = torch.randint(0, 32, (3, 5))
    a = m(tok, carry=True)
    b = m(tok, carry=True)          # continues from a's final state
    m.reset_hidden_state()
    c = m(tok, carry=True)
    assert a.shape == (5, 3, 32)
    assert torch.allclose(a, c) and not torch.allclose(a, b)


def test_bilstm_encoder_shape():
    m = BiLSTMEncoder(6, 8, 2, 3)
    assert m(torch.randn(7, 2, 6)).shape == (7, 2, 3)


def _losses(log):
    out = {}
    for m in _STEP.finditer(log):
        out.setdefault(int(m.group(1)), []).append(float(m.group(3)))
    return out


def test_lm_ddp_invariance(tmp_path):
    args = ["-m", "pytorch_distributed_rnn_amd.lm_cli", "--hidden", "16", "--embed", "8", "--seq-len", "16",
            "--batch-size", "8", "--synthetic-tokens", "4000", "--max-steps", "4", "--log-interval", "1",
            "--device", "cpu", "--vocab", "64"]
    local = _losses(run(["python"] + args + ["local"], cwd=ROOT))[0]
    dist = _losses(torchrun(args + ["distributed"], 2, cwd=ROOT))
    mean = [(a + b) / 2 for a, b in zip(dist[0], dist[1])]
    assert len(mean) == len(local) == 4
    for x, y in zip(mean, local):
        assert abs(x - y) < 5e-5, (mean, local)


def test_lm_checkpoint_resume(tmp_path):
    args = ["python", "-m", "pytorch_distributed_rnn_amd.lm_cli", "--hidden", "16", "--embed", "8", "--seq-len", "16",
            "--batch-size", "4", "--synthetic-tokens", "3000", "--max-steps", "3", "--log-interval", "0",
            "--device", "cpu", "--vocab", "64", "--checkpoint-directory", str(tmp_path)]
    run(args + ["local"], cwd=ROOT)
    ck = tmp_path / "charlm-epoch0.pt"
    assert ck.exists()
    state = torch.load(ck, weights_only=True)
    assert state["epoch"] == 1 and "embedding.weight" in state["model_state"]
    run(args + ["--resume", str(ck), "local"], cwd=ROOT)
    assert (tmp_path / "charlm-epoch1.pt").exists()


def test_lm_trainer_settle_is_a_no_op_on_cpu():
    """The deferred persistent-path verification (train/lm.py settle) only
    engages on a GPU in per-step verification mode; on the CPU a step returns
    its loss directly and settle() has nothing to confirm."""
    import torch
    from pytorch_distributed_rnn_amd.data.charlm import CharCorpus
    from pytorch_distributed_rnn_amd.models.charlm import CharLM
    from pytorch_distributed_rnn_amd.train.lm import LMTrainer
    torch.manual_seed(0)
    corpus = CharCorpus.synthetic(20_000, seed=1)
    tr = LMTrainer(CharLM(corpus.vocab_size, 16, 32, 1, 0.0, torch.float32), corpus, 4, 8, device=torch.device("cpu"),
                   log_interval=0)
    assert not tr._deferred_verify()
    inp, tgt = next(iter(CharCorpus.segments(tr.streams, 8, 1)))
    loss = tr.train_step(inp, tgt)
    assert torch.isfinite(loss) and tr.settle() == 0 and tr._pending == []


def test_gru_forward_sequences_per_workgroup_override(monkeypatch):
    """ops/lstm.py gru_fwd_nb: PDRNN_TUNE nb_fwd overrides the residency rule
    (which needs a GPU to count CUs; 1 without one)."""
    from pytorch_distributed_rnn_amd.ops.lstm import gru_fwd_nb
    set_tune(monkeypatch, nb_fwd="2")
    assert gru_fwd_nb(100, 32) == 2
    set_tune(monkeypatch, nb_fwd=None)
    import torch
    if not torch.cuda.is_available():
        assert gru_fwd_nb(1440, 32) == 1
    assert gru_fwd_nb(1440, 16) == 1


def test_gemm_helpers_accumulate_into_cpu():
    """ops/gemm.py mm_kk / col_sum ``accumulate_into`` (the direct-gradient
    sinks' products) on the torch fallback: the result is added into the
    given tensors."""
    from pytorch_distributed_rnn_amd.ops.gemm import col_sum, mm_kk
    torch.manual_seed(0)
    a, b, a2, b2 = torch.randn(40, 8), torch.randn(40, 6), torch.randn(10, 8), torch.randn(10, 6)
    o = torch.randn(8, 6)
    ref = o + a.t() @ b + a2.t() @ b2
    assert mm_kk([(a, b), (a2, b2)], accumulate_into=o) is o
    torch.testing.assert_close(o, ref)
    x = torch.randn(30, 5)
    o1, o2 = torch.randn(5), torch.randn(5)
    r1, r2 = o1 + x.sum(0), o2 + x.sum(0)
    col_sum(x, accumulate_into=[o1, o2])
    torch.testing.assert_close(o1, r1)
    torch.testing.assert_close(o2, r2)


def test_time_major_tokens_one_copy_for_shifted_windows():
    """LMTrainer._time_major: the overlapping (input, target) windows of one
    stream become sequence-major [T, B] tensors out of ONE [T + 1, B] copy;
    unrelated windows fall back to a transpose copy each."""
    from pytorch_distributed_rnn_amd.data.charlm import CharCorpus
    from pytorch_distributed_rnn_amd.train.lm import LMTrainer
    streams = torch.randint(0, 256, (4, 50))
    for inp, tgt in CharCorpus.segments(streams, 7, 3):
        a, b = LMTrainer._time_major(inp, tgt)
        assert torch.equal(a, inp.t()) and torch.equal(b, tgt.t())
        assert a.is_contiguous() and b.is_contiguous()
        assert a.untyped_storage().data_ptr() == b.untyped_storage().data_ptr()  # one buffer
    x, y = torch.randint(0, 9, (3, 5)), torch.randint(0, 9, (3, 5))
    a, b = LMTrainer._time_major(x, y)
    assert torch.equal(a, x.t()) and torch.equal(b, y.t())
