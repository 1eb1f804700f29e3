"""GPU: the fused whole-step path equals the autograd path (same math)."""
import copy

import pytest
import torch

from _tune import set_tune

pytestmark = pytest.mark.gpu


def _trainer(model, data, fused: bool):
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    t = Trainer(model, data, batch_size=96, learning_rate=2.5e-3, device=torch.device("cuda"))
    if not fused:
        t._fused = None  # force the autograd path
    return t


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_fused_step_matches_autograd(cell):
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    torch.manual_seed(0)
    train, _, _ = synthetic_motion(n_train=384, n_validation=2, n_test=2, seed=3)
    m1 = MotionModel(9, 32, 2, 6, cell=cell)
    m2 = copy.deepcopy(m1)
    t1, t2 = _trainer(m1, train, True), _trainer(m2, train, False)
    assert t1._fused_step() is not None, "fused step not selected on GPU"
    b1, b2 = list(t1.train_loader), list(t2.train_loader)
    for x1, x2 in zip(b1, b2):
        s1, n1 = t1.train_batch(x1)
        s2, n2 = t2.train_batch(x2)
        assert n1 == n2
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
        assert int(s1[2]) == int(s2[2])
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


@pytest.mark.parametrize("cell,hidden,layers", [("lstm", 16, 1), ("lstm", 32, 3), ("lstm", 16, 4),
                                                 ("gru", 16, 2), ("gru", 32, 1)])
def test_one_launch_step_shapes_match_autograd(cell, hidden, layers):
    """The one-launch step (B = 64: one sequence per workgroup) at other
    hidden sizes / depths equals the autograd step."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    torch.manual_seed(1)
    train, _, _ = synthetic_motion(n_train=128, n_validation=2, n_test=2, seed=5)
    m1 = MotionModel(9, hidden, layers, 6, cell=cell)
    m2 = copy.deepcopy(m1)
    t1 = Trainer(m1, train, batch_size=64, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2 = Trainer(m2, train, batch_size=64, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2._fused = None
    if t1._fused_step() is None:
        pytest.skip("fused step does not cover this shape")
    mod = _ext.native(torch.device("cuda", 0))
    assert mod.lstm_small_step_one_launch(hidden, layers, 128, 64, 1, 0, 1, 0)
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
        assert int(s1[2]) == int(s2[2])
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


def test_one_launch_step_selected_in_latency_regime():
    """B <= one resident round: forward + head/CE + BPTT run as one launch
    (the B=96 runs of test_fused_step_matches_autograd go through it); the
    headline B=1440 keeps the separate launches."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.ops.lstm import fused_bwd_nb, small_launch_config
    mod = _ext.native(torch.device("cuda", 0))
    for b, expect in ((96, True), (180, True), (1440, False)):
        nb_f, sp_f, _, sp_b = small_launch_config(b, 32, 2)
        got = mod.lstm_small_step_one_launch(32, 2, 128, b, nb_f, sp_f, fused_bwd_nb(b, 32, 2), sp_b)
        assert got == expect, (b, got)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("nb", [2, 3])
def test_fused_multi_sequence_backward_matches_autograd(cell, nb, monkeypatch):
    """Sequences interleaved in one workgroup of the fused step's register-dW
    backward (PDRNN_TUNE nb_bwd; the GRU stays single-sequence) against the
    autograd path; 380 samples in batches of 96 leave a last batch of 92, so
    tiles with unused slots run."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, nb_bwd=str(nb))
    torch.manual_seed(1)
    train, _, _ = synthetic_motion(n_train=380, n_validation=2, n_test=2, seed=4)
    m1 = MotionModel(9, 32, 2, 6, cell=cell)
    m2 = copy.deepcopy(m1)
    t1, t2 = _trainer(m1, train, True), _trainer(m2, train, False)
    assert t1._fused_step() is not None
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


@pytest.mark.parametrize("nb", [1, 3])
def test_fused_step_headline_batch_matches_autograd(nb, monkeypatch):
    """B = 1440 (the headline per-GPU batch): the deferred-dW backward (nb 1)
    and the register-dW backward with 3 sequences per workgroup."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    set_tune(monkeypatch, nb_bwd=str(nb))
    torch.manual_seed(2)
    train, _, _ = synthetic_motion(n_train=2880, n_validation=2, n_test=2, seed=5)
    m1 = MotionModel(9, 32, 2, 6)
    m2 = copy.deepcopy(m1)
    t1 = Trainer(m1, train, batch_size=1440, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2 = Trainer(m2, train, batch_size=1440, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2._fused = None
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


def test_fused_gru_step_headline_batch_matches_autograd():
    """GRU at B = 1440 and its short batch 1128: above one residency round
    the gate-split forward takes two sequences per workgroup (ops/lstm.py
    gru_fwd_nb) -- against the autograd path on the same kernels' math."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.ops.lstm import gru_fwd_nb
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    assert gru_fwd_nb(1440, 32) == 2
    torch.manual_seed(3)
    train, _, _ = synthetic_motion(n_train=2568, n_validation=2, n_test=2, seed=6)
    m1 = MotionModel(9, 32, 2, 6, cell="gru")
    m2 = copy.deepcopy(m1)
    t1 = Trainer(m1, train, batch_size=1440, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2 = Trainer(m2, train, batch_size=1440, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2._fused = None
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


@pytest.mark.parametrize("cell,hidden,layers,seq,features", [
    ("lstm", 32, 2, 128, 9), ("lstm", 16, 1, 37, 9), ("lstm", 32, 3, 21, 5),
    ("lstm", 16, 2, 6, 16), ("gru", 32, 2, 128, 9), ("gru", 16, 2, 9, 3)])
def test_deferred_dw_backward_matches_autograd(cell, hidden, layers, seq, features, monkeypatch):
    """The BPTT with the weight gradients deferred to the matrix-core kernel
    (lstm_small_dw.hip) -- forced at B = 96 so that every shape runs it; 382
    samples leave a last batch of 94 (with odd T: B*T not a multiple of the
    4-row MFMA step), T from 6 to 128, chunks straddling sequences, 3..16
    input features (x tiles masked)."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, dwout="force")
    assert _ext.native(torch.device("cuda")).lstm_small_step_deferred_dw(hidden, layers, seq, 96)
    torch.manual_seed(3)
    train, _, _ = synthetic_motion(n_train=382, n_validation=2, n_test=2, seq_length=seq, num_features=features,
                                   seed=6)
    m1 = MotionModel(features, hidden, layers, 6, cell=cell)
    m2 = copy.deepcopy(m1)
    t1, t2 = _trainer(m1, train, True), _trainer(m2, train, False)
    if t1._fused_step() is None:
        pytest.skip("fused step does not cover this shape")
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
        assert int(s1[2]) == int(s2[2])
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


def _fused_grads(model, train, B):
    """Gradients of one fused step (no optimizer update) on the first batch."""
    from pytorch_distributed_rnn_amd.ops.lstm import fused_bwd_nb, small_launch_config
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    t = Trainer(model, train, batch_size=B, learning_rate=2.5e-3, device=torch.device("cuda"))
    f = t._fused_step()
    assert f is not None
    feats, labels, idx = t.train_loader.make_batch(t.train_loader.batch_indices()[0])
    nb_f, sp_f, _, _ = small_launch_config(idx.numel(), f.H, f.NL)
    ws = f.weights
    if f.gru:
        from pytorch_distributed_rnn_amd.ops.gru_fused import _pack
        ws = _pack(f.weights, f.NL, f.H, f.flat.data)
        nb_f, sp_f = 1, 1
    f.flat.attach_grads()
    stats = torch.zeros(3, device="cuda")
    f.mod.lstm_head_train_step(feats, idx, labels, ws, f.m.fc.weight, f.m.fc.bias, f.flat.grad, stats, f.H, f.NL,
                               sp_f, 0, nb_f, fused_bwd_nb(idx.numel(), f.H, f.NL), None, None,
                               1 if f.gru else 0, f.colmap)
    return [p.grad.detach().double() for p in f.m.parameters()], feats.index_select(0, idx), \
        labels.index_select(0, idx).reshape(-1)


@pytest.mark.parametrize("cell,hidden,layers,seq", [("lstm", 64, 1, 16), ("lstm", 32, 2, 128), ("gru", 64, 1, 12)])
def test_deferred_dw_gradients_match_fp64(cell, hidden, layers, seq, monkeypatch):
    """Gradients of the deferred-dW step (before Adam) against fp64 autograd:
    max error <= 2e-6 of each parameter's largest gradient (the Adam-trajectory
    test above cannot take H = 64 at T = 16: Adam's first step is sign(g) * lr,
    so elements whose gradient is at rounding level flip either way)."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, dwout="force")
    torch.manual_seed(3)
    train, _, _ = synthetic_motion(n_train=190, n_validation=2, n_test=2, seq_length=seq, seed=6)
    m0 = MotionModel(9, hidden, layers, 6, cell=cell)
    grads, x, y = _fused_grads(copy.deepcopy(m0), train, 95)
    ref = copy.deepcopy(m0).cuda().double()
    torch.nn.functional.cross_entropy(ref(x.double()), y).backward()
    for (k, r), g in zip(ref.named_parameters(), grads):
        scale = r.grad.abs().max().item()
        assert (g - r.grad).abs().max().item() <= 2e-6 * scale + 1e-12, k


@pytest.mark.parametrize("B,nb", [(1440, "2"), (1152, "2"), (1440, "1")])
def test_headline_batch_gradients_match_fp64(B, nb, monkeypatch):
    """The headline step at the epoch's two batch sizes (1440 and the short
    last 1152 of a 6912-sequence epoch): gradients of the fused HIP step
    (deferred-dW BPTT with one or two sequences per workgroup; the weight
    gradients formed by the matrix-core launch over 256 K chunks; the
    one-pass slab reduction) before Adam against fp64 torch autograd on the same weights
    and batch -- an oracle independent of the HIP kernels."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, dwout=None)
    monkeypatch.setenv("PDRNN_SW", "0")  # the gate-split / K-split family (sequence-in-wave: test below)
    set_tune(monkeypatch, dwout_nb=nb)
    mod = _ext.native(torch.device("cuda", 0))
    assert mod.lstm_small_step_deferred_dw(32, 2, 128, B)
    torch.manual_seed(11)
    train, _, _ = synthetic_motion(n_train=B, n_validation=2, n_test=2, seed=12)
    m0 = MotionModel(9, 32, 2, 6)
    grads, x, y = _fused_grads(copy.deepcopy(m0), train, B)
    ref = copy.deepcopy(m0).cuda().double()
    torch.nn.functional.cross_entropy(ref(x.double()), y).backward()
    for (k, r), g in zip(ref.named_parameters(), grads):
        scale = r.grad.abs().max().item()
        assert (g - r.grad).abs().max().item() <= 2e-6 * scale + 1e-12, k


def _fp64_check(m0, train, B, tol=2e-6):
    grads, x, y = _fused_grads(copy.deepcopy(m0), train, B)
    ref = copy.deepcopy(m0).cuda().double()
    torch.nn.functional.cross_entropy(ref(x.double()), y).backward()
    for (k, r), g in zip(ref.named_parameters(), grads):
        scale = r.grad.abs().max().item()
        assert (g - r.grad).abs().max().item() <= tol * scale + 1e-12, k


@pytest.mark.parametrize("B,layers,mode", [(1440, 2, ""), (1152, 2, ""), (720, 2, ""), (360, 2, ""), (180, 2, ""),
                                           (144, 2, ""), (97, 2, ""), (1440, 2, "2"), (180, 2, "3"),
                                           (97, 2, "6"), (720, 2, "3/2"), (1152, 2, "2/3"), (360, 2, "6/2"), (180, 2, "2/2"), (512, 2, "2/4"), (97, 2, "5/2"), (360, 2, "5/3"),
                                           (180, 1, ""), (1440, 1, ""), (180, 2, "0")])
def test_seq_in_wave_step_gradients_match_fp64(B, layers, mode, monkeypatch):
    """The sequence-in-wave step (kernels/lstm_sw.hip: each sequence's
    recurrence inside one wave, or one wave per layer; deferred matrix-core
    dW; one-pass reduction) at every per-rank batch of the 1/2/4/8-GPU
    strong-scaling runs (1440 / 720 / 360 / 180, and the epoch's short last
    batches 1152 / 144), an odd batch (a half-empty two-sequence wave), each
    wave map forced once, and the single-layer config-2 shape: gradients
    before Adam against fp64 torch autograd on the same weights and batch."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    monkeypatch.delenv("PDRNN_SW", raising=False)
    fm, _, bm = mode.partition("/")  # "F/B": forward and backward maps forced apart
    set_tune(monkeypatch, sw_mode=fm or None, sw_bwd_mode=bm or None)
    mod = _ext.native(torch.device("cuda", 0))
    assert mod.lstm_sw_ok(32, 9, layers, 0)
    torch.manual_seed(13 + B)
    train, _, _ = synthetic_motion(n_train=B, n_validation=2, n_test=2, seed=14)
    _fp64_check(MotionModel(9, 32, layers, 6), train, B)


@pytest.mark.parametrize("B,layers,mode", [(1440, 2, ""), (1152, 2, ""), (720, 2, ""), (512, 2, ""), (180, 2, ""),
                                           (144, 2, ""), (97, 2, ""), (1440, 2, "2"), (180, 2, "3"), (97, 2, "6/3"),
                                           (180, 2, "2/2"), (360, 2, "5/3"), (512, 2, "2/4"),
                                           (180, 1, ""), (1440, 1, ""), (97, 1, "1")])
def test_seq_in_wave_gru_step_gradients_match_fp64(B, layers, mode, monkeypatch):
    """The GRU on the sequence-in-wave map (kernels/lstm_sw.hip, CELL = 1:
    the packed 4-block stack's products on the LSTM lanes, n = tanh(n_x + r
    n_h) and h = n + z (h_prev - n) after two DPP swaps; BPTT row phase with
    the direct dh z path; deferred matrix-core dW) at the headline / short /
    per-rank batches (B <= 512: the one-launch four-wave forward + register-dW
    BPTT) and forced wave maps: gradients before Adam against fp64 nn.GRU
    autograd on the same weights and batch."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    monkeypatch.delenv("PDRNN_SW", raising=False)
    fm, _, bm = mode.partition("/")
    set_tune(monkeypatch, sw_mode=fm or None, sw_bwd_mode=bm or None)
    mod = _ext.native(torch.device("cuda", 0))
    assert mod.lstm_sw_ok(32, 9, layers, 1)
    torch.manual_seed(17 + B)
    train, _, _ = synthetic_motion(n_train=B, n_validation=2, n_test=2, seed=18)
    _fp64_check(MotionModel(9, 32, layers, 6, cell="gru"), train, B)


@pytest.mark.parametrize("cell", ["lstm", "gru"])
@pytest.mark.parametrize("B", [512, 180, 97])
def test_seq_in_wave_latency_regime_separate_launches_match_fp64(B, cell, monkeypatch):
    """The latency regime (forward mode 5, backward mode 4) as separate
    forward / BPTT launches (PDRNN_SW=2) against fp64 autograd; the default
    one-launch step runs at every B <= 512 of the parametrisation above."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, sw_mode=None, sw_bwd_mode=None)
    monkeypatch.setenv("PDRNN_SW", "2")
    mod = _ext.native(torch.device("cuda", 0))
    assert mod.lstm_sw_step_ok(2, B, 128)
    torch.manual_seed(31 + B)
    train, _, _ = synthetic_motion(n_train=B, n_validation=2, n_test=2, seed=32)
    _fp64_check(MotionModel(9, 32, 2, 6, cell=cell), train, B)


def test_one_launch_sw_step_selection():
    """The one-launch step (forward + BPTT in one kernel) covers two-layer
    stacks up to two workgroups per CU (B <= 512 on 256 CUs) at T % 4 == 0;
    the headline batch keeps the separate launches."""
    from pytorch_distributed_rnn_amd import _ext
    mod = _ext.native(torch.device("cuda", 0))
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for B in (97, 144, 180, 360, 2 * cus):
        assert mod.lstm_sw_step_ok(2, B, 128), B
    for B, T in ((2 * cus + 1, 128), (720, 128), (1440, 128), (180, 126)):
        assert not mod.lstm_sw_step_ok(2, B, T), (B, T)


def test_seq_in_wave_batch_past_descriptor_range_falls_back(monkeypatch):
    """the sequence-in-wave kernels address every act / hseq row as
    a 32-bit offset under one 2 GiB buffer descriptor.  A batch whose rows
    pass that range (NL * B * T * 640 B >= 2^31: B = 13200 at T = 128) must
    take the per-sequence-rebased kernel family, and its gradients must still
    match fp64 autograd."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    monkeypatch.delenv("PDRNN_SW", raising=False)
    mod = _ext.native(torch.device("cuda", 0))
    B = 13200
    assert mod.lstm_sw_fits(2, 13000, 128) and not mod.lstm_sw_fits(2, B, 128)
    torch.manual_seed(17)
    train, _, _ = synthetic_motion(n_train=B, n_validation=2, n_test=2, seed=18)
    _fp64_check(MotionModel(9, 32, 2, 6), train, B, tol=4e-6)


@pytest.mark.parametrize("cell,B", [("gru", 180), ("gru", 144), ("lstm", 180), ("lstm", 144)])
def test_one_launch_gradients_match_fp64(cell, B, monkeypatch):
    """the one-launch step kernel (lstm_small_step_gs_kernel,
    forward + head/CE + register-dW BPTT per workgroup) at the 8-GPU epoch's
    per-rank batches against fp64 autograd: the GRU's path, and the LSTM's
    with the sequence-in-wave kernels switched off (PDRNN_SW=0)."""
    from pytorch_distributed_rnn_amd import _ext
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.ops.lstm import fused_bwd_nb, small_launch_config
    monkeypatch.setenv("PDRNN_SW", "0")
    set_tune(monkeypatch, dwout=None)
    mod = _ext.native(torch.device("cuda", 0))
    nb_f, sp_f, _, sp_b = small_launch_config(B, 32, 2)
    if cell == "gru":
        nb_f, sp_f = 1, 1
    assert mod.lstm_small_step_one_launch(32, 2, 128, B, nb_f, sp_f, fused_bwd_nb(B, 32, 2), sp_b)
    torch.manual_seed(21 + B)
    train, _, _ = synthetic_motion(n_train=B, n_validation=2, n_test=2, seed=22)
    _fp64_check(MotionModel(9, 32, 2, 6, cell=cell), train, B)


def test_deferred_dw_pairs_sequences_at_headline_batch(monkeypatch):
    """B = 1440 / 1152: two sequences per workgroup of the deferred-dW BPTT,
    all of them resident in one round (the grid fits the occupancy)."""
    from pytorch_distributed_rnn_amd import _ext
    set_tune(monkeypatch, dwout_nb=None)
    mod = _ext.native(torch.device("cuda", 0))
    for B in (1440, 1152):
        nb, grid = mod.lstm_small_dwout_geometry(32, 2, 128, B)
        assert (nb, grid) == (2, B // 2), (B, nb, grid)


def test_deferred_dw_selected_above_one_round(monkeypatch):
    """Default selection: the headline B = 1440 (three residency rounds of the
    register-dW backward) takes the deferred-dW path, the 8-GPU per-rank batch
    (180, one round) keeps the one-launch step."""
    from pytorch_distributed_rnn_amd import _ext
    set_tune(monkeypatch, dwout=None)
    mod = _ext.native(torch.device("cuda", 0))
    assert mod.lstm_small_step_deferred_dw(32, 2, 128, 1440)
    assert not mod.lstm_small_step_deferred_dw(32, 2, 128, 180)
    set_tune(monkeypatch, dwout="0")
    assert not mod.lstm_small_step_deferred_dw(32, 2, 128, 1440)


def test_deferred_dw_bf16_inputs_match_autograd(monkeypatch):
    """bf16 inputs (BASELINE config 2) through the deferred-dW backward: the dW
    kernel widens the gathered bf16 x rows itself."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    set_tune(monkeypatch, dwout="force")
    torch.manual_seed(0)
    train, _, _ = synthetic_motion(n_train=384, n_validation=2, n_test=2, seed=3)
    m1 = MotionModel(9, 32, 1, 6, compute_dtype=torch.bfloat16)
    m2 = copy.deepcopy(m1)
    t1, t2 = _trainer(m1, train, True), _trainer(m2, train, False)
    assert t1._fused_step() is not None and t1.train_loader.features.dtype == torch.bfloat16
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


def test_local_trainer_epoch_on_gpu(tmp_path):
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    torch.manual_seed(1)
    train, val, test = synthetic_motion(n_train=960, n_validation=96, n_test=96, seed=1)
    t = Trainer(MotionModel(9, 32, 2, 6), train, batch_size=480, learning_rate=2.5e-3,
                validation_set=val, test_set=test, checkpoint_dir=tmp_path)
    _, th, vh = t.train(3)
    assert len(th) == 3 and len(vh) == 3
    assert (tmp_path / "best-model.pt").exists()
    ck = torch.load(tmp_path / "best-model.pt", weights_only=True)
    assert "lstm.weight_ih_l0" in ck["model_state"]


def test_bf16_fused_step_matches_autograd():
    """BASELINE config 2: single-layer motion model, bf16 inputs/recurrent
    weights, fused whole-step path == autograd path."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    torch.manual_seed(0)
    train, _, _ = synthetic_motion(n_train=384, n_validation=2, n_test=2, seed=3)
    m1 = MotionModel(9, 32, 1, 6, compute_dtype=torch.bfloat16)
    m2 = copy.deepcopy(m1)
    t1, t2 = _trainer(m1, train, True), _trainer(m2, train, False)
    assert t1._fused_step() is not None and t1.train_loader.features.dtype == torch.bfloat16
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=2e-5, rtol=1e-4), k


def test_bf16_lstm_matches_rounded_fp64_reference():
    from pytorch_distributed_rnn_amd.models.rnn import LSTM
    torch.manual_seed(2)
    m = LSTM(9, 32, 1, batch_first=True).cuda()
    ref = torch.nn.LSTM(9, 32, 1, batch_first=True).cuda().double()
    with torch.no_grad():
        for p, q in zip(m.parameters(), ref.parameters()):
            q.copy_(p.to(torch.bfloat16).double())
    x = torch.randn(20, 128, 9, device="cuda").to(torch.bfloat16)
    out, (hn, _) = m(x)
    out_r, (hn_r, _) = ref(x.double())
    torch.testing.assert_close(out.double(), out_r, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(hn.double(), hn_r, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("T", [126, 61])
def test_seq_in_wave_short_sequences_fall_back_from_mode4(T, monkeypatch):
    """Backward mode 4 (the BPTT workgroups form their own weight gradients)
    takes K steps of 4 time steps: at T % 4 != 0 the binding runs mode 2 plus
    the dW kernel instead -- gradients against fp64 at B = 180 for such T."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    monkeypatch.delenv("PDRNN_SW", raising=False)
    set_tune(monkeypatch, sw_mode=None, sw_bwd_mode=None)
    torch.manual_seed(21)
    train, _, _ = synthetic_motion(n_train=180, n_validation=2, n_test=2, seq_length=T, seed=22)
    _fp64_check(MotionModel(9, 32, 2, 6), train, 180)


@pytest.mark.parametrize("cell", ["lstm"])
def test_direct_grads_match_autograd_accumulation(cell):
    """fp32 H = 128 motion model on the autograd path: the stacked-layer
    pipeline and the narrow head accumulating their weight gradients straight
    into the flat .grad views (ops/gradsink.py, single process) against the
    same steps with autograd adding returned gradients -- equal parameters
    after a few steps and equal gradients of one backward."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.ops import gradsink
    from pytorch_distributed_rnn_amd.train.trainer import Trainer
    torch.manual_seed(6)
    train, _, _ = synthetic_motion(n_train=160, n_validation=2, n_test=2, seed=9)
    m1 = MotionModel(9, 128, 2, 6, cell=cell)
    m2 = copy.deepcopy(m1)
    t1 = Trainer(m1, train, batch_size=64, learning_rate=2.5e-3, device=torch.device("cuda"))
    t2 = Trainer(m2, train, batch_size=64, learning_rate=2.5e-3, device=torch.device("cuda"))
    t1._fused = t2._fused = None
    assert t1._direct_grads_ok()
    t2._direct_grads_ok = lambda: False
    for x1, x2 in zip(list(t1.train_loader), list(t2.train_loader)):
        s1, _ = t1.train_batch(x1)
        s2, _ = t2.train_batch(x2)
        assert abs(float(s1[0]) - float(s2[0])) < 1e-5
    for (k, p), q in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=1e-6, rtol=1e-5), k
    # the Functions wrote the flat views themselves: with direct mode on, a
    # backward leaves exactly the reference gradient in them
    x = next(iter(t1.train_loader))
    grads = []
    for on in (True, False):
        t1.optimizer.zero_grad()
        with gradsink.direct_grads(on):
            out, lab = t1._forward(x)
            t1.loss_fn(out, lab.long().reshape(-1)).backward()
        grads.append([p.grad.clone() for p in m1.parameters()])
    for (k, _), g1, g2 in zip(m1.named_parameters(), *grads):
        assert torch.allclose(g1, g2, atol=1e-7, rtol=1e-5), k


@pytest.mark.parametrize("n_train,bs", [(448, 96), (6912, 1440)])
def test_single_process_epoch_graph_matches_eager(n_train, bs):
    """One process: every step of an epoch replayed as ONE HIP graph (fused
    step with Adam folded into the reduction, whose last workgroup advances
    the device step count) equals the eager per-step launches -- statistics,
    parameters and the optimizer's step count -- over five epochs, the ring
    slots shifted out of step once (the copy fallback)."""
    from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
    from pytorch_distributed_rnn_amd.models.motion import MotionModel
    from pytorch_distributed_rnn_amd.ops.adam import FusedAdam
    from pytorch_distributed_rnn_amd.train.fused_step import MotionTrainStep
    from pytorch_distributed_rnn_amd.utils.flat import flatten_module
    torch.manual_seed(6)
    train, _, _ = synthetic_motion(n_train=n_train, n_validation=1, n_test=1, seed=6)
    feats, labels = train.features.cuda(), train.labels.cuda().reshape(-1)
    m1 = MotionModel(9, 32, 2, 6).cuda()
    m2 = copy.deepcopy(m1)
    flatten_module(m1)
    flatten_module(m2)
    o1, o2 = FusedAdam(m1.parameters(), lr=2.5e-3), FusedAdam(m2.parameters(), lr=2.5e-3)
    s1 = MotionTrainStep(m1, o1, None, cuda_graph=True)
    s2 = MotionTrainStep(m2, o2, None)
    assert s1.cuda_graph and not s2.cuda_graph
    g = torch.Generator().manual_seed(3)
    replays = 0
    for e in range(5):
        idx_list = list(torch.split(torch.randperm(n_train, generator=g).cuda(), bs))
        if e == 4:
            s1._slot = (s1._slot + 3) % s1.RING
        res = s1.run_steps(feats, labels, idx_list)
        if res is None:
            res = [s1(feats, labels, i) for i in idx_list]
        else:
            replays += 1
        a = [r.clone() for r in res]
        assert s2.run_steps(feats, labels, idx_list) is None
        b = [s2(feats, labels, i).clone() for i in idx_list]
        for k, (x, y) in enumerate(zip(a, b)):
            torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6, msg=lambda m: f"epoch {e} step {k}: {m}")
    assert replays == 3, "the epoch was never replayed from a graph"
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    steps = 5 * len(idx_list)
    assert o1.state_dict()["state"][0]["step"] == o2.state_dict()["state"][0]["step"] == steps
