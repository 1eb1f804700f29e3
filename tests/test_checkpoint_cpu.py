"""Checkpoint dict/key layout and resume (reference: base.py:164-177)."""
import torch

from pytorch_distributed_rnn_amd.data.motion import synthetic_motion
from pytorch_distributed_rnn_amd.models.motion import MotionModel
from pytorch_distributed_rnn_amd.train.checkpoint import adapt_state_dict_keys, save_checkpoint
from pytorch_distributed_rnn_amd.train.trainer import Trainer


def test_roundtrip_and_layout(tmp_path):
    m = MotionModel(9, 8, 2, 6)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    p = save_checkpoint(tmp_path / "best-model.pt", 3, m, opt, 0.5)
    ck = torch.load(p, weights_only=True)
    assert set(ck.keys()) == {"epoch", "model_state", "optimizer_state", "loss"}
    assert ck["epoch"] == 4 and abs(ck["loss"] - 0.5) < 1e-9
    assert list(ck["model_state"].keys())[0] == "lstm.weight_ih_l0"


def test_module_prefix_adaptation():
    m = MotionModel(9, 8, 2, 6)
    pref = {"module." + k: v for k, v in m.state_dict().items()}
    assert adapt_state_dict_keys(pref, m).keys() == m.state_dict().keys()


def test_trainer_epoch_checkpoint_and_resume(tmp_path):
    torch.manual_seed(0)
    train, val, test = synthetic_motion(n_train=192, n_validation=32, n_test=32, seed=0)
    m = MotionModel(9, 8, 2, 6)
    t = Trainer(model=m, training_set=train, validation_set=val, test_set=test, batch_size=96,
                learning_rate=2.5e-3, checkpoint_dir=tmp_path, device=torch.device("cpu"))
    _, th, vh = t.train(epochs=2)
    assert len(th) == 2 and len(vh) == 2
    files = sorted(x.name for x in tmp_path.iterdir())
    assert "best-model.pt" in files
    m2 = MotionModel(9, 8, 2, 6)
    t2 = Trainer(model=m2, training_set=train, batch_size=96, learning_rate=2.5e-3,
                 checkpoint_dir=tmp_path / "r", device=torch.device("cpu"))
    nxt = t2.resume(tmp_path / "best-model.pt")
    assert nxt >= 1
    ck = torch.load(tmp_path / "best-model.pt", weights_only=True)
    for k, v in m2.state_dict().items():
        torch.testing.assert_close(v, ck["model_state"][k])
