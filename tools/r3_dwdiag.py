"""Diagnostic: gradients of the fused step with the deferred-dW backward vs
the register-dW backward vs autograd, per parameter (max abs / rel error)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_rnn_amd.data.motion import synthetic_motion  # noqa: E402
from pytorch_distributed_rnn_amd.models.motion import MotionModel  # noqa: E402
from pytorch_distributed_rnn_amd.train.trainer import Trainer  # noqa: E402


def grads_fused(model, train, mode, B):
    os.environ["PDRNN_LSTM_DWOUT"] = mode
    t = Trainer(model, train, batch_size=B, learning_rate=2.5e-3, device=torch.device("cuda"))
    f = t._fused_step()
    feats, labels, idx = t.train_loader.make_batch(t.train_loader.batch_indices()[0])
    from pytorch_distributed_rnn_amd.ops.lstm import fused_bwd_nb, small_launch_config
    nb_f, sp_f, _, _ = small_launch_config(idx.numel(), f.H, f.NL)
    stats = torch.zeros(3, device="cuda")
    ws = f.weights
    if f.gru:
        from pytorch_distributed_rnn_amd.ops.gru_fused import _pack
        ws = _pack(f.weights, f.NL, f.H, f.flat.data)
        nb_f, sp_f = 1, 1
    f.flat.attach_grads()
    f.mod.lstm_head_train_step(feats, idx, labels, ws, f.m.fc.weight, f.m.fc.bias, f.flat.grad, stats, f.H, f.NL,
                               sp_f, 0, nb_f, fused_bwd_nb(idx.numel(), f.H, f.NL), None, None,
                               1 if f.gru else 0, f.colmap)
    torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in f.m.parameters()], (feats, labels, idx)


def main():
    shapes = [("lstm", 64, 1, 16, 9), ("lstm", 32, 2, 128, 9), ("lstm", 16, 1, 37, 9), ("gru", 32, 2, 128, 9)]
    for cell, H, NL, T, F in shapes:
        torch.manual_seed(3)
        train, _, _ = synthetic_motion(n_train=382, n_validation=2, n_test=2, seq_length=T, num_features=F, seed=6)
        m0 = MotionModel(F, H, NL, 6, cell=cell)
        g_dw, (feats, labels, idx) = grads_fused(copy.deepcopy(m0), train, "force", 96)
        g_reg, _ = grads_fused(copy.deepcopy(m0), train, "0", 96)
        # autograd in fp64
        ref = copy.deepcopy(m0).cuda().double()
        x = feats.index_select(0, idx).double()
        y = labels.index_select(0, idx).reshape(-1)
        loss = torch.nn.functional.cross_entropy(ref(x), y)
        loss.backward()
        g_ref = [p.grad for p in ref.parameters()]
        names = [n for n, _ in m0.named_parameters()]
        print(f"== {cell} H={H} NL={NL} T={T} F={F}")
        for n, a, b, r in zip(names, g_dw, g_reg, g_ref):
            scale = r.abs().max().item() + 1e-30
            e_dw = (a.double() - r).abs().max().item() / scale
            e_reg = (b.double() - r).abs().max().item() / scale
            worst = (a.double() - r).abs().argmax().item()
            print(f"  {n:22s} |g|max={scale:.3e} rel_err dwout={e_dw:.2e} reg={e_reg:.2e} worst_idx={worst}")


if __name__ == "__main__":
    main()
