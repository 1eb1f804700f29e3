"""Short fixed workload for PMC passes: the in-tree GEMM on the bi-LSTM Xp L1
(NT x NT) and dW_ih L1 (KM x KM) shapes and hipBLASLt on the Xp shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_rnn_amd import _ext  # noqa: E402

mod = _ext.require()
r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).half()  # noqa: E731
A, B = r(32768, 8192), r(32768, 8192)
G, X = r(32768, 16384), r(32768, 8192)
for _ in range(2):
    mod.gemm16(A, False, B, False, out16=True, variant=3)
    mod.gemm16(G, True, X, True, variant=3)
    torch.mm(A, B.t())
torch.cuda.synchronize()
print("ok")
