"""Diagnostic: cycles per recurrence step of the fused LSTM kernels (PDRNN_LSTM_STAMPS=1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["PDRNN_LSTM_STAMPS"] = "1"
import torch  # noqa: E402

from pytorch_distributed_rnn_amd.ops.lstm import lstm_forward  # noqa: E402

for B in [int(b) for b in (sys.argv[1] if len(sys.argv) > 1 else "180,1440").split(",")]:
    ref = torch.nn.LSTM(9, 32, 2, batch_first=True).cuda()
    ws = [p.detach().clone().requires_grad_() for p in ref.parameters()]
    x = torch.randn(B, 128, 9, device="cuda")
    for _ in range(3):
        out, hn, cn = lstm_forward(x, ws, hidden=32, num_layers=2, batch_first=True)
        hn[-1].sum().backward()
        torch.cuda.synchronize()
    print(f"--- B={B}", file=sys.stderr, flush=True)
