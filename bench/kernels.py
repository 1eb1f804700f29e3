"""Micro-benchmark of the fused LSTM kernels vs torch nn.LSTM (MIOpen) on one GPU."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def timeit(fn, warmup=3, iters=20):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1440,720,360,180")
    ap.add_argument("--hidden", type=int, default=32)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--input", type=int, default=9)
    ap.add_argument("--seq", type=int, default=128)
    a = ap.parse_args()
    from pytorch_distributed_rnn_amd.ops.lstm import lstm_forward
    dev = torch.device("cuda")
    res = []
    for B in [int(b) for b in a.batches.split(",")]:
        ref = torch.nn.LSTM(a.input, a.hidden, a.layers, batch_first=True).to(dev)
        ws = [p.detach().clone().requires_grad_() for p in ref.parameters()]
        x = torch.randn(B, a.seq, a.input, device=dev)

        def fused_fwd():
            with torch.no_grad():
                lstm_forward(x, ws, hidden=a.hidden, num_layers=a.layers, batch_first=True,
                             need_out=False)

        def fused_fwd_save():
            out, hn, cn = lstm_forward(x, ws, hidden=a.hidden, num_layers=a.layers, batch_first=True)
            return hn

        def fused_fwdbwd():
            out, hn, cn = lstm_forward(x, ws, hidden=a.hidden, num_layers=a.layers, batch_first=True)
            hn[-1].sum().backward()

        def ref_fwd():
            with torch.no_grad():
                ref(x)

        def ref_fwdbwd():
            out, (hn, cn) = ref(x)
            hn[-1].sum().backward()

        r = dict(B=B, tune=os.environ.get("PDRNN_TUNE", ""),
                 fused_fwd_ms=timeit(fused_fwd), fused_fwd_save_ms=timeit(fused_fwd_save),
                 fused_train_ms=timeit(fused_fwdbwd),
                 torch_fwd_ms=timeit(ref_fwd), torch_train_ms=timeit(ref_fwdbwd))
        print(json.dumps(r), flush=True)
        res.append(r)


if __name__ == "__main__":
    main()
