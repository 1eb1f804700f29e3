"""Forward kernel lane maps at the motion shapes: gate-split (split=1) vs the
K-split map (split = lanes per unit), sequences per workgroup nb.

    python bench/fwd_split.py [--batches 1440,180]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1440,720,180")
    a = ap.parse_args()
    from pytorch_distributed_rnn_amd import _ext
    mod = _ext.require()
    dev = torch.device("cuda")
    H, NL, I, T = 32, 2, 9, 128
    ref = torch.nn.LSTM(I, H, NL, batch_first=True).to(dev)
    ws = [p.detach().contiguous() for p in ref.parameters()]
    for B in [int(b) for b in a.batches.split(",")]:
        x = torch.randn(B, T, I, device=dev)
        for split in (1, 2, 4, 8):
            for nb in (1, 2):
                def run():
                    return mod.lstm_small_fwd(x, None, ws, None, None, H, NL, True, True, False, nb, split)
                try:
                    for _ in range(5):
                        run()
                    torch.cuda.synchronize()
                except RuntimeError as e:
                    print(f"B={B} split={split} nb={nb}: n/a ({str(e)[:60]})")
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(50):
                    run()
                e1.record()
                torch.cuda.synchronize()
                print(f"B={B} split={split} nb={nb}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
