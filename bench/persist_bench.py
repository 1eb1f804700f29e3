"""Large-H recurrence, one layer: persistent cooperative kernel (tile -1) vs
the per-step MFMA kernels (tile 0 / auto split-K), forward and BPTT timed
separately with HIP events.  Defaults: the char-LM layer (bf16, H 1024, B 128,
T 512); ``--hidden 128 --dtype fp32 --batch 1440 --seq 128`` is the motion
model's fp32 ``--hidden-units 128`` layer.

    python bench/persist_bench.py [--batch 128] [--seq 512] [--hidden 1024] [--dtype bf16] [--reps 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seq", type=int, default=512)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cell", type=int, default=0)
    ap.add_argument("--hidden", type=int, default=1024)
    ap.add_argument("--dtype", choices=("bf16", "fp16", "fp32"), default="bf16")
    ap.add_argument("--tiles", type=int, nargs="*", default=[0],
                    help="per-step tile ids to time besides the automatic choice (lstm_large.hip TILE_CFGS_X)")
    a = ap.parse_args()
    from pytorch_distributed_rnn_amd import _ext
    mod = _ext.require()
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[a.dtype]
    code = {"bf16": 0, "fp16": 1, "fp32": 2}[a.dtype]
    H, B, T = a.hidden, a.batch, a.seq
    torch.manual_seed(0)
    xp = (torch.randn(T, B, 4 * H, device="cuda") * 0.5).to(dt)
    w = [(torch.randn(4 * H, H, device="cuda") * 0.03).to(dt)]
    wt = [(torch.randn(H, 4 * H, device="cuda") * 0.03).to(dt)]
    dout = (torch.randn(T, B, H, device="cuda") * 0.1).to(dt)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        best = 1e30
        for _ in range(a.reps):
            ev[0].record()
            fn()
            ev[1].record()
            torch.cuda.synchronize()
            best = min(best, ev[0].elapsed_time(ev[1]))
        return best

    res = {"B": B, "T": T, "H": H, "dtype": a.dtype, "cell": a.cell,
           "persist_mt": mod.lstm_large_persist_mt(B, H, 1, code)}
    # tile -1: persistent when covered (PDRNN_LSTM_PERSIST=0 -> auto per-step
    # tile); tile 0: per-step 32x64 forward tiles, split-K backward
    for name, t in [("auto", -1)] + [(f"per_step_tile{t}", t) for t in a.tiles]:
        fw = lambda: mod.lstm_large_fwd(xp, w, None, None, H, 0, t, a.cell)
        hseq, cseq, acts = fw()
        bw = lambda: mod.lstm_large_bwd(dout, None, None, wt, cseq, acts, None, H, 0, t, a.cell)
        f_ms, b_ms = timed(fw), timed(bw)
        res[name] = {"fwd_ms": round(f_ms, 3), "bwd_ms": round(b_ms, 3),
                     "fwd_us_per_step": round(f_ms * 1e3 / T, 2), "bwd_us_per_step": round(b_ms * 1e3 / T, 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
