"""Time the fp32 weight-gradient GEMM shape of the motion --hidden-units 128
model (dW = G^T X: G [T*B, 4H] and X [T*B, H] both k-major, K = 184320) on
kernels/gemm_f32.hip, with the default split-K heuristic; for rocprofv3 PMC
passes (one shape, a few launches)."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_distributed_rnn_amd.ops.gemm import gemm_f32  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=184320)
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--splitk", type=int, default=0, help="K slices (0: the occupancy heuristic)")
    a = ap.parse_args()
    torch.manual_seed(0)
    G = torch.randn(a.rows, a.m, device="cuda")
    X = torch.randn(a.rows, a.n, device="cuda")
    sk = a.splitk or None
    for _ in range(3):
        gemm_f32(G, True, X, True, rowsum=True, splitk=sk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        gemm_f32(G, True, X, True, rowsum=True, splitk=sk)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    c, _ = gemm_f32(G, True, X, True, rowsum=True, splitk=sk)
    ref = (G.double().t() @ X.double()).float()
    err = float((c - ref).abs().max() / ref.abs().max())
    print(json.dumps({"splitk": a.splitk, "us": dt * 1e6, "tflops": 2 * a.rows * a.m * a.n / dt / 1e12, "rel_err": err}))


if __name__ == "__main__":
    main()
