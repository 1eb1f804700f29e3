"""Tile-shape sweep of the MFMA GEMM core (the large-H step GEMMs) vs hipBLASLt."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_rnn_amd import _ext  # noqa: E402


def bench(fn, it=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(it):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / it


mod = _ext.require()
for (M, N, K, what) in [(4096, 4096, 16384, "bwd step B4096 H4096"), (4096, 16384, 4096, "fwd step B4096 H4096"),
                        (256, 4096, 16384, "bwd step B256"), (128, 4096, 1024, "charlm fwd step"),
                        # input projections Xp = X W_ih^T of the bi-LSTM (both directions, M = T*B rows;
                        # 1/8 of the B4096 x T64 rows keeps the sweep short, same per-tile work)
                        (32768, 32768, 1024, "Xp layer0 (I1024)"), (32768, 32768, 8192, "Xp layer1 (I8192)")]:
    a = torch.randn(M, K, device="cuda").half()
    b = torch.randn(N, K, device="cuda").half()
    fl = 2.0 * M * N * K
    ref = bench(lambda: torch.mm(a, b.t()))
    line = f"{what:24s} M{M} N{N} K{K}  hipBLASLt {fl / ref / 1e12:7.1f} TF/s"
    for tile in (0, 1, 2, 3, 4, 10, 11, 12, 13):
        try:
            t = bench(lambda: mod.gemm_nt(a, b, tile))
            line += f" | t{tile} {fl / t / 1e12:6.1f}"
        except RuntimeError:
            line += f" | t{tile}   n/a"
    print(line, flush=True)
c = mod.gemm_nt(a, b, 10)
torch.testing.assert_close(c, a.float() @ b.float().t(), rtol=2e-2, atol=2e-1)
print("tile10 ok")
