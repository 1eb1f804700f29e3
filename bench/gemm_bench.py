"""In-tree time-batched GEMM (kernels/gemm.hip) vs hipBLASLt (torch) on the
large-H layer shapes (fp16, uniform random operands).  bi-LSTM rows are 1/8 of
B4096 x T64 (same per-tile work, shorter run); char-LM shapes are full size."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_distributed_rnn_amd import _ext  # noqa: E402


def bench(fn, it=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / it)
    return best


def rnd(*s):
    return (torch.rand(*s, device="cuda") * 2 - 1).half()


mod = _ext.require()
rows = []
for what, M, N, K, kind in [
        ("bi-LSTM Xp L0 (I1024)", 32768, 32768, 1024, "xp"), ("bi-LSTM Xp L1 (I8192)", 32768, 32768, 8192, "xp"),
        ("bi-LSTM dX L1 (2 dirs)", 32768, 8192, 16384, "dx"), ("bi-LSTM dW_hh", 16384, 4096, 32256, "dw"),
        ("bi-LSTM dW_ih L1", 16384, 8192, 32768, "dw"), ("bi-LSTM dW_ih L0", 16384, 1024, 32768, "dw"),
        ("char-LM Xp L1", 65536, 4096, 1024, "xp"), ("char-LM dW_hh", 4096, 1024, 65408, "dw"),
        ("char-LM dX L1", 65536, 1024, 4096, "dx1")]:
    if kind == "xp":
        A, B, b = rnd(M, K), rnd(N, K), torch.randn(N, device="cuda")
        b16 = b.half()
        ref = lambda: torch.addmm(b16, A, B.t())  # noqa: E731
        ours = lambda v=0: mod.gemm16(A, False, B, False, bias=b, out16=True, variant=v)  # noqa: E731
        fl = 2.0 * M * N * K
    elif kind == "dx":
        G0, G1, W0, W1 = rnd(M, K), rnd(M, K), rnd(K, N), rnd(K, N)

        def ref():
            d = torch.mm(G0, W0)
            d.addmm_(G1, W1)
            return d
        ours = lambda v=0: mod.gemm16(G0, False, W0, True, A2=G1, B2=W1, out16=True, variant=v)  # noqa: E731
        fl = 4.0 * M * N * K
    elif kind == "dx1":
        G0, W0 = rnd(M, K), rnd(K, N)
        ref = lambda: torch.mm(G0, W0)  # noqa: E731
        ours = lambda v=0: mod.gemm16(G0, False, W0, True, out16=True, variant=v)  # noqa: E731
        fl = 2.0 * M * N * K
    else:
        G, Hh = rnd(K, M), rnd(K, N)
        ref = lambda: torch.mm(G.t(), Hh, out_dtype=torch.float32)  # noqa: E731
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        sk = max(1, min(8, 512 // tiles)) if tiles < 256 else 1
        ours = lambda v=0: mod.gemm16(G, True, Hh, True, splitk=sk, variant=v)  # noqa: E731
        fl = 2.0 * M * N * K
    err = (ours().float() - ref().float()).abs().max().item()
    tr = bench(ref)
    VARS = tuple(int(v) for v in os.environ.get('GEMM_VARS', '3,35').split(','))
    tv = [bench(lambda v=v: ours(v)) for v in VARS]
    to = min(tv)
    line = (f"{what:24s} M{M} N{N} K{K}: hipBLASLt {fl / tr / 1e12:7.1f} TF/s ({tr * 1e3:7.3f} ms) | "
            f"in-tree {fl / to / 1e12:7.1f} TF/s ({to * 1e3:7.3f} ms) | x{tr / to:5.2f} | maxerr {err:.3g} | "
            "variants " + " ".join(f"v{v}:{fl / t / 1e12:.0f}" for v, t in zip(VARS, tv)))
    print(line, flush=True)
