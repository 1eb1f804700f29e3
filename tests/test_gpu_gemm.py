"""GPU: the time-batched MFMA GEMM (csrc/kernels/gemm.hip) against an fp32
PyTorch reference of the same product, for every operand layout the large-H
layers use (Xp: [M,K] x [N,K] + bias -> 16-bit; dX: [M,K] x [K,N] in two K
segments; dW: [K,M] x [K,N] (+ a second segment) -> fp32), with shapes that
leave partial 256-wide tiles and strided (row-stride > width) operands."""
import pytest
import torch

from pytorch_distributed_rnn_amd import _ext

pytestmark = pytest.mark.gpu


def _mod():
    mod = _ext.require()
    assert hasattr(mod, "gemm16")
    return mod


def _op(t, km):
    """logical [rows, K] operand from its storage (k-major storage is [K, rows])."""
    return t.float().t() if km else t.float()


VARIANTS = [35]  # the build's default ping-pong schedule (an A/B build adds one: kernels/gemm.hip)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("akm,bkm", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (520, 264, 192), (1000, 776, 448)])
def test_gemm16_layouts_fp32_out(dtype, akm, bkm, M, N, K, variant):
    mod = _mod()
    torch.manual_seed(M + N + K)
    A = torch.randn(*((K, M) if akm else (M, K)), device="cuda").to(dtype)
    B = torch.randn(*((K, N) if bkm else (N, K)), device="cuda").to(dtype)
    C = mod.gemm16(A, akm, B, bkm, variant=variant)
    ref = _op(A, akm) @ _op(B, bkm).t()
    torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-3 * K ** 0.5)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_gemm16_xp_bias_16bit_out(dtype, variant):
    mod = _mod()
    torch.manual_seed(1)
    M, N, K = 777, 1280, 320
    X = torch.randn(M, K, device="cuda").to(dtype)
    W = torch.randn(N, K, device="cuda").to(dtype) * 0.1
    b = torch.randn(N, device="cuda")
    C = mod.gemm16(X, False, W, False, bias=b, out16=True, variant=variant)
    assert C.dtype == dtype and C.shape == (M, N)
    ref = X.float() @ W.float().t() + b
    tol = 8e-3 if dtype == torch.bfloat16 else 1e-3
    torch.testing.assert_close(C.float(), ref, rtol=tol, atol=tol * 4)


@pytest.mark.parametrize("variant", VARIANTS)
def test_gemm16_dx_two_segments_strided(variant):
    """dX = G0 W0 + G1 W1 with G the two direction slices of one [M, 2*4H] tensor."""
    mod = _mod()
    torch.manual_seed(2)
    M, G4, I = 640, 512, 384
    G = torch.randn(M, 2 * G4, device="cuda").half()
    W0 = torch.randn(G4, I, device="cuda").half()
    W1 = torch.randn(G4, I, device="cuda").half()
    g0, g1 = G[:, :G4], G[:, G4:]
    C = mod.gemm16(g0, False, W0, True, A2=g1, B2=W1, out16=True, variant=variant)
    ref = g0.float() @ W0.float() + g1.float() @ W1.float()
    torch.testing.assert_close(C.float(), ref, rtol=2e-3, atol=0.15)


@pytest.mark.parametrize("variant", VARIANTS)
def test_gemm16_dw_segment_and_accumulate(variant):
    """dW_hh = G[B:]^T Hprev + G[:B]^T h0 (k-major operands, strided H view), then += into an existing grad."""
    mod = _mod()
    torch.manual_seed(3)
    T, Bsz, G4, H = 5, 64, 768, 256
    G = torch.randn(T * Bsz, G4, device="cuda").bfloat16()
    hseq = torch.randn(T * Bsz, 2 * H, device="cuda").bfloat16()
    h = hseq[:, :H]
    h0 = torch.randn(Bsz, H, device="cuda").bfloat16()
    C = mod.gemm16(G[Bsz:], True, h[:-Bsz], True, A2=G[:Bsz], B2=h0, variant=variant)
    ref = G[Bsz:].float().t() @ h[:-Bsz].float() + G[:Bsz].float().t() @ h0.float()
    torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-2)
    base = torch.randn(G4, H, device="cuda")
    out = base.clone()
    mod.gemm16(G, True, h, True, out=out, accumulate=True, variant=variant)
    torch.testing.assert_close(out, base + G.float().t() @ h.float(), rtol=1e-3, atol=1e-2)


def test_gemm16_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C write."""
    mod = _mod()
    n = 256
    A = torch.eye(n, device="cuda").half()
    B = (torch.arange(n * 128, device="cuda").view(n, 128) % 97).half()  # B stored [N=256][K=128]? use k-major
    Bk = (torch.arange(n * n, device="cuda").view(n, n) % 61).half()      # [K, N]
    C = mod.gemm16(A, False, Bk, True)
    torch.testing.assert_close(C, Bk.float())
    del B


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("splitk", [2, 3, 5])
def test_gemm16_splitk_with_segment(splitk, variant):
    """split-K partials (fixed-order sum) across a segment boundary, incl. accumulate into out."""
    mod = _mod()
    torch.manual_seed(4)
    K1, K2, M, N = 64 * 7, 64 * 3, 264, 520
    G, Hh = torch.randn(K1, M, device="cuda").half(), torch.randn(K1, N, device="cuda").half()
    G2, H2 = torch.randn(K2, M, device="cuda").half(), torch.randn(K2, N, device="cuda").half()
    C = mod.gemm16(G, True, Hh, True, A2=G2, B2=H2, splitk=splitk, variant=variant)
    ref = G.float().t() @ Hh.float() + G2.float().t() @ H2.float()
    torch.testing.assert_close(C, ref, rtol=1e-3, atol=1e-2)
    out = torch.ones(M, N, device="cuda")
    mod.gemm16(G, True, Hh, True, out=out, accumulate=True, splitk=splitk, variant=variant)
    torch.testing.assert_close(out, 1 + G.float().t() @ Hh.float(), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("variant", [0, 35, 3])
def test_gemm16_schedule_variants(variant):
    """The compiled schedule variants (0 = default) are exact; one not
    compiled into this build is refused, never silently replaced."""
    mod = _mod()
    if variant not in [0] + list(mod.gemm_variants()):
        A = torch.randn(64, 64, device="cuda").bfloat16()
        with pytest.raises(RuntimeError):
            mod.gemm16(A, False, A, False, variant=variant)
        return
    torch.manual_seed(5)
    for akm, bkm in [(False, False), (True, True), (False, True)]:
        M, N, K = 520, 776, 64 * 9
        A = torch.randn(*((K, M) if akm else (M, K)), device="cuda").bfloat16()
        B = torch.randn(*((K, N) if bkm else (N, K)), device="cuda").bfloat16()
        C = mod.gemm16(A, akm, B, bkm, variant=variant)
        torch.testing.assert_close(C, _op(A, akm) @ _op(B, bkm).t(), rtol=1e-3, atol=3e-2)
