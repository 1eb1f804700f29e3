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


# ---------------------------------------------------------------- fp32 GEMM
F32_SHAPES = [(520, 776, 64 * 9), (37, 29, 9), (1024, 512, 1000), (130, 32, 4096), (300, 64, 128)]


def _mk(shape_mk, kmajor, dtype, gen_scale=1.0):
    r, c = shape_mk
    t = torch.randn(*((c, r) if kmajor else (r, c)), device="cuda") * gen_scale
    return t.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("akm,bkm", [(False, False), (True, True), (False, True), (True, False)])
@pytest.mark.parametrize("M,N,K", F32_SHAPES)
def test_gemm_f32_layouts_against_fp64(dtype, akm, bkm, M, N, K):
    """The fp32-product MFMA GEMM (kernels/gemm_f32.hip) against an fp64
    matmul of the same (widened) operands: every layout, ragged M/N/K (K = 9:
    the layer-0 projection of the motion model), all three tile widths."""
    mod = _mod()
    torch.manual_seed(7)
    A = _mk((M, K), akm, dtype)
    B = _mk((N, K), bkm, dtype)
    C, rs = mod.gemm_f32(A, akm, B, bkm)
    ref = _op(A, akm).double() @ _op(B, bkm).double().t()
    torch.testing.assert_close(C.double(), ref, rtol=2e-5, atol=2e-4 * (K ** 0.5))


@pytest.mark.parametrize("splitk", [1, 3])
def test_gemm_f32_segment_rowsum_bias_accumulate(splitk):
    """dW_hh-shaped product: two K segments (shifted h sequence + the initial
    state), split-K partials summed in fixed order, the row sums of op(A) over
    K (= the bias gradient), and accumulation into an existing output."""
    mod = _mod()
    torch.manual_seed(8)
    K1, K2, M, N = 1900, 95, 512, 128
    G1, G2 = torch.randn(K1, M, device="cuda"), torch.randn(K2, M, device="cuda")
    H1, H2 = torch.randn(K1, N, device="cuda"), torch.randn(K2, N, device="cuda")
    C, rs = mod.gemm_f32(G1, True, H1, True, A2=G2, B2=H2, splitk=splitk, rowsum=True)
    ref = G1.double().t() @ H1.double() + G2.double().t() @ H2.double()
    torch.testing.assert_close(C.double(), ref, rtol=2e-5, atol=2e-3)
    torch.testing.assert_close(rs.double(), G1.double().sum(0) + G2.double().sum(0), rtol=2e-5, atol=1e-3)
    out = torch.ones(M, N, device="cuda")
    mod.gemm_f32(G1, True, H1, True, out=out, accumulate=True, splitk=splitk)
    torch.testing.assert_close(out.double(), 1 + G1.double().t() @ H1.double(), rtol=2e-5, atol=2e-3)
    # projection with bias, 16-bit output (narrow head: N = 32)
    X = torch.randn(700, 256, device="cuda").bfloat16()
    W = torch.randn(32, 256, device="cuda").bfloat16()
    b = torch.randn(32, device="cuda")
    Y, _ = mod.gemm_f32(X, False, W, False, bias=b, out16=True)
    assert Y.dtype == torch.bfloat16
    torch.testing.assert_close(Y.float(), (X.double() @ W.double().t() + b.double()).float().bfloat16().float(),
                               rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("rows,cols", [(184320, 512), (95, 7), (4096, 32), (1000, 1024), (33, 512)])
def test_col_sum_matches_fp64(dtype, rows, cols):
    """cols % 512 == 0 with 16-bit input takes the 8-column-per-thread kernel
    (the strided view below the 4-column one)."""
    mod = _mod()
    X = torch.randn(rows, cols, device="cuda").to(dtype)
    got = mod.col_sum(X)
    torch.testing.assert_close(got.double(), X.double().sum(0), rtol=1e-5, atol=1e-3)
    # a strided view (row stride > cols)
    Y = torch.randn(rows, cols + 5, device="cuda").to(dtype)[:, 2:2 + cols]
    torch.testing.assert_close(mod.col_sum(Y).double(), Y.double().sum(0), rtol=1e-5, atol=1e-3)
