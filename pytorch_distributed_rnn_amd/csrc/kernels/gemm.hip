// Time-batched GEMMs of the large-hidden LSTM / GRU layers for gfx950:
//
//   * input projection   Xp = X W_ih^T + b        (A [M][K], B [N][K], 16-bit out, fp32 bias)
//   * input gradient     dX = dG0 W0 + dG1 W1     (A [M][K], B [K][N], two K segments)
//   * weight gradients   dW = dG^T Hprev (+ dG0^T h0)  (A [K][M], B [K][N], fp32 out)
//
// These are the products SURVEY N1 puts on the matrix cores next to the
// recurrence kernels (lstm_large.hip); the reference trains the same cell
// through torch.nn.LSTM (reference: src/motion/model.py:9).
//
// One kernel template covers every operand layout: 256 x 256 output tile per
// workgroup, BK = 64, v_mfma_f32_16x16x32_{bf16,f16}, 8 waves as 2 (M) x 4 (N),
// each wave 128 x 64 outputs = 8 x 4 accumulator tiles (128 VGPRs).
//
// Staging.  LDS holds two K-tiles (slots) of four 16 KiB "quarter" images:
//   A_m0 / A_m1 : the tile rows a wave group computes in its first / second
//                 64-row half (rows {0-63, 128-191} / {64-127, 192-255}),
//   B_n0 / B_n1 : the tile columns a wave computes in its first / second
//                 32-column half.
// A quarter is filled by direct global->LDS DMA (global_load_lds_dwordx4,
// lane-linear destination, XOR swizzle applied on the per-lane source) and
// each quarter of slot t%2 is re-filled with K-tile t+2 as soon as its last
// reader phase of K-tile t has passed -- 6 to 7 phases of MFMA work cover a
// DMA's latency with only two slots of LDS.
//
// Phases.  A K-tile is 4 phases, one per accumulator quadrant (mq, nq) in the
// order (0,0) (0,1) (1,1) (1,0); a phase reads its fragments (A_m0 + B_n0,
// B_n1, A_m1, none), passes a barrier, then issues 16 MFMAs.  The two wave
// groups (wr = 0: M rows 0-127, wr = 1: rows 128-255) run one barrier apart
// (group 1 passes an extra barrier first): on every SIMD one wave reads LDS
// while the other one keeps the matrix pipe busy.  DMA completion is retired
// with counted `s_waitcnt vmcnt` one phase before the first reader, and raw
// s_barriers keep the DMAs in flight (a __syncthreads() would drain them).
//
// Operand images.  [M][K] / [N][K] operands (K contiguous) are stored as
// 128-byte rows (one row = 64 k of one m), 16-byte chunk c at slot c ^ (row & 7),
// and read with ds_read_b128.  [K][M] / [K][N] operands (k-major) are stored as
// 256-byte k-rows of 128 m, chunk c at slot c ^ f(k), f(k) = 2 ((k & 3) |
// ((k >> 3) & 1) << 2), and read with the transposing ds_read_b64_tr_b16 --
// conflict-free: the eight k-rows a 32-lane half touches land on eight distinct
// 32-byte bank groups.
//
// Epilogue: fp32 stores (optionally C += AB), or 16-bit output (+ fp32 column
// bias) through the now idle LDS so that every global store is a full 16-byte
// lane access.  Tile order: XCD-aware (each XCD gets a contiguous run of tile
// ids) and grouped 8 tile-rows at a time so concurrently resident tiles share
// A and B panels in their XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pdrnn/api.h"
#include "pdrnn/common.h"
#include "pdrnn/gemm_pp.h"

namespace pdrnn {
namespace {

using namespace pp;

struct GBF16 {
  static __device__ __forceinline__ g_f32x4 mfma(const uint4& a, const uint4& b, g_f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(g_bf16x8, a), __builtin_bit_cast(g_bf16x8, b),
                                                   c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t from_f(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
};
struct GF16 {
  static __device__ __forceinline__ g_f32x4 mfma(const uint4& a, const uint4& b, g_f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(g_f16x8, a), __builtin_bit_cast(g_f16x8, b),
                                                  c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t from_f(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
};

// The operand pointers arrive as __restrict__ arguments of this inlined body:
// hipcc then tags each LDS DMA with the scope of its global source and proves
// the ds_reads independent of it.  Without that it puts an `s_waitcnt
// vmcnt(0)` before every ds_read that may alias an outstanding LDS DMA (all of
// them), which drains the DMA pipeline every phase.  The counted waits and
// barriers below are what orders the accesses.
// V: schedule variant bits (tuning A/B): 1 = B_n1 refill in Q3 instead of Q2,
// 2 = issue a phase's DMA after its fragment reads
template <class DT, bool AKM, bool BKM, bool OUT16, int V>
__device__ __forceinline__ void gemm_body(const PdrnnGemmArgs& p, const uint16_t* __restrict__ Ab,
                                          const uint16_t* __restrict__ Bb, const uint16_t* __restrict__ A2b,
                                          const uint16_t* __restrict__ B2b, uint16_t* smem) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;

  // ---- tile id: XCD-contiguous runs, then groups of 8 tile-rows
  const int tiles_m = (p.M + TM - 1) / TM, tiles_n = (p.N + TN - 1) / TN;
  const int nwg = tiles_m * tiles_n;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  constexpr int GROUP = (V & 32) ? 4 : (V & 64) ? 16 : 8;  // tile-rows per raster group (V bits 32 / 64: tuning)
  const int per_group = GROUP * tiles_n;
  const int gidx = wg / per_group, first_m = gidx * GROUP;
  const int gsz = min(tiles_m - first_m, GROUP);
  const int tm = first_m + (wg % per_group) % gsz, tn = (wg % per_group) / gsz;
  const int m0 = tm * TM, n0 = tn * TN;

  // split-K: blockIdx.y takes K-tiles [ktb, kte) of the concatenated segments
  // and writes its fp32 partial to C + blockIdx.y * c_split_stride
  const int KT1 = p.K / TK, KTALL = KT1 + p.K2 / TK;
  const int ktb = (int)((int64_t)KTALL * blockIdx.y / gridDim.y);
  const int KT = (int)((int64_t)KTALL * (blockIdx.y + 1) / gridDim.y) - ktb;
  g_f32x4 acc[8][4];
  pp::mainloop<DT, AKM, BKM, V>(Ab, p.lda, Bb, p.ldb, A2b, p.lda2, B2b, p.ldb2, p.M, p.N, KT1, ktb, KT, m0, n0, smem,
                                acc);

  // ---- epilogue
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (!OUT16) {
    float* C = static_cast<float*>(p.C) + (int64_t)blockIdx.y * p.c_split_stride;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rb = m0 + wr * 128 + i * 16 + fq * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = n0 + wc * 64 + j * 16 + fr;
        if (col >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rb + r;
          if (row < p.M) {
            float* dst = C + (int64_t)row * p.ldc + col;
            *dst = p.accumulate ? *dst + acc[i][j][r] : acc[i][j][r];
          }
        }
      }
    }
  } else {
    // 16-bit output (+ fp32 column bias): each wave stages its 128 x 64 block
    // in LDS (column pairs packed per lane after a neighbour swap), then
    // writes 16-byte row chunks
    uint16_t* stg = smem + wid * (128 * 64);
    const float* bias = static_cast<const float*>(p.bias);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int lc = j * 16 + fr;
      const float bv = bias ? bias[min(n0 + wc * 64 + lc, p.N - 1)] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bv;
        float w[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = dpp_swap1(v[r]);
        const bool odd = fr & 1;
        const int c0 = lc & ~1;
        const int rr = i * 16 + fq * 4 + (odd ? 2 : 0);
        // even lane: rows r0, r0+1 of (c, c+1); odd lane: rows r0+2, r0+3 of (c-1, c)
        const float a0 = odd ? w[2] : v[0], b0 = odd ? v[2] : w[0];
        const float a1 = odd ? w[3] : v[1], b1 = odd ? v[3] : w[1];
        const uint32_t p0 = (uint32_t)DT::from_f(a0) | ((uint32_t)DT::from_f(b0) << 16);
        const uint32_t p1 = (uint32_t)DT::from_f(a1) | ((uint32_t)DT::from_f(b1) << 16);
        *reinterpret_cast<uint32_t*>(stg + rr * 64 + c0) = p0;
        *reinterpret_cast<uint32_t*>(stg + (rr + 1) * 64 + c0) = p1;
      }
    }
    wait_lds();
    uint16_t* C = static_cast<uint16_t*>(p.C);
    // 128 rows x 8 chunks of 16 B; 64 lanes -> 8 rows per pass
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int lr = it * 8 + (lane >> 3), ch = lane & 7;
      const int row = m0 + wr * 128 + lr, col = n0 + wc * 64 + ch * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(stg + lr * 64 + ch * 8);
      if (row < p.M && col < p.N) *reinterpret_cast<uint4*>(C + (int64_t)row * p.ldc + col) = v;
    }
  }
}

template <class DT, bool AKM, bool BKM, bool OUT16, int V>
__global__ void __launch_bounds__(512) gemm256_kernel(PdrnnGemmArgs p) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  gemm_body<DT, AKM, BKM, OUT16, V>(p, static_cast<const uint16_t*>(p.A), static_cast<const uint16_t*>(p.B),
                                 static_cast<const uint16_t*>(p.A2 ? p.A2 : p.A),
                                 static_cast<const uint16_t*>(p.B2 ? p.B2 : p.B), smem);
}

template <class DT, bool AKM, bool BKM, int V>
hipError_t launch_v(const PdrnnGemmArgs& a, hipStream_t st) {
  const int tiles = ((a.M + TM - 1) / TM) * ((a.N + TN - 1) / TN);
  const dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1);
  if (a.c_16bit)
    hipLaunchKernelGGL((gemm256_kernel<DT, AKM, BKM, true, V>), grid, dim3(512), LDS_BYTES, st, a);
  else
    hipLaunchKernelGGL((gemm256_kernel<DT, AKM, BKM, false, V>), grid, dim3(512), LDS_BYTES, st, a);
  return hipGetLastError();
}
// Schedule variants (V bits: 1 = B_n1 refill in Q3, 2 = DMA after the fragment
// reads, 32 / 64 = raster groups of 4 / 16 tile-rows).  The product build
// compiles the default, 35 (profiles/r3_gemm/raster.log); an A/B build adds
// ONE more: PDRNN_HIP_EXTRA_FLAGS=-DPDRNN_GEMM_AB=<V> python -m
// pytorch_distributed_rnn_amd._build, then gemm16(..., variant=<V>).
constexpr int kGemmDefaultVariant = 35;
template <class DT, bool AKM, bool BKM>
hipError_t launch(const PdrnnGemmArgs& a, hipStream_t st) {
#ifdef PDRNN_GEMM_AB
  if (a.variant == PDRNN_GEMM_AB) return launch_v<DT, AKM, BKM, PDRNN_GEMM_AB>(a, st);
#endif
  if (a.variant <= 0 || a.variant == kGemmDefaultVariant) return launch_v<DT, AKM, BKM, kGemmDefaultVariant>(a, st);
  return hipErrorInvalidValue;  // not compiled into this build
}

template <class DT>
hipError_t dispatch(const PdrnnGemmArgs& a, hipStream_t st) {
  if (a.a_kmajor) {
    if (a.b_kmajor) return launch<DT, true, true>(a, st);
    return launch<DT, true, false>(a, st);
  }
  if (a.b_kmajor) return launch<DT, false, true>(a, st);
  return launch<DT, false, false>(a, st);
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_gemm_supported(const PdrnnGemmArgs* a) {
  // K segments in whole K-tiles; k-major operands move in 8-element chunks;
  // 16-bit output rows in 16-byte chunks
  if (a->M < 8 || a->N < 8 || a->K <= 0 || a->K % 64 || a->K2 % 64 || a->K2 < 0) return 0;
  if ((a->a_kmajor && a->M % 8) || (a->b_kmajor && a->N % 8)) return 0;
  if (a->c_16bit && (a->N % 8 || a->ldc % 8 || a->accumulate)) return 0;
  if (a->K2 && (!a->A2 || !a->B2)) return 0;
  // split-K: fp32 partials only, at least one K-tile per split
  if (a->splitk > 1 && (a->c_16bit || a->accumulate || (a->K + a->K2) / 64 < a->splitk)) return 0;
  return 1;
}

int pdrnn_gemm_variants(int* out, int max) {
  int n = 0;
  if (n < max) out[n++] = pdrnn::kGemmDefaultVariant;
#ifdef PDRNN_GEMM_AB
  if (n < max && PDRNN_GEMM_AB != pdrnn::kGemmDefaultVariant) out[n++] = PDRNN_GEMM_AB;
#endif
  return n;
}

hipError_t pdrnn_gemm(const PdrnnGemmArgs* a, hipStream_t stream) {
  if (!pdrnn_gemm_supported(a)) return hipErrorInvalidValue;
  if (a->dtype == 0) return pdrnn::dispatch<pdrnn::GBF16>(*a, stream);
  return pdrnn::dispatch<pdrnn::GF16>(*a, stream);
}

}  // extern "C"
