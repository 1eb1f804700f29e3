// Large-hidden LSTM (H = 256 ... 4096+, bf16 / fp16 storage, fp32 accumulation
// and cell state) for gfx950.
//
// A layer is split into
//   * one big input-projection GEMM over all timesteps (library GEMM, issued
//     from the host: Xp[T, B, 4H] = X W_ih^T + b, gate-interleaved columns),
//   * T recurrent steps, each ONE launch of a hand-written MFMA kernel that
//     computes h_{t-1} W_hh^T (v_mfma_f32_16x16x32_{bf16,f16}, LDS
//     double-buffered, register-staged tiles) and applies the LSTM cell in the
//     epilogue: the 4 gates of a hidden unit sit in 4 adjacent output columns
//     (gate-interleaved weight rows) = one DPP quad of the MFMA C layout, so
//     the gate exchange is 16 quad broadcasts, no LDS round trip;
//   * the BPTT mirror: each reverse step is one MFMA kernel computing
//     dh_{t-1} = dgates_t W_hh (K = 4H) whose epilogue runs the cell backward
//     of step t-1 (per-element, no exchange) and emits dgates_{t-1};
//     weight gradients are then library GEMMs over all timesteps.
// Both directions of a bidirectional layer run in the same launch
// (blockIdx.z = direction), doubling the workgroups per step.
//
// Reference semantics: torch.nn.LSTM (gate order i, f, g, o), the op the
// reference's MotionModel uses (reference: src/motion/model.py:9,14).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));

// storage type tags
struct BF16 {
  typedef bf16x8 frag;
  static __device__ __forceinline__ float to_f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
  static __device__ __forceinline__ uint16_t from_f(float f) {
    const __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN-preserving
    return __builtin_bit_cast(uint16_t, b);
  }
  static __device__ __forceinline__ f32x4 mfma(const uint4& a, const uint4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                   c, 0, 0, 0);
  }
};
struct F16 {
  typedef f16x8 frag;
  static __device__ __forceinline__ float to_f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
  static __device__ __forceinline__ uint16_t from_f(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
  static __device__ __forceinline__ f32x4 mfma(const uint4& a, const uint4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                  c, 0, 0, 0);
  }
};

constexpr int BK = 64;  // K elements per LDS tile (8 x 16-byte chunks per row)

__device__ __forceinline__ float sigm(float x) { return fast_rcp(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_(float x) {
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) * fast_rcp(1.f + e), x);
}
__device__ __forceinline__ float qbcast(float v, int q) {
  switch (q) {
    case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x00, 0xF, 0xF, false));
    case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x55, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xAA, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xFF, 0xF, 0xF, false));
  }
}

// LDS image of a [ROWS x 64] 16-bit tile: 16-byte chunk c of row r lives at
// chunk slot (c ^ (r & 7)) -- the XOR swizzle spreads the 16 rows an MFMA
// fragment read touches over all bank groups.
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * BK + ((chunk ^ (row & 7)) << 3); }

// C[M, N] (+)= A[M, K] * Bt[N, K]^T for one BM x BN block tile; 4 waves as
// 2 x 2, each wave (BM/2) x (BN/2) = MT x NT MFMA 16x16 sub-tiles.  A / Bt are
// 16-bit, K-contiguous with leading dimensions lda / ldb.  Rows of A beyond M
// are clamped (their results are discarded by the caller).  K % 64 == 0.
template <class DT, int BM, int BN>
struct GemmNT {
  static constexpr int MT = BM / 32, NT = BN / 32;
  static constexpr int A_CHUNKS = BM * 8 / 256, B_CHUNKS = BN * 8 / 256;
  static constexpr int LDS_ELEMS = 2 * (BM + BN) * BK;  // double-buffered A | B

  __device__ static void run(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ Bt,
                             int64_t ldb, int M, int K, int m0, int n0, uint16_t* smem, f32x4 (&acc)[MT][NT]) {
    const int tid = threadIdx.x;
    const int lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const uint4* ga[A_CHUNKS];
    const uint4* gb[B_CHUNKS];
    int la[A_CHUNKS], lb[B_CHUNKS];
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const int id = tid + i * 256, r = id >> 3, c = id & 7;
      const int gr = min(m0 + r, M - 1);
      ga[i] = reinterpret_cast<const uint4*>(A + (int64_t)gr * lda + c * 8);
      la[i] = lds_off(r, c);
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const int id = tid + i * 256, r = id >> 3, c = id & 7;
      gb[i] = reinterpret_cast<const uint4*>(Bt + (int64_t)(n0 + r) * ldb + c * 8);
      lb[i] = lds_off(r, c);
    }
    uint16_t* sA[2] = {smem, smem + (BM + BN) * BK};
    uint16_t* sB[2] = {smem + BM * BK, smem + (BM + BN) * BK + BM * BK};

    uint4 ra[A_CHUNKS], rb[B_CHUNKS];
    const int KT = K / BK;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) ra[i] = ga[i][0];
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) rb[i] = gb[i][0];
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) *reinterpret_cast<uint4*>(sA[0] + la[i]) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) *reinterpret_cast<uint4*>(sB[0] + lb[i]) = rb[i];
    __syncthreads();

    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < KT; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < KT;
      if (more) {
        const int koff = (kt + 1) * (BK / 8);  // in uint4 units
#pragma unroll
        for (int i = 0; i < A_CHUNKS; ++i) ra[i] = ga[i][koff];
#pragma unroll
        for (int i = 0; i < B_CHUNKS; ++i) rb[i] = gb[i][koff];
      }
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        uint4 fa[MT], fb[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i)
          fa[i] = *reinterpret_cast<const uint4*>(sA[cur] + lds_off(wm * (BM / 2) + i * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int j = 0; j < NT; ++j)
          fb[j] = *reinterpret_cast<const uint4*>(sB[cur] + lds_off(wn * (BN / 2) + j * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = DT::mfma(fa[i], fb[j], acc[i][j]);
      }
      if (more) {
        const int nxt = cur ^ 1;
#pragma unroll
        for (int i = 0; i < A_CHUNKS; ++i) *reinterpret_cast<uint4*>(sA[nxt] + la[i]) = ra[i];
#pragma unroll
        for (int i = 0; i < B_CHUNKS; ++i) *reinterpret_cast<uint4*>(sB[nxt] + lb[i]) = rb[i];
      }
      __syncthreads();
    }
  }
};

// ---------------------------------------------------------------------------
// Forward step: gates = h_{t-1} Wp^T + xp_t  ->  (i, f, g, o), c_t, h_t.
// Columns are gate-interleaved: col = 4 u + q.
// ---------------------------------------------------------------------------
template <class DT, int BM, int BN>
__global__ void __launch_bounds__(256) lstm_large_fwd_step_kernel(PdrnnLstmLargeStepArgs args) {
  typedef GemmNT<DT, BM, BN> G;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_u16[];
  const PdrnnLstmLargeDir& d = args.dir[blockIdx.z];
  const int B = args.B, H = args.H;
  const int t = args.reverse_mask & (1 << blockIdx.z) ? args.T - 1 - args.step : args.step;
  const int tp = args.reverse_mask & (1 << blockIdx.z) ? t + 1 : t - 1;  // previous step in processing order
  const bool first = args.step == 0;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  // A operand: h_{prev} rows of the output sequence (or h0)
  const uint16_t* hA = first ? d.h0 : d.hseq + (int64_t)tp * d.hseq_st;
  const int64_t lda = first ? H : d.hseq_sb;
  f32x4 acc[G::MT][G::NT];
  if (first && d.h0 == nullptr) {
#pragma unroll
    for (int i = 0; i < G::MT; ++i)
#pragma unroll
      for (int j = 0; j < G::NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    G::run(hA, lda, d.w, H, B, H, m0, n0, smem_u16, acc);
  }

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int q = lane & 3;
  const uint16_t* xp = d.xp + (int64_t)t * d.xp_st;
  const float* cprev = first ? d.c0 : d.cseq + (int64_t)tp * B * H;
  float* cout = d.cseq + (int64_t)t * B * H;
  uint16_t* hout = d.hseq + (int64_t)t * d.hseq_st;
  uint16_t* acts = d.acts + (int64_t)t * B * 4 * H;
#pragma unroll
  for (int i = 0; i < G::MT; ++i) {
    const int rbase = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < G::NT; ++j) {
      const int col = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
      const int u = col >> 2;
      float a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = min(rbase + r, B - 1);
        const float z = acc[i][j][r] + DT::to_f(xp[(int64_t)row * d.xp_sb + col]);
        a[r] = q == 2 ? tanh_(z) : sigm(z);
        if (rbase + r < B) acts[(int64_t)row * 4 * H + col] = DT::from_f(a[r]);
      }
      // lane q of the quad finishes row rbase + q of unit u
      float ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float i_ = qbcast(a[r], 0), f_ = qbcast(a[r], 1), g_ = qbcast(a[r], 2), o_ = qbcast(a[r], 3);
        if (r == q) { ig = i_; fg = f_; gg = g_; og = o_; }
      }
      const int row = rbase + q;
      if (row < B) {
        const float cp = cprev ? cprev[(int64_t)row * H + u] : 0.f;
        const float cn = fmaf(fg, cp, ig * gg);
        const float h = og * tanh_(cn);
        cout[(int64_t)row * H + u] = cn;
        hout[(int64_t)row * d.hseq_sb + u] = DT::from_f(h);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Backward step: dh_{t'} = dgates_t Wp  (t' = the step processed before t in
// forward order) fused with the cell backward of step t':
//   dh = acc + dout_{t'};  dc = dc_carry + dh o (1 - tanh(c)^2)
//   dgates_{t'} = [dc g i(1-i), dc c_prev f(1-f), dc i (1-g^2), dh tanh(c) o(1-o)]
//   dc_carry = dc f
// With cell == 0 (after the first forward step): dh0 = acc, dc0 = dc_carry.
// ---------------------------------------------------------------------------
template <class DT, int BM, int BN>
__global__ void __launch_bounds__(256) lstm_large_bwd_step_kernel(PdrnnLstmLargeStepArgs args) {
  typedef GemmNT<DT, BM, BN> G;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_u16[];
  const PdrnnLstmLargeDir& d = args.dir[blockIdx.z];
  const int B = args.B, H = args.H, T = args.T;
  const bool rev = args.reverse_mask & (1 << blockIdx.z);
  // args.step counts backward steps: s = 0 consumes dgates of the LAST forward step
  const int s = args.step;
  const int t = rev ? s : T - 1 - s;            // step whose dgates are the GEMM input
  const int tn = rev ? t + 1 : t - 1;           // step whose cell backward the epilogue runs
  const bool cell = rev ? tn < T : tn >= 0;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  f32x4 acc[G::MT][G::NT];
  G::run(d.dgates + (int64_t)t * B * 4 * H, 4 * H, d.wt, 4 * H, B, 4 * H, m0, n0, smem_u16, acc);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int i = 0; i < G::MT; ++i) {
    const int rbase = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < G::NT; ++j) {
      const int u = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = rbase + r;
        if (b >= B) continue;
        const int64_t bu = (int64_t)b * H + u;
        float dh = acc[i][j][r];
        if (!cell) {
          if (d.dh0) d.dh0[bu] = dh;
          if (d.dc0) d.dc0[bu] = d.dc_carry[bu];
          continue;
        }
        if (d.dout) dh += DT::to_f(d.dout[(int64_t)tn * d.dout_st + (int64_t)b * d.dout_sb + u]);
        const u16x4 av = *reinterpret_cast<const u16x4*>(d.acts + ((int64_t)tn * B + b) * 4 * H + 4 * u);
        const float ig = DT::to_f(av.x), fg = DT::to_f(av.y), gg = DT::to_f(av.z), og = DT::to_f(av.w);
        const float c = d.cseq[(int64_t)tn * B * H + bu];
        const int tpp = rev ? tn + 1 : tn - 1;
        const bool has_prev = rev ? tpp < T : tpp >= 0;
        const float cp = has_prev ? d.cseq[(int64_t)tpp * B * H + bu] : (d.c0 ? d.c0[bu] : 0.f);
        const float tc = tanh_(c);
        const float dc = fmaf(dh * og, 1.f - tc * tc, d.dc_carry[bu]);
        u16x4 dg;
        dg.x = DT::from_f(dc * gg * ig * (1.f - ig));
        dg.y = DT::from_f(dc * cp * fg * (1.f - fg));
        dg.z = DT::from_f(dc * ig * (1.f - gg * gg));
        dg.w = DT::from_f(dh * tc * og * (1.f - og));
        *reinterpret_cast<u16x4*>(d.dgates + ((int64_t)tn * B + b) * 4 * H + 4 * u) = dg;
        d.dc_carry[bu] = dc * fg;
      }
    }
  }
}

// Cell backward of the LAST forward step (no recurrent dh yet):
// dh = dout_T-1 + dhn, dc = dcn.  One thread per (b, u).
template <class DT>
__global__ void lstm_large_bwd_first_kernel(PdrnnLstmLargeStepArgs args) {
  const PdrnnLstmLargeDir& d = args.dir[blockIdx.z];
  const int B = args.B, H = args.H, T = args.T;
  const bool rev = args.reverse_mask & (1 << blockIdx.z);
  const int tn = rev ? 0 : T - 1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * H) return;
  const int b = (int)(e / H), u = (int)(e - (int64_t)b * H);
  float dh = d.dhn ? d.dhn[e] : 0.f;
  if (d.dout) dh += DT::to_f(d.dout[(int64_t)tn * d.dout_st + (int64_t)b * d.dout_sb + u]);
  const u16x4 av = *reinterpret_cast<const u16x4*>(d.acts + ((int64_t)tn * B + b) * 4 * H + 4 * u);
  const float ig = DT::to_f(av.x), fg = DT::to_f(av.y), gg = DT::to_f(av.z), og = DT::to_f(av.w);
  const float c = d.cseq[(int64_t)tn * B * H + e];
  const int tpp = rev ? tn + 1 : tn - 1;
  const bool has_prev = rev ? tpp < T : tpp >= 0;
  const float cp = has_prev ? d.cseq[(int64_t)tpp * B * H + e] : (d.c0 ? d.c0[e] : 0.f);
  const float tc = tanh_(c);
  const float dc = fmaf(dh * og, 1.f - tc * tc, d.dcn ? d.dcn[e] : 0.f);
  u16x4 dg;
  dg.x = DT::from_f(dc * gg * ig * (1.f - ig));
  dg.y = DT::from_f(dc * cp * fg * (1.f - fg));
  dg.z = DT::from_f(dc * ig * (1.f - gg * gg));
  dg.w = DT::from_f(dh * tc * og * (1.f - og));
  *reinterpret_cast<u16x4*>(d.dgates + ((int64_t)tn * B + b) * 4 * H + 4 * u) = dg;
  d.dc_carry[e] = dc * fg;
}

// Plain NT GEMM on the same core (tests / fallbacks): C[M,N] fp32 = A Bt^T.
template <class DT, int BM, int BN>
__global__ void __launch_bounds__(256) gemm_nt_kernel(const uint16_t* A, int64_t lda, const uint16_t* Bt,
                                                      int64_t ldb, float* C, int64_t ldc, int M, int N, int K) {
  typedef GemmNT<DT, BM, BN> G;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem_u16[];
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  f32x4 acc[G::MT][G::NT];
  G::run(A, lda, Bt, ldb, M, K, m0, n0, smem_u16, acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int j = 0; j < G::NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * (BM / 2) + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * (BN / 2) + j * 16 + (lane & 15);
        if (row < M && col < N) C[(int64_t)row * ldc + col] = acc[i][j][r];
      }
}

template <class DT, int BM, int BN>
hipError_t launch_step(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, hipStream_t st) {
  const int N = backward ? a->H : 4 * a->H;
  dim3 grid(N / BN, (a->B + BM - 1) / BM, ndir);
  const size_t lds = sizeof(uint16_t) * GemmNT<DT, BM, BN>::LDS_ELEMS;
  if (backward)
    hipLaunchKernelGGL((lstm_large_bwd_step_kernel<DT, BM, BN>), grid, dim3(256), lds, st, *a);
  else
    hipLaunchKernelGGL((lstm_large_fwd_step_kernel<DT, BM, BN>), grid, dim3(256), lds, st, *a);
  return hipGetLastError();
}

// Tile choice: enough workgroups to cover the CUs (256) at small batch,
// bigger tiles (more MFMA per LDS byte) once the batch allows.
template <class DT>
hipError_t dispatch_step(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, int tile, hipStream_t st) {
  const int N = backward ? a->H : 4 * a->H;
  if (tile <= 0) {
    const int64_t t64 = (int64_t)(N / 64) * ((a->B + 63) / 64) * ndir;
    const int64_t t128 = (int64_t)(N / 128) * ((a->B + 127) / 128) * ndir;
    tile = t128 >= 512 ? 128 : (t64 >= 256 ? 64 : 32);
  }
  switch (tile) {
    case 32: return launch_step<DT, 32, 64>(a, ndir, backward, st);
    case 64: return launch_step<DT, 64, 64>(a, ndir, backward, st);
    case 128:
      if (N % 128) return launch_step<DT, 64, 64>(a, ndir, backward, st);
      return launch_step<DT, 128, 128>(a, ndir, backward, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_lstm_large_supported(int H) { return H >= 64 && H % 64 == 0; }

hipError_t pdrnn_lstm_large_step(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, int dtype, int tile,
                                 hipStream_t stream) {
  if (!pdrnn_lstm_large_supported(a->H) || ndir < 1 || ndir > 2) return hipErrorInvalidValue;
  if (dtype == 0) return pdrnn::dispatch_step<pdrnn::BF16>(a, ndir, backward != 0, tile, stream);
  return pdrnn::dispatch_step<pdrnn::F16>(a, ndir, backward != 0, tile, stream);
}

hipError_t pdrnn_lstm_large_bwd_first(const PdrnnLstmLargeStepArgs* a, int ndir, int dtype, hipStream_t stream) {
  const int64_t n = (int64_t)a->B * a->H;
  dim3 grid((unsigned)((n + 255) / 256), 1, ndir);
  if (dtype == 0)
    hipLaunchKernelGGL(pdrnn::lstm_large_bwd_first_kernel<pdrnn::BF16>, grid, dim3(256), 0, stream, *a);
  else
    hipLaunchKernelGGL(pdrnn::lstm_large_bwd_first_kernel<pdrnn::F16>, grid, dim3(256), 0, stream, *a);
  return hipGetLastError();
}

hipError_t pdrnn_gemm_nt(const uint16_t* A, int64_t lda, const uint16_t* Bt, int64_t ldb, float* C, int64_t ldc,
                         int M, int N, int K, int dtype, hipStream_t stream) {
  if (K % 64 || N % 64) return hipErrorInvalidValue;
  dim3 grid(N / 64, (M + 63) / 64);
  const size_t lds = sizeof(uint16_t) * pdrnn::GemmNT<pdrnn::BF16, 64, 64>::LDS_ELEMS;
  if (dtype == 0)
    hipLaunchKernelGGL((pdrnn::gemm_nt_kernel<pdrnn::BF16, 64, 64>), grid, dim3(256), lds, stream, A, lda, Bt, ldb,
                       C, ldc, M, N, K);
  else
    hipLaunchKernelGGL((pdrnn::gemm_nt_kernel<pdrnn::F16, 64, 64>), grid, dim3(256), lds, stream, A, lda, Bt, ldb,
                       C, ldc, M, N, K);
  return hipGetLastError();
}

}  // extern "C"
