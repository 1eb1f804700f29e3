// fp32-product GEMM on the matrix cores (v_mfma_f32_16x16x4_f32) for the
// large-H layers' time-batched products that the 16-bit ping-pong GEMM
// (kernels/gemm.hip) does not serve:
//   * fp32 models (the reference trains in fp32 with a user-set hidden size:
//     reference src/motion/main.py:20-21, src/motion/model.py:9): the input
//     projection Xp = X W_ih^T + b, dW_hh, dW_ih (+ db as the row sums of
//     dgates^T, fused into the same pass) and dX of ops/lstm_large.py /
//     ops/gru_large.py for H >= 128;
//   * narrow outputs (N < 128, e.g. the bi-LSTM's 32-wide head) with 16-bit
//     inputs, which would idle most of a 256-wide ping-pong tile.
// 16-bit inputs are widened to fp32 on their way into LDS (exact) and multiplied
// on v_mfma_f32_16x16x16{bf16,f16} (one instruction per 16-deep k-tile); fp32
// inputs on v_mfma_f32_16x16x4_f32.  Products exact, accumulation fp32 (the
// numerics of torch's matmul up to summation order).
//
//   C[M, N] (= or +=) sum over the K segments of op(A) op(B) (+ bias[n])
//   A: a_kmajor ? (m, k) at A[k * lda + m] : A[m * lda + k]    (same for B / n)
//   segment 2 (K2 > 0): A2 / B2 with lda2 / ldb2, same layouts
//   rowsum (optional): [splitk][M] sums over K of op(A)(m, k) -- the bias
//   gradient of a dW = dgates^T x product, free beside the MFMAs
//   splitk > 1: fp32 partials at C + s * c_split_stride (ldc = N), summed in a
//   fixed order by pdrnn_splitk_sum (deterministic).
//
// Tile: 128 x BN (BN in {32, 64, 128}) x 16, 256 threads = 4 waves, each wave
// a (128 / WAVES_M) x (BN / WAVES_N) block of 16 x 16 MFMA tiles.  Operands
// are staged k-major in LDS ([k][m] / [k][n], rows padded by 16 floats: the 4
// k-rows a fragment read touches land on 4 distinct 16-bank groups), double
// buffered with the next tile's global loads in registers during the MFMAs.
#include "pdrnn/api.h"
#include "pdrnn/common.h"

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

namespace pdrnn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int GF_BM = 128, GF_THREADS = 256, GF_PAD = 16;
// k-tile depth: 32 for fp32 inputs with a k-major A (the weight-gradient
// products G^T X: 8 MFMA k-steps between barriers, -4 % / -18 % on the fp32
// motion model's dW shapes), 16 otherwise (a row-major A is transposed into
// LDS element by element -- 32 made those shapes 8-31 % slower; 16-bit inputs
// take one v_mfma_f32_16x16x16 per tile).  profiles/r4/h3/ vs profiles/r4/rd5/.
template <int IN, bool AKM>
constexpr int gf_bk() { return IN == 2 && AKM ? 32 : 16; }

template <int IN>
__device__ __forceinline__ float ld1(const void* p, int64_t i) {
  if constexpr (IN == 2) return static_cast<const float*>(p)[i];
  else if constexpr (IN == 0) return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
  else return __half2float(static_cast<const __half*>(p)[i]);
}

// 4 consecutive elements of a row starting at column c (of `cols`), row r (of
// `rows`); out-of-range elements read 0.  vec: row stride and base allow one
// aligned vector load when the whole quad is in range.
template <int IN>
__device__ __forceinline__ float4 quad(const void* p, int64_t ld, int r, int c, int rows, int cols, bool vec) {
  const int64_t i = (int64_t)r * ld + c;
  if (vec && r < rows && c + 3 < cols) {
    if constexpr (IN == 2) {
      return *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    } else {
      const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
      if constexpr (IN == 0) {
        return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                           __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        const __half2 h0 = __builtin_bit_cast(__half2, u.x), h1 = __builtin_bit_cast(__half2, u.y);
        return make_float4(__low2float(h0), __high2float(h0), __low2float(h1), __high2float(h1));
      }
    }
  }
  float v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = (r < rows && c + j < cols) ? ld1<IN>(p, i + j) : 0.f;
  return make_float4(v[0], v[1], v[2], v[3]);
}

// the same without bounds checks (a tile known to be in range, vec layout)
template <int IN>
__device__ __forceinline__ float4 quad_nb(const void* p, int64_t i) {
  if constexpr (IN == 2) {
    return *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
    if constexpr (IN == 0) {
      return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                         __uint_as_float(u.y & 0xffff0000u));
    } else {
      const __half2 h0 = __builtin_bit_cast(__half2, u.x), h1 = __builtin_bit_cast(__half2, u.y);
      return make_float4(__low2float(h0), __high2float(h0), __low2float(h1), __high2float(h1));
    }
  }
}

template <int BN, int GF_BK>
struct GfCfg {
  static constexpr int WN_WAVES = BN == 128 ? 2 : 1;
  static constexpr int WM_WAVES = 4 / WN_WAVES;
  static constexpr int WM = GF_BM / WM_WAVES, WN = BN / WN_WAVES;
  static constexpr int MI = WM / 16, NI = WN / 16;
  static constexpr int A_QUADS = GF_BM * GF_BK / 4 / GF_THREADS;     // per thread (2 or 4)
  static constexpr int B_QUADS = (BN * GF_BK / 4 + GF_THREADS - 1) / GF_THREADS;
  static constexpr int LDA_S = GF_BM + GF_PAD, LDB_S = BN + GF_PAD;
};

template <int IN, bool AKM, bool BKM, int BN>
__global__ void __launch_bounds__(GF_THREADS) gemm_f32_kernel(PdrnnGemmF32Args p) {
  constexpr int GF_BK = gf_bk<IN, AKM>();
  using Cfg = GfCfg<BN, GF_BK>;
  __shared__ __attribute__((aligned(16))) float As[2][GF_BK][Cfg::LDA_S];
  __shared__ __attribute__((aligned(16))) float Bs[2][GF_BK][Cfg::LDB_S];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / Cfg::WN_WAVES, wn = wave % Cfg::WN_WAVES;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * GF_BM, n0 = tn * BN;
  const int nt1 = (p.K + GF_BK - 1) / GF_BK, nt2 = p.K2 > 0 ? (p.K2 + GF_BK - 1) / GF_BK : 0;
  const int nt = nt1 + nt2;
  const int split = blockIdx.y, nsplit = gridDim.y;
  const int t_begin = (int)((int64_t)nt * split / nsplit), t_end = (int)((int64_t)nt * (split + 1) / nsplit);
  const bool vec = p.vec != 0;
  const bool do_rs = p.rowsum != nullptr && tn == 0 && wn == 0;

  float4 ra[Cfg::A_QUADS], rb[Cfg::B_QUADS];
  // global -> registers: the quads of k-tile t (segment 1 or 2)
  auto load = [&](int t, float4 (&xa)[Cfg::A_QUADS], float4 (&xb)[Cfg::B_QUADS]) {
    const bool s2 = t >= nt1;
    const void* A = s2 ? p.A2 : p.A;
    const void* B = s2 ? p.B2 : p.B;
    const int64_t lda = s2 ? p.lda2 : p.lda, ldb = s2 ? p.ldb2 : p.ldb;
    const int K = s2 ? p.K2 : p.K;
    const int k0 = (s2 ? t - nt1 : t) * GF_BK;
#pragma unroll
    for (int j = 0; j < Cfg::A_QUADS; ++j) {
      const int q = tid + j * GF_THREADS;
      if constexpr (AKM) xa[j] = quad<IN>(A, lda, k0 + q / (GF_BM / 4), m0 + (q % (GF_BM / 4)) * 4, K, p.M, vec);
      else xa[j] = quad<IN>(A, lda, m0 + q / (GF_BK / 4), k0 + (q % (GF_BK / 4)) * 4, p.M, K, vec);
    }
#pragma unroll
    for (int j = 0; j < Cfg::B_QUADS; ++j) {
      const int q = tid + j * GF_THREADS;
      if (q < BN * GF_BK / 4) {
        if constexpr (BKM) xb[j] = quad<IN>(B, ldb, k0 + q / (BN / 4), n0 + (q % (BN / 4)) * 4, K, p.N, vec);
        else xb[j] = quad<IN>(B, ldb, n0 + q / (GF_BK / 4), k0 + (q % (GF_BK / 4)) * 4, p.N, K, vec);
      }
    }
  };
  // the same for a tile known to be in range (vec layout): straight-line
  // vector loads.  Run from a loop of its own: with the bounds-checked loads
  // in the same loop, the divergent branches around them made the compiler
  // join register copies of the loaded values -- and wait for every load
  // (s_waitcnt vmcnt(0)) -- before the MFMAs, so the next tile's loads never
  // overlapped them (profiles/r4/gemm_probe/)
  auto load_fast = [&](int t, float4 (&xa)[Cfg::A_QUADS], float4 (&xb)[Cfg::B_QUADS]) {
    const bool s2 = t >= nt1;
    const void* A = s2 ? p.A2 : p.A;
    const void* B = s2 ? p.B2 : p.B;
    const int64_t lda = s2 ? p.lda2 : p.lda, ldb = s2 ? p.ldb2 : p.ldb;
    const int k0 = (s2 ? t - nt1 : t) * GF_BK;
#pragma unroll
    for (int j = 0; j < Cfg::A_QUADS; ++j) {
      const int q = tid + j * GF_THREADS;
      if constexpr (AKM) xa[j] = quad_nb<IN>(A, (int64_t)(k0 + q / (GF_BM / 4)) * lda + m0 + (q % (GF_BM / 4)) * 4);
      else xa[j] = quad_nb<IN>(A, (int64_t)(m0 + q / (GF_BK / 4)) * lda + k0 + (q % (GF_BK / 4)) * 4);
    }
#pragma unroll
    for (int j = 0; j < Cfg::B_QUADS; ++j) {
      const int q = tid + j * GF_THREADS;
      if ((BN * GF_BK / 4) % GF_THREADS == 0 || q < BN * GF_BK / 4) {  // (compile-time true when B tiles evenly)
        if constexpr (BKM) xb[j] = quad_nb<IN>(B, (int64_t)(k0 + q / (BN / 4)) * ldb + n0 + (q % (BN / 4)) * 4);
        else xb[j] = quad_nb<IN>(B, (int64_t)(n0 + q / (GF_BK / 4)) * ldb + k0 + (q % (GF_BK / 4)) * 4);
      }
    }
  };
  // registers -> LDS (k-major images)
  auto store = [&](int buf, const float4 (&xa)[Cfg::A_QUADS], const float4 (&xb)[Cfg::B_QUADS]) {
#pragma unroll
    for (int j = 0; j < Cfg::A_QUADS; ++j) {
      const int q = tid + j * GF_THREADS;
      if constexpr (AKM) {
        *reinterpret_cast<float4*>(&As[buf][q / (GF_BM / 4)][(q % (GF_BM / 4)) * 4]) = xa[j];
      } else {
        const int m = q / (GF_BK / 4), k = (q % (GF_BK / 4)) * 4;
        As[buf][k][m] = xa[j].x; As[buf][k + 1][m] = xa[j].y; As[buf][k + 2][m] = xa[j].z; As[buf][k + 3][m] = xa[j].w;
      }
    }
#pragma unroll
    for (int j = 0; j < Cfg::B_QUADS; ++j) {
      const int q = tid + j * GF_THREADS;
      if (q < BN * GF_BK / 4) {
        if constexpr (BKM) {
          *reinterpret_cast<float4*>(&Bs[buf][q / (BN / 4)][(q % (BN / 4)) * 4]) = xb[j];
        } else {
          const int n = q / (GF_BK / 4), k = (q % (GF_BK / 4)) * 4;
          Bs[buf][k][n] = xb[j].x; Bs[buf][k + 1][n] = xb[j].y; Bs[buf][k + 2][n] = xb[j].z; Bs[buf][k + 3][n] = xb[j].w;
        }
      }
    }
  };

  f32x4 acc[Cfg::MI][Cfg::NI];
#pragma unroll
  for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float rs[Cfg::MI];
#pragma unroll
  for (int i = 0; i < Cfg::MI; ++i) rs[i] = 0.f;

  const int fr = lane & 15, fk = lane >> 4;  // fragment row / column, k within a 4-step
  const int am = wm * Cfg::WM + fr, bn = wn * Cfg::WN + fr;
  auto compute = [&](int buf) {
    if constexpr (IN == 2) {
      // fp32: 4 k-steps of v_mfma_f32_16x16x4_f32 (lane: row fr, k = 4 ks + fk)
#pragma unroll
      for (int ks = 0; ks < GF_BK / 4; ++ks) {
        const int k = ks * 4 + fk;
        float a[Cfg::MI], b[Cfg::NI];
#pragma unroll
        for (int i = 0; i < Cfg::MI; ++i) a[i] = As[buf][k][am + i * 16];
#pragma unroll
        for (int j = 0; j < Cfg::NI; ++j) b[j] = Bs[buf][k][bn + j * 16];
#pragma unroll
        for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
          for (int j = 0; j < Cfg::NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        if (do_rs) {
#pragma unroll
          for (int i = 0; i < Cfg::MI; ++i) rs[i] += a[i];
        }
      }
    } else {
      // 16-bit inputs (staged as exact fp32): the whole k-tile in ONE
      // v_mfma_f32_16x16x16{bf16,f16} per output tile (lane: row fr, k = 4 fk + e),
      // the fp32 -> 16-bit re-pack exact
      typedef short s16x4 __attribute__((ext_vector_type(4)));
      typedef _Float16 h16x4 __attribute__((ext_vector_type(4)));
      s16x4 a[Cfg::MI], b[Cfg::NI];
      auto pack = [](float x0, float x1, float x2, float x3) {
        s16x4 v;
        if constexpr (IN == 0) {
          v = s16x4{(short)(__float_as_uint(x0) >> 16), (short)(__float_as_uint(x1) >> 16),
                    (short)(__float_as_uint(x2) >> 16), (short)(__float_as_uint(x3) >> 16)};
        } else {
          const h16x4 h = h16x4{(_Float16)x0, (_Float16)x1, (_Float16)x2, (_Float16)x3};
          v = __builtin_bit_cast(s16x4, h);
        }
        return v;
      };
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i) {
        const float x0 = As[buf][4 * fk][am + i * 16], x1 = As[buf][4 * fk + 1][am + i * 16];
        const float x2 = As[buf][4 * fk + 2][am + i * 16], x3 = As[buf][4 * fk + 3][am + i * 16];
        a[i] = pack(x0, x1, x2, x3);
        if (do_rs) rs[i] += (x0 + x1) + (x2 + x3);
      }
#pragma unroll
      for (int j = 0; j < Cfg::NI; ++j)
        b[j] = pack(Bs[buf][4 * fk][bn + j * 16], Bs[buf][4 * fk + 1][bn + j * 16], Bs[buf][4 * fk + 2][bn + j * 16],
                    Bs[buf][4 * fk + 3][bn + j * 16]);
#pragma unroll
      for (int i = 0; i < Cfg::MI; ++i)
#pragma unroll
        for (int j = 0; j < Cfg::NI; ++j) {
          if constexpr (IN == 0)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a[i], b[j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x16f16(__builtin_bit_cast(h16x4, a[i]),
                                                              __builtin_bit_cast(h16x4, b[j]), acc[i][j], 0, 0, 0);
        }
    }
  };
  // one k-tile of loads in flight during the MFMAs of the current one (two
  // register sets for fp32 inputs measured no faster and the dX / Xp shapes
  // slower: profiles/r4/h2/h2tb_motion_h128_kernel_stats.md vs rd5)
  int buf = 0;
  if (t_begin < t_end) {
    load(t_begin, ra, rb);
    store(0, ra, rb);
  }
  __syncthreads();
  if (vec && m0 + GF_BM <= p.M && n0 + BN <= p.N && p.K % GF_BK == 0 && p.K2 % GF_BK == 0) {
    for (int t = t_begin; t < t_end; ++t) {  // every tile in range
      const bool more = t + 1 < t_end;
      if (more) load_fast(t + 1, ra, rb);  // in flight during the MFMAs below
      compute(buf);
      if (more) store(buf ^ 1, ra, rb);
      __syncthreads();
      buf ^= 1;
    }
  } else {
    for (int t = t_begin; t < t_end; ++t) {
      const bool more = t + 1 < t_end;
      if (more) load(t + 1, ra, rb);
      compute(buf);
      if (more) store(buf ^ 1, ra, rb);
      __syncthreads();
      buf ^= 1;
    }
  }

  // ---- epilogue: lane holds rows 4 fk + r, column fr of every 16 x 16 tile
  const bool partial = nsplit > 1;
  float* Cf = static_cast<float*>(p.C) + (partial ? (int64_t)split * p.c_split_stride : 0);
#pragma unroll
  for (int i = 0; i < Cfg::MI; ++i) {
#pragma unroll
    for (int j = 0; j < Cfg::NI; ++j) {
      const int n = n0 + wn * Cfg::WN + j * 16 + fr;
      if (n >= p.N) continue;
      const float bias = (!partial && p.bias) ? p.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * Cfg::WM + i * 16 + 4 * fk + r;
        if (m >= p.M) continue;
        const int64_t o = (int64_t)m * p.ldc + n;
        float v = acc[i][j][r] + bias;
        if (p.out_dtype == 2 || partial) {
          if (p.accumulate && !partial) v += Cf[o];
          Cf[o] = v;
        } else if (p.out_dtype == 0) {
          static_cast<__hip_bfloat16*>(p.C)[o] = __float2bfloat16(v);
        } else {
          static_cast<__half*>(p.C)[o] = __float2half(v);
        }
      }
    }
  }
  if (do_rs) {
#pragma unroll
    for (int i = 0; i < Cfg::MI; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const int m = m0 + wm * Cfg::WM + i * 16 + fr;
      if (fk == 0 && m < p.M) p.rowsum[(int64_t)split * p.M + m] = v;
    }
  }
}

template <int IN, bool AKM, bool BKM>
hipError_t launch_f32(const PdrnnGemmF32Args& a, hipStream_t st) {
  const int bn = a.N <= 32 ? 32 : a.N <= 64 ? 64 : 128;
  const int tiles = ((a.M + GF_BM - 1) / GF_BM) * ((a.N + bn - 1) / bn);
  const dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1);
  switch (bn) {
    case 32: hipLaunchKernelGGL((gemm_f32_kernel<IN, AKM, BKM, 32>), grid, dim3(GF_THREADS), 0, st, a); break;
    case 64: hipLaunchKernelGGL((gemm_f32_kernel<IN, AKM, BKM, 64>), grid, dim3(GF_THREADS), 0, st, a); break;
    default: hipLaunchKernelGGL((gemm_f32_kernel<IN, AKM, BKM, 128>), grid, dim3(GF_THREADS), 0, st, a); break;
  }
  return hipGetLastError();
}

template <int IN>
hipError_t dispatch_f32(const PdrnnGemmF32Args& a, hipStream_t st) {
  if (a.a_kmajor) return a.b_kmajor ? launch_f32<IN, true, true>(a, st) : launch_f32<IN, true, false>(a, st);
  return a.b_kmajor ? launch_f32<IN, false, true>(a, st) : launch_f32<IN, false, false>(a, st);
}

// out[i] (= or +=) sum_s part[s * n + i], fixed order (deterministic)
__global__ void __launch_bounds__(256) splitk_sum_kernel(const float* __restrict__ part, int splitk, int64_t n,
                                                         float* __restrict__ out, int accumulate) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = accumulate ? out[i] : 0.f;
    float acc = 0.f;
    int k = 0;
    // 8 partial rows in flight per thread, added in the same k order
    for (; k + 8 <= splitk; k += 8) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = part[(int64_t)(k + j) * n + i];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j];
    }
    for (; k < splitk; ++k) acc += part[(int64_t)k * n + i];
    out[i] = s + acc;
  }
}

// Column sums of a [rows, cols] matrix (row stride ld), pass 1: block (cx, ry)
// sums columns [256 cx, 256 cx + 256) over row group ry into part[ry][cols];
// the row groups are then summed by splitk_sum_kernel (fixed order).  A thread
// owns 4 consecutive columns (one 8- or 16-byte load per row where aligned)
// and every 4th row of the group, 4 rows in flight: a wave reads 256 columns
// of a row per instruction.
template <int IN>
__global__ void __launch_bounds__(256) col_sum_kernel(const void* __restrict__ X, int64_t rows, int64_t cols,
                                                      int64_t ld, float* __restrict__ part, int vec) {
  __shared__ float4 red[256];
  const int c4 = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = (int)blockIdx.x * 256 + 4 * c4;
  const int64_t r0 = rows * blockIdx.y / gridDim.y, r1 = rows * (blockIdx.y + 1) / gridDim.y;
  const int ncols = (int)cols;
  float4 acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col < ncols) {
    int64_t r = r0 + g;
    for (; r + 12 < r1; r += 16) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = quad<IN>(X, ld, (int)(r + 4 * k), col, (int)r1, ncols, vec != 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[k].x += v[k].x; acc[k].y += v[k].y; acc[k].z += v[k].z; acc[k].w += v[k].w;
      }
    }
    for (int k = 0; r < r1; r += 4, ++k) {
      const float4 v = quad<IN>(X, ld, (int)r, col, (int)r1, ncols, vec != 0);
      acc[k & 3].x += v.x; acc[k & 3].y += v.y; acc[k & 3].z += v.z; acc[k & 3].w += v.w;
    }
  }
  float4 t;
  t.x = (acc[0].x + acc[1].x) + (acc[2].x + acc[3].x);
  t.y = (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y);
  t.z = (acc[0].z + acc[1].z) + (acc[2].z + acc[3].z);
  t.w = (acc[0].w + acc[1].w) + (acc[2].w + acc[3].w);
  red[threadIdx.x] = t;
  __syncthreads();
  if (g == 0 && col < ncols) {
    const float4 a = red[c4], b = red[64 + c4], c = red[128 + c4], d = red[192 + c4];
    const float o[4] = {(a.x + b.x) + (c.x + d.x), (a.y + b.y) + (c.y + d.y), (a.z + b.z) + (c.z + d.z),
                        (a.w + b.w) + (c.w + d.w)};
    float* dst = part + (int64_t)blockIdx.y * cols + col;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (col + j < ncols) dst[j] = o[j];
  }
}

// 16-bit column sums, 8 columns per thread (one 16-byte load per row) and 8
// rows in flight: twice the bytes per load and twice the loads in flight of
// col_sum_kernel, which left the bi-LSTM's 8.6 GB db pass at ~3.5 TB/s.  Same
// fixed summation order per (column, row group) (deterministic).
template <int IN>
__global__ void __launch_bounds__(256) col_sum16_kernel(const uint16_t* __restrict__ X, int64_t rows, int64_t cols,
                                                        int64_t ld, float* __restrict__ part) {
  __shared__ float red[4][64][9];
  const int c8 = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.x * 512 + 8 * c8;
  const int64_t r0 = rows * blockIdx.y / gridDim.y, r1 = rows * (blockIdx.y + 1) / gridDim.y;
  float acc[2][8];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
  auto add = [&](float (&dst)[8], const uint4& u) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (IN == 0) {
        dst[2 * j] += __uint_as_float(w[j] << 16);
        dst[2 * j + 1] += __uint_as_float(w[j] & 0xffff0000u);
      } else {
        const __half2 h = __builtin_bit_cast(__half2, w[j]);
        dst[2 * j] += __low2float(h);
        dst[2 * j + 1] += __high2float(h);
      }
    }
  };
  if (col < cols) {
    int64_t r = r0 + g;
    for (; r + 28 < r1; r += 32) {
      uint4 v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const uint4*>(X + (r + 4 * k) * ld + col);
#pragma unroll
      for (int k = 0; k < 8; ++k) add(acc[k & 1], v[k]);
    }
    for (int k = 0; r < r1; r += 4, ++k) add(acc[k & 1], *reinterpret_cast<const uint4*>(X + r * ld + col));
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[g][c8][j] = acc[0][j] + acc[1][j];
  __syncthreads();
  if (g == 0 && col < cols) {
    float* dst = part + (int64_t)blockIdx.y * cols + col;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[j] = (red[0][c8][j] + red[1][c8][j]) + (red[2][c8][j] + red[3][c8][j]);
  }
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_gemm_f32_supported(const PdrnnGemmF32Args* a) {
  if (a->M < 1 || a->N < 1 || a->K < 1 || a->K2 < 0 || (a->K2 > 0 && (!a->A2 || !a->B2))) return 0;
  if (a->in_dtype < 0 || a->in_dtype > 2 || (a->out_dtype != 2 && a->out_dtype != a->in_dtype)) return 0;
  if (a->splitk > 1 && (a->out_dtype != 2 || a->accumulate || a->bias)) return 0;
  if (a->out_dtype != 2 && a->accumulate) return 0;
  return 1;
}

hipError_t pdrnn_gemm_f32(const PdrnnGemmF32Args* a, hipStream_t stream) {
  if (!pdrnn_gemm_f32_supported(a)) return hipErrorInvalidValue;
  switch (a->in_dtype) {
    case 0: return pdrnn::dispatch_f32<0>(*a, stream);
    case 1: return pdrnn::dispatch_f32<1>(*a, stream);
    default: return pdrnn::dispatch_f32<2>(*a, stream);
  }
}

hipError_t pdrnn_splitk_sum(const float* part, int splitk, int64_t n, float* out, int accumulate, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pdrnn::splitk_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, part, splitk, n, out,
                     accumulate);
  return hipGetLastError();
}

int pdrnn_col_sum_groups(int64_t rows, int64_t cols) {
  // ~4 workgroups per CU, at least 64 rows per group
  const int64_t cblocks = (cols + 255) / 256;
  int64_t g = (1024 + cblocks - 1) / cblocks;
  if (g > rows / 64) g = rows / 64;
  if (g > 1024) g = 1024;
  return g < 1 ? 1 : (int)g;
}

hipError_t pdrnn_col_sum(const void* X, int dtype, int64_t rows, int64_t cols, int64_t ld, float* part, int groups,
                         hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (rows >= (1LL << 31) || cols >= (1LL << 31)) return hipErrorInvalidValue;
  const int esz = dtype == 2 ? 4 : 2;
  const int vec = (ld % 4 == 0 && reinterpret_cast<uintptr_t>(X) % (4 * esz) == 0) ? 1 : 0;
  if (dtype != 2 && cols % 512 == 0 && ld % 8 == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0) {
    const dim3 g8((unsigned)(cols / 512), (unsigned)groups);
    const uint16_t* X16 = static_cast<const uint16_t*>(X);
    if (dtype == 0) hipLaunchKernelGGL(pdrnn::col_sum16_kernel<0>, g8, dim3(256), 0, stream, X16, rows, cols, ld, part);
    else hipLaunchKernelGGL(pdrnn::col_sum16_kernel<1>, g8, dim3(256), 0, stream, X16, rows, cols, ld, part);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((cols + 255) / 256), (unsigned)groups);
  switch (dtype) {
    case 0: hipLaunchKernelGGL(pdrnn::col_sum_kernel<0>, grid, dim3(256), 0, stream, X, rows, cols, ld, part, vec); break;
    case 1: hipLaunchKernelGGL(pdrnn::col_sum_kernel<1>, grid, dim3(256), 0, stream, X, rows, cols, ld, part, vec); break;
    default: hipLaunchKernelGGL(pdrnn::col_sum_kernel<2>, grid, dim3(256), 0, stream, X, rows, cols, ld, part, vec); break;
  }
  return hipGetLastError();
}

}  // extern "C"
