// Large-hidden LSTM (H = 64k: bf16 / fp16 storage on v_mfma_f32_16x16x32, or
// fp32 storage on v_mfma_f32_16x16x4_f32; fp32 accumulation and cell state)
// for gfx950.
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
// The same kernels serve the large-H GRU (CELL = 1, ops/gru_large.py): its
// gates ride on the LSTM quad as [r | z | n_x | n_h] with zero weight blocks.
//
// Reference semantics: torch.nn.LSTM (gate order i, f, g, o), the op the
// reference's MotionModel uses (reference: src/motion/model.py:9,14).
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <type_traits>

#include "pdrnn/api.h"
#include "pdrnn/common.h"
#include "pdrnn/gemm_pp.h"

namespace pdrnn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// storage type tags.  S: element type in HBM / LDS; EPC: elements per 16-byte
// chunk (an LDS tile row is 8 chunks = 128 bytes: BK = 8 * EPC elements);
// mfma: one 16-byte chunk per operand and lane -> one K-slab of the tile.
struct BF16 {
  typedef uint16_t S;
  static constexpr int EPC = 8;
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
  typedef uint16_t S;
  static constexpr int EPC = 8;
  static __device__ __forceinline__ float to_f(uint16_t v) { return (float)__builtin_bit_cast(_Float16, v); }
  static __device__ __forceinline__ uint16_t from_f(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }
  static __device__ __forceinline__ f32x4 mfma(const uint4& a, const uint4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b),
                                                  c, 0, 0, 0);
  }
};
// fp32 storage on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32
// accumulation; 157 TF/s dense = the fp32 vector peak, reached by the matrix
// pipe without VALU issue pressure).  A lane's 16-byte chunk holds 4
// consecutive k; the k-slab of chunk c is split into 4 MFMAs, MFMA m taking
// component m -- lane group fq of MFMA m then covers k = 4 (ks*4 + fq) + m,
// identical for A and B, so the 4 MFMAs sum the slab exactly once.
struct F32 {
  typedef float S;
  static constexpr int EPC = 4;
  static __device__ __forceinline__ float to_f(float v) { return v; }
  static __device__ __forceinline__ float from_f(float f) { return f; }
  static __device__ __forceinline__ f32x4 mfma(const uint4& a, const uint4& b, f32x4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), c, 0, 0, 0);
  }
};

// 8 consecutive elements of storage type DT (16 or 32 bytes)
template <class DT>
struct V8 {
  uint4 v[sizeof(typename DT::S) / 2];
  __device__ __forceinline__ float get(int k) const { return DT::to_f(reinterpret_cast<const typename DT::S*>(v)[k]); }
  __device__ __forceinline__ void set(int k, float f) { reinterpret_cast<typename DT::S*>(v)[k] = DT::from_f(f); }
};
template <class DT>
__device__ __forceinline__ V8<DT> ld_v8(const typename DT::S* p) { return *reinterpret_cast<const V8<DT>*>(p); }
template <class DT>
__device__ __forceinline__ void st_v8(typename DT::S* p, const V8<DT>& v) { *reinterpret_cast<V8<DT>*>(p) = v; }

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

// LDS image of a [ROWS x 8 chunks] tile (128 bytes per row): 16-byte chunk c
// of row r lives at chunk slot (c ^ (r & 7)) -- the XOR swizzle spreads the
// 16 rows an MFMA fragment read touches over all bank groups.  Offsets in
// elements of DT::S.
template <class DT>
__device__ __forceinline__ int lds_off(int row, int chunk) {
  return row * 8 * DT::EPC + (chunk ^ (row & 7)) * DT::EPC;
}

// C[M, N] = A[M, K] * Bt[N, K]^T for one BM x BN block tile, WM x WN waves,
// each wave (BM/WM) x (BN/WN) = MT x NT 16x16 MFMA sub-tiles.  A / Bt are
// DT::S, K-contiguous (lda / ldb).  Rows of A beyond M are clamped (the
// caller discards their results).  K % BK == 0 (BK = 64 16-bit / 32 fp32).
//
// Staging: direct global->LDS DMA (global_load_lds_dwordx4, 1 KiB per wave
// instruction) into a STAGES-deep ring of [BM+BN][64] tiles, prefetch distance
// STAGES-1 k-tiles, retired by a counted `s_waitcnt vmcnt` + raw s_barrier so
// the DMAs stay in flight across barriers (a __syncthreads() would drain
// them).  The XOR swizzle of the LDS image is applied on the per-lane global
// SOURCE address (the DMA destination is lane-linear).  All LDS is the one
// dynamic array (a second __shared__ object makes hipcc drain vmcnt before
// every ds_read).
template <class DT, int BM, int BN, int WM, int WN, int STAGES>
struct GemmPipe {
  typedef typename DT::S S;
  static constexpr int BK = 8 * DT::EPC;        // K elements per LDS tile row
  static constexpr int NWAVES = WM * WN, NTHREADS = NWAVES * 64;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int MT = WTM / 16, NT = WTN / 16;
  static constexpr int ROWS = BM + BN;
  static constexpr int STAGE_ELEMS = ROWS * BK;
  static constexpr int GROUPS = ROWS * 8 / 64;  // 1 KiB DMA groups per stage
  static constexpr int G = GROUPS / NWAVES;     // DMA instructions per wave per stage
  static constexpr int LDS_ELEMS = STAGES * STAGE_ELEMS;
  static_assert(GROUPS % NWAVES == 0, "DMA groups must split evenly over the waves");
  static_assert(MT >= 1 && NT >= 1 && BM % 8 == 0, "tile shape");

  template <int N>
  __device__ static __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  }

  __device__ static void run(const S* __restrict__ A, int64_t lda, const S* __restrict__ Bt,
                             int64_t ldb, int M, int K, int m0, int n0, S* smem, f32x4 (&acc)[MT][NT]) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid / WN, wn = wid % WN;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const S* src[G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int cid = (wid * G + i) * 64 + lane;
      const int row = cid >> 3, slot = cid & 7;
      const int lc = slot ^ (row & 7);
      src[i] = row < BM ? A + (int64_t)min(m0 + row, M - 1) * lda + lc * DT::EPC
                        : Bt + (int64_t)(n0 + row - BM) * ldb + lc * DT::EPC;
    }
    auto issue = [&](int kt, int st) {
      constexpr int GE = 64 * DT::EPC;  // elements per 1 KiB DMA group
      S* base = smem + st * STAGE_ELEMS + wid * G * GE;
#pragma unroll
      for (int i = 0; i < G; ++i)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(src[i] + kt * BK),
                                         (__attribute__((address_space(3))) void*)(base + i * GE), 16, 0, 0);
    };
    const int KT = K / BK;
#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
      if (p < KT) issue(p, p);

    const int fr = lane & 15, fq = lane >> 4;
    for (int kt = 0; kt < KT; ++kt) {
      // tiles issued after kt that may stay in flight: min(STAGES-2, KT-1-kt)
      const int ahead = min(STAGES - 2, KT - 1 - kt);
      if constexpr (STAGES >= 4) {
        if (ahead >= 2) wait_vm<2 * G>();
        else if (ahead == 1) wait_vm<G>();
        else wait_vm<0>();
      } else {
        if (ahead >= 1) wait_vm<G>();
        else wait_vm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (kt + STAGES - 1 < KT) issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
      const S* sA = smem + (kt % STAGES) * STAGE_ELEMS;
      const S* sB = sA + BM * BK;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {  // 2 k-slabs of 4 chunks per tile row
        uint4 fa[MT], fb[NT];
#pragma unroll
        for (int i = 0; i < MT; ++i)
          fa[i] = *reinterpret_cast<const uint4*>(sA + lds_off<DT>(wm * WTM + i * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int j = 0; j < NT; ++j)
          fb[j] = *reinterpret_cast<const uint4*>(sB + lds_off<DT>(wn * WTN + j * 16 + fr, ks * 4 + fq));
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j] = DT::mfma(fa[i], fb[j], acc[i][j]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
};

// Tile configurations (BM, BN, WM, WN, STAGES)
#define TILE_CFGS_X(X)   \
  X(0, 32, 64, 1, 4, 4)      \
  X(1, 64, 64, 2, 2, 4)      \
  X(2, 128, 128, 2, 2, 3)    \
  X(3, 256, 128, 4, 2, 3)    \
  X(4, 32, 32, 2, 2, 4)

// ---------------------------------------------------------------------------
// Forward step: gates = h_{t-1} Wp^T + xp_t  ->  (i, f, g, o), c_t, h_t.
// Columns are gate-interleaved: col = 4 u + q.
// ---------------------------------------------------------------------------
// CELL 1 = GRU on the same quad (host packing in ops/gru_large.py): the four
// columns of a unit are [r | z | n_x | n_h] (n_x = W_in x + b_in from xp,
// n_h = W_hn h + b_hn), cseq holds the fp32 hidden state h_t, and the saved
// quad is (r, z, n, n_h).
template <class DT, int BM, int BN, int WM, int WN, int ST, int CELL>
__global__ void __launch_bounds__(WM * WN * 64) lstm_large_fwd_step_kernel(PdrnnLstmLargeStepArgs args) {
  typedef GemmPipe<DT, BM, BN, WM, WN, ST> G;
  typedef typename DT::S S;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  S* const smem = reinterpret_cast<S*>(smem_raw);
  const PdrnnLstmLargeDir& d = args.dir[blockIdx.z];
  const int B = args.B, H = args.H;
  const int t = args.reverse_mask & (1 << blockIdx.z) ? args.T - 1 - args.step : args.step;
  const int tp = args.reverse_mask & (1 << blockIdx.z) ? t + 1 : t - 1;  // previous step in processing order
  const bool first = args.step == 0;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  // A operand: h_{prev} rows of the output sequence (or h0)
  const S* hA = first ? static_cast<const S*>(d.h0) : static_cast<const S*>(d.hseq) + (int64_t)tp * d.hseq_st;
  const int64_t lda = first ? H : d.hseq_sb;
  f32x4 acc[G::MT][G::NT];
  if (first && d.h0 == nullptr) {
#pragma unroll
    for (int i = 0; i < G::MT; ++i)
#pragma unroll
      for (int j = 0; j < G::NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    G::run(hA, lda, static_cast<const S*>(d.w), H, B, H, m0, n0, smem, acc);
  }

  // Epilogue through LDS: the C tile is parked as fp32 [BM][BN+4] in the
  // (now idle) staging ring, then every thread owns 8 consecutive columns
  // (= 2 hidden units x 4 gates) of a row: 16-byte loads of xp, 16-byte
  // stores of the activated gates, 8-byte c and 4-byte h -- instead of
  // 2-byte scattered accesses straight from the MFMA C layout.
  constexpr int LDC = BN + 4;
  static_assert(BM * LDC * 4 <= G::LDS_ELEMS * sizeof(S), "C tile must fit in the staging ring");
  float* cs = reinterpret_cast<float*>(smem_raw);
  {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / WN, wn = wid % WN;
#pragma unroll
    for (int i = 0; i < G::MT; ++i)
#pragma unroll
      for (int j = 0; j < G::NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(wm * G::WTM + i * 16 + (lane >> 4) * 4 + r) * LDC + wn * G::WTN + j * 16 + (lane & 15)] = acc[i][j][r];
  }
  __syncthreads();
  const S* xp = static_cast<const S*>(d.xp) + (int64_t)t * d.xp_st;
  const float* cprev = first ? d.c0 : d.cseq + (int64_t)tp * B * H;
  float* cout = d.cseq + (int64_t)t * B * H;
  S* hout = static_cast<S*>(d.hseq) + (int64_t)t * d.hseq_st;
  S* acts = static_cast<S*>(d.acts) + (int64_t)t * B * 4 * H;
  constexpr int C8 = BN / 8;
  // Every item's global operands (xp, c_prev) and C-tile slice are loaded
  // first, then the cell math and stores run: the loads of all items are in
  // flight together instead of one HBM round trip per item (with one
  // workgroup per CU the epilogue is not hidden behind another workgroup's
  // MFMA loop).
  constexpr int ITEMS = (BM * C8 + G::NTHREADS - 1) / G::NTHREADS;
  V8<DT> xv[ITEMS];
  float2 cpv[ITEMS];
  float4 za[ITEMS], zb[ITEMS];
#pragma unroll
  for (int it = 0; it < ITEMS; ++it) {
    const int e = min((int)threadIdx.x + it * G::NTHREADS, BM * C8 - 1);
    const int row = e / C8, c8 = e - row * C8;
    const int b = min(m0 + row, B - 1);
    const int col = n0 + c8 * 8;
    xv[it] = ld_v8<DT>(xp + (int64_t)b * d.xp_sb + col);
    cpv[it] = cprev ? *reinterpret_cast<const float2*>(cprev + (int64_t)b * H + (col >> 2)) : make_float2(0.f, 0.f);
    za[it] = *reinterpret_cast<const float4*>(cs + row * LDC + c8 * 8);
    zb[it] = *reinterpret_cast<const float4*>(cs + row * LDC + c8 * 8 + 4);
  }
#pragma unroll
  for (int it = 0; it < ITEMS; ++it) {
    const int e = threadIdx.x + it * G::NTHREADS;
    const int row = e / C8, c8 = e - row * C8;
    const int b = m0 + row;
    if (e >= BM * C8 || b >= B) continue;
    const int col = n0 + c8 * 8;
    const float z[8] = {za[it].x, za[it].y, za[it].z, za[it].w, zb[it].x, zb[it].y, zb[it].z, zb[it].w};
    float g[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float zz = z[k] + xv[it].get(k);
      if constexpr (CELL == 0) g[k] = (k & 3) == 2 ? tanh_(zz) : sigm(zz);
      else g[k] = (k & 3) < 2 ? sigm(zz) : zz;  // GRU: r, z activated; n_x, n_h linear
    }
    const int u = col >> 2;
    const float2 cp = cpv[it];
    float s0, s1, h0v, h1v;
    if constexpr (CELL == 0) {
      s0 = fmaf(g[1], cp.x, g[0] * g[2]);
      s1 = fmaf(g[5], cp.y, g[4] * g[6]);
      h0v = g[3] * tanh_(s0);
      h1v = g[7] * tanh_(s1);
    } else {
      // n = tanh(n_x + r n_h) takes n_x's slot in the saved quad;
      // h = n + z (h_prev - n) with the fp32 h_prev
      g[2] = tanh_(fmaf(g[0], g[3], g[2]));
      g[6] = tanh_(fmaf(g[4], g[7], g[6]));
      s0 = h0v = fmaf(g[1], cp.x - g[2], g[2]);
      s1 = h1v = fmaf(g[5], cp.y - g[6], g[6]);
    }
    V8<DT> av;
#pragma unroll
    for (int k = 0; k < 8; ++k) av.set(k, g[k]);
    st_v8<DT>(acts + (int64_t)b * 4 * H + col, av);
    *reinterpret_cast<float2*>(cout + (int64_t)b * H + u) = make_float2(s0, s1);
    if constexpr (sizeof(S) == 2) {
      const uint32_t hv = (uint32_t)DT::from_f(h0v) | ((uint32_t)DT::from_f(h1v) << 16);
      *reinterpret_cast<uint32_t*>(hout + (int64_t)b * d.hseq_sb + u) = hv;
    } else {
      *reinterpret_cast<float2*>(hout + (int64_t)b * d.hseq_sb + u) = make_float2(h0v, h1v);
    }
  }
}

// Cell backward of step tn for one (b, u), given the recurrent dh from the
// step GEMM and the carry of the step after tn (LSTM: dc; GRU: the direct
// path dh_{tn+1} z_{tn+1}): emits dgates_tn and the new carry; after the
// first forward step (cell == false) it emits dh0 / dc0 instead.
template <class DT, int CELL, bool COH = false>
__device__ __forceinline__ void cell_bwd_elem(const PdrnnLstmLargeDir& d, int B, int H, int T, bool rev, int tn,
                                              bool cell, int b, int u, float dh, float carry) {
  const int64_t bu = (int64_t)b * H + u;
  if constexpr (CELL == 1) dh += carry;
  if (!cell) {
    if (d.dh0) d.dh0[bu] = dh;
    if (CELL == 0 && d.dc0) d.dc0[bu] = carry;
    return;
  }
  typedef typename DT::S S;
  if (d.dout) dh += DT::to_f(static_cast<const S*>(d.dout)[(int64_t)tn * d.dout_st + (int64_t)b * d.dout_sb + u]);
  const S* ap = static_cast<const S*>(d.acts) + ((int64_t)tn * B + b) * 4 * H + 4 * u;
  const float a0 = DT::to_f(ap[0]), a1 = DT::to_f(ap[1]), a2 = DT::to_f(ap[2]), a3 = DT::to_f(ap[3]);
  const int tpp = rev ? tn + 1 : tn - 1;
  const bool has_prev = rev ? tpp < T : tpp >= 0;
  // LSTM: c_{tn-1};  GRU: h_{tn-1} (both fp32 in cseq, c0 = initial state)
  const float sp = has_prev ? d.cseq[(int64_t)tpp * B * H + bu] : (d.c0 ? d.c0[bu] : 0.f);
  struct { S x, y, z, w; } dg;
  float next;
  if constexpr (CELL == 0) {
    const float ig = a0, fg = a1, gg = a2, og = a3;
    const float tc = tanh_(d.cseq[(int64_t)tn * B * H + bu]);
    const float dc = fmaf(dh * og, 1.f - tc * tc, carry);
    dg.x = DT::from_f(dc * gg * ig * (1.f - ig));
    dg.y = DT::from_f(dc * sp * fg * (1.f - fg));
    dg.z = DT::from_f(dc * ig * (1.f - gg * gg));
    dg.w = DT::from_f(dh * tc * og * (1.f - og));
    next = dc * fg;
  } else {
    // h = n + z (h_prev - n), n = tanh(n_x + r n_h):
    // [dr r(1-r) | dz z(1-z) | dpre_n (x side) | dpre_n r (n_h side)]
    const float r = a0, z = a1, n = a2, nh = a3;
    const float dpn = dh * (1.f - z) * (1.f - n * n);
    dg.x = DT::from_f(dpn * nh * r * (1.f - r));
    dg.y = DT::from_f(dh * (sp - n) * z * (1.f - z));
    dg.z = DT::from_f(dpn);
    dg.w = DT::from_f(dpn * r);
    next = dh * z;
  }
  // gate-BLOCKED layout (torch's row order): the next step GEMM pairs it with
  // W_hh^T as stored, and the weight-gradient GEMMs land directly in the
  // parameters' layout (no permutation copies)
  S* dgp = static_cast<S*>(d.dgates) + ((int64_t)tn * B + b) * 4 * H + u;
  if constexpr (COH) {
    // persistent kernel: read by the other workgroups of the batch block
    // within the launch (device-coherent stores, see ps_ld16)
    const __amdgpu_buffer_rsrc_t r = uniform_rsrc(static_cast<S*>(d.dgates) + (int64_t)tn * B * 4 * H);
    const uint32_t o = (uint32_t)(((int64_t)b * 4 * H + u) * sizeof(S));
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, dg.x), r, o, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, dg.y), r, o + H * sizeof(S), 0, 16);
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, dg.z), r, o + 2 * H * sizeof(S), 0, 16);
    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, dg.w), r, o + 3 * H * sizeof(S), 0, 16);
  } else {
    dgp[0] = dg.x; dgp[H] = dg.y; dgp[2 * H] = dg.z; dgp[3 * H] = dg.w;
  }
  d.dc_carry[bu] = next;
}

// 8-float (2 x 16-byte) row accesses
__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), c = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// Cell backward of 8 consecutive units u0 .. u0+7 of row b (u0 % 8 == 0):
// cell_bwd_elem's math with 16-byte accesses, split into a load phase and a
// compute phase so that the epilogue of the backward step kernel puts the
// global loads of several items in flight before the first one is consumed.
template <class DT>
struct CellBwdOps8 {
  float carry[8], sp[8], cur[8];
  V8<DT> av[4];  // 8 units x 4 gates
  V8<DT> dv;
};

template <class DT, int CELL>
__device__ __forceinline__ void cell_bwd_load8(const PdrnnLstmLargeDir& d, int B, int H, int T, bool rev, int tn,
                                               bool cell, int b, int u0, CellBwdOps8<DT>& o) {
  typedef typename DT::S S;
  const int64_t bu = (int64_t)b * H + u0;
  ld8(d.dc_carry + bu, o.carry);
  if (!cell) return;
  if (d.dout) o.dv = ld_v8<DT>(static_cast<const S*>(d.dout) + (int64_t)tn * d.dout_st + (int64_t)b * d.dout_sb + u0);
  else o.dv = V8<DT>{};
  const S* ap = static_cast<const S*>(d.acts) + ((int64_t)tn * B + b) * 4 * H + 4 * u0;
#pragma unroll
  for (int q = 0; q < 4; ++q) o.av[q] = ld_v8<DT>(ap + 8 * q);
  const int tpp = rev ? tn + 1 : tn - 1;
  const bool has_prev = rev ? tpp < T : tpp >= 0;
  if (has_prev) ld8(d.cseq + (int64_t)tpp * B * H + bu, o.sp);
  else if (d.c0) ld8(d.c0 + bu, o.sp);
  else {
#pragma unroll
    for (int k = 0; k < 8; ++k) o.sp[k] = 0.f;
  }
  if constexpr (CELL == 0) ld8(d.cseq + (int64_t)tn * B * H + bu, o.cur);
}

template <class DT, int CELL>
__device__ __forceinline__ void cell_bwd_compute8(const PdrnnLstmLargeDir& d, int B, int H, bool cell, int tn, int b,
                                                  int u0, float (&dh)[8], const CellBwdOps8<DT>& o) {
  typedef typename DT::S S;
  const int64_t bu = (int64_t)b * H + u0;
  float carry[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) carry[k] = o.carry[k];
  if constexpr (CELL == 1) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dh[k] += carry[k];
  }
  if (!cell) {
    if (d.dh0) st8(d.dh0 + bu, dh);
    if (CELL == 0 && d.dc0) st8(d.dc0 + bu, carry);
    return;
  }
  if (d.dout) {
#pragma unroll
    for (int k = 0; k < 8; ++k) dh[k] += o.dv.get(k);
  }
  // unit k: gates 4k .. 4k+3 of the 32 loaded (V8 q holds units 2q, 2q+1)
  auto act = [&](int e) { return o.av[e >> 3].get(e & 7); };
  alignas(16) S g[4][8];
  float next[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float a0 = act(4 * k), a1 = act(4 * k + 1);
    const float a2 = act(4 * k + 2), a3 = act(4 * k + 3);
    if constexpr (CELL == 0) {
      const float tc = tanh_(o.cur[k]);
      const float dc = fmaf(dh[k] * a3, 1.f - tc * tc, carry[k]);
      g[0][k] = DT::from_f(dc * a2 * a0 * (1.f - a0));
      g[1][k] = DT::from_f(dc * o.sp[k] * a1 * (1.f - a1));
      g[2][k] = DT::from_f(dc * a0 * (1.f - a2 * a2));
      g[3][k] = DT::from_f(dh[k] * tc * a3 * (1.f - a3));
      next[k] = dc * a1;
    } else {
      const float dpn = dh[k] * (1.f - a1) * (1.f - a2 * a2);
      g[0][k] = DT::from_f(dpn * a3 * a0 * (1.f - a0));
      g[1][k] = DT::from_f(dh[k] * (o.sp[k] - a2) * a1 * (1.f - a1));
      g[2][k] = DT::from_f(dpn);
      g[3][k] = DT::from_f(dpn * a0);
      next[k] = dh[k] * a1;
    }
  }
  S* dgp = static_cast<S*>(d.dgates) + ((int64_t)tn * B + b) * 4 * H + u0;
#pragma unroll
  for (int q = 0; q < 4; ++q) st_v8<DT>(dgp + q * H, *reinterpret_cast<const V8<DT>*>(g[q]));
  st8(d.dc_carry + bu, next);
}

// ---------------------------------------------------------------------------
// Backward step: dh_{t'} = dgates_t Wp  (t' = the step processed before t in
// forward order) fused with the cell backward of step t':
//   dh = acc + dout_{t'};  dc = dc_carry + dh o (1 - tanh(c)^2)
//   dgates_{t'} = [dc g i(1-i), dc c_prev f(1-f), dc i (1-g^2), dh tanh(c) o(1-o)]
//   dc_carry = dc f
// With cell == 0 (after the first forward step): dh0 = acc, dc0 = dc_carry.
// ---------------------------------------------------------------------------
template <class DT, int BM, int BN, int WM, int WN, int ST, int CELL>
__global__ void __launch_bounds__(WM * WN * 64) lstm_large_bwd_step_kernel(PdrnnLstmLargeStepArgs args) {
  typedef GemmPipe<DT, BM, BN, WM, WN, ST> G;
  typedef typename DT::S S;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  S* const smem = reinterpret_cast<S*>(smem_raw);
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
  G::run(static_cast<const S*>(d.dgates) + (int64_t)t * B * 4 * H, 4 * H, static_cast<const S*>(d.wt), 4 * H, B,
         4 * H, m0, n0, smem, acc);

  // Epilogue through LDS (as in the forward): the dh tile is parked as fp32
  // [BM][BN+4] in the idle staging ring, then each thread runs the cell
  // backward of 8 consecutive units of one row with 16-byte loads / stores
  // (acts, c, carry, dout, and one store per gate block of dgates) instead of
  // per-element 2-byte accesses straight from the MFMA C layout.
  constexpr int LDC = BN + 4;
  static_assert(BM * LDC * 4 <= G::LDS_ELEMS * sizeof(S), "C tile must fit in the staging ring");
  float* cs = reinterpret_cast<float*>(smem_raw);
  {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / WN, wn = wid % WN;
#pragma unroll
    for (int i = 0; i < G::MT; ++i)
#pragma unroll
      for (int j = 0; j < G::NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(wm * G::WTM + i * 16 + (lane >> 4) * 4 + r) * LDC + wn * G::WTN + j * 16 + (lane & 15)] = acc[i][j][r];
  }
  __syncthreads();
  constexpr int C8 = BN / 8;
  // items in batches of IB: every item's global operands of a batch are in
  // flight together (see the forward epilogue)
  constexpr int ITEMS = (BM * C8 + G::NTHREADS - 1) / G::NTHREADS;
  constexpr int IB = ITEMS < 2 ? ITEMS : 2;
#pragma unroll
  for (int i0 = 0; i0 < ITEMS; i0 += IB) {
    CellBwdOps8<DT> ops[IB];
#pragma unroll
    for (int ib = 0; ib < IB; ++ib) {
      const int e = min((int)threadIdx.x + (i0 + ib) * G::NTHREADS, BM * C8 - 1);
      const int row = e / C8, c8 = e - row * C8;
      cell_bwd_load8<DT, CELL>(d, B, H, T, rev, tn, cell, min(m0 + row, B - 1), n0 + c8 * 8, ops[ib]);
    }
#pragma unroll
    for (int ib = 0; ib < IB; ++ib) {
      const int e = threadIdx.x + (i0 + ib) * G::NTHREADS;
      const int row = e / C8, c8 = e - row * C8;
      const int b = m0 + row;
      if (e >= BM * C8 || b >= B) continue;
      float dh[8];
      const float4 z0 = *reinterpret_cast<const float4*>(cs + row * LDC + c8 * 8);
      const float4 z1 = *reinterpret_cast<const float4*>(cs + row * LDC + c8 * 8 + 4);
      dh[0] = z0.x; dh[1] = z0.y; dh[2] = z0.z; dh[3] = z0.w;
      dh[4] = z1.x; dh[5] = z1.y; dh[6] = z1.z; dh[7] = z1.w;
      cell_bwd_compute8<DT, CELL>(d, B, H, cell, tn, b, n0 + c8 * 8, dh, ops[ib]);
    }
  }
}

// Split-K form of the backward step for small batches (few output tiles, long
// K = 4H): blockIdx.z = direction * S + slice; each workgroup writes its fp32
// partial tile to ws[slice][dir][B][H]; the cell kernel sums the S partials
// in fixed order (deterministic) and runs the cell backward.
template <class DT, int BM, int BN, int WM, int WN, int ST>
__global__ void __launch_bounds__(WM * WN * 64) lstm_large_bwd_splitk_kernel(PdrnnLstmLargeStepArgs args) {
  typedef GemmPipe<DT, BM, BN, WM, WN, ST> G;
  typedef typename DT::S Sd;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int S = args.splitk;
  const int dir = blockIdx.z / S, sl = blockIdx.z - dir * S;
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const int B = args.B, H = args.H, T = args.T;
  const bool rev = args.reverse_mask & (1 << dir);
  const int t = rev ? args.step : T - 1 - args.step;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int Ks = 4 * H / S, k0 = sl * Ks;
  f32x4 acc[G::MT][G::NT];
  G::run(static_cast<const Sd*>(d.dgates) + (int64_t)t * B * 4 * H + k0, 4 * H, static_cast<const Sd*>(d.wt) + k0,
         4 * H, B, Ks, m0, n0, reinterpret_cast<Sd*>(smem_raw), acc);
  float* ws = args.ws + ((int64_t)sl * 2 + dir) * B * H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int j = 0; j < G::NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int b = m0 + wm * G::WTM + i * 16 + (lane >> 4) * 4 + r;
        const int u = n0 + wn * G::WTN + j * 16 + (lane & 15);
        if (b < B) ws[(int64_t)b * H + u] = acc[i][j][r];
      }
}

template <class DT, int CELL>
__global__ void lstm_large_bwd_cell_kernel(PdrnnLstmLargeStepArgs args) {
  const int dir = blockIdx.z;
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const int B = args.B, H = args.H, T = args.T, S = args.splitk;
  const bool rev = args.reverse_mask & (1 << dir);
  const int t = rev ? args.step : T - 1 - args.step;
  const int tn = rev ? t + 1 : t - 1;
  const bool cell = rev ? tn < T : tn >= 0;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * H) return;
  float dh = 0.f;
  for (int sl = 0; sl < S; ++sl) dh += args.ws[((int64_t)sl * 2 + dir) * B * H + e];
  const int b = (int)(e / H), u = (int)(e - (int64_t)b * H);
  cell_bwd_elem<DT, CELL>(d, B, H, T, rev, tn, cell, b, u, dh, d.dc_carry[e]);
}

// The same with 8 consecutive units per thread (16-byte loads / stores of
// dh, acts, c, carry, dout and one store per gate block of dgates): the cell
// half of the large-batch backward (ping-pong GEMM + cell), S = 1.
template <class DT, int CELL>
__global__ void __launch_bounds__(256) lstm_large_bwd_cell8_kernel(PdrnnLstmLargeStepArgs args) {
  const int dir = blockIdx.z;
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const int B = args.B, H = args.H, T = args.T;
  const bool rev = args.reverse_mask & (1 << dir);
  const int t = rev ? args.step : T - 1 - args.step;
  const int tn = rev ? t + 1 : t - 1;
  const bool cell = rev ? tn < T : tn >= 0;
  const int64_t e8 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int H8 = H >> 3;
  if (e8 >= (int64_t)B * H8) return;
  const int b = (int)(e8 / H8), u0 = (int)(e8 - (int64_t)b * H8) * 8;
  CellBwdOps8<DT> ops;
  cell_bwd_load8<DT, CELL>(d, B, H, T, rev, tn, cell, b, u0, ops);
  float dh[8];
  ld8(args.ws + (int64_t)dir * B * H + (int64_t)b * H + u0, dh);
  cell_bwd_compute8<DT, CELL>(d, B, H, cell, tn, b, u0, dh, ops);
}

// Cell backward of the LAST forward step (no recurrent dh yet):
// dh = dout_T-1 + dhn, carry = dcn (LSTM) / 0 (GRU).  One thread per (b, u).
template <class DT, int CELL>
__global__ void lstm_large_bwd_first_kernel(PdrnnLstmLargeStepArgs args) {
  const PdrnnLstmLargeDir& d = args.dir[blockIdx.z];
  const int B = args.B, H = args.H, T = args.T;
  const bool rev = args.reverse_mask & (1 << blockIdx.z);
  const int tn = rev ? 0 : T - 1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)B * H) return;
  const int b = (int)(e / H), u = (int)(e - (int64_t)b * H);
  const float carry = (CELL == 0 && d.dcn) ? d.dcn[e] : 0.f;
  cell_bwd_elem<DT, CELL>(d, B, H, T, rev, tn, true, b, u, d.dhn ? d.dhn[e] : 0.f, carry);
}

// Plain NT GEMM on the same core (tests / fallbacks): C[M,N] fp32 = A Bt^T.
template <class DT, int BM, int BN, int WM, int WN, int ST>
__global__ void __launch_bounds__(WM * WN * 64) gemm_nt_kernel(const typename DT::S* A, int64_t lda,
                                                               const typename DT::S* Bt, int64_t ldb, float* C,
                                                               int64_t ldc, int M, int N, int K) {
  typedef GemmPipe<DT, BM, BN, WM, WN, ST> G;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  f32x4 acc[G::MT][G::NT];
  G::run(A, lda, Bt, ldb, M, K, m0, n0, reinterpret_cast<typename DT::S*>(smem_raw), acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / WN, wn = wid % WN;
#pragma unroll
  for (int i = 0; i < G::MT; ++i)
#pragma unroll
    for (int j = 0; j < G::NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * G::WTM + i * 16 + (lane >> 4) * 4 + r;
        const int col = n0 + wn * G::WTN + j * 16 + (lane & 15);
        if (row < M && col < N) C[(int64_t)row * ldc + col] = acc[i][j][r];
      }
}

// ---------------------------------------------------------------------------
// Large-batch form of the forward step kernel on the ping-pong GEMM main loop
// (pdrnn/gemm_pp.h: 256 x 256 tile, 8 waves, LDS-DMA quarter ring, counted
// vmcnt, staggered wave groups) -- the same cell epilogues as above, run in
// two passes over the tile's row halves because a 256 x 256 fp32 C tile does
// not fit in LDS: the wave group owning rows h*128 .. h*128+127 parks them as
// fp32 [128][256+4], then every thread runs the cell math of 8 consecutive
// columns of a row.
constexpr int kPpLdc = 256 + 4;
constexpr size_t kPpLds = (size_t)128 * kPpLdc * 4;  // >= the main loop's 128 KiB

template <class DT>
__device__ __forceinline__ void pp_park(float* cs, const pp::g_f32x4 (&acc)[8][4], int half) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  if (wr == half) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          cs[(i * 16 + (lane >> 4) * 4 + r) * kPpLdc + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
  }
}

template <class DT, int CELL>
__global__ void __launch_bounds__(512) lstm_large_fwd_step_pp_kernel(PdrnnLstmLargeStepArgs args) {
  typedef typename DT::S S;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const PdrnnLstmLargeDir& d = args.dir[blockIdx.z];
  const int B = args.B, H = args.H;
  const int t = args.reverse_mask & (1 << blockIdx.z) ? args.T - 1 - args.step : args.step;
  const int tp = args.reverse_mask & (1 << blockIdx.z) ? t + 1 : t - 1;
  const bool first = args.step == 0;
  const int m0 = blockIdx.y * 256, n0 = blockIdx.x * 256;
  const S* hA = first ? static_cast<const S*>(d.h0) : static_cast<const S*>(d.hseq) + (int64_t)tp * d.hseq_st;
  const int64_t lda = first ? H : d.hseq_sb;
  pp::g_f32x4 acc[8][4];
  if (first && d.h0 == nullptr) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = pp::g_f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
    const uint16_t* a16 = reinterpret_cast<const uint16_t*>(hA);
    const uint16_t* w16 = static_cast<const uint16_t*>(d.w);
    pp::mainloop<DT, false, false, 3, false>(a16, lda, w16, H, a16, lda, w16, H, B, 4 * H, H / 64, 0, H / 64, m0, n0,
                                      reinterpret_cast<uint16_t*>(smem_raw), acc);
  }
  float* cs = reinterpret_cast<float*>(smem_raw);
  const int tid = threadIdx.x;
  const S* xp = static_cast<const S*>(d.xp) + (int64_t)t * d.xp_st;
  const float* cprev = first ? d.c0 : d.cseq + (int64_t)tp * B * H;
  float* cout = d.cseq + (int64_t)t * B * H;
  S* hout = static_cast<S*>(d.hseq) + (int64_t)t * d.hseq_st;
  S* acts = static_cast<S*>(d.acts) + (int64_t)t * B * 4 * H;
  // items in batches of IB (the accumulators stay live through both passes:
  // a batch's loads in flight together within the remaining registers)
  constexpr int C8 = 32, ITEMS = 128 * C8 / 512, IB = 4;
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    pp_park<DT>(cs, acc, half);
    __syncthreads();
#pragma unroll
  for (int i0 = 0; i0 < ITEMS; i0 += IB) {
    V8<DT> xv[IB];
    float2 cpv[IB];
    float4 za[IB], zb[IB];
#pragma unroll
    for (int it = 0; it < IB; ++it) {
      const int e = tid + (i0 + it) * 512;
      const int row = e / C8, c8 = e - row * C8;
      const int b = min(m0 + half * 128 + row, B - 1);
      const int col = n0 + c8 * 8;
      xv[it] = ld_v8<DT>(xp + (int64_t)b * d.xp_sb + col);
      cpv[it] = cprev ? *reinterpret_cast<const float2*>(cprev + (int64_t)b * H + (col >> 2)) : make_float2(0.f, 0.f);
      za[it] = *reinterpret_cast<const float4*>(cs + row * kPpLdc + c8 * 8);
      zb[it] = *reinterpret_cast<const float4*>(cs + row * kPpLdc + c8 * 8 + 4);
    }
#pragma unroll
    for (int it = 0; it < IB; ++it) {
      const int e = tid + (i0 + it) * 512;
      const int row = e / C8, c8 = e - row * C8;
      const int b = m0 + half * 128 + row;
      if (b >= B) continue;
      const int col = n0 + c8 * 8;
      const float z[8] = {za[it].x, za[it].y, za[it].z, za[it].w, zb[it].x, zb[it].y, zb[it].z, zb[it].w};
      float g[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float zz = z[k] + xv[it].get(k);
        if constexpr (CELL == 0) g[k] = (k & 3) == 2 ? tanh_(zz) : sigm(zz);
        else g[k] = (k & 3) < 2 ? sigm(zz) : zz;
      }
      const int u = col >> 2;
      const float2 cp = cpv[it];
      float s0, s1, h0v, h1v;
      if constexpr (CELL == 0) {
        s0 = fmaf(g[1], cp.x, g[0] * g[2]);
        s1 = fmaf(g[5], cp.y, g[4] * g[6]);
        h0v = g[3] * tanh_(s0);
        h1v = g[7] * tanh_(s1);
      } else {
        g[2] = tanh_(fmaf(g[0], g[3], g[2]));
        g[6] = tanh_(fmaf(g[4], g[7], g[6]));
        s0 = h0v = fmaf(g[1], cp.x - g[2], g[2]);
        s1 = h1v = fmaf(g[5], cp.y - g[6], g[6]);
      }
      V8<DT> av;
#pragma unroll
      for (int k = 0; k < 8; ++k) av.set(k, g[k]);
      st_v8<DT>(acts + (int64_t)b * 4 * H + col, av);
      *reinterpret_cast<float2*>(cout + (int64_t)b * H + u) = make_float2(s0, s1);
      const uint32_t hv = (uint32_t)DT::from_f(h0v) | ((uint32_t)DT::from_f(h1v) << 16);
      *reinterpret_cast<uint32_t*>(hout + (int64_t)b * d.hseq_sb + u) = hv;
    }
  }
    __syncthreads();
  }
}

// Backward step as two launches at large batch: the ping-pong GEMM dh_t =
// dgates_t W_hh with a plain fp32 epilogue into ws[dir][B][H] (no cell
// epilogue registers live beside the accumulators), then
// lstm_large_bwd_cell_kernel (S = 1).  The fused GemmPipe kernel's epilogue
// saves the dh round trip, but its 256x128 tiles run the GEMM slower.
template <class DT>
__global__ void __launch_bounds__(512) lstm_large_bwd_gemm_pp_kernel(PdrnnLstmLargeStepArgs args) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int dir = blockIdx.z;
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const int B = args.B, H = args.H, T = args.T;
  const bool rev = args.reverse_mask & (1 << dir);
  const int t = rev ? args.step : T - 1 - args.step;
  const int m0 = blockIdx.y * 256, n0 = blockIdx.x * 256;
  pp::g_f32x4 acc[8][4];
  const uint16_t* g16 = static_cast<const uint16_t*>(d.dgates) + (int64_t)t * B * 4 * H;
  const uint16_t* w16 = static_cast<const uint16_t*>(d.wt);
  pp::mainloop<DT, false, false, 3, false>(g16, 4 * H, w16, 4 * H, g16, 4 * H, w16, 4 * H, B, H, 4 * H / 64, 0,
                                           4 * H / 64, m0, n0, reinterpret_cast<uint16_t*>(smem_raw), acc);
  float* ws = args.ws + (int64_t)dir * B * H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wr = wid >> 2, wc = wid & 3;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = m0 + wr * 128 + i * 16 + (lane >> 4) * 4 + r;
      if (b >= B) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) ws[(int64_t)b * H + n0 + wc * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
    }
}

// the ping-pong forward step: 16-bit storage, 4H a multiple of 256, >= one
// workgroup per CU (bi-LSTM B 4096, H 4096, fp16: 1165 -> 930 us per step).
// The same fused form for the backward step measured 2353 us (its two-pass
// cell epilogue kept too many registers live beside the accumulators and the
// fp16 build spilled inside the main loop; profiles/r3_pp_step/) and was
// replaced by the GEMM + cell pair below.  PDRNN_TUNE large_pp=0 opts out,
// =2 takes it at any legal shape (tests).
inline bool use_pp_step(int B, int N, int ndir, int dsize, bool backward) {
  const int env = pdrnn_tune_int("large_pp", 1);
  if (!env || backward || dsize != 2 || N % 256) return false;
  if (env == 2) return true;
  return B >= 128 && (int64_t)(N / 256) * ((B + 255) / 256) * ndir >= 256;
}

template <class DT, int CELL>
hipError_t launch_step_pp(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, hipStream_t st) {
  const int N = backward ? a->H : 4 * a->H;
  dim3 grid(N / 256, (a->B + 255) / 256, ndir);
  if (backward) return hipErrorInvalidValue;
  hipLaunchKernelGGL((lstm_large_fwd_step_pp_kernel<DT, CELL>), grid, dim3(512), kPpLds, st, *a);
  return hipGetLastError();
}

template <class DT, int CELL, int BM, int BN, int WM, int WN, int ST>
hipError_t launch_step(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, hipStream_t st) {
  typedef GemmPipe<DT, BM, BN, WM, WN, ST> G;
  const int N = backward ? a->H : 4 * a->H;
  if (N % BN) return hipErrorInvalidValue;
  dim3 grid(N / BN, (a->B + BM - 1) / BM, ndir);
  const size_t lds = sizeof(typename DT::S) * G::LDS_ELEMS;
  if (backward)
    hipLaunchKernelGGL((lstm_large_bwd_step_kernel<DT, BM, BN, WM, WN, ST, CELL>), grid, dim3(G::NTHREADS), lds, st, *a);
  else
    hipLaunchKernelGGL((lstm_large_fwd_step_kernel<DT, BM, BN, WM, WN, ST, CELL>), grid, dim3(G::NTHREADS), lds, st, *a);
  return hipGetLastError();
}

// Tile choice: the largest tile that still gives >= 256 workgroups (one per
// CU) and does not waste more than half of its rows on a small batch.
// Fallback when no tile reaches one workgroup per CU: the 32x32 tile (most
// workgroups; the recurrent step is latency-bound there).
inline int pick_tile(int M, int N, int ndir) {
  const int bm[4] = {32, 64, 128, 256}, bn[4] = {64, 64, 128, 128};
  for (int c = 3; c >= 0; --c) {
    if (N % bn[c]) continue;
    if (c > 0 && M <= bm[c] / 2) continue;
    const int64_t blocks = (int64_t)(N / bn[c]) * ((M + bm[c] - 1) / bm[c]) * ndir;
    if (blocks >= 256) return c;
  }
  return 4;
}

template <class DT, int CELL>
hipError_t dispatch_step(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, int tile, hipStream_t st) {
  const int N = backward ? a->H : 4 * a->H;
  if constexpr (sizeof(typename DT::S) == 2) {
    if (backward && a->bwd_pp && a->ws && a->splitk == 1 && a->H % 256 == 0) {
      dim3 grid(a->H / 256, (a->B + 255) / 256, ndir);
      hipLaunchKernelGGL((lstm_large_bwd_gemm_pp_kernel<DT>), grid, dim3(512), 131072, st, *a);
      PDRNN_HIP_CHECK(hipGetLastError());
      const int64_t n8 = (int64_t)a->B * a->H / 8;
      hipLaunchKernelGGL((lstm_large_bwd_cell8_kernel<DT, CELL>), dim3((unsigned)((n8 + 255) / 256), 1, ndir),
                         dim3(256), 0, st, *a);
      return hipGetLastError();
    }
  }
  if (backward && a->splitk > 1 && a->ws) {
    // S K-slices (32x32 tiles for small batches, 128x128 once the batch fills
    // them), then the fixed-order sum + cell backward
    if ((4 * a->H) % (64 * a->splitk)) return hipErrorInvalidValue;
    if (a->splitk_big && N % 128 == 0) {
      typedef GemmPipe<DT, 128, 128, 2, 2, 3> G;
      dim3 grid(N / 128, (a->B + 127) / 128, ndir * a->splitk);
      hipLaunchKernelGGL((lstm_large_bwd_splitk_kernel<DT, 128, 128, 2, 2, 3>), grid, dim3(G::NTHREADS),
                         sizeof(typename DT::S) * G::LDS_ELEMS, st, *a);
    } else {
      typedef GemmPipe<DT, 32, 32, 2, 2, 4> G;
      if (N % 32) return hipErrorInvalidValue;
      dim3 grid(N / 32, (a->B + 31) / 32, ndir * a->splitk);
      hipLaunchKernelGGL((lstm_large_bwd_splitk_kernel<DT, 32, 32, 2, 2, 4>), grid, dim3(G::NTHREADS),
                         sizeof(typename DT::S) * G::LDS_ELEMS, st, *a);
    }
    PDRNN_HIP_CHECK(hipGetLastError());
    const int64_t n = (int64_t)a->B * a->H;
    hipLaunchKernelGGL((lstm_large_bwd_cell_kernel<DT, CELL>), dim3((unsigned)((n + 255) / 256), 1, ndir), dim3(256), 0, st,
                       *a);
    return hipGetLastError();
  }
  if constexpr (sizeof(typename DT::S) == 2) {
    if (tile < 0 && use_pp_step(a->B, N, ndir, 2, backward)) return launch_step_pp<DT, CELL>(a, ndir, backward, st);
  }
  if (tile < 0 || tile > 4) tile = pick_tile(a->B, N, ndir);
  switch (tile) {
#define TILE_CASE(ID, BM_, BN_, WM_, WN_, ST_) \
  case ID: return launch_step<DT, CELL, BM_, BN_, WM_, WN_, ST_>(a, ndir, backward, st);
    TILE_CFGS_X(TILE_CASE)
#undef TILE_CASE
    default: return hipErrorInvalidValue;
  }
}

// Tile shapes reachable only through the plain GEMM entry (tile-shape
// experiments for the large-batch step GEMMs; ids >= 10).
#define GEMM_ONLY_CFGS_X(X) \
  X(10, 256, 256, 2, 4, 2)      \
  X(11, 128, 128, 2, 2, 4)      \
  X(12, 128, 256, 2, 4, 3)      \
  X(13, 128, 128, 2, 2, 2)

template <class DT>
hipError_t gemm_nt_dispatch(const void* Av, int64_t lda, const void* Btv, int64_t ldb, float* C, int64_t ldc,
                            int M, int N, int K, int tile, hipStream_t st) {
  const typename DT::S* A = static_cast<const typename DT::S*>(Av);
  const typename DT::S* Bt = static_cast<const typename DT::S*>(Btv);
  if (tile < 0 || (tile > 4 && tile < 10) || tile > 13) tile = pick_tile(M, N, 1);
  switch (tile) {
#define TILE_CASE(ID, BM_, BN_, WM_, WN_, ST_)                                                      \
  case ID: {                                                                                        \
    typedef GemmPipe<DT, BM_, BN_, WM_, WN_, ST_> G;                                                 \
    if (N % BN_) return hipErrorInvalidValue;                                                        \
    dim3 grid(N / BN_, (M + BM_ - 1) / BM_);                                                         \
    hipLaunchKernelGGL((gemm_nt_kernel<DT, BM_, BN_, WM_, WN_, ST_>), grid, dim3(G::NTHREADS),       \
                       sizeof(typename DT::S) * G::LDS_ELEMS, st, A, lda, Bt, ldb, C, ldc, M, N, K); \
    return hipGetLastError();                                                                        \
  }
    TILE_CFGS_X(TILE_CASE)
    GEMM_ONLY_CFGS_X(TILE_CASE)
#undef TILE_CASE
    default: return hipErrorInvalidValue;
  }
}


// ---------------------------------------------------------------------------
// Persistent recurrence (one launch for all T steps of a layer).
//
// The per-step kernels above re-stream W_hh (8 MB at H = 1024 bf16) from
// L2 / MALL every timestep and pay a launch per step; at small batch (char-LM
// B = 128) that is what a step costs, not the MFMA work.  Here each workgroup
// keeps its slice of W_hh in REGISTERS for the whole sequence -- 8 waves x 32
// KiB of MFMA B fragments -- and the grid synchronises per timestep through a
// per-(direction, batch-block) arrival counter instead of kernel boundaries.
//
//   * workgroup = 512 threads (8 waves), owns NU = 32 hidden units x 16*MT
//     batch rows; the K dimension of the step GEMM is split over the 8 waves
//     (forward K = H, backward K = 4H), partial tiles are summed through LDS;
//   * forward: gates[16 MT x 128] = h_{t-1} W_slice^T, then the cell of the
//     block's 16 MT x 32 (row, unit) pairs, one per thread (c stays fp32);
//   * backward: dh[16 MT x 32] = dgates_t W_hh[:, units], then the cell
//     backward (cell_bwd_elem above) of the same pairs;
//   * grid sync: h_t / dgates_t are written and read with device-coherent
//     (SC1) buffer accesses; every thread drains its stores (vmcnt 0), the
//     workgroup barriers, and one thread bumps the arrival counter of its
//     batch block (relaxed agent-scope atomic); before the next step one
//     thread spins on that counter until all NCB column blocks of the batch
//     block have arrived.  No L2 write-back / invalidate per step (an
//     acquire/release pair costs a whole-L2 maintenance operation on every
//     spin and arrival: measured 2x slower than the per-step kernels).  Only the 32 workgroups that share rows wait for
//     each other; the spin is bounded (~2 s of wall clock; *err is set) so a
//     fault can never hang the GPU;
//   * blockIdx -> (column block, batch block) puts the batch block in the
//     low bits: workgroups are dispatched round-robin over the 8 XCDs, so the
//     workgroups of one XCD read the same A rows out of their shared L2.
// The grid must be co-resident (checked against the kernel's occupancy,
// persist_go below); the host falls back to the per-step kernels otherwise.
// ---------------------------------------------------------------------------
constexpr int PS_NU = 32;       // hidden units per workgroup
constexpr int PS_WAVES = 8;
constexpr int PS_THREADS = PS_WAVES * 64;

struct PersistSync {
  int* cnt;   // [ndir][NMB] arrival counters, zero at launch
  int* err;   // set to 1 when a spin timed out (this launch: releases every waiter)
  int* sticky;  // also set on a timeout; never cleared (the host checks it)
  int mode;   // diagnostics (wrong results): bit 0 no waits, bit 1 no step GEMM, bit 2 no store drain,
              // bit 4 flag the launch as timed out (tests of the host's recovery)
  long long* stamps;  // mode bit 3: workgroup 0 records s_memtime at 8 points of steps 0..63
  uint32_t* xchg;     // tagged forward exchange (16-bit types): [nslots][ndir][B][H] dwords, zero
                      // at launch, or null for the arrival-counter protocol (see ps_poll_h)
  int nslots;         // exchange ring length (>= 2)
};
#define PS_STAMP(k)                                                                          \
  if ((sync.mode & 8) && blockIdx.x == 0 && threadIdx.x == 0 && s < 64)                      \
    sync.stamps[s * 8 + (k)] = (long long)__builtin_amdgcn_s_memtime();

__device__ __forceinline__ void ps_arrive(int* c, int mode = 0) {
  // every wave's device-coherent stores are complete before the count moves
  if (!(mode & 4)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void ps_wait(int* c, int target, int* err, int* sticky) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      // once any workgroup has timed out nobody waits any more (the launch
      // drains in ~2 s instead of 2 s per remaining step)
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
      if (wall_clock64() - t0 > 200000000ull) {  // 100 MHz constant clock: 2 s
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (sticky) __hip_atomic_store(sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// Device-coherent (SC1 = agent scope) 16-byte loads / 2-byte stores for the
// data exchanged between workgroups inside the launch (h_t, dgates_t): they
// bypass the per-CU L1 and the XCD-private L2 copies, so no cache
// write-back / invalidate is needed around the arrival counter.
constexpr int PS_SC1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ps_rsrc(const void* p) { return uniform_rsrc(p); }
__device__ __forceinline__ uint4 ps_ld16(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off_bytes, 0, PS_SC1);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void ps_st2(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes, uint16_t v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, r, off_bytes, 0, PS_SC1);
}
__device__ __forceinline__ void ps_st(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes, uint16_t v) { ps_st2(r, off_bytes, v); }
__device__ __forceinline__ void ps_st(__amdgpu_buffer_rsrc_t r, uint32_t off_bytes, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off_bytes, 0, PS_SC1);
}
// the 4 gate values of one (row, unit) pair in storage type S (8 or 16 bytes)
template <class S>
using Quad = typename std::conditional<sizeof(S) == 2, uint2, uint4>::type;
template <class DT>
__device__ __forceinline__ Quad<typename DT::S> pack4(float a, float b, float c, float d) {
  Quad<typename DT::S> q;
  typename DT::S* v = reinterpret_cast<typename DT::S*>(&q);
  v[0] = DT::from_f(a); v[1] = DT::from_f(b); v[2] = DT::from_f(c); v[3] = DT::from_f(d);
  return q;
}

// workgroup -> (direction, column block, batch block)
__device__ __forceinline__ void ps_coords(int NCB, int NMB, int& dir, int& cb, int& mb) {
  const int per_dir = NCB * NMB;
  dir = blockIdx.x / per_dir;
  const int l = blockIdx.x - dir * per_dir;
  mb = l % NMB;
  cb = l / NMB;
}

// Tagged forward exchange (16-bit types; PersistSync::xchg non-null).  The
// arrival-counter protocol costs a step ~43% of its cycles on the char-LM
// shape (wait 34% + store drain and count 9%,
// profiles/r6/persist_fwd_step_cycles.md): every producer drains its h_t
// stores before counting, and the reader loads h_{t-1} only after it has seen
// the count.  Here h_t travels as one dword per value -- bf16/f16 bits in the
// low half, the step tag s + 1 in the high half -- in a ring of nslots >= 2
// exchange slots [nslots][ndir][B][H], zero at launch.  A reader of step s
// polls its A-fragment chunks of slot (s - 1) % nslots until every dword
// carries tag s, so the data IS the flag: no drain, no counter, and the loads
// that succeed are the operands.  Reusing a slot is safe: a producer writes
// slot s % nslots again at step s + nslots >= s + 2 only after it has read
// h_{s+1} of every column block of its batch block, i.e. after all of them
// finished step s + 1, whose reads of the slot precede their cell phase.
// Tags are unique within a launch (T < 65535, checked by the host).  The spin
// is bounded like ps_wait (~2 s, *err releases every other poller).
// Measured slower than the counters (PDRNN_TUNE persist_tagx, default off;
// profiles/r6/persist_fwd_step_cycles.md).
template <int MT, int KS>
__device__ __forceinline__ void ps_poll_h(uint4 (&af)[MT][KS], const PersistSync& sync, const uint32_t* slot,
                                          uint32_t want, int mb, int fr, int fq, int k0, int B, int H) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t rx = ps_rsrc(slot);
  const uint64_t t0 = wall_clock64();
  // probe: re-reading the whole operand every round (8 KiB a wave, 16 MiB a
  // grid round on the char-LM shape) congests the device-coherent path and
  // was 30% slower than the counters; one dword a lane watches the last unit
  // of producer block (fq mod KS) of its row, and the full load is issued
  // when every probe shows the tag (re-polled in full if any chunk lags)
  bool probing = true;
  for (;;) {
    bool ok = true;
    if (probing) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int row = min(mb * 16 * MT + mt * 16 + fr, B - 1);
        const uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(
            rx, (uint32_t)((row * H + k0 + (fq % KS) * PS_NU + PS_NU - 1) * 4), 0, PS_SC1);
        ok = ok && (v >> 16) == want;
      }
      if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
        probing = false;
        continue;
      }
    } else {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int row = min(mb * 16 * MT + mt * 16 + fr, B - 1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const uint32_t off = (uint32_t)((row * H + k0 + ks * 32 + fq * 8) * 4);
          const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, PS_SC1);
          const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rx, off + 16, 0, PS_SC1);
          ok = ok && (lo.x >> 16) == want && (lo.y >> 16) == want && (lo.z >> 16) == want && (lo.w >> 16) == want &&
               (hi.x >> 16) == want && (hi.y >> 16) == want && (hi.z >> 16) == want && (hi.w >> 16) == want;
          af[mt][ks] = make_uint4((lo.x & 0xffffu) | (lo.y << 16), (lo.z & 0xffffu) | (lo.w << 16),
                                  (hi.x & 0xffffu) | (hi.y << 16), (hi.z & 0xffffu) | (hi.w << 16));
        }
      }
      if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
    }
    __builtin_amdgcn_s_sleep(1);
    const int e = __builtin_amdgcn_readfirstlane(__hip_atomic_load(sync.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (e != 0) break;
    if (wall_clock64() - t0 > 200000000ull) {  // 100 MHz constant clock: 2 s
      if ((threadIdx.x & 63) == 0) {
        __hip_atomic_store(sync.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (sync.sticky) __hip_atomic_store(sync.sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      break;
    }
  }
}

// Per-step epilogue state lives in registers: the cell state c (forward) and
// the carry (backward) never leave the thread that owns the (row, unit) pair;
// the operands of the next step that do not depend on other workgroups (xp;
// acts / c / dout) are loaded right after the arrival, so their latency hides
// behind the wait; only the exchanged stores (h_t / dgates_t) precede the
// arrival -- the saved activations and c_t are stored after it.
template <class DT, int CELL, int KS, int MT, bool TAGX>
__global__ void __launch_bounds__(PS_THREADS) lstm_large_persist_fwd_kernel(PdrnnLstmLargeStepArgs args,
                                                                            PersistSync sync) {
  typedef typename DT::S S;
  constexpr int CT = 4 * PS_NU / 16;  // 8 column tiles of 16 gate columns
  constexpr int LDR = 4 * PS_NU + 4;  // partial-tile row stride (floats)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* red = reinterpret_cast<float*>(smem_raw);  // [wave][MT][16][LDR]
  const int B = args.B, H = args.H, T = args.T;
  if ((sync.mode & 16) && blockIdx.x == 0 && threadIdx.x == 0) {  // test hook: this launch "timed out"
    __hip_atomic_store(sync.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sync.sticky) __hip_atomic_store(sync.sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int NCB = H / PS_NU, NMB = (B + 16 * MT - 1) / (16 * MT);
  int dir, cb, mb;
  ps_coords(NCB, NMB, dir, cb, mb);
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const bool rev = args.reverse_mask & (1 << dir);
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = cb * 4 * PS_NU;        // first gate column (gate-interleaved)
  const int k0 = wid * (H / PS_WAVES);  // this wave's K range
  int* cnt = sync.cnt + dir * NMB + mb;
  // exchange slot of step s: s mod the ring length, this direction (TAGX)
  const int ndirs = gridDim.x / (NCB * NMB);
  auto xslot = [&](int s, int dr) { return sync.xchg + ((int64_t)((s % sync.nslots) * ndirs + dr)) * B * H; };

  // W_hh slice as MFMA B fragments, resident for the whole sequence
  uint4 wf[KS][CT];
  {
    const S* w = static_cast<const S*>(d.w);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < CT; ++j)
        wf[ks][j] = *reinterpret_cast<const uint4*>(w + (int64_t)(n0 + j * 16 + fr) * H + k0 + ks * 4 * DT::EPC + fq * DT::EPC);
  }
  // this thread's (row, unit) pairs of the cell epilogue: 16 rows x 32 units
  const int eu = threadIdx.x & (PS_NU - 1), er = threadIdx.x / PS_NU;
  const int u = cb * PS_NU + eu;
  int brow[MT];
  float cst[MT];   // cell state (LSTM c / GRU h), fp32, register-resident
  Quad<S> xpn[MT];  // next step's 4 gate pre-activations
  // step range of this launch (a later range resumes from c_{t0 - 1} in cseq
  // and h_{t0 - 1} in hseq)
  const int S0 = args.s1 > 0 ? args.s0 : 0, S1 = args.s1 > 0 ? args.s1 : T;
  const int t_first = rev ? T - 1 - S0 : S0;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    brow[mt] = min(mb * 16 * MT + mt * 16 + er, B - 1);
    const int tp0 = rev ? t_first + 1 : t_first - 1;
    cst[mt] = S0 > 0 ? d.cseq[(int64_t)tp0 * B * H + (int64_t)brow[mt] * H + u]
                     : (d.c0 ? d.c0[(int64_t)brow[mt] * H + u] : 0.f);
  }
  auto load_xp = [&](int t) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      xpn[mt] = *reinterpret_cast<const Quad<S>*>(static_cast<const S*>(d.xp) + (int64_t)t * d.xp_st +
                                                (int64_t)brow[mt] * d.xp_sb + 4 * u);
  };
  load_xp(t_first);

  for (int s = S0; s < S1; ++s) {
    const int t = rev ? T - 1 - s : s;
    const int tp = rev ? t + 1 : t - 1;
    const bool first = s == 0;
    Quad<S> xcur[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) xcur[mt] = xpn[mt];
    PS_STAMP(0)
    if constexpr (!TAGX) {
      if (s > S0 && !(sync.mode & 1)) ps_wait(cnt, s * NCB, sync.err, sync.sticky);
    }
    PS_STAMP(1)

    f32x4 acc[MT][CT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < CT; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const S* hA = first ? static_cast<const S*>(d.h0) : static_cast<const S*>(d.hseq) + (int64_t)tp * d.hseq_st;
    if (hA != nullptr && !(sync.mode & 2)) {
      const int64_t lda = first ? H : d.hseq_sb;
      const __amdgpu_buffer_rsrc_t ra = ps_rsrc(hA);
      uint4 af[MT][KS];
      if (TAGX && s > S0) {
        ps_poll_h<MT, KS>(af, sync, xslot(s - 1, dir), (uint32_t)s, mb, fr, fq, k0, B, H);
      } else {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int row = min(mb * 16 * MT + mt * 16 + fr, B - 1);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks)
            af[mt][ks] = ps_ld16(ra, (uint32_t)((row * lda + k0 + ks * 4 * DT::EPC + fq * DT::EPC) * sizeof(S)));
        }
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int j = 0; j < CT; ++j) acc[mt][j] = DT::mfma(af[mt][ks], wf[ks][j], acc[mt][j]);
    }
    PS_STAMP(2)
    // partial tiles -> LDS
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          red[((wid * MT + mt) * 16 + fq * 4 + i) * LDR + j * 16 + fr] = acc[mt][j][i];
    __syncthreads();
    PS_STAMP(3)
    float gs[MT][4];
    const __amdgpu_buffer_rsrc_t rh = ps_rsrc(static_cast<S*>(d.hseq) + (int64_t)t * d.hseq_st);
    const __amdgpu_buffer_rsrc_t rxw = ps_rsrc(TAGX ? static_cast<const void*>(xslot(s, dir)) : static_cast<const void*>(sync.cnt));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const S* xv = reinterpret_cast<const S*>(&xcur[mt]);
      float z[4] = {DT::to_f(xv[0]), DT::to_f(xv[1]), DT::to_f(xv[2]), DT::to_f(xv[3])};
#pragma unroll
      for (int w = 0; w < PS_WAVES; ++w) {
        const float4 p = *reinterpret_cast<const float4*>(red + ((w * MT + mt) * 16 + er) * LDR + 4 * eu);
        z[0] += p.x; z[1] += p.y; z[2] += p.z; z[3] += p.w;
      }
      float* g = gs[mt];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if constexpr (CELL == 0) g[k] = k == 2 ? tanh_(z[k]) : sigm(z[k]);
        else g[k] = k < 2 ? sigm(z[k]) : z[k];
      }
      float hv;
      if constexpr (CELL == 0) {
        cst[mt] = fmaf(g[1], cst[mt], g[0] * g[2]);
        hv = g[3] * tanh_(cst[mt]);
      } else {
        g[2] = tanh_(fmaf(g[0], g[3], g[2]));
        cst[mt] = hv = fmaf(g[1], cst[mt] - g[2], g[2]);
      }
      const int b = mb * 16 * MT + mt * 16 + er;
      if constexpr (TAGX) {
        // h_t to hseq (read after the launch: a plain store) and, tagged with
        // s + 1, to this step's exchange slot (read by the next step's polls)
        if (b < B) {
          const uint16_t hb = DT::from_f(hv);
          static_cast<S*>(d.hseq)[(int64_t)t * d.hseq_st + (int64_t)b * d.hseq_sb + u] = hb;
          __builtin_amdgcn_raw_buffer_store_b32(((uint32_t)(s + 1) << 16) | hb, rxw, (uint32_t)((b * H + u) * 4), 0,
                                                PS_SC1);
        }
      } else {
        if (b < B) ps_st(rh, (uint32_t)((b * d.hseq_sb + u) * sizeof(S)), DT::from_f(hv));
      }
    }
    PS_STAMP(4)
    if (TAGX || s + 1 == T) __syncthreads();  // (LDS reuse only: nobody counts arrivals)
    else ps_arrive(cnt, sync.mode);
    PS_STAMP(5)
    if (s + 1 < S1) load_xp(rev ? t - 1 : t + 1);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int b = mb * 16 * MT + mt * 16 + er;
      if (b >= B) continue;
      const int64_t bu = (int64_t)b * H + u;
      const float* g = gs[mt];
      *reinterpret_cast<Quad<S>*>(static_cast<S*>(d.acts) + (int64_t)t * B * 4 * H + 4 * bu) =
          pack4<DT>(g[0], g[1], g[2], g[3]);
      d.cseq[(int64_t)t * B * H + bu] = cst[mt];
    }
    PS_STAMP(6)
  }
}

// Backward: step s consumes dgates_t (t = T-1-s forward order) and runs the
// cell backward of tn (the step before t), or emits dh0 / dc0 after the
// first forward step.  dgates_{T-1} and the initial carry come from
// lstm_large_bwd_first_kernel.  Same cell math as cell_bwd_elem.
template <class DT, int CELL, int KS, int MT>
__global__ void __launch_bounds__(PS_THREADS) lstm_large_persist_bwd_kernel(PdrnnLstmLargeStepArgs args,
                                                                            PersistSync sync) {
  typedef typename DT::S S;
  constexpr int CT = PS_NU / 16;  // 2 column tiles of 16 units
  constexpr int LDR = PS_NU + 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* red = reinterpret_cast<float*>(smem_raw);  // [wave][MT][16][LDR]
  const int B = args.B, H = args.H, T = args.T;
  if ((sync.mode & 16) && blockIdx.x == 0 && threadIdx.x == 0) {  // test hook: this launch "timed out"
    __hip_atomic_store(sync.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sync.sticky) __hip_atomic_store(sync.sticky, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int NCB = H / PS_NU, NMB = (B + 16 * MT - 1) / (16 * MT);
  int dir, cb, mb;
  ps_coords(NCB, NMB, dir, cb, mb);
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const bool rev = args.reverse_mask & (1 << dir);
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = cb * PS_NU;
  const int k0 = wid * (4 * H / PS_WAVES);
  int* cnt = sync.cnt + dir * NMB + mb;

  uint4 wf[KS][CT];
  {
    const S* wt = static_cast<const S*>(d.wt);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < CT; ++j)
        wf[ks][j] = *reinterpret_cast<const uint4*>(wt + (int64_t)(n0 + j * 16 + fr) * 4 * H + k0 + ks * 4 * DT::EPC +
                                                    fq * DT::EPC);
  }
  const int eu = threadIdx.x & (PS_NU - 1), er = threadIdx.x / PS_NU;
  const int u = cb * PS_NU + eu;
  int brow[MT];
  float carry[MT];
  // next cell-backward operands: dout, the 4 saved gates, c_tn, c_{tn-1}
  float nd[MT], ncur[MT], nsp[MT];
  Quad<S> nact[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    brow[mt] = min(mb * 16 * MT + mt * 16 + er, B - 1);
    carry[mt] = d.dc_carry[(int64_t)brow[mt] * H + u];
  }
  auto load_ops = [&](int tn) {
    const int tpp = rev ? tn + 1 : tn - 1;
    const bool has_prev = rev ? tpp < T : tpp >= 0;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int64_t bu = (int64_t)brow[mt] * H + u;
      nd[mt] = d.dout ? DT::to_f(static_cast<const S*>(d.dout)[(int64_t)tn * d.dout_st +
                                                                (int64_t)brow[mt] * d.dout_sb + u])
                      : 0.f;
      nact[mt] = *reinterpret_cast<const Quad<S>*>(static_cast<const S*>(d.acts) + ((int64_t)tn * B) * 4 * H + 4 * bu);
      ncur[mt] = CELL == 0 ? d.cseq[(int64_t)tn * B * H + bu] : 0.f;
      nsp[mt] = has_prev ? d.cseq[(int64_t)tpp * B * H + bu] : (d.c0 ? d.c0[bu] : 0.f);
    }
  };
  // step range of this launch: a later range resumes from dgates_t (written
  // by the earlier range's last step) and the carry it left in dc_carry
  const int S0 = args.s1 > 0 ? args.s0 : 0, S1 = args.s1 > 0 ? args.s1 : T;
  {
    const int t0 = rev ? S0 : T - 1 - S0, tn0 = rev ? t0 + 1 : t0 - 1;
    if (rev ? tn0 < T : tn0 >= 0) load_ops(tn0);
  }

  for (int s = S0; s < S1; ++s) {
    const int t = rev ? s : T - 1 - s;
    const int tn = rev ? t + 1 : t - 1;
    const bool cell = rev ? tn < T : tn >= 0;
    float od[MT], ocur[MT], osp[MT];
    Quad<S> oact[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) { od[mt] = nd[mt]; ocur[mt] = ncur[mt]; osp[mt] = nsp[mt]; oact[mt] = nact[mt]; }
    // dgates_t of the whole batch block: written by every column block (the
    // first one by the separate first-step kernel, ordered by the launch)
    if (s > S0 && !(sync.mode & 1)) ps_wait(cnt, s * NCB, sync.err, sync.sticky);
    f32x4 acc[MT][CT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < CT; ++j) acc[mt][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const __amdgpu_buffer_rsrc_t ra = ps_rsrc(static_cast<const S*>(d.dgates) + (int64_t)t * B * 4 * H);
    // K loop in 4 chunks: a chunk's loads are all in flight before its MFMAs
    constexpr int KC = KS >= 4 ? KS / 4 : 1;
    if (!(sync.mode & 2)) {
#pragma unroll
      for (int kc = 0; kc < KS; kc += KC) {
        uint4 af[MT][KC];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          const int row = min(mb * 16 * MT + mt * 16 + fr, B - 1);
#pragma unroll
          for (int k = 0; k < KC; ++k)
            af[mt][k] = ps_ld16(ra, (uint32_t)((row * 4 * H + k0 + (kc + k) * 4 * DT::EPC + fq * DT::EPC) * sizeof(S)));
        }
#pragma unroll
        for (int k = 0; k < KC; ++k)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int j = 0; j < CT; ++j) acc[mt][j] = DT::mfma(af[mt][k], wf[kc + k][j], acc[mt][j]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          red[((wid * MT + mt) * 16 + fq * 4 + i) * LDR + j * 16 + fr] = acc[mt][j][i];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rg = ps_rsrc(static_cast<S*>(d.dgates) + (int64_t)(cell ? tn : 0) * B * 4 * H);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float dh = 0.f;
#pragma unroll
      for (int w = 0; w < PS_WAVES; ++w) dh += red[((w * MT + mt) * 16 + er) * LDR + eu];
      const int b = mb * 16 * MT + mt * 16 + er;
      if (b >= B) continue;
      const int64_t bu = (int64_t)b * H + u;
      if constexpr (CELL == 1) dh += carry[mt];
      if (!cell) {
        if (d.dh0) d.dh0[bu] = dh;
        if (CELL == 0 && d.dc0) d.dc0[bu] = carry[mt];
        continue;
      }
      dh += od[mt];
      const S* av = reinterpret_cast<const S*>(&oact[mt]);
      const float a0 = DT::to_f(av[0]), a1 = DT::to_f(av[1]), a2 = DT::to_f(av[2]), a3 = DT::to_f(av[3]);
      float g0, g1, g2, g3;
      if constexpr (CELL == 0) {
        const float tc = tanh_(ocur[mt]);
        const float dc = fmaf(dh * a3, 1.f - tc * tc, carry[mt]);
        g0 = dc * a2 * a0 * (1.f - a0);
        g1 = dc * osp[mt] * a1 * (1.f - a1);
        g2 = dc * a0 * (1.f - a2 * a2);
        g3 = dh * tc * a3 * (1.f - a3);
        carry[mt] = dc * a1;
      } else {
        const float dpn = dh * (1.f - a1) * (1.f - a2 * a2);
        g0 = dpn * a3 * a0 * (1.f - a0);
        g1 = dh * (osp[mt] - a2) * a1 * (1.f - a1);
        g2 = dpn;
        g3 = dpn * a0;
        carry[mt] = dh * a1;
      }
      // gate-blocked dgates_tn (read by the batch block's other workgroups
      // at the next step: device-coherent stores)
      const uint32_t o = (uint32_t)(((int64_t)b * 4 * H + u) * sizeof(S));
      ps_st(rg, o, DT::from_f(g0));
      ps_st(rg, o + H * sizeof(S), DT::from_f(g1));
      ps_st(rg, o + 2 * H * sizeof(S), DT::from_f(g2));
      ps_st(rg, o + 3 * H * sizeof(S), DT::from_f(g3));
    }
    if (s + 1 < T) {
      ps_arrive(cnt, sync.mode);
      const int tn2 = rev ? tn + 1 : tn - 1;  // cell-backward step of s + 1
      if (s + 1 < S1 && (rev ? tn2 < T : tn2 >= 0)) load_ops(tn2);
    }
  }
  if (S1 < T) {  // the next range's carry
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int b = mb * 16 * MT + mt * 16 + er;
      if (b < B) d.dc_carry[(int64_t)b * H + u] = carry[mt];
    }
  }
}

// Every workgroup of a batch block must be resident at once (they wait for
// each other every step).  The grid is checked against the kernel's occupancy
// on an idle device and launched as an ordinary dispatch: cooperative
// launches gave the same placement, and under rocprofv3 their processes
// segfaulted at exit (char-LM and fp32 --hidden 128 runs, round 4).  Residency
// lost to other work at run time (RCCL kernels beside it) ends in the bounded
// spin and the host's fallback, as before.
template <class K>
hipError_t persist_go(K kernel, dim3 grid, size_t lds, hipStream_t st, const PdrnnLstmLargeStepArgs& args,
                      const PersistSync& sy, int* occ_cache) {
  if (*occ_cache < 0) {
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, reinterpret_cast<const void*>(kernel), PS_THREADS, lds) !=
        hipSuccess)
      occ = 0;
    *occ_cache = occ;
  }
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return hipErrorInvalidDevice;
  if ((int64_t)*occ_cache * cus < (int64_t)grid.x) return hipErrorCooperativeLaunchTooLarge;
  hipLaunchKernelGGL(kernel, grid, dim3(PS_THREADS), lds, st, args, sy);
  return hipGetLastError();
}

template <class DT, int CELL, int MT, int KSF, int KSB>
hipError_t persist_launch(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, PersistSync sy, hipStream_t st) {
  // the K split: 8 waves x KS chunk steps x 4 lane groups x EPC elements
  if (a->H != PS_WAVES * KSF * 4 * DT::EPC || 4 * a->H != PS_WAVES * KSB * 4 * DT::EPC) return hipErrorInvalidValue;
  const int NCB = a->H / PS_NU, NMB = (a->B + 16 * MT - 1) / (16 * MT);
  const dim3 grid(NCB * NMB * ndir);
  static int occ_bwd = -1, occ_fwd = -1;
  if (backward) {
    const size_t lds = (size_t)PS_WAVES * MT * 16 * (PS_NU + 4) * 4;
    return persist_go(lstm_large_persist_bwd_kernel<DT, CELL, KSB, MT>, grid, lds, st, *a, sy, &occ_bwd);
  }
  if constexpr (DT::EPC != 8) {
    // fp32: no persistent forward (8.3 vs 7.1 us a step for the per-step
    // kernels at H = 128, profiles/r4/h2/h2_persist_f32_cell*.json; the
    // planner never asks for it, bindings.cpp large_persist_plan)
    (void)occ_fwd;
    return hipErrorInvalidValue;
  } else {
    const size_t lds = (size_t)PS_WAVES * MT * 16 * (4 * PS_NU + 4) * 4;
    static int occ_fwd_tag = -1;
    if (sy.xchg != nullptr)
      return persist_go(lstm_large_persist_fwd_kernel<DT, CELL, KSF, MT, true>, grid, lds, st, *a, sy, &occ_fwd_tag);
    return persist_go(lstm_large_persist_fwd_kernel<DT, CELL, KSF, MT, false>, grid, lds, st, *a, sy, &occ_fwd);
  }
}

// 16-bit storage: H = 1024 (forward K-steps per wave H/256 = 4, backward
// 4H/256 = 16: 32 fragments of 16 B per wave either way = 128 VGPRs).
// fp32 storage: H = 128 (1 / 4 chunk steps of 16 k: 8 fragments) or H = 256
// (2 / 8) -- the fp32 models' hidden sizes, whose per-step kernels were
// latency-bound at 7-9 us a step.
template <class DT, int CELL>
hipError_t persist_dispatch(const PdrnnLstmLargeStepArgs* a, int ndir, bool backward, int mt, PersistSync sy,
                            hipStream_t st) {
  if constexpr (DT::EPC == 8) {
    return mt == 1 ? persist_launch<DT, CELL, 1, 4, 16>(a, ndir, backward, sy, st)
                   : persist_launch<DT, CELL, 2, 4, 16>(a, ndir, backward, sy, st);
  } else {
    if (a->H == 128)
      return mt == 1 ? persist_launch<DT, CELL, 1, 1, 4>(a, ndir, backward, sy, st)
                     : persist_launch<DT, CELL, 2, 1, 4>(a, ndir, backward, sy, st);
    return mt == 1 ? persist_launch<DT, CELL, 1, 2, 8>(a, ndir, backward, sy, st)
                   : persist_launch<DT, CELL, 2, 2, 8>(a, ndir, backward, sy, st);
  }
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_lstm_large_supported(int H) { return H >= 64 && H % 64 == 0; }

// K-slices for the backward step GEMM (1 = no split) and their tile
// (*big: 128x128 instead of 32x32).  Large batches: 128x128 tiles with the
// fewest slices reaching one workgroup per CU (bi-LSTM h4096 B256: 2 slices,
// -6 % step time); small batches: 32x32 tiles, slices while < 512 workgroups
// and each slice keeps >= 8 k-tiles (char-LM h1024 B128: 4 slices).
int pdrnn_lstm_large_bwd_pp(int B, int H, int ndir, int dtype) {
  const int env = pdrnn_tune_int("large_pp_bwd", 1);  // (0 off, 2 at any legal shape)
  if (!env || (dtype != 0 && dtype != 1) || H % 256) return 0;
  if (env == 2) return 1;
  return B >= 128 && (int64_t)(H / 256) * ((B + 255) / 256) * ndir >= 256;
}

int pdrnn_lstm_large_bwd_splitk(int B, int H, int ndir, int* big) {
  *big = 0;
  const int kt = 4 * H / 64;
  if (B >= 128 && H % 128 == 0) {
    const int64_t t128 = (int64_t)(H / 128) * ((B + 127) / 128) * ndir;
    if (t128 >= 256) return 1;
    for (int s = 2; s <= 4; s *= 2)
      if (t128 * s >= 256 && kt / s >= 8) { *big = 1; return s; }
  }
  const int64_t tiles = (int64_t)(H / 32) * ((B + 31) / 32) * ndir;
  if (tiles >= 256) return 1;
  int s = 1;
  while (tiles * s * 2 <= 512 && kt / (s * 2) >= 8) s *= 2;
  return s;
}

hipError_t pdrnn_lstm_large_step(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, int dtype, int tile,
                                 hipStream_t stream) {
  if (!pdrnn_lstm_large_supported(a->H) || ndir < 1 || ndir > 2) return hipErrorInvalidValue;
  if (a->cell != 0 && a->cell != 1) return hipErrorInvalidValue;
  const bool bw = backward != 0;
  if (dtype == 0)
    return a->cell ? pdrnn::dispatch_step<pdrnn::BF16, 1>(a, ndir, bw, tile, stream)
                   : pdrnn::dispatch_step<pdrnn::BF16, 0>(a, ndir, bw, tile, stream);
  if (dtype == 2)
    return a->cell ? pdrnn::dispatch_step<pdrnn::F32, 1>(a, ndir, bw, tile, stream)
                   : pdrnn::dispatch_step<pdrnn::F32, 0>(a, ndir, bw, tile, stream);
  return a->cell ? pdrnn::dispatch_step<pdrnn::F16, 1>(a, ndir, bw, tile, stream)
                 : pdrnn::dispatch_step<pdrnn::F16, 0>(a, ndir, bw, tile, stream);
}

// Persistent recurrence (see above): batch rows per workgroup / 16 (1 or 2)
// for a grid that fits one workgroup per CU, or 0 when the shape is not
// covered (16-bit storage with H = 1024, fp32 with H = 128 / 256; grid <= cus).
int pdrnn_lstm_large_persist_mt(int B, int H, int ndir, int dtype, int cus) {
  if (dtype < 0 || dtype > 2) return 0;
  if ((dtype == 2 ? (H != 128 && H != 256) : H != 1024) || ndir < 1 || ndir > 2) return 0;
  for (int mt = 1; mt <= 2; ++mt) {
    const int64_t grid = (int64_t)(H / pdrnn::PS_NU) * ((B + 16 * mt - 1) / (16 * mt)) * ndir;
    if (grid <= cus) return mt;
  }
  return 0;
}

hipError_t pdrnn_lstm_large_persist(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, int dtype, int mt,
                                    int* counters, int* err, int* sticky, int mode, uint32_t* xchg,
                                    int nslots, hipStream_t stream) {
  if ((mt != 1 && mt != 2) || dtype < 0 || dtype > 2) return hipErrorInvalidValue;
  if (xchg != nullptr && (backward || dtype == 2 || a->T >= 65535 || nslots < 2 || (reinterpret_cast<uintptr_t>(xchg) & 15)))
    return hipErrorInvalidValue;
  if (dtype == 2 ? (a->H != 128 && a->H != 256) : a->H != 1024) return hipErrorInvalidValue;
  if (a->cell != 0 && a->cell != 1) return hipErrorInvalidValue;
  const pdrnn::PersistSync sy{counters, err, sticky, mode,
                              reinterpret_cast<long long*>((reinterpret_cast<uintptr_t>(err + 1) + 7) & ~(uintptr_t)7),
                              xchg, nslots};
  const bool bw = backward != 0;
  if (dtype == 0)
    return a->cell ? pdrnn::persist_dispatch<pdrnn::BF16, 1>(a, ndir, bw, mt, sy, stream)
                   : pdrnn::persist_dispatch<pdrnn::BF16, 0>(a, ndir, bw, mt, sy, stream);
  if (dtype == 2)
    return a->cell ? pdrnn::persist_dispatch<pdrnn::F32, 1>(a, ndir, bw, mt, sy, stream)
                   : pdrnn::persist_dispatch<pdrnn::F32, 0>(a, ndir, bw, mt, sy, stream);
  return a->cell ? pdrnn::persist_dispatch<pdrnn::F16, 1>(a, ndir, bw, mt, sy, stream)
                 : pdrnn::persist_dispatch<pdrnn::F16, 0>(a, ndir, bw, mt, sy, stream);
}

hipError_t pdrnn_lstm_large_bwd_first(const PdrnnLstmLargeStepArgs* a, int ndir, int dtype, hipStream_t stream) {
  const int64_t n = (int64_t)a->B * a->H;
  dim3 grid((unsigned)((n + 255) / 256), 1, ndir);
  if (a->cell != 0 && a->cell != 1) return hipErrorInvalidValue;
  if (dtype == 0) {
    if (a->cell) hipLaunchKernelGGL((pdrnn::lstm_large_bwd_first_kernel<pdrnn::BF16, 1>), grid, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL((pdrnn::lstm_large_bwd_first_kernel<pdrnn::BF16, 0>), grid, dim3(256), 0, stream, *a);
  } else if (dtype == 2) {
    if (a->cell) hipLaunchKernelGGL((pdrnn::lstm_large_bwd_first_kernel<pdrnn::F32, 1>), grid, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL((pdrnn::lstm_large_bwd_first_kernel<pdrnn::F32, 0>), grid, dim3(256), 0, stream, *a);
  } else {
    if (a->cell) hipLaunchKernelGGL((pdrnn::lstm_large_bwd_first_kernel<pdrnn::F16, 1>), grid, dim3(256), 0, stream, *a);
    else hipLaunchKernelGGL((pdrnn::lstm_large_bwd_first_kernel<pdrnn::F16, 0>), grid, dim3(256), 0, stream, *a);
  }
  return hipGetLastError();
}

hipError_t pdrnn_gemm_nt(const void* A, int64_t lda, const void* Bt, int64_t ldb, float* C, int64_t ldc,
                         int M, int N, int K, int dtype, int tile, hipStream_t stream) {
  if (K % 64 || N % 32) return hipErrorInvalidValue;
  if (dtype == 0) return pdrnn::gemm_nt_dispatch<pdrnn::BF16>(A, lda, Bt, ldb, C, ldc, M, N, K, tile, stream);
  if (dtype == 2) return pdrnn::gemm_nt_dispatch<pdrnn::F32>(A, lda, Bt, ldb, C, ldc, M, N, K, tile, stream);
  return pdrnn::gemm_nt_dispatch<pdrnn::F16>(A, lda, Bt, ldb, C, ldc, M, N, K, tile, stream);
}

}  // extern "C"
