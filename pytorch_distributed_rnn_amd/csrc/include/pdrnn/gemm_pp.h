// Ping-pong MFMA GEMM main loop for gfx950 (shared by kernels/gemm.hip and
// the large-H recurrent step kernels of kernels/lstm_large.hip).
//
// 256 x 256 output tile per 512-thread workgroup, BK = 64,
// v_mfma_f32_16x16x32_{bf16,f16}, 8 waves as 2 (M) x 4 (N), each wave 128 x 64
// outputs = acc[8][4].  Operand staging, phase schedule and barrier stagger:
// see the header comment of kernels/gemm.hip.  A caller provides the tile
// origin (m0, n0), the K-tile range and 128 KiB of dynamic LDS, and runs its
// own epilogue on acc (wave wr = wid >> 2 owns tile rows wr*128 + i*16 + ...,
// wave wc = wid & 3 owns columns wc*64 + j*16 + ...; C layout of the 16x16
// MFMA: row 4 (lane >> 4) + r, column lane & 15).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pdrnn {
namespace pp {

typedef __bf16 g_bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 g_f16x8 __attribute__((ext_vector_type(8)));
typedef float g_f32x4 __attribute__((ext_vector_type(4)));
typedef short g_s16x4 __attribute__((ext_vector_type(4)));

constexpr int TM = 256, TN = 256, TK = 64;
constexpr int QELEMS = 8192;  // elements (16-bit) per quarter image = 16 KiB
constexpr int LDS_BYTES = 8 * QELEMS * 2;

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void bar() { __builtin_amdgcn_s_barrier(); }
// lgkmcnt(0) through the builtin (vmcnt / expcnt fields at their maxima): the
// compiler's waitcnt pass sees it, so it does not add its own lgkmcnt(0) in
// front of the next MFMA for fragment reads this wait already retired
__device__ __forceinline__ void wait_lds() { __builtin_amdgcn_s_waitcnt(0xC07F); }

// k-major image swizzle (chunk units, even: chunk pairs stay together)
__device__ __forceinline__ int kswz(int k) { return (((k & 3) | (((k >> 3) & 1) << 2)) << 1); }

// local row of an A quarter -> tile row; local column of a B quarter -> tile column
__device__ __forceinline__ int a_tile_row(int mq, int ml) { return (ml >> 6) * 128 + mq * 64 + (ml & 63); }
__device__ __forceinline__ int b_tile_col(int nq, int nl) { return (nl >> 5) * 64 + nq * 32 + (nl & 31); }

// One operand (A or B) of the GEMM: the per-lane DMA sources of its two
// quarters (2 global_load_lds per wave per quarter).
template <bool KM>
struct Operand {
  const uint16_t* src[2][2];  // [quarter][instr]
  int64_t kstep;              // elements to advance per K-tile

  // base: operand pointer, ld: leading dimension (elements), lim: rows (KM: columns) in range,
  // r0: first tile row/col of this workgroup, isA: A (m-quarters) or B (n-quarters)
  __device__ __forceinline__ void init(const uint16_t* base, int64_t ld, int lim, int r0, bool isA, int wid,
                                       int lane) {
    kstep = KM ? (int64_t)TK * ld : (int64_t)TK;
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int g = wid * 2 + i;  // 1 KiB DMA group of the quarter
        if constexpr (!KM) {
          const int row = g * 8 + (lane >> 3), slot = lane & 7;
          const int c = slot ^ (row & 7);
          const int tr = isA ? a_tile_row(q, row) : b_tile_col(q, row);
          const int gr = min(r0 + tr, lim - 1);
          src[q][i] = base + (int64_t)gr * ld + c * 8;
        } else {
          const int kr = g * 4 + (lane >> 4), slot = lane & 15;
          const int c = slot ^ kswz(kr);
          const int tc = isA ? a_tile_row(q, c * 8) : b_tile_col(q, c * 8);
          const int gc = min(r0 + tc, lim - 8);
          src[q][i] = base + (int64_t)kr * ld + gc;
        }
      }
  }
  __device__ __forceinline__ void skip(int tiles) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 2; ++i) src[q][i] += tiles * kstep;
  }
  // issue quarter q of the next K-tile into LDS quarter image `dst`
  __device__ __forceinline__ void issue(int q, uint16_t* dst, int wid) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src[q][i],
                                       (__attribute__((address_space(3))) void*)(dst + (wid * 2 + i) * 512), 16, 0,
                                       0);
      src[q][i] += kstep;
    }
  }
};

// Fragment reads.  NT image (K contiguous): 16 rows x 8 k per lane group.
__device__ __forceinline__ uint4 frag_row(const uint16_t* img, int row, int ks, int lane) {
  const int r = row + (lane & 15);
  const int c = ks * 4 + (lane >> 4);
  return *reinterpret_cast<const uint4*>(img + r * 64 + ((c ^ (r & 7)) << 3));
}
// k-major image: two transposing reads (k = 8g + {0..3}, 8g + {4..7}) of the
// 16 columns col .. col+15.
__device__ __forceinline__ uint4 frag_tr(const uint16_t* img, int col, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int cc = col + 4 * p;
  const int ch = cc >> 3, within = cc & 7;
  const int k0 = ks * 32 + 8 * g + q, k1 = k0 + 4;
  const g_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) g_s16x4*)(img + k0 * 128 + ((ch ^ kswz(k0)) << 3) + within));
  const g_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) g_s16x4*)(img + k1 * 128 + ((ch ^ kswz(k1)) << 3) + within));
  uint4 r;
  r.x = (uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16);
  r.y = (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16);
  r.z = (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16);
  r.w = (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16);
  return r;
}
template <bool KM>
__device__ __forceinline__ uint4 frag(const uint16_t* img, int base, int ks, int lane) {
  if constexpr (KM) return frag_tr(img, base, ks, lane);
  else return frag_row(img, base, ks, lane);
}

// The operand pointers arrive as __restrict__ arguments of this inlined body:
// hipcc then tags each LDS DMA with the scope of its global source and proves
// the ds_reads independent of it.  Without that it puts an `s_waitcnt
// vmcnt(0)` before every ds_read that may alias an outstanding LDS DMA (all of
// them), which drains the DMA pipeline every phase.  The counted waits and
// barriers below are what orders the accesses.
//
// K-tiles [ktb, ktb + KT) of the concatenation (segment 1: K-tiles [0, KT1) of
// A / B; segment 2: A2 / B2).  V: schedule variant bits (tuning A/B): 1 = B_n1
// refill in Q3 instead of Q2, 2 = issue a phase's DMA after its fragment reads.
// SEG2 = false: one K segment (the segment-switch code and the per-lane
// values it re-derives are compiled out -- fewer registers live in the loop).
// Returns with all LDS DMA retired and a full workgroup barrier passed: the
// caller may reuse the 128 KiB of LDS.
template <class DT, bool AKM, bool BKM, int V, bool SEG2 = true>
__device__ __forceinline__ void mainloop(const uint16_t* __restrict__ Ab, int64_t lda,
                                         const uint16_t* __restrict__ Bb, int64_t ldb,
                                         const uint16_t* __restrict__ A2b, int64_t lda2,
                                         const uint16_t* __restrict__ B2b, int64_t ldb2, int M, int N, int KT1,
                                         int ktb, int KT, int m0, int n0, uint16_t* smem, g_f32x4 (&acc)[8][4]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  Operand<AKM> opA;
  Operand<BKM> opB;
  if (ktb < KT1) {
    opA.init(Ab, lda, M, m0, true, wid, lane);
    opB.init(Bb, ldb, N, n0, false, wid, lane);
    opA.skip(ktb);
    opB.skip(ktb);
  } else {
    opA.init(A2b, lda2, M, m0, true, wid, lane);
    opB.init(B2b, ldb2, N, n0, false, wid, lane);
    opA.skip(ktb - KT1);
    opB.skip(ktb - KT1);
  }

  // quarter images: slot s, quarter kind (0 A_m0, 1 A_m1, 2 B_n0, 3 B_n1)
  auto img = [&](int s, int kind) -> uint16_t* { return smem + (s * 4 + kind) * QELEMS; };
  // tile t's quarter (kind) issue; switches to the second K segment at KT1
  auto issueA = [&](int t, int mq) {
    if (SEG2 && t + ktb == KT1 && t > 0) {
      // second K segment (dW: h0 pairing, dX: second direction)
      opA.init(A2b, lda2, M, m0, true, wid, lane);
    }
    opA.issue(mq, img(t & 1, mq), wid);
  };
  auto issueB = [&](int t, int nq) {
    if (SEG2 && t + ktb == KT1 && t > 0) opB.init(B2b, ldb2, N, n0, false, wid, lane);
    opB.issue(nq, img(t & 1, 2 + nq), wid);
  };
  // per-tile issue order: B_n0, A_m0, B_n1, A_m1 (the vmcnt counts below assume it);
  // a segment switch happens on the first quarter of a kind issued for tile KT1 --
  // B_n0 / A_m0 for B and A respectively, so init() runs once per operand.
  auto issue_all = [&](int t) {
    issueB(t, 0);
    issueA(t, 0);
    opB.issue(1, img(t & 1, 3), wid);
    opA.issue(1, img(t & 1, 1), wid);
  };

#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = g_f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-tiles 0 and 1 in flight, retire B_n0(0), A_m0(0)
  issue_all(0);
  if (KT > 1) {
    issue_all(1);
    wait_vm<12>();
  } else {
    wait_vm<4>();
  }
  bar();
  if (wr == 1) bar();  // group 1 runs one barrier behind

  uint4 fa[4][2], fb0[2][2], fb1[2][2];
  const int arow = wr * 64, bcol = wc * 32;

  auto mfma_quad = [&](int mq, int nq, const uint4 (&fb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
          acc[mq * 4 + mi][nq * 2 + nj] = DT::mfma(fa[mi][ks], fb[nj][ks], acc[mq * 4 + mi][nq * 2 + nj]);
    __builtin_amdgcn_s_setprio(0);
  };

  for (int t = 0; t < KT; ++t) {
    const int s = t & 1;
    const bool more1 = t + 1 < KT, more2 = t + 2 < KT;
    // ---- Q0 (0,0): retire B_n1(t); read A_m0, B_n0
    if (more1) wait_vm<10>();
    else wait_vm<2>();
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[mi][ks] = frag<AKM>(img(s, 0), arow + mi * 16, ks, lane);
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb0[nj][ks] = frag<BKM>(img(s, 2), bcol + nj * 16, ks, lane);
    wait_lds();
    bar();
    mfma_quad(0, 0, fb0);
    bar();
    // ---- Q1 (0,1): retire A_m1(t); refill B_n0 with t+2; read B_n1
    if (more1) wait_vm<8>();
    else wait_vm<0>();
    if (!(V & 2) && more2) issueB(t + 2, 0);
#pragma unroll
    for (int nj = 0; nj < 2; ++nj)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fb1[nj][ks] = frag<BKM>(img(s, 3), bcol + nj * 16, ks, lane);
    if ((V & 2) && more2) issueB(t + 2, 0);
    wait_lds();
    bar();
    mfma_quad(0, 1, fb1);
    bar();
    // ---- Q2 (1,1): refill A_m0 (and B_n1) with t+2; read A_m1
    if (!(V & 2) && more2) {
      issueA(t + 2, 0);
      if (!(V & 1)) opB.issue(1, img(s, 3), wid);
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) fa[mi][ks] = frag<AKM>(img(s, 1), arow + mi * 16, ks, lane);
    if ((V & 2) && more2) {
      issueA(t + 2, 0);
      if (!(V & 1)) opB.issue(1, img(s, 3), wid);
    }
    wait_lds();
    bar();
    mfma_quad(1, 1, fb1);
    bar();
    // ---- Q3 (1,0): retire B_n0(t+1), A_m0(t+1); refill A_m1 (and B_n1) with t+2
    if (more2) {
      if constexpr (V & 1) wait_vm<8>();
      else wait_vm<10>();
    } else if (more1) {
      wait_vm<4>();
    }
    if (more2) {
      if constexpr (V & 1) opB.issue(1, img(s, 3), wid);
      opA.issue(1, img(s, 1), wid);
    }
    bar();
    mfma_quad(1, 0, fb0);
    bar();
  }
  if (wr == 0) bar();  // even out the barrier count
  wait_vm<0>();
  wait_lds();
  __syncthreads();

}

}  // namespace pp
}  // namespace pdrnn
