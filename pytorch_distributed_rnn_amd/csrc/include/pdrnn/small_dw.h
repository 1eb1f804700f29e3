// Weight-gradient reduction body of the fused small-H LSTM/GRU stack on the
// fp32 matrix cores (v_mfma_f32_16x16x4_f32), shared by the stand-alone dW
// kernel (kernels/lstm_small_dw.hip: one workgroup per K chunk) and the BPTT
// kernel whose workgroups form the dW of their own sequences right after
// their recurrence (kernels/lstm_small.hip, lstm_small_bwd_dw_kernel).
// Mapping and pipeline: see the comment at the top of lstm_small_dw.hip.
#pragma once

#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// (b,t) rows per pipeline stage (4 per MFMA K step).  32-row stages (twice
// the MFMA work per barrier) measured no faster at H = 32: 67-69 vs 68 us at
// B = 1440, 16.5 vs 14.1 at B = 180 (profiles/r5/sw/sw13_dw32.log) -- the
// kernel sits near both its HBM (~280 MB a step) and its MFMA floor at ~50 %
// of each (profiles/r5/pmc/dw_b1440.md).  Twice the chunks (two workgroups
// per CU, two MFMA waves per SIMD) is slower too: 72.8 vs 68.7 us at B = 1440,
// 40.8 vs 37.3 at 720 (profiles/r5/sw/dw_chunks_256_vs_512.log).
template <int H>
constexpr int dw_rows() { return 16; }
static_assert(dw_rows<32>() <= PDRNN_DW_PAD_ROWS, "dW stages read past the padding");

template <int H>
constexpr int dw_stages() { return H >= 64 ? 3 : 4; }
// LDS floats per stage: gate gradients [RW][4H] | h_{t-1} rows [RW][H] | input rows [RW][H]
template <int H>
constexpr int dw_stage_floats() { return dw_rows<H>() * 6 * H; }

template <int N>
__device__ __forceinline__ void dw_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt takes an immediate: a wave-uniform count in [0, 16] by a switch
__device__ __forceinline__ void dw_wait_vm_n(int n) {
  switch (n) {
    case 0: dw_wait_vm<0>(); break;
    case 1: dw_wait_vm<1>(); break;
    case 2: dw_wait_vm<2>(); break;
    case 3: dw_wait_vm<3>(); break;
    case 4: dw_wait_vm<4>(); break;
    case 5: dw_wait_vm<5>(); break;
    case 6: dw_wait_vm<6>(); break;
    case 7: dw_wait_vm<7>(); break;
    case 8: dw_wait_vm<8>(); break;
    case 9: dw_wait_vm<9>(); break;
    case 10: dw_wait_vm<10>(); break;
    case 11: dw_wait_vm<11>(); break;
    case 12: dw_wait_vm<12>(); break;
    case 13: dw_wait_vm<13>(); break;
    case 14: dw_wait_vm<14>(); break;
    case 15: dw_wait_vm<15>(); break;
    default: dw_wait_vm<16>(); break;
  }
}

// DMA jobs of one stage (one dwordx4 wave instruction each, 64 lanes x 16 B):
//   A   : H/4 jobs, 64/H gate-gradient rows of 16H bytes each
//   Bh  : H/16 jobs, the stage's 16 h_{t-1} rows = 16 contiguous h rows
//   Bin : layer >= 1: H/16 jobs (h of the layer below);
//         layer 0: ceil(16 IP / 256) jobs of the contiguous x rows (IP = I
//         rounded up to 4)
// Every wave issues exactly JPW = ceil(jobs / waves) of them per stage (the
// surplus re-issues job 0: same bytes to the same place), so that one vmcnt
// count retires a stage for every wave.  A job's per-lane source pointer and
// LDS destination are fixed for the whole loop; each stage only adds the
// stage stride.  Reads past the last row land in the buffers' padding (see
// PdrnnLstmSmallDwArgs) and are masked at use: no clamps in the loop.
// Stages [st0, st1) of layer l (rows k < k_end), partial sums to slab row
// `slab_row`.  MASKA: gate-gradient rows at or past k_end are zeroed at use (a
// caller whose last stage may read rows that hold no finite values yet).
template <int H, bool X0, bool MASKA = false>
__device__ __forceinline__ void lstm_small_dw_range(const PdrnnLstmSmallDwArgs& a, int l, int st0, int st1,
                                                   int64_t k_end, int64_t slab_row) {
  constexpr int G = H / 16;   // float4 A fragments per K step (64 gates each)
  constexpr int MT = 4 * G;   // virtual 16-row m-tiles
  constexpr int R = dw_stages<H>();
  constexpr int SF = dw_stage_floats<H>();
  constexpr int RW = dw_rows<H>();
  constexpr int OFF_BH = RW * 4 * H, OFF_BIN = RW * 5 * H;
  constexpr int JA = RW * H / 64, JH = RW * H / 256;
  constexpr int MAXJ = 8;  // jobs per wave and stage, upper bound (launcher-checked)
  // ONE dynamic LDS array (a second __shared__ object makes hipcc drain vmcnt
  // before ds_reads): the R stage slots
  extern __shared__ __attribute__((aligned(16))) float lds[];

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int i = lane & 15, kk = lane >> 4;
  const int B = a.B, T = a.T;
  const int Iin = X0 ? a.I : H;
  const int IP = X0 ? a.xg_ld : H;
  const int NI = (Iin + 15) / 16;
  const int NW = NI + H / 16;
  const int64_t BT = (int64_t)B * T;
  const int nst = st1 - st0;
  const int JX = X0 ? (RW * IP + 255) / 256 : JH;
  const int J = JA + JH + JX;
  const int JPW = (J + NW - 1) / NW;  // wave-uniform; (R - 2) * JPW <= 16, JPW <= MAXJ
  const bool active = w < NW && nst > 0;  // idle waves of the narrower layer only join barriers

  // this wave's jobs: source pointer at stage st0 (per lane), byte stride per
  // stage, LDS offset in a slot (floats)
  const char* jsrc[MAXJ];
  int64_t jstride[MAXJ];
  int jdst[MAXJ];
  {
    const int64_t k0 = (int64_t)st0 * RW;
    const float* dg_l = a.dg + (int64_t)l * BT * a.dg_st;
    const float* h_own = a.hseq + (int64_t)l * BT * H;
    const float* h_below = a.hseq + (int64_t)(l > 0 ? l - 1 : 0) * BT * H;
#pragma unroll
    for (int q = 0; q < MAXJ; ++q) {
      int j = w + q * NW;
      j = j < J ? j : 0;
      const float* src;
      int64_t stride;
      int dst;
      if (j < JA) {  // gate-gradient rows
        constexpr int RPJ = 64 / H;
        src = dg_l + (k0 + j * RPJ + lane / H) * a.dg_st + (lane % H) * 4;
        stride = RW * a.dg_st;
        dst = j * 256;
      } else if (j < JA + JH) {  // h_{t-1}: h rows k0-1 .. k0+RW-2 (row -1 is front padding)
        const int jj = j - JA;
        src = h_own + (k0 - 1) * H + (jj * 64 + lane) * 4;
        stride = RW * H;
        dst = OFF_BH + jj * 256;
      } else if (!X0) {  // layer below's h rows k0 .. k0+RW-1
        const int jj = j - JA - JH;
        src = h_below + k0 * H + (jj * 64 + lane) * 4;
        stride = RW * H;
        dst = OFF_BIN + jj * 256;
      } else {  // x rows k0 .. k0+RW-1 (row stride IP)
        const int jj = j - JA - JH;
        src = a.xg + k0 * IP + (jj * 64 + lane) * 4;
        stride = RW * IP;
        dst = OFF_BIN + jj * 256;
      }
      jsrc[q] = reinterpret_cast<const char*>(src);
      jstride[q] = stride * (int64_t)sizeof(float);
      jdst[q] = dst;
    }
  }
  auto issue = [&](int s, int slot) {  // stage st0 + s into ring slot `slot`
    float* base = lds + slot * SF;
#pragma unroll
    for (int q = 0; q < MAXJ; ++q) {
      if (q < JPW)
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(jsrc[q] + s * jstride[q]),
                                         (__attribute__((address_space(3))) void*)(base + jdst[q]), 16, 0, 0);
    }
  };

  const bool is_in = w < NI;
  const int c0 = is_in ? w : w - NI;
  const int col = 16 * c0 + i;
  const bool col_ok = is_in ? col < Iin : true;
  const bool db_wave = w == NI;
  const int boff = is_in ? OFF_BIN + col : OFF_BH + col;  // B element of row r: sA[boff + r * IPB]
  const int IPB = is_in ? IP : H;

  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float dbacc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) dbacc[m] = 0.f;

  if (active) {
#pragma unroll
    for (int p = 0; p < R - 1; ++p)
      if (p < nst) issue(p, p);
  }
  int t0 = (int)(((int64_t)st0 * RW + kk) % T);  // t of this lane's first row in the stage
  for (int s = 0; s < nst; ++s) {
    // retire this wave's DMAs of stage s (up to R-2 later stages stay in
    // flight), then a barrier: every wave's DMAs of stage s have landed, and
    // every wave is done with the slot that the refill below overwrites
    if (active) dw_wait_vm_n(min(R - 2, nst - 1 - s) * JPW);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (active && s + R - 1 < nst) issue(s + R - 1, (s + R - 1) % R);
    if (!active) continue;
    const float* sA = lds + (s % R) * SF;
    const int64_t k0 = (int64_t)(st0 + s) * RW;
    // the stage's fragments first (all RW / 4 K steps: one LDS latency per
    // stage), then its RW / 4 x 4G MFMAs back to back
    constexpr int KS = RW / 4;
    f32x4 av[KS][G];
    float bv[KS];
    int t = t0;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int r = 4 * ks + kk;
#pragma unroll
      for (int g = 0; g < G; ++g) av[ks][g] = *reinterpret_cast<const f32x4*>(sA + r * 4 * H + 64 * g + 4 * i);
      if constexpr (MASKA) {
        const bool a_ok = k0 + r < k_end;
#pragma unroll
        for (int g = 0; g < G; ++g) av[ks][g] = a_ok ? av[ks][g] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
      const float bval = sA[boff + r * IPB];
      const bool b_ok = (k0 + r < k_end) & col_ok & (is_in | (t > 0));
      bv[ks] = b_ok ? bval : 0.f;
      t += 4;
      t = t >= T ? t - T : t;
    }
    t0 = t;  // KS K steps x 4 rows = one stage: the next stage starts here
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        acc[4 * g + 0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks][g].x, bv[ks], acc[4 * g + 0], 0, 0, 0);
        acc[4 * g + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks][g].y, bv[ks], acc[4 * g + 1], 0, 0, 0);
        acc[4 * g + 2] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks][g].z, bv[ks], acc[4 * g + 2], 0, 0, 0);
        acc[4 * g + 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ks][g].w, bv[ks], acc[4 * g + 3], 0, 0, 0);
      }
    }
    if (db_wave) {  // wave-uniform branch, no loads inside
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const float am = k0 + 4 * ks + kk < k_end ? 1.f : 0.f;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          dbacc[4 * g + 0] = fmaf(am, av[ks][g].x, dbacc[4 * g + 0]);
          dbacc[4 * g + 1] = fmaf(am, av[ks][g].y, dbacc[4 * g + 1]);
          dbacc[4 * g + 2] = fmaf(am, av[ks][g].z, dbacc[4 * g + 2]);
          dbacc[4 * g + 3] = fmaf(am, av[ks][g].w, dbacc[4 * g + 3]);
        }
      }
    }
  }
  if (!active) return;

  // ---- epilogue: partial sums of this chunk -> slab row ----------------------
  float* slab = a.slab + slab_row * a.P;
  const int lo = lane >> 4, j = lane & 15;
  if (col_ok) {
    const int64_t off = is_in ? a.off_wih[l] : a.off_whh[l];
    const int ld = is_in ? Iin : H;
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 64 * g + 16 * lo + 4 * r + c;
          slab[off + (int64_t)m * ld + 16 * c0 + j] = acc[4 * g + c][r];
        }
      }
    }
  }
  if (db_wave) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float v = dbacc[m];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      dbacc[m] = v;
    }
    if (kk == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int m = 64 * g + 4 * i + c;
          if (a.off_bih[l] >= 0) slab[a.off_bih[l] + m] = dbacc[4 * g + c];
          if (a.off_bhh[l] >= 0) slab[a.off_bhh[l] + m] = dbacc[4 * g + c];
        }
      }
    }
  }
}

}  // namespace pdrnn
