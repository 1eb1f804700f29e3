// Sequence-in-wave LSTM / GRU stack (H = 32, 1-2 layers), forward and lean
// BPTT, fp32, gfx950.  The motion model's recurrence (reference: nn.LSTM in
// src/motion/model.py:9,14, trained by src/motion/trainer/base.py:111,116;
// the GRU cell through the packed 4-block stack, CELL = 1, see load_fwd_w).
//
// Why a second small-H family (docs/DESIGN.md §2b): the gate-split kernels of
// lstm_small.hip spread one sequence over 4 waves (a layer = 128 lanes, one
// gate row each), so every step broadcasts the 64-float operand vector from
// LDS to all 4 waves (16 ds_read_b128 per lane, the LDS serialises the four
// waves' reads: ~276 of 966 cycles at B = 180) and crosses an s_barrier
// (~216 cycles).  Here a sequence never leaves its wave:
//
//  * lane = (unit u = lane >> 1, K half s = lane & 1).  A lane holds the four
//    gate rows q*H + u of [W_ih | W_hh] over ITS half of the operand vector
//    (layer >= 1: s = 0 the input h^{l-1}_t, s = 1 the own h_{t-1}; layer 0:
//    s = 0 x_t (12 columns, zero-padded) + h[0, 12), s = 1 h[12, 32)), as k
//    pairs for v_pk_fma_f32.  Half the operand vector per lane: 8 (layer 1) /
//    6 (layer 0) ds_read_b128 per step, the two halves' addresses on disjoint
//    banks.  One DPP swap adds the partner's partial sums.
//  * lane s = 0 activates i, g and lane s = 1 f, o (rows pre-scaled by
//    -log2 e, x2 for g: sigma = 1 / (1 + 2^z), tanh(g) = 2 sigma(2g) - 1); two
//    DPP swaps give both lanes all four gates; both update c, h.
//  * h_t goes to a per-wave LDS slot and is read back by the same wave next
//    step: LDS operations of one wave execute in order, so no barrier and no
//    waitcnt beyond the reads' own.  Mode 2 runs each layer of a 2-layer
//    stack in its own wave (one barrier per step, h^0 handed over through
//    parity slots) for the latency regime.
//  * BPTT, per layer: lane (u, s) owns column u of W_hh (and W_ih for
//    layers >= 1: the input gradient feeding the layer below) over gate rows
//    [64 s, 64 s + 64); the row phase makes the lane's two pre-activation gate
//    gradients (s = 0: i, f; s = 1: g, o) from the saved activations, writes
//    them to LDS and over the activation slots (deferred dW, lstm_small_dw.hip),
//    and the column phase reads its 64 rows back (16 ds_read_b128) for
//    W^T dz; one DPP swap completes the sums.  Layer 1's input gradient
//    stays in registers for layer 0's next step (mode 2: LDS parity slots).
//  * Whole sequences per wave, so the grid is B / NB waves, at most one wave
//    per SIMD (~300-400 VGPRs: every weight in registers).
#include "pdrnn/api.h"
#include "pdrnn/common.h"
#include "pdrnn/motion_head.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace pdrnn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kH = 32;
constexpr float kA = -1.4426950408889634f;  // -log2(e): rows pre-scaled so sigma(z) = 1 / (1 + 2^acc)
constexpr int kHB = 36;                     // h slot: 32 values + a zero chunk (layer 0, s = 1, chunk 5)
constexpr int kXS = 12;                     // staged x row: I <= 12 columns, zero-padded
constexpr int kDZ = 4 * kH + 4;             // dz vector, rows >= 64 shifted by 4 floats (bank spread)
constexpr uint32_t kOOR = 0x80000000u;      // buffer offset past the range: the store is dropped

// bf16 models: fp32 masters rounded to bf16 as they load (round to nearest even)
PDRNN_DEVICE float wround(float v, int w_bf16) { return w_bf16 ? (float)(__bf16)v : v; }
PDRNN_DEVICE float sig2(float z) { return fast_rcp(1.f + __builtin_amdgcn_exp2f(z)); }
PDRNN_DEVICE float tanh_c(float c) { return fmaf(sig2(c * (2.f * kA)), 2.f, -1.f); }
PDRNN_DEVICE float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
PDRNN_DEVICE pdrnn_f2 lo2(float4 v) { return pdrnn_f2{v.x, v.y}; }
PDRNN_DEVICE pdrnn_f2 hi2(float4 v) { return pdrnn_f2{v.z, v.w}; }
PDRNN_DEVICE pdrnn_f2 pfma(pdrnn_f2 a, pdrnn_f2 b, pdrnn_f2 c) { return __builtin_elementwise_fma(a, b, c); }
PDRNN_DEVICE void bstore(float v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, so, 0);
}
PDRNN_DEVICE int dz_slot(int r) { return r + (r >= 2 * kH ? 4 : 0); }
// sum of this lane's value and its K-half partner's (lanes 2u, 2u + 1)
PDRNN_DEVICE float pair_sum(float v) { return v + dpp_swap1(v); }

template <int NB>
PDRNN_DEVICE int pick(const int (&v)[NB], int n) {
  if constexpr (NB == 1) return v[0];
  else if constexpr (NB == 2) return n == 0 ? v[0] : v[1];
  else return n == 0 ? v[0] : n == 1 ? v[1] : v[2];
}
// sequences per wave of a mode: 1 (0, 2, 4, 5, 6), 2 (1, 3).  (Three per
// layer wave -- the mode-2 map at 960 waves for B = 1440, one per SIMD --
// measured slower in both passes: forward +28 us, BPTT +20 us against modes
// 6 / 3, profiles/r6/m7_ab.md; removed.)
constexpr int sw_nb(int mode) { return (mode == 1 || mode == 3) ? 2 : 1; }

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------
// This lane's four gate rows over NC float4 chunks of its operand half, k
// pairs, in the order (m0, x0, m1, x1): m0 / m1 are the gates this lane
// activates (s = 0: i, g; s = 1: f, o) and x0 / x1 the ones its partner
// activates.  After the loop the sum of w[0] is this lane's own partial of
// m0 and the sum of w[1] the partial its partner needs (and likewise for
// m1): one DPP add per gate finishes the K-split sum, with no select.  The
// biases of m0 / m1 seed their accumulators.
template <int NC>
struct FwdW {
  pdrnn_f2 w[4][2 * NC];
  float bias[2];
};

// Column of chunk c, element e (-1: zero) -- see the file comment.
PDRNN_DEVICE int fwd_col(int l, int s, int c, int e, int Iin, bool& from_ih) {
  if (l == 0) {
    if (s == 0) {
      if (c < 3) { from_ih = true; const int k = 4 * c + e; return k < Iin ? k : -1; }
      from_ih = false; return 4 * (c - 3) + e;
    }
    from_ih = false; return c < 5 ? 12 + 4 * c + e : -1;
  }
  from_ih = s == 0;
  return 4 * c + e;
}

// CELL 1 = GRU, packed by the host as a 4-row-block stack with zero blocks
// (W_ih: [W_ir; W_iz; W_in; 0], W_hh: [W_hr; W_hz; 0; W_hn], ops/gru_fused.py),
// so the products are the LSTM's: rows (r, z, n_x, n_h) with n_x / n_h scaled
// by 2 kA (tanh(n_x + r n_h) = 2 sigma(2 (n_x + r n_h)) - 1 is linear in both).
template <int NC, int CELL = 0>
PDRNN_DEVICE FwdW<NC> load_fwd_w(const PdrnnLstmSmallFwdArgs& a, int l, int u, int s) {
  FwdW<NC> W;
  const int Iin = l == 0 ? a.I : kH;
  const float* wih = a.w_ih[l];
  const float* whh = a.w_hh[l];
  const int gq[4] = {s, 1 - s, 2 + s, 3 - s};  // (m0, x0, m1, x1)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = gq[j];
    const int r = q * kH + u;
    const float sc = kA * ((CELL == 0 ? q == 2 : q >= 2) ? 2.f : 1.f);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bool ih = false;
        const int k = fwd_col(l, s, c, e, Iin, ih);
        float x = 0.f;
        if (k >= 0) x = ih ? wih[(int64_t)r * Iin + k] : whh[(int64_t)r * kH + k];
        v[e] = wround(x, a.w_bf16) * sc;
      }
      W.w[j][2 * c] = pdrnn_f2{v[0], v[1]};
      W.w[j][2 * c + 1] = pdrnn_f2{v[2], v[3]};
    }
    if (!(j & 1))
      W.bias[j >> 1] = ((a.b_ih[l] ? wround(a.b_ih[l][r], a.w_bf16) : 0.f) +
                        (a.b_hh[l] ? wround(a.b_hh[l][r], a.w_bf16) : 0.f)) * sc;
  }
  return W;
}

// p[0] / p[2]: own partials of m0 / m1 (+ bias), p[1] / p[3]: the partner's
// (eight accumulators instead of four -- a gate's lo / hi halves apart, no
// back-to-back dependent v_pk_fma_f32 -- measured no faster: a wave alone on
// its SIMD issues v_pk_fma_f32 at ~8 cycles, so the products are issue-bound,
// profiles/r6/fwd_phase_stamps.md)
template <int NC>
PDRNN_DEVICE void fwd_dot(const FwdW<NC>& W, const float4 (&v)[NC], float (&p)[4]) {
  pdrnn_f2 acc[4] = {{W.bias[0], 0.f}, {0.f, 0.f}, {W.bias[1], 0.f}, {0.f, 0.f}};
#ifdef SW_PROBE_HALF_K  // timing probe only (wrong numerics): half the products
#pragma unroll
  for (int c = 0; c < NC / 2; ++c) {
#else
#pragma unroll
  for (int c = 0; c < NC; ++c) {
#endif
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc[j] = pfma(W.w[j][2 * c], lo2(v[c]), acc[j]);
      acc[j] = pfma(W.w[j][2 * c + 1], hi2(v[c]), acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] = acc[j].x + acc[j].y;
}

struct Cell {
  float a0, a1, c, h;
};
// DPP quad_perm [1, 1, 3, 3]: both lanes of a pair read the odd lane
PDRNN_DEVICE float from_odd(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xF5, 0xF, 0xF, false));
}
// The K-split sums -> this lane's two activations (s = 0: i, g; s = 1: f, o;
// `gk` = {2, -1} on even lanes: tanh(g) = 2 sigma(2g) - 1, {1, 0} on odd) and
// the unit's new c, h on both lanes: c = f c + i g is the sum of one product
// per lane (odd: f c, even: i g), h = o tanh(c) with o read from the odd lane.
PDRNN_DEVICE Cell fwd_cell(const float (&p)[4], pdrnn_f2 gk, float c, bool odd) {
  const float z0 = p[0] + dpp_swap1(p[1]);
  const float z1 = p[2] + dpp_swap1(p[3]);
  Cell r;
  r.a0 = sig2(z0);
  r.a1 = fmaf(sig2(z1), gk.x, gk.y);
  const float term = r.a0 * (odd ? c : r.a1);
  r.c = term + dpp_swap1(term);
  r.h = from_odd(r.a1) * tanh_c(r.c);
  return r;
}
// GRU: lane s = 0 holds r and n_x, s = 1 z and n_h (2 kA-scaled); one DPP
// swap each gives both lanes all four, then n = tanh(n_x + r n_h) and
// h = n + z (h_prev - n) on both.  Saved slots: a0 = r | z, a1 = n_x | n_h
// (unscaled; the BPTT reads n_h), c = n.
PDRNN_DEVICE Cell fwd_cell_gru(const float (&p)[4], float hprev, bool odd) {
  const float z0 = p[0] + dpp_swap1(p[1]);
  const float z1 = p[2] + dpp_swap1(p[3]);
  Cell r;
  r.a0 = sig2(z0);
  const float a0p = dpp_swap1(r.a0), z1p = dpp_swap1(z1);
  const float rg = odd ? a0p : r.a0, zg = odd ? r.a0 : a0p;
  const float nx = odd ? z1p : z1, nh = odd ? z1 : z1p;
  r.a1 = z1 * (1.f / (2.f * kA));
  r.c = fmaf(sig2(fmaf(rg, nh, nx)), 2.f, -1.f);
  r.h = fmaf(zg, hprev - r.c, r.c);
  return r;
}
template <int CELL>
PDRNN_DEVICE Cell fwd_cell_any(const float (&p)[4], pdrnn_f2 gk, float c, float hprev, bool odd) {
  if constexpr (CELL == 0) return fwd_cell(p, gk, c, odd);
  else return fwd_cell_gru(p, hprev, odd);
}
template <int NL, int NB>
PDRNN_DEVICE constexpr int fwd_lds_floats_hb() { return NB * NL * 2 * kHB; }

// x staging (forward prologue): NB sequences' [T, I] input rows into the LDS
// rows xs[(n T + t) kXS + k] (zero-padded to kXS; the caller zeroed xs) and,
// when xg_out is set, the fp32 rows [b T + t][xg_ld] of the deferred dW (pad
// columns written as zeros).  A sequence's rows are one contiguous block of the
// motion batch: 16-byte loads of the block, all of a thread's rounds in flight
// at once (element-wise loads, one dependent round per 4 elements per thread,
// cost the single-layer forward 16 us of ~100 at B = 1440, 23 with bf16 x,
// profiles/r6/x_staging.md).  Returns false when the layout does not allow it.
template <int NB>
PDRNN_DEVICE bool stage_x_vec(const PdrnnLstmSmallFwdArgs& a, float* xs, const int (&bsrc)[NB], const int (&bidx)[NB],
                              const int (&vint)[NB], int tid, int nthr) {
  const int T = a.T, I = a.I;
  const int esz = a.x_bf16 ? 2 : 4;
  const int per = T * I;
  if (a.x_st != I || a.x_sb != (int64_t)per || (per * esz) % 16 != 0 ||
      (reinterpret_cast<uintptr_t>(a.x) & 15) != 0)
    return false;
  const int cpe = 16 / esz;  // elements per 16-byte chunk
  const int nch = per / cpe;
  const int tot = NB * nch;
  const int xg_ld = a.xg_ld;
  const char* xb = reinterpret_cast<const char*>(a.x);
  constexpr int R = 8;  // chunks per thread in flight
  for (int c0 = tid; c0 < tot; c0 += R * nthr) {
    uint4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = min(c0 + r * nthr, tot - 1);
      const int n = c / nch, q = c - n * nch;
      v[r] = *reinterpret_cast<const uint4*>(xb + ((int64_t)pick<NB>(bsrc, n) * per + (int64_t)q * cpe) * esz);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int c = c0 + r * nthr;
      if (c < tot) {
        const int n = c / nch, q = c - n * nch;
        const uint32_t w[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
        const int e0 = q * cpe;
        int t = e0 / I, k = e0 - t * I;  // (one division per chunk, then stepped)
        float* xrow = xs + (n * T + t) * kXS;
        float* grow = a.xg_out ? a.xg_out + ((int64_t)pick<NB>(bidx, n) * T + t) * xg_ld : nullptr;
        const bool gv = grow != nullptr && pick<NB>(vint, n);
        for (int j = 0; j < cpe; ++j) {
          const float val = esz == 2 ? __uint_as_float((j & 1 ? w[j >> 1] >> 16 : w[j >> 1] & 0xFFFFu) << 16)
                                     : __uint_as_float(w[j]);
          xrow[k] = val;
          if (gv && k < xg_ld) grow[k] = val;
          if (++k == I) {
            k = 0;
            xrow += kXS;
            if (grow) grow += xg_ld;
          }
        }
      }
    }
  }
  if (a.xg_out && xg_ld > I) {  // the dW kernel reads xg_ld columns: zero pads
    const int padw = xg_ld - I;
    for (int e = tid; e < NB * T * padw; e += nthr) {
      const int n = e / (T * padw), rem = e - n * (T * padw);
      const int t = rem / padw, k = I + rem - t * padw;
      if (pick<NB>(vint, n)) a.xg_out[((int64_t)pick<NB>(bidx, n) * T + t) * xg_ld + k] = 0.f;
    }
  }
  return true;
}

// NL = 1 or 2.  MODE 0/1: one wave runs all layers of NB = 1 / 2 sequences.
// MODE 2/3 (NL = 2): wave l runs layer l of NB = 1 / 2 sequences, one
// barrier per step (layer 0's h_t handed over through parity slots).
// mode 2 holds <= 168 VGPRs: three waves per SIMD, so B = 1440 (2880 layer
// waves on 1024 SIMDs) is one residency round with every SIMD loaded evenly
template <int NL, int MODE, int CELL = 0>
__global__ void __launch_bounds__(MODE >= 2 ? 64 * NL : 64) __attribute__((amdgpu_waves_per_eu(MODE == 6 ? 3 : 1)))
lstm_sw_fwd_kernel(PdrnnLstmSmallFwdArgs a) {
  constexpr int NB = sw_nb(MODE);
  constexpr bool SPLIT = MODE >= 2;
  static_assert(NL == 1 || NL == 2, "one or two layers");
  static_assert(!SPLIT || NL == 2, "layer-split mode needs two layers");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x, nthr = blockDim.x;
  const uint64_t sr_in = (a.stamps && tid == 0) ? stamp_real() : 0;  // (entry: the prologue's cost)
  const int lane = tid & 63;
  const int wv = SPLIT ? __builtin_amdgcn_readfirstlane(tid >> 6) : 0;
  const int u = lane >> 1;
  const bool odd = (lane & 1) != 0;
  const int B = a.B, T = a.T, I = a.I;
  const int bbase = blockIdx.x * NB;
  float* hb = smem;
  float* xs = smem + fwd_lds_floats_hb<NL, NB>();
  auto hbuf = [&](int n, int l, int p) { return hb + ((n * NL + l) * 2 + p) * kHB; };

  int bidx[NB], bsrc[NB], vint[NB];
  bool valid[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    valid[n] = b < B;
    vint[n] = valid[n] ? 1 : 0;
    bidx[n] = valid[n] ? b : B - 1;  // an empty slot recomputes the last sequence, stores nothing
    bsrc[n] = a.idx ? (int)a.idx[bidx[n]] : bidx[n];
  }

  // ---- prologue: zero the h slots (h_{-1} = 0, pad chunks), stage x ------
  // (the vector staging writes only the I real columns: xs zeroed first; two
  // sequences per workgroup only -- with one, the zeroing pass and barrier
  // cost more than the element loads: mode 6 136.2 vs 133.6 us at B = 1440)
  const bool xvec = NB == 2 && a.x_st == I && a.x_sb == (int64_t)T * I;
  for (int e = tid; e < fwd_lds_floats_hb<NL, NB>() + (xvec ? NB * T * kXS : 0); e += nthr) hb[e] = 0.f;
  if (xvec) lds_barrier();
  if (!(xvec && stage_x_vec<NB>(a, xs, bsrc, bidx, vint, tid, nthr))) {
    const int per = T * kXS, tot = NB * per;
    const int xg_ld = a.xg_ld;
    for (int e0 = tid; e0 < tot; e0 += 4 * nthr) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = min(e0 + r * nthr, tot - 1);
        const int n = e / per, rem = e - n * per;
        const int t = rem / kXS, k = rem - t * kXS;
        const float x = ldx(a.x, (int64_t)pick<NB>(bsrc, n) * a.x_sb + (int64_t)t * a.x_st + min(k, I - 1), a.x_bf16);
        v[r] = k < I ? x : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = e0 + r * nthr;
        if (e < tot) {
          const int n = e / per, rem = e - n * per;
          const int t = rem / kXS, k = rem - t * kXS;
          xs[e] = v[r];
          if (a.xg_out && k < xg_ld && pick<NB>(vint, n))
            a.xg_out[((int64_t)pick<NB>(bidx, n) * T + t) * xg_ld + k] = v[r];
        }
      }
    }
  }
  // the LDS rows are in place; the xg_out stores (read by a later launch) need
  // not drain here -- a __syncthreads() would wait for them (~1-3 us)
  lds_barrier();

  const __amdgpu_buffer_rsrc_t r_act = uniform_rsrc(a.act);
  const __amdgpu_buffer_rsrc_t r_h = uniform_rsrc(a.hseq);
  const uint32_t s_ = odd ? 1u : 0u;
  const uint32_t vo_a0 = (s_ * kH + u) * 4, vo_a1 = ((2 + s_) * kH + u) * 4, vo_c = (4 * kH + u) * 4, vo_h = u * 4;
  uint32_t vmask[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) vmask[n] = valid[n] ? 0u : kOOR;
  // byte offset of row (l, b, t) in act (5H floats per row) and hseq (H)
  auto row = [&](int l, int n, int t) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((uint32_t)(((l * B + pick<NB>(bidx, n)) * T + t)));
  };

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  // state: c and the last committed h per (layer, sequence)
  float cst[NL][NB], hst[NL][NB];
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int n = 0; n < NB; ++n) { cst[l][n] = 0.f; hst[l][n] = 0.f; }

  // Layer 0 at time t (active unless t == T) / layer 1 at time t (active
  // unless t < 0), for all NB sequences, split into the operand reads and the
  // rest: a caller running both layers issues both layers' reads first (their
  // LDS order against the other layer's h write would otherwise serialise
  // the two independent chains).
  auto rd0 = [&](int t, float4 (&v)[NB][6]) {
    const int tc = min(t, T - 1);
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const float* hp = hbuf(n, 0, (t - 1) & 1);
      const float* pa = odd ? hp + 12 : xs + (n * T + tc) * kXS;
      const float* pb = odd ? hp + 24 : hp;
#pragma unroll
      for (int c = 0; c < 3; ++c) v[n][c] = ld4(pa + 4 * c);
#pragma unroll
      for (int c = 0; c < 3; ++c) v[n][3 + c] = ld4(pb + 4 * c);
    }
  };
  auto rd1 = [&](int t, float4 (&v)[NB][8]) {
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const float* pc = odd ? hbuf(n, 1, (t - 1) & 1) : hbuf(n, 0, t & 1);
#pragma unroll
      for (int c = 0; c < 8; ++c) v[n][c] = ld4(pc + 4 * c);
    }
  };
  auto commit = [&](int l, int n, int t, bool act, const Cell& r) {
    cst[l][n] = act ? r.c : cst[l][n];
    hst[l][n] = act ? r.h : hst[l][n];
    hbuf(n, l, t & 1)[u] = hst[l][n];
    const uint32_t rw = row(l, n, min(max(t, 0), T - 1));
    const uint32_t m = act ? vmask[n] : kOOR;
    bstore(r.a0, r_act, vo_a0 | m, rw * (5 * kH * 4));
    bstore(r.a1, r_act, vo_a1 | m, rw * (5 * kH * 4));
    bstore(r.c, r_act, vo_c | m, rw * (5 * kH * 4));
    bstore(r.h, r_h, vo_h | m, rw * (kH * 4));
  };
  const pdrnn_f2 gk = odd ? pdrnn_f2{1.f, 0.f} : pdrnn_f2{2.f, -1.f};
  auto cmp0 = [&](const FwdW<6>& W, int t, const float4 (&v)[NB][6]) {
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      float p[4];
      fwd_dot<6>(W, v[n], p);
      commit(0, n, t, t < T, fwd_cell_any<CELL>(p, gk, cst[0][n], hst[0][n], odd));
    }
  };
  auto cmp1 = [&](const FwdW<8>& W, int t, const float4 (&v)[NB][8]) {
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      float p[4];
      fwd_dot<8>(W, v[n], p);
      commit(NL - 1, n, t, t >= 0, fwd_cell_any<CELL>(p, gk, cst[NL - 1][n], hst[NL - 1][n], odd));
    }
  };

  if constexpr (NL == 1) {
    const FwdW<6> W0 = load_fwd_w<6, CELL>(a, 0, u, odd ? 1 : 0);
    for (int t = 0; t < T; ++t) {
      float4 v0[NB][6];
      rd0(t, v0);
      cmp0(W0, t, v0);
    }
  } else if constexpr (!SPLIT) {
    const FwdW<6> W0 = load_fwd_w<6, CELL>(a, 0, u, odd ? 1 : 0);
    const FwdW<8> W1 = load_fwd_w<8, CELL>(a, 1, u, odd ? 1 : 0);
    // layer 0 at t = it, layer 1 at t = it - 1: both read h^0_{it-1}
    for (int it = 0; it <= T; ++it) {
      float4 v0[NB][6], v1[NB][8];
      rd0(it, v0);
      rd1(it - 1, v1);
      cmp0(W0, it, v0);
      cmp1(W1, it - 1, v1);
    }
  } else {
    // mode 2: every operand read of the step in flight before the first
    // FMA (one LDS latency per step); mode 6 (the same map at <= 168 VGPRs,
    // three waves per SIMD for B > one wave per SIMD) leaves the reads to the
    // scheduler, which pairs them to stay within its registers
    if (wv == 0) {
      const FwdW<6> W0 = load_fwd_w<6, CELL>(a, 0, u, odd ? 1 : 0);
      for (int it = 0; it <= T; ++it) {
        if (it < T) {
          float4 v0[NB][6];
          rd0(it, v0);
          if constexpr (MODE != 6) __builtin_amdgcn_sched_barrier(0);
          cmp0(W0, it, v0);
        }
        lds_barrier();
      }
    } else {
      const FwdW<8> W1 = load_fwd_w<8, CELL>(a, 1, u, odd ? 1 : 0);
      for (int it = 0; it <= T; ++it) {
        if (it > 0) {
          float4 v1[NB][8];
          rd1(it - 1, v1);
          if constexpr (MODE != 6) __builtin_amdgcn_sched_barrier(0);
          cmp1(W1, it - 1, v1);
        }
        lds_barrier();
      }
    }
  }
  uint64_t sr1 = 0;
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    sr1 = stamp_real();
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = sr1;
  }

  // ---- epilogue: h_n / c_n, then the fused head on the top layer's h_T ----
  // (two sequences per wave: both heads' operands loaded first, their
  // dependent loads in flight together, not behind the first head's stores;
  // one sequence loads inline -- the VGPR-capped mode 6 would spill)
  const bool top_wave = !SPLIT || wv == NL - 1;
  HeadIn hin[NB];
  if constexpr (NB > 1) {
    if (a.head_w && top_wave) {
#pragma unroll
      for (int n = 0; n < NB; ++n) hin[n] = head_load(a, pick<NB>(bidx, n), u);
    }
  }
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    if (!valid[n]) continue;
    const int b = bbase + n;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      if (SPLIT && l != wv) continue;
      if (!odd && a.hn) a.hn[((int64_t)l * B + b) * kH + u] = hst[l][n];
      if (!odd && a.cn) a.cn[((int64_t)l * B + b) * kH + u] = cst[l][n];
    }
    if (a.head_w && top_wave) {
      if constexpr (NB > 1) motion_head(a, b, hst[NL - 1][n], u, odd, hin[n]);
      else motion_head(a, b, hst[NL - 1][n], u, odd);
    }
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[4] = sr_in; st[5] = stamp_real(); st[6] = stamp_cu();
  }
}

// ---------------------------------------------------------------------------
// Forward, four waves per sequence (mode 5, two-layer stacks in the latency
// regime): wave w runs layer w >> 1, units 16 (w & 1) .. + 15.  lane =
// (unit ul = lane >> 2, K quarter q = lane & 3): a lane holds the four gate
// rows of its unit over a quarter of the operand vector (layer 0: x | h[0,12)
// | h[12,24) | h[24,32) + zero pad, 3 float4 chunks; layer 1: h^0[0,16) |
// h^0[16,32) | h^1[0,16) | h^1[16,32), 4 chunks), half of mode 2's products
// per lane.  A quad reduce-scatter (xor 2, then xor 1) leaves lane q with the
// full pre-activation of gate q (i, f, g, o): one activation per lane; quad
// broadcasts give every lane of the unit i, f, g, o for c and h.  The two
// waves of a layer meet in the per-layer h slots: one barrier per step, as in
// mode 2.
// ---------------------------------------------------------------------------
template <int NC>
struct Fwd4W {
  pdrnn_f2 w[4][2 * NC];
};

PDRNN_DEVICE float quad_bcast(float v, int k) {
  switch (k) {
    case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x00, 0xF, 0xF, false));
    case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x55, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xAA, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xFF, 0xF, 0xF, false));
  }
}

// column of layer l, quarter q, chunk c, element e (-1: zero)
PDRNN_DEVICE int fwd4_col(int l, int q, int c, int e, int Iin, bool& from_ih) {
  const int k = 4 * c + e;
  if (l == 0) {
    if (q == 0) { from_ih = true; return k < Iin ? k : -1; }
    from_ih = false;
    const int hk = 12 * (q - 1) + k;
    return hk < kH ? hk : -1;
  }
  from_ih = q < 2;
  return 16 * (q & 1) + k;
}

template <int NC, int CELL = 0>
PDRNN_DEVICE Fwd4W<NC> load_fwd4_w(const PdrnnLstmSmallFwdArgs& a, int l, int u, int q, float (&bias)[4]) {
  Fwd4W<NC> W;
  const int Iin = l == 0 ? a.I : kH;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = j * kH + u;
    const float sc = kA * ((CELL == 0 ? j == 2 : j >= 2) ? 2.f : 1.f);  // (GRU: see load_fwd_w)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bool ih = false;
        const int k = fwd4_col(l, q, c, e, Iin, ih);
        float x = 0.f;
        if (k >= 0) x = ih ? a.w_ih[l][(int64_t)r * Iin + k] : a.w_hh[l][(int64_t)r * kH + k];
        v[e] = wround(x, a.w_bf16) * sc;
      }
      W.w[j][2 * c] = pdrnn_f2{v[0], v[1]};
      W.w[j][2 * c + 1] = pdrnn_f2{v[2], v[3]};
    }
    bias[j] = q == 0 ? ((a.b_ih[l] ? wround(a.b_ih[l][r], a.w_bf16) : 0.f) +
                        (a.b_hh[l] ? wround(a.b_hh[l][r], a.w_bf16) : 0.f)) * sc
                     : 0.f;
  }
  return W;
}

// PH: per-phase stamps (diagnostics build, PDRNN_TUNE sw_phase=1 with
// PDRNN_LSTM_STAMPS): s_memtime at the loop top (after the barrier), after the
// operand reads landed, after the products, after the quad reduce, after the
// cell and its stores; per-phase cycle sums over steps [16, T - 16) of waves 0
// (layer 0) and 2 (layer 1), written behind the loop stamps (row of 24).
template <int CELL = 0, bool PH = false>
PDRNN_DEVICE void fwd4_body(const PdrnnLstmSmallFwdArgs& a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const uint64_t sr_in = (a.stamps && tid == 0) ? stamp_real() : 0;  // (entry: the prologue's cost)
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = wv >> 1;
  const int ul = lane >> 2, q = lane & 3;
  const int u = 16 * (wv & 1) + ul;
  const int B = a.B, T = a.T, I = a.I;
  const int b = blockIdx.x;  // one sequence per workgroup
  const int bsrc = a.idx ? (int)a.idx[b] : b;
  float* hb = smem;                                  // [layer][parity][kHB]
  float* xs = smem + 2 * 2 * kHB;                    // [T][kXS]
  auto hbuf = [&](int ll, int p) { return hb + (ll * 2 + p) * kHB; };

  // (vector staging as in lstm_sw_fwd_kernel: xs zeroed first)
  const bool xvec = a.x_st == I && a.x_sb == (int64_t)T * I;
  for (int e = tid; e < 2 * 2 * kHB + (xvec ? T * kXS : 0); e += 256) hb[e] = 0.f;
  if (xvec) lds_barrier();
  const int bsrc1[1] = {bsrc}, bidx1[1] = {b}, vint1[1] = {1};
  if (!(xvec && stage_x_vec<1>(a, xs, bsrc1, bidx1, vint1, tid, 256))) {
    for (int e = tid; e < T * kXS; e += 256) {
      const int t = e / kXS, k = e - t * kXS;
      const float x = ldx(a.x, (int64_t)bsrc * a.x_sb + (int64_t)t * a.x_st + min(k, I - 1), a.x_bf16);
      const float v = k < I ? x : 0.f;
      xs[e] = v;
      if (a.xg_out && k < a.xg_ld) a.xg_out[((int64_t)b * T + t) * a.xg_ld + k] = v;
    }
  }
  lds_barrier();  // (as in lstm_sw_fwd_kernel; the one-launch step's __syncthreads drains them before its BPTT)

  const __amdgpu_buffer_rsrc_t r_act = uniform_rsrc(a.act);
  const __amdgpu_buffer_rsrc_t r_h = uniform_rsrc(a.hseq);
  const uint32_t vo_a = (q * kH + u) * 4, vo_c = (4 * kH + u) * 4, vo_h = u * 4;
  const uint32_t lead = q == 0 ? 0u : kOOR;  // c / h stored by lane q = 0 of the unit
  const pdrnn_f2 gk = q == 2 ? pdrnn_f2{2.f, -1.f} : pdrnn_f2{1.f, 0.f};
  float cst = 0.f, hst = 0.f;

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  // quad reduce-scatter of the four gate partials -> this lane's gate (q)
  auto gate_sum = [&](const float (&p)[4]) {
    const bool hi = q >= 2;
    const float k0 = hi ? p[2] : p[0], k1 = hi ? p[3] : p[1];
    const float s0 = hi ? p[0] : p[2], s1 = hi ? p[1] : p[3];
    const float m0 = k0 + dpp_swap2(s0), m1 = k1 + dpp_swap2(s1);
    const bool od = (q & 1) != 0;
    return (od ? m1 : m0) + dpp_swap1(od ? m0 : m1);
  };
  auto cell = [&](int t, bool act, float z) {
    float av, cn, hn;
    if constexpr (CELL == 0) {
      av = fmaf(sig2(z), gk.x, gk.y);  // i, f, tanh g or o of this lane
      const float ig = quad_bcast(av, 0), fg = quad_bcast(av, 1), gg = quad_bcast(av, 2), og = quad_bcast(av, 3);
      cn = fmaf(fg, cst, ig * gg);
      hn = og * tanh_c(cn);
    } else {  // GRU: r, z, or the 2 kA-scaled n_x / n_h of this lane; cn carries n
      const float sg = sig2(z);
      const float v = q < 2 ? sg : z;
      const float rg = quad_bcast(v, 0), zg = quad_bcast(v, 1), nx = quad_bcast(v, 2), nh = quad_bcast(v, 3);
      cn = fmaf(sig2(fmaf(rg, nh, nx)), 2.f, -1.f);
      hn = fmaf(zg, hst - cn, cn);
      av = q < 2 ? sg : z * (1.f / (2.f * kA));  // saved unscaled
    }
    cst = act ? cn : cst;
    hst = act ? hn : hst;
    if (q == 0) hbuf(l, t & 1)[u] = hst;
    const uint32_t rw = __builtin_amdgcn_readfirstlane((uint32_t)((l * B + b) * T + min(max(t, 0), T - 1)));
    const uint32_t m = act ? 0u : kOOR;
    bstore(av, r_act, vo_a | m, rw * (5 * kH * 4));
    bstore(cn, r_act, vo_c | m | lead, rw * (5 * kH * 4));
    bstore(hn, r_h, vo_h | m | lead, rw * (kH * 4));
  };
  // phase stamps (PH only; compiled out otherwise)
  uint64_t ph_t[5] = {0, 0, 0, 0, 0}, ph_sum[5] = {0, 0, 0, 0, 0}, ph_prev = 0, ph_n = 0;
  auto ph_now = [&]() -> uint64_t {
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t v = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return v;
  };
  auto ph_mark = [&](int k, float dep) {
    if constexpr (PH) {
      asm volatile("" ::"v"(dep));  // (the value this phase produced exists before the stamp)
      ph_t[k] = ph_now();
    }
  };
  auto ph_reads = [&]() {
    if constexpr (PH) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ph_t[1] = ph_now();
    }
  };
  auto ph_step = [&](int it) {  // after the barrier: close step it, open it + 1
    if constexpr (PH) {
      const uint64_t now = ph_now();
      if (it >= 16 && it < T - 16) {
        ph_sum[0] += ph_t[1] - ph_t[0];  // barrier -> operand reads landed
        ph_sum[1] += ph_t[2] - ph_t[1];  // products
        ph_sum[2] += ph_t[3] - ph_t[2];  // quad reduce (DPP)
        ph_sum[3] += ph_t[4] - ph_t[3];  // activations, cell, stores issued
        ph_sum[4] += now - ph_t[4];      // barrier wait
        ++ph_n;
      }
      (void)ph_prev;
      ph_t[0] = now;
    }
  };
  if constexpr (PH) ph_t[0] = ph_now();

  if (l == 0) {
    float bias[4];
    const Fwd4W<3> W = load_fwd4_w<3, CELL>(a, 0, u, q, bias);
    for (int it = 0; it <= T; ++it) {
      if (it < T) {
        const int t = it;
        const float* src = q == 0 ? xs + t * kXS : hbuf(0, (t - 1) & 1) + 12 * (q - 1);
        float4 v[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) v[c] = ld4(src + 4 * c);
        __builtin_amdgcn_sched_barrier(0);
        ph_reads();
        pdrnn_f2 acc[4] = {{bias[0], 0.f}, {bias[1], 0.f}, {bias[2], 0.f}, {bias[3], 0.f}};
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] = pfma(W.w[j][2 * c], lo2(v[c]), acc[j]);
            acc[j] = pfma(W.w[j][2 * c + 1], hi2(v[c]), acc[j]);
          }
        float p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j] = acc[j].x + acc[j].y;
        ph_mark(2, p[3]);
        const float z = gate_sum(p);
        ph_mark(3, z);
        cell(t, true, z);
        ph_mark(4, 0.f);
      }
      lds_barrier();
      ph_step(it);
    }
  } else {
    float bias[4];
    const Fwd4W<4> W = load_fwd4_w<4, CELL>(a, 1, u, q, bias);
    for (int it = 0; it <= T; ++it) {
      if (it > 0) {
        const int t = it - 1;
        const float* src = q < 2 ? hbuf(0, t & 1) + 16 * q : hbuf(1, (t - 1) & 1) + 16 * (q - 2);
        float4 v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = ld4(src + 4 * c);
        __builtin_amdgcn_sched_barrier(0);
        ph_reads();
        pdrnn_f2 acc[4] = {{bias[0], 0.f}, {bias[1], 0.f}, {bias[2], 0.f}, {bias[3], 0.f}};
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            acc[j] = pfma(W.w[j][2 * c], lo2(v[c]), acc[j]);
            acc[j] = pfma(W.w[j][2 * c + 1], hi2(v[c]), acc[j]);
          }
        float p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j] = acc[j].x + acc[j].y;
        ph_mark(2, p[3]);
        const float z = gate_sum(p);
        ph_mark(3, z);
        cell(t, true, z);
        ph_mark(4, 0.f);
      }
      lds_barrier();
      ph_step(it);
    }
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * (PH ? 24 : 8);
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
    st[4] = sr_in; st[6] = stamp_cu();  // (exit: after the head, below)
  }
  if constexpr (PH) {
    if ((wv == 0 || wv == 2) && lane == 0) {
      uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 24 + 8 + (wv == 2 ? 8 : 0);
#pragma unroll
      for (int k = 0; k < 5; ++k) st[k] = ph_sum[k];
      st[5] = ph_n;
    }
  }
  // ---- epilogue: h_n / c_n; the head reads the top layer's h_T from its slot
  if (q == 0) {
    if (a.hn) a.hn[((int64_t)l * B + b) * kH + u] = hst;
    if (a.cn) a.cn[((int64_t)l * B + b) * kH + u] = cst;
  }
  if (a.head_w) {
    // (the last barrier of the loop ordered every h_T write before this read:
    // layer 1's last step t = T-1 went to slot (T-1) & 1)
    if (wv == 2) {
      const int hu = lane >> 1;
      motion_head(a, b, hbuf(1, (T - 1) & 1)[hu], hu, (lane & 1) != 0);
    }
  }
  if (a.stamps && tid == 0) a.stamps[(uint64_t)blockIdx.x * (PH ? 24 : 8) + 5] = stamp_real();
}
template <int CELL, bool PH = false>
__global__ void __launch_bounds__(256) lstm_sw_fwd4_kernel(PdrnnLstmSmallFwdArgs a) { fwd4_body<CELL, PH>(a); }

// ---------------------------------------------------------------------------
// Backward (lean contract: zero initial state, dL/dh_T of the top layer only,
// weight gradients deferred to pdrnn_lstm_small_dw)
// ---------------------------------------------------------------------------
struct Ops {
  float i, f, g, o, c, cp;
};

// column u of W_hh (and W_ih) over rows [64 s, 64 s + 64), row pairs
struct BwdCol {
  pdrnn_f2 w[32];
};
PDRNN_DEVICE BwdCol load_bwd_col(const float* w, int ld, int col, bool live, int u, int s, int wbf) {
  BwdCol W;
  (void)u;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const int r = 64 * s + 2 * j;
    const float x0 = w[(int64_t)r * ld + col], x1 = w[(int64_t)(r + 1) * ld + col];
    W.w[j] = live ? pdrnn_f2{wround(x0, wbf), wround(x1, wbf)} : pdrnn_f2{0.f, 0.f};
  }
  return W;
}

// gate gradients of this lane (d0: i | g, d1: f | o) from the saved
// activations; dc carries dL/dc_t into step t - 1
PDRNN_DEVICE void row_phase(const Ops& o, float dht, float& dc, bool odd, bool has_prev, float& d0, float& d1) {
  const float cp = has_prev ? o.cp : 0.f;
  const float tc = tanh_c(o.c);
  const float dcp = fmaf(dht * o.o, fmaf(-tc, tc, 1.f), dc);
  const float X = odd ? o.i : o.g;
  const float Y = odd ? fmaf(-o.g, o.g, 1.f) : fmaf(-o.i, o.i, o.i);
  d0 = dcp * X * Y;
  const float P = odd ? dht : dcp;
  const float Q = odd ? tc : cp;
  const float R = odd ? fmaf(-o.o, o.o, o.o) : fmaf(-o.f, o.f, o.f);
  d1 = P * Q * R;
  dc = dcp * o.f;
}

// GRU (saved r, z, n_h, n; cp = h_{t-1}): the gate-gradient vector is
// [dr r(1-r) | dz z(1-z) | dpn | dpn r] with dpn = dh (1-z) (1-n^2) (s = 0:
// the r, z blocks; s = 1: n_x, n_h), so the column phase W^T dz over the
// packed stack is the LSTM's; dc carries the direct path dh_t z_t into t - 1.
PDRNN_DEVICE void row_phase_gru(const Ops& o, float dht, float& dc, bool odd, bool has_prev, float& d0, float& d1) {
  const float hp = has_prev ? o.cp : 0.f;
  const float dh = dht + dc;
  const float n = o.c, r = o.i, z = o.f;
  const float dpn = dh * (1.f - z) * fmaf(-n, n, 1.f);
  d0 = odd ? dpn : dpn * o.o * fmaf(-r, r, r);
  d1 = odd ? dpn * r : dh * (hp - n) * fmaf(-z, z, z);
  dc = dh * z;
}

PDRNN_DEVICE float col_dot(const BwdCol& W, const float4 (&g)[16]) {
  pdrnn_f2 a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    a0 = pfma(W.w[2 * c], lo2(g[c]), a0);
    a1 = pfma(W.w[2 * c + 1], hi2(g[c]), a1);
  }
  const pdrnn_f2 s = a0 + a1;
  return pair_sum(s.x + s.y);
}

// (no occupancy target: at 168 VGPRs the split backward spills, and it only
// runs at B <= one wave per SIMD)
template <int NL, int MODE, int CELL = 0>
PDRNN_DEVICE void bwd_body(const PdrnnLstmSmallBwdArgs& a) {
  constexpr int NB = sw_nb(MODE);
  constexpr bool SPLIT = MODE >= 2;
  // mode 4: the mode-2 map plus two waves that accumulate the weight
  // gradients on the matrix cores (no gate-gradient stores, no dW launch).
  // (A four-wave BPTT map -- two waves per layer, unit x row quarter -- was
  // correct but slower: 92.7 vs 55.3 us at B = 180, the column phase waiting
  // behind the barrier for the other wave's dz; profiles/r5/sw/bwd5_probe.log;
  // removed in round 6.)
  constexpr bool DWACC = MODE == 4;
  constexpr int ZR = DWACC ? 8 : 2;  // dz slots per (sequence, layer): a ring that holds a dW K step
  static_assert(NL == 1 || NL == 2, "one or two layers");
  static_assert(!SPLIT || NL == 2, "layer-split mode needs two layers");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int tid = threadIdx.x;
  const uint64_t sr_in = (a.stamps && tid == 0) ? stamp_real() : 0;  // (entry: the prologue's cost)
  const int lane = tid & 63;
  const int wv = SPLIT ? __builtin_amdgcn_readfirstlane(tid >> 6) : 0;
  const int u = lane >> 1;
  const int s = lane & 1;
  const bool odd = s != 0;
  const int B = a.B, T = a.T;
  const int bbase = blockIdx.x * NB;
  float* dzb = smem;                          // [NB][NL][ZR][kDZ]
  float* dxb = smem + NB * NL * ZR * kDZ;     // [NB][2][32] (modes 2/3: layer 1 -> layer 0)
  auto dzbuf = [&](int n, int l, int t) { return dzb + ((n * NL + l) * ZR + (t & (ZR - 1))) * kDZ; };

  int bidx[NB];
  bool valid[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    valid[n] = b < B;
    bidx[n] = valid[n] ? b : B - 1;
  }
  uint32_t vmask[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) vmask[n] = valid[n] ? 0u : kOOR;

  // the dW kernel streams whole stages: the PDRNN_DW_PAD_ROWS padding rows
  // behind the last layer's gate gradients must hold finite values
  if (!DWACC && blockIdx.x == 0) {
    float* pad = a.dg_out + (int64_t)NL * B * T * a.dg_st;
    for (int e = tid; e < PDRNN_DW_PAD_ROWS * a.dg_st; e += blockDim.x) pad[e] = 0.f;
  }

  const __amdgpu_buffer_rsrc_t r_act = uniform_rsrc(a.act);
  const __amdgpu_buffer_rsrc_t r_dg = uniform_rsrc(a.dg_out);
  const __amdgpu_buffer_rsrc_t r_hs = uniform_rsrc(a.hseq);  // GRU: h_{t-1}
  const uint32_t st_act = 5 * kH * 4, st_dg = (uint32_t)a.dg_st * 4;
  const uint32_t vo_i = u * 4, vo_f = (kH + u) * 4, vo_g = (2 * kH + u) * 4, vo_o = (3 * kH + u) * 4;
  const uint32_t vo_c = (4 * kH + u) * 4;
  const uint32_t vo_d0 = (2 * s * kH + u) * 4, vo_d1 = ((2 * s + 1) * kH + u) * 4;
  const int slot0 = dz_slot(2 * s * kH + u), slot1 = dz_slot((2 * s + 1) * kH + u);
  const int colbase = dz_slot(64 * s);

  auto rowidx = [&](int l, int n, int t) -> uint32_t {
    return __builtin_amdgcn_readfirstlane((uint32_t)((l * B + pick<NB>(bidx, n)) * T + t));
  };
  // branch-free operand loads of layer l, step t (clamped; masked at use)
  auto load_ops = [&](int l, int n, int t) {
    const int tc = min(max(t, 0), T - 1);
    const uint32_t ra = rowidx(l, n, tc) * st_act;
    const uint32_t rp = __builtin_amdgcn_readfirstlane(tc > 0 ? ra - st_act : ra);
    Ops o;
    o.i = bload(r_act, vo_i, ra);
    o.f = bload(r_act, vo_f, ra);
    o.o = bload(r_act, vo_o, ra);
    o.c = bload(r_act, vo_c, ra);
    if constexpr (CELL == 0) {
      o.g = bload(r_act, vo_g, ra);
      o.cp = bload(r_act, vo_c, rp);
    } else {  // GRU: n_x unused; h_{t-1} of the unit from the saved h sequence
      o.g = 0.f;
      const uint32_t rh = rowidx(l, n, tc) * (kH * 4);
      o.cp = bload(r_hs, u * 4, __builtin_amdgcn_readfirstlane(tc > 0 ? rh - kH * 4 : rh));
    }
    return o;
  };

  // per (layer, sequence) state
  float dhrec[NL][NB], dc[NL][NB], dx1[NB];
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int n = 0; n < NB; ++n) { dhrec[l][n] = 0.f; dc[l][n] = 0.f; }
  float dhtop[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    dx1[n] = 0.f;
    dhtop[n] = a.dhn[(int64_t)bidx[n] * kH + u];
  }
  if (SPLIT) {
    for (int e = tid; e < NB * 2 * 32; e += blockDim.x) dxb[e] = 0.f;
  }

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  // Iteration `it`: the top layer at t = T-1-it, layer 0 (of a 2-layer stack)
  // at t = T-it (lag 1: its dh input is layer 1's input gradient of step t).
  // The body is branch-free (inactive steps compute on clamped operands and
  // their stores are dropped): a branch join would make the waitcnt pass wait
  // for the prefetches of the next two iterations.
  const int iters = T + NL - 1;

  // DWACC: the weight gradients on the matrix cores of two extra waves of the
  // workgroup (wave 2: layer 0, wave 3: layer 1), so the BPTT waves never
  // wait on a busy matrix core.  dW_hh / dW_ih of a layer are 16x16 C tiles
  // of v_mfma_f32_16x16x4_f32 (M = 128 gate rows in 8 tiles, N = 32 columns
  // in 2, K = 4 consecutive time steps).  A K step's A operands (the layer's
  // dz from the 8-slot LDS ring) are captured in the iteration after its
  // last step is written; its 32 MFMAs issue a quarter (two m-tiles) per
  // iteration.  The B operands (h_{t-1} and the layer input, no recurrence
  // dependency) are loaded one group ahead.  The BPTT waves keep their two
  // gate rows' bias sums in registers.
  float dbs[2] = {0.f, 0.f};
  const int xld = a.xg_ld;
  // B operands of the K step over times t .. t+3 (lane: time t + (lane >> 4),
  // column lane & 15 of each 16-column tile)
  auto dw_loadb = [&](int l, int t, float (&bv)[4]) {
    const int tk = t + (lane >> 4), c = lane & 15;
    const int64_t b = bidx[0];
    const float* hown = a.hseq + ((int64_t)(l * B + b) * T + max(tk - 1, 0)) * kH;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) bv[nt] = tk > 0 ? hown[16 * nt + c] : 0.f;
    if (l > 0) {
      const float* hin = a.hseq + ((int64_t)((l - 1) * B + b) * T + tk) * kH;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) bv[2 + nt] = hin[16 * nt + c];
    } else {
      bv[2] = c < xld ? a.xg_out[((int64_t)b * T + tk) * xld + c] : 0.f;
      bv[3] = 0.f;
    }
  };
  // the dW wave of layer L (compile time); its iteration `it` is the BPTT
  // waves' iteration (one barrier each)
  auto dw_wave = [&](auto lc) {
    constexpr int L = decltype(lc)::value;
    constexpr int NI = L > 0 ? 2 : 1;  // input column tiles (layer 0: I <= 16)
    f32x4 ahh[8][2], aih[8][NI];
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) ahh[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int nt = 0; nt < NI; ++nt) aih[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float pav[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f}, bnext[4];
    dw_loadb(L, T - 4, bnext);
    // (branch-free: before the first K step is complete the A operands are
    // zeros; a branch would put the accumulators through copies at its joins)
    auto capture = [&](int g, bool live) {
      const float* zb = dzbuf(0, L, g + (lane >> 4));
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const float z = zb[dz_slot(16 * mt + (lane & 15))];
        pav[mt] = live ? z : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) pb[k] = bnext[k];
      dw_loadb(L, max(g - 4, 0), bnext);
    };
    auto quarter = [&](auto qc) {
      constexpr int q = decltype(qc)::value;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        constexpr int m0 = 2 * q;
        const int mt = m0 + j;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          ahh[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pav[mt], pb[nt], ahh[mt][nt], 0, 0, 0);
#pragma unroll
        for (int nt = 0; nt < NI; ++nt)
          aih[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(pav[mt], pb[2 + nt], aih[mt][nt], 0, 0, 0);
      }
    };
    using Q0 = std::integral_constant<int, 0>;
    using Q1 = std::integral_constant<int, 1>;
    using Q2 = std::integral_constant<int, 2>;
    using Q3 = std::integral_constant<int, 3>;
    // T % 4 == 0.  Layer 1's group g (times g .. g+3) is complete after
    // iteration T-1-g, layer 0's after T-g: capture at it = T-g (layer 1) or
    // T-g+1 (layer 0), i.e. at it % 4 == LAG, then one quarter per iteration.
    constexpr int LAG = L == 1 ? 0 : 1;
    auto pos = [&](int it, auto pc) {
      constexpr int p = decltype(pc)::value;
      constexpr int q = (p - LAG + 4) & 3;
      if constexpr (q == 0) capture(T - it + LAG, it >= 4 + LAG);
      quarter(std::integral_constant<int, q>{});
      __builtin_amdgcn_sched_barrier(0);  // (a quarter per iteration, not clumped)
      lds_barrier();
    };
    __syncthreads();
    const int iters = T + 1;
    int it = 0;
    for (; it + 3 < iters; it += 4) {
      pos(it, Q0{});
      pos(it + 1, Q1{});
      pos(it + 2, Q2{});
      pos(it + 3, Q3{});
    }
    pos(it, Q0{});  // it = T
    // (after the last barrier every dz is in the ring)
    if constexpr (L == 1) {
      quarter(Q1{}); quarter(Q2{}); quarter(Q3{});
    } else {
      capture(0, true);
      quarter(Q0{}); quarter(Q1{}); quarter(Q2{}); quarter(Q3{});
    }
    // this workgroup's slab row (an empty slot recomputed sequence B - 1: its
    // row must still be written, as zeros, since the reduction sums every row)
    const __amdgpu_buffer_rsrc_t r_slab = uniform_rsrc(a.slab);
    const uint32_t srow = (uint32_t)blockIdx.x * (uint32_t)a.P;  // (element offsets; the slab is far below 2 GiB)
    auto sst = [&](int64_t e, float v) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r_slab, (uint32_t)(srow + e) * 4u, 0, 0);
    };
    const int Iin = L == 0 ? a.I : kH;
    const int c = lane & 15, r4 = 4 * (lane >> 4);
    const float keep = valid[0] ? 1.f : 0.f;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + r4 + r;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) sst(a.off_whh[L] + (int64_t)row * kH + 16 * nt + c, keep * ahh[mt][nt][r]);
#pragma unroll
        for (int nt = 0; nt < NI; ++nt) {
          const int col = 16 * nt + c;
          if (col < Iin) sst(a.off_wih[L] + (int64_t)row * Iin + col, keep * aih[mt][nt][r]);
        }
      }
  };
  auto db_store = [&](int l) {
    const __amdgpu_buffer_rsrc_t r_slab = uniform_rsrc(a.slab);
    const uint32_t srow = (uint32_t)blockIdx.x * (uint32_t)a.P;
    auto sst = [&](int64_t e, float v) {
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r_slab, (uint32_t)(srow + e) * 4u, 0, 0);
    };
    const float d0 = valid[0] ? dbs[0] : 0.f, d1 = valid[0] ? dbs[1] : 0.f;
    const int r0 = 2 * s * kH + u, r1 = r0 + kH;
    if (a.off_bih[l] >= 0) { sst(a.off_bih[l] + r0, d0); sst(a.off_bih[l] + r1, d1); }
    if (a.off_bhh[l] >= 0) { sst(a.off_bhh[l] + r0, d0); sst(a.off_bhh[l] + r1, d1); }
  };

  // layer-generic pieces
  // (carrying c_{t-1} into the next step instead of re-loading it as that
  // step's c_t measured slower: BPTT 141 vs 128 us at B = 1440)
  auto rows = [&](int l, int n, int t, const Ops& o, float dh_in, bool act) {
    float d0, d1, dcn = dc[l][n];
    if constexpr (CELL == 0) row_phase(o, dhrec[l][n] + dh_in, dcn, odd, t > 0, d0, d1);
    else row_phase_gru(o, dhrec[l][n] + dh_in, dcn, odd, t > 0, d0, d1);
    dc[l][n] = act ? dcn : dc[l][n];
    float* zb = dzbuf(n, l, t);
    zb[slot0] = d0;
    zb[slot1] = d1;
    if constexpr (DWACC) {
      dbs[0] += act ? d0 : 0.f;
      dbs[1] += act ? d1 : 0.f;
    } else {
      const uint32_t so = rowidx(l, n, min(max(t, 0), T - 1)) * st_dg;
      const uint32_t m = act ? vmask[n] : kOOR;
      bstore(d0, r_dg, vo_d0 | m, so);
      bstore(d1, r_dg, vo_d1 | m, so);
    }
  };
  auto read_dz = [&](int l, int n, int t, float4 (&g)[16]) {
    const float* zb = dzbuf(n, l, t) + colbase;
#pragma unroll
    for (int c = 0; c < 16; ++c) g[c] = ld4(zb + 4 * c);
  };

  if constexpr (NL == 1) {
    const BwdCol Whh = load_bwd_col(a.w_hh[0], kH, u, true, u, s, a.w_bf16);
    Ops opA[NB], opB[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) opA[n] = load_ops(0, n, T - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NB; ++n) opB[n] = load_ops(0, n, T - 2);
    __builtin_amdgcn_sched_barrier(0);
    auto body = [&](int it, Ops (&op)[NB]) {
      const int t = T - 1 - it;
      const bool act = t >= 0;
#pragma unroll
      for (int n = 0; n < NB; ++n) rows(0, n, t, op[n], it == 0 ? dhtop[n] : 0.f, act);
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        float4 g[16];
        read_dz(0, n, t, g);
        const float v = col_dot(Whh, g);
        dhrec[0][n] = act ? v : dhrec[0][n];
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) op[n] = load_ops(0, n, t - 2);
    };
    int it = 0;
    for (; it + 1 < iters; it += 2) {
      body(it, opA);
      body(it + 1, opB);
    }
    if (it < iters) body(it, opA);
  } else if constexpr (!SPLIT) {
    const BwdCol Whh1 = load_bwd_col(a.w_hh[1], kH, u, true, u, s, a.w_bf16);
    const BwdCol Wih1 = load_bwd_col(a.w_ih[1], kH, u, true, u, s, a.w_bf16);
    const BwdCol Whh0 = load_bwd_col(a.w_hh[0], kH, u, true, u, s, a.w_bf16);
    Ops opA[2][NB], opB[2][NB];
    // issue order pinned (A's loads, then B's, each layer 1 then layer 0): the
    // loop's counted vmcnt waits are the max over its entry edges
#pragma unroll
    for (int n = 0; n < NB; ++n) { opA[1][n] = load_ops(1, n, T - 1); opA[0][n] = load_ops(0, n, T); }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NB; ++n) { opB[1][n] = load_ops(1, n, T - 2); opB[0][n] = load_ops(0, n, T - 1); }
    __builtin_amdgcn_sched_barrier(0);
    auto body = [&](int it, Ops (&op)[2][NB]) {
      const int t1 = T - 1 - it, t0 = T - it;
      const bool act1 = t1 >= 0, act0 = t0 < T;
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        rows(1, n, t1, op[1][n], it == 0 ? dhtop[n] : 0.f, act1);
        rows(0, n, t0, op[0][n], dx1[n], act0);
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        float4 g1[16], g0[16];
        read_dz(1, n, t1, g1);
        read_dz(0, n, t0, g0);
        const float vh1 = col_dot(Whh1, g1);
        const float vx1 = col_dot(Wih1, g1);
        const float vh0 = col_dot(Whh0, g0);
        dhrec[1][n] = act1 ? vh1 : dhrec[1][n];
        dx1[n] = act1 ? vx1 : 0.f;
        dhrec[0][n] = act0 ? vh0 : dhrec[0][n];
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) { op[1][n] = load_ops(1, n, t1 - 2); op[0][n] = load_ops(0, n, t0 - 2); }
    };
    int it = 0;
    for (; it + 1 < iters; it += 2) {
      body(it, opA);
      body(it + 1, opB);
    }
    if (it < iters) body(it, opA);
  } else {
    // modes 2/3: wave 1 = layer 1 (t = T-1-it), wave 0 = layer 0 (t = T-it),
    // one barrier per iteration; layer 1's input gradient of step t reaches
    // layer 0 through dxb[n][t & 1]
    if (wv == 1) {
      const BwdCol Whh1 = load_bwd_col(a.w_hh[1], kH, u, true, u, s, a.w_bf16);
      const BwdCol Wih1 = load_bwd_col(a.w_ih[1], kH, u, true, u, s, a.w_bf16);
      Ops opA[NB], opB[NB];
#pragma unroll
      for (int n = 0; n < NB; ++n) opA[n] = load_ops(1, n, T - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NB; ++n) opB[n] = load_ops(1, n, T - 2);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      auto body = [&](int it, Ops (&op)[NB]) {
        const int t = T - 1 - it;
        const bool act = t >= 0;
#pragma unroll
        for (int n = 0; n < NB; ++n) rows(1, n, t, op[n], it == 0 ? dhtop[n] : 0.f, act);
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          float4 g[16];
          read_dz(1, n, t, g);
          const float vh = col_dot(Whh1, g);
          const float vx = col_dot(Wih1, g);
          dhrec[1][n] = act ? vh : dhrec[1][n];
          if (!odd) dxb[(n * 2 + (t & 1)) * 32 + u] = act ? vx : 0.f;
          // one sequence's 64-float dz slice in registers at a time (two
          // would push the wave past 256 VGPRs: one wave per SIMD)
          if (NB > 1) __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int n = 0; n < NB; ++n) op[n] = load_ops(1, n, t - 2);
        lds_barrier();
      };
      int it = 0;
      for (; it + 1 < iters; it += 2) {
        body(it, opA);
        body(it + 1, opB);
      }
      if (it < iters) body(it, opA);
      if constexpr (DWACC) db_store(1);
    } else if (wv == 0) {
      const BwdCol Whh0 = load_bwd_col(a.w_hh[0], kH, u, true, u, s, a.w_bf16);
      Ops opA[NB], opB[NB];
#pragma unroll
      for (int n = 0; n < NB; ++n) opA[n] = load_ops(0, n, T);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NB; ++n) opB[n] = load_ops(0, n, T - 1);
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      auto body = [&](int it, Ops (&op)[NB]) {
        const int t = T - it;
        const bool act = t < T;
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          const float dxin = dxb[(n * 2 + (t & 1)) * 32 + u];  // layer 1's step-t input gradient
          rows(0, n, t, op[n], act ? dxin : 0.f, act);
        }
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          float4 g[16];
          read_dz(0, n, t, g);
          const float vh = col_dot(Whh0, g);
          dhrec[0][n] = act ? vh : dhrec[0][n];
          if (NB > 1) __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int n = 0; n < NB; ++n) op[n] = load_ops(0, n, t - 2);
        lds_barrier();
      };
      int it = 0;
      for (; it + 1 < iters; it += 2) {
        body(it, opA);
        body(it + 1, opB);
      }
      if (it < iters) body(it, opA);
      if constexpr (DWACC) db_store(0);
    } else if constexpr (DWACC) {
      if (wv == 2) dw_wave(std::integral_constant<int, 0>{});
      else dw_wave(std::integral_constant<int, 1>{});
    }
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    const uint64_t sr1 = stamp_real();
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = sr1;
    st[4] = sr_in; st[5] = sr1; st[6] = stamp_cu();
  }
}
template <int NL, int MODE, int CELL = 0>
__global__ void __launch_bounds__(MODE == 4 ? 256 : MODE >= 2 ? 64 * NL : 64)
lstm_sw_bwd_kernel(PdrnnLstmSmallBwdArgs a) {
  bwd_body<NL, MODE, CELL>(a);
}

// ---------------------------------------------------------------------------
// One-launch step (latency regime: B <= two workgroups per CU, two layers).
// Workgroup b runs sequence b's four-wave forward (mode 5) with the head/CE,
// then -- no grid-wide dependency between the passes -- the same sequence's
// BPTT with its two matrix-core dW waves (mode 4): each sequence's backward
// starts the moment its own forward ends instead of after the slowest
// workgroup of a forward launch.  Every operand the backward reads (act,
// hseq, the staged x rows, dh_T) was written by the same workgroup: a
// __syncthreads() (which drains vmcnt on gfx950) orders them.  The slab
// reduction stays a launch of its own: inside this one (device-coherent slab
// stores, an arrival counter, every workgroup summing a column slice) it cost
// 15 us against 7 for the separate launch, and a release fence instead of
// the coherent stores 35 (profiles/r6/one_launch_step.md).
// ---------------------------------------------------------------------------
template <int CELL>
__global__ void __launch_bounds__(256) lstm_sw_step_kernel(PdrnnLstmSmallFwdArgs f, PdrnnLstmSmallBwdArgs bk) {
  fwd4_body<CELL>(f);
  __syncthreads();  // the forward's outputs (act, hseq, x rows, dh_T) before the backward reads them
  bwd_body<2, 4, CELL>(bk);
}

// ---- host side -------------------------------------------------------------
int sw_cus() {
  static thread_local int c_dev = -1, c_val = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev != c_dev) {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    c_dev = dev;
    c_val = cus > 0 ? cus : 1;
  }
  return c_val;
}

size_t fwd_lds(int NL, int nb, int T) { return sizeof(float) * ((size_t)nb * NL * 2 * kHB + (size_t)nb * T * kXS); }
size_t bwd_lds(int NL, int nb, int zr = 2) { return sizeof(float) * ((size_t)nb * NL * zr * kDZ + (size_t)nb * 2 * 32); }
int mode_nb(int mode) { return sw_nb(mode); }

template <int NL, int MODE>
hipError_t launch_fwd(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  constexpr int NB = sw_nb(MODE);
  const int grid = (a->B + NB - 1) / NB;
  const int block = MODE >= 2 ? 64 * NL : 64;
  if (a->cell == 1)
    hipLaunchKernelGGL((lstm_sw_fwd_kernel<NL, MODE, 1>), dim3(grid), dim3(block), fwd_lds(NL, NB, a->T), st, *a);
  else
    hipLaunchKernelGGL((lstm_sw_fwd_kernel<NL, MODE, 0>), dim3(grid), dim3(block), fwd_lds(NL, NB, a->T), st, *a);
  return hipGetLastError();
}
hipError_t launch_fwd4(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  const size_t lds = sizeof(float) * (2 * 2 * kHB + (size_t)a->T * kXS);
  if (a->phase_stamps && a->stamps && a->cell == 0)
    hipLaunchKernelGGL((lstm_sw_fwd4_kernel<0, true>), dim3(a->B), dim3(256), lds, st, *a);
  else if (a->cell == 1) hipLaunchKernelGGL(lstm_sw_fwd4_kernel<1>, dim3(a->B), dim3(256), lds, st, *a);
  else hipLaunchKernelGGL(lstm_sw_fwd4_kernel<0>, dim3(a->B), dim3(256), lds, st, *a);
  return hipGetLastError();
}
template <int NL, int MODE>
hipError_t launch_bwd(const PdrnnLstmSmallBwdArgs* a, hipStream_t st) {
  constexpr int NB = sw_nb(MODE);
  const int grid = (a->B + NB - 1) / NB;
  const int block = MODE == 4 ? 256 : MODE >= 2 ? 64 * NL : 64;
  const size_t lds = bwd_lds(NL, NB, MODE >= 4 ? 8 : 2);
  if (a->cell == 1) hipLaunchKernelGGL((lstm_sw_bwd_kernel<NL, MODE, 1>), dim3(grid), dim3(block), lds, st, *a);
  else hipLaunchKernelGGL((lstm_sw_bwd_kernel<NL, MODE, 0>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

}  // namespace
}  // namespace pdrnn

using namespace pdrnn;


extern "C" int pdrnn_lstm_sw_ok(int H, int I, int NL, int cell) {
  return (H == kH && I >= 1 && I <= kXS && (NL == 1 || NL == 2) && (cell == 0 || cell == 1)) ? 1 : 0;
}

// Every (layer, sequence, step) row of `act` (5H floats) and `hseq` is
// addressed as a 32-bit byte offset under ONE buffer descriptor whose range
// is 2 GiB (uniform_rsrc): past it loads return 0 and stores are dropped.
// The launchers refuse batches whose last row (plus the deferred-dW padding
// rows) would not fit; the caller then takes the gate-split family, which
// rebases its descriptors per sequence.
extern "C" int pdrnn_lstm_sw_fits(int NL, int B, int T) {
  const int64_t rows = (int64_t)NL * B * T + PDRNN_DW_PAD_ROWS;
  return (NL >= 1 && B >= 1 && T >= 1 && rows * 5 * kH * 4 < ((int64_t)1 << 31)) ? 1 : 0;
}

// Measured (bench/sw_probe.cpp, profiles/r5/sw): two-layer stacks run one
// wave per layer up to one wave per SIMD (mode 2) -- the forward two waves
// per layer up to half a wave per SIMD (mode 5: 56.5 vs 62.0 us at B = 180,
// 73.1 vs 81.8 at 512, slower above, profiles/r5/sw/fwd4_probe.log); above, the forward keeps
// that map at three waves per SIMD (mode 6) and the backward takes two
// sequences per wave (mode 3).  Up to two workgroups per CU the backward
// forms the weight gradients itself (mode 4: two more waves per workgroup on
// the matrix cores, no dW launch; 55.7 us against 54.7 + 16.9 at B = 180,
// profiles/r5/sw/dw4_probe.log; T % 4 == 0, the caller falls back to mode 2
// otherwise).  One layer: one wave per sequence (mode 0),
// two above one wave per SIMD (mode 1).  PDRNN_TUNE sw_mode / sw_bwd_mode
// override (sw_mode alone: both passes).
extern "C" int pdrnn_lstm_sw_mode(int NL, int B, int backward) {
  int m = pdrnn_tune_int(backward ? "sw_bwd_mode" : "sw_mode", -1);
  if (m < 0 && backward) m = pdrnn_tune_int("sw_mode", -1);
  if (m >= 0) {
    if (m >= 0 && m <= 6 && (m < 2 || NL == 2) && (m != 6 || !backward) && (m != 4 || backward) &&
        (m != 5 || !backward))
      return m;
  }
  const int simds = 4 * sw_cus();
  // (modes 4 / 5: four waves per workgroup, two workgroups per CU)
  if (NL == 2 && 2 * B <= simds) return backward ? 4 : 5;
  if (NL == 2) return B <= simds ? 2 : backward ? 3 : 6;
  return B <= simds ? 0 : 1;
}

extern "C" int pdrnn_lstm_sw_nb(int mode) { return mode_nb(mode); }

namespace {
size_t step_lds(int T) { return std::max(sizeof(float) * (2 * 2 * kHB + (size_t)T * kXS), bwd_lds(2, 1, 8)); }
}  // namespace

extern "C" int pdrnn_lstm_sw_step_ok(int NL, int B, int T) {
  if (NL != 2 || B <= 0 || T <= 0 || T % 4 || !pdrnn_lstm_sw_fits(NL, B, T)) return 0;
  if (pdrnn_lstm_sw_mode(NL, B, 0) != 5 || pdrnn_lstm_sw_mode(NL, B, 1) != 4) return 0;
  return step_lds(T) <= 64 * 1024 ? 1 : 0;
}

extern "C" hipError_t pdrnn_lstm_sw_step(const PdrnnLstmSmallFwdArgs* f, const PdrnnLstmSmallBwdArgs* b,
                                         hipStream_t st) {
  if (!pdrnn_lstm_sw_ok(kH, f->I, f->NL, f->cell) || f->NL != 2 || f->h0 || f->c0 || b->cell != f->cell)
    return hipErrorInvalidValue;
  if (!f->act || !f->hseq || f->B <= 0 || f->T <= 0 || f->T % 4 || !pdrnn_lstm_sw_fits(f->NL, f->B, f->T))
    return hipErrorInvalidValue;
  if (!f->head_w || f->C > 16 || f->C < 1 || !f->labels || !f->slab || !f->dh_top) return hipErrorInvalidValue;
  if (!f->xg_out || f->xg_ld < f->I || f->xg_ld > 16) return hipErrorInvalidValue;
  if (b->B != f->B || b->T != f->T || b->NL != 2 || b->act != f->act || b->hseq != f->hseq || b->dhn != f->dh_top ||
      !b->dhn_top_only || !b->slab || b->xg_out != f->xg_out || b->h0 || b->c0 || b->dout || b->dcn || b->dx ||
      b->dh0 || b->dc0)
    return hipErrorInvalidValue;
  const size_t lds = step_lds(f->T);
  if (lds > 64 * 1024) return hipErrorInvalidConfiguration;
  if (f->cell == 1) hipLaunchKernelGGL(lstm_sw_step_kernel<1>, dim3(f->B), dim3(256), lds, st, *f, *b);
  else hipLaunchKernelGGL(lstm_sw_step_kernel<0>, dim3(f->B), dim3(256), lds, st, *f, *b);
  return hipGetLastError();
}

extern "C" hipError_t pdrnn_lstm_sw_fwd(const PdrnnLstmSmallFwdArgs* a, int mode, hipStream_t st) {
  if (!pdrnn_lstm_sw_ok(kH, a->I, a->NL, a->cell) || a->h0 || a->c0) return hipErrorInvalidValue;
  if (!a->act || !a->hseq || a->B <= 0 || a->T <= 0) return hipErrorInvalidValue;
  if (!pdrnn_lstm_sw_fits(a->NL, a->B, a->T)) return hipErrorInvalidValue;  // 2 GiB descriptor range
  if (a->head_w && (a->C > 16 || a->C < 1 || !a->labels || !a->slab || !a->dh_top)) return hipErrorInvalidValue;
  if (a->xg_out && (a->xg_ld < a->I || a->xg_ld > kXS)) return hipErrorInvalidValue;
  if (fwd_lds(a->NL, mode_nb(mode), a->T) > 64 * 1024) return hipErrorInvalidConfiguration;
  if (a->NL == 1) {
    if (mode == 0) return launch_fwd<1, 0>(a, st);
    if (mode == 1) return launch_fwd<1, 1>(a, st);
    return hipErrorInvalidValue;
  }
  if (mode == 0) return launch_fwd<2, 0>(a, st);
  if (mode == 1) return launch_fwd<2, 1>(a, st);
  if (mode == 2) return launch_fwd<2, 2>(a, st);
  if (mode == 3) return launch_fwd<2, 3>(a, st);
  if (mode == 6) return launch_fwd<2, 6>(a, st);
  if (mode == 5) return launch_fwd4(a, st);
  return hipErrorInvalidValue;
}

extern "C" hipError_t pdrnn_lstm_sw_bwd(const PdrnnLstmSmallBwdArgs* a, int mode, hipStream_t st) {
  if (!pdrnn_lstm_sw_ok(kH, a->I, a->NL, a->cell)) return hipErrorInvalidValue;
  if (a->h0 || a->c0 || a->dout || a->dcn || a->dx || a->dh0 || a->dc0 || !a->dhn || !a->dhn_top_only)
    return hipErrorInvalidValue;  // lean contract only
  if (!a->act || !a->dg_out || a->dg_st < 4 * kH || a->B <= 0 || a->T <= 0) return hipErrorInvalidValue;
  if (!pdrnn_lstm_sw_fits(a->NL, a->B, a->T)) return hipErrorInvalidValue;  // 2 GiB descriptor range
  if (a->NL == 1) {
    if (mode == 0) return launch_bwd<1, 0>(a, st);
    if (mode == 1) return launch_bwd<1, 1>(a, st);
    return hipErrorInvalidValue;
  }
  if (mode == 0) return launch_bwd<2, 0>(a, st);
  if (mode == 1) return launch_bwd<2, 1>(a, st);
  if (mode == 2) return launch_bwd<2, 2>(a, st);
  if (mode == 3) return launch_bwd<2, 3>(a, st);
  if (mode == 4) {  // register dW: one slab row per workgroup; reads the x rows and the h sequence
    if (a->T % 4 || !a->slab || !a->xg_out || a->xg_ld > 16 || !a->hseq) return hipErrorInvalidValue;
    return launch_bwd<2, 4>(a, st);
  }
  return hipErrorInvalidValue;
}
