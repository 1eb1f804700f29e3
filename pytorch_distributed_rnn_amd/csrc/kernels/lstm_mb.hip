// bf16 matrix-core recurrence of the motion LSTM (H = 32, 1-2 layers) for
// bf16 models (BASELINE config 2: weights and inputs in bf16, fp32 cell state
// and accumulation).  Forward and lean BPTT, gfx950.
// Reference model: nn.LSTM + Linear, src/motion/model.py:9-17.
//
// The fp32 kernels (lstm_sw.hip) spend every recurrence step on v_pk_fma_f32:
// at bf16 the matrix cores do the step's products 16x faster, so here a
// workgroup owns a tile of 16 sequences (the MFMA N dimension) and each step
// is v_mfma_f32_16x16x32_bf16 work:
//
//  * forward, layer l: gates^T[128 x 16] = W[128 x K] [x_t | h_{t-1}]^T, as 8
//    M-tiles of 16 gate rows.  M-tile mt holds units {mt, 8+mt, 16+mt, 24+mt}
//    gate-interleaved (row 4 slot + q), so the accumulator rows of lane l
//    (4 (l>>4) .. +3, column l&15) are the four gates of ONE unit of ONE
//    sequence: the cell runs in registers with no lane exchange.  The unit
//    permutation also makes the h a lane produces (units 8 (l>>4) + mt) the
//    B-operand slice (k = 8 (l>>4) .. +7) of its column: the four waves of the
//    tile (two M-tiles each) meet in one LDS image of h_t per step (one 4-byte
//    write and one 16-byte read per lane, one barrier).  x_t enters through one
//    more v_mfma_f32_16x16x32_bf16 per M-tile (K = 16 staged columns + 16
//    zeros) from an LDS-staged bf16 image: one MFMA shape in every accumulate
//    chain (a 16x16x16 result chained into a 16x16x32 as SrcC came out
//    corrupted, run-to-run different, at t >= 1: profiles/r5/sw/mb9_dump.log).
//  * backward, layer l: four waves, wave s owns K-step s of the gate rows
//    (units 8 s .. 8 s + 7): lane l computes the pre-activation gate
//    gradients of units 8 s + 2 (l>>4) + {0, 1} for sequence l&15 -- exactly
//    its B-operand slice of dz -- and dh = W_hh^T dz (+ dx = W_ih^T dz for
//    the layer below) is a split-K MFMA over the four waves, whose partial
//    tiles meet in LDS (parity buffers, one barrier per step).
//  * rounding: h_t, x_t and dz are rounded to bf16 as MFMA operands; products
//    and sums are fp32 (the bf16 model's precision contract); activations,
//    cell state and the saved tensors stay fp32, so the deferred weight
//    gradients (lstm_small_dw.hip) are unchanged.
#include "pdrnn/api.h"
#include "pdrnn/common.h"
#include "pdrnn/motion_head.h"

#include <cstdlib>

namespace pdrnn {
namespace {

constexpr int kH = 32;
constexpr int kN = 16;                      // sequences per workgroup (MFMA columns)
constexpr int kXK = 16;                     // staged x columns (I <= 16, zero-padded)
constexpr float kL2E = 1.4426950408889634f;
constexpr uint32_t kOOR = 0x80000000u;      // buffer offset past the range: the store is dropped
constexpr int kSR = 6 * kH + 4;             // staging row: i f g o c h (+ pad: 16-byte rows, fewer bank conflicts)
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

PDRNN_DEVICE uint32_t bfb(float v) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)v); }
PDRNN_DEVICE uint32_t pk(float a, float b) { return bfb(a) | (bfb(b) << 16); }
PDRNN_DEVICE float rbf(float v) { return (float)(__bf16)v; }
PDRNN_DEVICE float sgm(float z) { return fast_rcp(1.f + __builtin_amdgcn_exp2f(-kL2E * z)); }
PDRNN_DEVICE float tnh(float z) { return fmaf(sgm(2.f * z), 2.f, -1.f); }
PDRNN_DEVICE f32x4 mfma32(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}
PDRNN_DEVICE void bst(float v, __amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, vo, so, 0);
}
PDRNN_DEVICE float bld(__amdgpu_buffer_rsrc_t r, uint32_t vo, uint32_t so) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}

// 8 consecutive bf16 of row r, columns c0 .. c0 + 7 (a row-major [4H, ld] weight)
PDRNN_DEVICE u32x4 wrow8(const float* w, int ld, int r, int c0) {
  const float* p = w + (int64_t)r * ld + c0;
  return u32x4{pk(p[0], p[1]), pk(p[2], p[3]), pk(p[4], p[5]), pk(p[6], p[7])};
}

// ---------------------------------------------------------------------------
// Forward: 4 waves per 16-sequence tile, wave w owns M-tiles 2w, 2w + 1 of
// every layer; iteration `it` runs layer 0 at t = it and layer 1 at t = it - 1.
// ---------------------------------------------------------------------------
template <int NL>
__global__ void __launch_bounds__(256) lstm_mb_fwd_kernel(PdrnnLstmSmallFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int HBF = NL * 2 * kN * kH / 2;  // h images, in floats (bf16 pairs)
  uint16_t* hb16 = reinterpret_cast<uint16_t*>(smem);
  float* htop = smem + HBF;                  // [16][32] fp32: the top layer's h_T for the head
  uint16_t* xs = reinterpret_cast<uint16_t*>(htop + kN * kH);  // [T][16][16] bf16
  // [2 parity][NL][16 seq][kSR] fp32: a step's act rows (i f g o c) and h,
  // written by the cells in MFMA-accumulator order and stored row-coalesced
  // after the step's barrier (direct stores spanned 16 sequences per
  // instruction: the CU's vector-memory pipe set the step time)

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, n = lane & 15;
  const int B = a.B, T = a.T, I = a.I;
  const int b0 = blockIdx.x * kN;
  const bool valid = b0 + n < B;
  const int bn = valid ? b0 + n : B - 1;
  auto hbuf = [&](int l, int p) { return hb16 + (l * 2 + p) * kN * kH; };
  float* stg = reinterpret_cast<float*>(xs + (size_t)T * kN * kXK);

  // ---- prologue: zero the h images (h_{-1} = 0), stage x as bf16 ---------
  for (int e = tid; e < HBF; e += 256) smem[e] = 0.f;
  {
    const int tot = T * kN * kXK;
    for (int e0 = tid; e0 < tot; e0 += 4 * 256) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = min(e0 + r * 256, tot - 1);
        const int t = e / (kN * kXK), rem = e - t * (kN * kXK);
        const int nn = rem / kXK, k = rem - nn * kXK;
        const int bb = min(b0 + nn, B - 1);
        const int src = a.idx ? (int)a.idx[bb] : bb;
        const float x = ldx(a.x, (int64_t)src * a.x_sb + (int64_t)t * a.x_st + min(k, I - 1), a.x_bf16);
        v[r] = k < I ? x : 0.f;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int e = e0 + r * 256;
        if (e < tot) {
          const int t = e / (kN * kXK), rem = e - t * (kN * kXK);
          const int nn = rem / kXK, k = rem - nn * kXK;
          xs[e] = (uint16_t)bfb(v[r]);
          // the deferred-dW kernel's fp32 copy of the (bf16) layer-0 input rows
          if (a.xg_out && k < a.xg_ld && b0 + nn < B)
            a.xg_out[((int64_t)(b0 + nn) * T + t) * a.xg_ld + k] = rbf(v[r]);
        }
      }
    }
  }

  // ---- weights: A fragments of this wave's two M-tiles ----------------------
  // A row i = lane & 15 of M-tile mt: unit 8 (i >> 2) + mt, gate i & 3
  const int ai = lane & 15, ak = lane >> 4;
  // (W_ih of layer 0 as a K = 32 operand: k < 16 the staged x columns, k >= 16
  // zero -- one MFMA shape for the whole accumulate chain)
  u32x4 ax[2], ah0[2], aih1[2], ahh1[2];
  float bias[NL][2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int mt = 2 * w + m;
    const int row = (ai & 3) * kH + 8 * (ai >> 2) + mt;
    {
      const float* p = a.w_ih[0] + (int64_t)row * I;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * ak + j;
        const float x = p[min(k, I - 1)];
        v[j] = k < I ? x : 0.f;
      }
      ax[m] = u32x4{pk(v[0], v[1]), pk(v[2], v[3]), pk(v[4], v[5]), pk(v[6], v[7])};
    }
    ah0[m] = wrow8(a.w_hh[0], kH, row, 8 * ak);
    if constexpr (NL == 2) {
      aih1[m] = wrow8(a.w_ih[1], kH, row, 8 * ak);
      ahh1[m] = wrow8(a.w_hh[1], kH, row, 8 * ak);
    }
    // accumulator rows of this lane: gates 0..3 of unit 8 g + mt
#pragma unroll
    for (int l = 0; l < NL; ++l)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = q * kH + 8 * g + mt;
        bias[l][m][q] = (a.b_ih[l] ? rbf(a.b_ih[l][r]) : 0.f) + (a.b_hh[l] ? rbf(a.b_hh[l][r]) : 0.f);
      }
  }
  __syncthreads();

  float cst[NL][2], hst[NL][2];
#pragma unroll
  for (int l = 0; l < NL; ++l)
#pragma unroll
    for (int m = 0; m < 2; ++m) { cst[l][m] = 0.f; hst[l][m] = 0.f; }

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  // epilogue of layer l's M-tile m at time t (active: commit; the outputs go
  // to the step's staging rows, parity p)
  auto cell = [&](int l, int m, int t, bool act, f32x4 acc, int p) {
    const int mt = 2 * w + m;
    const int u = 8 * g + mt;
    const float ig = sgm(acc[0] + bias[l][m][0]);
    const float fg = sgm(acc[1] + bias[l][m][1]);
    const float gg = tnh(acc[2] + bias[l][m][2]);
    const float og = sgm(acc[3] + bias[l][m][3]);
    const float cn = fmaf(fg, cst[l][m], ig * gg);
    const float h = og * tnh(cn);
    cst[l][m] = act ? cn : cst[l][m];
    hst[l][m] = act ? h : hst[l][m];
    (void)t;
    float* sr = stg + ((p * NL + l) * kN + n) * kSR;
    sr[0 * kH + u] = ig;
    sr[1 * kH + u] = fg;
    sr[2 * kH + u] = gg;
    sr[3 * kH + u] = og;
    sr[4 * kH + u] = cn;
    sr[5 * kH + u] = h;
  };
  // the staged rows of iteration `it` (layer l at t = it - l) to act / hseq:
  // 48 float4 per (layer, sequence) row, 6 per thread
  auto flush = [&](int it, int p) {
#pragma unroll
    for (int j = 0; j < NL * kN * 48 / 256; ++j) {
      const int e = tid + 256 * j;
      const int l = e / (kN * 48), rem = e - l * (kN * 48);
      const int nn = rem / 48, c4 = rem - nn * 48;
      const int t = it - l;
      if (t < 0 || t >= T || b0 + nn >= B) continue;
      const float4 v = *reinterpret_cast<const float4*>(stg + ((p * NL + l) * kN + nn) * kSR + 4 * c4);
      const int64_t row = ((int64_t)l * B + b0 + nn) * T + t;
      float* dst = c4 < 40 ? a.act + row * (5 * kH) + 4 * c4 : a.hseq + row * kH + 4 * (c4 - 40);
      *reinterpret_cast<float4*>(dst) = v;
    }
  };
  auto publish = [&](int l, int t) {  // this lane's two h (units 8g + 2w, + 1) into the step-t image
    uint32_t* dst = reinterpret_cast<uint32_t*>(hbuf(l, t & 1) + n * kH + 8 * g + 2 * w);
    *dst = pk(hst[l][0], hst[l][1]);
  };
  auto bfrag = [&](int l, int t) {  // B operand: h_t of units 8g .. 8g+7, sequence n
    return *reinterpret_cast<const u32x4*>(hbuf(l, t & 1) + n * kH + 8 * g);
  };
  // x_t as the K = 32 B operand: lanes g < 2 hold staged columns 8g .. 8g+7
  const u32x4 zx = {0u, 0u, 0u, 0u};
  auto xfrag = [&](int t) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(xs + (min(t, T - 1) * kN + n) * kXK + 8 * (g & 1));
    return g < 2 ? v : zx;
  };
  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};

  const int iters = T + NL - 1;
  for (int it = 0; it < iters; ++it) {
    const int t0 = it, t1 = it - 1;
    const u32x4 bh0 = bfrag(0, t0 - 1);
#ifdef MB_DEBUG
    if (it == 1 && blockIdx.x == 0 && w == 0 && a.stamps) {  // the step-0 h image as read (probe dump)
      uint32_t* dbg = reinterpret_cast<uint32_t*>(a.stamps) + 256;  // past the stamps of workgroup 0
      for (int j = 0; j < 4; ++j) dbg[lane * 4 + j] = bh0[j];
      for (int j = 0; j < 4; ++j) dbg[256 + lane * 4 + j] = ah0[0][j];
    }
#endif
    const u32x4 bx = xfrag(t0);
    u32x4 bh1;
    if constexpr (NL == 2) bh1 = bfrag(1, t1 - 1);
    f32x4 acc0[2], acc1[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) acc0[m] = mfma32(ah0[m], bh0, mfma32(ax[m], bx, z4));
    if constexpr (NL == 2) {
#pragma unroll
      for (int m = 0; m < 2; ++m) acc1[m] = mfma32(ahh1[m], bh1, mfma32(aih1[m], bh0, z4));
    }
    const int p = it & 1;
#pragma unroll
    for (int m = 0; m < 2; ++m) cell(0, m, t0, t0 < T, acc0[m], p);
    publish(0, t0);
    if constexpr (NL == 2) {
#pragma unroll
      for (int m = 0; m < 2; ++m) cell(1, m, t1, t1 >= 0, acc1[m], p);
      publish(1, t1);
    }
    lds_barrier();
    flush(it, p);
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
  }

  // ---- epilogue: h_n / c_n, the head on the top layer's h_T ---------------
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int u = 8 * g + 2 * w + m;
    if (valid) {
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        if (a.hn) a.hn[((int64_t)l * B + bn) * kH + u] = hst[l][m];
        if (a.cn) a.cn[((int64_t)l * B + bn) * kH + u] = cst[l][m];
      }
    }
    htop[n * kH + u] = hst[NL - 1][m];
  }
  __syncthreads();
  if (a.head_w) {
    const int hu = lane >> 1;
    const bool odd = (lane & 1) != 0;
    for (int s = 0; s < 4; ++s) {
      const int nn = 4 * w + s;
      if (b0 + nn < B) motion_head(a, b0 + nn, htop[nn * kH + hu], hu, odd);
    }
  }
}

// ---------------------------------------------------------------------------
// Backward: 4 waves per layer; wave s of layer l owns gate-row K-step s (units
// 8 s .. 8 s + 7); iteration `it` runs the top layer at t = T-1-it and layer 0
// of a 2-layer stack at t = T-it.
// ---------------------------------------------------------------------------
struct Ops {
  float v[2][6];  // per unit e: i, f, g, o, c_t, c_{t-1}
};

template <int NL>
__global__ void __launch_bounds__(256 * NL) lstm_mb_bwd_kernel(PdrnnLstmSmallBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int PT = kN * kH;                 // one partial tile [16 seq][32 units] fp32
  float* pdh = smem;                          // [2 parity][NL][4 waves] tiles
  float* pdx = smem + 2 * NL * 4 * PT;        // [2 parity][4 waves] tiles (layer 1 -> layer 0)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wg = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l = wg >> 2, s = wg & 3;
  const int g = lane >> 4, n = lane & 15;
  const int B = a.B, T = a.T;
  const int b0 = blockIdx.x * kN;
  const bool valid = b0 + n < B;
  const int bn = valid ? b0 + n : B - 1;
  const int u0 = 8 * s + 2 * g;               // this lane's units u0, u0 + 1
  auto ptile = [&](float* base, int p, int k) { return base + (p * (base == pdh ? NL * 4 : 4) + k) * PT; };

  for (int e = tid; e < (2 * NL * 4 + 2 * 4) * PT; e += 256 * NL) smem[e] = 0.f;
  if (blockIdx.x == 0) {
    float* pad = a.dg_out + (int64_t)NL * B * T * a.dg_st;
    for (int e = tid; e < PDRNN_DW_PAD_ROWS * a.dg_st; e += 256 * NL) pad[e] = 0.f;
  }

  // A fragments: W^T for this wave's K-step.  M-tile mt row i = lane & 15 is
  // input unit 16 mt + i; K element 8 (lane>>4) + j is gate j & 3 of unit
  // 8 s + 2 (lane>>4) + (j >> 2)
  const int ai = lane & 15, ak = lane >> 4;
  u32x4 ahh[2], aih[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    float vh[8], vx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int r = (j & 3) * kH + 8 * s + 2 * ak + (j >> 2);
      vh[j] = a.w_hh[l][(int64_t)r * kH + 16 * mt + ai];
      vx[j] = (l > 0) ? a.w_ih[l][(int64_t)r * kH + 16 * mt + ai] : 0.f;
    }
    ahh[mt] = u32x4{pk(vh[0], vh[1]), pk(vh[2], vh[3]), pk(vh[4], vh[5]), pk(vh[6], vh[7])};
    aih[mt] = u32x4{pk(vx[0], vx[1]), pk(vx[2], vx[3]), pk(vx[4], vx[5]), pk(vx[6], vx[7])};
  }

  const __amdgpu_buffer_rsrc_t r_act = uniform_rsrc(a.act);
  const __amdgpu_buffer_rsrc_t r_dg = uniform_rsrc(a.dg_out);
  const uint32_t rowbase = (uint32_t)((l * B + bn) * T);
  const uint32_t vmask = valid ? 0u : kOOR;
  const bool top = l == NL - 1;
  float dhtop[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) dhtop[e] = top ? a.dhn[(int64_t)bn * kH + u0 + e] : 0.f;

  // step of this wave's layer at iteration it
  auto tstep = [&](int it) { return top ? T - 1 - it : T - it; };
  auto load_ops = [&](int t) {
    const int tc = min(max(t, 0), T - 1);
    const uint32_t ra = (rowbase + (uint32_t)tc) * (5 * kH * 4);
    const uint32_t rp = tc > 0 ? ra - 5 * kH * 4 : ra;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)0);
    Ops o;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const uint32_t u = (uint32_t)(u0 + e);
#pragma unroll
      for (int q = 0; q < 5; ++q) o.v[e][q] = bld(r_act, ra + (q * kH + u) * 4, so);
      o.v[e][5] = bld(r_act, rp + (4 * kH + u) * 4, so);
    }
    return o;
  };

  float dc[2] = {0.f, 0.f};
  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  Ops opA = load_ops(tstep(0));
  __builtin_amdgcn_sched_barrier(0);
  Ops opB = load_ops(tstep(1));
  __builtin_amdgcn_sched_barrier(0);
  __syncthreads();

  const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int iters = T + NL - 1;
  auto body = [&](int it, Ops& op) {
    const int t = tstep(it);
    const bool act = t >= 0 && t < T;
    const int p = it & 1, pp = p ^ 1;
    // dh of this lane's units: the 4 waves' split-K partials of the previous
    // iteration (own layer: dh_rec; layer 0 also layer 1's input gradient)
    float dh[2] = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float2 v = *reinterpret_cast<const float2*>(ptile(pdh, pp, l * 4 + k) + n * kH + u0);
      dh[0] += v.x;
      dh[1] += v.y;
      if (!top) {
        const float2 x = *reinterpret_cast<const float2*>(ptile(pdx, pp, k) + n * kH + u0);
        dh[0] += x.x;
        dh[1] += x.y;
      }
    }
    if (top && it == 0) { dh[0] += dhtop[0]; dh[1] += dhtop[1]; }
    float dz[2][4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float ig = op.v[e][0], fg = op.v[e][1], gg = op.v[e][2], og = op.v[e][3];
      const float cp = t > 0 ? op.v[e][5] : 0.f;
      const float tc = tnh(op.v[e][4]);
      const float dcp = fmaf(dh[e] * og, fmaf(-tc, tc, 1.f), dc[e]);
      dz[e][0] = dcp * gg * fmaf(-ig, ig, ig);
      dz[e][1] = dcp * cp * fmaf(-fg, fg, fg);
      dz[e][2] = dcp * ig * fmaf(-gg, gg, 1.f);
      dz[e][3] = dh[e] * tc * fmaf(-og, og, og);
      dc[e] = act ? dcp * fg : dc[e];
#pragma unroll
      for (int q = 0; q < 4; ++q) dz[e][q] = act ? dz[e][q] : 0.f;
    }
    // the gate gradients over the consumed activation slots (deferred dW)
    {
      const uint32_t ra = (rowbase + (uint32_t)min(max(t, 0), T - 1)) * ((uint32_t)a.dg_st * 4);
      const uint32_t m_ = act ? vmask : kOOR;
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)0);
#pragma unroll
      for (int e = 0; e < 2; ++e)
#pragma unroll
        for (int q = 0; q < 4; ++q) bst(dz[e][q], r_dg, (ra + (q * kH + u0 + e) * 4) | m_, so);
    }
    const u32x4 bdz = {pk(dz[0][0], dz[0][1]), pk(dz[0][2], dz[0][3]), pk(dz[1][0], dz[1][1]), pk(dz[1][2], dz[1][3])};
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const f32x4 d = mfma32(ahh[mt], bdz, z4);
      *reinterpret_cast<f32x4*>(ptile(pdh, p, l * 4 + s) + n * kH + 16 * mt + 4 * g) = d;
      if (l > 0) {
        const f32x4 x = mfma32(aih[mt], bdz, z4);
        *reinterpret_cast<f32x4*>(ptile(pdx, p, s) + n * kH + 16 * mt + 4 * g) = x;
      }
    }
    op = load_ops(tstep(it + 2));
    lds_barrier();
  };
  int it = 0;
  for (; it + 1 < iters; it += 2) {
    body(it, opA);
    body(it + 1, opB);
  }
  if (it < iters) body(it, opA);
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
  }
}

size_t fwd_lds(int NL, int T) {
  return sizeof(float) * ((size_t)NL * 2 * kN * kH / 2 + kN * kH) + sizeof(uint16_t) * (size_t)T * kN * kXK +
         sizeof(float) * (size_t)2 * NL * kN * kSR;
}
size_t bwd_lds(int NL) { return sizeof(float) * (size_t)(2 * NL * 4 + 2 * 4) * kN * kH; }

}  // namespace
}  // namespace pdrnn

using namespace pdrnn;

extern "C" int pdrnn_lstm_mb_ok(int H, int I, int NL, int cell, int T) {
  return (H == kH && I >= 1 && I <= kXK && (NL == 1 || NL == 2) && cell == 0 && T >= 1 &&
          fwd_lds(NL, T) <= 160 * 1024) ? 1 : 0;
}

extern "C" hipError_t pdrnn_lstm_mb_fwd(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  if (!pdrnn_lstm_mb_ok(kH, a->I, a->NL, a->cell, a->T) || a->h0 || a->c0) return hipErrorInvalidValue;
  if (!a->act || !a->hseq || a->B <= 0) return hipErrorInvalidValue;
  if (a->head_w && (a->C > 16 || a->C < 1 || !a->labels || !a->slab || !a->dh_top)) return hipErrorInvalidValue;
  if (a->xg_out && (a->xg_ld < a->I || a->xg_ld > kXK)) return hipErrorInvalidValue;
  const int grid = (a->B + kN - 1) / kN;
  const size_t lds = fwd_lds(a->NL, a->T);
  if (a->NL == 1) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)lstm_mb_fwd_kernel<1>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lstm_mb_fwd_kernel<1>), dim3(grid), dim3(256), lds, st, *a);
  } else {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)lstm_mb_fwd_kernel<2>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((lstm_mb_fwd_kernel<2>), dim3(grid), dim3(256), lds, st, *a);
  }
  return hipGetLastError();
}

extern "C" hipError_t pdrnn_lstm_mb_bwd(const PdrnnLstmSmallBwdArgs* a, hipStream_t st) {
  if (!pdrnn_lstm_mb_ok(kH, a->I, a->NL, a->cell, a->T)) return hipErrorInvalidValue;
  if (a->h0 || a->c0 || a->dout || a->dcn || a->dx || a->dh0 || a->dc0 || !a->dhn || !a->dhn_top_only)
    return hipErrorInvalidValue;  // lean contract only
  if (!a->act || !a->dg_out || a->dg_st < 4 * kH || a->B <= 0) return hipErrorInvalidValue;
  const int grid = (a->B + kN - 1) / kN;
  if (a->NL == 1) hipLaunchKernelGGL((lstm_mb_bwd_kernel<1>), dim3(grid), dim3(256), bwd_lds(1), st, *a);
  else hipLaunchKernelGGL((lstm_mb_bwd_kernel<2>), dim3(grid), dim3(512), bwd_lds(2), st, *a);
  return hipGetLastError();
}
