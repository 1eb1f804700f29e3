// Throughput BPTT for the fused small-H training step (LSTM / GRU), fp32, gfx950.
//
// Same unit-group lane map and wave-pipelined layer schedule as the latency
// kernel in lstm_small.hip (lane (u, j) owns column u of the rows of gate j of
// W_hh / W_ih in VGPRs and accumulates dW for them across the whole launch),
// sized for batches larger than one resident wave of single-sequence
// workgroups (the motion model's B = 1440 on one GPU):
//
//  * NB sequences per workgroup share the register-resident W and dW: the
//    per-(sequence, step) cost is the 64 packed FMAs of the column phase plus
//    the cell math, and a B = 1440 batch finishes in ONE residency round (480
//    workgroups of 3 on 256 CUs x 2) instead of three rounds of 512.
//  * Register budget (256 VGPRs at 2 waves / SIMD): W + dW 128, one gate-
//    gradient slice 32, operand prefetch (5 floats x 2 steps x NB) and per-
//    sequence state.  Every operand stream is ONE workgroup-uniform buffer
//    descriptor per layer (SGPRs) with the sequence and timestep folded into
//    the scalar offset, so NB costs no VGPR / SGPR addresses.
//  * Layer-0 inputs are staged into LDS compactly ([T][I], not zero-padded to
//    H): NB = 3 sequences of the motion shape take 14 KB.
//  * Lean contract only (zero initial state, loss through the top layer's
//    h_T): the fused training step (csrc/bindings.cpp lstm_head_train_step).
//
// Reference behaviour replaced: autograd through torch.nn.LSTM on CPU
// (reference: src/motion/model.py:9,14; loss.backward() in
// src/motion/trainer/base.py:63-70).
#include "pdrnn/api.h"
#include "pdrnn/common.h"

#include <type_traits>

#ifndef PDRNN_TP_CHUNK
#define PDRNN_TP_CHUNK 4
#endif

namespace pdrnn {
namespace {

// steps per DMA chunk of staged operands (even: step parity is compile-time)
constexpr int kTpChunk = PDRNN_TP_CHUNK;

// Operand staging geometry (per layer, per chunk of TC steps), in 16-byte
// units: three stream regions, each padded to whole DMA rounds (64 units per
// wave-instruction x the layer's waves) so that every DMA instruction reads
// ONE stream -- its base pointer is then compile-time, not a per-lane select
// (which the compiler lowers to a lookup table in scratch):
//   act[NB][TC+1][5H/4]  saved activations [i f g o | c]; row r = time t_lo-1+r
//                        (row t-1 supplies c_{t-1})
//   own[NB][TC][H/4]     the layer's own h; row r = time t_lo-1+r (h_{t-1})
//   in [NB][TC][H/4]     layer-below h (layers above 0); row r = time t_lo+r
template <int H, int NB, int TC, bool FIRST>
struct TpStage {
  static constexpr int A4 = 5 * H / 4, H4 = H / 4;
  static constexpr int WPL = 4 * H / 64;                    // waves per layer group
  static constexpr int RND = 64 * WPL;                      // units per DMA round
  static constexpr int pad(int u) { return (u + RND - 1) / RND * RND; }
  static constexpr int ACT_U = NB * (TC + 1) * A4, H_U = NB * TC * H4;
  static constexpr int OWN = pad(ACT_U);                    // region starts (units)
  static constexpr int IN = OWN + pad(H_U);
  static constexpr int UNITS = IN + (FIRST ? 0 : pad(H_U));
  static constexpr int ROUNDS = UNITS / RND;                // DMA instructions per wave
};
template <int H, int NB, int TC>
constexpr int tp_stage_floats(int NL) {
  // layer 0 has no input rows; every other layer has the same geometry
  return 2 * 4 * (TpStage<H, NB, TC, true>::UNITS + (NL - 1) * TpStage<H, NB, TC, false>::UNITS);
}

// One body per layer (NL <= 2).  `layer` is wave-uniform but differs between
// the waves of a workgroup: instantiating each layer's body makes every
// per-step choice and every LDS address offset compile-time -- no uniform
// branches (and the register copies at their joins) inside the recurrence,
// and LDS addresses are one lane base plus instruction offsets.
//
// Per-step operands never pass through VGPRs on their way in: every TC steps
// each layer group DMAs the next chunk of its saved activations / hidden
// states straight into LDS (global_load_lds_dwordx4, double-buffered, waited
// for with one vmcnt(0) a whole chunk later), and the steps read them with
// ds_read at compile-time offsets.  That frees the 2-deep register prefetch
// (5 floats x 2 x NB) which, next to 128 VGPRs of W / dW, is what limits how
// many sequences a workgroup can interleave.
template <int H, int NB, int CELL, int NL, int LAYER>
__device__ __forceinline__ void tp_body(const PdrnnLstmSmallBwdArgs& a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int R = 4 * H;
  constexpr int RS = H;              // rows per lane: lane j of a unit owns gate j's rows
  constexpr int LANES = 4 * H;
  constexpr int RP = R + 16;         // 4-float pad after each gate slice (bank spread)
  constexpr int TC = kTpChunk;
  constexpr bool FIRST = LAYER == 0, TOP = LAYER == NL - 1;
  constexpr int layer = LAYER;
  using SG = TpStage<H, NB, TC, FIRST>;
  const int B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const int lg = tid - layer * LANES;
  const int lane = tid & 63;
  const int wl = __builtin_amdgcn_readfirstlane(lg >> 6);  // wave within the layer group
  const int u = lg >> 2;
  const int j = lg & 3;
  const int Iin = FIRST ? I : H;
  constexpr int lag = 2 * (NL - 1 - layer);

  // LDS: dg[NB][NL][2][RP] | dha[NB][NL][2][H] | stage[2][layers] | xs[NB][T][I]
  float* dg_s = smem;
  float* dha_s = dg_s + NB * NL * 2 * RP;
  float* stage_s = dha_s + NB * NL * 2 * H;
  float* xs = stage_s + tp_stage_floats<H, NB, TC>(NL);
  auto dgbuf = [&](int n, int l, int p) { return dg_s + ((n * NL + l) * 2 + p) * RP; };
  auto dhabuf = [&](int n, int l, int p) { return dha_s + ((n * NL + l) * 2 + p) * H; };
  // this layer's staging region of buffer `buf`
  constexpr int L0U = TpStage<H, NB, TC, true>::UNITS, LU = TpStage<H, NB, TC, false>::UNITS;
  // float offset (into smem) of this layer's staging region of buffer `buf`
  // (integer offsets, not pointers: a pointer carried through the chunk
  // loop loses its LDS address space and the reads become flat loads, which
  // also wait on the in-flight DMAs)
  constexpr int stage_base = NB * NL * 2 * RP + NB * NL * 2 * H;
  auto stage = [&](int buf) {
    return stage_base + 4 * (buf * (L0U + (NL - 1) * LU) + (FIRST ? 0 : L0U + (layer - 1) * LU));
  };

  const int r0 = j * RS;
  const bool ih_live = u < Iin;
  const float xmask = u < I ? 1.f : 0.f;
  float m[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) m[q] = j == q ? 1.f : 0.f;
  pdrnn_f2 whh[RS / 2], wih[RS / 2], dwhh[RS / 2], dwih[RS / 2];
  {
    const float* ph = a.w_hh[layer] + (int64_t)r0 * H + u;
    const float* pi = a.w_ih[layer] + (int64_t)r0 * Iin + min(u, Iin - 1);
#pragma unroll
    for (int rr = 0; rr < RS / 2; ++rr) {
      whh[rr] = pdrnn_f2{ph[(2 * rr) * H], ph[(2 * rr + 1) * H]};
      const float x0 = pi[(int64_t)(2 * rr) * Iin], x1 = pi[(int64_t)(2 * rr + 1) * Iin];
      wih[rr] = ih_live ? pdrnn_f2{x0, x1} : pdrnn_f2{0.f, 0.f};
      dwhh[rr] = pdrnn_f2{0.f, 0.f};
      dwih[rr] = pdrnn_f2{0.f, 0.f};
    }
  }
  float db = 0.f;
  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  const float* act_l = a.act + (int64_t)layer * B * T * 5 * H;
  const float* own_l = a.hseq + (int64_t)layer * B * T * H;
  const float* in_l = a.hseq + (int64_t)(FIRST ? 0 : layer - 1) * B * T * H;
  constexpr int dha_tgt = FIRST ? NL - 1 : layer - 1;  // top layer's dha slots are never read
  const int t_first = T - 1 + lag;
  const int iters = T + 2 * (NL - 1);
  const int nchunks = (iters + TC - 1) / TC;

  for (int b0 = blockIdx.x * NB; b0 < B; b0 += gridDim.x * NB) {
    bool valid[NB];
    float dh[NB], dc[NB], dha_r[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      valid[n] = b0 + n < B;
      dh[n] = TOP ? a.dhn[(int64_t)min(b0 + n, B - 1) * H + u] : 0.f;
      dc[n] = 0.f;
      dha_r[n] = 0.f;
      if (lg < H) {
        dhabuf(n, layer, 0)[lg] = 0.f;
        dhabuf(n, layer, 1)[lg] = 0.f;
      }
    }
    // layer-0 inputs, compact [T][I] per sequence
    for (int n = 0; n < NB; ++n) {
      const int bn = min(b0 + n, B - 1);
      const int64_t src = (int64_t)(a.idx ? (int)a.idx[bn] : bn) * a.x_sb;
      float* dst = xs + (int64_t)n * T * I;
      for (int e = tid; e < T * I; e += blockDim.x) {
        const int t = e / I, k = e - t * I;
        dst[e] = ldx(a.x, src + (int64_t)t * a.x_st + k, a.x_bf16);
      }
    }

    // DMA chunk c (steps it = c*TC .. c*TC+TC-1, times t_lo .. t_lo+TC-1)
    // into staging buffer c & 1.  Times outside [0, T) are clamped: those
    // steps are inactive and their operands masked.
    auto issue = [&](int c) {
      const int t_lo = t_first - (c + 1) * TC + 1;
      float* base = smem + stage(c & 1);
#pragma unroll
      for (int g = 0; g < SG::ROUNDS; ++g) {
        const int grp = g * SG::WPL + wl;
        const int k = grp * 64 + lane;                 // unit within the layer region
        const bool is_act = g * SG::RND < SG::OWN;     // compile-time per round
        const bool is_own = !is_act && g * SG::RND < SG::IN;
        const int kr = k - (is_act ? 0 : (is_own ? SG::OWN : SG::IN));
        const int w4 = is_act ? SG::A4 : SG::H4;
        const int rows = is_act ? TC + 1 : TC;
        const int n = min(kr / (rows * w4), NB - 1);   // padding lanes re-read the last rows
        const int rr = kr - n * rows * w4;
        const int r = min(rr / w4, rows - 1), c4 = rr - (rr / w4) * w4;
        const int64_t seq = min(b0 + n, B - 1);
        const int tt = min(max(t_lo - (is_act || is_own ? 1 : 0) + r, 0), T - 1);
        const float* src = is_act ? act_l + (seq * T + tt) * 5 * H + min(c4, w4 - 1) * 4
                                  : (is_own ? own_l : in_l) + (seq * T + tt) * H + min(c4, w4 - 1) * 4;
        __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(base + grp * 256), 16, 0, 0);
      }
    };
    issue(0);

    // one step; S = it - c*TC (compile-time), P = it & 1
    auto step = [&](int it, int sb, auto sc, auto pc) {
      constexpr int S = decltype(sc)::value;
      constexpr int p = decltype(pc)::value;
      constexpr int ra = TC - S;                  // activation row of time t (row 0 = t_lo - 1)
      constexpr int rh = TC - 1 - S;              // own row holding h_{t-1}; input row of t
      const int t = t_first - it;
      const bool active = t >= 0 && t < T;
      // ---------------- row phase: gate gradients of (u, gate j) ----------
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float* sn = smem + sb + n * (TC + 1) * SG::A4 * 4;    // act rows of sequence n
        const float* so = smem + sb + SG::OWN * 4 + n * TC * H;      // own h rows
        const float aq = sn[ra * SG::A4 * 4 + j * H + u];
        const float ct = sn[ra * SG::A4 * 4 + 4 * H + u];
        const float dht = TOP ? dh[n] : dh[n] + dha_r[n];
        const float ig = quad_bcast(aq, 0), fg = quad_bcast(aq, 1);
        const float gg = quad_bcast(aq, 2), og = quad_bcast(aq, 3);
        // per-lane gate selection by arithmetic with 0/1 lane masks: selects
        // (even of precomputed values) compile into divergent branches over
        // j here, with exec-mask joins inside the recurrence
        const float own = aq;
        float dgv, dcn;
        if constexpr (CELL == 0) {
          // opaque: keeps the read unconditional (the compiler otherwise sinks
          // it into a divergent branch over j around the select below)
          const float cpv = opaque_copy(sn[(ra - 1) * SG::A4 * 4 + 4 * H + u]);
          const float cp = t > 0 ? cpv : 0.f;
          const float tc = tanhf_fast(ct);
          const float dcp = fmaf(dht * og, 1.f - tc * tc, dc[n]);
          // i: dcp gg s'(i)  f: dcp cp s'(f)  g: dcp ig t'(g)  o: dht tc s'(o)
          const float oth = fmaf(m[0], gg, fmaf(m[1], cp, fmaf(m[2], ig, m[3] * tc)));
          const float src = fmaf(m[3], dht - dcp, dcp);
          const float der = fmaf(m[2], 1.f - own, own) - own * own;
          dgv = src * oth * der;
          dcn = dcp * fg;
        } else {  // GRU: ig = r, fg = z, og = n_h, ct = n
          const float hpv = opaque_copy(so[rh * H + u]);
          const float hp = t > 0 ? hpv : 0.f;
          const float nn = ct;
          const float dpn = dht * (1.f - fg) * (1.f - nn * nn);
          // r: dpn n_h s'(r)  z: dht (h - n) s'(z)  n_x: dpn  n_h: dpn r
          const float a0 = fmaf(m[1], dht - dpn, dpn);
          const float a1 = fmaf(m[0], og, fmaf(m[1], hp - nn, fmaf(m[3], ig, m[2])));
          const float a2 = fmaf(m[0] + m[1], own - own * own - 1.f, 1.f);
          dgv = a0 * a1 * a2;
          dcn = dht * fg;  // direct path into dh_{t-1}
        }
        dgv = active ? dgv : 0.f;
        dc[n] = active ? dcn : dc[n];
        dgbuf(n, layer, p)[j * (H + 4) + u] = dgv;
        db += valid[n] ? dgv : 0.f;
      }
      lds_barrier();
      // ---------------- column phase: W^T dg and dW += dg (x) input --------
      const int tcl = min(max(t, 0), T - 1);
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float hpv = smem[sb + SG::OWN * 4 + n * TC * H + rh * H + u];
        const float hprev = t > 0 ? hpv : 0.f;
        float xin;
        if constexpr (FIRST) xin = xmask * xs[(n * T + tcl) * I + min(u, I - 1)];
        else xin = smem[sb + SG::IN * 4 + n * TC * H + rh * H + u];
        const float hw = valid[n] ? hprev : 0.f, xw = valid[n] ? xin : 0.f;
        const float4* g4 = reinterpret_cast<const float4*>(dgbuf(n, layer, p) + j * (H + 4));
        float4 gv[RS / 4];
#pragma unroll
        for (int r4 = 0; r4 < RS / 4; ++r4) gv[r4] = g4[r4];
        pdrnn_f2 sh[2] = {{0.f, 0.f}, {0.f, 0.f}}, sx[2] = {{0.f, 0.f}, {0.f, 0.f}};
        const pdrnn_f2 hb = {hw, opaque_copy(hw)}, xb = {xw, opaque_copy(xw)};
#pragma unroll
        for (int r4 = 0; r4 < RS / 4; ++r4) {
          const float4 g = gv[r4];
          const pdrnn_f2 g01 = {g.x, g.y}, g23 = {g.z, g.w};
          sh[0] = __builtin_elementwise_fma(whh[2 * r4], g01, sh[0]);
          sh[1] = __builtin_elementwise_fma(whh[2 * r4 + 1], g23, sh[1]);
          sx[0] = __builtin_elementwise_fma(wih[2 * r4], g01, sx[0]);
          sx[1] = __builtin_elementwise_fma(wih[2 * r4 + 1], g23, sx[1]);
          dwhh[2 * r4] = __builtin_elementwise_fma(g01, hb, dwhh[2 * r4]);
          dwhh[2 * r4 + 1] = __builtin_elementwise_fma(g23, hb, dwhh[2 * r4 + 1]);
          dwih[2 * r4] = __builtin_elementwise_fma(g01, xb, dwih[2 * r4]);
          dwih[2 * r4 + 1] = __builtin_elementwise_fma(g23, xb, dwih[2 * r4 + 1]);
        }
        // pin the dW updates to this step: they feed nothing until the
        // epilogue, and left free the scheduler sinks them past later steps'
        // barriers (keeping several steps' gate-gradient slices live -> spills)
#pragma unroll
        for (int rr = 0; rr < RS / 2; ++rr) asm volatile("" : "+v"(dwhh[rr]), "+v"(dwih[rr]));
        const pdrnn_f2 shs = sh[0] + sh[1], sxs = sx[0] + sx[1];
        float dhn_ = group_sum<4>(shs.x + shs.y);
        if constexpr (CELL == 1) dhn_ += dc[n];
        dh[n] = active ? dhn_ : dh[n];
        dhabuf(n, dha_tgt, p)[u] = group_sum<4>(sxs.x + sxs.y);  // consumed by the layer below at it+2
      }
      if constexpr (!TOP) {
#pragma unroll
        for (int n = 0; n < NB; ++n) dha_r[n] = dhabuf(n, layer, p ^ 1)[u];
      }
    };

    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    static_assert(TC % 2 == 0, "parity of it is compile-time within a chunk");
    for (int c = 0; c < nchunks; ++c) {
      // chunk c's DMA (issued a whole chunk ago) has landed for this wave; the
      // barrier makes every wave's part visible and retires all reads of the
      // buffer the next DMA overwrites
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      if (c + 1 < nchunks) issue(c + 1);
      const int sb = stage(c & 1);
      const int it0 = c * TC;
      step(it0 + 0, sb, I0{}, I0{});
      step(it0 + 1, sb, I1{}, I1{});
      if constexpr (TC >= 4) {
        step(it0 + 2, sb, std::integral_constant<int, 2>{}, I0{});
        step(it0 + 3, sb, std::integral_constant<int, 3>{}, I1{});
      }
    }
    __syncthreads();  // LDS is reused by the next tile
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 4;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
  }

  float* slab = a.slab + (int64_t)blockIdx.x * a.P;
  {
    float* dst = slab + a.off_whh[layer] + (int64_t)r0 * H + u;
#pragma unroll
    for (int rr = 0; rr < RS / 2; ++rr) {
      dst[(2 * rr) * H] = dwhh[rr].x;
      dst[(2 * rr + 1) * H] = dwhh[rr].y;
    }
  }
  if (ih_live) {
    float* dst = slab + a.off_wih[layer] + (int64_t)r0 * Iin + u;
#pragma unroll
    for (int rr = 0; rr < RS / 2; ++rr) {
      dst[(int64_t)(2 * rr) * Iin] = dwih[rr].x;
      dst[(int64_t)(2 * rr + 1) * Iin] = dwih[rr].y;
    }
  }
  if (a.off_bih[layer] >= 0) slab[a.off_bih[layer] + j * H + u] = db;
  if (a.off_bhh[layer] >= 0) slab[a.off_bhh[layer] + j * H + u] = db;
}

template <int H, int NB, int CELL>
__global__ void __attribute__((amdgpu_flat_work_group_size(64, 256), amdgpu_waves_per_eu(2, 2)))
lstm_small_bwd_tp_kernel(PdrnnLstmSmallBwdArgs a) {
  const int layer = __builtin_amdgcn_readfirstlane((int)threadIdx.x / (4 * H));
  if (a.NL == 1) tp_body<H, NB, CELL, 1, 0>(a);
  else if (layer == 0) tp_body<H, NB, CELL, 2, 0>(a);
  else tp_body<H, NB, CELL, 2, 1>(a);
}

size_t tp_lds(int H, int nb, int NL, int T, int I) {
  size_t stage = 0;
#define PDRNN_TP_STAGE(HH, NN) \
  if (H == HH && nb == NN) stage = tp_stage_floats<HH, NN, kTpChunk>(NL);
  PDRNN_TP_STAGE(16, 2) PDRNN_TP_STAGE(16, 3) PDRNN_TP_STAGE(16, 4)
  PDRNN_TP_STAGE(32, 2) PDRNN_TP_STAGE(32, 3) PDRNN_TP_STAGE(32, 4)
#undef PDRNN_TP_STAGE
  return sizeof(float) * ((size_t)nb * NL * 2 * (4 * H + 16) + (size_t)nb * NL * 2 * H + stage + (size_t)nb * T * I);
}

template <int H, int NB, int CELL>
int tp_resident(int NL, size_t lds) {
  static thread_local int c_dev = -1, c_nl = -1, c_val = 0;
  static thread_local size_t c_lds = 0;
  int per_cu = 0, cus = 0, dev = 0;
  hipGetDevice(&dev);
  if (dev == c_dev && NL == c_nl && lds == c_lds) return c_val;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_small_bwd_tp_kernel<H, NB, CELL>, NL * 4 * H, lds);
  if (per_cu < 1) per_cu = 1;
  if (cus < 1) cus = 1;
  c_dev = dev; c_nl = NL; c_lds = lds; c_val = per_cu * cus;
  return c_val;
}

template <int H, int NB, int CELL>
int tp_grid(int NL, int T, int I, int B) {
  const int cap = tp_resident<H, NB, CELL>(NL, tp_lds(H, NB, NL, T, I));
  const int tiles = (B + NB - 1) / NB;
  return tiles < cap ? tiles : cap;
}

template <int H, int CELL>
int tp_grid_nb(int NL, int T, int I, int B, int nb) {
  switch (nb) {
    case 2: return tp_grid<H, 2, CELL>(NL, T, I, B);
    case 3: return tp_grid<H, 3, CELL>(NL, T, I, B);
    case 4: return tp_grid<H, 4, CELL>(NL, T, I, B);
    default: return -1;
  }
}

template <int H, int NB, int CELL>
hipError_t tp_launch(const PdrnnLstmSmallBwdArgs* a, int grid, hipStream_t st) {
  if (grid <= 0) grid = tp_grid<H, NB, CELL>(a->NL, a->T, a->I, a->B);
  hipLaunchKernelGGL((lstm_small_bwd_tp_kernel<H, NB, CELL>), dim3(grid), dim3(a->NL * 4 * H),
                     tp_lds(H, NB, a->NL, a->T, a->I), st, *a);
  return hipGetLastError();
}

template <int H, int CELL>
hipError_t tp_dispatch(const PdrnnLstmSmallBwdArgs* a, int nb, int grid, hipStream_t st) {
  switch (nb) {
    case 2: return tp_launch<H, 2, CELL>(a, grid, st);
    case 3: return tp_launch<H, 3, CELL>(a, grid, st);
    case 4: return tp_launch<H, 4, CELL>(a, grid, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_lstm_small_bwd_tp_ok(int H, int NL, int T, int I, int B, int nb) {
  if (H != 16 && H != 32) return 0;
  if (nb < 2 || nb > 4 || NL < 1 || NL > 2 || I < 1 || I > H || T < 1) return 0;
  // scalar byte offsets of the per-layer streams stay 32-bit
  if ((uint64_t)B * T * 5 * H * 4 >= (1ull << 31)) return 0;
  if (pdrnn::tp_lds(H, nb, NL, T, I) > 80 * 1024) return 0;
  return 1;
}

int pdrnn_lstm_small_bwd_tp_grid(int H, int NL, int T, int I, int B, int nb, int cell) {
  if (!pdrnn_lstm_small_bwd_tp_ok(H, NL, T, I, B, nb)) return -1;
  if (H == 16) return cell ? pdrnn::tp_grid_nb<16, 1>(NL, T, I, B, nb) : pdrnn::tp_grid_nb<16, 0>(NL, T, I, B, nb);
  return cell ? pdrnn::tp_grid_nb<32, 1>(NL, T, I, B, nb) : pdrnn::tp_grid_nb<32, 0>(NL, T, I, B, nb);
}

hipError_t pdrnn_lstm_small_bwd_tp(const PdrnnLstmSmallBwdArgs* a, int H, int nb, int grid, hipStream_t stream) {
  if (!pdrnn_lstm_small_bwd_tp_ok(H, a->NL, a->T, a->I, a->B, nb) || !a->dhn || !a->dhn_top_only || a->h0 ||
      a->c0 || a->dout || a->dcn || a->dx || a->dh0 || a->dc0)
    return hipErrorInvalidConfiguration;
  if (H == 16) return a->cell ? pdrnn::tp_dispatch<16, 1>(a, nb, grid, stream) : pdrnn::tp_dispatch<16, 0>(a, nb, grid, stream);
  return a->cell ? pdrnn::tp_dispatch<32, 1>(a, nb, grid, stream) : pdrnn::tp_dispatch<32, 0>(a, nb, grid, stream);
}

}  // extern "C"
