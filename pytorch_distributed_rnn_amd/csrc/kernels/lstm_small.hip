// Fused small-hidden LSTM stack, forward and BPTT backward, fp32, gfx950.
//
// Replaces the ATen CPU `_VF.lstm` the reference drives through nn.LSTM
// (reference: src/motion/model.py:9,14; per-step cell math in SURVEY.md §3.5).
//
// Design (MI355X-first, see docs/DESIGN.md):
//  * One workgroup owns NB whole sequences for all T timesteps and all NL
//    layers: the recurrence never leaves the CU, no per-timestep launches.
//  * Layers are wave-pipelined: at iteration `it` layer l processes t = it - l,
//    so the stack costs T + NL - 1 dependent steps instead of NL * T.  One
//    workgroup barrier per iteration; layer hand-offs go through double-
//    buffered LDS vectors.
//  * Forward lane map: a layer group is H*S lanes, lane = (unit u, K-slice s).
//    Each lane keeps ITS rows of [W_ih | W_hh] (4 gates x 2H/S columns) in
//    VGPRs for the whole launch and reads its K-slice of [x_t | h_{t-1}] from
//    LDS with broadcast ds_read_b128.  The S partial dot products of a unit
//    are combined with DPP quad permutes (no LDS), after which every lane of
//    the unit holds all four gates and updates c/h redundantly.
//  * Backward lane map (per layer group of 2H*S2 lanes): a "row" role (lane =
//    gate row r = q*H+u, computes dgates) and a "column" role (lane = column k
//    of [W_ih | W_hh] x row-slice s2) that owns W[r-slice][k] AND accumulates
//    dW[r-slice][k] in registers across all timesteps and all NB sequences
//    (the weight gradient never round-trips through HBM per timestep).  The
//    column role produces dh_{t-1} (recurrent) and d(input) for the layer
//    below with the same FMAs.  Partial per-workgroup dW are written to a slab
//    that a deterministic two-pass reduction sums (pdrnn_slab_reduce).
//  * Layer-0 input is zero-padded to H columns so every layer has K = 2H:
//    layers are load-balanced in the pipeline and there is one code path.
#include "pdrnn/api.h"
#include "pdrnn/common.h"

#include <cstring>

namespace pdrnn {
namespace {

// x sequence preloaded into LDS once (zero-padded to H columns) when it fits:
// layer 0 then reads its input slice straight from LDS every step -- no
// per-step global load on the recurrence's critical path.
constexpr int kXldsBytes = 48 * 1024;

// bf16 models keep fp32 master weights; the kernels use them rounded to bf16
// (round-to-nearest-even, v_cvt_pk_bf16_f32) as they load them
__device__ __forceinline__ float wround(float v, int w_bf16) { return w_bf16 ? (float)(__bf16)v : v; }


// Stage one sequence's inputs x[t][0..I) into the LDS image xs[t][0..H)
// (columns >= I zero): only the I real columns are loaded (not H), 4 loads
// in flight per thread, so the prologue is one memory round trip instead of
// T*H/blockDim dependent ones.
// xg (optional): the staged rows are also written, widened to fp32, to a
// contiguous [T][I] image (the deferred-dW kernel's layer-0 operand: no
// per-row gather or bf16 handling there).
template <int H>
__device__ __forceinline__ void stage_x(float* dst, const float* x, int64_t base, int64_t x_st, int T, int I,
                                        int bf, bool valid, float* xg = nullptr, int xg_ld = 0) {
  const int nthr = blockDim.x;
  for (int e = threadIdx.x; e < T * H; e += nthr) {
    const int k = e % H;
    if (k >= I || !valid) dst[e] = 0.f;
  }
  if (!valid) return;
  const int n = T * I;
  for (int e0 = threadIdx.x; e0 < n; e0 += 4 * nthr) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = min(e0 + r * nthr, n - 1);
      const int t = e / I, k = e - t * I;
      v[r] = ldx(x, base + (int64_t)t * x_st + k, bf);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = e0 + r * nthr;
      if (e < n) {
        const int t = e / I, k = e - t * I;
        dst[t * H + k] = v[r];
        if (xg) xg[t * xg_ld + k] = v[r];
      }
    }
  }
}

template <int H, int NB>
__device__ __forceinline__ void preload_x(float* xs, const PdrnnLstmSmallFwdArgs& a, const int* bsrc,
                                          const bool* valid) {
  for (int n = 0; n < NB; ++n)
    stage_x<H>(xs + (int64_t)n * a.T * H, a.x, (int64_t)bsrc[n] * a.x_sb, a.x_st, a.T, a.I, a.x_bf16, valid[n]);
}

// Fused classifier head + cross-entropy on the top layer's h_T (motion
// training step), shared by the gate-split and K-split forward kernels: both
// leave h_T in the top layer's hidden slot of the LDS operand buffers
// ([NB][NL][2][2H], parity T & 1).  Wave n handles sequence n of the tile.
// Label and head-weight column of this lane, loaded before the recurrence
// (the one-launch step): the epilogue's idx -> label -> logits chain then
// starts from registers instead of two dependent global round trips.
struct HeadPre {
  int64_t lab;
  float w[16];
};
template <int H, int NB>
__device__ __forceinline__ HeadPre head_prefetch(const PdrnnLstmSmallFwdArgs& a, int bbase) {
  HeadPre pre{};
  const int n = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int b = bbase + n;
  if (n < NB && b < a.B) {
    pre.lab = a.labels[a.idx ? a.idx[b] : b];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) pre.w[cc] = (cc < a.C && lane < H) ? a.head_w[cc * H + lane] : 0.f;
  }
  return pre;
}

template <int H, int NB>
__device__ __forceinline__ void fwd_head_epilogue(const PdrnnLstmSmallFwdArgs& a, const float* smem, int bbase,
                                                  const HeadPre* pre = nullptr, float* dh_lds = nullptr) {
  constexpr int K = 2 * H;
  const int NL = a.NL, B = a.B, T = a.T;
  const int tid = threadIdx.x;
  auto vin = [&](int n, int l, int p) -> const float* { return smem + ((n * NL + l) * 2 + p) * K; };
  static_assert(NB <= 4, "one wave per sequence of the tile");
  const int n = tid >> 6;
  const int b = bbase + n;
  if (n < NB && b < B) {
    const int lane = tid & 63;
    const float* hT = vin(n, NL - 1, T & 1) + H;
    const float hv = lane < H ? hT[lane] : 0.f;
    const int64_t lab = pre ? pre->lab : a.labels[a.idx ? a.idx[b] : b];
    const int C = a.C;
    float m = -INFINITY, logit_y = 0.f;
    int amax = 0;
    float lg_c[16];
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      if (cc < C) {
        const float wv = pre ? pre->w[cc] : (lane < H ? a.head_w[cc * H + lane] : 0.f);
        float z = wave_sum(wv * hv) + (a.head_b ? a.head_b[cc] : 0.f);
        lg_c[cc] = z;
        if (z > m) { m = z; amax = cc; }
        if (cc == lab) logit_y = z;
      }
    }
    float se = 0.f;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc)
      if (cc < C) se += expf(lg_c[cc] - m);
    const float lse = m + logf(se);
    const float inv_se = 1.f / se;
    float* srow = a.slab + (int64_t)b * a.slab_P;
    float dh = 0.f;
#pragma unroll
    for (int cc = 0; cc < 16; ++cc) {
      if (cc < C) {
        const float d = (expf(lg_c[cc] - m) * inv_se - (cc == lab ? 1.f : 0.f)) * a.inv_batch;
        if (lane < H) {
          dh = fmaf(pre ? pre->w[cc] : a.head_w[cc * H + lane], d, dh);
          srow[a.head_off_w + cc * H + lane] = d * hv;
        }
        if (lane == 0 && a.head_b) srow[a.head_off_b + cc] = d;
      }
    }
    if (lane < H) {
      a.dh_top[(int64_t)b * H + lane] = dh;
      if (dh_lds) dh_lds[lane] = dh;  // one-launch step: handed to the backward half through LDS
    }
    if (lane == 0) {  // [mean-loss contribution, count, correct] -> column sums are the batch stats
      srow[a.stat_off + 0] = (lse - logit_y) * a.inv_batch;
      srow[a.stat_off + 1] = 1.f;
      srow[a.stat_off + 2] = amax == lab ? 1.f : 0.f;
    }
  }
}

constexpr float kNegLog2eK = -1.4426950408889634f;

// H <= 32: at most 168 VGPRs, three waves per SIMD -- the B = 1440 forward
// (2880 waves on 1024 SIMDs) must stay one residency round (170 VGPRs with
// the packed K loop would drop it to two: 135 -> 184 us)
template <int H, int S, int NB, bool SAVE, bool XLDS, bool HEAD = false>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(H <= 32 ? 3 : 1)))
lstm_small_fwd_kernel(PdrnnLstmSmallFwdArgs a) {
  constexpr int K = 2 * H;
  constexpr int KS = K / S;
  constexpr int LANES = H * S;
  static_assert(KS % 4 == 0 && H % KS == 0, "K slice must be float4 aligned and not straddle");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int NL = a.NL, B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const uint64_t sr_in = (a.stamps && tid == 0) ? stamp_real() : 0;
  const int layer = __builtin_amdgcn_readfirstlane(tid / LANES);
  const int lg = tid - layer * LANES;
  const int u = lg / S;
  const int s = lg % S;
  const int k0 = s * KS;  // first column of this lane's K slice
  const int bbase = blockIdx.x * NB;
  const int Iin = layer == 0 ? I : H;

  // LDS: vin[n][l][p][K] (k < H layer input, k >= H own hidden) | xs[n][T][H]
  float* xs = smem + NB * NL * 2 * K;
  auto vin = [&](int n, int l, int p) -> float* { return smem + ((n * NL + l) * 2 + p) * K; };

  // ---- this lane's rows q*H+u of [W_ih | W_hh], columns k0 .. k0+KS-1 ----
  float w[4][KS];
  float bias[4];
  {
    const bool in_part = k0 < H;
    const float* src = in_part ? a.w_ih[layer] : a.w_hh[layer];
    const int ld = in_part ? Iin : H;
    const int c0 = in_part ? k0 : k0 - H;
    // float4 row loads where the slice is aligned (every h part, the input
    // part of layers >= 1): each lane reads a different row, so every load
    // instruction touches 64 cache lines -- 4x fewer instructions matter at
    // B = 1440, where all workgroups load the weights at once (the prologue
    // was ~27 us with scalar loads)
    const bool vec = (ld % 4) == 0 && (!in_part || Iin == H);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = q * H + u;
      if (vec) {
#pragma unroll
        for (int k4 = 0; k4 < KS / 4; ++k4) {
          const float4 v = *reinterpret_cast<const float4*>(src + r * ld + c0 + 4 * k4);
          w[q][4 * k4 + 0] = wround(v.x, a.w_bf16); w[q][4 * k4 + 1] = wround(v.y, a.w_bf16);
          w[q][4 * k4 + 2] = wround(v.z, a.w_bf16); w[q][4 * k4 + 3] = wround(v.w, a.w_bf16);
        }
      } else {
        // only the live columns are loaded: for the layer-0 input slice
        // (I << KS) the guard is uniform over the slice's lanes, so the
        // zero-padded tail issues no loads at all (128 -> 4 I per lane)
        const int lim = in_part ? Iin : H;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int c = c0 + kk;
          float v = 0.f;
          if (c < lim) v = src[r * ld + c];
          w[q][kk] = wround(v, a.w_bf16);
        }
      }
      bias[q] = (a.b_ih[layer] ? wround(a.b_ih[layer][r], a.w_bf16) : 0.f) +
                (a.b_hh[layer] ? wround(a.b_hh[layer][r], a.w_bf16) : 0.f);
    }
    if constexpr (S == 2) {
      // pre-scaled rows (as in the gate-split map): the pre-activation comes
      // out as -log2(e) z (x2 for the g gate), so sigmoid = 1 / (1 + 2^acc)
      // and tanh(g) = 2 sigmoid(2g) - 1 with no scaling in the recurrence
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float sc = kNegLog2eK * (q == 2 ? 2.f : 1.f);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) w[q][kk] *= sc;
        bias[q] *= sc;
      }
    }
  }

  pdrnn_f2 w2[4][KS / 2];  // k pairs of the slice (packed FMA operands)
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < KS / 2; ++j) w2[q][j] = pdrnn_f2{w[q][2 * j], w[q][2 * j + 1]};

  int bsrc[NB];
  bool valid[NB];
  float c[NB], hl[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    valid[n] = b < B;
    bsrc[n] = valid[n] ? (a.idx ? (int)a.idx[b] : b) : 0;
    const int bc = min(b, B - 1);
    const float h_init = (a.h0 && valid[n]) ? a.h0[((int64_t)layer * B + bc) * H + u] : 0.f;
    c[n] = (a.c0 && valid[n]) ? a.c0[((int64_t)layer * B + bc) * H + u] : 0.f;
    hl[n] = h_init;
    if (s == 0) vin(n, layer, 0)[H + u] = h_init;
    if (!XLDS && layer == 0 && lg < H)
      vin(n, 0, 0)[lg] = (valid[n] && lg < I) ? a.x[bsrc[n] * a.x_sb + lg] : 0.f;
  }
  if constexpr (XLDS) preload_x<H, NB>(xs, a, bsrc, valid);
  __syncthreads();

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }
  const int iters = T + NL - 1;
  for (int it = 0; it < iters; ++it) {
    prio_by_progress(it, iters, a.prio);
    const int t = it - layer;
    if (t >= 0 && t < T) {
      const int p = t & 1;
      float xnext[NB];
      if (!XLDS && layer == 0 && lg < H) {
        const int tn = min(t + 1, T - 1);
        const int kx = min(lg, I - 1);
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          const float v = a.x[bsrc[n] * a.x_sb + (int64_t)tn * a.x_st + kx];  // unconditional load
          xnext[n] = (t + 1 < T && valid[n] && lg < I) ? v : 0.f;
        }
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float* src = vin(n, layer, p) + k0;
        if (XLDS && layer == 0 && k0 < H) src = xs + ((int64_t)n * T + t) * H + k0;
        const float4* v4 = reinterpret_cast<const float4*>(src);
        // packed fp32 FMAs over k pairs (v_pk_fma_f32: 2 MACs per lane and
        // instruction, 64 instead of 128 per step), halves summed at the end
        pdrnn_f2 acc2[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
#pragma unroll
        for (int k4 = 0; k4 < KS / 4; ++k4) {
          const float4 v = v4[k4];
          const pdrnn_f2 vlo = {v.x, v.y}, vhi = {v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc2[q] = __builtin_elementwise_fma(w2[q][2 * k4], vlo, acc2[q]);
            acc2[q] = __builtin_elementwise_fma(w2[q][2 * k4 + 1], vhi, acc2[q]);
          }
        }
        float acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = group_sum<S>(acc2[q].x + acc2[q].y) + bias[q];
        if constexpr (S == 2 && NB == 1 && SAVE) {
          // the unit's two lanes split the activations (lane 0: i, g; lane
          // 1: f, o; one DPP swap exchanges them) and the stores: every lane
          // writes one LDS slot and three global words, no branches
          const float z0 = s == 0 ? acc[0] : acc[1];
          const float z1 = s == 0 ? acc[2] : acc[3];
          const float a0 = fast_rcp(1.f + __builtin_amdgcn_exp2f(z0));               // i | f
          const float s1 = fast_rcp(1.f + __builtin_amdgcn_exp2f(z1));
          const float a1 = s == 0 ? fmaf(s1, 2.f, -1.f) : s1;                         // g | o
          const float b0 = dpp_swap1(a0), b1 = dpp_swap1(a1);
          const float ig = s == 0 ? a0 : b0, fg = s == 0 ? b0 : a0;
          const float gg = s == 0 ? a1 : b1, og = s == 0 ? b1 : a1;
          const float cn = fmaf(fg, c[n], ig * gg);
          const float th = fmaf(fast_rcp(1.f + __builtin_amdgcn_exp2f(cn * (2.f * kNegLog2eK))), 2.f, -1.f);
          const float h = og * th;
          c[n] = cn;
          hl[n] = h;
          // lane 0: own-h slot of the next step; lane 1: the next layer's
          // input slot (top layer: its own slot again, same value)
          float* hslot = (s == 0 || layer == NL - 1) ? vin(n, layer, p ^ 1) + H + u : vin(n, layer + 1, p) + u;
          *hslot = h;
          const int64_t row = ((int64_t)layer * B + bbase + n) * T + t;
          float* act = a.act + row * 5 * H + u;
          act[(s == 0 ? 0 : 1) * H] = s == 0 ? ig : fg;
          act[(s == 0 ? 2 : 3) * H] = s == 0 ? gg : og;
          float* w3 = s == 0 ? act + 4 * H : a.hseq + row * H + u;
          *w3 = s == 0 ? cn : h;
          continue;
        }
        const float ig = sigmoidf_fast(acc[0]);
        const float fg = sigmoidf_fast(acc[1]);
        const float gg = tanhf_fast(acc[2]);
        const float og = sigmoidf_fast(acc[3]);
        const float cn = fmaf(fg, c[n], ig * gg);
        const float h = og * tanhf_fast(cn);
        c[n] = cn;
        hl[n] = h;
        if (s == 0) vin(n, layer, p ^ 1)[H + u] = h;
        if (layer < NL - 1 && s == (S > 1 ? 1 : 0)) vin(n, layer + 1, p)[u] = h;
        if (valid[n]) {
          const int b = bbase + n;
          if constexpr (SAVE) {
            const int64_t row = ((int64_t)layer * B + b) * T + t;
            if (s == 0) a.hseq[row * H + u] = h;
            float* act = a.act + row * 5 * H;
            const float items[5] = {ig, fg, gg, og, cn};
#pragma unroll
            for (int item = 0; item < 5; ++item)
              if (item % S == s) act[item * H + u] = items[item];
          } else {
            if (a.out && layer == NL - 1 && s == 0) a.out[b * a.o_sb + (int64_t)t * a.o_st + u] = h;
          }
        }
      }
      if (!XLDS && layer == 0 && lg < H) {
#pragma unroll
        for (int n = 0; n < NB; ++n) vin(n, 0, p ^ 1)[lg] = xnext[n];
      }
    }
    lds_barrier();
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
  }

#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    if (valid[n] && s == 0) {
      a.hn[((int64_t)layer * B + b) * H + u] = hl[n];
      a.cn[((int64_t)layer * B + b) * H + u] = c[n];
    }
  }
  if constexpr (HEAD) fwd_head_epilogue<H, NB>(a, smem, bbase);
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[4] = sr_in; st[5] = stamp_real(); st[6] = stamp_cu();
  }
  // the second wave's SIMD (bit 32 marks the slot as written)
  if (a.stamps && tid == 64) a.stamps[(uint64_t)blockIdx.x * 8 + 7] = stamp_cu() | (1ull << 32);
}

// ---------------------------------------------------------------------------
// Forward, gate-split lane map (default): a layer group is 4H lanes, lane =
// (unit u, gate q) with the 4 gates of a unit in one DPP quad.  Each lane owns
// ONE full row of [W_ih | W_hh] (pre-scaled by -log2(e), and by 2 for the g
// gate so tanh(x) = 2*sigmoid(2x) - 1), computes its dot product with packed
// fp32 FMAs (v_pk_fma_f32, 2 MACs per instruction), applies ONE transcendental
// activation, and the quad exchanges the four activated gates with DPP quad
// broadcasts.  Compared with the K-split map this removes the cross-lane
// partial-sum tree and three of the four activations from every lane's
// per-timestep dependency chain (the recurrence is latency-bound: one wave per
// SIMD at motion batch sizes).
// ---------------------------------------------------------------------------
constexpr float kNegLog2e = -1.4426950408889634f;

// CELL 1 = GRU on the same lane map: the quad's four rows are [r | z | n_x |
// n_h] (n_x = W_in x + b_in and n_h = W_hn h + b_hn kept linear), packed by the
// host as a 4-block stack with zero blocks (W_ih: [W_ir; W_iz; W_in; 0], W_hh:
// [W_hr; W_hz; 0; W_hn]); n = tanh(n_x + r n_h), h = n + z (h_prev - n).  The
// saved activation slots hold r, z, n_x, n_h and n (in the cell-state slot).
template <int H, int NB, bool SAVE, bool XLDS, bool HEAD, int CELL = 0>
// xs_off >= 0: x is staged at smem + xs_off (the one-launch step puts it
// where its backward half expects it, so the backward does not stage it again)
__device__ __forceinline__ void lstm_small_fwd_gs_body(const PdrnnLstmSmallFwdArgs& a, int xs_off = -1,
                                                       bool head_pre = false, float* dh_lds = nullptr) {
  constexpr int K = 2 * H;
  constexpr int LANES = 4 * H;
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int NL = a.NL, B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const uint64_t sr_in = (a.stamps && tid == 0) ? stamp_real() : 0;
  const int layer = __builtin_amdgcn_readfirstlane(tid / LANES);
  const int lg = tid - layer * LANES;
  const int u = lg >> 2;
  const int q = lg & 3;
  const int r = q * H + u;
  const int bbase = blockIdx.x * NB;
  const int Iin = layer == 0 ? I : H;

  float* xs = smem + (xs_off >= 0 ? xs_off : NB * NL * 2 * K);
  auto vin = [&](int n, int l, int p) -> float* { return smem + ((n * NL + l) * 2 + p) * K; };
  HeadPre hpre{};
  if constexpr (HEAD) {
    if (head_pre) hpre = head_prefetch<H, NB>(a, bbase);
  }

  // activation: sigma(z) with z pre-scaled, then a = sigma * am + ab
  // (GRU n_x / n_h rows stay linear: unscaled weights, activation skipped)
  const bool lin = CELL == 1 && q >= 2;
  const float gsc = (CELL == 0 && q == 2) ? 2.f : 1.f;
  const float am = gsc;
  const float ab = (CELL == 0 && q == 2) ? -1.f : 0.f;
  const float wsc = lin ? 1.f : kNegLog2e * gsc;

  pdrnn_f2 w2[K / 2];
  float bias;
  {
    const float* wih = a.w_ih[layer] + (int64_t)r * Iin;
    const float* whh = a.w_hh[layer] + (int64_t)r * H;
#pragma unroll
    for (int kk = 0; kk < K / 2; ++kk) {
      float v0, v1;
      const int k = 2 * kk;
      if (k < H) {  // compile-time per unrolled kk
        const float t0 = wih[min(k, Iin - 1)], t1 = wih[min(k + 1, Iin - 1)];
        v0 = k < Iin ? t0 : 0.f;
        v1 = k + 1 < Iin ? t1 : 0.f;
      } else {
        v0 = whh[k - H];
        v1 = whh[k + 1 - H];
      }
      w2[kk] = pdrnn_f2{wround(v0, a.w_bf16) * wsc, wround(v1, a.w_bf16) * wsc};
    }
    bias = ((a.b_ih[layer] ? wround(a.b_ih[layer][r], a.w_bf16) : 0.f) +
            (a.b_hh[layer] ? wround(a.b_hh[layer][r], a.w_bf16) : 0.f)) * wsc;
  }

  int bsrc[NB];
  bool valid[NB];
  float c[NB], hl[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    valid[n] = b < B;
    bsrc[n] = valid[n] ? (a.idx ? (int)a.idx[b] : b) : 0;
    const int bc = min(b, B - 1);
    const float h_init = (a.h0 && valid[n]) ? a.h0[((int64_t)layer * B + bc) * H + u] : 0.f;
    c[n] = (a.c0 && valid[n]) ? a.c0[((int64_t)layer * B + bc) * H + u] : 0.f;
    hl[n] = h_init;
    if (q == 0) vin(n, layer, 0)[H + u] = h_init;
    if (!XLDS && layer == 0 && lg < H)
      vin(n, 0, 0)[lg] = (valid[n] && lg < I) ? a.x[bsrc[n] * a.x_sb + lg] : 0.f;
  }
  if constexpr (XLDS) preload_x<H, NB>(xs, a, bsrc, valid);
  __syncthreads();

  // per-lane output streams (advanced by one timestep per active iteration)
  // lane q writes act item q (i,f,g,o); q==0 also writes c_t, q==1 writes h_t
  float* out1[NB];
  float* out2[NB];
  int64_t step1 = 0, step2 = 0;
  if constexpr (SAVE) {
    step1 = 5 * H;
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const int bc = min(bbase + n, B - 1);
      const int64_t row0 = ((int64_t)layer * B + bc) * T;
      out1[n] = a.act + row0 * 5 * H + q * H + u;
      out2[n] = q == 0 ? a.act + row0 * 5 * H + 4 * H + u : a.hseq + row0 * H + u;
    }
    step2 = q == 0 ? 5 * H : H;
  } else {
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      out1[n] = a.out ? a.out + (int64_t)min(bbase + n, B - 1) * a.o_sb + u : nullptr;
      out2[n] = nullptr;
    }
    step1 = a.o_st;
  }
  const bool write2 = SAVE && q < 2;
  const bool write1 = SAVE || (a.out != nullptr && layer == NL - 1 && q == 0);

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }
  const int iters = T + NL - 1;
  for (int it = 0; it < iters; ++it) {
    prio_by_progress(it, iters, a.prio);
    const int t = it - layer;
    if (t >= 0 && t < T) {
      const int p = t & 1;
      float xnext[NB];
      if (!XLDS && layer == 0 && lg < H) {
        const int tn = min(t + 1, T - 1);
        const int kx = min(lg, I - 1);
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          const float v = a.x[bsrc[n] * a.x_sb + (int64_t)tn * a.x_st + kx];
          xnext[n] = (t + 1 < T && valid[n] && lg < I) ? v : 0.f;
        }
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float* src_in = vin(n, layer, p);
        if (XLDS && layer == 0) src_in = xs + ((int64_t)n * T + t) * H;
        const float* src_h = vin(n, layer, p) + H;
        pdrnn_f2 acc[4] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};
        // the whole [x_t; h_{t-1}] operand vector in flight at once (one LDS
        // latency per step; left to itself the scheduler keeps 2-3 reads in
        // flight to save VGPRs and exposes the latency ~6 times per step)
        float4 vin4[K / 4];
#pragma unroll
        for (int k4 = 0; k4 < K / 4; ++k4)
          vin4[k4] = (4 * k4 < H) ? reinterpret_cast<const float4*>(src_in)[k4]
                                  : reinterpret_cast<const float4*>(src_h)[k4 - H / 4];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k4 = 0; k4 < K / 4; ++k4) {
          const float4 v = vin4[k4];
          acc[(2 * k4) & 3] = __builtin_elementwise_fma(w2[2 * k4], pdrnn_f2{v.x, v.y}, acc[(2 * k4) & 3]);
          acc[(2 * k4 + 1) & 3] =
              __builtin_elementwise_fma(w2[2 * k4 + 1], pdrnn_f2{v.z, v.w}, acc[(2 * k4 + 1) & 3]);
        }
        const pdrnn_f2 s2 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        const float z = (s2.x + s2.y) + bias;  // = -log2(e) * gsc * preactivation
        const float sg = fast_rcp(1.f + __builtin_amdgcn_exp2f(z));
        const float act = lin ? z : fmaf(sg, am, ab);  // sigmoid, or tanh for the g gate
        const float ig = quad_bcast(act, 0);
        const float fg = quad_bcast(act, 1);
        const float gg = quad_bcast(act, 2);
        const float og = quad_bcast(act, 3);
        float cn, h;
        if constexpr (CELL == 0) {
          cn = fmaf(fg, c[n], ig * gg);
          const float th = fmaf(fast_rcp(1.f + __builtin_amdgcn_exp2f(cn * (2.f * kNegLog2e))), 2.f, -1.f);
          h = og * th;
        } else {  // GRU: ig = r, fg = z, gg = n_x, og = n_h; cn carries n
          const float pre = fmaf(ig, og, gg);
          cn = fmaf(fast_rcp(1.f + __builtin_amdgcn_exp2f(pre * (2.f * kNegLog2e))), 2.f, -1.f);
          h = fmaf(fg, hl[n] - cn, cn);
        }
        c[n] = cn;
        hl[n] = h;
        if (q == 0) vin(n, layer, p ^ 1)[H + u] = h;
        if (q == 1 && layer < NL - 1) vin(n, layer + 1, p)[u] = h;
        if (valid[n]) {
          if (write1) out1[n][(int64_t)t * step1] = SAVE ? act : h;
          if (write2) out2[n][(int64_t)t * step2] = q == 0 ? cn : h;
        }
      }
      if (!XLDS && layer == 0 && lg < H) {
#pragma unroll
        for (int n = 0; n < NB; ++n) vin(n, 0, p ^ 1)[lg] = xnext[n];
      }
    }
    lds_barrier();
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
  }
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    if (valid[n] && q == 0) {
      a.hn[((int64_t)layer * B + b) * H + u] = hl[n];
      if (CELL == 0) a.cn[((int64_t)layer * B + b) * H + u] = c[n];
    }
  }
  if constexpr (HEAD) fwd_head_epilogue<H, NB>(a, smem, bbase, head_pre ? &hpre : nullptr, dh_lds);
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[4] = sr_in; st[5] = stamp_real(); st[6] = stamp_cu();
  }
}

template <int H, int NB, bool SAVE, bool XLDS, bool HEAD, int CELL = 0>
__global__ void __launch_bounds__(512) lstm_small_fwd_gs_kernel(PdrnnLstmSmallFwdArgs a) {
  lstm_small_fwd_gs_body<H, NB, SAVE, XLDS, HEAD, CELL>(a);
}

template <int H, int S2, int NB, bool XLDS>
__global__ void __launch_bounds__(512) lstm_small_bwd_kernel(PdrnnLstmSmallBwdArgs a) {
  constexpr int R = 4 * H;        // gate rows
  constexpr int K = 2 * H;        // columns of [W_ih | W_hh] (input padded to H)
  constexpr int RS = R / S2;      // rows per column lane
  constexpr int G = K * S2;       // lanes per layer group
  constexpr int CH = 4;           // float4 chunks per LDS read burst (bounds VGPRs)
  static_assert(G >= R, "S2 must be >= 2");
  static_assert(RS % (4 * CH) == 0, "row slice must be a multiple of the chunk");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int NL = a.NL, B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const int layer = __builtin_amdgcn_readfirstlane(tid / G);
  const int lg = tid - layer * G;
  const int bbase = blockIdx.x * NB;
  const int Iin = layer == 0 ? I : H;

  // LDS carve: dg[NB][NL][R] | dhrec[NB][NL][H] | dha[NB][NL][H] | xs[NB][T][H]
  float* dg_s = smem;
  float* dhrec_s = dg_s + NB * NL * R;
  float* dha_s = dhrec_s + NB * NL * H;
  float* xs = dha_s + NB * NL * H;
  auto dg = [&](int n, int l) { return dg_s + (n * NL + l) * R; };
  auto dhrec = [&](int n, int l) { return dhrec_s + (n * NL + l) * H; };
  auto dha = [&](int n, int l) { return dha_s + (n * NL + l) * H; };

  // Row role (lanes < 4H): gate row r = q*H + u.
  const bool is_row = lg < R;
  const int q = lg / H;
  const int u = lg % H;
  // Column role: column k of [W_ih | W_hh], row slice s2.
  const int k = lg / S2;
  const int s2 = lg % S2;

  // This lane's column: rows s2*RS .. s2*RS+RS-1 at a fixed stride
  // (branch-free addressing; zero-padded input columns k >= I).
  const bool col_in = k < H;
  const bool col_live = !col_in || k < Iin;
  const int64_t col_stride = col_in ? Iin : H;
  const int64_t col_off = col_in ? (int64_t)s2 * RS * Iin + k : (int64_t)s2 * RS * H + (k - H);
  float W[RS], dW[RS];
  {
    const float* base = (col_in ? a.w_ih[layer] : a.w_hh[layer]) + (col_live ? col_off : 0);
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const float v = base[j * col_stride];
      W[j] = col_live ? wround(v, a.w_bf16) : 0.f;
      dW[j] = 0.f;
    }
  }
  float db = 0.f;
  float dc[NB];
  int bsrc[NB];
  bool valid[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    valid[n] = b < B;
    bsrc[n] = valid[n] ? (a.idx ? (int)a.idx[b] : b) : 0;
    const int bc = min(b, B - 1);
    dc[n] = (is_row && a.dcn && valid[n]) ? a.dcn[((int64_t)layer * B + bc) * H + u] : 0.f;
    if (lg < H) {
      dhrec(n, layer)[lg] = (a.dhn && valid[n]) ? a.dhn[((int64_t)layer * B + bc) * H + lg] : 0.f;
      dha(n, layer)[lg] = 0.f;
    }
  }
  if constexpr (XLDS) {
    for (int n = 0; n < NB; ++n) {
      float* dst = xs + (int64_t)n * T * H;
      const int64_t base = (int64_t)bsrc[n] * a.x_sb;
      for (int e = tid; e < T * H; e += blockDim.x) {
        const int t = e / H, kk = e - t * H;
        const float v = ldx(a.x, base + (int64_t)t * a.x_st + min(kk, I - 1), a.x_bf16);
        dst[e] = (valid[n] && kk < I) ? v : 0.f;
      }
    }
  }

  // ---- per-timestep operands, prefetched TWO steps ahead (ping-pong sets) --
  // Loads are unconditional on clamped, always-valid addresses and masked
  // afterwards: no control flow around them and no register copies between
  // iterations, so the compiler's waitcnt tracking keeps them in flight
  // across both barriers of the step in between.
  // Raw values only: masking happens at the point of use (a select on a
  // freshly loaded register would force the wait right at the load).
  struct RowOps { float i, f, g, o, c, cp, dout; };
  const bool top = layer == NL - 1;
  auto load_row = [&](int t, int n) {
    const int b = min(bbase + n, B - 1);
    const int tc = min(max(t, 0), T - 1);
    const float* act = a.act + (((int64_t)layer * B + b) * T + tc) * 5 * H + u;
    RowOps r;
    r.i = act[0 * H]; r.f = act[1 * H]; r.g = act[2 * H]; r.o = act[3 * H]; r.c = act[4 * H];
    const float* cpp = tc > 0 ? act - H : (a.c0 ? a.c0 + ((int64_t)layer * B + b) * H + u : act);
    r.cp = *cpp;
    const float* dp = (top && a.dout) ? a.dout + b * a.d_sb + (int64_t)tc * a.d_st + u : act;
    r.dout = *dp;
    return r;
  };
  // global part of the column input (everything except layer-0 x under XLDS)
  auto load_in = [&](int t, int n) -> float {
    const int b = min(bbase + n, B - 1);
    const int tc = min(max(t, 0), T - 1);
    const float* p;
    if (k < H) {
      const float* px = a.x + bsrc[n] * a.x_sb + (int64_t)tc * a.x_st + min(k, I - 1);
      const float* ph = a.hseq + (((int64_t)(layer > 0 ? layer - 1 : 0) * B + b) * T + tc) * H + k;
      p = layer == 0 ? px : ph;
    } else {
      const int kh = k - H;
      const float* ph = a.hseq + (((int64_t)layer * B + b) * T + max(tc - 1, 0)) * H + kh;
      const float* p0 = a.h0 ? a.h0 + ((int64_t)layer * B + b) * H + kh : ph;
      p = tc > 0 ? ph : p0;
    }
    return *p;
  };
  // masks, recomputed where the values are consumed
  auto in_live = [&](int t, int n) -> bool {
    if (!valid[n] || t < 0 || t >= T) return false;
    if (k < H) return layer > 0 || k < I;
    return t > 0 || a.h0 != nullptr;
  };
  const bool in_from_lds = XLDS && layer == 0 && k < H;

  const int t_first = T - 1 + (NL - 1 - layer);  // this layer's t at it = 0
  RowOps ropA[NB], ropB[NB];
  float inA[NB], inB[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    ropA[n] = load_row(t_first, n);
    inA[n] = load_in(t_first, n);
    ropB[n] = load_row(t_first - 1, n);
    inB[n] = load_in(t_first - 1, n);
  }
  __syncthreads();

  auto step = [&](int it, RowOps (&rop)[NB], float (&inp)[NB]) {
    const int t = t_first - it;
    const bool active = t >= 0 && t < T;
    // ---------------- row phase: dgates ----------------
    if (active && is_row) {
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const RowOps& r = rop[n];
        const float cp = (t > 0 || a.c0) ? r.cp : 0.f;
        float dh = dhrec(n, layer)[u] + ((top && a.dout) ? r.dout : 0.f);
        if (layer < NL - 1) dh += dha(n, layer)[u];
        const float tc = tanhf_fast(r.c);
        const float dcp = fmaf(dh * r.o, 1.f - tc * tc, dc[n]);
        const float d_i = dcp * r.g * r.i * (1.f - r.i);
        const float d_f = dcp * cp * r.f * (1.f - r.f);
        const float d_g = dcp * r.i * (1.f - r.g * r.g);
        const float d_o = dh * tc * r.o * (1.f - r.o);
        float dgv = q == 0 ? d_i : (q == 1 ? d_f : (q == 2 ? d_g : d_o));
        if (!valid[n]) dgv = 0.f;
        dc[n] = dcp * r.f;
        dg(n, layer)[lg] = dgv;
        db += dgv;
      }
    }
    // refill this set for step t-2 (consumed two iterations from now)
#pragma unroll
    for (int n = 0; n < NB; ++n) rop[n] = load_row(t - 2, n);
    lds_barrier();
    // ---------------- column phase: dh_{t-1}, d(input), dW ----------------
    if (active) {
      float in_v[NB];
#pragma unroll
      for (int n = 0; n < NB; ++n)
        in_v[n] = in_from_lds ? xs[((int64_t)n * T + t) * H + k] : (in_live(t, n) ? inp[n] : 0.f);
      float ds[NB][4];  // 4 independent chains per sequence (FMA latency)
#pragma unroll
      for (int n = 0; n < NB; ++n) ds[n][0] = ds[n][1] = ds[n][2] = ds[n][3] = 0.f;
#pragma unroll
      for (int c0 = 0; c0 < RS / 4; c0 += CH) {
        float4 g[NB][CH];
#pragma unroll
        for (int n = 0; n < NB; ++n) {
          const float4* g4 = reinterpret_cast<const float4*>(dg(n, layer) + s2 * RS);
#pragma unroll
          for (int cc = 0; cc < CH; ++cc) g[n][cc] = g4[c0 + cc];
        }
#pragma unroll
        for (int cc = 0; cc < CH; ++cc) {
          const int j = 4 * (c0 + cc);
#pragma unroll
          for (int n = 0; n < NB; ++n) {
            ds[n][0] = fmaf(W[j + 0], g[n][cc].x, ds[n][0]);
            ds[n][1] = fmaf(W[j + 1], g[n][cc].y, ds[n][1]);
            ds[n][2] = fmaf(W[j + 2], g[n][cc].z, ds[n][2]);
            ds[n][3] = fmaf(W[j + 3], g[n][cc].w, ds[n][3]);
            dW[j + 0] = fmaf(g[n][cc].x, in_v[n], dW[j + 0]);
            dW[j + 1] = fmaf(g[n][cc].y, in_v[n], dW[j + 1]);
            dW[j + 2] = fmaf(g[n][cc].z, in_v[n], dW[j + 2]);
            dW[j + 3] = fmaf(g[n][cc].w, in_v[n], dW[j + 3]);
          }
        }
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float tot = group_sum<S2>((ds[n][0] + ds[n][1]) + (ds[n][2] + ds[n][3]));
        if (s2 == 0) {
          if (k >= H) {
            dhrec(n, layer)[k - H] = tot;
          } else if (layer > 0) {
            dha(n, layer - 1)[k] = tot;
          } else if (a.dx && valid[n] && k < I) {
            a.dx[(bbase + n) * a.dx_sb + (int64_t)t * a.dx_st + k] = tot;
          }
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NB; ++n) inp[n] = in_from_lds ? 0.f : load_in(t - 2, n);
    lds_barrier();
  };

  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }
  const int iters = T + NL - 1;
  int it = 0;
  for (; it + 1 < iters; it += 2) {
    prio_by_progress(it / 2, iters / 2, a.prio);
    step(it, ropA, inA);
    step(it + 1, ropB, inB);
  }
  if (it < iters) step(it, ropA, inA);
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
  }

  // ---------------- epilogue: initial-state grads + partial dW slab --------
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    if (!valid[n]) continue;
    if (a.dh0 && lg < H) a.dh0[((int64_t)layer * B + b) * H + lg] = dhrec(n, layer)[lg];
    if (a.dc0 && is_row && q == 0) a.dc0[((int64_t)layer * B + b) * H + u] = dc[n];
  }
  float* slab = a.slab + (int64_t)blockIdx.x * a.P;
  if (col_live) {
    float* dst = slab + (col_in ? a.off_wih[layer] : a.off_whh[layer]) + col_off;
#pragma unroll
    for (int j = 0; j < RS; ++j) dst[j * col_stride] = dW[j];
  }
  if (is_row) {
    if (a.off_bih[layer] >= 0) slab[a.off_bih[layer] + lg] = db;
    if (a.off_bhh[layer] >= 0) slab[a.off_bhh[layer] + lg] = db;
  }
}

// ---------------------------------------------------------------------------
// Backward, unit-group lane map (default): a layer group is H*L lanes, lane =
// (unit u, j) with the L lanes of a unit adjacent.  Lane j owns the row slice
// [j*RS, (j+1)*RS) (RS = 4H/L) of COLUMN u of both W_hh and W_ih, and the
// matching dW accumulators.  Per timestep:
//   row phase : lanes j<4 compute dgate_j[u] (the quad exchanges the saved
//               activations with DPP), publish it to LDS (parity buffer);
//   barrier   : the only one of the step;
//   col phase : every lane reads its RS dgates, forms partial
//               dh_{t-1}[u] = sum_r W_hh[r][u] dg[r] and d(input)[u], and
//               accumulates dW[r][u] += dg[r] * input; an L-lane DPP reduction
//               gives every lane of the group the full dh_{t-1}[u] -- kept in a
//               register for the next row phase (no LDS round trip, no second
//               barrier); d(input) goes to the layer below through a parity
//               buffer that it reads two iterations later (layer lag 2).
// Packed fp32 FMAs (v_pk_fma_f32) throughout.
// ---------------------------------------------------------------------------
// LEAN: the fused training-step configuration (zero initial states, loss only
// through h_T of the top layer, no dx / dh0 / dc0 outputs) with every optional
// operand folded away at compile time -- fewer live pointers and no per-step
// branches on the hot path.
// CELL 1 = GRU (packing as in the forward): the gate-gradient vector is
// [dr*r(1-r) | dz*z(1-z) | dpre_n | dpre_n*r] with dpre_n = dh (1-z) (1-n^2),
// so the column phase (W^T g, dW += g h^T / g x^T) is the LSTM's unchanged;
// the direct path dh_{t-1} += dh_t z rides in the dc register.
// W columns (u) of this lane's rows j*RS.. as float2 pairs along rows
// (W_hh and W_ih; W_ih columns past the layer input are zero).
template <int H, int L>
struct BwdCols {
  pdrnn_f2 whh[4 * H / L / 2], wih[4 * H / L / 2];
};
template <int H, int L>
__device__ __forceinline__ BwdCols<H, L> bwd_load_cols(const PdrnnLstmSmallBwdArgs& a) {
  constexpr int RS = 4 * H / L;
  constexpr int LANES = H * L;
  const int tid = threadIdx.x;
  const int layer = __builtin_amdgcn_readfirstlane(tid / LANES);
  const int lg = tid - layer * LANES;
  const int u = lg / L, j = lg % L;
  const int Iin = layer == 0 ? a.I : H;
  const int r0 = j * RS;
  const bool ih_live = u < Iin;
  BwdCols<H, L> w;
  const float* ph = a.w_hh[layer] + (int64_t)r0 * H + u;
  const float* pi = a.w_ih[layer] + (int64_t)r0 * Iin + min(u, Iin - 1);
#pragma unroll
  for (int rr = 0; rr < RS / 2; ++rr) {
    w.whh[rr] = pdrnn_f2{wround(ph[(2 * rr) * H], a.w_bf16), wround(ph[(2 * rr + 1) * H], a.w_bf16)};
    const float x0 = pi[(int64_t)(2 * rr) * Iin], x1 = pi[(int64_t)(2 * rr + 1) * Iin];
    w.wih[rr] = ih_live ? pdrnn_f2{wround(x0, a.w_bf16), wround(x1, a.w_bf16)} : pdrnn_f2{0.f, 0.f};
  }
  return w;
}

template <int H, int L, int NB, bool XLDS, bool LEAN, int CELL = 0, bool DWOUT = false>
// xs_off >= 0: x already staged at smem + xs_off by the forward half of the
// one-launch step (same layout, same workgroup): not loaded again.
// wpre: the W columns, loaded by the caller ahead of time (one-launch step:
// issued before the forward so their latency hides behind it).
// dh_lds: the top layer's dh_T of this workgroup's (single) sequence in LDS.
// DWOUT: no register-resident dW / db accumulators and no slab row; every
// step's gate gradients go to a.dg_out instead (one 4-byte store per row lane,
// overwriting the activation slot that lane has just consumed when dg_out ==
// act) and lstm_small_dw.hip forms the weight gradients on the matrix cores.
// The 64 accumulator VGPRs it frees raise the resident workgroups per CU
// (B = 1440: three residency rounds become two), and the per-step rank-1
// updates (~1/3 of a step's VALU issue) leave the recurrence's critical path.
__device__ __forceinline__ void lstm_small_bwd_gs_body(const PdrnnLstmSmallBwdArgs& a, int xs_off = -1,
                                                       const BwdCols<H, L>* wpre = nullptr,
                                                       const float* dh_lds = nullptr) {
  constexpr int R = 4 * H;
  constexpr int RS = R / L;          // rows per lane
  constexpr int LANES = H * L;
  static_assert(L >= 4 && RS % 4 == 0, "need >= 4 lanes per unit, float4 row slices");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int NL = a.NL, B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const uint64_t sr_in = (a.stamps && tid == 0) ? stamp_real() : 0;
  const int layer = __builtin_amdgcn_readfirstlane(tid / LANES);
  const int lg = tid - layer * LANES;
  const int u = lg / L;
  const int j = lg % L;
  const int q = j & 3;
  const bool rowlane = j < 4;
  const int Iin = layer == 0 ? I : H;
  const bool top = layer == NL - 1;
  const int lag = 2 * (NL - 1 - layer);
  const float* const h0p = LEAN ? nullptr : a.h0;
  const float* const c0p = LEAN ? nullptr : a.c0;
  const float* const doutp = LEAN ? nullptr : a.dout;
  const float* const dcnp = LEAN ? nullptr : a.dcn;
  float* const dxp = LEAN ? nullptr : a.dx;
  float* const dh0p = LEAN ? nullptr : a.dh0;
  float* const dc0p = LEAN ? nullptr : a.dc0;
  const bool top_only = LEAN ? true : a.dhn_top_only;

  // LDS: dg[NB][NL][2][RP] | dha[NB][NL][2][H] | xs[NB][T][H]
  // The gate-gradient vector is stored with a 4-float pad after every RS-row
  // slice: the L lanes of a unit read slices j*RS.. as float4s, and with an
  // unpadded RS = 32 slices j and j + 2 hit the same banks (2-way conflict,
  // ~150 cycles per step, profiles/r2_small_kernels_pmc.md).
  constexpr int RP = R + L * 4;
  float* dg_s = smem;
  float* dha_s = dg_s + NB * NL * 2 * RP;
  float* xs = xs_off >= 0 ? smem + xs_off : dha_s + NB * NL * 2 * H;
  auto dgbuf = [&](int n, int l, int p) { return dg_s + ((n * NL + l) * 2 + p) * RP; };
  auto dhabuf = [&](int n, int l, int p) { return dha_s + ((n * NL + l) * 2 + p) * H; };

  // ---- W columns (u) for rows j*RS.., as float2 pairs along rows ----------
  // Loaded ONCE and shared by the NB sequences a workgroup interleaves; the
  // grid is persistent over batch tiles (workgroup g handles tiles g, g+G, ...)
  // and the dW accumulators run across all of them, so a workgroup writes one
  // slab row however many sequences it processed.
  const int r0 = j * RS;
  const bool ih_live = u < Iin;
  float gm[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) gm[g] = q == g ? 1.f : 0.f;
  pdrnn_f2 whh[RS / 2], wih[RS / 2], dwhh[RS / 2], dwih[RS / 2];
  if (wpre) {
#pragma unroll
    for (int rr = 0; rr < RS / 2; ++rr) {
      whh[rr] = wpre->whh[rr];
      wih[rr] = wpre->wih[rr];
    }
  } else {
    const BwdCols<H, L> w = bwd_load_cols<H, L>(a);
#pragma unroll
    for (int rr = 0; rr < RS / 2; ++rr) {
      whh[rr] = w.whh[rr];
      wih[rr] = w.wih[rr];
    }
  }
#pragma unroll
  for (int rr = 0; rr < RS / 2; ++rr) {
    dwhh[rr] = pdrnn_f2{0.f, 0.f};
    dwih[rr] = pdrnn_f2{0.f, 0.f};
  }
  float db = 0.f;
  uint64_t st0 = 0, sr0 = 0;
  if (a.stamps && tid == 0) { st0 = stamp_cycles(); sr0 = stamp_real(); }

  struct Ops { float aq, ct, cp, dout, hprev, xin; };
  for (int b0 = blockIdx.x * NB; b0 < B; b0 += gridDim.x * NB) {
    int bs[NB], bsrc[NB];
    bool valid[NB];
    float dh[NB], dc[NB], dha_r[NB];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      valid[n] = b0 + n < B;
      bs[n] = min(b0 + n, B - 1);  // invalid slots recompute the last sequence, never store
      bsrc[n] = a.idx ? (int)a.idx[bs[n]] : bs[n];
      dh[n] = 0.f;
      dha_r[n] = 0.f;
      if (dh_lds) {
        dh[n] = top ? dh_lds[u] : 0.f;
      } else if (a.dhn) {
        if (top_only) dh[n] = top ? a.dhn[(int64_t)bs[n] * H + u] : 0.f;
        else dh[n] = a.dhn[((int64_t)layer * B + bs[n]) * H + u];
      }
      dc[n] = dcnp ? dcnp[((int64_t)layer * B + bs[n]) * H + u] : 0.f;
      if (lg < H) {
        dhabuf(n, layer, 0)[lg] = 0.f;
        dhabuf(n, layer, 1)[lg] = 0.f;
      }
    }
    if constexpr (XLDS) {
      if (xs_off < 0) {
#pragma unroll
        for (int n = 0; n < NB; ++n)
          stage_x<H>(xs + (int64_t)n * T * H, a.x, (int64_t)bsrc[n] * a.x_sb, a.x_st, T, I, a.x_bf16, true,
                     (DWOUT && valid[n]) ? a.xg_out + (int64_t)bs[n] * T * a.xg_ld : nullptr, a.xg_ld);
      }
    }

    // ---- raw per-timestep operands (prefetched 2 steps ahead, masked at use)
    // Every stream is a buffer descriptor on a wave-uniform base (SGPRs), a
    // per-lane byte offset fixed for the whole loop (VGPR) and a per-step
    // scalar offset: one buffer_load per operand, no per-step VALU address
    // arithmetic.  Out-of-range steps are clamped, the values masked at use.
    // NB > 1 with x in LDS: the NB sequences of a tile are consecutive rows
    // (bs[n] >= bs[0]), so ONE descriptor per stream serves all of them and a
    // sequence's rows are a wave-uniform byte delta folded into the scalar
    // offset -- 4 SGPRs per stream instead of 4 NB (the paired-sequence BPTT
    // spilled SGPRs into VGPR lanes inside the recurrence)
    constexpr bool kShared = XLDS && NB > 1;
    constexpr int ND = kShared ? 1 : NB;
    __amdgpu_buffer_rsrc_t r_act[ND], r_own[ND], r_in[ND];
    uint32_t d_act[NB], d_h[NB], d_dg[NB];
    const int x_layer0 = layer == 0 && !XLDS;
#pragma unroll
    for (int n = 0; n < ND; ++n) {
      const int64_t lb = (int64_t)layer * B + bs[n];
      r_act[n] = uniform_rsrc(a.act + lb * T * 5 * H);
      r_own[n] = uniform_rsrc(a.hseq + lb * T * H);
      r_in[n] = uniform_rsrc(x_layer0 ? a.x + (int64_t)bsrc[n] * a.x_sb
                                      : a.hseq + ((int64_t)(layer > 0 ? layer - 1 : 0) * B + bs[n]) * T * H);
    }
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const uint32_t dn = kShared ? (uint32_t)(bs[n] - bs[0]) * (uint32_t)T : 0u;
      d_act[n] = __builtin_amdgcn_readfirstlane(dn * 5u * H * 4u);
      d_h[n] = __builtin_amdgcn_readfirstlane(dn * (uint32_t)H * 4u);
      d_dg[n] = DWOUT ? __builtin_amdgcn_readfirstlane(dn * (uint32_t)a.dg_st * 4u) : 0u;
    }
    const bool has_dout = top && doutp != nullptr;
    // deferred dW: this row's gate-gradient stream (same row layout as act)
    __amdgpu_buffer_rsrc_t r_dg[ND];
    uint32_t st_dg = 0;
    if constexpr (DWOUT) {
      st_dg = (uint32_t)a.dg_st * 4;
#pragma unroll
      for (int n = 0; n < ND; ++n) r_dg[n] = uniform_rsrc(a.dg_out + ((int64_t)layer * B + bs[n]) * T * a.dg_st);
    }
    const uint32_t vo_q = (q * H + u) * 4, vo_c = (4 * H + u) * 4, vo_u = u * 4;
    const uint32_t vo_x = (x_layer0 ? min(u, I - 1) : u) * 4;
    const uint32_t st_act = 5 * H * 4, st_h = H * 4;
    const uint32_t st_x = x_layer0 ? (uint32_t)a.x_st * 4 : st_h;
    // Branch-free: every operand is loaded every step and masked at use.  A
    // load under a branch makes the waitcnt pass fall back to vmcnt(0) at the
    // join, which would wait for the prefetches issued for later steps too.
    auto load_ops = [&](int n, int t) {
      // scalar offsets (readfirstlane: provably uniform -> SGPR soffset, no waterfall)
      const uint32_t tc = __builtin_amdgcn_readfirstlane((uint32_t)min(max(t, 0), T - 1));
      const uint32_t tp = tc > 0 ? tc - 1 : 0;
      const uint32_t so_a = __builtin_amdgcn_readfirstlane(tc * st_act);
      const uint32_t so_ap = __builtin_amdgcn_readfirstlane(tp * st_act);
      const uint32_t so_h = __builtin_amdgcn_readfirstlane(tp * st_h);
      const uint32_t so_x = __builtin_amdgcn_readfirstlane(tc * st_x);
      Ops o;
      const int nd = kShared ? 0 : n;
      o.aq = bload(r_act[nd], vo_q, so_a + d_act[n]);
      o.ct = bload(r_act[nd], vo_c, so_a + d_act[n]);
      o.cp = bload(r_act[nd], vo_c, so_ap + d_act[n]);
      // optional operands (generic kernel only): descriptors built on demand
      // to keep the SGPR budget of the hot loop
      const int64_t lb = (int64_t)layer * B + bs[n];
      if (c0p && tc == 0) o.cp = bload(uniform_rsrc(c0p + lb * H), vo_u, 0);
      o.dout = has_dout ? bload(uniform_rsrc(doutp + bs[n] * a.d_sb), vo_u,
                                __builtin_amdgcn_readfirstlane(tc * (uint32_t)a.d_st * 4))
                        : 0.f;
      o.hprev = bload(r_own[nd], vo_u, so_h + d_h[n]);
      if (h0p && tc == 0) o.hprev = bload(uniform_rsrc(h0p + lb * H), vo_u, 0);
      o.xin = bload(r_in[nd], vo_x, so_x + (x_layer0 ? 0u : d_h[n]));
      return o;
    };

    const int t_first = T - 1 + lag;
    Ops opA[NB], opB[NB];
    // issue order pinned (A's loads, then B's): the loop's counted vmcnt waits
    // are the max over its entry edges, so a reordered prologue would make
    // every in-loop wait conservative
#pragma unroll
    for (int n = 0; n < NB; ++n) opA[n] = load_ops(n, t_first);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int n = 0; n < NB; ++n) opB[n] = load_ops(n, t_first - 1);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();

    // The step body is branch-free (inactive steps compute and mask): a branch
    // join makes the waitcnt pass conservative, and every conservative
    // vmcnt here would wait for the prefetches of the next two steps.
    const int dha_tgt = layer > 0 ? layer - 1 : NL - 1;  // top layer's dha slots are never read
    // the lean contract wants no input gradient: layer 0 skips W_ih^T g (a
    // quarter to a half of its column-phase FMAs) -- unless the dW updates
    // still need the column loop's operands (they do not depend on it)
    const bool need_dx = !LEAN || layer > 0;
    auto step = [&](int it, Ops* op) {
      const int t = t_first - it;
      const bool active = t >= 0 && t < T;
      const int p = it & 1;
      // ---------------- row phase ----------------
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        float dht = dh[n] + (has_dout ? op[n].dout : 0.f);
        if (!top) dht += dha_r[n];  // dh from the layer above (prefetched, see the column phase)
        const float ig = quad_bcast(op[n].aq, 0), fg = quad_bcast(op[n].aq, 1);
        const float gg = quad_bcast(op[n].aq, 2), og = quad_bcast(op[n].aq, 3);
        // this lane's gate gradient by arithmetic with 0/1 lane masks
        // (gm[q] = [q == lane's gate]): a select chain over q compiles into
        // divergent exec-masked branches inside the recurrence
        const float own = op[n].aq;
        float dgv, dcn;
        if constexpr (CELL == 0) {
          const float cp = (t > 0 || c0p) ? op[n].cp : 0.f;
          const float tc = tanhf_fast(op[n].ct);
          const float dcp = fmaf(dht * og, 1.f - tc * tc, dc[n]);
          // i: dcp gg s'(i)  f: dcp cp s'(f)  g: dcp ig t'(g)  o: dht tc s'(o)
          const float oth = fmaf(gm[0], gg, fmaf(gm[1], cp, fmaf(gm[2], ig, gm[3] * tc)));
          const float src = fmaf(gm[3], dht - dcp, dcp);
          const float der = fmaf(gm[2], 1.f - own, own) - own * own;
          dgv = src * oth * der;
          dcn = dcp * fg;
        } else {  // GRU: ig = r, fg = z, og = n_h, ct = n
          const float hp = (t > 0 || h0p) ? op[n].hprev : 0.f;
          const float nn = op[n].ct;
          const float dpn = dht * (1.f - fg) * (1.f - nn * nn);
          // r: dpn n_h s'(r)  z: dht (h - n) s'(z)  n_x: dpn  n_h: dpn r
          const float a0 = fmaf(gm[1], dht - dpn, dpn);
          const float a1 = fmaf(gm[0], og, fmaf(gm[1], hp - nn, fmaf(gm[3], ig, gm[2])));
          const float a2 = fmaf(gm[0] + gm[1], own - own * own - 1.f, 1.f);
          dgv = a0 * a1 * a2;
          dcn = dht * fg;  // direct path into dh_{t-1}
        }
        dgv = active ? dgv : 0.f;  // inactive: zero gate gradients (dW, db, dh unaffected)
        dc[n] = active ? dcn : dc[n];
        if (L == 4 || rowlane) {
          dgbuf(n, layer, p)[q * H + u + ((q * H + u) / RS) * 4] = dgv;
          if constexpr (!DWOUT) db += valid[n] ? dgv : 0.f;
        }
        if constexpr (DWOUT) {
          // branch-free: a step outside [0, T), an unused batch slot or a
          // duplicate lane (L = 8) stores out of the buffer's range, which the
          // hardware drops (a branch around it would make the loop's vmcnt
          // waits conservative, see load_ops)
          const bool st_ok = active && valid[n] && (L == 4 || rowlane);
          const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)min(max(t, 0), T - 1) * st_dg);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, dgv), r_dg[kShared ? 0 : n],
                                                st_ok ? vo_q : 0x80000000u, so + d_dg[n], 0);
        }
      }
      lds_barrier();
      // ---------------- column phase ----------------
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float hprev = (t > 0 || h0p) ? op[n].hprev : 0.f;
        // both candidates live at once (a select, not a branch): otherwise the
        // LDS read reuses the prefetch register and waits on in-flight loads
        const int tcl = min(max(t, 0), T - 1);
        const float xsv = XLDS ? xs[((int64_t)n * T + tcl) * H + u] : 0.f;
        const float xgv = (layer > 0 || u < I) ? op[n].xin : 0.f;
        const float xin = (XLDS && layer == 0) ? xsv : xgv;
        // an invalid slot still runs the recurrence but contributes nothing to dW
        const float hw = valid[n] ? hprev : 0.f, xw = valid[n] ? xin : 0.f;
        const float4* g4 = reinterpret_cast<const float4*>(dgbuf(n, layer, p) + r0 + j * 4);
        // all of this lane's gate-gradient slice in flight at once: one
        // LDS latency per step instead of one per read batch
        float4 gv[RS / 4];
#pragma unroll
        for (int r4 = 0; r4 < RS / 4; ++r4) gv[r4] = g4[r4];
        __builtin_amdgcn_sched_barrier(0);
        pdrnn_f2 sh[2] = {{0.f, 0.f}, {0.f, 0.f}}, sx[2] = {{0.f, 0.f}, {0.f, 0.f}};
        const pdrnn_f2 hb = {hw, opaque_copy(hw)}, xb = {xw, opaque_copy(xw)};
#pragma unroll
        for (int r4 = 0; r4 < RS / 4; ++r4) {
          const float4 g = gv[r4];
          const pdrnn_f2 g01 = {g.x, g.y}, g23 = {g.z, g.w};
          sh[0] = __builtin_elementwise_fma(whh[2 * r4], g01, sh[0]);
          sh[1] = __builtin_elementwise_fma(whh[2 * r4 + 1], g23, sh[1]);
          if (need_dx) {  // wave-uniform (one layer per wave); no loads inside
            sx[0] = __builtin_elementwise_fma(wih[2 * r4], g01, sx[0]);
            sx[1] = __builtin_elementwise_fma(wih[2 * r4 + 1], g23, sx[1]);
          }
          if constexpr (!DWOUT) {
            dwhh[2 * r4] = __builtin_elementwise_fma(g01, hb, dwhh[2 * r4]);
            dwhh[2 * r4 + 1] = __builtin_elementwise_fma(g23, hb, dwhh[2 * r4 + 1]);
            dwih[2 * r4] = __builtin_elementwise_fma(g01, xb, dwih[2 * r4]);
            dwih[2 * r4 + 1] = __builtin_elementwise_fma(g23, xb, dwih[2 * r4 + 1]);
          }
        }
        // pin this step's dW updates here: they feed nothing until the
        // epilogue, and left free the scheduler sinks them into the next
        // step (keeping this step's gate-gradient slice live across it)
        if constexpr (!DWOUT) {
#pragma unroll
          for (int rr = 0; rr < RS / 2; ++rr) asm volatile("" : "+v"(dwhh[rr]), "+v"(dwih[rr]));
        }
        const pdrnn_f2 shs = sh[0] + sh[1], sxs = sx[0] + sx[1];
        float dhn_ = group_sum<L>(shs.x + shs.y);  // dh_{t-1}[u] on every lane of the unit
        if constexpr (CELL == 1) dhn_ += dc[n];
        dh[n] = active ? dhn_ : dh[n];
        if (need_dx) {
          const float dx = group_sum<L>(sxs.x + sxs.y);
          // every lane of the unit holds dx: all write the same value (no
          // branch); consumed by layer-1 at it+2 (same parity)
          dhabuf(n, dha_tgt, p)[u] = dx;
          if (!LEAN && layer == 0 && dxp && active && j == 0 && u < I && valid[n])
            dxp[bs[n] * a.dx_sb + (int64_t)t * a.dx_st + u] = dx;
        }
      }
      // dh the layer above wrote for the NEXT iteration (its column phase of
      // it-1, published by this iteration's barrier): read now, off the next
      // row phase's critical path.  Its next overwrite is after the next barrier.
      if (!top) {
#pragma unroll
        for (int n = 0; n < NB; ++n) dha_r[n] = dhabuf(n, layer, (it + 1) & 1)[u];
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        op[n] = load_ops(n, t - 2);  // refill for two steps ahead
      }
    };

    const int iters = T + 2 * (NL - 1);
    // progress over all of this workgroup's tiles, in step pairs
    const int tiles = (B - (int)blockIdx.x * NB + (int)gridDim.x * NB - 1) / ((int)gridDim.x * NB);
    const int tile = (b0 - (int)blockIdx.x * NB) / ((int)gridDim.x * NB);
    const int hp = (iters + 1) / 2;
    int it = 0;
    for (; it + 1 < iters; it += 2) {
      prio_by_progress(tile * hp + it / 2, tiles * hp, a.prio);
      step(it, opA);
      step(it + 1, opB);
    }
    if (it < iters) step(it, opA);

    if (j == 0) {
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        if (!valid[n]) continue;
        if (dh0p) dh0p[((int64_t)layer * B + bs[n]) * H + u] = dh[n];
        if (CELL == 0 && dc0p) dc0p[((int64_t)layer * B + bs[n]) * H + u] = dc[n];
      }
    }
    __syncthreads();  // LDS is reused by the next tile
  }
  if (a.stamps && tid == 0) {
    uint64_t* st = a.stamps + (uint64_t)blockIdx.x * 8;
    st[0] = st0; st[1] = stamp_cycles(); st[2] = sr0; st[3] = stamp_real();
    st[4] = sr_in; st[5] = st[3]; st[6] = stamp_cu();
  }

  // ---------------- epilogue: this workgroup's partial dW / db ----------
  if constexpr (DWOUT) {
    // the dW kernel streams whole stages: the PDRNN_DW_PAD_ROWS padding rows
    // behind the last layer's gate gradients must hold finite values (masked
    // operands are multiplied by zero there, and NaN * 0 = NaN)
    if (blockIdx.x == 0) {
      float* pad = a.dg_out + (int64_t)NL * B * T * a.dg_st;
      for (int e = threadIdx.x; e < PDRNN_DW_PAD_ROWS * a.dg_st; e += blockDim.x) pad[e] = 0.f;
    }
    return;
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
  if (rowlane) {
    if (a.off_bih[layer] >= 0) slab[a.off_bih[layer] + q * H + u] = db;
    if (a.off_bhh[layer] >= 0) slab[a.off_bhh[layer] + q * H + u] = db;
  }
}

template <int H, int L, int NB, bool XLDS, bool LEAN, int CELL = 0>
__global__ void __launch_bounds__(512) lstm_small_bwd_gs_kernel(PdrnnLstmSmallBwdArgs a) {
  lstm_small_bwd_gs_body<H, L, NB, XLDS, LEAN, CELL>(a);
}

// Lean BPTT with the weight gradients deferred to lstm_small_dw.hip.
// NB = 2: two sequences per workgroup share the register-resident W columns
// (64 of the ~147 VGPRs of a lane), so a workgroup carries twice the batch at
// about the same register cost: B = 1440 (1152) fits ONE residency round of
// 720 (576) workgroups at 3 waves per SIMD instead of two rounds of one
// sequence each -- the recurrence's 130 dependent steps are paid once, each
// step issuing both sequences' independent chains.
template <int H, int L, int NB, bool XLDS, int CELL>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(NB > 1 ? 3 : 1)))
lstm_small_bwd_dwout_kernel(PdrnnLstmSmallBwdArgs a) {
  lstm_small_bwd_gs_body<H, L, NB, XLDS, true, CELL, true>(a);
}

// ---------------------------------------------------------------------------
// Whole training step of the latency regime in ONE launch: when the backward
// grid is one sequence per workgroup (B <= resident workgroups) and both maps
// use the same NL*4H lanes (gate-split forward, L = 4 unit-group backward),
// workgroup b runs sequence b's forward + head/CE epilogue and then its own
// BPTT.  Every operand the backward reads (saved activations, h sequence,
// dh_T) was written by this workgroup, so no grid-wide dependency exists: the
// kernel boundary between the two launches (tail of the slowest forward
// workgroup + the backward's launch and wave start) disappears, and each
// workgroup goes straight from its forward into its backward.
// ---------------------------------------------------------------------------
template <int H, bool XLDS, int CELL>
__global__ void __launch_bounds__(512) lstm_small_step_gs_kernel(PdrnnLstmSmallFwdArgs f, PdrnnLstmSmallBwdArgs b) {
  extern __shared__ __attribute__((aligned(16))) float smem_step[];
  static_assert(H <= 32, "dh_T slot must fit the L = 8 padding slack (NL * 2 * 16 floats >= H)");
  // x staged once, past the backward's gate-gradient / dh buffers (the larger
  // of the two halves' operand areas, bwd_gs_lds<H, 1> with L = 4 lanes)
  const int xs_off = XLDS ? f.NL * 2 * (4 * H + 4 * 4 + H) : -1;
  // the backward's W columns and the head's label / weights are issued now:
  // their latency hides behind the forward recurrence (registers are free --
  // the backward half sets the kernel's VGPR budget)
  const BwdCols<H, 4> wcols = bwd_load_cols<H, 4>(b);
  // dh_T slot: the launch's LDS slack past x (bwd_gs_lds pads for L = 8)
  float* dh_lds = XLDS ? smem_step + xs_off + f.T * H : nullptr;
  lstm_small_fwd_gs_body<H, 1, true, XLDS, true, CELL>(f, xs_off, true, dh_lds);
  // this workgroup's global stores (activations, h, dh_T) before its own
  // backward loads them: a workgroup-scope release/acquire (the barrier's
  // own fences) is enough -- every wave of the workgroup shares the CU's
  // L1, which holds no line of these buffers (the forward never loads them,
  // and the L1 is invalidated at kernel start).  An agent-scope fence here
  // would write back the XCD's L2 (measured: +6 us/step at B = 180).  The
  // LDS operand buffers are reused by the backward.
  __syncthreads();
  lstm_small_bwd_gs_body<H, 4, 1, XLDS, true, CELL>(b, xs_off, &wcols, dh_lds);
}

// Column-sum of a [rows, P] slab: pass 1 sums row chunks into work[split, P].
__global__ void slab_reduce_pass1(const float* __restrict__ slab, int64_t rows, int64_t P,
                                  float* __restrict__ work, int split) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int sp = blockIdx.y;
  if (p >= P) return;
  const int64_t r0 = rows * sp / split, r1 = rows * (sp + 1) / split;
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
  int64_t r = r0;
  for (; r + 4 <= r1; r += 4) {
    acc0 += slab[(r + 0) * P + p];
    acc1 += slab[(r + 1) * P + p];
    acc2 += slab[(r + 2) * P + p];
    acc3 += slab[(r + 3) * P + p];
  }
  for (; r < r1; ++r) acc0 += slab[r * P + p];
  work[(int64_t)sp * P + p] = (acc0 + acc1) + (acc2 + acc3);
}

__global__ void slab_reduce_pass2(const float* __restrict__ work, int64_t P, int split,
                                  float* __restrict__ out, float beta) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  float acc = 0.f;
  for (int sp = 0; sp < split; ++sp) acc += work[(int64_t)sp * P + p];
  out[p] = beta == 0.f ? acc : fmaf(beta, out[p], acc);
}

// pass 1 over two slabs side by side: columns [0, PA) from A, [PA, PA+PB) from B.
// colmap (optional): output column p < PA reads A column colmap[p] of an A
// slab with leading dimension ldA (the GRU's packed 4-block layout -> nn.GRU
// parameter order, zero blocks dropped).
__global__ void slab2_reduce_pass1(const float* __restrict__ A, int64_t rowsA, int64_t PA,
                                   const float* __restrict__ Bs, int64_t rowsB, int64_t PB,
                                   float* __restrict__ work, int split, const int* __restrict__ colmap,
                                   int64_t ldA) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int sp = blockIdx.y;
  const int64_t P = PA + PB;
  if (p >= P) return;
  const bool inA = p < PA;
  const float* src = inA ? A + (colmap ? colmap[p] : p) : Bs + (p - PA);
  const int64_t ld = inA ? ldA : PB;
  const int64_t rows = inA ? rowsA : rowsB;
  const int64_t r0 = rows * sp / split, r1 = rows * (sp + 1) / split;
  // 8 independent loads in flight per thread (the head slab has B rows over
  // ~200 columns: few threads, long columns -- latency-bound otherwise)
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += src[(r + k) * ld];
  }
  for (int k = 0; r < r1; ++r, ++k) acc[k] += src[r * ld];
  work[(int64_t)sp * P + p] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
}

__global__ void slab_reduce_pass2_split(const float* __restrict__ work, int64_t P, int64_t Pa, int split,
                                        float* __restrict__ out_a, float* __restrict__ out_b) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  float acc = 0.f;
  for (int sp = 0; sp < split; ++sp) acc += work[(int64_t)sp * P + p];
  if (p < Pa) out_a[p] = acc;
  else out_b[p - Pa] = acc;
}

template <int H, int S, int NB, bool SAVE>
hipError_t launch_fwd(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  constexpr int LANES = H * S;
  const int grid = (a->B + NB - 1) / NB;
  const int block = a->NL * LANES;
  const size_t lds = sizeof(float) * NB * a->NL * 2 * (2 * H);
  const size_t xbytes = sizeof(float) * (size_t)NB * a->T * H;
  if constexpr (SAVE) {
    if (a->head_w) {  // fused training step: classifier head + CE epilogue
      if (a->C > 16) return hipErrorInvalidValue;
      if (xbytes <= (size_t)kXldsBytes)
        hipLaunchKernelGGL((lstm_small_fwd_kernel<H, S, NB, true, true, true>), dim3(grid), dim3(block), lds + xbytes, st, *a);
      else
        hipLaunchKernelGGL((lstm_small_fwd_kernel<H, S, NB, true, false, true>), dim3(grid), dim3(block), lds, st, *a);
      return hipGetLastError();
    }
  }
  if (xbytes <= (size_t)kXldsBytes)
    hipLaunchKernelGGL((lstm_small_fwd_kernel<H, S, NB, SAVE, true>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  else
    hipLaunchKernelGGL((lstm_small_fwd_kernel<H, S, NB, SAVE, false>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

template <int H, int NB, bool SAVE>
hipError_t launch_fwd_gs(const PdrnnLstmSmallFwdArgs* a, hipStream_t st);

// GRU forward: NB sequences per workgroup (2 above one residency round: one
// sequence per 4-wave workgroup holds ~150 VGPRs, 3 workgroups per CU); the
// classifier head + CE epilogue of the fused training step (SAVE + head_w) is
// shared with the LSTM.
template <int H, int NB, bool SAVE>
hipError_t launch_fwd_gs_gru(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  const int grid = (a->B + NB - 1) / NB;
  const int block = a->NL * 4 * H;
  const size_t lds = sizeof(float) * NB * a->NL * 2 * (2 * H);
  const size_t xbytes = sizeof(float) * (size_t)NB * a->T * H;
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if (a->head_w) {
    if constexpr (SAVE) {
      if (a->C > 16) return hipErrorInvalidValue;
      if (xl) hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, true, true, true, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
      else hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, true, false, true, 1>), dim3(grid), dim3(block), lds, st, *a);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (xl)
    hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, SAVE, true, false, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  else
    hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, SAVE, false, false, 1>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

template <int H, int NB, bool SAVE>
hipError_t launch_fwd_gs(const PdrnnLstmSmallFwdArgs* a, hipStream_t st);

// GRU forward: one sequence per workgroup; the classifier head + CE epilogue
// of the fused training step (SAVE + head_w) is shared with the LSTM.
template <int H, bool SAVE>
hipError_t launch_fwd_gs_gru(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  const int grid = a->B;
  const int block = a->NL * 4 * H;
  const size_t lds = sizeof(float) * a->NL * 2 * (2 * H);
  const size_t xbytes = sizeof(float) * (size_t)a->T * H;
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if (a->head_w) {
    if constexpr (SAVE) {
      if (a->C > 16) return hipErrorInvalidValue;
      if (xl) hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, 1, true, true, true, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
      else hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, 1, true, false, true, 1>), dim3(grid), dim3(block), lds, st, *a);
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (xl)
    hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, 1, SAVE, true, false, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  else
    hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, 1, SAVE, false, false, 1>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

template <int H, int NB, bool SAVE>
hipError_t launch_fwd_gs(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  const int grid = (a->B + NB - 1) / NB;
  const int block = a->NL * 4 * H;
  const size_t lds = sizeof(float) * NB * a->NL * 2 * (2 * H);
  const size_t xbytes = sizeof(float) * (size_t)NB * a->T * H;
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if constexpr (SAVE) {
    if (a->head_w) {
      if (a->C > 16) return hipErrorInvalidValue;
      if (xl) hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, true, true, true>), dim3(grid), dim3(block), lds + xbytes, st, *a);
      else hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, true, false, true>), dim3(grid), dim3(block), lds, st, *a);
      return hipGetLastError();
    }
  }
  if (xl)
    hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, SAVE, true, false>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  else
    hipLaunchKernelGGL((lstm_small_fwd_gs_kernel<H, NB, SAVE, false, false>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

// lanes per hidden unit of the unit-group backward: 8 at H = 64 (row slices
// of 32), else 4
template <int H>
int bwd_gs_lanes(int NL) {
  (void)NL;
  return H == 64 ? 8 : 4;
}

// Persistent grid for the backward: as many workgroups as can be resident
// (occupancy query x CU count), capped by the number of batch tiles.
template <int H, int L, int NB, bool XLDS, bool LEAN>
int bwd_gs_resident(int NL, size_t lds) {
  // one-entry cache per instantiation (the query costs a driver round trip)
  static thread_local int c_dev = -1, c_nl = -1, c_val = 0;
  static thread_local size_t c_lds = 0;
  int per_cu = 0, cus = 0, dev = 0;
  hipGetDevice(&dev);
  if (dev == c_dev && NL == c_nl && lds == c_lds) return c_val;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_small_bwd_gs_kernel<H, L, NB, XLDS, LEAN>, NL * H * L, lds);
  if (per_cu < 1) per_cu = 1;
  if (cus < 1) cus = 1;
  c_dev = dev; c_nl = NL; c_lds = lds; c_val = per_cu * cus;
  return c_val;
}

template <int H, int NB>
size_t bwd_gs_lds(int NL) {
  // dg slices padded by 4 floats per lane slice (L <= 8 lanes per unit)
  return sizeof(float) * NB * NL * 2 * (4 * H + 8 * 4 + H);
}
template <int H, int NB>
size_t bwd_gs_xbytes(int T) { return sizeof(float) * (size_t)NB * T * H; }

inline bool bwd_lean(const PdrnnLstmSmallBwdArgs* a) {
  return !a->h0 && !a->c0 && !a->dout && !a->dcn && !a->dx && !a->dh0 && !a->dc0 && a->dhn && a->dhn_top_only;
}

template <int H, int L, int NB>
int bwd_gs_grid(const PdrnnLstmSmallBwdArgs* a) {
  const size_t lds = bwd_gs_lds<H, NB>(a->NL), xbytes = bwd_gs_xbytes<H, NB>(a->T);
  const bool xl = xbytes <= (size_t)kXldsBytes;
  int cap;
  if (bwd_lean(a)) cap = xl ? bwd_gs_resident<H, L, NB, true, true>(a->NL, lds + xbytes)
                            : bwd_gs_resident<H, L, NB, false, true>(a->NL, lds);
  else cap = xl ? bwd_gs_resident<H, L, NB, true, false>(a->NL, lds + xbytes)
                : bwd_gs_resident<H, L, NB, false, false>(a->NL, lds);
  const int tiles = (a->B + NB - 1) / NB;
  return tiles < cap ? tiles : cap;
}

template <int H, int L>
hipError_t launch_bwd_gs_gru(const PdrnnLstmSmallBwdArgs* a, hipStream_t st, int grid) {
  const int block = a->NL * H * L;
  const size_t lds = bwd_gs_lds<H, 1>(a->NL), xbytes = bwd_gs_xbytes<H, 1>(a->T);
  if (grid <= 0) grid = bwd_gs_grid<H, L, 1>(a);
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if (bwd_lean(a)) {  // fused training step: zero initial state, loss through h_T only
    if (xl) hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, 1, true, true, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
    else hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, 1, false, true, 1>), dim3(grid), dim3(block), lds, st, *a);
  } else {
    if (xl) hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, 1, true, false, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
    else hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, 1, false, false, 1>), dim3(grid), dim3(block), lds, st, *a);
  }
  return hipGetLastError();
}

template <int H, int L, int NB>
hipError_t launch_bwd_gs(const PdrnnLstmSmallBwdArgs* a, hipStream_t st, int grid) {
  const int block = a->NL * H * L;
  const size_t lds = bwd_gs_lds<H, NB>(a->NL), xbytes = bwd_gs_xbytes<H, NB>(a->T);
  if (grid <= 0) grid = bwd_gs_grid<H, L, NB>(a);
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if (bwd_lean(a)) {
    if (xl) hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, NB, true, true>), dim3(grid), dim3(block), lds + xbytes, st, *a);
    else hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, NB, false, true>), dim3(grid), dim3(block), lds, st, *a);
  } else {
    if (xl) hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, NB, true, false>), dim3(grid), dim3(block), lds + xbytes, st, *a);
    else hipLaunchKernelGGL((lstm_small_bwd_gs_kernel<H, L, NB, false, false>), dim3(grid), dim3(block), lds, st, *a);
  }
  return hipGetLastError();
}

template <int H, int S2, int NB>
hipError_t launch_bwd(const PdrnnLstmSmallBwdArgs* a, hipStream_t st) {
  constexpr int G = 2 * H * S2;
  const int grid = (a->B + NB - 1) / NB;
  const int block = a->NL * G;
  const size_t lds = sizeof(float) * NB * a->NL * (4 * H + 2 * H);
  const size_t xbytes = sizeof(float) * (size_t)NB * a->T * H;
  if (xbytes <= (size_t)kXldsBytes)
    hipLaunchKernelGGL((lstm_small_bwd_kernel<H, S2, NB, true>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  else
    hipLaunchKernelGGL((lstm_small_bwd_kernel<H, S2, NB, false>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

// Valid lane splits.  Forward: lanes per layer H*S (multiple of 64),
// K slice 2H/S float4-aligned and inside one half of [x | h].  Backward:
// lanes per layer 2H*S2, row slice 4H/S2 a multiple of 16.  Workgroup size
// NL * lanes <= 512 (launch bound: keeps 256 VGPRs per lane available).
constexpr bool fwd_ok(int H, int S) {
  return (H * S) % 64 == 0 && (2 * H / S) % 4 == 0 && H % (2 * H / S) == 0;
}
constexpr bool bwd_ok(int H, int S2) { return S2 >= 2 && (4 * H / S2) % 16 == 0 && (2 * H * S2) % 64 == 0; }

template <int H, int S>
hipError_t dispatch_fwd_s(const PdrnnLstmSmallFwdArgs* a, int nb, int save, hipStream_t st) {
  if constexpr (!fwd_ok(H, S)) {
    return hipErrorInvalidValue;
  } else {
    if (a->NL * H * S > 512) return hipErrorInvalidConfiguration;
    if (save) {
      if (nb == 1) return launch_fwd<H, S, 1, true>(a, st);
      if (nb == 2) return launch_fwd<H, S, 2, true>(a, st);
    } else {
      if (nb == 1) return launch_fwd<H, S, 1, false>(a, st);
      if (nb == 2) return launch_fwd<H, S, 2, false>(a, st);
    }
    return hipErrorInvalidValue;
  }
}

template <int H>
hipError_t dispatch_fwd(const PdrnnLstmSmallFwdArgs* a, int nb, int split, int save, hipStream_t st) {
  if (a->cell == 1 && split != 1) return hipErrorInvalidConfiguration;  // GRU: gate-split map only
  if (split == 1) {  // gate-split map (4 lanes per unit, one gate each)
    if (a->NL * 4 * H > 512) return hipErrorInvalidConfiguration;

    if (a->cell == 1) {
      if (nb == 2) return save ? launch_fwd_gs_gru<H, 2, true>(a, st) : launch_fwd_gs_gru<H, 2, false>(a, st);
      return save ? launch_fwd_gs_gru<H, 1, true>(a, st) : launch_fwd_gs_gru<H, 1, false>(a, st);
    }
    if (save) return nb == 2 ? launch_fwd_gs<H, 2, true>(a, st) : launch_fwd_gs<H, 1, true>(a, st);
    return nb == 2 ? launch_fwd_gs<H, 2, false>(a, st) : launch_fwd_gs<H, 1, false>(a, st);
  }
  // (K splits of 4 / 8 lanes per unit are never the widest valid map -- a
  // stack that fits them fits the gate-split map -- and are not built)
  if (split == 2) return dispatch_fwd_s<H, 2>(a, nb, save, st);
  return hipErrorInvalidValue;
}

template <int H, int S2>
hipError_t dispatch_bwd_s(const PdrnnLstmSmallBwdArgs* a, int nb, hipStream_t st) {
  if constexpr (!bwd_ok(H, S2)) {
    return hipErrorInvalidValue;
  } else {
    if (a->NL * 2 * H * S2 > 512) return hipErrorInvalidConfiguration;
    if (nb == 1) return launch_bwd<H, S2, 1>(a, st);
    return hipErrorInvalidValue;
  }
}

template <int H>
hipError_t dispatch_bwd(const PdrnnLstmSmallBwdArgs* a, int nb, int split, hipStream_t st, int grid_hint) {
  if (a->cell == 1 && (split != 1 || nb != 1)) return hipErrorInvalidConfiguration;
  if (split == 1) {  // unit-group map, L lanes per unit (row slices of 4H/L)
    if (a->cell == 1) {
      if (a->NL * H * (H >= 64 ? 8 : 4) > 512) return hipErrorInvalidConfiguration;
      if constexpr (H >= 64) return launch_bwd_gs_gru<H, 8>(a, st, grid_hint);
      else return launch_bwd_gs_gru<H, 4>(a, st, grid_hint);
    }
    if (bwd_gs_lanes<H>(a->NL) == 8) {
      if constexpr (H <= 32) {
        switch (nb) {
          case 1: return launch_bwd_gs<H, 8, 1>(a, st, grid_hint);
          case 2: return launch_bwd_gs<H, 8, 2>(a, st, grid_hint);
          case 3: return launch_bwd_gs<H, 8, 3>(a, st, grid_hint);
          default: return hipErrorInvalidConfiguration;
        }
      }
      if constexpr (H == 64) {
        switch (nb) {
          case 1: return launch_bwd_gs<H, 8, 1>(a, st, grid_hint);
          default: return hipErrorInvalidConfiguration;
        }
      }
    }
    constexpr int L = 4;
    if constexpr (H <= 32) {
      if (a->NL * H * L > 512) return hipErrorInvalidConfiguration;
      switch (nb) {
        case 1: return launch_bwd_gs<H, L, 1>(a, st, grid_hint);
        case 2: return launch_bwd_gs<H, L, 2>(a, st, grid_hint);
        case 3: return launch_bwd_gs<H, L, 3>(a, st, grid_hint);
        default: return hipErrorInvalidConfiguration;
      }
    }
    return hipErrorInvalidConfiguration;
  }
  // (likewise the 4-slice row split: a stack that fits it fits the unit-group map)
  if (split == 2) return dispatch_bwd_s<H, 2>(a, nb, st);
  return hipErrorInvalidValue;
}

template <int H>
hipError_t launch_step_gs(const PdrnnLstmSmallFwdArgs* f, const PdrnnLstmSmallBwdArgs* b, hipStream_t st) {
  if (f->NL * 4 * H > 512 || f->B != b->B || f->T != b->T || f->NL != b->NL) return hipErrorInvalidConfiguration;
  if (!f->head_w || f->C > 16 || !bwd_lean(b)) return hipErrorInvalidValue;
  const int grid = f->B;
  const int block = f->NL * 4 * H;  // = NL * H * L with L = 4
  const size_t lds_f = sizeof(float) * f->NL * 2 * (2 * H);
  const size_t lds_b = bwd_gs_lds<H, 1>(f->NL);
  const size_t lds = lds_f > lds_b ? lds_f : lds_b;
  const size_t xbytes = sizeof(float) * (size_t)f->T * H;
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if (f->cell == 1) {
    if (xl) hipLaunchKernelGGL((lstm_small_step_gs_kernel<H, true, 1>), dim3(grid), dim3(block), lds + xbytes, st, *f, *b);
    else hipLaunchKernelGGL((lstm_small_step_gs_kernel<H, false, 1>), dim3(grid), dim3(block), lds, st, *f, *b);
  } else {
    if (xl) hipLaunchKernelGGL((lstm_small_step_gs_kernel<H, true, 0>), dim3(grid), dim3(block), lds + xbytes, st, *f, *b);
    else hipLaunchKernelGGL((lstm_small_step_gs_kernel<H, false, 0>), dim3(grid), dim3(block), lds, st, *f, *b);
  }
  return hipGetLastError();
}

// ---- deferred-dW backward (DWOUT) ----------------------------------------
template <int H>
constexpr int dwout_lanes() { return H >= 64 ? 8 : 4; }

template <int H, int NB, bool XLDS, int CELL>
int bwd_dwout_resident(int NL, size_t lds) {
  constexpr int L = dwout_lanes<H>();
  static thread_local int c_dev = -1, c_nl = -1, c_val = 0;
  static thread_local size_t c_lds = 0;
  int per_cu = 0, cus = 0, dev = 0;
  hipGetDevice(&dev);
  if (dev == c_dev && NL == c_nl && lds == c_lds) return c_val;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lstm_small_bwd_dwout_kernel<H, L, NB, XLDS, CELL>,
                                               NL * H * L, lds);
  if (per_cu < 1) per_cu = 1;
  if (cus < 1) cus = 1;
  c_dev = dev; c_nl = NL; c_lds = lds; c_val = per_cu * cus;
  return c_val;
}

template <int H, int NB>
int bwd_dwout_cap(int NL, int T, int cell) {
  const size_t lds = bwd_gs_lds<H, NB>(NL), xbytes = bwd_gs_xbytes<H, NB>(T);
  const bool xl = xbytes <= (size_t)kXldsBytes;
  return cell == 1 ? (xl ? bwd_dwout_resident<H, NB, true, 1>(NL, lds + xbytes)
                         : bwd_dwout_resident<H, NB, false, 1>(NL, lds))
                   : (xl ? bwd_dwout_resident<H, NB, true, 0>(NL, lds + xbytes)
                         : bwd_dwout_resident<H, NB, false, 0>(NL, lds));
}

// Sequences per workgroup of the deferred-dW backward: 2 when pairing the
// sequences takes fewer residency rounds than one per workgroup (B = 1152 /
// 1440 at H = 32: one round instead of two), else 1.  PDRNN_TUNE dwout_nb=1|2
// forces one (A/B measurements).
template <int H>
int bwd_dwout_nb(int NL, int T, int B, int cell) {
  const int env = pdrnn_tune_int("dwout_nb", 0);  // per call: tests flip it in-process
  if (env == 1 || env == 2) return env;
  if (H > 32 || NL * H * dwout_lanes<H>() > 512) return 1;
  const int cap1 = bwd_dwout_cap<H, 1>(NL, T, cell), cap2 = bwd_dwout_cap<H, 2>(NL, T, cell);
  const int r1 = (B + cap1 - 1) / cap1, r2 = ((B + 1) / 2 + cap2 - 1) / cap2;
  return r2 < r1 ? 2 : 1;
}

// Balanced persistent grid: the fewest residency rounds, then the fewest
// workgroups that still finish in that many rounds -- every workgroup walks
// the same number of batch tiles (B = 1440 at 768 resident: 720 x 2, not a
// second round of 672 behind a first of 768), and fewer co-resident waves
// make each recurrence step cheaper.
template <int H>
int bwd_dwout_grid(int NL, int T, int B, int cell, int nb) {
  const int cap = nb == 2 ? bwd_dwout_cap<H, 2>(NL, T, cell) : bwd_dwout_cap<H, 1>(NL, T, cell);
  const int tiles = (B + nb - 1) / nb;
  if (tiles <= cap) return tiles;
  const int rounds = (tiles + cap - 1) / cap;
  return (tiles + rounds - 1) / rounds;
}

template <int H, int NB>
hipError_t launch_bwd_dwout_nb(const PdrnnLstmSmallBwdArgs* a, hipStream_t st, int grid) {
  constexpr int L = dwout_lanes<H>();
  const int block = a->NL * H * L;
  const size_t lds = bwd_gs_lds<H, NB>(a->NL), xbytes = bwd_gs_xbytes<H, NB>(a->T);
  const bool xl = xbytes <= (size_t)kXldsBytes;
  if (!xl || !a->xg_out) return hipErrorInvalidConfiguration;  // x staged once per sequence (writes xg_out)
  if (grid <= 0) grid = bwd_dwout_grid<H>(a->NL, a->T, a->B, a->cell, NB);
  if (a->cell == 1) hipLaunchKernelGGL((lstm_small_bwd_dwout_kernel<H, L, NB, true, 1>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  else hipLaunchKernelGGL((lstm_small_bwd_dwout_kernel<H, L, NB, true, 0>), dim3(grid), dim3(block), lds + xbytes, st, *a);
  return hipGetLastError();
}

template <int H>
hipError_t launch_bwd_dwout(const PdrnnLstmSmallBwdArgs* a, hipStream_t st, int grid, int nb) {
  constexpr int L = dwout_lanes<H>();
  if (a->NL * H * L > 512) return hipErrorInvalidConfiguration;
  if (!bwd_lean(a) || !a->dg_out || a->dg_st < 4 * H) return hipErrorInvalidValue;
  if (nb == 2) {
    if constexpr (H <= 32) return launch_bwd_dwout_nb<H, 2>(a, st, grid);
    return hipErrorInvalidConfiguration;
  }
  return launch_bwd_dwout_nb<H, 1>(a, st, grid);
}

}  // namespace
}  // namespace pdrnn

extern "C" {

// PDRNN_TUNE dwout=0 disables the deferred-dW backward, dwout=force selects it at
// every batch size (tests: the one-launch step would otherwise take B <= one
// residency round).  Returns 0 (not covered), 1 (covered), 2 (covered, forced).
int pdrnn_lstm_small_dwout_ok(int H, int NL, int T) {
  // read per call (one host query per training step): tests flip it in-process
  char e[16];
  const int mode = !pdrnn_tune_str("dwout", e, (int)sizeof(e)) ? 1 : (e[0] == '0' ? 0 : (strcmp(e, "force") == 0 ? 2 : 1));
  if (mode == 0 || T < 4 || NL < 1 || NL > PDRNN_MAX_LAYERS) return 0;
  if (H != 16 && H != 32 && H != 64) return 0;
  if ((size_t)T * H * sizeof(float) > (size_t)pdrnn::kXldsBytes) return 0;  // LDS-resident x only
  return NL * H * (H >= 64 ? 8 : 4) <= 512 ? mode : 0;
}

int pdrnn_lstm_small_bwd_dwout_nb(int H, int NL, int T, int B) {
  // LSTM and GRU instantiations share the register budget (same VGPR class);
  // the LSTM's is the one queried
  switch (H) {
    case 16: return pdrnn::bwd_dwout_nb<16>(NL, T, B, 0);
    case 32: return pdrnn::bwd_dwout_nb<32>(NL, T, B, 0);
    case 64: return pdrnn::bwd_dwout_nb<64>(NL, T, B, 0);
    default: return -1;
  }
}

int pdrnn_lstm_small_bwd_dwout_grid(int H, int NL, int T, int B, int nb) {
  switch (H) {
    case 16: return pdrnn::bwd_dwout_grid<16>(NL, T, B, 0, nb);
    case 32: return pdrnn::bwd_dwout_grid<32>(NL, T, B, 0, nb);
    case 64: return pdrnn::bwd_dwout_grid<64>(NL, T, B, 0, nb);
    default: return -1;
  }
}

hipError_t pdrnn_lstm_small_bwd_dwout(const PdrnnLstmSmallBwdArgs* a, int H, int grid, int nb, hipStream_t stream) {
  if (a->x_bf16 && (size_t)a->T * H * sizeof(float) * (nb > 1 ? nb : 1) > (size_t)pdrnn::kXldsBytes)
    return hipErrorInvalidConfiguration;
  if (nb != 1 && nb != 2) return hipErrorInvalidValue;
  switch (H) {
    case 16: return pdrnn::launch_bwd_dwout<16>(a, stream, grid, nb);
    case 32: return pdrnn::launch_bwd_dwout<32>(a, stream, grid, nb);
    case 64: return pdrnn::launch_bwd_dwout<64>(a, stream, grid, nb);
    default: return hipErrorInvalidValue;
  }
}

// 1 when the fused one-launch step covers (H, NL, B, launch config): the
// gate-split forward with one sequence per workgroup, the L = 4 unit-group
// backward, and a backward grid of one sequence per workgroup (gridb == B).
int pdrnn_lstm_small_step_ok(int H, int NL, int B, int nb_fwd, int split_fwd, int nb_bwd, int split_bwd,
                             int gridb) {
  if ((H != 16 && H != 32) || nb_fwd != 1 || split_fwd != 1 || nb_bwd != 1 || split_bwd != 1) return 0;
  if (NL * 4 * H > 512 || gridb != B) return 0;
  const int lanes = H == 16 ? pdrnn::bwd_gs_lanes<16>(NL) : pdrnn::bwd_gs_lanes<32>(NL);
  return lanes == 4 ? 1 : 0;
}

// Fused forward + head/CE + BPTT launch of the latency regime (see
// lstm_small_step_gs_kernel); H in {16, 32}.
hipError_t pdrnn_lstm_small_step(const PdrnnLstmSmallFwdArgs* f, const PdrnnLstmSmallBwdArgs* b, int H,
                                 hipStream_t stream) {
  if (f->x_bf16 && (size_t)f->T * H * sizeof(float) > (size_t)pdrnn::kXldsBytes) return hipErrorInvalidConfiguration;
  switch (H) {
    case 16: return pdrnn::launch_step_gs<16>(f, b, stream);
    case 32: return pdrnn::launch_step_gs<32>(f, b, stream);
    default: return hipErrorInvalidValue;
  }
}

int pdrnn_lstm_small_supported(int H, int I, int NL) {
  const bool h_ok = H == 16 || H == 32 || H == 64;
  if (!h_ok || I < 1 || I > H || NL < 1 || NL > PDRNN_MAX_LAYERS) return 0;
  const int s_min = H == 32 ? 2 : 4;   // smallest valid forward split
  const int s2_min = H == 64 ? 4 : 2;  // smallest valid backward split
  return (NL * H * s_min <= 512 && NL * 2 * H * s2_min <= 512) ? 1 : 0;
}

// Largest split whose workgroup fits: more lanes per unit = shorter
// per-timestep critical path (latency-bound small batches); the host may
// request a smaller one for throughput-bound large batches.
int pdrnn_lstm_small_max_split(int H, int NL, int backward) {
  if (backward) {
    if (NL * H * (H >= 64 ? 8 : 4) <= 512) return 1;  // unit-group map
    if (NL * 4 * H <= 512 && (2 * H) % 16 == 0) return 2;  // 2-slice row split
    return 0;
  }
  if (NL * 4 * H <= 512) return 1;  // gate-split map
  if (NL * H * 2 <= 512 && (H * 2) % 64 == 0) return 2;  // 2-lane K split
  return 0;
}

int pdrnn_lstm_small_grid(int H, int B, int nb) {
  (void)H;
  return (B + nb - 1) / nb;
}

hipError_t pdrnn_lstm_small_fwd(const PdrnnLstmSmallFwdArgs* a, int H, int nb, int split, int save,
                                hipStream_t stream) {
  // bf16 inputs are widened while staging x into LDS: needs the LDS-resident x path
  if (a->x_bf16 && (size_t)a->T * H * sizeof(float) * (nb > 1 ? nb : 1) > (size_t)pdrnn::kXldsBytes)
    return hipErrorInvalidConfiguration;
  switch (H) {
    case 16: return pdrnn::dispatch_fwd<16>(a, nb, split, save, stream);
    case 32: return pdrnn::dispatch_fwd<32>(a, nb, split, save, stream);
    case 64: return pdrnn::dispatch_fwd<64>(a, nb, split, save, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t pdrnn_lstm_small_bwd(const PdrnnLstmSmallBwdArgs* a, int H, int nb, int split, int grid,
                                hipStream_t stream) {
  if (a->x_bf16 && (split != 1 || (size_t)a->T * H * sizeof(float) * (nb > 1 ? nb : 1) > (size_t)pdrnn::kXldsBytes))
    return hipErrorInvalidConfiguration;
  switch (H) {
    case 16: return pdrnn::dispatch_bwd<16>(a, nb, split, stream, grid);
    case 32: return pdrnn::dispatch_bwd<32>(a, nb, split, stream, grid);
    case 64: return pdrnn::dispatch_bwd<64>(a, nb, split, stream, grid);
    default: return hipErrorInvalidValue;
  }
}

// Slab rows (= grid) the backward will use for (H, NL, T, B, split).
int pdrnn_lstm_small_bwd_grid(int H, int NL, int T, int B, int nb, int split) {
  if (split != 1) return (B + nb - 1) / nb;
  PdrnnLstmSmallBwdArgs a{};
  a.NL = NL; a.T = T; a.B = B;
#define BWD_GRID_CASE(HH, LL)                                   \
  switch (nb) {                                                  \
    case 1: return pdrnn::bwd_gs_grid<HH, LL, 1>(&a);            \
    case 2: return pdrnn::bwd_gs_grid<HH, LL, 2>(&a);            \
    case 3: return pdrnn::bwd_gs_grid<HH, LL, 3>(&a);            \
    default: return -1;                                          \
  }
  switch (H) {
    case 16:
      if (pdrnn::bwd_gs_lanes<16>(NL) == 8) { BWD_GRID_CASE(16, 8) }
      BWD_GRID_CASE(16, 4)
    case 32:
      if (pdrnn::bwd_gs_lanes<32>(NL) == 8) { BWD_GRID_CASE(32, 8) }
      BWD_GRID_CASE(32, 4)
    case 64:
      if (nb != 1) return -1;
      return pdrnn::bwd_gs_grid<64, 8, 1>(&a);
    default: return -1;
  }
#undef BWD_GRID_CASE
}

hipError_t pdrnn_slab_reduce(const float* slab, int64_t rows, int64_t P, float* out, float beta,
                             float* work, int split, hipStream_t stream) {
  if (split < 1) split = 1;
  if (split > 64) split = 64;
  if (split > rows) split = (int)rows > 0 ? (int)rows : 1;
  const int threads = 256;
  dim3 g1((unsigned)((P + threads - 1) / threads), (unsigned)split);
  hipLaunchKernelGGL(pdrnn::slab_reduce_pass1, g1, dim3(threads), 0, stream, slab, rows, P, work, split);
  PDRNN_HIP_CHECK(hipGetLastError());
  dim3 g2((unsigned)((P + threads - 1) / threads));
  hipLaunchKernelGGL(pdrnn::slab_reduce_pass2, g2, dim3(threads), 0, stream, work, P, split, out, beta);
  return hipGetLastError();
}

hipError_t pdrnn_slab_reduce2(const float* slab, int64_t rows, int64_t P, int64_t P_a, float* out_a,
                              float* out_b, float* work, int split, hipStream_t stream) {
  if (split < 1) split = 1;
  if (split > 64) split = 64;
  if (split > rows) split = (int)rows > 0 ? (int)rows : 1;
  const int threads = 256;
  dim3 g1((unsigned)((P + threads - 1) / threads), (unsigned)split);
  hipLaunchKernelGGL(pdrnn::slab_reduce_pass1, g1, dim3(threads), 0, stream, slab, rows, P, work, split);
  PDRNN_HIP_CHECK(hipGetLastError());
  dim3 g2((unsigned)((P + threads - 1) / threads));
  hipLaunchKernelGGL(pdrnn::slab_reduce_pass2_split, g2, dim3(threads), 0, stream, work, P, P_a, split, out_a, out_b);
  return hipGetLastError();
}

hipError_t pdrnn_slab2_reduce_pass1(const float* A, int64_t rowsA, int64_t PA, const float* Bs, int64_t rowsB,
                                   int64_t PB, float* work, int split, const int* colmap, int64_t ldA,
                                   hipStream_t stream) {
  if (split < 1) split = 1;
  if (split > 64) split = 64;
  const int64_t P = PA + PB;
  const int threads = 256;
  dim3 g1((unsigned)((P + threads - 1) / threads), (unsigned)split);
  hipLaunchKernelGGL(pdrnn::slab2_reduce_pass1, g1, dim3(threads), 0, stream, A, rowsA, PA, Bs, rowsB, PB, work, split,
                     colmap, colmap ? ldA : PA);
  return hipGetLastError();
}

hipError_t pdrnn_slab2_reduce(const float* A, int64_t rowsA, int64_t PA, const float* Bs, int64_t rowsB, int64_t PB,
                              int64_t n_out, float* out, float* out_tail, float* work, int split, const int* colmap,
                              int64_t ldA, hipStream_t stream) {
  if (split < 1) split = 1;
  if (split > 64) split = 64;
  const int64_t P = PA + PB;
  const int threads = 256;
  dim3 g1((unsigned)((P + threads - 1) / threads), (unsigned)split);
  hipLaunchKernelGGL(pdrnn::slab2_reduce_pass1, g1, dim3(threads), 0, stream, A, rowsA, PA, Bs, rowsB, PB, work, split,
                     colmap, colmap ? ldA : PA);
  PDRNN_HIP_CHECK(hipGetLastError());
  dim3 g2((unsigned)((P + threads - 1) / threads));
  hipLaunchKernelGGL(pdrnn::slab_reduce_pass2_split, g2, dim3(threads), 0, stream, work, P, n_out, split, out, out_tail);
  return hipGetLastError();
}

}  // extern "C"
