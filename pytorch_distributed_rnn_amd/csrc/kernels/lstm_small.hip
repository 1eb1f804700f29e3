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

namespace pdrnn {
namespace {

template <int H, int S, int NB, bool SAVE>
__global__ void __launch_bounds__(512) lstm_small_fwd_kernel(PdrnnLstmSmallFwdArgs a) {
  constexpr int K = 2 * H;
  constexpr int KS = K / S;
  constexpr int LANES = H * S;
  static_assert(KS % 4 == 0, "K slice must be float4 aligned");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int NL = a.NL, B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const int layer = __builtin_amdgcn_readfirstlane(tid / LANES);
  const int lg = tid - layer * LANES;
  const int u = lg / S;
  const int s = lg % S;
  const int bbase = blockIdx.x * NB;
  const int Iin = layer == 0 ? I : H;

  // vin[n][l][p][k]: k < H layer input, k >= H own hidden state.
  auto vin = [&](int n, int l, int p) -> float* { return smem + ((n * NL + l) * 2 + p) * K; };

  // ---- weights for this lane: rows q*H+u, columns s*KS .. s*KS+KS-1 -------
  float w[4][KS];
  float bias[4];
  {
    const float* Wih = a.w_ih[layer];
    const float* Whh = a.w_hh[layer];
    const float* Bih = a.b_ih[layer];
    const float* Bhh = a.b_hh[layer];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = q * H + u;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const int k = s * KS + kk;
        float v;
        if (k < H) v = k < Iin ? Wih[r * Iin + k] : 0.f;
        else v = Whh[r * H + (k - H)];
        w[q][kk] = v;
      }
      bias[q] = (Bih ? Bih[r] : 0.f) + (Bhh ? Bhh[r] : 0.f);
    }
  }

  int bsrc[NB];
  bool valid[NB];
  float c[NB], hl[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    valid[n] = b < B;
    bsrc[n] = valid[n] ? (a.idx ? (int)a.idx[b] : b) : 0;
    const float h_init = (a.h0 && valid[n]) ? a.h0[((int64_t)layer * B + b) * H + u] : 0.f;
    c[n] = (a.c0 && valid[n]) ? a.c0[((int64_t)layer * B + b) * H + u] : 0.f;
    hl[n] = h_init;
    if (s == 0) vin(n, layer, 0)[H + u] = h_init;
    if (layer == 0 && lg < H)
      vin(n, 0, 0)[lg] = (valid[n] && lg < I) ? a.x[bsrc[n] * a.x_sb + lg] : 0.f;
  }
  __syncthreads();

  const int iters = T + NL - 1;
  for (int it = 0; it < iters; ++it) {
    const int t = it - layer;
    if (t >= 0 && t < T) {
      const int p = t & 1;
      float xnext[NB];
      if (layer == 0 && lg < H) {
#pragma unroll
        for (int n = 0; n < NB; ++n)
          xnext[n] = (t + 1 < T && valid[n] && lg < I)
                         ? a.x[bsrc[n] * a.x_sb + (int64_t)(t + 1) * a.x_st + lg]
                         : 0.f;
      }
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const float4* v4 = reinterpret_cast<const float4*>(vin(n, layer, p) + s * KS);
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k4 = 0; k4 < KS / 4; ++k4) {
          const float4 v = v4[k4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            acc[q] = fmaf(w[q][4 * k4 + 0], v.x, acc[q]);
            acc[q] = fmaf(w[q][4 * k4 + 1], v.y, acc[q]);
            acc[q] = fmaf(w[q][4 * k4 + 2], v.z, acc[q]);
            acc[q] = fmaf(w[q][4 * k4 + 3], v.w, acc[q]);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = group_sum<S>(acc[q]) + bias[q];
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
      if (layer == 0 && lg < H) {
#pragma unroll
        for (int n = 0; n < NB; ++n) vin(n, 0, p ^ 1)[lg] = xnext[n];
      }
    }
    __syncthreads();
  }

#pragma unroll
  for (int n = 0; n < NB; ++n) {
    const int b = bbase + n;
    if (valid[n] && s == 0) {
      a.hn[((int64_t)layer * B + b) * H + u] = hl[n];
      a.cn[((int64_t)layer * B + b) * H + u] = c[n];
    }
  }
}

template <int H, int S2, int NB>
__global__ void __launch_bounds__(512) lstm_small_bwd_kernel(PdrnnLstmSmallBwdArgs a) {
  constexpr int R = 4 * H;        // gate rows
  constexpr int K = 2 * H;        // columns of [W_ih | W_hh] (input padded to H)
  constexpr int RS = R / S2;      // rows per column lane
  constexpr int G = K * S2;       // lanes per layer group
  static_assert(G >= R, "S2 must be >= 2");
  static_assert(RS % 4 == 0, "row slice must be float4 aligned");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int NL = a.NL, B = a.B, T = a.T, I = a.I;
  const int tid = threadIdx.x;
  const int layer = __builtin_amdgcn_readfirstlane(tid / G);
  const int lg = tid - layer * G;
  const int bbase = blockIdx.x * NB;
  const int Iin = layer == 0 ? I : H;

  // LDS carve: dg[NB][NL][R] | dhrec[NB][NL][H] | dha[NB][NL][H]
  float* dg_s = smem;
  float* dhrec_s = dg_s + NB * NL * R;
  float* dha_s = dhrec_s + NB * NL * H;
  auto dg = [&](int n, int l) { return dg_s + (n * NL + l) * R; };
  auto dhrec = [&](int n, int l) { return dhrec_s + (n * NL + l) * H; };
  auto dha = [&](int n, int l) { return dha_s + (n * NL + l) * H; };

  // Row role.
  const bool is_row = lg < R;
  const int q = lg / H;
  const int u = lg % H;
  // Column role.
  const int k = lg / S2;
  const int s2 = lg % S2;

  float W[RS], dW[RS];
  {
    const float* Wih = a.w_ih[layer];
    const float* Whh = a.w_hh[layer];
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      const int r = s2 * RS + j;
      float v;
      if (k < H) v = k < Iin ? Wih[r * Iin + k] : 0.f;
      else v = Whh[r * H + (k - H)];
      W[j] = v;
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
    dc[n] = (is_row && a.dcn && valid[n]) ? a.dcn[((int64_t)layer * B + b) * H + u] : 0.f;
    if (lg < H) {
      dhrec(n, layer)[lg] = (a.dhn && valid[n]) ? a.dhn[((int64_t)layer * B + b) * H + lg] : 0.f;
      dha(n, layer)[lg] = 0.f;
    }
  }
  __syncthreads();

  const int iters = T + NL - 1;
  for (int it = 0; it < iters; ++it) {
    const int t = T - 1 - it + (NL - 1 - layer);
    const bool active = t >= 0 && t < T;
    // ---------------- row phase: dgates ----------------
    if (active && is_row) {
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        float dgv = 0.f;
        if (valid[n]) {
          const int b = bbase + n;
          const int64_t row = ((int64_t)layer * B + b) * T + t;
          const float* act = a.act + row * 5 * H;
          const float ig = act[0 * H + u], fg = act[1 * H + u], gg = act[2 * H + u],
                      og = act[3 * H + u], ct = act[4 * H + u];
          float cp;
          if (t > 0) cp = act[-5 * H + 4 * H + u];
          else cp = a.c0 ? a.c0[((int64_t)layer * B + b) * H + u] : 0.f;
          float dh = dhrec(n, layer)[u];
          if (layer < NL - 1) dh += dha(n, layer)[u];
          else if (a.dout) dh += a.dout[b * a.d_sb + (int64_t)t * a.d_st + u];
          const float tc = tanhf_fast(ct);
          const float dcp = fmaf(dh * og, 1.f - tc * tc, dc[n]);
          const float d_i = dcp * gg * ig * (1.f - ig);
          const float d_f = dcp * cp * fg * (1.f - fg);
          const float d_g = dcp * ig * (1.f - gg * gg);
          const float d_o = dh * tc * og * (1.f - og);
          dgv = q == 0 ? d_i : (q == 1 ? d_f : (q == 2 ? d_g : d_o));
          dc[n] = dcp * fg;
        }
        dg(n, layer)[lg] = dgv;
        db += dgv;
      }
    }
    __syncthreads();
    // ---------------- column phase: dh_{t-1}, d(input), dW ----------------
    if (active) {
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        const int b = bbase + n;
        float in = 0.f;
        if (valid[n]) {
          if (k < H) {
            if (layer == 0) {
              if (k < I) in = a.x[bsrc[n] * a.x_sb + (int64_t)t * a.x_st + k];
            } else {
              in = a.hseq[(((int64_t)(layer - 1) * B + b) * T + t) * H + k];
            }
          } else {
            const int kh = k - H;
            if (t > 0) in = a.hseq[(((int64_t)layer * B + b) * T + (t - 1)) * H + kh];
            else if (a.h0) in = a.h0[((int64_t)layer * B + b) * H + kh];
          }
        }
        const float4* g4 = reinterpret_cast<const float4*>(dg(n, layer) + s2 * RS);
        float ds0 = 0.f, ds1 = 0.f;
#pragma unroll
        for (int j4 = 0; j4 < RS / 4; ++j4) {
          const float4 g = g4[j4];
          ds0 = fmaf(W[4 * j4 + 0], g.x, ds0);
          ds1 = fmaf(W[4 * j4 + 1], g.y, ds1);
          ds0 = fmaf(W[4 * j4 + 2], g.z, ds0);
          ds1 = fmaf(W[4 * j4 + 3], g.w, ds1);
          dW[4 * j4 + 0] = fmaf(g.x, in, dW[4 * j4 + 0]);
          dW[4 * j4 + 1] = fmaf(g.y, in, dW[4 * j4 + 1]);
          dW[4 * j4 + 2] = fmaf(g.z, in, dW[4 * j4 + 2]);
          dW[4 * j4 + 3] = fmaf(g.w, in, dW[4 * j4 + 3]);
        }
        const float ds = group_sum<S2>(ds0 + ds1);
        if (s2 == 0) {
          if (k >= H) {
            dhrec(n, layer)[k - H] = ds;
          } else if (layer > 0) {
            dha(n, layer - 1)[k] = ds;
          } else if (a.dx && valid[n] && k < I) {
            a.dx[b * a.dx_sb + (int64_t)t * a.dx_st + k] = ds;
          }
        }
      }
    }
    __syncthreads();
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
#pragma unroll
  for (int j = 0; j < RS; ++j) {
    const int r = s2 * RS + j;
    if (k < H) {
      if (k < Iin) slab[a.off_wih[layer] + (int64_t)r * Iin + k] = dW[j];
    } else {
      slab[a.off_whh[layer] + (int64_t)r * H + (k - H)] = dW[j];
    }
  }
  if (is_row) {
    if (a.off_bih[layer] >= 0) slab[a.off_bih[layer] + lg] = db;
    if (a.off_bhh[layer] >= 0) slab[a.off_bhh[layer] + lg] = db;
  }
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

template <int H, int S, int NB, bool SAVE>
hipError_t launch_fwd(const PdrnnLstmSmallFwdArgs* a, hipStream_t st) {
  constexpr int LANES = H * S;
  const int grid = (a->B + NB - 1) / NB;
  const int block = a->NL * LANES;
  const size_t lds = sizeof(float) * NB * a->NL * 2 * (2 * H);
  hipLaunchKernelGGL((lstm_small_fwd_kernel<H, S, NB, SAVE>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

template <int H, int S2, int NB>
hipError_t launch_bwd(const PdrnnLstmSmallBwdArgs* a, hipStream_t st) {
  constexpr int G = 2 * H * S2;
  const int grid = (a->B + NB - 1) / NB;
  const int block = a->NL * G;
  const size_t lds = sizeof(float) * NB * a->NL * (4 * H + 2 * H);
  hipLaunchKernelGGL((lstm_small_bwd_kernel<H, S2, NB>), dim3(grid), dim3(block), lds, st, *a);
  return hipGetLastError();
}

// Forward split S per hidden size: lanes per layer = H*S must be a multiple of
// 64 and 4*2H/S weight registers must stay <= 128.
template <int H> struct FwdSplit;
template <> struct FwdSplit<16> { static constexpr int S = 4; };
template <> struct FwdSplit<32> { static constexpr int S = 2; };
template <> struct FwdSplit<64> { static constexpr int S = 4; };
// Backward split S2: lanes per layer = 2H*S2, rows per column lane 4H/S2.
template <int H> struct BwdSplit;
template <> struct BwdSplit<16> { static constexpr int S2 = 2; };
template <> struct BwdSplit<32> { static constexpr int S2 = 2; };
template <> struct BwdSplit<64> { static constexpr int S2 = 4; };

template <int H>
hipError_t dispatch_fwd(const PdrnnLstmSmallFwdArgs* a, int nb, int save, hipStream_t st) {
  constexpr int S = FwdSplit<H>::S;
  if (save) {
    if (nb == 1) return launch_fwd<H, S, 1, true>(a, st);
    if (nb == 2) return launch_fwd<H, S, 2, true>(a, st);
    if (nb == 4) return launch_fwd<H, S, 4, true>(a, st);
  } else {
    if (nb == 1) return launch_fwd<H, S, 1, false>(a, st);
    if (nb == 2) return launch_fwd<H, S, 2, false>(a, st);
    if (nb == 4) return launch_fwd<H, S, 4, false>(a, st);
  }
  return hipErrorInvalidValue;
}

template <int H>
hipError_t dispatch_bwd(const PdrnnLstmSmallBwdArgs* a, int nb, hipStream_t st) {
  constexpr int S2 = BwdSplit<H>::S2;
  if (nb == 1) return launch_bwd<H, S2, 1>(a, st);
  if (nb == 2) return launch_bwd<H, S2, 2>(a, st);
  if (nb == 4) return launch_bwd<H, S2, 4>(a, st);
  return hipErrorInvalidValue;
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_lstm_small_supported(int H, int I, int NL) {
  const bool h_ok = H == 16 || H == 32 || H == 64;
  if (!h_ok || I < 1 || I > H || NL < 1 || NL > PDRNN_MAX_LAYERS) return 0;
  // Workgroup size limit (1024 threads) for the backward: NL * 2H * S2.
  const int s2 = H == 64 ? 4 : 2;
  return NL * 2 * H * s2 <= 1024 ? 1 : 0;
}

int pdrnn_lstm_small_grid(int H, int B, int nb) {
  (void)H;
  return (B + nb - 1) / nb;
}

hipError_t pdrnn_lstm_small_fwd(const PdrnnLstmSmallFwdArgs* a, int H, int nb, int save,
                                hipStream_t stream) {
  switch (H) {
    case 16: return pdrnn::dispatch_fwd<16>(a, nb, save, stream);
    case 32: return pdrnn::dispatch_fwd<32>(a, nb, save, stream);
    case 64: return pdrnn::dispatch_fwd<64>(a, nb, save, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t pdrnn_lstm_small_bwd(const PdrnnLstmSmallBwdArgs* a, int H, int nb, hipStream_t stream) {
  switch (H) {
    case 16: return pdrnn::dispatch_bwd<16>(a, nb, stream);
    case 32: return pdrnn::dispatch_bwd<32>(a, nb, stream);
    case 64: return pdrnn::dispatch_bwd<64>(a, nb, stream);
    default: return hipErrorInvalidValue;
  }
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

}  // extern "C"
