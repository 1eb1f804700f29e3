// Row-owning recurrence for fp32 storage at H = 128 (the reference's
// precision with `--hidden-units 128`, reference src/motion/main.py:20-21,
// src/motion/model.py:9): one launch per layer pass, every workgroup owns 16
// batch rows and ALL 4H gate columns, so h_t of its rows depends only on its
// own h_{t-1} -- no grid synchronisation at all (unlike the persistent
// column-block kernels of lstm_large.hip, whose 8-wave K split and per-step
// grid sync cost more than the per-step kernels at this size:
// profiles/r4/h2/h2_persist_f32_cell*.json).
//
//   * 512 threads = 8 waves; the whole W_hh (512 x 128 fp32 = 256 KiB) lives
//     in registers as MFMA B fragments, 128 VGPRs per lane: forward, wave w
//     owns gate columns [64 w, 64 w + 64) (units 16 w .. 16 w + 15,
//     gate-interleaved) over the full K = H; backward, wave w owns units
//     [16 w, 16 w + 16) over the full K = 4H;
//   * fragments are 16-byte chunks of 4 consecutive k split over 4
//     v_mfma_f32_16x16x4_f32 (F32::mfma in lstm_large.hip: exact fp32
//     products, fp32 accumulation);
//   * h_{t-1} (forward) / dgates_t (backward) of the block's 16 rows are
//     double-buffered in LDS: one workgroup barrier per step;
//   * forward: the gate tile goes through a per-wave LDS patch so each lane
//     reads the 4 gates of its (row, unit) pairs as one float4 and runs the
//     cell with c in registers; backward: a lane's dh tile IS its (row, unit)
//     pairs, the cell backward runs straight from the accumulators.
// Same semantics (gate packing, GRU [r|z|n_x|n_h] cell, saved activations,
// gate-blocked dgates, dh0 / dc0) as lstm_large_persist_{fwd,bwd}_kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int RH = 128;           // hidden size covered
constexpr int RW = 8;             // waves
constexpr int RT = RW * 64;       // threads
constexpr int RLDH = RH + 4;      // h row stride in LDS (floats)
constexpr int RLDG = 4 * RH + 4;  // dgates row stride in LDS
constexpr int RLDP = 64 + 4;      // per-wave gate patch row stride

// the activations of the per-step / persistent kernels (common.h)
__device__ __forceinline__ float r_sigm(float x) { return sigmoidf_fast(x); }
__device__ __forceinline__ float r_tanh(float x) { return tanhf_fast(x); }

// 4 MFMAs over one 16-byte chunk: MFMA m takes component m of both operands
__device__ __forceinline__ f32x4 mfma4(const float4& a, const float4& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
}

template <int CELL>
__global__ void __launch_bounds__(RT) lstm_rows_f32_fwd_kernel(PdrnnLstmLargeStepArgs args) {
  __shared__ __attribute__((aligned(16))) float hl[2][16][RLDH];
  __shared__ __attribute__((aligned(16))) float gp[RW][16][RLDP];
  const int dir = blockIdx.y;
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const int B = args.B, T = args.T;
  const bool rev = args.reverse_mask & (1 << dir);
  const int r0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // W_hh (gate-interleaved rows) as B fragments: column n = 64 w + 16 ct + fr
  float4 wf[RH / 16][4];
  {
    const float* W = static_cast<const float*>(d.w);
#pragma unroll
    for (int kc = 0; kc < RH / 16; ++kc)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        wf[kc][ct] = *reinterpret_cast<const float4*>(W + (int64_t)(64 * w + 16 * ct + fr) * RH + kc * 16 + fq * 4);
  }
  // cell pairs of this lane: unit 16 w + (lane & 15), rows (lane >> 4) + 4 i
  const int ul = lane & 15, u = 16 * w + ul;
  int brow[4];
  float cst[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    brow[i] = min(r0 + (lane >> 4) + 4 * i, B - 1);
    cst[i] = d.c0 ? d.c0[(int64_t)brow[i] * RH + u] : 0.f;
  }
  // h_{t-1} of the first step
  for (int e = threadIdx.x; e < 16 * RH; e += RT) {
    const int row = e / RH, k = e - row * RH;
    const int b = min(r0 + row, B - 1);
    hl[0][row][k] = d.h0 ? static_cast<const float*>(d.h0)[(int64_t)b * RH + k] : 0.f;
  }
  float4 xpn[4];
  auto load_xp = [&](int t) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xpn[i] = *reinterpret_cast<const float4*>(static_cast<const float*>(d.xp) + (int64_t)t * d.xp_st +
                                                (int64_t)brow[i] * d.xp_sb + 4 * u);
  };
  load_xp(rev ? T - 1 : 0);
  __syncthreads();

  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = rev ? T - 1 - s : s;
    float4 xc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xc[i] = xpn[i];
    if (s + 1 < T) load_xp(rev ? t - 1 : t + 1);  // in flight during the MFMAs
    f32x4 acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (s > 0 || d.h0) {
#pragma unroll
      for (int kc = 0; kc < RH / 16; ++kc) {
        const float4 a = *reinterpret_cast<const float4*>(&hl[cur][fr][kc * 16 + fq * 4]);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc[ct] = mfma4(a, wf[kc][ct], acc[ct]);
      }
    }
    // gate tile -> this wave's patch [row][64 columns]: lane holds rows 4 fq + i, column 16 ct + fr
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int i = 0; i < 4; ++i) gp[w][4 * fq + i][16 * ct + fr] = acc[ct][i];
    // the wave's own patch: its LDS writes are done before any lane reads
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float* hn = &hl[cur ^ 1][0][0];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (lane >> 4) + 4 * i;
      const float4 p = *reinterpret_cast<const float4*>(&gp[w][row][4 * ul]);
      float z[4] = {xc[i].x + p.x, xc[i].y + p.y, xc[i].z + p.z, xc[i].w + p.w};
      float g[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if constexpr (CELL == 0) g[k] = k == 2 ? r_tanh(z[k]) : r_sigm(z[k]);
        else g[k] = k < 2 ? r_sigm(z[k]) : z[k];
      }
      float hv;
      if constexpr (CELL == 0) {
        cst[i] = fmaf(g[1], cst[i], g[0] * g[2]);
        hv = g[3] * r_tanh(cst[i]);
      } else {
        g[2] = r_tanh(fmaf(g[0], g[3], g[2]));
        cst[i] = hv = fmaf(g[1], cst[i] - g[2], g[2]);
      }
      hn[row * RLDH + u] = hv;
      const int b = r0 + row;
      if (b < B) {
        const int64_t bu = (int64_t)b * RH + u;
        static_cast<float*>(d.hseq)[(int64_t)t * d.hseq_st + (int64_t)b * d.hseq_sb + u] = hv;
        *reinterpret_cast<float4*>(static_cast<float*>(d.acts) + (int64_t)t * B * 4 * RH + 4 * bu) =
            make_float4(g[0], g[1], g[2], g[3]);
        d.cseq[(int64_t)t * B * RH + bu] = cst[i];
      }
    }
    lds_barrier();  // h_t of every wave in LDS before the next step's reads (stores stay in flight)
    cur ^= 1;
  }
}

template <int CELL>
__global__ void __launch_bounds__(RT) lstm_rows_f32_bwd_kernel(PdrnnLstmLargeStepArgs args) {
  __shared__ __attribute__((aligned(16))) float dl[2][16][RLDG];
  const int dir = blockIdx.y;
  const PdrnnLstmLargeDir& d = args.dir[dir];
  const int B = args.B, T = args.T;
  const bool rev = args.reverse_mask & (1 << dir);
  const int r0 = blockIdx.x * 16;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  constexpr int KC = 4 * RH / 16;  // 32 chunk steps over K = 4H

  // W_hh^T (torch gate-blocked columns) as B fragments: unit n = 16 w + fr
  float4 wf[KC];
  {
    const float* Wt = static_cast<const float*>(d.wt);
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      wf[kc] = *reinterpret_cast<const float4*>(Wt + (int64_t)(16 * w + fr) * 4 * RH + kc * 16 + fq * 4);
  }
  // this lane's (row, unit) pairs = its accumulator tile: rows 4 fq + i, unit 16 w + fr
  const int u = 16 * w + fr;
  int brow[4];
  float carry[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    brow[i] = min(r0 + 4 * fq + i, B - 1);
    carry[i] = (CELL == 0 && d.dcn) ? d.dcn[(int64_t)brow[i] * RH + u] : 0.f;  // the dc_n flowing in
  }
  // next cell-backward operands: dout, the 4 saved gates, c_tn, c_{tn-1}
  float nd[4], ncur[4], nsp[4];
  float4 nact[4];
  auto load_ops = [&](int tn) {
    const int tpp = rev ? tn + 1 : tn - 1;
    const bool has_prev = rev ? tpp < T : tpp >= 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t bu = (int64_t)brow[i] * RH + u;
      nd[i] = d.dout ? static_cast<const float*>(d.dout)[(int64_t)tn * d.dout_st + (int64_t)brow[i] * d.dout_sb + u]
                     : 0.f;
      nact[i] = *reinterpret_cast<const float4*>(static_cast<const float*>(d.acts) + (int64_t)tn * B * 4 * RH + 4 * bu);
      ncur[i] = CELL == 0 ? d.cseq[(int64_t)tn * B * RH + bu] : 0.f;
      nsp[i] = has_prev ? d.cseq[(int64_t)tpp * B * RH + bu] : (d.c0 ? d.c0[bu] : 0.f);
    }
  };
  // the cell backward of step tn for pair i: dgates_tn (gate-blocked) into
  // LDS (the next step's A operand) and global, the dc carry advanced
  auto cell_step = [&](int i, float dh, float dd, float4 act, float cc, float sp, float* dn, int tn) {
    const int row = 4 * fq + i;
    const int b = r0 + row;
    dh += dd;
    const float a0 = act.x, a1 = act.y, a2 = act.z, a3 = act.w;
    float g0, g1, g2, g3;
    if constexpr (CELL == 0) {
      const float tc = r_tanh(cc);
      const float dc = fmaf(dh * a3, 1.f - tc * tc, carry[i]);
      g0 = dc * a2 * a0 * (1.f - a0);
      g1 = dc * sp * a1 * (1.f - a1);
      g2 = dc * a0 * (1.f - a2 * a2);
      g3 = dh * tc * a3 * (1.f - a3);
      carry[i] = dc * a1;
    } else {
      const float dpn = dh * (1.f - a1) * (1.f - a2 * a2);
      g0 = dpn * a3 * a0 * (1.f - a0);
      g1 = dh * (sp - a2) * a1 * (1.f - a1);
      g2 = dpn;
      g3 = dpn * a0;
      carry[i] = dh * a1;
    }
    float* dr = dn + row * RLDG + u;
    dr[0] = g0; dr[RH] = g1; dr[2 * RH] = g2; dr[3 * RH] = g3;
    if (b < B) {
      float* o = static_cast<float*>(d.dgates) + (int64_t)tn * B * 4 * RH + (int64_t)b * 4 * RH + u;
      o[0] = g0; o[RH] = g1; o[2 * RH] = g2; o[3 * RH] = g3;
    }
  };
  // The first processed step (the layer's last forward step) has no
  // recurrent product: dh = dh_n.  Done here instead of a separate
  // lstm_large_bwd_first launch before this one (a dispatch per layer and
  // pipeline chunk on the fp32 hidden-128 model, profiles/r6/glue).
  const int t0 = rev ? 0 : T - 1, tn0 = rev ? t0 + 1 : t0 - 1;
  load_ops(t0);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    cell_step(i, d.dhn ? d.dhn[(int64_t)brow[i] * RH + u] : 0.f, nd[i], nact[i], ncur[i], nsp[i], &dl[0][0][0], t0);
  if (rev ? tn0 < T : tn0 >= 0) load_ops(tn0);
  __syncthreads();

  int cur = 0;
  for (int s = 0; s < T; ++s) {
    const int t = rev ? s : T - 1 - s;
    const int tn = rev ? t + 1 : t - 1;
    const bool cell = rev ? tn < T : tn >= 0;
    float od[4], ocur[4], osp[4];
    float4 oact[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { od[i] = nd[i]; ocur[i] = ncur[i]; osp[i] = nsp[i]; oact[i] = nact[i]; }
    if (cell) {  // operands of the next step's cell backward, in flight during the MFMAs
      const int tn2 = rev ? tn + 1 : tn - 1;
      if (rev ? tn2 < T : tn2 >= 0) load_ops(tn2);
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const float4 a = *reinterpret_cast<const float4*>(&dl[cur][fr][kc * 16 + fq * 4]);
      acc = mfma4(a, wf[kc], acc);
    }
    float* dn = &dl[cur ^ 1][0][0];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 4 * fq + i;
      const int b = r0 + row;
      float dh = acc[i];
      if constexpr (CELL == 1) dh += carry[i];
      if (!cell) {
        if (b < B) {
          const int64_t bu = (int64_t)b * RH + u;
          if (d.dh0) d.dh0[bu] = dh;
          if (CELL == 0 && d.dc0) d.dc0[bu] = carry[i];
        }
        continue;
      }
      cell_step(i, dh, od[i], oact[i], ocur[i], osp[i], dn, tn);
    }
    lds_barrier();  // dgates_tn of every wave in LDS before the next step's reads
    cur ^= 1;
  }
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_lstm_rows_f32_supported(int H, int dtype) { return dtype == 2 && H == pdrnn::RH; }

// One layer pass (ndir directions) of the row-owning fp32 recurrence.  The
// backward runs the first processed step's cell backward itself (from dhn /
// dcn; no pdrnn_lstm_large_bwd_first launch before it, unlike the persistent
// backward).
hipError_t pdrnn_lstm_rows_f32(const PdrnnLstmLargeStepArgs* a, int ndir, int backward, hipStream_t stream) {
  if (a->H != pdrnn::RH || ndir < 1 || ndir > 2 || a->B < 1 || a->T < 1) return hipErrorInvalidValue;
  if (a->cell != 0 && a->cell != 1) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((a->B + 15) / 16), (unsigned)ndir);
  if (backward) {
    if (a->cell) hipLaunchKernelGGL(pdrnn::lstm_rows_f32_bwd_kernel<1>, grid, dim3(pdrnn::RT), 0, stream, *a);
    else hipLaunchKernelGGL(pdrnn::lstm_rows_f32_bwd_kernel<0>, grid, dim3(pdrnn::RT), 0, stream, *a);
  } else {
    if (a->cell) hipLaunchKernelGGL(pdrnn::lstm_rows_f32_fwd_kernel<1>, grid, dim3(pdrnn::RT), 0, stream, *a);
    else hipLaunchKernelGGL(pdrnn::lstm_rows_f32_fwd_kernel<0>, grid, dim3(pdrnn::RT), 0, stream, *a);
  }
  return hipGetLastError();
}

}  // extern "C"
