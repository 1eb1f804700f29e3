// Weight gradients of the fused small-H LSTM/GRU stack on the fp32 matrix cores.
//
// The reference's backward (src/motion/trainer/base.py:116 -> ATen LSTM
// backward for nn.LSTM at src/motion/model.py:9) forms, per layer,
//   dW_ih = sum_{b,t} dgates_t^T x_t,   dW_hh = sum_{b,t} dgates_t^T h_{t-1},
//   db    = sum_{b,t} dgates_t.
// The lean BPTT (lstm_small.hip, DWOUT) leaves the gate gradients in memory;
// this kernel does the three reductions over K = B*T rows with
// v_mfma_f32_16x16x4_f32 (exact fp32 products and accumulation: the same
// numerics as a k-ordered fmaf chain, SURVEY.md §2b N1 "MFMA GEMMs for dW").
//
// Mapping (one workgroup per (K chunk, layer); one wave per 16-column output
// tile of [in | h_prev]; every wave holds ALL 4H gate rows of its columns):
//   * K step = 4 consecutive (b,t) rows; lane (i = lane & 15, kk = lane >> 4)
//     handles row kk of the step.
//   * A operand (gate gradients): one float4 per 64 gates, read straight from
//     the row (coalesced 256 B per row quarter): component c of the float4 at
//     gate 64g + 4i is the A fragment of the "virtual" m-tile (g, c) whose MFMA
//     row i is gate 64g + 4i + c -- 4 m-tiles per load, no LDS, no transpose.
//   * B operand: element 16 c0 + i of the row's input (x, as the gathered fp32
//     rows the BPTT wrote while staging them, or the layer below's h_t) or of
//     h_{t-1} (zero at t = 0).
//   * C tile (g, c) of lane l: rows 4(l >> 4) + r -> gate 64g + 16(l >> 4) + 4r
//     + c, column l & 15.
//   * The waves of a workgroup re-read the same gate-gradient rows (L1/L2
//     hits); HBM sees each byte once.
//   * db: the first h_prev wave also sums its A fragments on the VALU (free
//     beside the MFMAs) and reduces them over the 4 row lanes at the end.
//   * Operands reach LDS by DMA (global_load_lds, no VGPR staging): a ring
//     of 16-row stages (dw_rows, small_dw.h), stages in flight past the one being consumed,
//     retired by a counted vmcnt + raw barrier (a __syncthreads() would drain
//     the ring); every wave issues an equal share of a stage's DMA jobs.
// Chunk c writes its partial sums to slab row c; pdrnn_slab_reduce_adam sums
// the rows in a fixed order (deterministic) and applies Adam.
#include "pdrnn/api.h"
#include "pdrnn/common.h"
#include "pdrnn/small_dw.h"

namespace pdrnn {
namespace {

// grid (chunks, NL): one workgroup per (K chunk, layer)
template <int H>
__global__ void __launch_bounds__(512) lstm_small_dw_kernel(PdrnnLstmSmallDwArgs a) {
  const int64_t BT = (int64_t)a.B * a.T;
  constexpr int RW = dw_rows<H>();
  const int nstage_all = (int)((BT + RW - 1) / RW);
  const int st0 = (int)((int64_t)nstage_all * blockIdx.x / a.chunks);
  const int st1 = (int)((int64_t)nstage_all * (blockIdx.x + 1) / a.chunks);
  const int64_t k_end = min((int64_t)st1 * RW, BT);
  if (blockIdx.y == 0) lstm_small_dw_range<H, true>(a, 0, st0, st1, k_end, blockIdx.x);
  else lstm_small_dw_range<H, false>(a, blockIdx.y, st0, st1, k_end, blockIdx.x);
}
template <int H>
hipError_t launch_dw(const PdrnnLstmSmallDwArgs* a, hipStream_t st) {
  const size_t lds = sizeof(float) * (size_t)dw_stages<H>() * dw_stage_floats<H>();
  const int nw0 = (a->I + 15) / 16 + H / 16, nw1 = 2 * (H / 16);
  constexpr int RW = dw_rows<H>();
  const int jobs0 = RW * H / 64 + RW * H / 256 + (RW * a->xg_ld + 255) / 256, jobs1 = RW * H / 64 + 2 * (RW * H / 256);
  const int jpw0 = (jobs0 + nw0 - 1) / nw0, jpw1 = (jobs1 + nw1 - 1) / nw1;
  constexpr int ahead = dw_stages<H>() - 2;  // stages each wave keeps in flight past the one it waits for
  if (ahead * jpw0 > 16 || ahead * jpw1 > 16 || jpw0 > 8 || jpw1 > 8) return hipErrorInvalidConfiguration;
  const int nw = a->NL > 1 && nw1 > nw0 ? nw1 : nw0;
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)lstm_small_dw_kernel<H>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((lstm_small_dw_kernel<H>), dim3((unsigned)a->chunks, (unsigned)a->NL), dim3(64 * nw), lds, st, *a);
  return hipGetLastError();
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_lstm_small_dw_chunks(int H, int NL, int B, int T) {
  (void)NL;
  const int rw = H >= 64 ? pdrnn::dw_rows<64>() : pdrnn::dw_rows<32>();
  const int64_t stages = ((int64_t)B * T + rw - 1) / rw;
  int64_t c = 256;
  if (c > stages / 4) c = stages / 4;  // at least 4 stages per chunk (amortise the pipeline fill)
  if (c < 1) c = 1;
  return (int)c;
}

hipError_t pdrnn_lstm_small_dw(const PdrnnLstmSmallDwArgs* a, int H, hipStream_t stream) {
  if (a->T < 4 || a->chunks < 1 || a->NL < 1 || a->NL > PDRNN_MAX_LAYERS || a->I < 1 || a->I > H || !a->xg ||
      a->xg_ld < a->I || a->xg_ld % 4 != 0 || a->dg_st % 4 != 0)
    return hipErrorInvalidValue;
  switch (H) {
    case 16: return pdrnn::launch_dw<16>(a, stream);
    case 32: return pdrnn::launch_dw<32>(a, stream);
    case 64: return pdrnn::launch_dw<64>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // extern "C"
