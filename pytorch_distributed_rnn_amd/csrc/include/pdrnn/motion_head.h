// Fused classifier head + softmax cross-entropy of the motion training step,
// one wave per sequence, H = 32 (kernels/lstm_sw.hip).
#pragma once

#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {

// The head's operands of sequence b for lane unit u: the label (through the
// batch gather) and the head weights / biases.  Loaded by a caller ahead of
// the head (the single-layer forward's epilogue: the dependent index -> label
// loads of its two sequences in flight together instead of one after the
// other behind the first head's stores, profiles/r6/x_staging.md).
struct HeadIn {
  int64_t lab;
  float w[16], bias[16];
};
PDRNN_DEVICE HeadIn head_load(const PdrnnLstmSmallFwdArgs& a, int b, int u) {
  HeadIn in;
  in.lab = a.labels[a.idx ? a.idx[b] : b];
#pragma unroll
  for (int cc = 0; cc < 16; ++cc) {
    in.w[cc] = cc < a.C ? a.head_w[cc * 32 + u] : 0.f;
    in.bias[cc] = (cc < a.C && a.head_b) ? a.head_b[cc] : 0.f;
  }
  return in;
}

// Head + softmax-CE on h_T (lane (u, s) holds h_T[u]): logits, loss, argmax,
// dlogits; dW_head / db_head / [loss, 1, correct] into the sequence's head
// slab row, dL/dh_T into dh_top (the fused training step; reference loss:
// src/motion/trainer/base.py:15,112).
PDRNN_DEVICE void motion_head(const PdrnnLstmSmallFwdArgs& a, int b, float h, int u, bool odd, const HeadIn& in) {
  const int64_t lab = in.lab;
  const int C = a.C;
  float lg[16];
  float m = -INFINITY, logit_y = 0.f;
  int amax = 0;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc) {
    if (cc < C) {
      const float wv = in.w[cc];
      const float z = wave_sum(odd ? 0.f : wv * h) + in.bias[cc];
      lg[cc] = z;
      if (z > m) { m = z; amax = cc; }
      if (cc == lab) logit_y = z;
    }
  }
  float se = 0.f;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc)
    if (cc < C) se += expf(lg[cc] - m);
  const float lse = m + logf(se);
  const float inv_se = 1.f / se;
  const __amdgpu_buffer_rsrc_t r_slab = uniform_rsrc(a.slab);
  const uint32_t srow = (uint32_t)b * (uint32_t)a.slab_P;
  auto sst = [&](int e, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r_slab, (srow + (uint32_t)e) * 4u, 0, 0);
  };
  float dh = 0.f;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc) {
    if (cc < C) {
      const float d = (expf(lg[cc] - m) * inv_se - (cc == lab ? 1.f : 0.f)) * a.inv_batch;
      dh = fmaf(in.w[cc], d, dh);
      if (!odd) sst(a.head_off_w + cc * 32 + u, d * h);
      if (lane == 0 && a.head_b) sst(a.head_off_b + cc, d);
    }
  }
  if (!odd) a.dh_top[(int64_t)b * 32 + u] = dh;
  if (lane == 0) {
    sst(a.stat_off + 0, (lse - logit_y) * a.inv_batch);
    sst(a.stat_off + 1, 1.f);
    sst(a.stat_off + 2, amax == lab ? 1.f : 0.f);
  }
}

PDRNN_DEVICE void motion_head(const PdrnnLstmSmallFwdArgs& a, int b, float h, int u, bool odd) {
  motion_head(a, b, h, u, odd, head_load(a, b, u));
}

}  // namespace pdrnn
