// Fused classifier head + softmax cross-entropy of the motion training step,
// one wave per sequence, H = 32 (kernels/lstm_sw.hip).
#pragma once

#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {

// Head + softmax-CE on h_T (lane (u, s) holds h_T[u]): logits, loss, argmax,
// dlogits; dW_head / db_head / [loss, 1, correct] into the sequence's head
// slab row, dL/dh_T into dh_top (the fused training step; reference loss:
// src/motion/trainer/base.py:15,112).
PDRNN_DEVICE void motion_head(const PdrnnLstmSmallFwdArgs& a, int b, float h, int u, bool odd) {
  const int64_t lab = a.labels[a.idx ? a.idx[b] : b];
  const int C = a.C;
  float lg[16];
  float m = -INFINITY, logit_y = 0.f;
  int amax = 0;
#pragma unroll
  for (int cc = 0; cc < 16; ++cc) {
    if (cc < C) {
      const float wv = a.head_w[cc * 32 + u];
      const float z = wave_sum(odd ? 0.f : wv * h) + (a.head_b ? a.head_b[cc] : 0.f);
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
      dh = fmaf(a.head_w[cc * 32 + u], d, dh);
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

}  // namespace pdrnn
