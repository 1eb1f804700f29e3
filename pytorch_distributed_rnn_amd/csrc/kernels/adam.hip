// Fused Adam / AdamW step over ONE flat fp32 parameter buffer.
//
// Replaces torch 1.4's per-parameter Python loop of ATen ops that the
// reference runs every step (reference: src/motion/trainer/base.py:43,117;
// SURVEY.md §2b N5).  Models built by this framework keep all parameters,
// gradients and optimizer moments in contiguous flat buffers, so the whole
// optimizer step is a single streaming launch (16 B per lane, grid-stride).
// The update follows torch.optim.Adam's single-tensor formula term by term
// (lerp for exp_avg, addcmul for exp_avg_sq, sqrt(v)/sqrt(bc2)+eps,
// addcdiv by lr/bc1).  `grad_scale` folds the 1/world average of a sum
// all-reduce into the read of the gradient.
#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {
namespace {

struct AdamScalars {
  float lr, b1, b2, eps, wd, bc1, bc2_sqrt, gscale;
  int decoupled, maximize, amsgrad;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float* vmax,
                                          const AdamScalars& s) {
  g *= s.gscale;
  if (s.maximize) g = -g;
  if (s.wd != 0.f) {
    if (s.decoupled) p *= 1.f - s.lr * s.wd;
    else g = fmaf(s.wd, p, g);
  }
  // exp_avg.lerp_(grad, 1 - beta1)   (weight < 0.5 branch of torch's lerp)
  m = m + (1.f - s.b1) * (g - m);
  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1-beta2)
  v = v * s.b2 + (1.f - s.b2) * (g * g);
  float vv = v;
  if (s.amsgrad) { *vmax = fmaxf(*vmax, v); vv = *vmax; }
  const float denom = sqrtf(vv) / s.bc2_sqrt + s.eps;
  const float step_size = s.lr / s.bc1;
  p = p - step_size * (m / denom);
}

__global__ void __launch_bounds__(256) adam_flat_kernel(PdrnnAdamArgs a) {
  if (a.skip && *a.skip != 0) return;  // uniform: every workgroup reads the same word
  AdamScalars s;
  s.lr = a.lr_ptr ? *a.lr_ptr : a.lr;
  s.b1 = a.beta1; s.b2 = a.beta2; s.eps = a.eps; s.wd = a.weight_decay;
  const float st_new = a.step_advance ? *a.step_advance + 1.f : 0.f;
  if (a.step_advance) {
    s.bc1 = 1.f - powf(a.beta1, st_new);
    s.bc2_sqrt = sqrtf(1.f - powf(a.beta2, st_new));
  } else if (a.step_ptr) {
    const float st = *a.step_ptr;
    s.bc1 = 1.f - powf(a.beta1, st);
    s.bc2_sqrt = sqrtf(1.f - powf(a.beta2, st));
  } else {
    s.bc1 = a.bias_correction1;
    s.bc2_sqrt = a.bias_correction2_sqrt;
  }
  s.gscale = a.grad_scale; s.decoupled = a.decoupled; s.maximize = a.maximize;
  s.amsgrad = a.max_exp_avg_sq != nullptr;

  const int64_t n = a.n;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool aligned = ((reinterpret_cast<uintptr_t>(a.param) | reinterpret_cast<uintptr_t>(a.grad) |
                         reinterpret_cast<uintptr_t>(a.exp_avg) | reinterpret_cast<uintptr_t>(a.exp_avg_sq)) & 15) == 0 &&
                       !s.amsgrad;
  int64_t done = 0;
  if (aligned) {
    const int64_t n4 = n / 4;
    float4* P = reinterpret_cast<float4*>(a.param);
    const float4* Gr = reinterpret_cast<const float4*>(a.grad);
    float4* M = reinterpret_cast<float4*>(a.exp_avg);
    float4* V = reinterpret_cast<float4*>(a.exp_avg_sq);
    for (int64_t i = tid; i < n4; i += stride) {
      float4 p = P[i], m = M[i], v = V[i];
      const float4 g = Gr[i];
      adam_elem(p.x, g.x, m.x, v.x, nullptr, s);
      adam_elem(p.y, g.y, m.y, v.y, nullptr, s);
      adam_elem(p.z, g.z, m.z, v.z, nullptr, s);
      adam_elem(p.w, g.w, m.w, v.w, nullptr, s);
      P[i] = p; M[i] = m; V[i] = v;
    }
    done = n4 * 4;
  }
  for (int64_t i = done + tid; i < n; i += stride) {
    float p = a.param[i], m = a.exp_avg[i], v = a.exp_avg_sq[i];
    adam_elem(p, a.grad[i], m, v, s.amsgrad ? a.max_exp_avg_sq + i : nullptr, s);
    a.param[i] = p; a.exp_avg[i] = m; a.exp_avg_sq[i] = v;
  }
  if (a.step_advance) {
    // every workgroup read the old count above (it fed bc1/bc2); the last one
    // to arrive publishes the new count and re-arms the ticket for the next
    // launch (kernel-boundary visibility)
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(a.ticket, 1u) == gridDim.x - 1) {
      *a.step_advance = st_new;
      *a.ticket = 0u;
    }
  }
}

// Adam fused with the last reduction pass of the fused training step: the
// gradient of element i is the fixed-order sum of `split` partial rows
// (work[s][i], exactly the second pass of the deterministic slab reduction),
// written to grad_out and consumed in registers; the trailing n_stats
// columns are the batch statistics.  One launch instead of two, no
// gradient re-read.
__global__ void __launch_bounds__(256) adam_partials_kernel(PdrnnAdamArgs a, const float* __restrict__ work,
                                                            int split, int64_t P_total, float* __restrict__ grad_out,
                                                            float* __restrict__ stats_out, int n_stats) {
  AdamScalars s;
  s.lr = a.lr; s.b1 = a.beta1; s.b2 = a.beta2; s.eps = a.eps; s.wd = a.weight_decay;
  s.bc1 = a.bias_correction1; s.bc2_sqrt = a.bias_correction2_sqrt;
  s.gscale = a.grad_scale; s.decoupled = a.decoupled; s.maximize = a.maximize;
  s.amsgrad = 0;
  const int64_t n = a.n;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n + n_stats; i += stride) {
    // the split partial sums with 8 loads in flight (fixed order: deterministic)
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int sp = 0;
    for (; sp + 8 <= split; sp += 8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += work[(int64_t)(sp + k) * P_total + i];
    }
    for (int k = 0; sp < split; ++sp, ++k) acc[k] += work[(int64_t)sp * P_total + i];
    const float g = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    if (i < n) {
      grad_out[i] = g;
      float p = a.param[i], m = a.exp_avg[i], v = a.exp_avg_sq[i];
      adam_elem(p, g, m, v, nullptr, s);
      a.param[i] = p; a.exp_avg[i] = m; a.exp_avg_sq[i] = v;
    } else {
      stats_out[i - n] = g;
    }
  }
}

// One-pass column reduction of the fused step's two gradient slabs into the
// flat gradient, with the Adam update folded in (a.param != nullptr; the
// single-process step) -- replaces the two-pass reduction (slab2_reduce_pass1
// + adam_partials / slab_reduce_pass2_split) and one launch.
//   A: [rowsA, ldA] recurrent dW rows, one per backward workgroup, read
//      through colmap (GRU packed layout) when given;
//   B: [rowsB, PB] per-sequence head rows (head dW, db, [loss, n, correct]).
// A 1024-thread workgroup owns CW consecutive columns (one wave reads 64
// consecutive floats of a row: coalesced) and splits the rows over 1024 / CW
// row groups (A: 64 x 16, B: 16 x 64 -- the head slab has B rows over ~200
// columns), each thread keeps 8 loads in flight, and the row-group partials
// are summed in a fixed order through LDS (deterministic).
__global__ void __launch_bounds__(1024) slab_reduce_adam_kernel(
    PdrnnAdamArgs a, const float* __restrict__ A, int64_t rowsA, int64_t PA, int64_t ldA,
    const int* __restrict__ colmap, const float* __restrict__ Bs, int64_t rowsB, int64_t PB, int64_t n_out,
    float* __restrict__ grad_out, float* __restrict__ tail_out, int nblkA, const float* __restrict__ slot_step,
    int slot_offset, int ring_rows) {
  __shared__ float red[1024];
  const int tid = threadIdx.x;
  const bool inA = (int)blockIdx.x < nblkA;
  // a.step_advance (single-process graph replay): the step used is the
  // device count + 1, published by the last workgroup to arrive (ticket);
  // the count also names the statistics ring row (slot_step, same buffer)
  const float st_new = a.step_advance ? *a.step_advance + 1.f : 0.f;
  const int cw = inA ? 64 : 16;
  const int nrg = 1024 / cw;
  const int ci = tid % cw, rg = tid / cw;
  const int64_t col = inA ? (int64_t)blockIdx.x * 64 + ci : (int64_t)(blockIdx.x - nblkA) * 16 + ci;
  const bool live = col < (inA ? PA : PB);
  const int64_t p = inA ? col : PA + col;  // flat index: [A columns | B columns]
  // the Adam operands of this column first: their latency hides behind the
  // slab reads instead of adding a dependent round trip after the reduction
  const bool adam = a.param && tid < cw && live && p < n_out;
  float pv = 0.f, m = 0.f, v = 0.f;
  if (adam) { pv = a.param[p]; m = a.exp_avg[p]; v = a.exp_avg_sq[p]; }
  // 16 loads in flight per thread (a column's rows split over nrg groups)
  float acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = 0.f;
  if (live) {
    const float* src = inA ? A + (colmap ? colmap[col] : col) : Bs + col;
    const int64_t ld = inA ? ldA : PB;
    const int64_t rows = inA ? rowsA : rowsB;
    const int64_t r0 = rows * rg / nrg, r1 = rows * (rg + 1) / nrg;
    int64_t r = r0;
    for (; r + 16 <= r1; r += 16) {
#pragma unroll
      for (int k = 0; k < 16; ++k) acc[k] += src[(r + k) * ld];
    }
    for (int k = 0; r < r1; ++r, ++k) acc[k] += src[r * ld];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] += acc[k + 8];
  red[tid] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (tid < cw && live) {
  float g = 0.f;
  for (int k = 0; k < nrg; ++k) g += red[k * cw + tid];
  if (p < n_out) {
    grad_out[p] = g;
    if (adam) {
      AdamScalars s;
      s.lr = a.lr; s.b1 = a.beta1; s.b2 = a.beta2; s.eps = a.eps; s.wd = a.weight_decay;
      if (a.step_advance) {
        s.bc1 = 1.f - powf(a.beta1, st_new);
        s.bc2_sqrt = sqrtf(1.f - powf(a.beta2, st_new));
      } else {
        s.bc1 = a.bias_correction1; s.bc2_sqrt = a.bias_correction2_sqrt;
      }
      s.gscale = a.grad_scale; s.decoupled = a.decoupled; s.maximize = a.maximize;
      s.amsgrad = 0;
      adam_elem(pv, g, m, v, nullptr, s);
      a.param[p] = pv; a.exp_avg[p] = m; a.exp_avg_sq[p] = v;
    }
  } else {
    // tail (batch statistics): row ((int)*slot_step + slot_offset) mod
    // ring_rows of a [ring_rows, tail] ring when slot_step is given -- a
    // graph-replayed step then writes its statistics straight into the
    // epoch ring slot the host assigned it (no copy after the replay)
    int64_t row = 0;
    if (slot_step) {
      const int64_t r = ((int64_t)(*slot_step) + slot_offset) % ring_rows;
      row = r < 0 ? r + ring_rows : r;
    }
    const int64_t nt = PA + PB - n_out;
    tail_out[row * nt + p - n_out] = g;
  }
  }
  if (a.step_advance) {
    // every workgroup has read the old count (bias corrections, ring row)
    // before it arrives; the last one publishes the new count and re-arms
    // the ticket (kernel-boundary visibility for the next launch)
    __syncthreads();
    if (tid == 0 && atomicAdd(a.ticket, 1u) == gridDim.x - 1) {
      *a.step_advance = st_new;
      *a.ticket = 0u;
    }
  }
}

// Gradient-norm clipping of a flat fp32 gradient, deterministic and without
// a host sync: pass 1 -- per-workgroup sums of squares (each thread a fixed
// strided set, then a fixed LDS tree); pass 2 -- one workgroup sums the
// partials in order and writes scale = min(1, max_norm / (norm + eps)) (and
// the norm); pass 3 -- g *= scale.  The reference's trainers do not clip; the
// LM trainer does (train/lm.py).
__global__ void __launch_bounds__(256) sumsq_partial_kernel(const float* __restrict__ g, int64_t n,
                                                            float* __restrict__ part) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc = fmaf(g[i], g[i], acc);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) clip_finalize_kernel(const float* __restrict__ part, int nparts, float max_norm,
                                                            float eps, float* __restrict__ out) {
  __shared__ float red[256];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) acc += part[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0]);
    out[0] = fminf(max_norm / (norm + eps), 1.f);
    out[1] = norm;
  }
}

__global__ void __launch_bounds__(256) scale_flat_kernel(float* __restrict__ g, int64_t n, const float* __restrict__ scale) {
  const float s = scale[0];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) g[i] *= s;
}

}  // namespace
}  // namespace pdrnn

extern "C" hipError_t pdrnn_slab_reduce_adam(const PdrnnAdamArgs* a, const float* A, int64_t rowsA, int64_t PA,
                                            int64_t ldA, const int* colmap, const float* Bs, int64_t rowsB,
                                            int64_t PB, int64_t n_out, float* grad_out, float* tail_out,
                                            const float* slot_step, int slot_offset, int ring_rows,
                                            hipStream_t stream) {
  if (slot_step && ring_rows <= 0) return hipErrorInvalidValue;
  if (PA + PB <= 0) return hipSuccess;
  if (PA + PB > n_out && tail_out == nullptr) return hipErrorInvalidValue;
  PdrnnAdamArgs none{};
  const int nblkA = (int)((PA + 63) / 64);
  const int nblkB = (int)((PB + 15) / 16);
  hipLaunchKernelGGL(pdrnn::slab_reduce_adam_kernel, dim3((unsigned)(nblkA + nblkB)), dim3(1024), 0, stream,
                     a ? *a : none, A, rowsA, PA, ldA, colmap, Bs, rowsB, PB, n_out, grad_out, tail_out, nblkA,
                     slot_step, slot_offset, ring_rows);
  return hipGetLastError();
}

extern "C" hipError_t pdrnn_adam_partials(const PdrnnAdamArgs* a, const float* work, int split, int64_t P_total,
                                          float* grad_out, float* stats_out, int n_stats, hipStream_t stream) {
  const int64_t total = a->n + n_stats;
  if (total <= 0) return hipSuccess;
  // 64-thread blocks: one element per thread and enough workgroups to spread
  // a small model (14k parameters) over the CUs
  int64_t blocks = (total + 63) / 64;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pdrnn::adam_partials_kernel, dim3((unsigned)blocks), dim3(64), 0, stream, *a, work, split,
                     P_total, grad_out, stats_out, n_stats);
  return hipGetLastError();
}

extern "C" hipError_t pdrnn_clip_flat(float* g, int64_t n, float max_norm, float eps, float* work, int nparts,
                                      float* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (nparts < 1 || nparts > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pdrnn::sumsq_partial_kernel, dim3((unsigned)nparts), dim3(256), 0, stream, g, n, work);
  PDRNN_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(pdrnn::clip_finalize_kernel, dim3(1), dim3(256), 0, stream, work, nparts, max_norm, eps, out);
  PDRNN_HIP_CHECK(hipGetLastError());
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pdrnn::scale_flat_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, g, n, out);
  return hipGetLastError();
}

extern "C" hipError_t pdrnn_adam_flat(const PdrnnAdamArgs* a, hipStream_t stream) {
  if (a->n <= 0) return hipSuccess;
  int64_t blocks = (a->n / 4 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pdrnn::adam_flat_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, *a);
  return hipGetLastError();
}
