// Fused softmax cross-entropy (mean over non-ignored rows) + accuracy.
//
// Replaces CrossEntropyLoss + argmax/eq/sum of the reference training step
// (reference: src/motion/trainer/base.py:15,112,114).
// One wave per row: max, sum-exp and the first-index argmax are reduced with
// wave64 shuffles; the unscaled gradient softmax(x) - onehot(y) is written in
// the same pass so the backward is a single scale by grad_out / n_valid.
// Block partials (loss, n_valid, n_correct) are summed by a second one-block
// pass in a fixed order -> bitwise reproducible loss.
#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {
namespace {

constexpr int kThreads = 256;
constexpr int kWavesPerBlock = kThreads / 64;

template <typename T>
__device__ __forceinline__ float load_as_f32(const T* p);
template <>
__device__ __forceinline__ float load_as_f32<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float load_as_f32<uint16_t>(const uint16_t* p) { return bf16_to_f32(*p); }
template <>
__device__ __forceinline__ float load_as_f32<_Float16>(const _Float16* p) { return (float)*p; }

template <typename T>
__global__ void __launch_bounds__(kThreads) xent_rows_kernel(PdrnnXentArgs a, int rows_per_block) {
  __shared__ float red[kWavesPerBlock][3];
  const T* logits = reinterpret_cast<const T*>(a.logits);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int64_t row0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t row1 = min(row0 + rows_per_block, a.N);
  float loss_acc = 0.f, valid_acc = 0.f, correct_acc = 0.f;
  for (int64_t row = row0 + wave; row < row1; row += kWavesPerBlock) {
    const T* x = logits + row * a.ld;
    const int64_t label = a.labels[row];
    PDRNN_DEVICE_ASSERT(label == a.ignore_index || (label >= 0 && label < a.C));
    // pass 1: max + first argmax
    float m = -INFINITY;
    int64_t am = a.C;
    for (int64_t c = lane; c < a.C; c += 64) {
      const float v = load_as_f32<T>(x + c);
      if (v > m || (v == m && c < am) || (v != v && m == m)) { m = v; am = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(m, o, 64);
      const int64_t oa = __shfl_xor(am, o, 64);
      if (om > m || (om == m && oa < am)) { m = om; am = oa; }
    }
    // pass 2: sum exp
    float s = 0.f;
    for (int64_t c = lane; c < a.C; c += 64) s += expf(load_as_f32<T>(x + c) - m);
    s = wave_sum(s);
    const float lse = m + logf(s);
    const bool valid = label != a.ignore_index && label >= 0 && label < a.C;
    if (a.dlogits) {
      float* d = a.dlogits + row * a.C;
      const float inv = 1.f / s;
      for (int64_t c = lane; c < a.C; c += 64) {
        float p = valid ? expf(load_as_f32<T>(x + c) - m) * inv : 0.f;
        if (valid && c == label) p -= 1.f;
        d[c] = p;
      }
    }
    float rl = 0.f;
    if (valid) rl = lse - load_as_f32<T>(x + label);
    if (lane == 0) {
      if (a.row_loss) a.row_loss[row] = rl;
      loss_acc += rl;
      valid_acc += valid ? 1.f : 0.f;
      correct_acc += (valid && am == label) ? 1.f : 0.f;
    }
  }
  if (lane == 0) {
    red[wave][0] = loss_acc;
    red[wave][1] = valid_acc;
    red[wave][2] = correct_acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float l = 0.f, v = 0.f, c = 0.f;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) { l += red[w][0]; v += red[w][1]; c += red[w][2]; }
    a.partial[blockIdx.x * 3 + 0] = l;
    a.partial[blockIdx.x * 3 + 1] = v;
    a.partial[blockIdx.x * 3 + 2] = c;
  }
}

__global__ void __launch_bounds__(256) xent_finalize_kernel(const float* partial, int nblocks, float* out) {
  __shared__ float red[3][256];
  float l = 0.f, v = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < nblocks; i += 256) {
    l += partial[i * 3 + 0];
    v += partial[i * 3 + 1];
    c += partial[i * 3 + 2];
  }
  red[0][threadIdx.x] = l;
  red[1][threadIdx.x] = v;
  red[2][threadIdx.x] = c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
      red[2][threadIdx.x] += red[2][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float nv = red[1][0];
    out[0] = nv > 0.f ? red[0][0] / nv : NAN;
    out[1] = nv;
    out[2] = red[2][0];
  }
}

// dst = src * (grad_out[0] / stats[1])
// OD: output 0 bf16, 1 fp16, 2 fp32 -- a 16-bit head takes its logits
// gradient in its own dtype straight from here (no separate cast dispatch)
template <int OD>
__global__ void xent_bwd_kernel(const float* __restrict__ src, const float* grad_out, const float* stats,
                                void* __restrict__ dst, int64_t n) {
  const float scale = grad_out[0] / stats[1];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = src[i] * scale;
    if constexpr (OD == 2) {
      static_cast<float*>(dst)[i] = v;
    } else if constexpr (OD == 1) {
      static_cast<uint16_t*>(dst)[i] = __builtin_bit_cast(uint16_t, (_Float16)v);
    } else {
      const uint32_t u = __float_as_uint(v);  // round to nearest even (finite inputs)
      static_cast<uint16_t*>(dst)[i] = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
  }
}

int rows_per_block_for(int64_t N, int64_t C) {
  // Enough blocks to fill the chip for large N; whole rows per wave.
  (void)C;
  int64_t rpb = (N + 1023) / 1024;
  if (rpb < kWavesPerBlock) rpb = kWavesPerBlock;
  if (rpb > 64) rpb = 64;
  return (int)rpb;
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int pdrnn_xent_partial_blocks(int64_t N, int64_t C) {
  const int rpb = pdrnn::rows_per_block_for(N, C);
  return (int)((N + rpb - 1) / rpb);
}

hipError_t pdrnn_xent_fwd(const PdrnnXentArgs* a, hipStream_t stream) {
  const int rpb = pdrnn::rows_per_block_for(a->N, a->C);
  const int nblocks = (int)((a->N + rpb - 1) / rpb);
  if (nblocks > 0) {
    switch (a->dtype) {
      case 0: hipLaunchKernelGGL(pdrnn::xent_rows_kernel<float>, dim3(nblocks), dim3(pdrnn::kThreads), 0, stream, *a, rpb); break;
      case 1: hipLaunchKernelGGL(pdrnn::xent_rows_kernel<uint16_t>, dim3(nblocks), dim3(pdrnn::kThreads), 0, stream, *a, rpb); break;
      case 2: hipLaunchKernelGGL(pdrnn::xent_rows_kernel<_Float16>, dim3(nblocks), dim3(pdrnn::kThreads), 0, stream, *a, rpb); break;
      default: return hipErrorInvalidValue;
    }
    PDRNN_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(pdrnn::xent_finalize_kernel, dim3(1), dim3(256), 0, stream, a->partial, nblocks, a->out);
  return hipGetLastError();
}

hipError_t pdrnn_xent_bwd(const float* dlogits, const float* grad_out, const float* stats, void* dst,
                          int64_t n, int out_dtype, hipStream_t stream) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  if (out_dtype == 0)
    hipLaunchKernelGGL(pdrnn::xent_bwd_kernel<0>, dim3(blocks), dim3(256), 0, stream, dlogits, grad_out, stats, dst, n);
  else if (out_dtype == 1)
    hipLaunchKernelGGL(pdrnn::xent_bwd_kernel<1>, dim3(blocks), dim3(256), 0, stream, dlogits, grad_out, stats, dst, n);
  else if (out_dtype == 2)
    hipLaunchKernelGGL(pdrnn::xent_bwd_kernel<2>, dim3(blocks), dim3(256), 0, stream, dlogits, grad_out, stats, dst, n);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // extern "C"
