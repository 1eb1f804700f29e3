// Embedding lookup (gather) and deterministic backward (CSR segmented sum).
//
// New capability required by BASELINE config 4 (char-LM); the reference has no
// embedding (SURVEY.md §0 discrepancies table).  Forward: one wave per output
// row, 16 B per lane.  Backward: instead of float atomics (order-dependent
// rounding, ~1.3 TB/s chip-wide cap) the indices are stably sorted once on
// the host side of the op and each vocabulary row sums its contribution rows
// in a fixed order -> bitwise reproducible gradients, plain coalesced loads.
#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {
namespace {

__global__ void __launch_bounds__(256) emb_fwd_kernel(const float* __restrict__ w, const int64_t* __restrict__ idx,
                                                      float* __restrict__ out, int64_t n, int64_t dim,
                                                      int64_t V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const bool vec = (dim % 4) == 0;
  for (int64_t r = wave; r < n; r += nwaves) {
    int64_t v = idx[r];
    if (v < 0) v += V;
    PDRNN_DEVICE_ASSERT(v >= 0 && v < V);
    const float* src = w + v * dim;
    float* dst = out + r * dim;
    if (vec) {
      const float4* s4 = reinterpret_cast<const float4*>(src);
      float4* d4 = reinterpret_cast<float4*>(dst);
      for (int64_t c = lane; c < dim / 4; c += 64) d4[c] = s4[c];
    } else {
      for (int64_t c = lane; c < dim; c += 64) dst[c] = src[c];
    }
  }
}

// Gather with the cast to the 16-bit compute dtype fused in (bf16: dtype 0,
// fp16: dtype 1): the LSTM's input projection consumes it directly.
template <int DT>
__global__ void __launch_bounds__(256) emb_fwd16_kernel(const float* __restrict__ w, const int64_t* __restrict__ idx,
                                                        uint16_t* __restrict__ out, int64_t n, int64_t dim,
                                                        int64_t V) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < n; r += nwaves) {
    int64_t v = idx[r];
    if (v < 0) v += V;
    PDRNN_DEVICE_ASSERT(v >= 0 && v < V);
    const float* src = w + v * dim;
    uint16_t* dst = out + r * dim;
    for (int64_t c = lane; c < dim; c += 64) {
      const float f = src[c];
      dst[c] = DT == 0 ? __builtin_bit_cast(uint16_t, (__bf16)f) : __builtin_bit_cast(uint16_t, (_Float16)f);
    }
  }
}

// dweight[v] = sum over j in [off[v], off[v+1]) of dout[perm[j]]; padding row -> 0.
__global__ void __launch_bounds__(256) emb_bwd_csr_kernel(const float* __restrict__ dout,
                                                          const int64_t* __restrict__ perm,
                                                          const int64_t* __restrict__ off,
                                                          float* __restrict__ dw, int64_t V, int64_t dim,
                                                          int64_t padding_idx) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < V; v += nwaves) {
    const int64_t j0 = off[v], j1 = off[v + 1];
    float* dst = dw + v * dim;
    for (int64_t c = lane; c < dim; c += 64) {
      float acc = 0.f;
      if (v != padding_idx)
        for (int64_t j = j0; j < j1; ++j) acc += dout[perm[j] * dim + c];
      dst[c] = acc;
    }
  }
}

// Same contract, latency-hiding form: one wave per (vocab row, 64-column
// slice); the contribution list is walked 8 rows at a time (8 independent
// index loads, then 8 independent row loads, summed in list order -- still
// bitwise deterministic).  dout may be fp32 / bf16 / fp16 (DT 2 / 0 / 1).
template <int DT>
__device__ __forceinline__ float ld_as_f(const void* p, int64_t i) {
  if constexpr (DT == 2) return reinterpret_cast<const float*>(p)[i];
  const uint16_t v = reinterpret_cast<const uint16_t*>(p)[i];
  if constexpr (DT == 0) return __uint_as_float(((uint32_t)v) << 16);
  return (float)__builtin_bit_cast(_Float16, v);
}

template <int DT>
__global__ void __launch_bounds__(256) emb_bwd_csr8_kernel(const void* __restrict__ dout,
                                                           const int64_t* __restrict__ perm,
                                                           const int64_t* __restrict__ off, float* __restrict__ dw,
                                                           int64_t V, int64_t dim, int64_t padding_idx) {
  const int lane = threadIdx.x & 63;
  const int64_t slices = (dim + 63) / 64;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave; w < V * slices; w += nwaves) {
    const int64_t v = w / slices;
    const int64_t c = (w - v * slices) * 64 + lane;
    const int64_t cc = c < dim ? c : dim - 1;
    const int64_t j0 = off[v], j1 = off[v + 1];
    float acc = 0.f;
    if (v != padding_idx) {
      for (int64_t j = j0; j < j1; j += 8) {
        int64_t p[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) p[k] = perm[min(j + k, j1 - 1)];
        float x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = ld_as_f<DT>(dout, p[k] * dim + cc);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += (j + k < j1) ? x[k] : 0.f;
      }
    }
    if (c < dim) dw[v * dim + c] = acc;
  }
}

// Small vocabularies (char-LM: V = 256 rows, 65536 contributions per step):
// one wave per vocab row leaves only V x dim/64 waves, each walking a list of
// hundreds to thousands of rows (frequent characters) -- latency-bound at
// ~0.9 ms.  Here each row's list is cut into P equal pieces, one wave per
// (row, slice, piece) writes a partial sum, and a second pass adds the P
// partials in piece order (still bitwise deterministic).
template <int DT>
__global__ void __launch_bounds__(256) emb_bwd_pieces_kernel(const void* __restrict__ dout,
                                                             const int64_t* __restrict__ perm,
                                                             const int64_t* __restrict__ off,
                                                             float* __restrict__ part, int64_t V, int64_t dim,
                                                             int P) {
  const int lane = threadIdx.x & 63;
  const int64_t slices = (dim + 63) / 64;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave; w < V * slices * P; w += nwaves) {
    const int64_t vp = w / slices;  // v * P + piece
    const int64_t v = vp / P;
    const int piece = (int)(vp - v * P);
    const int64_t c = (w - vp * slices) * 64 + lane;
    const int64_t cc = c < dim ? c : dim - 1;
    const int64_t a = off[v], n = off[v + 1] - a;
    const int64_t j0 = a + n * piece / P, j1 = a + n * (piece + 1) / P;
    float acc = 0.f;
    for (int64_t j = j0; j < j1; j += 8) {
      int64_t p[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) p[k] = perm[min(j + k, j1 - 1)];
      float x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = ld_as_f<DT>(dout, p[k] * dim + cc);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += (j + k < j1) ? x[k] : 0.f;
    }
    if (c < dim) part[vp * dim + c] = acc;
  }
}

__global__ void __launch_bounds__(256) emb_bwd_pieces_sum_kernel(const float* __restrict__ part,
                                                                 float* __restrict__ dw, int64_t V, int64_t dim,
                                                                 int P, int64_t padding_idx) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= V * dim) return;
  const int64_t v = e / dim, c = e - v * dim;
  float acc = 0.f;
  if (v != padding_idx)
    for (int p = 0; p < P; ++p) acc += part[(v * P + p) * dim + c];
  dw[e] = acc;
}

int blocks_for(int64_t rows) {
  int64_t b = (rows + 3) / 4;  // 4 waves per block, one row per wave
  if (b < 1) b = 1;
  if (b > 8192) b = 8192;
  return (int)b;
}

}  // namespace
}  // namespace pdrnn

extern "C" {

hipError_t pdrnn_embedding_fwd(const float* weight, const int64_t* idx, float* out, int64_t n_idx, int64_t dim,
                               int64_t num_embeddings, hipStream_t stream) {
  if (n_idx <= 0) return hipSuccess;
  hipLaunchKernelGGL(pdrnn::emb_fwd_kernel, dim3(pdrnn::blocks_for(n_idx)), dim3(256), 0, stream, weight, idx, out,
                     n_idx, dim, num_embeddings);
  return hipGetLastError();
}

hipError_t pdrnn_embedding_fwd16(const float* weight, const int64_t* idx, uint16_t* out, int64_t n_idx, int64_t dim,
                                 int64_t num_embeddings, int dtype, hipStream_t stream) {
  if (n_idx <= 0) return hipSuccess;
  if (dtype == 0)
    hipLaunchKernelGGL(pdrnn::emb_fwd16_kernel<0>, dim3(pdrnn::blocks_for(n_idx)), dim3(256), 0, stream, weight, idx,
                       out, n_idx, dim, num_embeddings);
  else
    hipLaunchKernelGGL(pdrnn::emb_fwd16_kernel<1>, dim3(pdrnn::blocks_for(n_idx)), dim3(256), 0, stream, weight, idx,
                       out, n_idx, dim, num_embeddings);
  return hipGetLastError();
}

hipError_t pdrnn_embedding_bwd_csr2(const void* dout, int dout_dtype, const int64_t* perm, const int64_t* offsets,
                                   float* dweight, int64_t num_embeddings, int64_t dim, int64_t padding_idx,
                                   hipStream_t stream) {
  const int64_t waves = num_embeddings * ((dim + 63) / 64);
  const dim3 grid(pdrnn::blocks_for(waves)), block(256);
  if (dout_dtype == 0)
    hipLaunchKernelGGL(pdrnn::emb_bwd_csr8_kernel<0>, grid, block, 0, stream, dout, perm, offsets, dweight,
                       num_embeddings, dim, padding_idx);
  else if (dout_dtype == 1)
    hipLaunchKernelGGL(pdrnn::emb_bwd_csr8_kernel<1>, grid, block, 0, stream, dout, perm, offsets, dweight,
                       num_embeddings, dim, padding_idx);
  else
    hipLaunchKernelGGL(pdrnn::emb_bwd_csr8_kernel<2>, grid, block, 0, stream, dout, perm, offsets, dweight,
                       num_embeddings, dim, padding_idx);
  return hipGetLastError();
}

hipError_t pdrnn_embedding_bwd_pieces(const void* dout, int dout_dtype, const int64_t* perm, const int64_t* offsets,
                                     float* partials, int pieces, float* dweight, int64_t num_embeddings, int64_t dim,
                                     int64_t padding_idx, hipStream_t stream) {
  if (pieces < 1) return hipErrorInvalidValue;
  const int64_t waves = num_embeddings * ((dim + 63) / 64) * pieces;
  const dim3 grid(pdrnn::blocks_for(waves)), block(256);
  if (dout_dtype == 0)
    hipLaunchKernelGGL(pdrnn::emb_bwd_pieces_kernel<0>, grid, block, 0, stream, dout, perm, offsets, partials,
                       num_embeddings, dim, pieces);
  else if (dout_dtype == 1)
    hipLaunchKernelGGL(pdrnn::emb_bwd_pieces_kernel<1>, grid, block, 0, stream, dout, perm, offsets, partials,
                       num_embeddings, dim, pieces);
  else
    hipLaunchKernelGGL(pdrnn::emb_bwd_pieces_kernel<2>, grid, block, 0, stream, dout, perm, offsets, partials,
                       num_embeddings, dim, pieces);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t n = num_embeddings * dim;
  hipLaunchKernelGGL(pdrnn::emb_bwd_pieces_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     partials, dweight, num_embeddings, dim, pieces, padding_idx);
  return hipGetLastError();
}

hipError_t pdrnn_embedding_bwd_csr(const float* dout, const int64_t* perm, const int64_t* offsets, float* dweight,
                                   int64_t num_embeddings, int64_t dim, int64_t padding_idx, hipStream_t stream) {
  hipLaunchKernelGGL(pdrnn::emb_bwd_csr_kernel, dim3(pdrnn::blocks_for(num_embeddings)), dim3(256), 0, stream, dout,
                     perm, offsets, dweight, num_embeddings, dim, padding_idx);
  return hipGetLastError();
}

}  // extern "C"
