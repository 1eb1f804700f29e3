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

// accumulate: dw += the sum (the weight's gradient buffer itself, ops/gradsink.py)
__global__ void __launch_bounds__(256) emb_bwd_pieces_sum_kernel(const float* __restrict__ part,
                                                                 float* __restrict__ dw, int64_t V, int64_t dim,
                                                                 int P, int64_t padding_idx, int accumulate) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= V * dim) return;
  const int64_t v = e / dim, c = e - v * dim;
  float acc = 0.f;
  if (v != padding_idx)
    for (int p = 0; p < P; ++p) acc += part[(v * P + p) * dim + c];
  dw[e] = accumulate ? dw[e] + acc : acc;
}

// ---- stable counting sort of the indices by vocabulary row (in-tree) ------
// Replaces a library radix / merge sort + searchsorted: the vocabulary is
// small (char-LM: 256), so a histogram per index block, one scan over
// (row, block) and a stable scatter give the same perm / offsets as a stable
// sort, deterministically and in three small launches.
constexpr int kSortTile = 256;     // indices per scatter sub-tile (= block size)
constexpr int kSortChunk = 4096;   // indices per histogram / scatter block

__device__ __forceinline__ int64_t wrap_idx(int64_t v, int64_t V) { return v < 0 ? v + V : v; }

// blockcounts[b][v] = occurrences of v in indices [b * chunk, (b + 1) * chunk)
__global__ void __launch_bounds__(256) emb_count_kernel(const int64_t* __restrict__ idx, int64_t n, int V,
                                                        int* __restrict__ bcount) {
  extern __shared__ int hist[];
  for (int v = threadIdx.x; v < V; v += blockDim.x) hist[v] = 0;
  __syncthreads();
  const int64_t j0 = (int64_t)blockIdx.x * kSortChunk, j1 = min(j0 + kSortChunk, n);
  for (int64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
    const int64_t v = wrap_idx(idx[j], V);
    PDRNN_DEVICE_ASSERT(v >= 0 && v < V);
    atomicAdd(&hist[v], 1);
  }
  __syncthreads();
  for (int v = threadIdx.x; v < V; v += blockDim.x) bcount[(int64_t)blockIdx.x * V + v] = hist[v];
}

// one workgroup: base[b][v] = offsets[v] + sum_{b' < b} bcount[b'][v];
// offsets[v] = sum_{v' < v} total[v'] (offsets[V] = n)
__global__ void __launch_bounds__(1024) emb_scan_kernel(int* __restrict__ bcount, int nb, int V,
                                                        int64_t* __restrict__ offsets) {
  extern __shared__ int tot[];  // [V] totals, then exclusive offsets
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    int run = 0;
    for (int b = 0; b < nb; ++b) {
      const int c = bcount[(int64_t)b * V + v];
      bcount[(int64_t)b * V + v] = run;
      run += c;
    }
    tot[v] = run;
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // V <= 16384: a serial scan of the totals is a few microseconds
    int run = 0;
    for (int v = 0; v < V; ++v) {
      const int c = tot[v];
      tot[v] = run;
      run += c;
    }
    offsets[V] = run;
  }
  __syncthreads();
  for (int v = threadIdx.x; v < V; v += blockDim.x) {
    offsets[v] = tot[v];
    for (int b = 0; b < nb; ++b) bcount[(int64_t)b * V + v] += tot[v];
  }
}

// perm[base[b][v] + (rank of j among the earlier indices of v in block b)] = j
__global__ void __launch_bounds__(kSortTile) emb_scatter_kernel(const int64_t* __restrict__ idx, int64_t n, int V,
                                                                const int* __restrict__ base,
                                                                int64_t* __restrict__ perm) {
  extern __shared__ int sh[];  // [V] running count of this block, [kSortTile] the tile's rows
  int* cnt = sh;
  int* tile = sh + V;
  for (int v = threadIdx.x; v < V; v += blockDim.x) cnt[v] = 0;
  const int64_t j0 = (int64_t)blockIdx.x * kSortChunk, j1 = min(j0 + kSortChunk, n);
  const int* bb = base + (int64_t)blockIdx.x * V;
  for (int64_t t0 = j0; t0 < j1; t0 += kSortTile) {
    const int64_t j = t0 + threadIdx.x;
    const int v = j < j1 ? (int)wrap_idx(idx[j], V) : -1;
    __syncthreads();  // the previous tile's counts are in, its rows read
    tile[threadIdx.x] = v;
    __syncthreads();
    if (v >= 0) {
      int rank = 0;
      for (int k = 0; k < (int)threadIdx.x; ++k) rank += tile[k] == v;
      perm[bb[v] + cnt[v] + rank] = j;
    }
    __syncthreads();  // every thread has read cnt[] for this tile
    if (v >= 0) atomicAdd(&cnt[v], 1);
  }
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
                                     int64_t padding_idx, int accumulate, hipStream_t stream) {
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
                     partials, dweight, num_embeddings, dim, pieces, padding_idx, accumulate);
  return hipGetLastError();
}

// Stable sort of n indices by row into perm (int64 [n]) and the row
// offsets (int64 [V + 1]); scratch: int32 [ceil(n / 4096) * V].  V <= 16384.
int64_t pdrnn_embedding_sort_scratch(int64_t n, int64_t V) {
  return ((n + pdrnn::kSortChunk - 1) / pdrnn::kSortChunk) * V;
}
hipError_t pdrnn_embedding_sort(const int64_t* idx, int64_t n, int64_t V, int* scratch, int64_t* perm,
                                int64_t* offsets, hipStream_t stream) {
  if (V < 1 || V > 16384 || n < 0 || n >= (int64_t)1 << 31) return hipErrorInvalidValue;
  const int nb = (int)((n + pdrnn::kSortChunk - 1) / pdrnn::kSortChunk);
  if (nb == 0) {
    hipLaunchKernelGGL(pdrnn::emb_scan_kernel, dim3(1), dim3(1024), sizeof(int) * (size_t)V, stream, scratch, 0,
                       (int)V, offsets);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(pdrnn::emb_count_kernel, dim3(nb), dim3(256), sizeof(int) * (size_t)V, stream, idx, n, (int)V,
                     scratch);
  hipLaunchKernelGGL(pdrnn::emb_scan_kernel, dim3(1), dim3(1024), sizeof(int) * (size_t)V, stream, scratch, nb,
                     (int)V, offsets);
  // the scatter stages V counters + one tile of keys: past 64 KiB of dynamic
  // LDS (V > 16384 - kSortTile) the launch needs the opt-in limit (160 KiB
  // per CU on gfx950), else it fails where the old at::sort path worked
  const size_t lds_scatter = sizeof(int) * ((size_t)V + pdrnn::kSortTile);
  if (lds_scatter > 64 * 1024) {
    const hipError_t ea = hipFuncSetAttribute((const void*)pdrnn::emb_scatter_kernel,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_scatter);
    if (ea != hipSuccess) return ea;
  }
  hipLaunchKernelGGL(pdrnn::emb_scatter_kernel, dim3(nb), dim3(pdrnn::kSortTile), lds_scatter, stream, idx, n,
                     (int)V, scratch, perm);
  return hipGetLastError();
}

hipError_t pdrnn_embedding_bwd_csr(const float* dout, const int64_t* perm, const int64_t* offsets, float* dweight,
                                   int64_t num_embeddings, int64_t dim, int64_t padding_idx, hipStream_t stream) {
  hipLaunchKernelGGL(pdrnn::emb_bwd_csr_kernel, dim3(pdrnn::blocks_for(num_embeddings)), dim3(256), 0, stream, dout,
                     perm, offsets, dweight, num_embeddings, dim, padding_idx);
  return hipGetLastError();
}

}  // extern "C"
