// Weight-shadow pack: every compute-layout copy of the fp32 master weights
// that went stale in an optimizer step, rebuilt in ONE launch.
//
// The kernels read the recurrent weights in layouts of their own -- gate-
// interleaved rows (forward step / input projection), transposed (BPTT step),
// the stored layout cast to 16 bit (dX GEMM), the GRU's zero-padded stacks,
// the folded projection biases (b_ih + b_hh, interleaved) -- cached on the
// parameters and rebuilt when their version counters move (ops/shadow.py).
// Done with torch, each is a strided converting copy or an add: about ten
// small dispatches per step on the char-LM (profiles/r6 glue trace) and on
// the fp32 hidden-128 motion model.  Here each layout is one job: a 3-D
// strided gather dst[i0, i1, i2] = src[i0, i1, i2] (+ src2[...]) with
// arbitrary element strides on either side, from fp32 (or 16-bit: the
// carried LSTM states, ops/lstm_large.py) converted to bf16 / fp16 / fp32.
// A workgroup moves a 64 x 64 tile of (i1, i2) through LDS, reading along
// whichever of i1 / i2 is unit-stride in the source and writing along the one
// that is unit-stride in the destination, so transposes stay coalesced on
// both sides.  Jobs are passed by value (kernel arguments, up to 16 a launch);
// a workgroup finds its job from the per-job first-tile prefix.
#include <hip/hip_runtime.h>

#include "pdrnn/api.h"

namespace pdrnn {
namespace {

constexpr int PK_T = 64;        // tile edge
constexpr int PK_THREADS = 256;

__device__ __forceinline__ uint16_t pk_bf16(float f) {
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);                  // round to nearest even
}

__global__ void __launch_bounds__(PK_THREADS) shadow_pack_kernel(PdrnnPackBatch b) {
  __shared__ float tile[PK_T][PK_T + 1];
  const int64_t blk = blockIdx.x;
  int j = 0;
  while (j + 1 < b.njobs && blk >= b.job[j + 1].tile0) ++j;
  const PdrnnPackJob& p = b.job[j];
  const int64_t l = blk - p.tile0;
  const int t2n = (p.n[2] + PK_T - 1) / PK_T, t1n = (p.n[1] + PK_T - 1) / PK_T;
  const int t2 = (int)(l % t2n);
  const int t1 = (int)((l / t2n) % t1n);
  const int64_t i0 = l / ((int64_t)t2n * t1n);
  const int a1 = t1 * PK_T, a2 = t2 * PK_T;
  if (p.vec) {
    // both sides unit-stride along i2, 4-element aligned (interleave / cast
    // jobs: most of the bytes): 4 elements a thread straight through, no LDS
    for (int e = threadIdx.x; e < PK_T * PK_T / 4; e += PK_THREADS) {
      const int r = e / (PK_T / 4), c = (e % (PK_T / 4)) * 4;
      if (a1 + r >= p.n[1] || a2 + c >= p.n[2]) continue;
      const int64_t so = i0 * p.ss[0] + (int64_t)(a1 + r) * p.ss[1] + (a2 + c);
      const int64_t dof = i0 * p.ds[0] + (int64_t)(a1 + r) * p.ds[1] + (a2 + c);
      float v[4];
      auto ld4 = [&](const void* base, float* o) {
        if (p.sdtype == 2) {
          const float4 f = *reinterpret_cast<const float4*>(static_cast<const float*>(base) + so);
          o[0] = f.x; o[1] = f.y; o[2] = f.z; o[3] = f.w;
        } else {
          const uint2 h = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(base) + so);
          const uint16_t hs[4] = {(uint16_t)h.x, (uint16_t)(h.x >> 16), (uint16_t)h.y, (uint16_t)(h.y >> 16)};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            o[q] = p.sdtype == 1 ? (float)__builtin_bit_cast(_Float16, hs[q]) : __uint_as_float((uint32_t)hs[q] << 16);
        }
      };
      ld4(p.src, v);
      if (p.src2) {
        float w2[4];
        ld4(p.src2, w2);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += w2[q];
      }
      if (p.dtype == 2) {
        *reinterpret_cast<float4*>(static_cast<float*>(p.dst) + dof) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        uint16_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          o[q] = p.dtype == 1 ? __builtin_bit_cast(uint16_t, (_Float16)v[q]) : pk_bf16(v[q]);
        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(p.dst) + dof) =
            make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
      }
    }
    return;
  }
  // read along the source's unit-stride dimension
  const bool s_in2 = p.ss[2] == 1 || p.ss[1] != 1;
  auto ld = [&](const void* base, int64_t o) -> float {
    if (p.sdtype == 2) return static_cast<const float*>(base)[o];
    const uint16_t h = static_cast<const uint16_t*>(base)[o];
    return p.sdtype == 1 ? (float)__builtin_bit_cast(_Float16, h) : __uint_as_float((uint32_t)h << 16);
  };
  const int64_t so = i0 * p.ss[0];
#pragma unroll 4
  for (int e = threadIdx.x; e < PK_T * PK_T; e += PK_THREADS) {
    const int r = s_in2 ? e / PK_T : e % PK_T, c = s_in2 ? e % PK_T : e / PK_T;
    if (a1 + r < p.n[1] && a2 + c < p.n[2]) {
      const int64_t o = so + (int64_t)(a1 + r) * p.ss[1] + (int64_t)(a2 + c) * p.ss[2];
      tile[r][c] = p.src2 ? ld(p.src, o) + ld(p.src2, o) : ld(p.src, o);
    }
  }
  __syncthreads();
  // write along the destination's unit-stride dimension
  const bool d_in2 = p.ds[2] == 1 || p.ds[1] != 1;
  for (int e = threadIdx.x; e < PK_T * PK_T; e += PK_THREADS) {
    const int r = d_in2 ? e / PK_T : e % PK_T, c = d_in2 ? e % PK_T : e / PK_T;
    if (a1 + r >= p.n[1] || a2 + c >= p.n[2]) continue;
    const int64_t o = i0 * p.ds[0] + (int64_t)(a1 + r) * p.ds[1] + (int64_t)(a2 + c) * p.ds[2];
    const float v = tile[r][c];
    if (p.dtype == 2) {
      static_cast<float*>(p.dst)[o] = v;
    } else if (p.dtype == 1) {
      static_cast<uint16_t*>(p.dst)[o] = __builtin_bit_cast(uint16_t, (_Float16)v);
    } else {
      static_cast<uint16_t*>(p.dst)[o] = pk_bf16(v);
    }
  }
}

}  // namespace
}  // namespace pdrnn

extern "C" {

int64_t pdrnn_shadow_pack_tiles(const PdrnnPackJob* j) {
  if (j->n[0] <= 0 || j->n[1] <= 0 || j->n[2] <= 0) return 0;
  return (int64_t)j->n[0] * ((j->n[1] + pdrnn::PK_T - 1) / pdrnn::PK_T) * ((j->n[2] + pdrnn::PK_T - 1) / pdrnn::PK_T);
}

hipError_t pdrnn_shadow_pack(PdrnnPackBatch* b, hipStream_t stream) {
  if (b->njobs < 1 || b->njobs > PDRNN_PACK_MAX_JOBS) return hipErrorInvalidValue;
  int64_t tiles = 0;
  for (int j = 0; j < b->njobs; ++j) {
    PdrnnPackJob& p = b->job[j];
    if (!p.src || !p.dst || p.dtype < 0 || p.dtype > 2 || p.sdtype < 0 || p.sdtype > 2) return hipErrorInvalidValue;
    p.tile0 = tiles;
    tiles += pdrnn_shadow_pack_tiles(&p);
    // the vector path: unit stride along i2 on both sides, every row start and
    // the extent a multiple of 4 elements, 16 / 8-byte aligned bases
    const int ses = p.sdtype == 2 ? 4 : 2, des = p.dtype == 2 ? 4 : 2;
    const uintptr_t al = (uintptr_t)p.src | (uintptr_t)p.src2 | 0;
    p.vec = p.ss[2] == 1 && p.ds[2] == 1 && p.n[2] % 4 == 0 && p.ss[1] % 4 == 0 && p.ds[1] % 4 == 0 &&
            p.ss[0] % 4 == 0 && p.ds[0] % 4 == 0 && (al % (4 * ses)) == 0 &&
            ((uintptr_t)p.dst % (4 * des)) == 0;
  }
  if (tiles == 0) return hipSuccess;
  if (tiles > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pdrnn::shadow_pack_kernel, dim3((unsigned)tiles), dim3(pdrnn::PK_THREADS), 0, stream, *b);
  return hipGetLastError();
}

}  // extern "C"
