// Shared device helpers for the gfx950 (CDNA4) kernels of pytorch_distributed_rnn_amd.
//
// Everything here is written for wave64 CDNA4: cross-lane reductions use DPP
// quad permutes (no LDS round trip), transcendental helpers map to the hardware
// v_exp_f32 / v_rcp_f32 instructions.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define PDRNN_HOST_DEVICE __host__ __device__

// Debug flavour (PDRNN_DEBUG_BUILD=1 python -m pytorch_distributed_rnn_amd._build):
// -O1 -g and device-side bounds asserts on data-dependent indices (token ids,
// labels).  A failing assert aborts the kernel with file:line on stderr --
// the on-GPU replacement for a sanitizer run, which this pool does not offer.
#ifndef PDRNN_DEBUG
#define PDRNN_DEBUG 0
#endif
#if PDRNN_DEBUG
#include <cassert>
#define PDRNN_DEVICE_ASSERT(cond) assert(cond)
#else
#define PDRNN_DEVICE_ASSERT(cond) ((void)0)
#endif
#define PDRNN_DEVICE __device__ __forceinline__

namespace pdrnn {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------
// Cross-lane helpers (DPP, wave64).  quad_perm control words:
//   [1,0,3,2] = 0xB1  (swap neighbours)      [2,3,0,1] = 0x4E (swap pairs)
// ---------------------------------------------------------------------------
PDRNN_DEVICE float dpp_swap1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}
PDRNN_DEVICE float dpp_swap2(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
}
// row_half_mirror (lane i of an 8-lane half-row reads lane 7-i) and row_mirror
// (lane i of a 16-lane row reads lane 15-i): after the quad sums these pair
// each quad with the other quad of the 8-group / each 8-group with the other
// half of the row, which completes the 8- and 16-lane butterflies.
PDRNN_DEVICE float dpp_half_mirror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
}
PDRNN_DEVICE float dpp_mirror(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
}

// Sum over groups of S adjacent lanes (S in {1,2,4,8,16}); every lane of the
// group receives the group total.
template <int S>
PDRNN_DEVICE float group_sum(float v) {
  if constexpr (S >= 2) v += dpp_swap1(v);
  if constexpr (S >= 4) v += dpp_swap2(v);
  if constexpr (S >= 8) v += dpp_half_mirror(v);
  if constexpr (S >= 16) v += dpp_mirror(v);
  return v;
}

PDRNN_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
PDRNN_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------
// Activations (fp32).  sigmoid via v_exp_f32 + v_rcp_f32; tanh from exp(-2|x|)
// so that small arguments keep their relative accuracy.
// ---------------------------------------------------------------------------
PDRNN_DEVICE float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
PDRNN_DEVICE float sigmoidf_fast(float x) { return fast_rcp(1.f + __expf(-x)); }
PDRNN_DEVICE float tanhf_fast(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) * fast_rcp(1.f + e);
  return copysignf(t, x);
}

// Workgroup barrier that orders LDS traffic only.  __syncthreads() on gfx950
// also drains vmcnt (every outstanding global load AND store of the wave)
// before s_barrier, which in a persistent recurrence serialises each timestep
// behind the HBM write latency of the previous one.  Cross-wave hand-offs in
// the recurrent kernels go exclusively through LDS, so waiting for lgkmcnt is
// sufficient; global prefetches and output stores stay in flight.
// Wave issue priority in the long small-H recurrences.  Co-resident
// workgroups start together and the SIMD's arbiter otherwise favours the
// oldest wave, so the workgroups dispatched last on a CU finish last and set
// the kernel's end (stamps: loop time rises with blockIdx in tiers of one
// workgroup per CU).  `prio` = mode | log2(period) << 4 | CUs << 8:
//   mode 1: priority falls with the wave's own progress (4 levels);
//   mode 2: priority rotates every `period` steps over the dispatch tiers
//           (tier = blockIdx / CUs, 3 levels), every tier leads a third of
//           the time.
// `it` is wave-uniform (scalar compares only).
PDRNN_DEVICE void set_prio_level(int lvl) {
  switch (lvl) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}
PDRNN_DEVICE void prio_by_progress(int it, int iters, int prio) {
  const int mode = prio & 15;
  // one workgroup per CU at most: nothing to arbitrate (and the B = 180
  // one-launch step measured 3 % slower with the setprio traffic)
  if ((int)gridDim.x <= max(prio >> 8, 1)) return;
  if (mode == 1) {
    if (it == 0) set_prio_level(3);
    else if (it == iters / 4) set_prio_level(2);
    else if (it == iters / 2) set_prio_level(1);
    else if (it == 3 * iters / 4) set_prio_level(0);
  } else if (mode == 2) {
    const int sh = (prio >> 4) & 15;
    if ((it & ((1 << sh) - 1)) == 0) {
      const int ncu = max(prio >> 8, 1);
      const int tier = (int)blockIdx.x / ncu;
      set_prio_level(((it >> sh) + tier) % 3);
    }
  }
}

PDRNN_DEVICE void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Opaque register copy.  Used to build a genuine {v, v} VGPR pair for a
// v_pk_fma_f32 broadcast operand: left to itself the compiler encodes the
// broadcast with op_sel on a register pair whose high half is an unrelated
// register -- often a prefetch still in flight, which then makes the waitcnt
// pass stall on that load.
PDRNN_DEVICE float opaque_copy(float v) {
  float r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// Diagnostic cycle stamps (shader clock and 100 MHz real-time clock).
PDRNN_DEVICE uint64_t stamp_cycles() { return __builtin_amdgcn_s_memtime(); }
PDRNN_DEVICE uint64_t stamp_real() { return __builtin_amdgcn_s_memrealtime(); }
// Which CU runs this wave (diagnostics: workgroup placement census): SIMD id
// << 24 | XCC id << 16 | the SE / SH / CU fields of HW_ID (bits 8..14).
PDRNN_DEVICE uint32_t stamp_cu() {
  const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  return (((hw >> 4) & 3) << 24) | ((xcc & 0xF) << 16) | ((hw >> 8) & 0x7F);
}

// bf16 <-> f32 (round to nearest even; NaN preserved by the hardware cvt).
PDRNN_DEVICE float bf16_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
PDRNN_DEVICE uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// ---------------------------------------------------------------------------
// Shared by the small-H recurrent kernels (lstm_small.hip, lstm_small_dw.hip)
// ---------------------------------------------------------------------------
// Buffer descriptor for a wave-uniform base pointer: the halves go through
// readfirstlane so the compiler can keep the descriptor in SGPRs (no
// waterfall loop around each buffer op).
PDRNN_DEVICE __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32));
  void* up = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(up, 0, 0x7FFFFFFF, 0x00020000);
}
PDRNN_DEVICE float bload(__amdgpu_buffer_rsrc_t r, uint32_t voff_bytes, uint32_t soff_bytes) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff_bytes, soff_bytes, 0));
}

// x element i as fp32 (x may be stored in bf16: mixed-precision inputs are
// widened once, while staging into LDS)
PDRNN_DEVICE float ldx(const float* x, int64_t i, int bf) {
  return bf ? bf16_to_f32(reinterpret_cast<const uint16_t*>(x)[i]) : x[i];
}

typedef float pdrnn_f2 __attribute__((ext_vector_type(2)));

PDRNN_DEVICE float quad_bcast(float v, int q) {
  // quad_perm [q,q,q,q]: every lane of the quad reads lane q of the quad
  switch (q) {
    case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x00, 0xF, 0xF, false));
    case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x55, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xAA, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xFF, 0xF, 0xF, false));
  }
}


}  // namespace pdrnn

#define PDRNN_HIP_CHECK(expr)                                                   \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) return _e;                                            \
  } while (0)
