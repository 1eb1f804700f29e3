// Diagnostics kernels (never on a training path).
//
// pdrnn_debug_spin: one wave that spins for a bounded wall-clock time
// (s_memrealtime, 100 MHz constant clock) -- used by the communicator
// watchdog test to stand in for a collective whose peer never arrives.  The
// wait is bounded by construction (no host flag, no data dependency), so the
// grid always drains.
#include "pdrnn/api.h"
#include "pdrnn/common.h"

namespace pdrnn {
namespace {

__global__ void __launch_bounds__(64) debug_spin_kernel(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

// pdrnn_debug_spin_cus: a grid of workgroups (threads, dynamic LDS as
// given) that spin for a bounded time each -- fills the CUs so that a
// persistent launch issued meanwhile on another stream cannot become
// co-resident (test of the persistent recurrence's timeout recovery).
__global__ void __launch_bounds__(1024) debug_spin_cus_kernel(uint64_t ticks) {
  extern __shared__ float hold[];  // occupancy only
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  if (ticks == 0) hold[threadIdx.x] = 0.f;  // keep the allocation referenced
}

}  // namespace
}  // namespace pdrnn

extern "C" hipError_t pdrnn_debug_spin_cus(uint64_t microseconds, int workgroups, int threads, int lds_bytes,
                                           hipStream_t stream) {
  if (microseconds > 10ull * 1000 * 1000) microseconds = 10ull * 1000 * 1000;  // bounded: 10 s
  if (workgroups < 1 || threads < 64 || threads > 1024 || threads % 64 || lds_bytes < 4 * threads ||
      lds_bytes > 160 * 1024)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(pdrnn::debug_spin_cus_kernel, dim3(workgroups), dim3(threads), (size_t)lds_bytes, stream,
                     microseconds * 100ull);
  return hipGetLastError();
}

extern "C" hipError_t pdrnn_debug_spin(uint64_t microseconds, hipStream_t stream) {
  // bounded: at most 60 s
  if (microseconds > 60ull * 1000 * 1000) microseconds = 60ull * 1000 * 1000;
  hipLaunchKernelGGL(pdrnn::debug_spin_kernel, dim3(1), dim3(64), 0, stream, microseconds * 100ull);
  return hipGetLastError();
}
