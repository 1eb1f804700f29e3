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

}  // namespace
}  // namespace pdrnn

extern "C" hipError_t pdrnn_debug_spin(uint64_t microseconds, hipStream_t stream) {
  // bounded: at most 60 s
  if (microseconds > 60ull * 1000 * 1000) microseconds = 60ull * 1000 * 1000;
  hipLaunchKernelGGL(pdrnn::debug_spin_kernel, dim3(1), dim3(64), 0, stream, microseconds * 100ull);
  return hipGetLastError();
}
