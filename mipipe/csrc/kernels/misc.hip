// Small utility kernels.
//
// gpu_sleep: one wave spins on s_memrealtime (100 MHz constant clock) for the
// requested time.  Used by the stream-overlap tests (upstream conftest's
// cuda_sleep idea): two sleeps on streams that truly overlap take ~max, not sum.
#include "common.h"
#include "kernels.h"

namespace mipipe {

namespace {
__global__ void sleep_kernel(uint64_t ticks) {
  const uint64_t start = __builtin_amdgcn_s_memrealtime();
  // Bounded spin: exits after `ticks` of the 100 MHz real-time counter.
  while (__builtin_amdgcn_s_memrealtime() - start < ticks) {
    __builtin_amdgcn_s_sleep(8);
  }
}
}  // namespace

void gpu_sleep(int64_t microseconds, hipStream_t s) {
  if (microseconds <= 0) return;
  const uint64_t ticks = (uint64_t)microseconds * 100ull;  // 100 MHz
  hipLaunchKernelGGL(sleep_kernel, dim3(1), dim3(64), 0, s, ticks);
}

}  // namespace mipipe
