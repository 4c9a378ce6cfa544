// Does hipMemcpyDeviceToDeviceNoCU keep a device-to-device copy off the CUs (the IPC links' "sdma" engine), and what
// does it cost?  Times 1..64 MiB copies with hipMemcpyDeviceToDevice (ROCm picks a blit kernel for same-device
// copies) and with hipMemcpyDeviceToDeviceNoCU (copy engines only), same device.  Run it under
// `rocprofv3 --kernel-trace --stats` to see which of the two launches a copy kernel.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/nocu_copy.hip -o tools/micro/bin/nocu_copy
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));          \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

static float time_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) CHECK(hipMemcpyAsync(dst, src, bytes, kind, s));
  const int iters = 20;
  CHECK(hipEventRecord(a, s));
  for (int i = 0; i < iters; ++i) CHECK(hipMemcpyAsync(dst, src, bytes, kind, s));
  CHECK(hipEventRecord(b, s));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
  return ms / iters;
}

int main() {
  const size_t max_bytes = 64ull << 20;
  void *src, *dst;
  CHECK(hipMalloc(&src, max_bytes));
  CHECK(hipMalloc(&dst, max_bytes));
  CHECK(hipMemset(src, 1, max_bytes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  printf("   MiB   D2D (us, GB/s)        D2D NoCU (us, GB/s)\n");
  for (size_t mib = 1; mib <= 64; mib *= 4) {
    const size_t bytes = mib << 20;
    const float t0 = time_copy(dst, src, bytes, hipMemcpyDeviceToDevice, s);
    const float t1 = time_copy(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, s);
    printf("%6zu   %8.1f %8.1f     %8.1f %8.1f\n", mib, t0 * 1e3, bytes / (t0 * 1e6), t1 * 1e3, bytes / (t1 * 1e6));
  }
  CHECK(hipStreamDestroy(s));
  CHECK(hipFree(src));
  CHECK(hipFree(dst));
  return 0;
}
