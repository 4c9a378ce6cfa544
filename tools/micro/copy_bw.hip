// Same-device (and, with >= 2 GPUs, peer) copy bandwidth on MI355X, 1-64 MiB:
//   memcpy  -- hipMemcpyAsync device-to-device (the runtime's engine choice;
//              HSA_ENABLE_SDMA=0/1 selects blit kernel / SDMA for the runtime)
//   blit    -- a plain 16-byte-per-lane copy kernel, 2048 workgroups
//   peer    -- hipMemcpyPeerAsync 0 -> 1 (peer access enabled), if 2 GPUs
//   peerblit-- the copy kernel on GPU 0 writing GPU 1's memory over xGMI
// Prints GB/s (median of 20) per size.  The pipeline's activation transfer at
// enc12 PP=8 is 32 x 128 x 4096 x 2 B = 32 MiB per micro-batch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

__global__ void __launch_bounds__(256) blit(const u32x4* __restrict__ src, u32x4* __restrict__ dst, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}

template <typename F>
float time_ms(F f, hipStream_t s) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  CK(hipStreamSynchronize(s));
  std::vector<float> ts;
  for (int i = 0; i < 20; ++i) {
    CK(hipEventRecord(a, s));
    f();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ts[ts.size() / 2];
}

int main() {
  int ndev = 0;
  CK(hipGetDeviceCount(&ndev));
  const size_t maxb = 64ull << 20;
  CK(hipSetDevice(0));
  void *src, *dst, *peer = nullptr;
  CK(hipMalloc(&src, maxb));
  CK(hipMalloc(&dst, maxb));
  CK(hipMemset(src, 1, maxb));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (ndev >= 2) {
    int ok = 0;
    CK(hipDeviceCanAccessPeer(&ok, 0, 1));
    if (ok) {
      CK(hipDeviceEnablePeerAccess(1, 0));
      CK(hipSetDevice(1));
      CK(hipMalloc(&peer, maxb));
      CK(hipDeviceEnablePeerAccess(0, 0));
      CK(hipSetDevice(0));
    }
  }
  printf("# %d GPU(s); GB/s (1e9 B/s), median of 20\n", ndev);
  printf("%8s %10s %10s %10s %10s\n", "MiB", "memcpy", "blit", "peer", "peerblit");
  for (size_t mib : {1, 4, 16, 32, 64}) {
    const size_t bytes = mib << 20;
    const size_t n = bytes / 16;
    const float t1 = time_ms([&] { CK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s)); }, s);
    const float t2 = time_ms([&] { hipLaunchKernelGGL(blit, dim3(2048), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n); }, s);
    float t3 = 0.f, t4 = 0.f;
    if (peer) {
      t3 = time_ms([&] { CK(hipMemcpyPeerAsync(peer, 1, src, 0, bytes, s)); }, s);
      t4 = time_ms([&] { hipLaunchKernelGGL(blit, dim3(2048), dim3(256), 0, s, (const u32x4*)src, (u32x4*)peer, n); }, s);
    }
    // same-device copies move the bytes twice (read + write); report the copy rate (bytes / time)
    printf("%8zu %10.1f %10.1f %10.1f %10.1f\n", mib, bytes / t1 / 1e6, bytes / t2 / 1e6, peer ? bytes / t3 / 1e6 : 0.0,
           peer ? bytes / t4 / 1e6 : 0.0);
  }
  return 0;
}
