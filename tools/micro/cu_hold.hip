// Holds k CUs with a resident spinning kernel shaped like RCCL's P2P kernel,
// to measure what a pre-posted RCCL receive costs the compute of a pipeline
// stage running beside it ("What's missing" #1).
//
// Footprint, from the code-object metadata of the RCCL that torch loads
// (torch/lib/librccl.so, gfx950 bundle; rcclGenericKernel<1..4, *>, the kernel
// every RCCL collective and send/recv runs):
//   256 threads, 19,744 B of LDS, 261-280 VGPRs (+17-32 AGPRs), 106 SGPRs.
// This kernel declares the same LDS and clobbers v255 and a16, so it allocates
// 256 VGPRs + 17 AGPRs = one wave per SIMD, like RCCL's.  One such block and a
// 512-thread GEMM block (2 waves per SIMD at ~240 VGPRs, 160 KiB of LDS) can
// never share a CU: each resident block takes a whole CU away from the GEMMs.
//
// Every wave exits either when the host releases it (a flag in host memory,
// read with vector loads) or after `max_s` seconds (s_memrealtime, 100 MHz),
// so the grid always drains.
//
// Usage: cu_hold <k> <max_s> <ready_file> <release_file>
//   launches k blocks, writes ready_file once every block runs, then waits for
//   release_file to exist, releases the blocks and exits 0.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/cu_hold.hip -o tools/micro/bin/cu_hold
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr int kLds = 19744;

__global__ void __launch_bounds__(256) hold(const int* release, int* started, unsigned long long limit) {
  __shared__ int lds[kLds / 4];
  const int t = threadIdx.x;
  lds[t] = t;
  asm volatile("" ::: "v255", "a16");  // RCCL-sized register allocation
  __syncthreads();
  if (t == 0) __hip_atomic_store(started + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int v = 0;
  for (;;) {
    v = __hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v != 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > limit) break;
    __builtin_amdgcn_s_sleep(32);
  }
  // keep the LDS live (never true: v is 0 or 1)
  if (v > 1 && lds[(t + 1) & 255] == -1) started[gridDim.x + blockIdx.x] = v;
}

static bool exists(const char* p) {
  struct stat st;
  return stat(p, &st) == 0;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: cu_hold <k> <max_s> <ready_file> <release_file>\n");
    return 2;
  }
  const int k = atoi(argv[1]);
  const double max_s = atof(argv[2]);
  const char* ready = argv[3];
  const char* rel = argv[4];
  int *release, *started;
  CK(hipHostMalloc((void**)&release, sizeof(int), hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&started, sizeof(int) * 2 * (k > 0 ? k : 1), hipHostMallocCoherent));
  *release = 0;
  for (int i = 0; i < 2 * (k > 0 ? k : 1); ++i) started[i] = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  if (k > 0) {
    hipLaunchKernelGGL(hold, dim3(k), dim3(256), 0, s, release, started, (unsigned long long)(max_s * 1e8));
    CK(hipGetLastError());
    for (int it = 0;; ++it) {  // all blocks resident (at most 30 s)
      int n = 0;
      for (int i = 0; i < k; ++i) n += __atomic_load_n(started + i, __ATOMIC_ACQUIRE);
      if (n == k) break;
      if (it > 30000) {
        fprintf(stderr, "cu_hold: only %d of %d blocks started\n", n, k);
        *release = 1;
        CK(hipStreamSynchronize(s));
        return 1;
      }
      usleep(1000);
    }
  }
  FILE* f = fopen(ready, "w");
  if (f) {
    fprintf(f, "%d\n", k);
    fclose(f);
  }
  for (int it = 0; !exists(rel) && it < (int)(max_s * 100); ++it) usleep(10000);
  __atomic_store_n(release, 1, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  printf("cu_hold: %d blocks released\n", k);
  return 0;
}
