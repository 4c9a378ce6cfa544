// Probe: which hipMemcpyAsync copies does the runtime run on the DMA engines, and which as a
// __amd_rocclr_copyBuffer kernel on the CUs?  Same-device device-to-device copies of growing size,
// with hipMemcpyDeviceToDeviceNoCU and hipMemcpyDeviceToDevice, on one non-blocking stream; a marker
// kernel separates the sizes so the trace can be read in order.  Run under
//   rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/scp -o scp -- tools/micro/bin/small_copy_probe
// and read with tools/small_copy_report.py.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/small_copy_probe.hip -o tools/micro/bin/small_copy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));             \
      exit(3);                                                                   \
    }                                                                            \
  } while (0)

__global__ void marker(int id, int* sink) {
  if (threadIdx.x == 0 && id < 0) sink[0] = id;  // never taken: the launch is the marker
}

int main() {
  const size_t sizes[] = {8, 64, 1024, 4096, 16384, 65536, 262144, 1048576, 4194304};
  const int nsizes = sizeof(sizes) / sizeof(sizes[0]);
  char *a = nullptr, *b = nullptr;
  int* sink = nullptr;
  CK(hipMalloc(&a, 8 << 20));
  CK(hipMalloc(&b, 8 << 20));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 1, 8 << 20));
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const hipMemcpyKind kinds[2] = {hipMemcpyDeviceToDeviceNoCU, hipMemcpyDeviceToDevice};
  const char* names[2] = {"D2D_NoCU", "D2D"};
  for (int k = 0; k < 2; ++k) {
    for (int i = 0; i < nsizes; ++i) {
      hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, s, k * 100 + i, sink);
      for (int r = 0; r < 3; ++r) {
        hipError_t e = hipMemcpyAsync(b, a, sizes[i], kinds[k], s);
        if (e != hipSuccess) {
          printf("%s %zu: refused (%s)\n", names[k], sizes[i], hipGetErrorString(e));
          (void)hipGetLastError();
        }
      }
      CK(hipStreamSynchronize(s));
      printf("marker %d = %s %zu B x 3\n", k * 100 + i, names[k], sizes[i]);
    }
  }
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
