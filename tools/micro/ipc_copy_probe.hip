// Probe: are small copies INTO IPC-mapped memory (hipIpcOpenMemHandle of another process's allocation, same
// GPU) run on the DMA engines with hipMemcpyDeviceToDeviceNoCU, or as __amd_rocclr_copyBuffer kernels?
//   ipc_copy_probe export FILE   allocates + exports a buffer (handle written to FILE), waits for FILE.done
//   ipc_copy_probe import FILE   opens it, copies growing sizes into it (one marker kernel before each size)
// Two independent processes (no fork), so the importer can run under rocprofv3; read the importer's trace with
// tools/small_copy_report.py --ipc.  (tools/gpu_runs/r6_g3.sh)
//   hipcc --offload-arch=gfx950 -O2 tools/micro/ipc_copy_probe.hip -o tools/micro/bin/ipc_copy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "[pid %d] %s failed: %s\n", getpid(), #x, hipGetErrorString(e_)); \
      exit(3);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void marker(int id, int* sink) {
  if (threadIdx.x == 0 && id < 0) sink[0] = id;
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s export|import FILE\n", argv[0]);
    return 2;
  }
  const std::string file = argv[2];
  const std::string done = file + ".done";
  CK(hipSetDevice(0));
  if (strcmp(argv[1], "export") == 0) {
    void *buf = nullptr, *small = nullptr;
    CK(hipMalloc(&buf, 8 << 20));
    CK(hipMalloc(&small, 4096));  // a small allocation, like the links' flag words
    hipIpcMemHandle_t h[2];
    CK(hipIpcGetMemHandle(&h[0], buf));
    CK(hipIpcGetMemHandle(&h[1], small));
    const std::string tmp = file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(h, sizeof h, 1, f) != 1) return 4;
    fclose(f);
    rename(tmp.c_str(), file.c_str());
    for (int i = 0; i < 60000 && access(done.c_str(), F_OK) != 0; ++i) usleep(1000);  // at most 60 s
    printf("exporter: done\n");
    return 0;
  }
  hipIpcMemHandle_t h[2];
  FILE* f = nullptr;
  for (int i = 0; i < 60000 && !(f = fopen(file.c_str(), "rb")); ++i) usleep(1000);
  if (!f || fread(h, sizeof h, 1, f) != 1) return 5;
  fclose(f);
  void *dst = nullptr, *dst_small = nullptr;
  CK(hipIpcOpenMemHandle(&dst, h[0], hipIpcMemLazyEnablePeerAccess));
  CK(hipIpcOpenMemHandle(&dst_small, h[1], hipIpcMemLazyEnablePeerAccess));
  const size_t sizes[] = {8, 4096, 65536, 262144, 1048576, 4194304};
  char* src = nullptr;
  int* sink = nullptr;
  CK(hipMalloc(&src, 8 << 20));
  CK(hipMalloc(&sink, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int i = 0; i < 6; ++i) {
    hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, s, i, sink);
    for (int r = 0; r < 3; ++r) CK(hipMemcpyAsync(dst, src, sizes[i], hipMemcpyDeviceToDeviceNoCU, s));
    CK(hipStreamSynchronize(s));
    printf("importer: marker %d = IPC dst, NoCU, %zu B x 3\n", i, sizes[i]);
  }
  // 8 bytes between small allocations: 4 KiB src -> 4 KiB IPC dst, 4 KiB src -> 8 MiB IPC dst,
  // 8 MiB src -> 4 KiB IPC dst (markers 6, 7, 8)
  char* src_small = nullptr;
  CK(hipMalloc(&src_small, 4096));
  const void* srcs[3] = {src_small, src_small, src};
  void* dsts[3] = {dst_small, dst, dst_small};
  for (int i = 0; i < 3; ++i) {
    hipLaunchKernelGGL(marker, dim3(1), dim3(64), 0, s, 6 + i, sink);
    for (int r = 0; r < 3; ++r) CK(hipMemcpyAsync(dsts[i], srcs[i], 8, hipMemcpyDeviceToDeviceNoCU, s));
    CK(hipStreamSynchronize(s));
    printf("importer: marker %d = 8 B, %s src -> %s IPC dst\n", 6 + i, i < 2 ? "4 KiB" : "8 MiB",
           i == 1 ? "8 MiB" : "4 KiB");
  }
  CK(hipIpcCloseMemHandle(dst));
  CK(hipIpcCloseMemHandle(dst_small));
  FILE* d = fopen(done.c_str(), "w");
  if (d) fclose(d);
  return 0;
}
