// Probe: can two processes sharing ONE MI355X exchange data through HIP IPC?
//  * hipIpcGetMemHandle / hipIpcOpenMemHandle (receiver-owned slot mapped by the sender)
//  * hipIpcGetEventHandle / hipIpcOpenEventHandle (interprocess events: the
//    receiver's stream waits on an event the sender records)
// Forks before any HIP call; each child initialises HIP on its own.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/ipc_probe.hip -o tools/micro/bin/ipc_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <thread>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "[pid %d] %s failed: %s\n", getpid(), #x, hipGetErrorString(e_)); \
      _exit(3);                                                                        \
    }                                                                                  \
  } while (0)

struct Msg {
  hipIpcMemHandle_t mem;
  hipIpcEventHandle_t ev;
  int ev_ok;
};

__global__ void fill(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

// busy-waits on the 100 MHz constant clock
__global__ void spin(unsigned long long ticks) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

int main() {
  const size_t n = 8u << 20;  // 32 MiB of floats
  int to_sender[2], to_recv[2];
  if (pipe(to_sender) || pipe(to_recv)) return 1;
  pid_t pid = fork();
  if (pid == 0) {
    // SENDER: opens the receiver's buffer, writes into it (hipMemcpy from a local
    // buffer, after a long spin kernel), records its own interprocess event.
    Msg m;
    if (read(to_sender[0], &m, sizeof m) != sizeof m) _exit(4);
    CK(hipSetDevice(0));
    void* remote = nullptr;
    CK(hipIpcOpenMemHandle(&remote, m.mem, hipIpcMemLazyEnablePeerAccess));
    float* local = nullptr;
    CK(hipMalloc(&local, n * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, s, local, n, 42.0f);
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 50000000ull);  // 0.5 s
    CK(hipMemcpyAsync(remote, local, n * 4, hipMemcpyDeviceToDevice, s));
    hipEvent_t ev;
    hipIpcEventHandle_t eh;
    int ev_ok = 0;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventInterprocess) == hipSuccess &&
        hipIpcGetEventHandle(&eh, ev) == hipSuccess) {
      ev_ok = 1;
      CK(hipEventRecord(ev, s));
    } else {
      (void)hipGetLastError();
    }
    Msg back{};
    back.ev = eh;
    back.ev_ok = ev_ok;
    auto t0 = std::chrono::steady_clock::now();
    if (write(to_recv[1], &back, sizeof back) != sizeof back) _exit(5);
    CK(hipStreamSynchronize(s));
    double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("sender: copy into the peer's buffer done %.1f ms after handing over (event ok=%d)\n", ms, ev_ok);
    char done;
    if (read(to_sender[0], &done, 1) != 1) _exit(6);
    CK(hipIpcCloseMemHandle(remote));
    _exit(0);
  }
  // RECEIVER
  CK(hipSetDevice(0));
  float* buf = nullptr;
  CK(hipMalloc(&buf, n * 4));
  CK(hipMemset(buf, 0, n * 4));
  CK(hipDeviceSynchronize());
  Msg m{};
  CK(hipIpcGetMemHandle(&m.mem, buf));
  if (write(to_sender[1], &m, sizeof m) != sizeof m) return 7;
  Msg back;
  if (read(to_recv[0], &back, sizeof back) != sizeof back) return 8;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* out = nullptr;
  CK(hipMalloc(&out, n * 4));
  int ok_ev = 0;
  auto t0 = std::chrono::steady_clock::now();
  if (back.ev_ok) {
    hipEvent_t ev;
    hipError_t e = hipIpcOpenEventHandle(&ev, back.ev);
    if (e == hipSuccess) {
      CK(hipStreamWaitEvent(s, ev, 0));
      ok_ev = 1;
    } else {
      printf("receiver: hipIpcOpenEventHandle failed: %s\n", hipGetErrorString(e));
      (void)hipGetLastError();
    }
  }
  CK(hipMemcpyAsync(out, buf, n * 4, hipMemcpyDeviceToDevice, s));
  CK(hipStreamSynchronize(s));
  double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  float h[4];
  CK(hipMemcpy(h, out + n - 4, 16, hipMemcpyDeviceToHost));
  printf("receiver: waited on the IPC event=%d, copy-out done after %.1f ms, last value %.1f (%s)\n", ok_ev, ms, h[3],
         h[3] == 42.0f ? "DATA ARRIVED: the stream wait held" : "stale: the wait did not hold");
  char done = 1;
  if (write(to_sender[1], &done, 1) != 1) return 9;
  int st = 0;
  waitpid(pid, &st, 0);
  printf("sender exit status %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);
  return 0;
}
