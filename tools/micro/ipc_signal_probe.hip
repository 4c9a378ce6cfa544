// Probe: can two processes sharing one MI355X order each other's streams on the
// GPU, with no host in the loop, through flags in IPC-exported device memory?
//   sender:   copy into the receiver's exported buffer, then hipStreamWriteValue64
//             of a sequence number into the receiver's exported flag word;
//   receiver: hipStreamWaitValue64(flag >= seq) on its compute stream, then use.
// Checks (1) the attribute, (2) data correctness behind a 0.3 s spin in the
// sender (the receiver's enqueue must return at once, its stream must wait),
// (3) GPU-side ping-pong latency with 1 MiB messages (one-way = round trip / 2),
// for flags from hipMalloc and from hipExtMallocWithFlags(hipMallocSignalMemory).
// Forks before any HIP call; each process initialises HIP on its own.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/ipc_signal_probe.hip -o tools/micro/bin/ipc_signal_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "[pid %d] %s failed: %s\n", getpid(), #x, hipGetErrorString(e_)); \
      _exit(3);                                                                        \
    }                                                                                  \
  } while (0)

struct Handles {
  hipIpcMemHandle_t data;   // receiver's data buffer
  hipIpcMemHandle_t flag;   // receiver's "full" flag (receiver waits on it)
  hipIpcMemHandle_t ack;    // sender's "freed" flag (sender waits on it)
};

__global__ void fill(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

__global__ void check(const float* p, size_t n, float v, unsigned* bad) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    if (p[i] != v) atomicAdd(bad, 1u);
}

__global__ void spin(unsigned long long ticks) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

static void* alloc_flag(bool signal) {
  void* p = nullptr;
  if (signal) CK(hipExtMallocWithFlags(&p, 4096, hipMallocSignalMemory));
  else CK(hipMalloc(&p, 4096));
  CK(hipMemset(p, 0, 4096));
  return p;
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int run(bool signal) {
  const size_t n = 256u << 10;  // 1 MiB of floats
  const int iters = 2000;
  int to_sender[2], to_recv[2];
  if (pipe(to_sender) || pipe(to_recv)) return 1;
  pid_t pid = fork();
  if (pid == 0) {  // ------------------------------------------------ sender
    Handles h;
    if (read(to_sender[0], &h, sizeof h) != sizeof h) _exit(4);
    CK(hipSetDevice(0));
    void *rdata = nullptr, *rflag = nullptr;
    CK(hipIpcOpenMemHandle(&rdata, h.data, hipIpcMemLazyEnablePeerAccess));
    CK(hipIpcOpenMemHandle(&rflag, h.flag, hipIpcMemLazyEnablePeerAccess));
    void* ack = alloc_flag(signal);
    Handles back = h;
    if (hipIpcGetMemHandle(&back.ack, ack) != hipSuccess) {
      fprintf(stderr, "sender: hipIpcGetMemHandle(ack, signal=%d) refused\n", (int)signal);
      _exit(5);
    }
    if (write(to_recv[1], &back, sizeof back) != sizeof back) _exit(4);
    float* local = nullptr;
    CK(hipMalloc(&local, n * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(fill, dim3(256), dim3(256), 0, s, local, n, 42.0f);
    // (2) correctness behind a long spin
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 30000000ull);  // 0.3 s
    CK(hipMemcpyAsync(rdata, local, n * 4, hipMemcpyDeviceToDevice, s));
    CK(hipStreamWriteValue64(s, rflag, 1, 0));
    CK(hipStreamSynchronize(s));
    // (3) ping-pong: message k -> flag = k + 2; wait ack >= k + 1 before reusing the buffer
    for (int k = 0; k < iters; ++k) {
      CK(hipStreamWaitValue64(s, ack, (uint64_t)k + 1, hipStreamWaitValueGte, ~0ull));
      CK(hipMemcpyAsync(rdata, local, n * 4, hipMemcpyDeviceToDevice, s));
      CK(hipStreamWriteValue64(s, rflag, (uint64_t)k + 2, 0));
    }
    CK(hipStreamSynchronize(s));
    char c;
    if (read(to_sender[0], &c, 1) != 1) _exit(4);  // receiver done before unmapping
    CK(hipIpcCloseMemHandle(rdata));
    CK(hipIpcCloseMemHandle(rflag));
    _exit(0);
  }
  // ---------------------------------------------------------------- receiver
  CK(hipSetDevice(0));
  int attr = -1;
  CK(hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0));
  float* data = nullptr;
  CK(hipMalloc(&data, n * 4));
  CK(hipMemset(data, 0, n * 4));
  void* flag = alloc_flag(signal);
  Handles h;
  CK(hipIpcGetMemHandle(&h.data, data));
  if (hipIpcGetMemHandle(&h.flag, flag) != hipSuccess) {
    printf("signal=%d: hipIpcGetMemHandle on the flag allocation refused\n", (int)signal);
    kill(pid, 9);
    waitpid(pid, nullptr, 0);
    return 0;
  }
  if (write(to_sender[1], &h, sizeof h) != sizeof h) return 1;
  Handles back;
  if (read(to_recv[0], &back, sizeof back) != sizeof back) {
    int st = 0;
    waitpid(pid, &st, 0);
    printf("signal=%d: sender failed (exit %d)\n", (int)signal, WEXITSTATUS(st));
    return 0;
  }
  void* rack = nullptr;
  CK(hipIpcOpenMemHandle(&rack, back.ack, hipIpcMemLazyEnablePeerAccess));
  unsigned* bad = nullptr;
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const double t0 = now();
  CK(hipStreamWaitValue64(s, flag, 1, hipStreamWaitValueGte, ~0ull));
  hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, s, data, n, 42.0f, bad);
  const double t_enq = now() - t0;
  CK(hipStreamSynchronize(s));
  const double t_sync = now() - t0;
  unsigned nbad = 0;
  CK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
  CK(hipMemset(data, 0, n * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  const double h0 = now();
  for (int k = 0; k < iters; ++k) {
    CK(hipStreamWriteValue64(s, rack, (uint64_t)k + 1, 0));  // buffer free for message k
    CK(hipStreamWaitValue64(s, flag, (uint64_t)k + 2, hipStreamWaitValueGte, ~0ull));
  }
  const double h_enq = now() - h0;
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  hipLaunchKernelGGL(check, dim3(256), dim3(256), 0, s, data, n, 42.0f, bad);
  unsigned nbad2 = 0;
  CK(hipMemcpy(&nbad2, bad, 4, hipMemcpyDeviceToHost));
  if (write(to_sender[1], "x", 1) != 1) return 1;
  int st = 0;
  waitpid(pid, &st, 0);
  printf("flags from %s: attr CanUseStreamWaitValue=%d; behind a 0.3 s sender spin: receiver enqueue %.1f us, "
         "stream done after %.3f s, %u bad words; ping-pong %d x 1 MiB: %.1f us per round trip (one-way %.1f us), "
         "host enqueue of the loop %.1f us per message, %u bad words after; sender exit %d\n",
         signal ? "hipMallocSignalMemory" : "hipMalloc", attr, t_enq * 1e6, t_sync, nbad, iters, ms * 1e3 / iters,
         ms * 1e3 / iters / 2, h_enq * 1e6 / iters, nbad2 - nbad, WEXITSTATUS(st));
  return 0;
}

int main() {
  // each mode in a child of its own: a process that has initialised HIP must not fork a HIP user
  for (int mode = 0; mode < 2; ++mode) {
    fflush(stdout);
    pid_t pid = fork();
    if (pid == 0) {
      run(mode == 1);
      fflush(stdout);
      _exit(0);
    }
    int st = 0;
    waitpid(pid, &st, 0);
  }
  return 0;
}
