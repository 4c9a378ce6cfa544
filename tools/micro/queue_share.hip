// Do kernels of different HIP streams that share a hardware queue run
// concurrently, or in submission order?  (GPU_MAX_HW_QUEUES is 4 on this pool.)
//
// Why it matters: an RCCL receive is a kernel that spins until the peer's data
// arrives.  The pipeline engine pre-posts its receives on the communicators'
// streams; if one of those streams shares a hardware queue with the compute
// stream AND the queue runs packets in order, compute kernels issued after the
// pre-posted receive cannot start until the receive completes -- which breaks
// the pipeline overlap, and deadlocks when the awaited data needs that compute
// (looping placements: rank 0 receives from rank n-1).
//
// Test: for each stream j != 0 of N streams, stream 0 runs a WAITER kernel
// that polls a flag (bounded: 100 ms by s_memrealtime, plus an iteration cap),
// then stream j runs a SETTER kernel that writes the flag (vector stores).
// Concurrent -> the waiter sees the flag within microseconds; serialised ->
// the waiter times out first.  Then the same with the waiter on a
// high-priority stream.
//
// Usage: queue_share [nstreams=8]   (run with GPU_MAX_HW_QUEUES=4 and =16)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void __launch_bounds__(64) waiter(int* flag, long long* out) {
  const int lane = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long limit = 10000000ull;  // 100 ms at the 100 MHz constant clock
  long long seen = -1;
  for (int it = 0; it < (1 << 22); ++it) {
    int v = __hip_atomic_load(flag + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
    if (v != 0) { seen = (long long)dt; break; }
    if (dt > limit) break;
    __builtin_amdgcn_s_sleep(2);
  }
  out[lane] = seen;
}

__global__ void __launch_bounds__(64) setter(int* flag) {
  __hip_atomic_store(flag + threadIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static void run(const char* what, hipStream_t ws, hipStream_t ss, int* flag, long long* out, long long* host) {
  CK(hipMemset(flag, 0, 64 * sizeof(int)));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, ws, flag, out);
  hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, ss, flag);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(host, out, 64 * sizeof(long long), hipMemcpyDeviceToHost));
  if (host[0] < 0)
    printf("%-40s SERIALISED (waiter timed out at 100 ms)\n", what);
  else
    printf("%-40s concurrent (flag seen after %.1f us)\n", what, host[0] / 100.0);
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 8;
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  printf("GPU_MAX_HW_QUEUES=%s, %d streams (+ one high-priority)\n", q ? q : "(unset)", n);
  int *flag;
  long long *out, host[64];
  CK(hipMalloc(&flag, 64 * sizeof(int)));
  CK(hipMalloc(&out, 64 * sizeof(long long)));
  std::vector<hipStream_t> s(n);
  for (int i = 0; i < n; ++i) CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
  int lo, hi;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t high;
  CK(hipStreamCreateWithPriority(&high, hipStreamNonBlocking, hi));
  char label[96];
  for (int j = 1; j < n; ++j) {
    snprintf(label, sizeof label, "waiter stream 0, setter stream %d", j);
    run(label, s[0], s[j], flag, out, host);
  }
  for (int j = 0; j < n; ++j) {
    snprintf(label, sizeof label, "waiter high-prio, setter stream %d", j);
    run(label, high, s[j], flag, out, host);
  }
  snprintf(label, sizeof label, "waiter stream 0, setter null stream");
  run(label, s[0], 0, flag, out, host);
  return 0;
}
