// ctypes-loadable waiter/setter kernels for tools/micro/queue_share_torch.py:
// the same bounded flag-poll test as queue_share.hip, launched on torch's own
// streams (the default stream and streams from torch's pool -- the pool
// ProcessGroupNCCL draws its communicator streams from).
#include <hip/hip_runtime.h>

__global__ void __launch_bounds__(64) qs_waiter(int* flag, long long* out) {
  const int lane = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  long long seen = -1;
  for (int it = 0; it < (1 << 22); ++it) {
    int v = __hip_atomic_load(flag + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
    if (v != 0) { seen = (long long)dt; break; }
    if (dt > 5000000ull) break;  // 50 ms
    __builtin_amdgcn_s_sleep(2);
  }
  out[lane] = seen;
}

__global__ void __launch_bounds__(64) qs_setter(int* flag) {
  __hip_atomic_store(flag + threadIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

extern "C" int qs_launch_waiter(void* stream, void* flag, void* out) {
  hipLaunchKernelGGL(qs_waiter, dim3(1), dim3(64), 0, (hipStream_t)stream, (int*)flag, (long long*)out);
  return (int)hipGetLastError();
}

extern "C" int qs_launch_setter(void* stream, void* flag) {
  hipLaunchKernelGGL(qs_setter, dim3(1), dim3(64), 0, (hipStream_t)stream, (int*)flag);
  return (int)hipGetLastError();
}
