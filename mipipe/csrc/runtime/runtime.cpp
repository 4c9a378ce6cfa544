// Native pipeline runtime.
//
// Streams: the scheduler needs chunks x stages copy streams; torch's pool has 32
// per priority per device and hands them out round-robin, so deep pipelines
// would alias copy streams and serialise unrelated transfers.  We create
// dedicated non-blocking HIP streams instead and keep them for the process
// lifetime (streams are cheap; destroying them while the allocator still holds
// events recorded on them is not).
//
// Events: every Copy/Wait needs an event record + stream wait.  Creating and
// destroying an event per call costs microseconds; a per-device pool of
// timing-disabled events reused round-robin costs one record + one wait.  A
// stream wait captures the event's state at call time, so re-recording the
// event later never affects an earlier wait -- the pool only has to be big
// enough that concurrent callers do not interleave a record and its wait,
// which the per-device mutex guarantees.
#include "runtime.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <array>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>

namespace mipipe {
namespace rt {

namespace {

constexpr int kMaxDevices = 64;
constexpr int kEventsPerDevice = 64;

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("mipipe runtime: ") + what + ": " + hipGetErrorString(e));
  }
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != d) check(hipSetDevice(d), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

struct EventPool {
  std::mutex mu;
  std::array<hipEvent_t, kEventsPerDevice> events{};
  int next = 0;
  bool init = false;

  hipEvent_t take(int device) {
    if (!init) {
      DeviceGuard g(device);
      for (auto& e : events) check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreateWithFlags");
      init = true;
    }
    hipEvent_t e = events[next];
    next = (next + 1) % kEventsPerDevice;
    return e;
  }
};

EventPool& pool(int device) {
  static std::array<EventPool, kMaxDevices> pools;
  if (device < 0 || device >= kMaxDevices) throw std::runtime_error("mipipe runtime: bad device index");
  return pools[device];
}

std::mutex g_stream_mu;
std::vector<hipStream_t>& streams() {
  static std::vector<hipStream_t> s;
  return s;
}

std::mutex g_peer_mu;

}  // namespace

hipStream_t stream_acquire(int device, int priority) {
  DeviceGuard g(device);
  int least = 0, greatest = 0;
  check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
  const int prio = priority < 0 ? greatest : least;
  hipStream_t s = nullptr;
  check(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio), "hipStreamCreateWithPriority");
  std::lock_guard<std::mutex> lock(g_stream_mu);
  streams().push_back(s);
  return s;
}

void stream_wait(hipStream_t waiting, hipStream_t waited, int device) {
  if (waiting == waited) return;
  EventPool& p = pool(device);
  std::lock_guard<std::mutex> lock(p.mu);
  hipEvent_t e = p.take(device);
  check(hipEventRecord(e, waited), "hipEventRecord");
  check(hipStreamWaitEvent(waiting, e, 0), "hipStreamWaitEvent");
}

// Grid-stride 16-byte copy.  A launch of <= 4 waves per CU (1024 blocks of
// 256) saturates HBM / an xGMI link without tying up the whole chip.
__global__ void __launch_bounds__(256) blit16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                     size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = src[i];
}

void blit_copy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  if (bytes == 0) return;
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes) & 15) {
    check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream), "hipMemcpyAsync(blit fallback)");
    return;
  }
  const size_t n = bytes / 16;
  const size_t want = (n + 255) / 256;
  const unsigned blocks = (unsigned)(want < 1024 ? want : 1024);
  hipLaunchKernelGGL(blit16_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<const uint4*>(src),
                     static_cast<uint4*>(dst), n);
  check(hipGetLastError(), "blit16_kernel launch");
}

void peer_copy(void* dst, int dst_device, const void* src, int src_device, size_t bytes, hipStream_t src_stream,
               hipStream_t dst_stream, int engine) {
  if (bytes == 0) return;
  {
    // The destination block may have been freed by work still pending on
    // dst_stream: the copy (on src_stream) must start after it.
    EventPool& p = pool(dst_device);
    std::lock_guard<std::mutex> lock(p.mu);
    hipEvent_t e = p.take(dst_device);
    check(hipEventRecord(e, dst_stream), "hipEventRecord(dst)");
    check(hipStreamWaitEvent(src_stream, e, 0), "hipStreamWaitEvent(src)");
  }
  {
    DeviceGuard g(src_device);
    if (engine == kCopyBlit) {
      blit_copy(dst, src, bytes, src_stream);
    } else if (dst_device == src_device) {
      check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, src_stream), "hipMemcpyAsync");
    } else {
      // the copy engines only (peer access is on: Pipe enables it): a peer copy must not hold CUs for the
      // whole xGMI transfer (profiles/nocu_copy_r5.txt); hipMemcpyPeerAsync if the runtime refuses the kind
      if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, src_stream) != hipSuccess) {
        (void)hipGetLastError();
        check(hipMemcpyPeerAsync(dst, dst_device, src, src_device, bytes, src_stream), "hipMemcpyPeerAsync");
      }
    }
  }
  {
    EventPool& p = pool(src_device);
    std::lock_guard<std::mutex> lock(p.mu);
    hipEvent_t e = p.take(src_device);
    check(hipEventRecord(e, src_stream), "hipEventRecord(src)");
    check(hipStreamWaitEvent(dst_stream, e, 0), "hipStreamWaitEvent(dst)");
  }
}

std::string copy_nocu(void* dst, const void* src, size_t bytes, hipStream_t stream) {
  const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, stream);
  if (e == hipSuccess) return std::string();
  (void)hipGetLastError();
  return hipGetErrorString(e);
}

bool can_access_peer(int device, int peer) {
  int ok = 0;
  check(hipDeviceCanAccessPeer(&ok, device, peer), "hipDeviceCanAccessPeer");
  return ok != 0;
}

void enable_peer_access(const std::vector<int>& devices) {
  std::lock_guard<std::mutex> lock(g_peer_mu);
  for (int d : devices) {
    for (int q : devices) {
      if (d == q || !can_access_peer(d, q)) continue;
      DeviceGuard g(d);
      hipError_t e = hipDeviceEnablePeerAccess(q, 0);
      if (e == hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        continue;
      }
      check(e, "hipDeviceEnablePeerAccess");
    }
  }
}

void range_push(const std::string& label) { roctxRangePushA(label.c_str()); }
void range_pop() { roctxRangePop(); }
void mark(const std::string& label) { roctxMarkA(label.c_str()); }

}  // namespace rt
}  // namespace mipipe
