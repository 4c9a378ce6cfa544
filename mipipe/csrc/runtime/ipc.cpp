// Device-memory P2P transport between processes: see ipc.h.
#include "ipc.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "runtime.h"

namespace mipipe {
namespace ipc {

namespace {

constexpr uint64_t kMagic = 0x6d69706970654c4bull;  // "mipipeLK"
constexpr int kMaxSlots = 1024;

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("mipipe ipc: ") + what + ": " + hipGetErrorString(e));
  }
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    if (d < 0) return;
    check(hipGetDevice(&prev), "hipGetDevice");
    if (prev != d) check(hipSetDevice(d), "hipSetDevice");
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

}  // namespace

struct alignas(64) SlotCtl {
  std::atomic<uint64_t> full;
  std::atomic<uint64_t> freed;
  uint64_t bytes;
  uint8_t pad[40];
};

// Shared-memory layout: header, per-slot control, then (host mode) the slots.
struct Shared {
  uint64_t magic;
  int64_t nslots;
  int64_t slot_bytes;
  int32_t device;        // receiver's device, -1 host mode
  int32_t use_events;
  std::atomic<uint32_t> aborted;
  std::atomic<uint32_t> sender_ready;
  std::atomic<uint32_t> sender_detached;     // the sender has closed its mapping of the ring
  hipIpcMemHandle_t mem;                     // the slot ring
  hipIpcEventHandle_t freed_ev[kMaxSlots];   // receiver's events, waited by the sender
  hipIpcEventHandle_t full_ev[kMaxSlots];    // sender's events, waited by the receiver
  SlotCtl slots[kMaxSlots];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics need lock-free 64-bit");

// ------------------------------------------------------------------ proxy
// Publishes a shared counter once a local event completes: the cross-process
// completion signal for links whose runtime lacks interprocess events.
namespace {

struct ProxyItem {
  hipEvent_t event;
  int device;
  std::atomic<uint64_t>* target;
  uint64_t value;
};

class Proxy {
 public:
  static Proxy& get() {
    static Proxy p;
    return p;
  }
  void push(const ProxyItem& it) {
    {
      std::lock_guard<std::mutex> l(mu_);
      q_.push_back(it);
      ++inflight_;
      if (!thread_.joinable()) thread_ = std::thread([this] { loop(); });
    }
    cv_.notify_one();
  }
  // Blocks until every pushed item has been published.
  void drain() {
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [this] { return inflight_ == 0; });
  }
  void shutdown() {
    {
      std::lock_guard<std::mutex> l(mu_);
      stop_ = true;
    }
    cv_.notify_one();
    if (thread_.joinable()) thread_.join();
    stop_ = false;
  }
  ~Proxy() { shutdown(); }

 private:
  void loop() {
    for (;;) {
      ProxyItem it;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop requested and drained
        it = q_.front();
        q_.pop_front();
      }
      if (it.device >= 0) {
        (void)hipSetDevice(it.device);
        (void)hipEventSynchronize(it.event);
        (void)hipEventDestroy(it.event);
      }
      it.target->store(it.value, std::memory_order_release);
      {
        std::lock_guard<std::mutex> l(mu_);
        --inflight_;
      }
      done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  int64_t inflight_ = 0;
  std::deque<ProxyItem> q_;
  std::thread thread_;
  bool stop_ = false;
};

}  // namespace

void proxy_shutdown() { Proxy::get().shutdown(); }

// ------------------------------------------------------------------ Link
static size_t map_size(int64_t nslots, int64_t slot_bytes, bool host) {
  size_t n = sizeof(Shared);
  n = (n + 4095) & ~size_t(4095);
  if (host) n += size_t(nslots) * size_t(slot_bytes);
  return n;
}

std::unique_ptr<Link> Link::create(const std::string& name, int device, int64_t nslots, int64_t slot_bytes,
                                   bool use_ipc_events) {
  if (nslots < 1 || nslots > kMaxSlots) throw std::runtime_error("mipipe ipc: nslots must be in [1, 1024]");
  if (slot_bytes < 16) throw std::runtime_error("mipipe ipc: slot_bytes too small");
  slot_bytes = (slot_bytes + 255) & ~int64_t(255);
  std::unique_ptr<Link> L(new Link());
  L->name_ = name;
  L->sender_ = false;
  L->device_ = device;
  const bool host = device < 0;
  L->map_bytes_ = map_size(nslots, slot_bytes, host);
  L->fd_ = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (L->fd_ < 0) throw std::runtime_error("mipipe ipc: shm_open(create) failed for " + name + ": " + strerror(errno));
  if (ftruncate(L->fd_, (off_t)L->map_bytes_) != 0) {
    shm_unlink(name.c_str());
    throw std::runtime_error("mipipe ipc: ftruncate failed: " + std::string(strerror(errno)));
  }
  void* p = mmap(nullptr, L->map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, L->fd_, 0);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    throw std::runtime_error("mipipe ipc: mmap failed: " + std::string(strerror(errno)));
  }
  L->sh_ = static_cast<Shared*>(p);
  Shared* sh = L->sh_;
  sh->nslots = nslots;
  sh->slot_bytes = slot_bytes;
  sh->device = device;
  sh->use_events = (!host && use_ipc_events) ? 1 : 0;
  sh->aborted.store(0);
  sh->sender_ready.store(0);
  sh->sender_detached.store(0);
  for (int k = 0; k < nslots; ++k) {
    sh->slots[k].full.store(0);
    sh->slots[k].freed.store(0);
    sh->slots[k].bytes = 0;
  }
  if (host) {
    L->data_ = reinterpret_cast<char*>(p) + ((sizeof(Shared) + 4095) & ~size_t(4095));
  } else {
    DeviceGuard g(device);
    void* d = nullptr;
    check(hipMalloc(&d, size_t(nslots) * size_t(slot_bytes)), "hipMalloc(slots)");
    L->data_ = static_cast<char*>(d);
    L->owns_data_ = true;
    check(hipIpcGetMemHandle(&sh->mem, d), "hipIpcGetMemHandle");
    if (sh->use_events) {
      L->local_events_ = new hipEvent_t[nslots];
      for (int k = 0; k < nslots; ++k) {
        check(hipEventCreateWithFlags(&L->local_events_[k], hipEventDisableTiming | hipEventInterprocess),
              "hipEventCreateWithFlags(interprocess)");
        check(hipIpcGetEventHandle(&sh->freed_ev[k], L->local_events_[k]), "hipIpcGetEventHandle");
      }
    }
  }
  std::atomic_thread_fence(std::memory_order_seq_cst);
  reinterpret_cast<std::atomic<uint64_t>*>(&sh->magic)->store(kMagic, std::memory_order_release);
  return L;
}

std::unique_ptr<Link> Link::attach(const std::string& name, int device, int engine, double timeout_s) {
  std::unique_ptr<Link> L(new Link());
  L->name_ = name;
  L->sender_ = true;
  L->device_ = device;
  L->engine_ = engine;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  for (;;) {
    L->fd_ = shm_open(name.c_str(), O_RDWR, 0600);
    if (L->fd_ >= 0) {
      struct stat st;
      if (fstat(L->fd_, &st) == 0 && (size_t)st.st_size >= sizeof(Shared)) break;
      close(L->fd_);
      L->fd_ = -1;
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("mipipe ipc: timed out attaching to " + name);
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  struct stat st;
  fstat(L->fd_, &st);
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, L->fd_, 0);
  if (p == MAP_FAILED) throw std::runtime_error("mipipe ipc: mmap(attach) failed");
  L->map_bytes_ = (size_t)st.st_size;
  L->sh_ = static_cast<Shared*>(p);
  Shared* sh = L->sh_;
  while (reinterpret_cast<std::atomic<uint64_t>*>(&sh->magic)->load(std::memory_order_acquire) != kMagic) {
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("mipipe ipc: " + name + " never became ready");
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  const bool host = sh->device < 0;
  if (host != (device < 0)) throw std::runtime_error("mipipe ipc: host/device mode mismatch on " + name);
  if (host) {
    L->data_ = reinterpret_cast<char*>(p) + ((sizeof(Shared) + 4095) & ~size_t(4095));
  } else {
    DeviceGuard g(device);
    void* d = nullptr;
    check(hipIpcOpenMemHandle(&d, sh->mem, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    L->data_ = static_cast<char*>(d);
    check(hipStreamCreateWithFlags(&L->copy_stream_, hipStreamNonBlocking), "hipStreamCreate(copy)");
    const int64_t n = sh->nslots;
    if (sh->use_events) {
      L->local_events_ = new hipEvent_t[n];
      L->remote_events_ = new hipEvent_t[n];
      for (int k = 0; k < n; ++k) {
        check(hipEventCreateWithFlags(&L->local_events_[k], hipEventDisableTiming | hipEventInterprocess),
              "hipEventCreateWithFlags(interprocess)");
        check(hipIpcGetEventHandle(&sh->full_ev[k], L->local_events_[k]), "hipIpcGetEventHandle");
        check(hipIpcOpenEventHandle(&L->remote_events_[k], sh->freed_ev[k]), "hipIpcOpenEventHandle");
      }
      L->remote_open_ = true;
    }
  }
  sh->sender_ready.store(1, std::memory_order_release);
  return L;
}

static bool ipc_debug() {
  static const bool on = [] {
    const char* v = getenv("MIPIPE_IPC_DEBUG");
    return v != nullptr && v[0] == '1';
  }();
  return on;
}

#define IPC_TRACE(...)                                     \
  do {                                                     \
    if (ipc_debug()) {                                     \
      fprintf(stderr, "[mipipe ipc %d] ", (int)getpid());  \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
    }                                                      \
  } while (0)

Link::~Link() {
  IPC_TRACE("destroy %s %s", sender_ ? "sender" : "receiver", name_.c_str());
  try {
    if (!host_mode() && sh_ != nullptr && !ipc_events()) Proxy::get().drain();  // no publish into a dead map
    IPC_TRACE("  proxy drained");
    if (!host_mode() && data_ != nullptr) {
      DeviceGuard g(device_);
      if (copy_stream_) (void)hipStreamSynchronize(copy_stream_);
      IPC_TRACE("  copy stream synchronized");
      if (sender_) {
        (void)hipIpcCloseMemHandle(data_);
        sh_->sender_detached.store(1, std::memory_order_release);
        IPC_TRACE("  unmapped the peer's ring");
      } else if (owns_data_) {
        // Free the ring only once no sender maps it: freeing memory a peer
        // process still maps can block until that peer lets go, and two
        // ranks tearing down their receivers first would wait on each other.
        // A ring still mapped is left to the process teardown.
        const bool mapped = sh_->sender_ready.load(std::memory_order_acquire) &&
                            !sh_->sender_detached.load(std::memory_order_acquire);
        if (!mapped) (void)hipFree(data_);
        IPC_TRACE("  ring %s", mapped ? "left mapped by the peer (not freed)" : "freed");
      }
      const int64_t n = sh_ ? sh_->nslots : 0;
      if (local_events_)
        for (int k = 0; k < n; ++k) (void)hipEventDestroy(local_events_[k]);
      if (remote_events_ && remote_open_)
        for (int k = 0; k < n; ++k) (void)hipEventDestroy(remote_events_[k]);
      if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
    }
  } catch (...) {
  }
  IPC_TRACE("  events destroyed");
  delete[] local_events_;
  delete[] remote_events_;
  if (sh_) munmap(sh_, map_bytes_);
  if (fd_ >= 0) close(fd_);
  if (!sender_) shm_unlink(name_.c_str());  // idempotent: ENOENT after unlink() is fine
}

int64_t Link::nslots() const { return sh_->nslots; }
int64_t Link::slot_bytes() const { return sh_->slot_bytes; }
bool Link::ipc_events() const { return sh_->use_events != 0; }

void Link::abort() { sh_->aborted.store(1, std::memory_order_release); }
void Link::unlink() { shm_unlink(name_.c_str()); }

std::string Link::describe() const {
  std::ostringstream o;
  o << (sender_ ? "sender" : "receiver") << " of " << name_ << " (" << sh_->nslots << " slots x " << sh_->slot_bytes
    << " B, " << (host_mode() ? "host" : ("device " + std::to_string(device_)))
    << (ipc_events() ? ", ipc events" : (host_mode() ? "" : ", proxy-completed")) << ", next seq " << next_seq_ << ")";
  return o.str();
}

void Link::wait_for(const char* what, uint64_t seq, int slot, bool full, double timeout_s) const {
  const SlotCtl& c = sh_->slots[slot];
  const std::atomic<uint64_t>& ctr = full ? c.full : c.freed;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  for (int spin = 0;; ++spin) {
    if (ctr.load(std::memory_order_acquire) >= seq) return;
    if (sh_->aborted.load(std::memory_order_acquire))
      throw std::runtime_error("mipipe ipc: " + describe() + ": the link was aborted while waiting for " + what);
    if (spin > 2000) {
      if (std::chrono::steady_clock::now() > deadline) {
        std::ostringstream o;
        o << "mipipe ipc: " << describe() << ": timed out after " << timeout_s << " s waiting for " << what
          << " (slot " << slot << ", need " << seq << ", have " << ctr.load() << ")";
        throw std::runtime_error(o.str());
      }
      std::this_thread::sleep_for(std::chrono::microseconds(spin > 20000 ? 200 : 5));
    }
  }
}

uint64_t Link::send(const void* src, size_t bytes, hipStream_t producer, double timeout_s) {
  if (!sender_) throw std::runtime_error("mipipe ipc: send on a receiving link");
  if ((int64_t)bytes > sh_->slot_bytes) {
    std::ostringstream o;
    o << "mipipe ipc: message of " << bytes << " B exceeds the slot size " << sh_->slot_bytes << " of " << name_;
    throw std::runtime_error(o.str());
  }
  const uint64_t s = next_seq_;
  const int64_t n = sh_->nslots;
  const int k = int(s % uint64_t(n));
  SlotCtl& c = sh_->slots[k];
  // the slot's previous message (s - n) must have been released
  if (s >= uint64_t(n)) wait_for("a free slot", s - uint64_t(n) + 1, k, false, timeout_s);
  char* dst = data_ + size_t(k) * size_t(sh_->slot_bytes);
  if (host_mode()) {
    std::memcpy(dst, src, bytes);
    c.bytes = bytes;
    c.full.store(s + 1, std::memory_order_release);
    ++next_seq_;
    return s;
  }
  DeviceGuard g(device_);
  if (s >= uint64_t(n) && ipc_events()) check(hipStreamWaitEvent(copy_stream_, remote_events_[k], 0), "wait freed");
  rt::stream_wait(copy_stream_, producer, device_);
  if (bytes) {
    if (engine_ == 1) {
      rt::blit_copy(dst, src, bytes, copy_stream_);
    } else {
      check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, copy_stream_), "hipMemcpyAsync(send)");
    }
  }
  c.bytes = bytes;
  if (ipc_events()) {
    check(hipEventRecord(local_events_[k], copy_stream_), "hipEventRecord(full)");
    c.full.store(s + 1, std::memory_order_release);
  } else {
    hipEvent_t e;
    check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate(proxy)");
    check(hipEventRecord(e, copy_stream_), "hipEventRecord(proxy)");
    Proxy::get().push({e, device_, &c.full, s + 1});
  }
  ++next_seq_;
  return s;
}

uint64_t Link::post() {
  if (sender_) throw std::runtime_error("mipipe ipc: post on a sending link");
  return next_seq_++;
}

void Link::open_remote_events() {
  if (remote_open_ || !ipc_events()) return;
  // the sender's event handles exist once it has attached
  while (!sh_->sender_ready.load(std::memory_order_acquire)) {
    if (sh_->aborted.load()) throw std::runtime_error("mipipe ipc: aborted before the sender attached");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  const int64_t n = sh_->nslots;
  remote_events_ = new hipEvent_t[n];
  for (int k = 0; k < n; ++k) check(hipIpcOpenEventHandle(&remote_events_[k], sh_->full_ev[k]), "hipIpcOpenEventHandle");
  remote_open_ = true;
}

void Link::wait(uint64_t seq, void* dst, size_t bytes, hipStream_t consumer, double timeout_s) {
  if (sender_) throw std::runtime_error("mipipe ipc: wait on a sending link");
  const int64_t n = sh_->nslots;
  const int k = int(seq % uint64_t(n));
  SlotCtl& c = sh_->slots[k];
  wait_for("the message", seq + 1, k, true, timeout_s);
  if (c.full.load(std::memory_order_acquire) != seq + 1) {
    std::ostringstream o;
    o << "mipipe ipc: " << describe() << ": slot " << k << " holds message " << c.full.load() - 1 << ", expected "
      << seq << " (receives posted out of order, or more than " << n << " in flight)";
    throw std::runtime_error(o.str());
  }
  if (c.bytes != bytes) {
    std::ostringstream o;
    o << "mipipe ipc: " << describe() << ": message " << seq << " is " << c.bytes << " B, the receive expects "
      << bytes;
    throw std::runtime_error(o.str());
  }
  const char* src = data_ + size_t(k) * size_t(sh_->slot_bytes);
  if (host_mode()) {
    std::memcpy(dst, src, bytes);
    c.freed.store(seq + 1, std::memory_order_release);
    return;
  }
  DeviceGuard g(device_);
  if (ipc_events()) {
    open_remote_events();
    check(hipStreamWaitEvent(consumer, remote_events_[k], 0), "wait full");
  }
  if (bytes) check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, consumer), "hipMemcpyAsync(recv)");
  if (ipc_events()) {
    check(hipEventRecord(local_events_[k], consumer), "hipEventRecord(freed)");
    c.freed.store(seq + 1, std::memory_order_release);
  } else {
    hipEvent_t e;
    check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate(proxy)");
    check(hipEventRecord(e, consumer), "hipEventRecord(proxy)");
    Proxy::get().push({e, device_, &c.freed, seq + 1});
  }
}

bool Link::done(uint64_t seq) const {
  const int k = int(seq % uint64_t(sh_->nslots));
  const SlotCtl& c = sh_->slots[k];
  return (sender_ ? c.full : c.freed).load(std::memory_order_acquire) >= seq + 1;
}

}  // namespace ipc
}  // namespace mipipe
