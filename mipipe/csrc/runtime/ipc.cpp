// Device-memory P2P transport between processes, completed on the GPU: see ipc.h.
#include "ipc.h"

#include <algorithm>
#include <vector>

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <sstream>
#include <stdexcept>
#include <thread>

#include "runtime.h"

namespace mipipe {
namespace ipc {

namespace {

constexpr uint64_t kMagic = 0x6d69706970654c32ull;  // "mipipeL2"
constexpr int kMaxSlots = 1024;
// Device mode: the slots live in allocations of at most ~1 GiB each (one IPC handle per chunk).  Importing a single
// 3 GiB allocation from another process stalled inside hipIpcOpenMemHandle (profiles/ipc_import_stall_r5.txt).
constexpr int64_t kChunkBytes = int64_t(1) << 30;
constexpr int kMaxChunks = 64;
constexpr int64_t kFlagStride = 64;  // one flag word per 64-byte line

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

int64_t flag_bytes(int64_t nslots) { return (nslots * kFlagStride + 4095) & ~int64_t(4095); }

}  // namespace

struct alignas(64) SlotCtl {  // host mode: the flags themselves; device mode: host-side counts for describe()
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
  int32_t device;                            // receiver's device, -1 host mode
  int32_t pad0;
  std::atomic<uint32_t> aborted;
  std::atomic<uint32_t> sender_ready;        // the sender has mapped the ring and exported its freed flags
  std::atomic<uint32_t> sender_detached;     // the sender has unmapped the ring
  std::atomic<uint32_t> receiver_detached;   // the receiver has unmapped the freed flags
  std::atomic<uint64_t> sent;                // messages the sender has enqueued
  std::atomic<uint64_t> released;            // messages the receiver has released (enqueued)
  hipIpcMemHandle_t ring;                    // receiver's full flags (device mode)
  hipIpcMemHandle_t freed;                   // sender's freed flags
  int32_t nchunks;                           // device mode: the slot allocations
  int32_t slots_per_chunk;
  hipIpcMemHandle_t chunk[kMaxChunks];
  SlotCtl slots[kMaxSlots];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics need lock-free 64-bit");

static size_t map_size(int64_t nslots, int64_t slot_bytes, bool host) {
  size_t n = (sizeof(Shared) + 4095) & ~size_t(4095);
  if (host) n += size_t(nslots) * size_t(slot_bytes);
  return n;
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

std::unique_ptr<Link> Link::create(const std::string& name, int device, int64_t nslots, int64_t slot_bytes) {
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
  sh->aborted.store(0);
  sh->sender_ready.store(0);
  sh->sender_detached.store(0);
  sh->receiver_detached.store(0);
  sh->sent.store(0);
  sh->released.store(0);
  for (int k = 0; k < nslots; ++k) {
    sh->slots[k].full.store(0);
    sh->slots[k].freed.store(0);
    sh->slots[k].bytes = 0;
  }
  if (host) {
    L->ring_ = reinterpret_cast<char*>(p) + ((sizeof(Shared) + 4095) & ~size_t(4095));
  } else {
    DeviceGuard g(device);
    void* d = nullptr;
    check(hipMalloc(&d, size_t(flag_bytes(nslots))), "hipMalloc(full flags)");
    check(hipMemset(d, 0, size_t(flag_bytes(nslots))), "hipMemset(full flags)");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize(ring)");
    L->ring_ = static_cast<char*>(d);
    L->owns_ring_ = true;
    check(hipIpcGetMemHandle(&sh->ring, d), "hipIpcGetMemHandle(full flags)");
    int64_t spc = std::max<int64_t>(1, std::min<int64_t>(nslots, kChunkBytes / slot_bytes));
    int64_t nch = (nslots + spc - 1) / spc;
    if (nch > kMaxChunks) {
      spc = (nslots + kMaxChunks - 1) / kMaxChunks;
      nch = (nslots + spc - 1) / spc;
    }
    sh->nchunks = int32_t(nch);
    sh->slots_per_chunk = int32_t(spc);
    for (int64_t c = 0; c < nch; ++c) {
      const int64_t n = std::min(spc, nslots - c * spc);
      void* q = nullptr;
      check(hipMalloc(&q, size_t(n) * size_t(slot_bytes)), "hipMalloc(slot chunk)");
      L->chunk_.push_back(static_cast<char*>(q));
      check(hipIpcGetMemHandle(&sh->chunk[c], q), "hipIpcGetMemHandle(slot chunk)");
    }
    IPC_TRACE("create %s: %lld slots of %lld B in %lld chunk(s)", name.c_str(), (long long)nslots,
              (long long)slot_bytes, (long long)nch);
    L->events_ = new hipEvent_t[nslots];
    for (int k = 0; k < nslots; ++k)
      check(hipEventCreateWithFlags(&L->events_[k], hipEventDisableTiming), "hipEventCreate(slot)");
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
  IPC_TRACE("attach %s: waiting for the block", name.c_str());
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
    L->ring_ = reinterpret_cast<char*>(p) + ((sizeof(Shared) + 4095) & ~size_t(4095));
  } else {
    DeviceGuard g(device);
    void* d = nullptr;
    IPC_TRACE("attach %s: opening the ring handle", name.c_str());
    check(hipIpcOpenMemHandle(&d, sh->ring, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(full flags)");
    L->ring_ = static_cast<char*>(d);
    for (int c = 0; c < sh->nchunks; ++c) {
      void* q = nullptr;
      check(hipIpcOpenMemHandle(&q, sh->chunk[c], hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(slot chunk)");
      L->chunk_.push_back(static_cast<char*>(q));
    }
    IPC_TRACE("attach %s: ring mapped (%d chunk(s))", name.c_str(), sh->nchunks);
    void* f = nullptr;
    check(hipMalloc(&f, size_t(flag_bytes(sh->nslots))), "hipMalloc(freed flags)");
    check(hipMemset(f, 0, size_t(flag_bytes(sh->nslots))), "hipMemset(freed flags)");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize(freed flags)");
    IPC_TRACE("attach %s: freed flags ready", name.c_str());
    L->freed_ = static_cast<char*>(f);
    L->owns_freed_ = true;
    check(hipIpcGetMemHandle(&sh->freed, f), "hipIpcGetMemHandle(freed flags)");
    check(hipStreamCreateWithFlags(&L->copy_stream_, hipStreamNonBlocking), "hipStreamCreate(copy)");
    const int64_t n = sh->nslots;
    L->events_ = new hipEvent_t[n];
    for (int k = 0; k < n; ++k)
      check(hipEventCreateWithFlags(&L->events_[k], hipEventDisableTiming), "hipEventCreate(slot)");
  }
  sh->sender_ready.store(1, std::memory_order_release);
  IPC_TRACE("attach %s: done", name.c_str());
  return L;
}


Link::~Link() {
  IPC_TRACE("destroy %s %s", sender_ ? "sender" : "receiver", name_.c_str());
  try {
    if (!host_mode() && sh_ != nullptr) {
      DeviceGuard g(device_);
      // Everything this side queued on the link has run before a mapping goes.
      // Each slot's event is recorded right after the flag write of the last
      // send (on the stream the copy used: the copy stream, or the producer's
      // for the inline engines) or the last release (the consumer's stream),
      // so those events cover every write into the peer's memory.  Bounded:
      // after a peer failure a send may wait forever for a slot the dead
      // receiver never frees -- then the mappings are left to process teardown
      // instead of hanging here (abort() releases this side's own waits).
      if (!drain(30.0)) {
        IPC_TRACE("  %s: queued work did not drain in 30 s; mappings left to teardown", name_.c_str());
        throw std::runtime_error("undrained");
      }
      if (sender_) {
        if (ring_) (void)hipIpcCloseMemHandle(ring_);
        for (char* q : chunk_) (void)hipIpcCloseMemHandle(q);
        sh_->sender_detached.store(1, std::memory_order_release);
        // The receiver maps our freed flags until it detaches; freeing memory a
        // peer still maps can block until it lets go (two ranks tearing down
        // in opposite orders would wait on each other), so a still-mapped
        // allocation is left to the process teardown.
        if (owns_freed_ && sh_->receiver_detached.load(std::memory_order_acquire)) (void)hipFree(freed_);
      } else {
        if (peer_open_ && freed_) (void)hipIpcCloseMemHandle(freed_);
        sh_->receiver_detached.store(1, std::memory_order_release);
        const bool mapped = sh_->sender_ready.load(std::memory_order_acquire) &&
                            !sh_->sender_detached.load(std::memory_order_acquire);
        if (owns_ring_ && !mapped) {
          (void)hipFree(ring_);
          for (char* q : chunk_) (void)hipFree(q);
        }
        IPC_TRACE("  ring %s", mapped ? "left mapped by the peer (not freed)" : "freed");
      }
      if (events_)
        for (int64_t k = 0; k < sh_->nslots; ++k) (void)hipEventDestroy(events_[k]);
      if (copy_stream_) (void)hipStreamDestroy(copy_stream_);
    }
  } catch (...) {
  }
  delete[] events_;
  if (sh_) munmap(sh_, map_bytes_);
  if (fd_ >= 0) close(fd_);
  if (!sender_) shm_unlink(name_.c_str());  // idempotent: ENOENT after unlink() is fine
}

int64_t Link::nslots() const { return sh_->nslots; }
int64_t Link::slot_bytes() const { return sh_->slot_bytes; }

bool Link::drain(double timeout_s) const {
  if (host_mode()) return true;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  auto quiet = [&](auto query) {
    for (;;) {
      const hipError_t e = query();
      if (e != hipErrorNotReady) return true;  // done (or an error: nothing left to wait for)
      if (std::chrono::steady_clock::now() > deadline) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  };
  if (events_)
    for (int64_t k = 0; k < sh_->nslots; ++k)
      if (!quiet([&] { return hipEventQuery(events_[k]); })) return false;
  if (copy_stream_ && !quiet([&] { return hipStreamQuery(copy_stream_); })) return false;
  return true;
}

void Link::abort() {
  sh_->aborted.store(1, std::memory_order_release);
  if (host_mode() || aborted_local_) return;
  aborted_local_ = true;
  // Device mode: every wait on this side is a hipStreamWaitValue64 on a flag
  // this side OWNS (receiver: the full flags at the head of its ring; sender:
  // its freed flags).  Saturating them lets every pending and future wait
  // pass, so the streams drain instead of blocking forever on a dead peer
  // (the step is being torn down with an error anyway; the slots' contents
  // no longer matter).  Written from a stream of our own, never the
  // compute stream that may be the one stuck in the wait.
  char* flags = sender_ ? freed_ : ring_;
  if (flags == nullptr || (sender_ && !owns_freed_)) return;
  try {
    DeviceGuard g(device_);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
    for (int64_t k = 0; k < sh_->nslots; ++k)
      (void)hipStreamWriteValue64(s, flags + k * kFlagStride, ~0ull, 0);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(5);
    while (hipStreamQuery(s) == hipErrorNotReady && std::chrono::steady_clock::now() < deadline)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    IPC_TRACE("abort %s: %lld flags saturated", name_.c_str(), (long long)sh_->nslots);
    // the stream is leaked if its writes are still queued (destroying it would block)
    if (hipStreamQuery(s) != hipErrorNotReady) (void)hipStreamDestroy(s);
  } catch (...) {
  }
}

int64_t Link::message_bytes(uint64_t seq) const {
  // the sender records each message's byte count in the shared block when it
  // enqueues the send; -1 while message seq has not been enqueued yet (or the
  // slot already holds a later one)
  const int k = int(seq % uint64_t(sh_->nslots));
  const uint64_t sent = sh_->sent.load(std::memory_order_acquire);
  if (sent < seq + 1) return -1;
  if (sent > seq + uint64_t(sh_->nslots)) return -2;
  return (int64_t)sh_->slots[k].bytes;
}
void Link::unlink() { shm_unlink(name_.c_str()); }

char* Link::slot(uint64_t seq) const {
  const int k = int(seq % uint64_t(sh_->nslots));
  if (host_mode()) return ring_ + int64_t(k) * sh_->slot_bytes;
  const int64_t spc = sh_->slots_per_chunk;
  return chunk_[size_t(int64_t(k) / spc)] + (int64_t(k) % spc) * sh_->slot_bytes;
}

std::string Link::describe() const {
  std::ostringstream o;
  o << (sender_ ? "sender" : "receiver") << " of " << name_ << " (" << sh_->nslots << " slots x " << sh_->slot_bytes
    << " B, " << (host_mode() ? "host" : ("device " + std::to_string(device_) + ", stream-ordered flags"))
    << ", next seq " << next_seq_ << ", peer-visible sent " << sh_->sent.load() << " / released "
    << sh_->released.load() << ")";
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
  char* dst = slot(s);
  if (host_mode()) {
    if (s >= uint64_t(n)) wait_for("a free slot", s - uint64_t(n) + 1, k, false, timeout_s);
    std::memcpy(dst, src, bytes);
    c.bytes = bytes;
    c.full.store(s + 1, std::memory_order_release);
    sh_->sent.store(s + 1, std::memory_order_release);
    ++next_seq_;
    return s;
  }
  DeviceGuard g(device_);
  // inline engines (2, 3) run the whole send on the producer's stream: no
  // cross-stream hop at all, the copy ordered behind the producer's later work
  const bool in_line = engine_ >= 2;
  hipStream_t cs = in_line ? producer : copy_stream_;
  if (!in_line) rt::stream_wait(copy_stream_, producer, device_);
  if (s >= uint64_t(n))  // the slot's previous message released by the receiver's stream
    check(hipStreamWaitValue64(cs, freed_ + int64_t(k) * kFlagStride, s - uint64_t(n) + 1,
                               hipStreamWaitValueGte, ~0ull),
          "hipStreamWaitValue64(freed)");
  if (bytes) {
    // engines 0 / 3 ("sdma", "inline-sdma"): the copy engines only -- hipMemcpyDeviceToDevice may pick a blit
    // kernel (CUs taken from compute, profiles/cu_hold_r5.txt); NoCU never does (tools/micro/nocu_copy.hip)
    if (engine_ == 1 || engine_ == 2) rt::blit_copy(dst, src, bytes, cs);
    else check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, cs), "hipMemcpyAsync(send, NoCU)");
  }
  check(hipStreamWriteValue64(cs, ring_ + int64_t(k) * kFlagStride, s + 1, 0), "hipStreamWriteValue64(full)");
  check(hipEventRecord(events_[k], cs), "hipEventRecord(sent)");
  c.bytes = bytes;
  sh_->sent.store(s + 1, std::memory_order_release);
  ++next_seq_;
  return s;
}

uint64_t Link::post() {
  if (sender_) throw std::runtime_error("mipipe ipc: post on a sending link");
  return next_seq_++;
}

void Link::open_peer_flags() {
  if (peer_open_ || host_mode()) return;
  // the sender exports its freed flags when it attaches
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(300);
  while (!sh_->sender_ready.load(std::memory_order_acquire)) {
    if (sh_->aborted.load()) throw std::runtime_error("mipipe ipc: aborted before the sender attached");
    if (std::chrono::steady_clock::now() > deadline) throw std::runtime_error("mipipe ipc: the sender never attached");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  void* f = nullptr;
  IPC_TRACE("receiver %s: opening the sender's freed flags", name_.c_str());
  check(hipIpcOpenMemHandle(&f, sh_->freed, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle(freed flags)");
  IPC_TRACE("receiver %s: freed flags mapped", name_.c_str());
  freed_ = static_cast<char*>(f);
  peer_open_ = true;
}

void* Link::acquire(uint64_t seq, hipStream_t consumer) {
  if (sender_) throw std::runtime_error("mipipe ipc: acquire on a sending link");
  if (host_mode()) throw std::runtime_error("mipipe ipc: acquire needs a device link (host mode copies)");
  const int k = int(seq % uint64_t(sh_->nslots));
  DeviceGuard g(device_);
  check(hipStreamWaitValue64(consumer, ring_ + int64_t(k) * kFlagStride, seq + 1, hipStreamWaitValueGte, ~0ull),
        "hipStreamWaitValue64(full)");
  return slot(seq);
}

void Link::release(uint64_t seq, hipStream_t consumer) {
  if (sender_) throw std::runtime_error("mipipe ipc: release on a sending link");
  const int k = int(seq % uint64_t(sh_->nslots));
  if (host_mode()) {
    sh_->slots[k].freed.store(seq + 1, std::memory_order_release);
  } else {
    DeviceGuard g(device_);
    open_peer_flags();
    check(hipStreamWriteValue64(consumer, freed_ + int64_t(k) * kFlagStride, seq + 1, 0),
          "hipStreamWriteValue64(freed)");
    check(hipEventRecord(events_[k], consumer), "hipEventRecord(released)");
  }
  if (seq + 1 > last_done_seq_) last_done_seq_ = seq + 1;
  sh_->released.store(last_done_seq_, std::memory_order_release);
}

void Link::wait(uint64_t seq, void* dst, size_t bytes, hipStream_t consumer, double timeout_s) {
  if (sender_) throw std::runtime_error("mipipe ipc: wait on a sending link");
  const int64_t n = sh_->nslots;
  const int k = int(seq % uint64_t(n));
  if ((int64_t)bytes > sh_->slot_bytes) throw std::runtime_error("mipipe ipc: receive larger than a slot");
  if (host_mode()) {
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
    std::memcpy(dst, slot(seq), bytes);
    release(seq, nullptr);
    return;
  }
  const void* src = acquire(seq, consumer);
  DeviceGuard g(device_);
  if (bytes) check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, consumer), "hipMemcpyAsync(recv)");
  release(seq, consumer);
}

bool Link::done(uint64_t seq) const {
  const int k = int(seq % uint64_t(sh_->nslots));
  if (host_mode()) {
    const SlotCtl& c = sh_->slots[k];
    return (sender_ ? c.full : c.freed).load(std::memory_order_acquire) >= seq + 1;
  }
  // the slot's event was last recorded for message seq or a later one
  if (sender_ ? sh_->sent.load() < seq + 1 : last_done_seq_ < seq + 1) return false;
  return hipEventQuery(events_[k]) == hipSuccess;
}

}  // namespace ipc
}  // namespace mipipe
