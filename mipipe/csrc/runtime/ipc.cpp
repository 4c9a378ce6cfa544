// Device-memory P2P transport between processes: see ipc.h.
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

constexpr uint64_t kMagic = 0x6d69706970654c33ull;  // "mipipeL3"
constexpr int kMaxSlots = 1024;
// Device mode: the slots live in allocations of at most 1 GiB each (one IPC handle per chunk).  Importing a single
// 3 GiB allocation from another process stalled inside hipIpcOpenMemHandle (profiles/ipc_import_stall_r5.txt), so
// no allocation may exceed kChunkBytes: a slot larger than that is refused, and there is a chunk handle per slot
// at most (kMaxChunks == kMaxSlots), so slots per chunk never has to grow past what fits.
constexpr int64_t kChunkBytes = int64_t(1) << 30;
constexpr int kMaxChunks = kMaxSlots;
// One flag per slot, at the start of a 64 KiB line that the sender's flag copy rewrites whole: torch's HIP runtime
// (7.0) runs a hipMemcpyDeviceToDeviceNoCU copy below 64 KiB as a __amd_rocclr_copyBuffer KERNEL, from 64 KiB on
// on the DMA engines (tools/nocu_torch_probe.py, profiles/ipc_cu_free_r6.txt).  64 KiB x 1024 slots = 64 MiB at
// most per link.
constexpr int64_t kFlagStride = int64_t(64) << 10;

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

int64_t flag_bytes(int64_t nslots) { return nslots * kFlagStride; }

// The full flag of a slot carries the LAP of the message in it (message s is lap s / nslots of slot s % nslots) as
// one bit per lap parity; the consumer waits for its lap's bit (hipStreamWaitValueAnd).  The previous lap's value
// has the other bit, the initial 0 neither, and abort()'s all-ones both -- so the flag never needs a monotonic
// value, and the sender writes it by copying one of two constant words.
uint64_t lap_tag(uint64_t lap) { return uint64_t(1) << (lap & 1); }

}  // namespace

struct alignas(64) SlotCtl {
  std::atomic<uint64_t> full;       // host mode: 1 + the message in the slot
  std::atomic<uint64_t> bytes_seq;  // 1 + the message `bytes` belongs to (published after bytes)
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
  std::atomic<uint32_t> sender_ready;        // the sender has mapped the ring
  std::atomic<uint32_t> sender_detached;     // the sender has unmapped the ring
  std::atomic<uint32_t> pad1;
  std::atomic<uint64_t> sent;                // messages the sender has enqueued
  std::atomic<uint64_t> released;            // messages the receiver has released (enqueued)
  // messages [0, freed) released and their releases EXECUTED: in device mode
  // written by the receiver's GPU (hipStreamWriteValue64 through the
  // registered mapping of this block), polled by the sender's host
  alignas(64) std::atomic<uint64_t> freed;
  uint8_t pad2[56];
  hipIpcMemHandle_t ring;                    // receiver's full flags (device mode)
  int32_t nchunks;                           // device mode: the slot allocations
  int32_t slots_per_chunk;
  hipIpcMemHandle_t chunk[kMaxChunks];
  SlotCtl slots[kMaxSlots];
};

static_assert(std::atomic<uint64_t>::is_always_lock_free, "cross-process atomics need lock-free 64-bit");

static size_t header_size() { return (sizeof(Shared) + 4095) & ~size_t(4095); }

static size_t map_size(int64_t nslots, int64_t slot_bytes, bool host) {
  size_t n = header_size();
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
  const bool host = device < 0;
  if (!host && slot_bytes > kChunkBytes) {
    std::ostringstream o;
    o << "mipipe ipc: a slot of " << slot_bytes << " B exceeds the 1 GiB IPC allocation limit (larger imports can "
      << "stall hipIpcOpenMemHandle, profiles/ipc_import_stall_r5.txt): use smaller micro-batches";
    throw std::runtime_error(o.str());
  }
  std::unique_ptr<Link> L(new Link());
  L->name_ = name;
  L->sender_ = false;
  L->device_ = device;
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
  sh->sent.store(0);
  sh->released.store(0);
  sh->freed.store(0);
  for (int k = 0; k < nslots; ++k) {
    sh->slots[k].full.store(0);
    sh->slots[k].bytes_seq.store(0);
    sh->slots[k].bytes = 0;
  }
  if (host) {
    L->ring_ = reinterpret_cast<char*>(p) + header_size();
  } else {
    DeviceGuard g(device);
    // the release counter lives in this (host) block: the receiver's GPU writes it, the sender's host reads it
    check(hipHostRegister(p, header_size(), hipHostRegisterMapped), "hipHostRegister(shared block)");
    L->registered_ = true;
    void* dp = nullptr;
    check(hipHostGetDevicePointer(&dp, p, 0), "hipHostGetDevicePointer(shared block)");
    L->freed_dev_ = reinterpret_cast<uint64_t*>(static_cast<char*>(dp) + offsetof(Shared, freed));
    void* d = nullptr;
    check(hipMalloc(&d, size_t(flag_bytes(nslots))), "hipMalloc(full flags)");
    check(hipMemset(d, 0, size_t(flag_bytes(nslots))), "hipMemset(full flags)");
    check(hipDeviceSynchronize(), "hipDeviceSynchronize(ring)");
    L->ring_ = static_cast<char*>(d);
    L->owns_ring_ = true;
    check(hipIpcGetMemHandle(&sh->ring, d), "hipIpcGetMemHandle(full flags)");
    const int64_t spc = std::max<int64_t>(1, std::min<int64_t>(nslots, kChunkBytes / slot_bytes));
    const int64_t nch = (nslots + spc - 1) / spc;  // <= nslots <= kMaxChunks
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
  if (engine < 0 || engine > 3) throw std::runtime_error("mipipe ipc: engine must be 0..3");
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
    L->ring_ = reinterpret_cast<char*>(p) + header_size();
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
    // the two lap tags a flag copy writes, one flag line each (device memory: a device-to-device copy)
    void* w = nullptr;
    check(hipMalloc(&w, size_t(2 * kFlagStride)), "hipMalloc(lap tags)");
    std::vector<uint64_t> tags(size_t(2 * kFlagStride) / sizeof(uint64_t));
    for (size_t i = 0; i < tags.size(); ++i) tags[i] = lap_tag(i < tags.size() / 2 ? 0 : 1);
    check(hipMemcpy(w, tags.data(), size_t(2 * kFlagStride), hipMemcpyHostToDevice), "hipMemcpy(lap tags)");
    L->tags_ = static_cast<char*>(w);
    // from the runtime's process-lifetime pool, never destroyed: torch's caching allocator records events on it
    // for every send source (record_stream) and may do so after the link is gone, when such a tensor is freed
    L->copy_stream_ = rt::stream_acquire(device, 0);
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
      // Each slot's event is recorded right after the flag copy of the last
      // send (on the stream the copy used) or the last release (the consumer's
      // stream), so those events cover every write into the peer's memory.  Bounded: after a peer failure
      // a consumer may wait forever for a message that never comes -- then the
      // mappings are left to process teardown instead of hanging here (abort()
      // releases this side's own waits).
      if (!drain(30.0)) {
        IPC_TRACE("  %s: queued work did not drain in 30 s; mappings left to teardown", name_.c_str());
        throw std::runtime_error("undrained");
      }
      if (sender_) {
        if (ring_) (void)hipIpcCloseMemHandle(ring_);
        for (char* q : chunk_) (void)hipIpcCloseMemHandle(q);
        sh_->sender_detached.store(1, std::memory_order_release);
        if (tags_) (void)hipFree(tags_);
      } else {
        const bool mapped = sh_->sender_ready.load(std::memory_order_acquire) &&
                            !sh_->sender_detached.load(std::memory_order_acquire);
        // freeing memory a peer still maps can block until it lets go (two ranks
        // tearing down in opposite orders would wait on each other): a still-mapped
        // ring is left to the process teardown
        if (owns_ring_ && !mapped) {
          (void)hipFree(ring_);
          for (char* q : chunk_) (void)hipFree(q);
        }
        if (registered_) (void)hipHostUnregister(sh_);
        IPC_TRACE("  ring %s", mapped ? "left mapped by the peer (not freed)" : "freed");
      }
      if (events_)
        for (int64_t k = 0; k < sh_->nslots; ++k) (void)hipEventDestroy(events_[k]);
      // copy_stream_ belongs to the runtime's stream pool (see attach)
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
  // Device mode: the only GPU-side waits are the receiver's
  // hipStreamWaitValue64s on the full flags it OWNS (a sender's waits are host
  // polls, which the aborted word ends).  Saturating the flags lets every
  // pending and future wait pass, so the streams drain instead of blocking
  // forever on a dead peer (the step is being torn down with an error anyway;
  // the slots' contents no longer matter).  Written from a stream of our own,
  // never the compute stream that may be the one stuck in the wait.
  if (sender_ || ring_ == nullptr) return;
  try {
    DeviceGuard g(device_);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
    for (int64_t k = 0; k < sh_->nslots; ++k)
      (void)hipStreamWriteValue64(s, ring_ + k * kFlagStride, ~0ull, 0);
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
  // enqueues the send, tagged with the message it belongs to (a sender running
  // a ring ahead may be rewriting the slot's count for a later message)
  const int k = int(seq % uint64_t(sh_->nslots));
  const SlotCtl& c = sh_->slots[k];
  const uint64_t tag = c.bytes_seq.load(std::memory_order_acquire);
  if (tag < seq + 1) return -1;
  if (tag > seq + 1) return -2;
  const uint64_t b = c.bytes;
  std::atomic_thread_fence(std::memory_order_acquire);
  if (c.bytes_seq.load(std::memory_order_relaxed) != seq + 1) return -2;
  return (int64_t)b;
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
    << " B, "
    << (host_mode() ? std::string("host")
                    : ("device " + std::to_string(device_) + ", " +
                       (sender_ ? (dma_engine() ? (nocu_refused_ ? "DMA copies refused by the runtime: default "
                                                                   "copy kind" : "DMA copies")
                                                : "blit copies")
                                : "stream-waited flags")))
    << ", next seq " << next_seq_ << ", peer-visible sent " << sh_->sent.load() << " / released "
    << sh_->released.load() << " / freed " << sh_->freed.load() << ")";
  return o.str();
}

void Link::wait_counter(const char* what, const void* counter, uint64_t need, double timeout_s) const {
  const auto& ctr = *static_cast<const std::atomic<uint64_t>*>(counter);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  for (int spin = 0;; ++spin) {
    if (ctr.load(std::memory_order_acquire) >= need) return;
    if (sh_->aborted.load(std::memory_order_acquire))
      throw std::runtime_error("mipipe ipc: " + describe() + ": the link was aborted while waiting for " + what);
    if (spin > 2000) {
      if (std::chrono::steady_clock::now() > deadline) {
        std::ostringstream o;
        o << "mipipe ipc: " << describe() << ": timed out after " << timeout_s << " s waiting for " << what
          << " (need " << need << ", have " << ctr.load() << ")";
        throw std::runtime_error(o.str());
      }
      std::this_thread::sleep_for(std::chrono::microseconds(spin > 20000 ? 200 : 5));
    }
  }
}

void Link::dma(void* dst, const void* src, size_t bytes, hipStream_t s, const char* what) {
  // the copy engines only: hipMemcpyDeviceToDevice may pick a blit kernel (CUs
  // taken from compute, profiles/cu_hold_r5.txt); NoCU never does
  // (tools/micro/nocu_copy.hip).  A runtime that refuses the kind gets the
  // default one from then on (as rt::peer_copy does).
  if (!nocu_refused_) {
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDeviceNoCU, s) == hipSuccess) return;
    (void)hipGetLastError();
    nocu_refused_ = true;
    IPC_TRACE("%s: hipMemcpyDeviceToDeviceNoCU refused; default copy kind from now on", name_.c_str());
  }
  check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s), what);
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
  // the slot's previous message (s - n) released, and that release executed: a
  // host poll of the shared counter, never a wait dispatched on the GPU
  if (s >= uint64_t(n)) wait_counter("a free slot", &sh_->freed, s - uint64_t(n) + 1, timeout_s);
  c.bytes = bytes;
  c.bytes_seq.store(s + 1, std::memory_order_release);
  if (host_mode()) {
    std::memcpy(dst, src, bytes);
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
  if (!in_line) rt::stream_wait(copy_stream_, producer, device_);  // an event wait: a barrier packet, no kernel
  char* flag = ring_ + int64_t(k) * kFlagStride;
  const uint64_t lap = s / uint64_t(n);
  if (dma_engine()) {
    // payload, then the lap tag into the receiver's flag: two device-to-device
    // DMA copies in stream order, no kernel on the stream
    if (bytes) dma(dst, src, bytes, cs, "hipMemcpyAsync(send)");
    dma(flag, tags_ + (lap & 1) * kFlagStride, size_t(kFlagStride), cs, "hipMemcpyAsync(flag)");
  } else {
    if (bytes) rt::blit_copy(dst, src, bytes, cs);
    check(hipStreamWriteValue64(cs, flag, lap_tag(lap), 0), "hipStreamWriteValue64(full)");
  }
  check(hipEventRecord(events_[k], cs), "hipEventRecord(sent)");
  sh_->sent.store(s + 1, std::memory_order_release);
  ++next_seq_;
  return s;
}

uint64_t Link::post() {
  if (sender_) throw std::runtime_error("mipipe ipc: post on a sending link");
  return next_seq_++;
}

void* Link::acquire(uint64_t seq, hipStream_t consumer) {
  if (sender_) throw std::runtime_error("mipipe ipc: acquire on a sending link");
  if (host_mode()) throw std::runtime_error("mipipe ipc: acquire needs a device link (host mode copies)");
  const int k = int(seq % uint64_t(sh_->nslots));
  DeviceGuard g(device_);
  check(hipStreamWaitValue64(consumer, ring_ + int64_t(k) * kFlagStride, lap_tag(seq / uint64_t(sh_->nslots)),
                             hipStreamWaitValueAnd, ~0ull),
        "hipStreamWaitValue64(full)");
  return slot(seq);
}

void Link::release(const std::vector<uint64_t>& seqs, hipStream_t consumer) {
  if (sender_) throw std::runtime_error("mipipe ipc: release on a sending link");
  if (seqs.empty()) return;
  const uint64_t before = last_done_seq_;
  for (uint64_t seq : seqs) {
    if (seq >= next_seq_) throw std::runtime_error("mipipe ipc: release of a message never posted");
    if (seq >= last_done_seq_) early_.insert(seq);
  }
  while (!early_.empty() && *early_.begin() == last_done_seq_) {
    early_.erase(early_.begin());
    ++last_done_seq_;
  }
  if (host_mode()) {
    if (last_done_seq_ > before) sh_->freed.store(last_done_seq_, std::memory_order_release);
  } else {
    DeviceGuard g(device_);
    // one write per call for the in-order prefix; releases above a gap wait for
    // the call that fills it (the engine releases in posting order)
    if (last_done_seq_ > before)
      check(hipStreamWriteValue64(consumer, freed_dev_, last_done_seq_, 0), "hipStreamWriteValue64(freed)");
    for (uint64_t seq : seqs)
      check(hipEventRecord(events_[int(seq % uint64_t(sh_->nslots))], consumer), "hipEventRecord(released)");
  }
  sh_->released.store(last_done_seq_, std::memory_order_release);
}

void Link::wait(uint64_t seq, void* dst, size_t bytes, hipStream_t consumer, double timeout_s) {
  if (sender_) throw std::runtime_error("mipipe ipc: wait on a sending link");
  const int64_t n = sh_->nslots;
  const int k = int(seq % uint64_t(n));
  if ((int64_t)bytes > sh_->slot_bytes) throw std::runtime_error("mipipe ipc: receive larger than a slot");
  if (host_mode()) {
    SlotCtl& c = sh_->slots[k];
    wait_counter("the message", &c.full, seq + 1, timeout_s);
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
    if (sender_) return sh_->slots[k].full.load(std::memory_order_acquire) >= seq + 1;
    return sh_->freed.load(std::memory_order_acquire) >= seq + 1;
  }
  // the slot's event was last recorded for message seq or a later one
  if (sender_ ? sh_->sent.load() < seq + 1 : last_done_seq_ < seq + 1) return false;
  return hipEventQuery(events_[k]) == hipSuccess;
}

}  // namespace ipc
}  // namespace mipipe
