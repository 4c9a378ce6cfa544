// Device-memory point-to-point transport between PROCESSES (SURVEY §5.8 (a),
// multi-process form): pipeline ranks that share a GPU -- or sit on different
// GPUs of a node -- move activations and gradients without RCCL and without
// host staging.
//
// One Link per directed rank pair.  The RECEIVER owns a ring of `nslots`
// device buffers (`slot_bytes` each) and exports them once (hipIpcGetMemHandle);
// the SENDER maps them (hipIpcOpenMemHandle) and copies each message into the
// next slot on a dedicated copy stream -- the DMA engines (hipMemcpyAsync) or a
// blit kernel -- so a transfer takes no CUs from the compute stream.  A shared
// control block (POSIX shm) carries per-slot sequence numbers:
//
//   full[k]  = 1 + sequence number of the last message written into slot k
//   freed[k] = 1 + sequence number of the last message the receiver released
//
// Completion crosses the process boundary either through interprocess events
// (the receiver's stream waits on the event the sender recorded after its
// copy: no host blocking on either side) or, where interprocess events are
// unavailable, through a proxy thread that publishes `full`/`freed` once the
// local copy event has completed.  Messages on a link are matched in order:
// the receiver posts receives in the order the sender sends (the engine's rule
// for every transport).
//
// Host mode (no GPU): the slots live in the shm segment and copies are
// memcpy -- the same protocol, exercised by the CPU tests.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>

namespace mipipe {
namespace ipc {

struct Shared;  // the shm layout (ipc.cpp)

class Link {
 public:
  // Receiver side: creates the shm control block `name` and the slot ring.
  // device < 0: host mode (slots in shared memory).
  static std::unique_ptr<Link> create(const std::string& name, int device, int64_t nslots, int64_t slot_bytes,
                                      bool use_ipc_events);
  // Sender side: attaches to the receiver's block (waits up to `timeout_s`
  // for it to appear).  engine: 0 = hipMemcpyAsync, 1 = blit kernel.
  static std::unique_ptr<Link> attach(const std::string& name, int device, int engine, double timeout_s);
  ~Link();

  bool is_sender() const { return sender_; }
  bool host_mode() const { return device_ < 0; }
  int64_t nslots() const;
  int64_t slot_bytes() const;
  bool ipc_events() const;
  // Copy stream of a sender (0 in host mode / on the receiver).
  hipStream_t copy_stream() const { return copy_stream_; }

  // Sender: enqueue message `bytes` from `src` after the work queued on
  // `producer` so far.  Returns the message's sequence number.
  uint64_t send(const void* src, size_t bytes, hipStream_t producer, double timeout_s);
  // Receiver: reserve the next sequence number (posting order = send order).
  uint64_t post();
  // Receiver: copy message `seq` into `dst` on `consumer` once it has arrived
  // (host-blocks until the sender has issued it).
  void wait(uint64_t seq, void* dst, size_t bytes, hipStream_t consumer, double timeout_s);
  // Sender / receiver: true once message `seq` is published (sender: copy
  // issued and, without ipc events, completed; receiver: slot released).
  bool done(uint64_t seq) const;

  // Unblocks both sides with an error (a failed peer, a watchdog).
  void abort();
  // Removes the shm name (after both sides are attached; the mapping stays).
  void unlink();
  std::string describe() const;

 private:
  Link() = default;
  void wait_for(const char* what, uint64_t seq, int slot, bool full, double timeout_s) const;
  void open_remote_events();

  std::string name_;
  bool sender_ = false;
  int device_ = -1;
  int engine_ = 0;
  Shared* sh_ = nullptr;
  size_t map_bytes_ = 0;
  int fd_ = -1;
  char* data_ = nullptr;          // slot ring (device pointer, or inside the shm map)
  bool owns_data_ = false;
  hipStream_t copy_stream_ = nullptr;
  hipEvent_t* local_events_ = nullptr;   // sender: full[k]; receiver: freed[k]
  hipEvent_t* remote_events_ = nullptr;  // sender: freed[k]; receiver: full[k] (opened lazily)
  bool remote_open_ = false;
  uint64_t next_seq_ = 0;
};

// Completed-copy publisher for links without interprocess events.
void proxy_shutdown();

}  // namespace ipc
}  // namespace mipipe
