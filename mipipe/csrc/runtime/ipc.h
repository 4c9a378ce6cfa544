// Device-memory point-to-point transport between PROCESSES (SURVEY §5.8 (a),
// multi-process form): pipeline ranks that share a GPU -- or sit on different
// GPUs of a node -- move activations and gradients without RCCL and without
// host staging, and without a host in the completion path.
//
// One Link per directed rank pair.  The RECEIVER owns a ring of `nslots`
// device buffers (`slot_bytes` each) behind an array of 64-byte "full" flag
// words, one device allocation exported once (hipIpcGetMemHandle); the SENDER
// owns an array of "freed" flag words, exported the same way.  Each side maps
// the other's allocation once (hipIpcOpenMemHandle).  Message s lands in slot
// k = s mod nslots:
//
//   sender,   on its copy stream:  wait producer; hipStreamWaitValue64(freed[k]
//             >= s - nslots + 1) (the slot's previous message released);
//             copy src -> slot k (DMA engines or a blit kernel);
//             hipStreamWriteValue64(full[k] = s + 1)   -- into the receiver's memory
//   receiver, on its compute stream: hipStreamWaitValue64(full[k] >= s + 1);
//             use slot k in place (zero copy) or copy it out; then
//             hipStreamWriteValue64(freed[k] = s + 1)  -- into the sender's memory
//
// Every wait is a stream-ordered command-processor wait: neither host blocks,
// a transfer overlaps whatever compute precedes the consumer's wait, and the
// message moves once (sender -> the receiver's slot; the slot is the receive
// buffer).  tools/micro/ipc_signal_probe.hip checks the primitive across two
// processes on one MI355X (profiles/ipc_stream_ordered.txt).  Pooled local
// events (one per slot, re-recorded) give the watchdog a non-blocking
// completion query.  Messages on a link are matched in order: the receiver
// posts receives in the order the sender sends (the engine's rule for every
// transport).
//
// Host mode (no GPU): the slots live in the shm segment, copies are memcpy
// and the flags are host atomics -- the same protocol, for the CPU tests.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace mipipe {
namespace ipc {

struct Shared;  // the shm layout (ipc.cpp)

class Link {
 public:
  // Receiver side: creates the shm control block `name` and the slot ring.
  // device < 0: host mode (slots in shared memory).
  static std::unique_ptr<Link> create(const std::string& name, int device, int64_t nslots, int64_t slot_bytes);
  // Sender side: attaches to the receiver's block (waits up to `timeout_s`
  // for it to appear).  engine: 0 = hipMemcpyAsync, 1 = blit kernel, on the
  // link's copy stream; 2 = blit kernel, 3 = hipMemcpyAsync, on the producer's
  // stream itself (inline: no cross-stream dependency per message).
  static std::unique_ptr<Link> attach(const std::string& name, int device, int engine, double timeout_s);
  ~Link();

  bool is_sender() const { return sender_; }
  bool host_mode() const { return device_ < 0; }
  int64_t nslots() const;
  int64_t slot_bytes() const;
  // Copy stream of a sender (0 in host mode / on the receiver).
  hipStream_t copy_stream() const { return copy_stream_; }
  // The sender copies on the producer's stream (engines 2, 3).
  bool inline_copy() const { return sender_ && engine_ >= 2; }

  // Sender: enqueue message `bytes` from `src` after the work queued on
  // `producer` so far.  Never blocks the host in device mode (host mode:
  // blocks while the slot is unreleased).  Returns the sequence number.
  uint64_t send(const void* src, size_t bytes, hipStream_t producer, double timeout_s);
  // Receiver: reserve the next sequence number (posting order = send order).
  uint64_t post();
  // Receiver, device mode: make `consumer` wait for message `seq` (no host
  // block); returns the slot holding it, valid until release(seq).
  void* acquire(uint64_t seq, hipStream_t consumer);
  // The slot message `seq` lands in (no wait: pair with acquire()).
  void* slot_ptr(uint64_t seq) const { return slot(seq); }
  // Receiver: mark message `seq`'s slot free for the sender, after the work
  // queued on `consumer` (device) / now (host).
  void release(uint64_t seq, hipStream_t consumer);
  // Receiver: acquire + copy into `dst` + release, on `consumer` (host mode:
  // blocks until the message is there, then memcpy).
  void wait(uint64_t seq, void* dst, size_t bytes, hipStream_t consumer, double timeout_s);
  // Sender: message `seq`'s copy has completed; receiver: its slot has been
  // released (device mode: an event query, never blocks).
  bool done(uint64_t seq) const;

  // A failed peer, a watchdog: unblocks host-mode waits with an error, and
  // (device mode) saturates the flags this side owns so its pending
  // hipStreamWaitValue64s pass instead of blocking the streams forever.
  void abort();
  // Waits (bounded) until everything this side queued on the link has run:
  // every slot's last send / release event and the copy stream.  False on
  // timeout.
  bool drain(double timeout_s) const;
  // Byte count of message seq as the sender enqueued it; -1 while the sender
  // has not enqueued it yet, -2 once its slot holds a later message.
  int64_t message_bytes(uint64_t seq) const;
  // Removes the shm name (after both sides are attached; the mapping stays).
  void unlink();
  // Receiver: maps the sender's freed flags (exported when it attached).  Done at
  // construction, one process at a time (mipipe/parallel/ipc.py): importing IPC
  // handles concurrently in a ring of processes can deadlock in the runtime.
  void open_peer_flags();
  std::string describe() const;

 private:
  Link() = default;
  void wait_for(const char* what, uint64_t seq, int slot, bool full, double timeout_s) const;
  char* slot(uint64_t seq) const;

  std::string name_;
  bool sender_ = false;
  int device_ = -1;
  int engine_ = 0;
  Shared* sh_ = nullptr;
  size_t map_bytes_ = 0;
  int fd_ = -1;
  char* ring_ = nullptr;          // device: the receiver's full flags; host: the slots in the shm map
  std::vector<char*> chunk_;      // device: the receiver's slot allocations (each <= ~1 GiB)
  bool owns_ring_ = false;
  char* freed_ = nullptr;         // sender's allocation: freed flags (device mode)
  bool owns_freed_ = false;
  bool peer_open_ = false;        // receiver: the sender's freed flags are mapped
  hipStream_t copy_stream_ = nullptr;
  hipEvent_t* events_ = nullptr;  // one per slot: sender after the copy, receiver after the release
  uint64_t next_seq_ = 0;
  bool aborted_local_ = false;     // abort() already saturated this side's flags
  uint64_t last_done_seq_ = 0;    // receiver: 1 + last released sequence (host bookkeeping)
};

}  // namespace ipc
}  // namespace mipipe
