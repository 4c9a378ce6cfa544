// Device-memory point-to-point transport between PROCESSES (SURVEY §5.8 (a),
// multi-process form): pipeline ranks that share a GPU -- or sit on different
// GPUs of a node -- move activations and gradients without RCCL and without
// host staging of the payload.
//
// One Link per directed rank pair.  The RECEIVER owns a ring of `nslots`
// device buffers (`slot_bytes` each, in allocations of <= 1 GiB) behind an
// array of "full" flag words (one per 64 KiB line) in its device memory, exported once
// (hipIpcGetMemHandle) and mapped once by the sender (hipIpcOpenMemHandle).
// Message s lands in slot k = s mod nslots:
//
//   sender host:   waits (host poll, never a GPU wait) until the receiver has
//                  released message s - nslots: the shared block's `freed`
//                  counter >= s - nslots + 1;
//   sender stream: event-wait for the producer (a barrier packet); copy
//                  src -> slot k; copy the lap tag of message s (lap
//                  s / nslots; one of two constant 64 KiB lines in the
//                  sender's device memory -- smaller NoCU copies run as a
//                  kernel) over full[k]'s line.  Engines 0 / 3 issue both
//                  copies with hipMemcpyDeviceToDeviceNoCU: the DMA engines
//                  only, so the link's copy stream dispatches NO kernel (no CU
//                  is ever taken from the GEMMs next to it); engines 1 / 2 are
//                  the kernel variants (blit copy + hipStreamWriteValue64);
//   receiver, on its compute stream: hipStreamWaitValue64(full[k] has the
//                  lap's bit) (in order with its own work: it only spins while
//                  that stream has nothing else to run), read slot k in place
//                  or copy it out, then hipStreamWriteValue64(freed = s + 1)
//                  into the shared block -- host memory registered with the
//                  receiver's GPU -- which the sender's host polls.
//
// The lap tag alternates between two bits (lap parity): the flag of slot k
// holds lap q - 1's bit until lap q's copy lands, and lap q + 1 cannot be
// sent before lap q was released -- so a bit test is exact without a
// monotonic value, and abort() can pass every pending wait by writing all
// ones.  Releases publish the in-order prefix: `freed` is the count of
// messages [0, freed) released.
//
// Pooled local events (one per slot, re-recorded) give the watchdog a
// non-blocking completion query.  Messages on a link are matched in order:
// the receiver posts receives in the order the sender sends (the engine's
// rule for every transport).
//
// Host mode (no GPU): the slots live in the shm segment, copies are memcpy
// and the flags are host atomics -- the same protocol, for the CPU tests.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <set>
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
  // for it to appear).  engine: 0 = DMA copies (NoCU), 1 = blit kernel, on the
  // link's copy stream; 2 = blit kernel, 3 = DMA copies, on the producer's
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
  // The sender's copies and flag writes run on the DMA engines (engines 0, 3).
  bool dma_engine() const { return sender_ && (engine_ == 0 || engine_ == 3); }

  // Sender: enqueue message `bytes` from `src` after the work queued on
  // `producer` so far.  Blocks the host only while the target slot still
  // holds an unreleased message (never with a slot per message of a step).
  // Returns the sequence number.
  uint64_t send(const void* src, size_t bytes, hipStream_t producer, double timeout_s);
  // Receiver: reserve the next sequence number (posting order = send order).
  uint64_t post();
  // Receiver, device mode: make `consumer` wait for message `seq` (no host
  // block); returns the slot holding it, valid until release(seq).
  void* acquire(uint64_t seq, hipStream_t consumer);
  // The slot message `seq` lands in (no wait: pair with acquire()).
  void* slot_ptr(uint64_t seq) const { return slot(seq); }
  // Receiver: mark messages `seqs` free for the sender, after the work queued
  // on `consumer` (device) / now (host).  One counter write per call, for the
  // in-order prefix released so far.
  void release(const std::vector<uint64_t>& seqs, hipStream_t consumer);
  void release(uint64_t seq, hipStream_t consumer) { release(std::vector<uint64_t>{seq}, consumer); }
  // Receiver: acquire + copy into `dst` + release, on `consumer` (host mode:
  // blocks until the message is there, then memcpy).
  void wait(uint64_t seq, void* dst, size_t bytes, hipStream_t consumer, double timeout_s);
  // Sender: message `seq`'s copy has completed; receiver: its slot has been
  // released (device mode: an event query, never blocks).
  bool done(uint64_t seq) const;

  // A failed peer, a watchdog: unblocks host waits with an error, and (device
  // mode, receiver) saturates the full flags this side owns so its pending
  // hipStreamWaitValue64s pass instead of blocking the stream forever.
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
  std::string describe() const;

 private:
  Link() = default;
  void wait_counter(const char* what, const void* counter, uint64_t need, double timeout_s) const;
  char* slot(uint64_t seq) const;
  void dma(void* dst, const void* src, size_t bytes, hipStream_t s, const char* what);

  std::string name_;
  bool sender_ = false;
  int device_ = -1;
  int engine_ = 0;
  Shared* sh_ = nullptr;
  size_t map_bytes_ = 0;
  int fd_ = -1;
  char* ring_ = nullptr;          // device: the receiver's full flags; host: the slots in the shm map
  std::vector<char*> chunk_;      // device: the receiver's slot allocations (each <= 1 GiB)
  bool owns_ring_ = false;
  char* tags_ = nullptr;          // sender: the two lap tags (device memory) the flag copies read
  bool registered_ = false;       // receiver: the shm header is registered with its GPU
  uint64_t* freed_dev_ = nullptr; // receiver: device address of the shared `freed` counter
  bool nocu_refused_ = false;     // the runtime refused hipMemcpyDeviceToDeviceNoCU: plain kinds instead
  hipStream_t copy_stream_ = nullptr;
  hipEvent_t* events_ = nullptr;  // one per slot: sender after the flag copy, receiver after the release
  uint64_t next_seq_ = 0;
  bool aborted_local_ = false;    // abort() already saturated this side's flags
  uint64_t last_done_seq_ = 0;    // receiver: the released in-order prefix [0, last_done_seq_)
  std::set<uint64_t> early_;      // receiver: released out of order, above the prefix
};

}  // namespace ipc
}  // namespace mipipe
