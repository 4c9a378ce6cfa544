// Native pipeline runtime: streams, events, peer copies, roctx ranges
// (§5.1).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace mipipe {
namespace rt {

// Dedicated non-blocking stream on `device` (never recycled while the process
// lives).  `priority`: 0 = normal, -1 = high (hipDeviceGetStreamPriorityRange).
hipStream_t stream_acquire(int device, int priority);

// `waiting` will not run work enqueued after this call before everything
// enqueued on `waited` so far has finished.  Uses a pooled event.
void stream_wait(hipStream_t waiting, hipStream_t waited, int device);

// Copy engines for peer_copy.
enum CopyEngine : int {
  kCopySdma = 0,  // hipMemcpy(Peer)Async: the DMA engines, no CUs used
  kCopyBlit = 1,  // a 16-byte-vector copy kernel on src_stream (push into the peer's HBM)
};

// Async copy of `bytes` from src (on src_device) to dst (on dst_device); the
// devices may be equal (a stage boundary between two partitions of one GPU).
// Ordering: dst_stream's prior work -> copy on src_stream -> dst_stream.
void peer_copy(void* dst, int dst_device, const void* src, int src_device, size_t bytes, hipStream_t src_stream,
               hipStream_t dst_stream, int engine = kCopySdma);

// The blit kernel alone, on `stream` of the current device (falls back to
// hipMemcpyAsync for pointers or sizes that are not 16-byte multiples).
void blit_copy(void* dst, const void* src, size_t bytes, hipStream_t stream);

// One hipMemcpyDeviceToDeviceNoCU copy on `stream` (the DMA engines only): "" if
// the runtime accepted it, else its error (diagnostics: which runtime refuses it).
std::string copy_nocu(void* dst, const void* src, size_t bytes, hipStream_t stream);

// Enables peer access between every ordered pair of `devices` (idempotent).
void enable_peer_access(const std::vector<int>& devices);
bool can_access_peer(int device, int peer);

void range_push(const std::string& label);
void range_pop();
void mark(const std::string& label);

}  // namespace rt
}  // namespace mipipe
