// scratch.hpp — temporary device buffers of the batched entry points (the Solinas PBS's switched mask, the PRE_SWITCHED
// lift, the external product's W1'-ordered GGSW, the generic f64 engine's digit spectra, pbs_large's accumulators, the
// keyswitch digits, the multi-GPU shard staging).
//
// A per-device pool of plain hipMalloc blocks, kept for reuse and grown on demand (scratch.cpp).  Ordering is by event,
// not by host synchronisation: each block carries the event recorded on the stream of its last user, and the next
// user's stream waits on it (hipStreamWaitEvent) before its first launch.  So a block is never reissued before the
// last kernel that read it retired, on any stream, and reusing a pooled block never blocks the host — on the legacy null
// stream or on a caller's stream alike.  Growing the pool does: a request no idle block fits (an idle block serves a
// request only if it is at most 4x or 64 MiB above it) hipMallocs a new block and first frees the idle blocks of that
// device too small for it, each after hipEventSynchronize on its last use.  The high-water mark is the largest set of
// blocks in use at once plus the idle ones kept (up to the 4 GiB chunks of a large-N blind rotation) until
// mi_scratch_trim.  The stream-ordered allocator (hipMallocAsync) is not used: DESIGN.md §5 records why.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace mi {

// a block of >= bytes on the current device, ordered after the block's previous user; *p = nullptr on failure
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s);
// returns the block to the pool once the work already queued on `s` has been enqueued (event recorded on `s`)
hipError_t scratch_free(void* p, hipStream_t s);
// frees every idle block of `device` (-1: all devices) after its last user retired; returns the bytes released
size_t scratch_trim(int device);
// the caller has synchronized `s` and is about to destroy it: blocks whose last user ran on `s` need no wait on the
// event recorded there (an event whose stream is gone cannot be waited on reliably; see scratch.cpp wait_last_use)
void scratch_stream_retired(hipStream_t s);
// bytes held by the pool on `device` (idle + in use)
size_t scratch_bytes(int device);

// Pooled non-blocking side streams of the current device, for an entry point that splits its batch over the caller's
// stream and up to MAX_SIDE more (pbs_large.hip, fft64_generic.hip): fork() orders each side stream after the work
// already queued on the caller's stream, join() orders the caller's stream after everything queued on the side
// streams and returns them to the pool.  No host synchronisation either way (events only).
class StreamFork {
 public:
  static constexpr int MAX_SIDE = 3;
  StreamFork() = default;
  StreamFork(const StreamFork&) = delete;
  StreamFork& operator=(const StreamFork&) = delete;
  ~StreamFork() { (void)join(); }
  // acquires up to n side streams (fewer on failure: sides() tells how many)
  hipError_t fork(hipStream_t s, int n = 1);
  hipError_t join();
  int sides() const { return n_; }
  hipStream_t side(int i = 0) const { return side_[i]; }

 private:
  hipStream_t caller_ = nullptr, side_[MAX_SIDE] = {};
  int device_ = 0, n_ = 0;
};

// lanes a batched blind rotation splits a chunk into: the caller's measured default for its shape, clamped to
// 1 ... 1 + MAX_SIDE (r6: no environment override; the lane sweeps of r4-r5 are in DESIGN.md section 4)
int pbs_lane_count(int dflt);

}  // namespace mi
