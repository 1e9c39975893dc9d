// scratch.cpp — the event-ordered scratch pool (scratch.hpp).
#include "scratch.hpp"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace mi {
namespace {

struct Block {
  void* p = nullptr;
  size_t bytes = 0;
  int device = 0;
  hipEvent_t last_use = nullptr;  // recorded on the stream of the block's last user
  hipStream_t stream = nullptr;   // that stream (scratch_stream_retired)
  bool recorded = false;
};

struct Pool {
  std::mutex mu;
  std::vector<Block> idle;
  std::unordered_map<void*, Block> busy;
};

Pool& pool() {
  static Pool* p = new Pool;  // never destroyed: the HIP runtime may be torn down before static destructors run
  return *p;
}

struct SidePool {
  std::mutex mu;
  std::vector<std::pair<int, hipStream_t>> idle;  // (device, stream)
};

SidePool& side_pool() {
  static SidePool* p = new SidePool;  // never destroyed, as pool()
  return *p;
}

// an idle side stream of `dev`, or a new non-blocking one
hipError_t side_acquire(int dev, hipStream_t* out) {
  SidePool& P = side_pool();
  {
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto it = P.idle.begin(); it != P.idle.end(); ++it)
      if (it->first == dev) {
        *out = it->second;
        P.idle.erase(it);
        return hipSuccess;
      }
  }
  return hipStreamCreateWithFlags(out, hipStreamNonBlocking);
}

void side_release(int dev, hipStream_t st) {
  SidePool& P = side_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  P.idle.emplace_back(dev, st);
}

// one event recorded on `from` and waited on by `to` (the event may be destroyed at once: the wait holds it)
hipError_t order_after(hipStream_t to, hipStream_t from) {
  hipEvent_t ev;
  hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  e = hipEventRecord(ev, from);
  if (e == hipSuccess) e = hipStreamWaitEvent(to, ev, 0);
  (void)hipEventDestroy(ev);
  return e;
}

constexpr size_t GRAIN = (size_t)1 << 20;  // blocks are whole MiB

// an idle block serves a request only when it is at most 4x the request or 64 MiB above it, so a small request does
// not take (and pin) a block sized for the large-N blind rotation while a concurrent large request allocates another
bool fits_snugly(size_t block, size_t request) {
  return block / 4 <= request || block - request <= ((size_t)64 << 20);
}

// waits for the block's last user.  The event was recorded on the caller's stream, which the caller may have destroyed
// since: on ROCm an event whose stream is gone can fail hipEventSynchronize / hipStreamWaitEvent (observed:
// hipErrorCapturedEvent with no capture anywhere in the process).  The fallback is a device-wide wait, and the runtime's
// sticky last error is cleared, so a later unrelated hipGetLastError (torch checks it after every launch) does not
// report it.
void wait_last_use(const Block& b) {
  if (!b.recorded) return;
  if (hipEventSynchronize(b.last_use) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipDeviceSynchronize();
    (void)hipGetLastError();
  }
}

// frees blocks that no longer have a pending user (their event has completed)
void release(std::vector<Block>& blocks) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (Block& b : blocks) {
    (void)hipSetDevice(b.device);
    wait_last_use(b);
    (void)hipEventDestroy(b.last_use);
    (void)hipFree(b.p);
    (void)hipGetLastError();
  }
  (void)hipSetDevice(cur);
}

// takes the smallest idle block of `dev` that holds `bytes` (snug ones only when `snug`) into the busy map
bool take_idle(Pool& P, int dev, size_t bytes, bool snug, Block* out) {
  auto best = P.idle.end();
  for (auto it = P.idle.begin(); it != P.idle.end(); ++it)
    if (it->device == dev && it->bytes >= bytes && (!snug || fits_snugly(it->bytes, bytes)) &&
        (best == P.idle.end() || it->bytes < best->bytes))
      best = it;
  if (best == P.idle.end()) return false;
  *out = *best;
  P.idle.erase(best);
  P.busy[out->p] = *out;
  return true;
}

// hands a reused block to the caller: its stream waits for the block's last user (host-side, if the event cannot be
// waited on by the stream: see wait_last_use)
hipError_t issue_reused(const Block& blk, void** out, hipStream_t s) {
  if (blk.recorded && hipStreamWaitEvent(s, blk.last_use, 0) != hipSuccess) {
    (void)hipGetLastError();
    wait_last_use(blk);
  }
  *out = blk.p;
  return hipSuccess;
}

}  // namespace

hipError_t scratch_alloc(void** out, size_t bytes, hipStream_t s) {
  *out = nullptr;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (bytes == 0) bytes = 1;
  Pool& P = pool();
  Block blk;
  bool found = false;
  std::vector<Block> smaller;  // idle blocks a new, larger block supersedes
  {
    std::lock_guard<std::mutex> lk(P.mu);
    found = take_idle(P, dev, bytes, true, &blk);
    if (!found) {
      // only the idle blocks too small for this request are superseded; a much larger idle block stays for the
      // large requests it was made for (a small request no longer takes the 4 GiB PBS block)
      auto keep = std::partition(P.idle.begin(), P.idle.end(),
                                 [&](const Block& b) { return b.device != dev || b.bytes >= bytes; });
      smaller.assign(keep, P.idle.end());
      P.idle.erase(keep, P.idle.end());
    }
  }
  if (found) return issue_reused(blk, out, s);
  release(smaller);
  blk = Block{};
  blk.device = dev;
  blk.bytes = (bytes + GRAIN - 1) / GRAIN * GRAIN;
  if ((e = hipMalloc(&blk.p, blk.bytes)) != hipSuccess) {
    (void)hipGetLastError();
    // out of device memory: serve the request from any idle block of this device that holds it, snug or
    // not (before the snug rule this request would have taken it); failing that, free every idle block of the device
    // once its last user has retired and try the allocation again
    {
      std::lock_guard<std::mutex> lk(P.mu);
      found = take_idle(P, dev, bytes, false, &blk);
    }
    if (found) return issue_reused(blk, out, s);
    (void)scratch_trim(dev);
    blk = Block{};
    blk.device = dev;
    blk.bytes = (bytes + GRAIN - 1) / GRAIN * GRAIN;
    if ((e = hipMalloc(&blk.p, blk.bytes)) != hipSuccess) {
      (void)hipGetLastError();
      return e;
    }
  }
  if ((e = hipEventCreateWithFlags(&blk.last_use, hipEventDisableTiming)) != hipSuccess) {
    (void)hipFree(blk.p);
    return e;
  }
  {
    std::lock_guard<std::mutex> lk(P.mu);
    P.busy[blk.p] = blk;
  }
  *out = blk.p;
  return hipSuccess;
}

hipError_t scratch_free(void* p, hipStream_t s) {
  if (!p) return hipSuccess;
  Pool& P = pool();
  Block blk;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto it = P.busy.find(p);
    if (it == P.busy.end()) return hipErrorInvalidValue;
    blk = it->second;
  }
  // the block is still owned by this caller: record before it becomes visible to others
  const hipError_t e = hipEventRecord(blk.last_use, s);
  blk.recorded = e == hipSuccess;
  blk.stream = s;
  if (!blk.recorded) {  // cannot order the next user: retire the block after the device drains
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> lk(P.mu);
    P.busy.erase(p);
    std::vector<Block> one{blk};
    release(one);
    return e;
  }
  std::lock_guard<std::mutex> lk(P.mu);
  P.busy.erase(p);
  P.idle.push_back(blk);
  return hipSuccess;
}

void scratch_stream_retired(hipStream_t s) {
  if (!s) return;  // the null stream is never destroyed
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  for (Block& b : P.idle)
    if (b.stream == s) b.recorded = false;  // the caller synchronized s: the block's last use has completed
  for (auto& kv : P.busy)
    if (kv.second.stream == s) kv.second.recorded = false;
}

size_t scratch_trim(int device) {
  Pool& P = pool();
  std::vector<Block> out;
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto keep = std::partition(P.idle.begin(), P.idle.end(),
                               [&](const Block& b) { return device >= 0 && b.device != device; });
    out.assign(keep, P.idle.end());
    P.idle.erase(keep, P.idle.end());
  }
  size_t bytes = 0;
  for (const Block& b : out) bytes += b.bytes;
  release(out);
  return bytes;
}

hipError_t StreamFork::fork(hipStream_t s, int n) {
  if (n_ > 0) return hipErrorInvalidValue;
  hipError_t e = hipGetDevice(&device_);
  if (e != hipSuccess) return e;
  caller_ = s;
  n = std::max(0, std::min(n, MAX_SIDE));
  while (n_ < n) {
    hipStream_t st = nullptr;
    if ((e = side_acquire(device_, &st)) != hipSuccess) break;
    if ((e = order_after(st, s)) != hipSuccess) {
      side_release(device_, st);
      break;
    }
    side_[n_++] = st;
  }
  return n_ == n ? hipSuccess : e;
}

hipError_t StreamFork::join() {
  hipError_t first = hipSuccess;
  for (int i = 0; i < n_; ++i) {
    const hipError_t e = order_after(caller_, side_[i]);
    if (e != hipSuccess) {
      (void)hipStreamSynchronize(side_[i]);  // cannot order by event: drain the side stream instead
      if (first == hipSuccess) first = e;
    }
    side_release(device_, side_[i]);
    side_[i] = nullptr;
  }
  n_ = 0;
  return first;
}

int pbs_lane_count(int dflt) { return std::max(1, std::min(dflt, 1 + StreamFork::MAX_SIDE)); }

size_t scratch_bytes(int device) {
  Pool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  size_t bytes = 0;
  for (const Block& b : P.idle)
    if (device < 0 || b.device == device) bytes += b.bytes;
  for (const auto& kv : P.busy)
    if (device < 0 || kv.second.device == device) bytes += kv.second.bytes;
  return bytes;
}

}  // namespace mi
