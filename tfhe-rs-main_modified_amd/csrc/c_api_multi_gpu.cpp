// c_api_multi_gpu.cpp — single-process multi-GPU helpers of the C ABI (mi_multi_gpu_*), the analogue of
// the CUDA backend's helper_multi_gpu (backends/tfhe-cuda-backend/cuda/src/utils/helper_multi_gpu.cu:10-98,
// helper_multi_gpu.cuh:150-265): a device set with one stream per device, the contiguous batch split,
// broadcast of read-only state, scatter / gather of LWE batches from / to the first device over
// peer-to-peer copies (xGMI on MI355X: each peer is fed over its own link), and a whole multi-GPU PBS.
//
// Bootstraps are independent: the data path has no collective; only the edges move
// data.  The one-process-per-GPU form of the same split (torch.distributed / RCCL) lives in
// tfhe_ntt_amd/multi_gpu.py and bench.py.
#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "scratch.hpp"
#include "c_api_internal.hpp"

using namespace mi::capi;

struct mi_multi_gpu {
  std::vector<int> devices;
  std::vector<hipStream_t> streams;  // non-blocking, one per entry of `devices`
  std::vector<hipEvent_t> events;    // one per entry, for cross-stream ordering
};

namespace {

constexpr uint32_t THRESHOLD_MULTI_GPU = 12;  // helper_multi_gpu.cu:9

// get_num_inputs_on_gpu / get_gpu_offset (helper_multi_gpu.cu:47-98): with fewer inputs than GPUs the
// first `total` GPUs take one each; otherwise contiguous chunks, the first total % count one larger.
void shard(size_t total, size_t index, size_t count, size_t* offset, size_t* n) {
  if (count > total) {
    *n = index < total ? 1 : 0;
    *offset = std::min(index, total);
    return;
  }
  const size_t base = total / count, extra = total % count;
  *n = base + (index < extra ? 1 : 0);
  *offset = index * base + std::min(index, extra);
}

// order `to` after everything queued so far on `from` (same or different device)
hipError_t after(hipStream_t to, hipStream_t from, hipEvent_t ev, int from_device) {
  DeviceGuard g(from_device);
  hipError_t e = hipEventRecord(ev, from);
  return e == hipSuccess ? hipStreamWaitEvent(to, ev, 0) : e;
}

}  // namespace

extern "C" {

int mi_multi_gpu_create(const int* devices, int count, mi_multi_gpu** out) {
  if (!out) return fail(MI_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  if (!devices || count < 1) return fail(MI_ERR_INVALID_ARG, "need at least one device");
  int visible = 0;
  if (hipGetDeviceCount(&visible) != hipSuccess || visible < 1) return fail(MI_ERR_HIP, "no HIP device visible");
  for (int i = 0; i < count; ++i)
    if (devices[i] < 0 || devices[i] >= visible) return fail(MI_ERR_INVALID_ARG, "device index out of range");
  // cuda_setup_multi_gpu (helper_multi_gpu.cu:11-40): bidirectional peer access between device 0 of the
  // set and every other device, enabled once per process and pair
  static std::mutex mu;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 1; i < count; ++i) {
      const int a = devices[0], b = devices[i];
      if (a == b) continue;
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, b, a) != hipSuccess || !ok) continue;  // falls back to staged copies
      for (auto [x, y] : {std::pair<int, int>{a, b}, std::pair<int, int>{b, a}}) {
        DeviceGuard g(x);
        const hipError_t e = hipDeviceEnablePeerAccess(y, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return hip_fail(e, "hipDeviceEnablePeerAccess");
        (void)hipGetLastError();  // clear the already-enabled status
      }
    }
  }
  mi_multi_gpu* m = new (std::nothrow) mi_multi_gpu;
  if (!m) return fail(MI_ERR_OOM, "host allocation failed");
  m->devices.assign(devices, devices + count);
  for (int i = 0; i < count; ++i) {
    DeviceGuard g(devices[i]);
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      if (s) (void)hipStreamDestroy(s);
      m->streams.push_back(nullptr);
      m->events.push_back(nullptr);
      mi_multi_gpu_destroy(m);
      return hip_fail(e, "stream creation");
    }
    m->streams.push_back(s);
    m->events.push_back(ev);
  }
  *out = m;
  return MI_OK;
}

int mi_multi_gpu_destroy(mi_multi_gpu* m) {
  if (!m) return MI_OK;
  for (size_t i = 0; i < m->devices.size() && i < m->streams.size(); ++i) {
    DeviceGuard g(m->devices[i]);
    if (m->streams[i]) {
      (void)hipStreamSynchronize(m->streams[i]);
      mi::scratch_stream_retired(m->streams[i]);
      (void)hipStreamDestroy(m->streams[i]);
    }
    if (i < m->events.size() && m->events[i]) (void)hipEventDestroy(m->events[i]);
  }
  delete m;
  return MI_OK;
}

int mi_multi_gpu_info(const mi_multi_gpu* m, int index, int* device, void** stream) {
  if (!m) return fail(MI_ERR_INVALID_ARG, "device set is NULL");
  if (index < 0 || index >= (int)m->devices.size()) return fail(MI_ERR_INVALID_ARG, "index out of range");
  if (device) *device = m->devices[index];
  if (stream) *stream = m->streams[index];
  return MI_OK;
}

int mi_multi_gpu_count(const mi_multi_gpu* m, int* count) {
  if (!m || !count) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  *count = (int)m->devices.size();
  return MI_OK;
}

int mi_multi_gpu_active_count(uint32_t num_inputs, uint32_t gpu_count, uint32_t* out) {
  if (!out || gpu_count == 0) return fail(MI_ERR_INVALID_ARG, "bad argument");
  const uint32_t ceil_div = std::max<uint32_t>(1, (num_inputs + THRESHOLD_MULTI_GPU - 1) / THRESHOLD_MULTI_GPU);
  *out = std::min(ceil_div, gpu_count);  // get_active_gpu_count (helper_multi_gpu.cu:42-49)
  return MI_OK;
}

int mi_multi_gpu_shard(size_t total, int index, int count, size_t* offset, size_t* n) {
  if (!offset || !n || count < 1 || index < 0 || index >= count) return fail(MI_ERR_INVALID_ARG, "bad shard request");
  shard(total, (size_t)index, (size_t)count, offset, n);
  return MI_OK;
}

int mi_multi_gpu_synchronize(const mi_multi_gpu* m) {
  if (!m) return fail(MI_ERR_INVALID_ARG, "device set is NULL");
  for (size_t i = 0; i < m->devices.size(); ++i) {
    DeviceGuard g(m->devices[i]);
    const hipError_t e = hipStreamSynchronize(m->streams[i]);
    if (e != hipSuccess) return hip_fail(e, "stream synchronize");
  }
  return MI_OK;
}

// dsts[i] on devices[i] receives `bytes` from src on devices[0]; dsts[i] == src is skipped.  Ordered
// after `stream` (on devices[0]); returns with the copies queued on the set's streams.
int mi_multi_gpu_broadcast(mi_multi_gpu* m, const void* src, void* const* dsts, size_t bytes, void* stream) {
  if (!m || !src || !dsts) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  const int d0 = m->devices[0];
  for (size_t i = 0; i < m->devices.size(); ++i) {
    if (!dsts[i]) return fail(MI_ERR_INVALID_ARG, "destination is NULL");
    if (dsts[i] == src || bytes == 0) continue;
    DeviceGuard g(m->devices[i]);
    hipError_t e = after(m->streams[i], (hipStream_t)stream, m->events[0], d0);
    if (e == hipSuccess) e = hipMemcpyPeerAsync(dsts[i], m->devices[i], src, d0, bytes, m->streams[i]);
    if (e != hipSuccess) return hip_fail(e, "broadcast copy");
  }
  return MI_OK;
}

// multi_gpu_scatter_lwe_async with the trivial index (helper_multi_gpu.cuh:150-176): shard i of the
// `total` units of `unit_bytes` at src (devices[0]) goes to dsts[i].
int mi_multi_gpu_scatter(mi_multi_gpu* m, const void* src, void* const* dsts, size_t total, size_t unit_bytes,
                         void* stream) {
  if (!m || !src || !dsts) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  const size_t G = m->devices.size();
  for (size_t i = 0; i < G; ++i) {
    size_t off = 0, n = 0;
    shard(total, i, G, &off, &n);
    if (n == 0) continue;
    if (!dsts[i]) return fail(MI_ERR_INVALID_ARG, "destination is NULL");
    const char* from = (const char*)src + off * unit_bytes;
    if (dsts[i] == from) continue;
    DeviceGuard g(m->devices[i]);
    hipError_t e = after(m->streams[i], (hipStream_t)stream, m->events[0], m->devices[0]);
    if (e == hipSuccess)
      e = hipMemcpyPeerAsync(dsts[i], m->devices[i], from, m->devices[0], n * unit_bytes, m->streams[i]);
    if (e != hipSuccess) return hip_fail(e, "scatter copy");
  }
  return MI_OK;
}

// multi_gpu_gather_lwe_async with the trivial index (helper_multi_gpu.cuh:211-238): srcs[i] (devices[i])
// back into shard i of dst (devices[0]); `stream` is ordered after every copy.
int mi_multi_gpu_gather(mi_multi_gpu* m, void* dst, const void* const* srcs, size_t total, size_t unit_bytes,
                        void* stream) {
  if (!m || !dst || !srcs) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  const size_t G = m->devices.size();
  for (size_t i = 0; i < G; ++i) {
    size_t off = 0, n = 0;
    shard(total, i, G, &off, &n);
    if (n == 0) continue;
    if (!srcs[i]) return fail(MI_ERR_INVALID_ARG, "source is NULL");
    char* to = (char*)dst + off * unit_bytes;
    DeviceGuard g(m->devices[i]);
    hipError_t e = hipSuccess;
    // the copy into dst waits for the work already queued on `stream` (whatever produced or cleared dst there: without
    // this a zero-fill of dst queued on `stream` could land after the copy, GPU test test_device_set_pbs_scatter_gather)
    if (srcs[i] != to) e = after(m->streams[i], (hipStream_t)stream, m->events[0], m->devices[0]);
    if (srcs[i] != to && e == hipSuccess)
      e = hipMemcpyPeerAsync(to, m->devices[0], srcs[i], m->devices[i], n * unit_bytes, m->streams[i]);
    if (e == hipSuccess) e = after((hipStream_t)stream, m->streams[i], m->events[i], m->devices[i]);
    if (e != hipSuccess) return hip_fail(e, "gather copy");
  }
  return MI_OK;
}

// The CUDA backend's multi-GPU bootstrap pattern: scatter the LWE batch from devices[0], one PBS launch per
// active device with that device's key and LUT copy, gather the outputs back.  Only the first
// get_active_gpu_count(batch, G) entries take part (helper_multi_gpu.cu:42-49, CudaStreams::active_gpu_subset,
// helper_multi_gpu.h:74-79): a batch of 13 on 8 entries runs on 2 devices (7 + 6), and the keys / LUTs of the
// inactive entries are not read.  keys[i] / luts[i] live on devices[i]; lwe_in / lwe_out on devices[0].
//
// Ordering: `stream` (devices[0]) is ordered before the whole call and after it.  producer_streams[i] (a stream of
// devices[i], NULL entry or NULL array = that device's legacy null stream) is the stream that produced luts[i] /
// keys[i]: shard i starts after the work queued on it so far, and it is ordered after shard i's last use of them,
// so the caller's allocator may free or reuse them on that stream as soon as the call returns.  Shard 0 runs in
// place on `stream`; the other shards use stream-ordered scratch on their device.
}  // extern "C"

namespace {
// what the multi-GPU bootstrap needs of a key: its device and shape, and its single-device batch launch
struct KeyShape {
  int device;
  size_t n_lwe, n;
  int k, variant;
};
KeyShape shape_of(const mi_pbs_ntt64_key* key) {
  return {key->plan->device, key->n_lwe, key->plan->n, key->k, key->variant};
}
KeyShape shape_of(const mi_fft64_pbs_key* key) { return {key->plan->device, key->n_lwe, key->plan->n, key->k, -1}; }
int pbs_batch(const mi_pbs_ntt64_key* key, uint64_t* out, const uint64_t* in, const uint64_t* lut, size_t n,
              int ms_mode, void* stream) {
  return mi_pbs_ntt64_batch(key, out, in, lut, n, ms_mode, stream);
}
int pbs_batch(const mi_fft64_pbs_key* key, uint64_t* out, const uint64_t* in, const uint64_t* lut, size_t n,
              int ms_mode, void* stream) {
  return mi_fft64_pbs_batch(key, out, in, lut, n, ms_mode, stream);
}

template <class Key>
int multi_gpu_pbs(mi_multi_gpu* m, const Key* const* keys, uint64_t* lwe_out, const uint64_t* lwe_in,
                  const uint64_t* const* luts, size_t batch, int ms_mode, void* stream, void* const* producer_streams) {
  if (!m || !keys || !luts) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  if (batch == 0) return MI_OK;
  if (!lwe_out || !lwe_in) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  uint32_t active = 0;
  mi_multi_gpu_active_count((uint32_t)batch, (uint32_t)m->devices.size(), &active);
  const size_t G = active;
  for (size_t i = 0; i < G; ++i) {
    if (!keys[i] || !luts[i]) return fail(MI_ERR_INVALID_ARG, "key / lut of an active entry is NULL");
    const KeyShape a = shape_of(keys[i]), b = shape_of(keys[0]);
    if (a.device != m->devices[i]) return fail(MI_ERR_INVALID_ARG, "keys[i] is not on devices[i]");
    if (a.n_lwe != b.n_lwe || a.k != b.k || a.variant != b.variant || a.n != b.n)
      return fail(MI_ERR_INVALID_ARG, "keys differ in shape");
  }
  const KeyShape k0 = shape_of(keys[0]);
  const size_t in_w = k0.n_lwe + 1, out_w = (size_t)k0.k * k0.n + 1;
  auto producer = [&](size_t i) -> hipStream_t {
    return producer_streams ? (hipStream_t)producer_streams[i] : nullptr;
  };
  std::vector<uint64_t*> ins(G, nullptr), outs(G, nullptr), scratch(G, nullptr);
  int st = MI_OK;
  for (size_t i = 0; i < G && st == MI_OK; ++i) {
    size_t off = 0, n = 0;
    shard(batch, i, G, &off, &n);
    if (i == 0 || n == 0) {
      ins[i] = const_cast<uint64_t*>(lwe_in) + off * in_w;
      outs[i] = lwe_out + off * out_w;
      continue;
    }
    DeviceGuard g(m->devices[i]);
    // shard i's work on the set's stream follows its producer stream (the key / LUT of devices[i])
    hipError_t e = after(m->streams[i], producer(i), m->events[i], m->devices[i]);
    if (e != hipSuccess) {
      st = hip_fail(e, "producer-stream ordering");
      break;
    }
    uint64_t* buf = nullptr;
    if (mi::scratch_alloc((void**)&buf, n * (in_w + out_w) * sizeof(uint64_t), m->streams[i]) != hipSuccess)
      st = fail(MI_ERR_OOM, "shard scratch allocation failed");
    scratch[i] = ins[i] = buf;
    outs[i] = buf ? buf + n * in_w : nullptr;
  }
  // shard 0 follows its producer stream too, when that is not the caller's stream itself
  if (st == MI_OK && producer(0) != (hipStream_t)stream) {
    hipError_t e = after((hipStream_t)stream, producer(0), m->events[0], m->devices[0]);
    if (e != hipSuccess) st = hip_fail(e, "producer-stream ordering");
  }
  // scatter / gather over the active prefix of the set only
  std::vector<void*> dsts(m->devices.size(), nullptr);
  std::vector<const void*> srcs(m->devices.size(), nullptr);
  for (size_t i = 0; i < G; ++i) {
    dsts[i] = ins[i];
    srcs[i] = outs[i];
  }
  mi_multi_gpu sub;
  sub.devices.assign(m->devices.begin(), m->devices.begin() + G);
  sub.streams.assign(m->streams.begin(), m->streams.begin() + G);
  sub.events.assign(m->events.begin(), m->events.begin() + G);
  if (st == MI_OK) st = mi_multi_gpu_scatter(&sub, lwe_in, dsts.data(), batch, in_w * 8, stream);
  // shard 0 runs on the caller's stream directly; the others on their device streams
  for (size_t i = 0; i < G && st == MI_OK; ++i) {
    size_t off = 0, n = 0;
    shard(batch, i, G, &off, &n);
    if (n == 0) continue;
    st = pbs_batch(keys[i], outs[i], ins[i], luts[i], n, ms_mode, i == 0 ? stream : m->streams[i]);
  }
  if (st == MI_OK) st = mi_multi_gpu_gather(&sub, lwe_out, srcs.data(), batch, out_w * 8, stream);
  for (size_t i = 1; i < G; ++i)
    if (scratch[i]) {
      DeviceGuard g(m->devices[i]);
      (void)mi::scratch_free(scratch[i], m->streams[i]);
    }
  // the producer streams follow the last use of their key / LUT (shard 0's is `stream`, which the gather ordered) —
  // also when a later step failed after some shards were already queued: the first error is still the one returned
  for (size_t i = 0; i < G; ++i) {
    hipStream_t ps = producer(i);
    if (i == 0 && ps == (hipStream_t)stream) continue;
    hipError_t e = after(ps, i == 0 ? (hipStream_t)stream : m->streams[i], m->events[i], m->devices[i]);
    if (e != hipSuccess && st == MI_OK) st = hip_fail(e, "producer-stream ordering");
  }
  return st;
}
}  // namespace

extern "C" {

int mi_pbs_ntt64_multi_gpu_ordered(mi_multi_gpu* m, const mi_pbs_ntt64_key* const* keys, uint64_t* lwe_out,
                                   const uint64_t* lwe_in, const uint64_t* const* luts, size_t batch, int ms_mode,
                                   void* stream, void* const* producer_streams) {
  return multi_gpu_pbs(m, keys, lwe_out, lwe_in, luts, batch, ms_mode, stream, producer_streams);
}

// the same sharding for the f64-FFT bootstrap (the default shortint PBS; the CUDA backend's multi-GPU PBS is the
// FFT one, helper_multi_gpu.cu)
int mi_fft64_pbs_multi_gpu_ordered(mi_multi_gpu* m, const mi_fft64_pbs_key* const* keys, uint64_t* lwe_out,
                                   const uint64_t* lwe_in, const uint64_t* const* luts, size_t batch, int ms_mode,
                                   void* stream, void* const* producer_streams) {
  return multi_gpu_pbs(m, keys, lwe_out, lwe_in, luts, batch, ms_mode, stream, producer_streams);
}

int mi_fft64_pbs_multi_gpu(mi_multi_gpu* m, const mi_fft64_pbs_key* const* keys, uint64_t* lwe_out,
                           const uint64_t* lwe_in, const uint64_t* const* luts, size_t batch, int ms_mode, void* stream) {
  return multi_gpu_pbs(m, keys, lwe_out, lwe_in, luts, batch, ms_mode, stream, nullptr);
}

int mi_pbs_ntt64_multi_gpu(mi_multi_gpu* m, const mi_pbs_ntt64_key* const* keys, uint64_t* lwe_out,
                           const uint64_t* lwe_in, const uint64_t* const* luts, size_t batch, int ms_mode, void* stream) {
  return mi_pbs_ntt64_multi_gpu_ordered(m, keys, lwe_out, lwe_in, luts, batch, ms_mode, stream, nullptr);
}

}  // extern "C"
