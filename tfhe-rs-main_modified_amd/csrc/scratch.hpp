// scratch.hpp — temporary device buffers of the batched entry points.  On a caller's stream they are stream-ordered
// (hipMallocAsync / hipFreeAsync: no device synchronisation per call).  On the legacy null stream (stream == NULL,
// the C ABI's default) they are plain allocations freed after the stream drains: with the /opt/rocm 7.2 runtime the
// C++ mirror suite saw stream-ordered scratch on the null stream come back with stale contents (an in-place Fourier
// reorder and a generic f64 external product at N = 8192, a few runs in a hundred; tools/fftg_rt_probe.cpp), which the
// plain allocation does not show.
#pragma once
#include <hip/hip_runtime.h>

namespace mi {

inline hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s) {
  return s ? hipMallocAsync(p, bytes, s) : hipMalloc(p, bytes);
}

inline hipError_t scratch_free(void* p, hipStream_t s) {
  if (!p) return hipSuccess;
  if (s) return hipFreeAsync(p, s);
  const hipError_t e = hipStreamSynchronize(nullptr);
  const hipError_t f = hipFree(p);
  return e != hipSuccess ? e : f;
}

}  // namespace mi
