// Diagnostic (GPU box): the in-place reorder sequence that came back stale in r3 (profiles/r3/null_stream_scratch/),
// restated without the library so each ingredient can be switched on its own.  Per rep, exactly as
// tools/fftg_rt_probe.cpp drives the f64 engine at N = 1024 (batch 2):
//   hipMalloc four / nat / back; K1 fills four; D2H four; K2 nat = perm(four); K3 back = perm^-1(nat); D2H back;
//   in place: tmp = scratch; copy tmp <- nat; K4 nat = perm^-1(tmp); release tmp; D2H nat (must equal four);
//   hipFree four / nat / back.
// mode bits: 1 = stage with an SDMA copy (hipMemcpyAsync D2D) instead of a copy kernel; 2 = stream-ordered scratch
// (hipMallocAsync / hipFreeAsync) instead of hipMalloc / hipFree after a sync; 4 = release threshold of the default
// pool = UINT64_MAX (the pool never returns memory to the device allocator); 8 = a created non-blocking stream
// instead of the legacy null stream.  Prints the wrong in-place results per mode and, for the first wrong rep, where
// the runtime says `tmp` lives against the rep's other buffers.
//   ./scratch_order_probe <n_complex> <reps> <mode> [<mode> ...]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void fill_kernel(double* out, size_t n, uint64_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = (double)((i + 1) * 0x9E3779B97F4A7C15ull ^ seed) * 0x1p-64;
}
// a fixed permutation of each polynomial's m complex values (a bit reversal), and its inverse
__device__ size_t rev(size_t x, int bits) { return __brevll(x) >> (64 - bits); }
__global__ void perm_kernel(double2* out, const double2* in, size_t polys, int logm) {
  const size_t m = (size_t)1 << logm, total = polys * m;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
    out[(i >> logm << logm) + rev(i & (m - 1), logm)] = in[i];
}
__global__ void copy_kernel(double2* out, const double2* in, size_t total) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

static const char* where(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return "unknown to the runtime";
  }
  return a.type == hipMemoryTypeDevice ? "device" : a.type == hipMemoryTypeHost ? "host" : "other";
}

int main(int argc, char** argv) {
  const size_t m = argc > 1 ? (size_t)atoll(argv[1]) : 512, reps = argc > 2 ? (size_t)atoll(argv[2]) : 6;
  int logm = 0;
  while (((size_t)1 << logm) < m) ++logm;
  const size_t polys = 2, total = polys * m, bytes = total * sizeof(double2);
  for (int ai = 3; ai < (argc > 3 ? argc : 4); ++ai) {
    const int mode = argc > 3 ? atoi(argv[ai]) : 3;
    const bool sdma = mode & 1, pool = mode & 2, keep = mode & 4, own = mode & 8;
    hipStream_t s = nullptr;
    if (own) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipMemPool_t mp;
    CK(hipDeviceGetDefaultMemPool(&mp, 0));
    uint64_t thr = keep ? ~0ull : 0ull;
    CK(hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &thr));
    int bad = 0;
    for (size_t r = 0; r < reps; ++r) {
      double2 *four = nullptr, *nat = nullptr, *back = nullptr, *tmp = nullptr;
      CK(hipMalloc(&four, bytes));
      CK(hipMalloc(&nat, bytes));
      CK(hipMalloc(&back, bytes));
      hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, s, (double*)four, 2 * total, (uint64_t)r);
      std::vector<double2> h0(total), h1(total);
      CK(hipMemcpyAsync(h0.data(), four, bytes, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      hipLaunchKernelGGL(perm_kernel, dim3(64), dim3(256), 0, s, nat, four, polys, logm);
      hipLaunchKernelGGL(perm_kernel, dim3(64), dim3(256), 0, s, back, nat, polys, logm);
      CK(hipMemcpyAsync(h1.data(), back, bytes, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      // in place: stage nat, then nat = perm^-1(tmp) (a bit reversal is its own inverse)
      if (pool) CK(hipMallocAsync((void**)&tmp, bytes, s));
      else CK(hipMalloc(&tmp, bytes));
      if (sdma) CK(hipMemcpyAsync(tmp, nat, bytes, hipMemcpyDeviceToDevice, s));
      else hipLaunchKernelGGL(copy_kernel, dim3(64), dim3(256), 0, s, tmp, nat, total);
      hipLaunchKernelGGL(perm_kernel, dim3(64), dim3(256), 0, s, nat, tmp, polys, logm);
      if (pool) CK(hipFreeAsync(tmp, s));
      std::vector<double2> h2(total);
      CK(hipMemcpyAsync(h2.data(), nat, bytes, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      if (!pool) CK(hipFree(tmp));
      size_t wrong = 0;
      for (size_t i = 0; i < total; ++i) wrong += h2[i].x != h0[i].x || h2[i].y != h0[i].y;
      const bool oop_ok = std::memcmp(h1.data(), h0.data(), bytes) == 0;
      if (wrong && !bad)
        std::printf("  mode %d rep %zu: %zu of %zu wrong (out-of-place %s); tmp %p (%s) four %p nat %p back %p\n", mode,
                    r, wrong, total, oop_ok ? "ok" : "WRONG", (void*)tmp, where(tmp), (void*)four, (void*)nat,
                    (void*)back);
      bad += wrong != 0;
      CK(hipFree(four));
      CK(hipFree(nat));
      CK(hipFree(back));
    }
    std::printf("mode %d (%s copy, %s scratch, release threshold %s, %s stream): %d of %zu in-place results wrong\n",
                mode, sdma ? "SDMA" : "kernel", pool ? "hipMallocAsync" : "hipMalloc", keep ? "max" : "0",
                own ? "non-blocking" : "null", bad, reps);
    if (own) CK(hipStreamDestroy(s));
  }
  return 0;
}
