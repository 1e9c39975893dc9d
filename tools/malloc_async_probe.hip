// Diagnostic (GPU box): is memory from hipMallocAsync on the legacy null stream safe to fill with hipMemcpyAsync and
// read by a kernel on that stream, across hipFreeAsync / hipMallocAsync of different sizes?  Mirrors the in-place
// reorder of the shape-generic f64 engine (launch_fftg_reorder).  Prints the number of wrong results per mode.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void copy_kernel(uint64_t* out, const uint64_t* in, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) out[i] = in[i] ^ 1;
}

int main(int argc, char** argv) {
  const hipStream_t s = argc > 1 ? nullptr : nullptr;
  int bad = 0, total = 0;
  const size_t sizes[] = {2048, 16384, 4096, 16384, 1 << 15, 2048, 16384};
  for (int rep = 0; rep < 20; ++rep)
    for (size_t n : sizes) {
      std::vector<uint64_t> h(n), g(n);
      for (size_t i = 0; i < n; ++i) h[i] = i * 0x9E3779B97F4A7C15ull + rep;
      uint64_t* buf = nullptr;
      hipMalloc(&buf, n * 8);
      hipMemcpy(buf, h.data(), n * 8, hipMemcpyHostToDevice);
      uint64_t* tmp = nullptr;
      if (hipMallocAsync((void**)&tmp, n * 8, s) != hipSuccess) { std::printf("alloc failed\n"); return 1; }
      hipMemcpyAsync(tmp, buf, n * 8, hipMemcpyDeviceToDevice, s);
      hipLaunchKernelGGL(copy_kernel, dim3(64), dim3(256), 0, s, buf, tmp, n);
      hipFreeAsync(tmp, s);
      hipMemcpy(g.data(), buf, n * 8, hipMemcpyDeviceToHost);
      size_t wrong = 0;
      for (size_t i = 0; i < n; ++i) wrong += g[i] != (h[i] ^ 1);
      bad += wrong != 0;
      ++total;
      hipFree(buf);
    }
  std::printf("malloc_async_probe: %d of %d rounds wrong\n", bad, total);
  return 0;
}
