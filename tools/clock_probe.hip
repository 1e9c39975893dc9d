// clock_probe.hip — diagnostic build (not part of the library): the twisted N = 2048 transform body
// (csrc/ntt64_tw_body.hpp, the same generated asm as ntt_tw_body_kernel) wrapped in s_memtime /
// s_memrealtime stamps, to read the clock the chip holds under this load (MI355X_MICROARCH.md, DVFS
// item 6: in-kernel clock = d(memtime) / d(memrealtime) x 100 MHz) and each wave's lifetime in cycles.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I tfhe-rs-main_modified_amd/csrc tools/clock_probe.hip -o tools/clock_probe
//   ./tools/clock_probe            (one JSON line)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "ntt64_tw_body.hpp"

using u64 = uint64_t;
static constexpr int WAVE_LDS2 = 1088;

template <bool FWD, bool STAMP>
__global__ __launch_bounds__(256, 4) void probe_kernel(u64* __restrict__ data, uint32_t batch, const u64* __restrict__ twist,
                                                       u64* __restrict__ stamps) {
  __shared__ u64 lds[4 * WAVE_LDS2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t poly = blockIdx.x * 4 + wv;
  if (poly >= batch) return;
  u64* p = data + (uint64_t)poly * 2048;
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8;
  const uint32_t t1w = S + (lane & 31) * 8;
  const uint32_t t1r = S + (i * 34 + par) * 8;
  const uint32_t lwo = par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2048;
  u64 c0 = 0, r0 = 0;
  if (STAMP) {
    c0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  if constexpr (FWD) {
    const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8;
    const uint32_t t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
    const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
    MI_TW_BODY_FWD([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r), [t2wl] "v"(t2wl), [t2wh] "v"(t2wh),
                   [t2r] "v"(t2r), [lwo] "v"(lwo));
  } else {
    const uint32_t t4w = S + ((i & 15) * 66 + par) * 8;
    const uint32_t t4r = S + lane * 8;
    MI_TW_BODY_INV([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r), [t4w] "v"(t4w), [t4r] "v"(t4r),
                   [lwo] "v"(lwo));
  }
  if (STAMP) {
    __builtin_amdgcn_s_waitcnt(0);
    const u64 c1 = __builtin_amdgcn_s_memtime();
    const u64 r1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0) {  // vector stores only
      stamps[4 * poly + 0] = c0;
      stamps[4 * poly + 1] = c1;
      stamps[4 * poly + 2] = r0;
      stamps[4 * poly + 3] = r1;
    }
  }
}

__global__ void empty_kernel(u64* d) {
  if (d == nullptr) d[0] = 0;
}

__global__ void fill(u64* d, size_t n, u64 seed) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    u64 x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    d[i] = x % 0xFFFFFFFF00000001ull;
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <bool FWD>
static int run(const char* name, u64* data, u64* twist, u64* stamps, uint32_t batch, hipStream_t s) {
  const unsigned grid = (batch + 3) / 4;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // >= 2 s of back-to-back launches so the clock settles (DVFS)
  for (int it = 0; it < 30000; ++it)
    hipLaunchKernelGGL((probe_kernel<FWD, false>), dim3(grid), dim3(256), 0, s, data, batch, twist, stamps);
  CK(hipEventRecord(e0, s));
  const int K = 200;
  for (int it = 0; it < K; ++it)
    hipLaunchKernelGGL((probe_kernel<FWD, false>), dim3(grid), dim3(256), 0, s, data, batch, twist, stamps);
  CK(hipEventRecord(e1, s));
  for (int it = 0; it < 50; ++it)  // stamped launches, the last one is read
    hipLaunchKernelGGL((probe_kernel<FWD, true>), dim3(grid), dim3(256), 0, s, data, batch, twist, stamps);
  CK(hipStreamSynchronize(s));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<u64> h((size_t)4 * batch);
  CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
  std::vector<double> clk, life;
  u64 cmin = ~0ull, cmax = 0, rmin = ~0ull, rmax = 0;
  for (uint32_t p = 0; p < batch; ++p) {
    const u64 c0 = h[4 * p], c1 = h[4 * p + 1], r0 = h[4 * p + 2], r1 = h[4 * p + 3];
    if (r1 > r0 + 20) clk.push_back((double)(c1 - c0) / (double)(r1 - r0) * 100.0);  // MHz
    life.push_back((double)(c1 - c0));
    cmin = std::min(cmin, c0), cmax = std::max(cmax, c1), rmin = std::min(rmin, r0), rmax = std::max(rmax, r1);
  }
  std::sort(clk.begin(), clk.end());
  std::sort(life.begin(), life.end());
  printf("{\"kernel\": \"%s\", \"us_per_launch\": %.2f, \"clock_mhz_median\": %.0f, \"clock_mhz_launch\": %.0f, "
         "\"wave_life_cycles_median\": %.0f, \"wave_life_cycles_p10\": %.0f, \"wave_life_cycles_p90\": %.0f, "
         "\"launch_span_us\": %.2f}\n",
         name, ms * 1000.0 / K, clk.empty() ? 0.0 : clk[clk.size() / 2],
         (double)(cmax - cmin) / (double)(rmax - rmin) * 100.0, life[life.size() / 2], life[life.size() / 10],
         life[life.size() * 9 / 10], (double)(rmax - rmin) / 100.0);
  return 0;
}

int main(int argc, char** argv) {
  const uint32_t batch = argc > 1 ? (uint32_t)atoi(argv[1]) : 8192;
  u64 *data, *twist, *stamps;
  CK(hipMalloc(&data, (size_t)batch * 2048 * 8));
  CK(hipMalloc(&twist, 8192 * 8));
  CK(hipMalloc(&stamps, (size_t)batch * 4 * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3((batch * 2048 + 255) / 256), dim3(256), 0, s, data, (size_t)batch * 2048, 7ull);
  hipLaunchKernelGGL(fill, dim3(32), dim3(256), 0, s, twist, (size_t)8192, 11ull);
  {  // dependent back-to-back launch cost of an empty kernel on this stream
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 1000; ++it) hipLaunchKernelGGL(empty_kernel, dim3(2048), dim3(256), 0, s, stamps);
    CK(hipEventRecord(e0, s));
    for (int it = 0; it < 5000; ++it) hipLaunchKernelGGL(empty_kernel, dim3(2048), dim3(256), 0, s, stamps);
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"empty_kernel_us_per_launch\": %.2f, \"batch\": %u}\n", ms * 1000.0 / 5000, batch);
  }
  if (run<true>("fwd", data, twist, stamps, batch, s)) return 1;
  if (run<false>("inv", data, twist, stamps, batch, s)) return 1;
  return 0;
}
