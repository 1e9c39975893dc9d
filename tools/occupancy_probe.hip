// occupancy_probe.hip — diagnostic (not part of the library): is the twisted N = 2048 transform bound by issue or by
// latency at its 4 waves per SIMD?  The library's own forward / inverse bodies (csrc/ntt64_tw_body.hpp, the wrapper of
// ntt64_tw.hip) run with extra dynamic LDS per workgroup so that fewer workgroups fit a CU: 4, 3, 2 and 1 resident
// waves per SIMD.  A latency-bound kernel slows down in proportion as waves are taken away; an issue-bound one keeps
// its time until too few waves remain to cover the dependency chains.  Times are interleaved in rotated rounds.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I tfhe-rs-main_modified_amd/csrc tools/occupancy_probe.hip \
//         -o tools/occupancy_probe && tools/occupancy_probe [batch] [warm-up launches] [launches per round] [rounds]
// (short settings for a PMC pass: tools/occupancy_probe 8192 200 4 1; the dynamic LDS size tells the residency apart)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "ntt64_tw_body.hpp"

using u64 = uint64_t;
static constexpr int WAVE_LDS2 = 1088;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// W waves per workgroup; dynamic LDS pads the workgroup to throttle residency
template <bool FWD, int W>
__global__ __launch_bounds__(64 * W) void body_kernel(u64* __restrict__ data, uint32_t batch,
                                                      const u64* __restrict__ twist) {
  __shared__ u64 lds[W * WAVE_LDS2];
  extern __shared__ u64 pad[];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = W == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t poly = blockIdx.x * W + wv;
  if (poly >= batch) return;
  if (lane == 64) pad[0] = 0;  // never true: keeps the dynamic allocation referenced
  u64* p = data + (uint64_t)poly * 2048;
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8;
  const uint32_t t1w = S + (lane & 31) * 8;
  const uint32_t t1r = S + (i * 34 + par) * 8;
  const uint32_t lwo = par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = FWD ? twist + 2048 : twist + 2 * (2048 + 32);
  if constexpr (FWD) {
    const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8;
    const uint32_t t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
    const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
    MI_TW_BODY_FWD([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r), [t2wl] "v"(t2wl), [t2wh] "v"(t2wh),
                   [t2r] "v"(t2r), [lwo] "v"(lwo));
  } else {
    const uint32_t t4w = S + ((i & 15) * 66 + par) * 8;
    const uint32_t t1x = S + (lane + (lane >> 5)) * 8;
    const uint32_t t1y = S + ((i & 15) * 66 + 33 * par) * 8;
    MI_TW_BODY_INV([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t4w] "v"(t4w), [t1x] "v"(t1x), [t1y] "v"(t1y), [lwo] "v"(lwo));
  }
}

__global__ void fill(u64* d, size_t n, u64 seed) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) d[i] = ((i + 1) * 0x9E3779B97F4A7C15ull ^ seed) % 0xFFFFFFFF00000001ull;
}

// residency target (waves per SIMD) -> dynamic LDS bytes per workgroup, for the forward's 1-wave and the inverse's
// 4-wave workgroups (160 KiB of LDS per CU, 4 SIMDs)
static size_t pad_for(int waves_per_simd, int W) {
  if (waves_per_simd >= 4) return 0;
  const double wgs = 4.0 * waves_per_simd / W;              // workgroups per CU wanted
  const double target = 160.0 * 1024 / (wgs + 0.5);          // wgs fit, wgs + 1 do not
  const double stat = (double)W * WAVE_LDS2 * 8;
  const size_t pad = (size_t)std::max(0.0, target - stat);
  return (pad + 511) / 512 * 512;
}

int main(int argc, char** argv) {
  const uint32_t batch = argc > 1 ? (uint32_t)atoi(argv[1]) : 8192;
  const size_t n = (size_t)batch * 2048;
  u64 *data, *twist;
  CK(hipMalloc(&data, n * 8));
  CK(hipMalloc(&twist, 8192 * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(fill, dim3(32), dim3(256), 0, s, twist, (size_t)8192, 11ull);
  hipLaunchKernelGGL(fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, data, n, 7ull);
  // both directions with one-wave workgroups here (the library's inverse uses four: 2.4 % faster at full residency),
  // so every residency target is reachable under the 64 KiB per-workgroup LDS limit
  CK(hipFuncSetAttribute((const void*)body_kernel<true, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 56 * 1024));
  CK(hipFuncSetAttribute((const void*)body_kernel<false, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 56 * 1024));
  const int occ[] = {4, 3, 2, 1};
  auto run = [&](bool fwd, int o) {
    if (fwd)
      hipLaunchKernelGGL((body_kernel<true, 1>), dim3(batch), dim3(64), pad_for(o, 1), s, data, batch, twist);
    else
      hipLaunchKernelGGL((body_kernel<false, 1>), dim3(batch), dim3(64), pad_for(o, 1), s, data, batch, twist);
  };
  const int warm = argc > 2 ? atoi(argv[2]) : 20000;
  for (int it = 0; it < warm; ++it) run(it & 1, 4);  // the clock settles under load
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int K = argc > 3 ? atoi(argv[3]) : 200, R = argc > 4 ? atoi(argv[4]) : 9;
  std::vector<double> t[2][4];
  for (int r = 0; r < R; ++r)
    for (int oi = 0; oi < 4; ++oi)
      for (int d = 0; d < 2; ++d) {
        const int o = occ[(oi + r) % 4];
        CK(hipEventRecord(e0, s));
        for (int it = 0; it < K; ++it) run(d == 0, o);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[d][4 - o].push_back(ms * 1000.0 / K);
      }
  CK(hipGetLastError());
  for (int o = 4; o >= 1; --o) {
    auto& f = t[0][4 - o];
    auto& v = t[1][4 - o];
    std::sort(f.begin(), f.end());
    std::sort(v.begin(), v.end());
    printf("{\"waves_per_simd\": %d, \"pad_fwd_B\": %zu, \"pad_inv_B\": %zu, \"fwd_us_median\": %.2f, "
           "\"inv_us_median\": %.2f}\n", o, pad_for(o, 1), pad_for(o, 1), f[R / 2], v[R / 2]);
  }
  return 0;
}
