// tw_debug.hip — dumps the twisted-transform registers after each phase (debug aid for
// tools/gen_tw_kernel.py).  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I tools
//   -I tfhe-rs-main_modified_amd/csrc tools/tw_debug.hip -o tools/tw_debug ; run: tools/tw_debug out.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "tw_dbg_body.hpp"

typedef uint64_t u64;
static constexpr int WAVE_LDS2 = 1088;

template <int STOP>
__global__ __launch_bounds__(256, 4) void kdbg(u64* data, const u64* twist) {
  __shared__ u64 lds[4 * WAVE_LDS2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  u64* p = data + (uint64_t)(blockIdx.x * 4 + wv) * 2048;
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8, t1w = S + (lane & 31) * 8, t1r = S + (i * 34 + par) * 8, lwo = par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2048;
  const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8, t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
  const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
#define ARGS [g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw), [l8] "v"(l8), \
             [t1w] "v"(t1w), [t1r] "v"(t1r), [t2wl] "v"(t2wl), [t2wh] "v"(t2wh), [t2r] "v"(t2r), [lwo] "v"(lwo)
  if (STOP == 0) MI_TW_BODY_FWD_G1(ARGS);
  if (STOP == 1) MI_TW_BODY_FWD_TWIST(ARGS);
  if (STOP == 2) MI_TW_BODY_FWD_T1(ARGS);
  if (STOP == 3) MI_TW_BODY_FWD_CYC(ARGS);
  if (STOP == 4) MI_TW_BODY_FWD_LAST(ARGS);
}

int main(int argc, char** argv) {
  const char* in = argc > 1 ? argv[1] : "gpurun_out/twdbg_in.bin";
  const char* out = argc > 2 ? argv[2] : "gpurun_out/twdbg_out.bin";
  std::vector<u64> h(4 * 2048 + 2080);
  FILE* f = fopen(in, "rb");
  if (!f || fread(h.data(), 8, h.size(), f) != h.size()) { printf("bad input\n"); return 1; }
  fclose(f);
  u64 *d, *tw;
  hipMalloc(&d, 4 * 2048 * 8);
  hipMalloc(&tw, 2080 * 8);
  hipMemcpy(tw, h.data() + 4 * 2048, 2080 * 8, hipMemcpyHostToDevice);
  std::vector<u64> res(5 * 4 * 2048);
  void (*ks[5])(u64*, const u64*) = {kdbg<0>, kdbg<1>, kdbg<2>, kdbg<3>, kdbg<4>};
  for (int s = 0; s < 5; ++s) {
    hipMemcpy(d, h.data(), 4 * 2048 * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[s], dim3(1), dim3(256), 0, 0, d, tw);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel %d failed\n", s); return 1; }
    hipMemcpy(res.data() + s * 4 * 2048, d, 4 * 2048 * 8, hipMemcpyDeviceToHost);
  }
  f = fopen(out, "wb");
  fwrite(res.data(), 8, res.size(), f);
  fclose(f);
  printf("ok\n");
  return 0;
}
