// select_probe.hip — diagnostic (not part of the library): what the compiler's Goldilocks arithmetic costs per operation
// on gfx950, against the same operations with the selects forced into the VOP3 form.  tools/valu_probe.hip measured a
// VOP2 v_cndmask_b32 (implicit VCC) at ~23 cycles per wave-instruction against 4.35 for the VOP3 form; hipcc emits the
// VOP2 form for most `c ? a : b` on 64-bit values (mi_arith.hpp's Goldilocks add / sub / reduce128).  Each kernel runs
// 8 independent chains of one operation per lane at 8 waves per SIMD; output: cycles per operation per wave.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I tfhe-rs-main_modified_amd/csrc tools/select_probe.hip \
//         -o tools/select_probe && tools/select_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "mi_arith.hpp"

using mi::Goldilocks;
using u64 = uint64_t;

#define ITERS 1024

// Goldilocks add with VOP3 carries and selects: s = a + b; U = s + EPS; result = (carry(s) | carry(U)) ? U : s
__device__ __forceinline__ u64 add_vop3(u64 a, u64 b) {
  uint32_t sl, sh, ul, uh, rl, rh;
  uint64_t c0, c1;
  asm volatile(
      "v_add_co_u32_e64 %0, %6, %8, %10\n\t"
      "v_addc_co_u32_e64 %1, %6, %9, %11, %6\n\t"
      "v_add_co_u32_e64 %2, %7, %0, -1\n\t"
      "v_addc_co_u32_e64 %3, %7, %1, 0, %7\n\t"
      "s_or_b64 %7, %7, %6\n\t"
      "v_cndmask_b32_e64 %4, %0, %2, %7\n\t"
      "v_cndmask_b32_e64 %5, %1, %3, %7"
      : "=&v"(sl), "=&v"(sh), "=&v"(ul), "=&v"(uh), "=&v"(rl), "=&v"(rh), "=&s"(c0), "=&s"(c1)
      : "v"((uint32_t)a), "v"((uint32_t)(a >> 32)), "v"((uint32_t)b), "v"((uint32_t)(b >> 32)));
  return ((u64)rh << 32) | rl;
}

#define CHAINS(OP)                                                                          \
  __global__ __launch_bounds__(256) void k_##OP(u64* out, u64 s0, u64 s1, uint64_t* clk) { \
    u64 x[8];                                                                               \
    const u64 y = (s1 ^ threadIdx.x) % Goldilocks::P;                                       \
    for (int i = 0; i < 8; ++i) x[i] = (s0 + threadIdx.x * 8 + i) % Goldilocks::P;          \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                       \
    for (int it = 0; it < ITERS; ++it) {                                                    \
      _Pragma("unroll") for (int i = 0; i < 8; ++i) x[i] = OP(x[i], y);                     \
    }                                                                                       \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                       \
    u64 acc = 0;                                                                            \
    for (int i = 0; i < 8; ++i) acc ^= x[i];                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;                                       \
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                        \
  }

__device__ __forceinline__ u64 gadd(u64 a, u64 b) { return Goldilocks::add(a, b); }
__device__ __forceinline__ u64 gsub(u64 a, u64 b) { return Goldilocks::sub(a, b); }
__device__ __forceinline__ u64 gmul(u64 a, u64 b) { return Goldilocks::mul(a, b); }
CHAINS(gadd)
CHAINS(gsub)
CHAINS(gmul)
CHAINS(add_vop3)

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount, blocks = cus * 8;
  u64* out;
  uint64_t *clk, h[4096];
  (void)hipMalloc(&out, (size_t)blocks * 256 * 8);
  (void)hipMalloc(&clk, (size_t)blocks * 8);
  struct K {
    const char* name;
    void (*f)(u64*, u64, u64, uint64_t*);
  } ks[] = {{"Goldilocks::add (compiler)", k_gadd}, {"Goldilocks::sub (compiler)", k_gsub},
            {"Goldilocks::mul (compiler)", k_gmul}, {"add, VOP3 selects (asm)", k_add_vop3}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (auto& k : ks) {
    float best = 1e30f;
    double cyc = 0;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3, 5, clk);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) {
        best = ms;
        (void)hipMemcpy(h, clk, (size_t)blocks * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; ++i) s += (double)h[i];
        cyc = s / blocks * 100.0 / 8;  // s_memtime is 100 MHz here? reported for reference only
      }
    }
    // per SIMD: blocks * 4 waves / (cus * 4 SIMDs) waves, each ITERS * 8 ops; time -> cycles at the measured clock
    const double ops_per_simd = (double)blocks * 4 / (cus * 4.0) * ITERS * 8;
    printf("%-30s %7.3f ms  %6.2f ns per op per SIMD  (%.2f cycles at 2.4 GHz)\n", k.name, best,
           best * 1e6 / ops_per_simd, best * 1e6 / ops_per_simd * 2.4);
    (void)cyc;
  }
  return 0;
}
