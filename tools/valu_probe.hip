// valu_probe.hip — measures the issue cost of the 32/64-bit integer VALU instructions the
// Goldilocks butterfly is built from (gfx950).  Each kernel runs ITERS x 8 independent
// instructions per lane (no dependency stalls) at full occupancy; the host converts the wall time
// into cycles per wave-instruction per SIMD using the in-kernel clock (s_memtime / s_memrealtime).
//
// Build+run:  hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o /tmp/valu_probe && /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 4096

#define BODY8(INS)                                                                   \
  INS(a0) INS(a1) INS(a2) INS(a3) INS(a4) INS(a5) INS(a6) INS(a7)

#define KERNEL(NAME, DECL, INS, SINK)                                                 \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t s0, uint32_t s1, uint64_t* clk) { \
    DECL;                                                                             \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                       \
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();                                   \
    for (int i = 0; i < ITERS; ++i) { BODY8(INS) }                                    \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                       \
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();                                   \
    out[blockIdx.x * blockDim.x + threadIdx.x] = SINK;                                \
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; } \
  }

#define D64 uint64_t a0 = s0 + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; uint32_t b = s1 ^ threadIdx.x, c = s0 + 77
#define D32 uint32_t a0 = s0 + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; uint32_t b = s1 ^ threadIdx.x, c = s0 + 77
#define SINK (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7)

#define I_MAD(x) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x), "=s"(cc) : "v"(b), "v"(c)); }
#define I_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_ADD32(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_ADDCO(x) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
#define I_LSHLADD64(x) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(x));
#define I_LSHL64(x) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(x));
#define I_CMP64(x) { uint64_t m; asm volatile("v_cmp_lt_u64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(a0)); }
#define I_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define I_MAD32(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define I_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define I_FMA64(x) asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(x));

KERNEL(k_mad64, D64, I_MAD, SINK)
KERNEL(k_mullo, D32, I_MULLO, SINK)
KERNEL(k_mulhi, D32, I_MULHI, SINK)
KERNEL(k_add32, D32, I_ADD32, SINK)
KERNEL(k_addco, D32, I_ADDCO, SINK)
KERNEL(k_lshladd64, D64, I_LSHLADD64, SINK)
KERNEL(k_lshl64, D64, I_LSHL64, SINK)
KERNEL(k_cmp64, D64, I_CMP64, SINK)
KERNEL(k_cnd, D32, I_CND, SINK)
KERNEL(k_mad24, D32, I_MAD32, SINK)
KERNEL(k_add3, D32, I_ADD3, SINK)
KERNEL(k_fma64, D64, I_FMA64, SINK)

typedef void (*kfn)(uint64_t*, uint32_t, uint32_t, uint64_t*);

int main() {
  struct { const char* name; kfn f; } ks[] = {
      {"v_mad_u64_u32", k_mad64}, {"v_mul_lo_u32", k_mullo}, {"v_mul_hi_u32", k_mulhi},
      {"v_add_u32", k_add32},     {"v_add_co_u32", k_addco}, {"v_lshl_add_u64", k_lshladd64},
      {"v_lshlrev_b64", k_lshl64}, {"v_cmp_lt_u64", k_cmp64}, {"v_cndmask_b32", k_cnd},
      {"v_mad_u32_u24", k_mad24}, {"v_add3_u32", k_add3},     {"v_fma_f64", k_fma64},
  };
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * 8;  // 8 x 256-thread blocks per CU = 8 waves per SIMD
  uint64_t *out, *clk;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  hipMalloc(&clk, (size_t)blocks * 16);
  uint64_t* h = (uint64_t*)malloc((size_t)blocks * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("CUs=%d\n", cus);
  for (auto& k : ks) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3, 5, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost);
    double sc = 0, sr = 0;
    for (int i = 0; i < blocks; ++i) { sc += h[2 * i]; sr += h[2 * i + 1]; }
    const double ghz = (sc / sr) * 0.1;  // memrealtime = 100 MHz
    const double wave_instr = (double)blocks * 4 * ITERS * 8;  // 4 waves per block
    const double cyc = ms * 1e-3 * ghz * 1e9;                  // kernel cycles at the in-kernel clock
    // per SIMD: cycles / (wave-instructions per SIMD)
    const double per_simd = cyc / (wave_instr / (cus * 4.0));
    printf("%-16s %8.3f ms  clk %.2f GHz  %.2f cycles per wave-instr per SIMD\n", k.name, ms, ghz, per_simd);
  }
  return 0;
}
