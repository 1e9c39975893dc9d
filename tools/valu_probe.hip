// valu_probe.hip — issue cost of the integer VALU instructions a Goldilocks butterfly is built
// from, on gfx950.  Each kernel runs ITERS x 8 independent instructions per lane at 8 waves per
// SIMD; carry/mask operands come from SGPRs written once before the loop (no hazard padding in the
// loop: checked in the .s).  Output: cycles per wave-instruction per SIMD at the in-kernel clock.
//
// Build+run:  hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o tools/valu_probe && tools/valu_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 2048

#define BODY8(INS) INS(a0, 0) INS(a1, 1) INS(a2, 2) INS(a3, 3) INS(a4, 4) INS(a5, 5) INS(a6, 6) INS(a7, 7)

#define KERNEL(NAME, T, INS)                                                                   \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t s0, uint32_t s1, uint64_t* clk) { \
    T a0 = s0 + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    uint32_t b = s1 ^ threadIdx.x, c = s0 + 77;                                              \
    uint64_t m0, m1;                                                                         \
    asm volatile("s_mov_b64 %0, exec\n\ts_mov_b64 %1, 0" : "=s"(m0), "=s"(m1));              \
    asm volatile("v_cmp_gt_u32_e32 vcc, 17, %0\n\ts_nop 7\n\ts_nop 7" :: "v"(b) : "memory", "vcc");     \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();                                          \
    for (int i = 0; i < ITERS; ++i) { BODY8(INS) }                                           \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();                                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; } \
  }

// 32-bit simple
#define I_ADD(x, k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_XOR(x, k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_MOV(x, k) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(b));
#define I_ADD3(x, k) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define I_ALIGN(x, k) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b));
// carries (VOP3 with explicit sdst / carry-in SGPR pairs)
#define I_ADDCO3(x, k) { uint64_t o; asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(x), "=s"(o) : "v"(b)); }
#define I_ADDC3(x, k) { uint64_t o; asm volatile("v_addc_co_u32 %0, %1, %0, %2, %3" : "+v"(x), "=s"(o) : "v"(b), "s"(m1)); }
#define I_SUBB3(x, k) { uint64_t o; asm volatile("v_subb_co_u32 %0, %1, %0, %2, %3" : "+v"(x), "=s"(o) : "v"(b), "s"(m1)); }
#define I_CND64(x, k) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "s"(m0));
#define I_CNDK(x, k) asm volatile("v_cndmask_b32 %0, 0, -1, %1" : "=v"(x) : "s"(m0));
// 64-bit
#define I_MAD(x, k) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(x), "=s"(cc) : "v"(b), "v"(c)); }
#define I_MAD0(x, k) { uint64_t cc; asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(x), "=s"(cc) : "v"(b), "v"(c)); }
#define I_LSHLADD64(x, k) asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(x));
#define I_CMP64(x, k) { uint64_t m; asm volatile("v_cmp_lt_u64 %0, %1, %2" : "=s"(m) : "v"(x), "v"(a0)); }
#define I_MOV64(x, k) asm volatile("v_mov_b64 %0, %0" : "+v"(x));
#define I_MULHI(x, k) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
// VOP2 forms with VCC (e32)
#define I_ADDCO32(x, k) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
#define I_CND32(x, k) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
#define I_SUBB32(x, k) asm volatile("v_subb_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
#define I_CND32B(x, k) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
#define I_CND64VCC(x, k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
#define I_SUBU32(x, k) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_LSHR32(x, k) asm volatile("v_lshrrev_b32_e32 %0, 7, %0" : "+v"(x));
#define I_LSHR64(x, k) asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(x));
#define I_NOT32(x, k) asm volatile("v_not_b32_e32 %0, %0" : "+v"(x));
#define I_MUL24(x, k) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_MULHI24(x, k) asm volatile("v_mul_hi_u32_u24_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_MULLO(x, k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define I_BFI(x, k) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define I_PERM(x, k) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define I_NOP0(x, k) asm volatile("s_nop 0");
#define I_NOP1(x, k) asm volatile("s_nop 1");
#define I_ADDPAIR(x, k) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1\n s_nop 1\n v_addc_co_u32_e32 %0, vcc, 0, %0, vcc" : "+v"(x) : "v"(b) : "vcc");
#define I_ADDPAIR_NONOP(x, k) asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1\n v_addc_co_u32_e32 %0, vcc, 0, %0, vcc" : "+v"(x) : "v"(b) : "vcc");

// cross-lane moves (pair stages): gfx950 half-swaps and a DPP quad_perm move
#define I_PL32(x, k) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(c));
#define I_PL16(x, k) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(c));
#define I_DPPQ(x, k) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(x) : "v"(b));
#define I_LSHL64(x, k) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(x));
#define I_MADI64(x, k) { uint64_t cc; asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(x), "=s"(cc) : "v"(b), "v"(c)); }

// f64 (FFT PBS path)
#define I_FADD(x, k) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(fb));
#define I_FMUL(x, k) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(fb));
#define I_FFMA(x, k) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x) : "v"(fb), "v"(fc));
#define I_FFMAC(x, k) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(x) : "v"(fb), "v"(fc));
#define I_FRND(x, k) asm volatile("v_rndne_f64 %0, %0" : "+v"(x));
#define I_FCVT(x, k) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(x) : "v"(b));
#define I_FPKFMA(x, k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(fb), "v"(fc));
#define FKERNEL(NAME, INS)                                                                   \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t s0, uint32_t s1, uint64_t* clk) { \
    double a0 = s0 + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    double fb = 1.0000001 * s1, fc = 0.5 * s0;                                               \
    uint32_t b = s1 ^ threadIdx.x;                                                           \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();                                          \
    for (int i = 0; i < ITERS; ++i) { BODY8(INS) }                                           \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();                                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7); \
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; } \
  }
FKERNEL(k_fadd, I_FADD)
FKERNEL(k_fmul, I_FMUL)
FKERNEL(k_ffma, I_FFMA)
FKERNEL(k_ffmac, I_FFMAC)
FKERNEL(k_frnd, I_FRND)
FKERNEL(k_fcvt, I_FCVT)
FKERNEL(k_fpkfma, I_FPKFMA)

KERNEL(k_add, uint32_t, I_ADD)
KERNEL(k_xor, uint32_t, I_XOR)
KERNEL(k_mov, uint32_t, I_MOV)
KERNEL(k_add3, uint32_t, I_ADD3)
KERNEL(k_align, uint32_t, I_ALIGN)
KERNEL(k_addco3, uint32_t, I_ADDCO3)
KERNEL(k_addc3, uint32_t, I_ADDC3)
KERNEL(k_subb3, uint32_t, I_SUBB3)
KERNEL(k_cnd64, uint32_t, I_CND64)
KERNEL(k_cndk, uint32_t, I_CNDK)
KERNEL(k_mad, uint64_t, I_MAD)
KERNEL(k_mad0, uint64_t, I_MAD0)
KERNEL(k_lshladd64, uint64_t, I_LSHLADD64)
KERNEL(k_cmp64, uint64_t, I_CMP64)
KERNEL(k_mov64, uint64_t, I_MOV64)
KERNEL(k_mulhi, uint32_t, I_MULHI)
KERNEL(k_addco32, uint32_t, I_ADDCO32)
KERNEL(k_cnd32, uint32_t, I_CND32)
KERNEL(k_subb32, uint32_t, I_SUBB32)
KERNEL(k_nop0, uint32_t, I_NOP0)
KERNEL(k_cnd32b, uint32_t, I_CND32B)
KERNEL(k_cnd64vcc, uint32_t, I_CND64VCC)
KERNEL(k_subu32, uint32_t, I_SUBU32)
KERNEL(k_lshr32, uint32_t, I_LSHR32)
KERNEL(k_lshr64, uint64_t, I_LSHR64)
KERNEL(k_not32, uint32_t, I_NOT32)
KERNEL(k_mul24, uint32_t, I_MUL24)
KERNEL(k_mulhi24, uint32_t, I_MULHI24)
KERNEL(k_mullo, uint32_t, I_MULLO)
KERNEL(k_bfi, uint32_t, I_BFI)
KERNEL(k_perm, uint32_t, I_PERM)
KERNEL(k_nop1, uint32_t, I_NOP1)
KERNEL(k_addpair, uint32_t, I_ADDPAIR)
KERNEL(k_addpair_nonop, uint32_t, I_ADDPAIR_NONOP)
KERNEL(k_pl32, uint32_t, I_PL32)
KERNEL(k_pl16, uint32_t, I_PL16)
KERNEL(k_dppq, uint32_t, I_DPPQ)
KERNEL(k_lshl64, uint64_t, I_LSHL64)
KERNEL(k_madi64, uint64_t, I_MADI64)

// VCC written by the SALU once before the loop (s_mov_b64 vcc, exec): the VOP2 select, and the same select with a DPP
// partner-lane source (quad_perm [1,0,3,2]: one instruction for the lane-pair regroup's move + select)
#define KERNEL_SVCC(NAME, T, INS)                                                              \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t s0, uint32_t s1, uint64_t* clk) { \
    T a0 = s0 + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
    uint32_t b = s1 ^ threadIdx.x;                                                           \
    uint64_t m0;                                                                             \
    asm volatile("s_mov_b64 %0, exec" : "=s"(m0));                                           \
    asm volatile("s_mov_b64 vcc, %0\n\ts_nop 7\n\ts_nop 7" :: "s"(m0) : "memory", "vcc");    \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();                                          \
    for (int i = 0; i < ITERS; ++i) { BODY8(INS) }                                           \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();                                          \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
    if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; } \
  }
#define I_CND32S(x, k) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x) : "v"(b));
#define I_CNDDPP(x, k) asm volatile("v_cndmask_b32_dpp %0, %1, %0, vcc quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" \
                                    : "+v"(x) : "v"(b));
#define I_ADDDPP(x, k) asm volatile("v_add_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" \
                                    : "+v"(x) : "v"(b));
KERNEL_SVCC(k_cnd32s, uint32_t, I_CND32S)
KERNEL_SVCC(k_cnddpp, uint32_t, I_CNDDPP)
KERNEL_SVCC(k_adddpp, uint32_t, I_ADDDPP)

typedef void (*kfn)(uint64_t*, uint32_t, uint32_t, uint64_t*);

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  struct { const char* name; kfn f; } ks[] = {
      {"v_add_u32", k_add},          {"v_xor_b32", k_xor},           {"v_mov_b32", k_mov},
      {"v_add3_u32", k_add3},        {"v_alignbit_b32", k_align},    {"v_add_co_u32(e64)", k_addco3},
      {"v_addc_co_u32(e64)", k_addc3}, {"v_subb_co_u32(e64)", k_subb3}, {"v_cndmask(sgpr)", k_cnd64},
      {"v_cndmask(0,-1,s)", k_cndk}, {"v_mad_u64_u32", k_mad},       {"v_mad_u64_u32(+0)", k_mad0},
      {"v_lshl_add_u64", k_lshladd64}, {"v_cmp_lt_u64", k_cmp64},    {"v_mov_b64", k_mov64},
      {"v_mul_hi_u32", k_mulhi},
      {"v_add_co_u32_e32(vcc)", k_addco32}, {"v_cndmask_e32(vcc)", k_cnd32}, {"v_subb_co_e32 chain", k_subb32},
      {"s_nop 0", k_nop0}, {"v_cndmask_e32(vcc valu-set)", k_cnd32b}, {"v_cndmask_e64(vcc)", k_cnd64vcc},
      {"v_sub_u32_e32", k_subu32}, {"v_lshrrev_b32_e32", k_lshr32}, {"v_lshrrev_b64", k_lshr64}, {"v_not_b32", k_not32},
      {"v_mul_u32_u24_e32", k_mul24}, {"v_mul_hi_u32_u24_e32", k_mulhi24}, {"v_mul_lo_u32", k_mullo}, {"v_bfi_b32", k_bfi},
      {"v_perm_b32", k_perm}, {"s_nop 1", k_nop1}, {"addco+nop1+addc (3 ins)", k_addpair}, {"addco+addc no nop", k_addpair_nonop},
      {"v_add_f64", k_fadd}, {"v_mul_f64", k_fmul}, {"v_fma_f64", k_ffma}, {"v_fmac_f64_e32", k_ffmac},
      {"v_rndne_f64", k_frnd}, {"v_cvt_f64_i32", k_fcvt}, {"v_pk_fma_f32", k_fpkfma},
      {"v_permlane32_swap_b32", k_pl32}, {"v_permlane16_swap_b32", k_pl16}, {"v_mov_b32_dpp quad_perm", k_dppq},
      {"v_lshlrev_b64", k_lshl64}, {"v_mad_i64_i32", k_madi64},
      {"v_cndmask_e32(vcc salu-set)", k_cnd32s}, {"v_cndmask_b32_dpp(vcc salu-set)", k_cnddpp},
      {"v_add_u32_dpp quad_perm", k_adddpp},
  };
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const int blocks = cus * (argc > 1 ? atoi(argv[1]) : 8);
  uint64_t *out, *clk;
  (void)hipMalloc(&out, (size_t)blocks * 256 * 8);
  (void)hipMalloc(&clk, (size_t)blocks * 16);
  uint64_t* h = (uint64_t*)malloc((size_t)blocks * 16);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("CUs=%d\n", cus);
  for (auto& k : ks) {
    float best = 1e30f;
    double ghz = 0;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 3, 5, clk);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) {
        best = ms;
        (void)hipMemcpy(h, clk, (size_t)blocks * 16, hipMemcpyDeviceToHost);
        double sc = 0, sr = 0;
        for (int i = 0; i < blocks; ++i) { sc += h[2 * i]; sr += h[2 * i + 1]; }
        ghz = (sc / sr) * 0.1;
      }
    }
    const double wave_instr = (double)blocks * 4 * ITERS * 8;
    const double cyc = best * 1e-3 * ghz * 1e9;
    printf("%-22s %7.3f ms  clk %.2f GHz  %5.2f cycles/wave-instr/SIMD\n", k.name, best, ghz,
           cyc / (wave_instr / (cus * 4.0)));
  }
  return 0;
}
