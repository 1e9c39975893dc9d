// pbs_tw.hip — programmable bootstrap, BNF flavour, decomposition level 1, on the twisted N = 2048
// Goldilocks transform (reference: tfhe/src/core_crypto/algorithms/lwe_programmable_bootstrapping/
// ntt64_bnf_pbs.rs:208-726, programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized).
//
// MI355X design: one 128-lane workgroup (2 waves) per LWE ciphertext.  Each wave keeps one GLWE
// polynomial of the accumulator in VGPRs (v128..v191) for the whole blind rotation and runs the
// complete CMUX step — rotation, decomposition, forward transform, GGSW multiply-accumulate (the
// partner's transformed polynomial comes through LDS), inverse transform, exact prime -> 2^64
// modulus switch — as one generated asm body (tools/gen_pbs_kernel.py -> pbs_tw_body.hpp).  256
// VGPRs and 32 KiB of LDS per workgroup: 2 waves per SIMD.  This wrapper computes the centered body
// correction (if asked) before the loop and does the final rotation by -ms(b) + sample extraction.
// Bit-exactness: the same restatement as pbs_kernels.hip (N^-1 folded into the key copy).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "pbs_tw_body.hpp"

namespace mi {
namespace pbstw {

static constexpr int N = 2048;
static constexpr unsigned LOG_MOD = 12;  // PolynomialSize::to_blind_rotation_input_modulus_log

__device__ __forceinline__ u64 modulus_switch(u64 input, unsigned log_modulus) {  // fft_impl/common.rs:10-23
  return (input + (1ull << (64u - log_modulus - 1u))) >> (64u - log_modulus);
}

// algorithms/modulus_switch.rs:60-104 centered_binary_ms_body_correction_to_add (128-lane reduction)
__device__ u64 centered_body_correction(const u64* __restrict__ lwe, uint32_t n_lwe, int t, u64* sh) {
  u64 sum_half = 0;
  int64_t sum_hed = 0;
  for (uint32_t i = t; i < n_lwe; i += 128) {
    const u64 a = lwe[i];
    const int64_t err = (int64_t)((modulus_switch(a, LOG_MOD) << (64u - LOG_MOD)) - a);
    const int64_t half = err / 2;  // truncating, as Rust's signed division
    sum_half += (u64)half;
    sum_hed += 2 * half - err;
  }
  sh[t] = sum_half;
  sh[128 + t] = (u64)sum_hed;
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (t < s) {
      sh[t] += sh[t + s];
      sh[128 + t] = (u64)((int64_t)sh[128 + t] + (int64_t)sh[128 + t + s]);
    }
    __syncthreads();
  }
  const u64 total_half = sh[0];
  const int64_t total_hed = (int64_t)sh[128];
  __syncthreads();
  return total_half - (u64)(total_hed / 2) - (1ull << (64u - LOG_MOD - 1u));
}

// The lane-pair twiddles of the forward and inverse transforms (tab[N..N+31], tab[2N+32+..]: the
// same for the plain and the N^-1-folded inverse tables) into LDS, read by the body's pair stage.
__device__ __forceinline__ void load_lane_pair_tables(u64* lwtab, const u64* __restrict__ tab, int t) {
  if (t < 64) lwtab[t] = t < 32 ? tab[N + t] : tab[2 * N + 32 + (t - 32)];
  __syncthreads();
}

// lwe_in: batch x (n+1); lut: 2 x N; bsk: n x 2 x 2 x N (NTT domain, N^-1 folded in);
// tab: [fwd twist (N) | fwd lane-pair twiddles (32) | inverse twist (N) | inverse lane-pair (32) | ...].
__global__ __launch_bounds__(128) void pbs_tw_kernel(u64* __restrict__ lwe_out, const u64* __restrict__ lwe_in,
                                                     const u64* __restrict__ lut, const u64* __restrict__ bsk,
                                                     uint32_t n_lwe, uint32_t batch, int base_log,
                                                     const u64* __restrict__ tab, int centered) {
  __shared__ u64 buf[2 * N];
  __shared__ u64 lwtab[64];
  const int t = threadIdx.x;
  const uint32_t lane = t & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;  // uniform per workgroup
  const u64* lwe = lwe_in + (size_t)b * (n_lwe + 1);
  load_lane_pair_tables(lwtab, tab, t);  // ends with a workgroup barrier
  u64 body_corr = 0;
  if (centered) body_corr = centered_body_correction(lwe, n_lwe, t, buf);

  const uint32_t S = (uint32_t)(uintptr_t)(buf + w * N), SP = (uint32_t)(uintptr_t)(buf + (1 - w) * N);
  const u64* lutw = lut + (size_t)w * N;
  const u64* gown = bsk + (size_t)3 * w * N;
  const u64* gpar = bsk + (size_t)(2 - w) * N;
  const uint32_t lut_lo = (uint32_t)(uintptr_t)lutw, lut_hi = (uint32_t)((uintptr_t)lutw >> 32);
  const uint32_t gown_lo = (uint32_t)(uintptr_t)gown, gown_hi = (uint32_t)((uintptr_t)gown >> 32);
  const uint32_t gpar_lo = (uint32_t)(uintptr_t)gpar, gpar_hi = (uint32_t)((uintptr_t)gpar >> 32);
  const uint32_t lwe_lo = (uint32_t)(uintptr_t)lwe, lwe_hi = (uint32_t)((uintptr_t)lwe >> 32);
  const uint32_t tab_lo = (uint32_t)(uintptr_t)tab, tab_hi = (uint32_t)((uintptr_t)tab >> 32);
  MI_PBS_BODY_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [lut_lo] "s"(lut_lo), [lut_hi] "s"(lut_hi),
                     [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi), [gpar_lo] "s"(gpar_lo),
                     [gpar_hi] "s"(gpar_hi), [lwe_lo] "s"(lwe_lo), [lwe_hi] "s"(lwe_hi), [n] "s"(n_lwe),
                     [tab_lo] "s"(tab_lo), [tab_hi] "s"(tab_hi), [bl] "s"(base_log),
                     [LW] "s"((uint32_t)(uintptr_t)lwtab));
  // buf[w N + e] = acc_w[e].  Final rotation by -ms(b) (ntt64_bnf_pbs.rs:262-270), then sample
  // extraction at nth = 0 (glwe_sample_extraction.rs:89-160): out[0] = A'[0], out[j] = -A'[N - j].
  const u64* acc = buf + w * N;
  const u64 body = modulus_switch(lwe[n_lwe] + body_corr, LOG_MOD);
  const int full = (int)(body / N) & 1, rem = (int)(body % N);
  u64* out = lwe_out + (size_t)b * (N + 1);
  if (w == 0) {
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const int j = 64 * r + (int)lane;
      const int m = (j == 0) ? 0 : N - j;
      u64 v = acc[(m + rem) & (N - 1)];
      if (full ^ (m >= N - rem)) v = (u64)0 - v;
      out[j] = (j == 0) ? v : (u64)0 - v;
    }
  } else if (lane == 0) {
    u64 v = acc[rem & (N - 1)];
    if (full) v = (u64)0 - v;
    out[N] = v;
  }
}

// external product / CMUX batch (config 3): one workgroup per GLWE pair, wave w on polynomial w
template <bool CMUX>
__global__ __launch_bounds__(128) void ext_tw_kernel(u64* __restrict__ out, u64* __restrict__ glwe,
                                                     const u64* __restrict__ ggsw, uint32_t batch, int base_log,
                                                     const u64* __restrict__ tab) {
  __shared__ u64 buf[2 * N];
  __shared__ u64 lwtab[64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;
  load_lane_pair_tables(lwtab, tab, threadIdx.x);
  const uint32_t S = (uint32_t)(uintptr_t)(buf + w * N), SP = (uint32_t)(uintptr_t)(buf + (1 - w) * N);
  u64* o = out + ((size_t)b * 2 + w) * N;
  u64* g = glwe + ((size_t)b * 2 + w) * N;
  const u64* gown = ggsw + (size_t)3 * w * N;
  const u64* gpar = ggsw + (size_t)(2 - w) * N;
  const uint32_t o_lo = (uint32_t)(uintptr_t)o, o_hi = (uint32_t)((uintptr_t)o >> 32);
  const uint32_t g_lo = (uint32_t)(uintptr_t)g, g_hi = (uint32_t)((uintptr_t)g >> 32);
  const uint32_t gown_lo = (uint32_t)(uintptr_t)gown, gown_hi = (uint32_t)((uintptr_t)gown >> 32);
  const uint32_t gpar_lo = (uint32_t)(uintptr_t)gpar, gpar_hi = (uint32_t)((uintptr_t)gpar >> 32);
  const uint32_t tab_lo = (uint32_t)(uintptr_t)tab, tab_hi = (uint32_t)((uintptr_t)tab >> 32);
  if constexpr (CMUX)
    MI_PBS_BODY_CMUX_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [glwe_lo] "s"(g_lo), [glwe_hi] "s"(g_hi),
                            [out_lo] "s"(o_lo), [out_hi] "s"(o_hi), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                            [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [tab_lo] "s"(tab_lo),
                            [tab_hi] "s"(tab_hi), [bl] "s"(base_log), [LW] "s"((uint32_t)(uintptr_t)lwtab));
  else
    MI_PBS_BODY_EXT_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [glwe_lo] "s"(g_lo), [glwe_hi] "s"(g_hi),
                           [out_lo] "s"(o_lo), [out_hi] "s"(o_hi), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                           [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [tab_lo] "s"(tab_lo),
                           [tab_hi] "s"(tab_hi), [bl] "s"(base_log), [LW] "s"((uint32_t)(uintptr_t)lwtab));
}

}  // namespace pbstw

hipError_t launch_ext_tw(bool cmux, uint64_t* out, uint64_t* glwe, const uint64_t* ggsw, size_t batch, int base_log,
                         const uint64_t* tab, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (base_log < 1 || base_log > 31) return hipErrorInvalidValue;
  if (cmux)
    hipLaunchKernelGGL(pbstw::ext_tw_kernel<true>, dim3((unsigned)batch), dim3(128), 0, s, out, glwe, ggsw,
                       (uint32_t)batch, base_log, tab);
  else
    hipLaunchKernelGGL(pbstw::ext_tw_kernel<false>, dim3((unsigned)batch), dim3(128), 0, s, out, glwe, ggsw,
                       (uint32_t)batch, base_log, tab);
  return hipGetLastError();
}

hipError_t launch_pbs_tw(uint64_t* out, const uint64_t* lwe_in, const uint64_t* lut, const uint64_t* bsk, size_t n_lwe,
                         size_t batch, int base_log, const uint64_t* tab, int centered, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (base_log < 1 || base_log > 31) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pbstw::pbs_tw_kernel, dim3((unsigned)batch), dim3(128), 0, s, out, lwe_in, lut, bsk,
                     (uint32_t)n_lwe, (uint32_t)batch, base_log, tab, centered);
  return hipGetLastError();
}

}  // namespace mi
