// pbs_device.hpp — device restatements of the scalar reference functions the PBS kernels share (pbs_kernels.hip:
// fused one-workgroup-per-ciphertext blind rotation; pbs_large.hip: the multi-kernel blind rotation of N > 8192).
// Reference paths relative to /root/reference/tfhe/src/core_crypto.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"

namespace mi {
namespace pbs {

static constexpr u64 P = GL_P;

// ---- scalar helpers (each restates one reference function) ----------------------------------

// commons/math/decomposition/decomposer.rs:156-185 (native u64)
__device__ __forceinline__ u64 decomp_init_native(u64 input, int base_log, int level) {
  const unsigned rep = base_log * level, non_rep = 64u - rep;
  u64 res = input >> (non_rep - 1);
  const u64 rounding_bit = res & 1u;
  res += 1;
  res >>= 1;
  res &= (~0ull) >> (64u - rep);
  const u64 need_balance = (((res - 1) | (rounding_bit << (rep - 1))) & res) >> (rep - 1);
  return res - (need_balance << rep);
}

// commons/math/decomposition/iter.rs:131-151
__device__ __forceinline__ u64 decompose_one_level(int base_log, u64& state) {
  const u64 mask = (1ull << base_log) - 1;
  const u64 res = state & mask;
  state = (u64)((int64_t)state >> base_log);
  const u64 carry = (((res - 1) | state) & res) >> (base_log - 1);
  state += carry;
  return res - (carry << base_log);
}

// decomposer.rs:25-49 native_closest_representable, then decomposer.rs:521-548 (q = p, 64 bits)
__device__ __forceinline__ u64 closest_abs_nonnative(u64 abs_value, int base_log, int level) {
  const unsigned shift = 64u - (unsigned)(level * base_log) - 1u;
  u64 res = abs_value >> shift;
  res += 1;
  res &= ~1ull;
  return res << shift;
}

// commons/math/ntt/ntt64.rs:184-197: ((v << 64) | (p >> 1)) / p for v < p, restated without a
// 128-bit division: 2^64 = p + EPS, so q = v + floor((v*EPS + h) / p) with h = p >> 1.
__device__ __forceinline__ u64 modswitch_prime_to_native(u64 v) {
  const unsigned __int128 R = (unsigned __int128)v * GL_EPS + (P >> 1);
  const u64 rh = (u64)(R >> 64), rl = (u64)R;
  unsigned __int128 R2 = (unsigned __int128)rh * GL_EPS + rl;  // R = rh*p + R2, R2 < 2^65
  u64 q = rh;
  if (R2 >= P) { R2 -= P; ++q; }
  if (R2 >= P) { ++q; }
  return v + q;
}

// fft_impl/common.rs:10-23
__device__ __forceinline__ u64 modulus_switch(u64 input, unsigned log_modulus) {
  return (input + (1ull << (64u - log_modulus - 1u))) >> (64u - log_modulus);
}

// ntt64_pbs.rs:540-549 + algorithms/misc.rs:6-18 divide_round
__device__ __forceinline__ u64 ms_non_native(u64 input, unsigned log_mod) {
  const unsigned __int128 num = ((unsigned __int128)input) << log_mod;
  // num / p with the 2^64 = p + EPS split (num < 2^(64 + log_mod))
  const u64 nh = (u64)(num >> 64), nl = (u64)num;
  unsigned __int128 r = (unsigned __int128)nh * GL_EPS + nl;  // num = nh*p + r
  u64 q = nh;
  while (r >= P) { r -= P; ++q; }
  return q + (r >= (P >> 1) ? 1 : 0);
}

__device__ __forceinline__ u64 neg_custom(u64 a) { return a == 0 ? 0 : P - a; }
__device__ __forceinline__ u64 sub_custom(u64 a, u64 b) { return a >= b ? a - b : a - b + P; }
__device__ __forceinline__ u64 add_custom(u64 a, u64 b) { return sub_custom(a, neg_custom(b)); }

template <bool BNF>
__device__ __forceinline__ u64 neg_q(u64 a) { return BNF ? (u64)0 - a : neg_custom(a); }

// algorithms/modulus_switch.rs:60-104 centered_binary_ms_body_correction_to_add, reduced over the
// workgroup (uses sh[0 .. 2T) and leaves it free again).
template <int T>
__device__ u64 centered_body_correction(const u64* __restrict__ lwe, uint32_t n_lwe, unsigned log_mod, int t, u64* sh) {
  u64 sum_half = 0;
  int64_t sum_hed = 0;
  for (uint32_t i = t; i < n_lwe; i += T) {
    const u64 a = lwe[i];
    const int64_t err = (int64_t)((modulus_switch(a, log_mod) << (64u - log_mod)) - a);
    const int64_t half = err / 2;  // truncating, as Rust's signed division
    sum_half += (u64)half;
    sum_hed += 2 * half - err;
  }
  sh[t] = sum_half;
  sh[T + t] = (u64)sum_hed;
  __syncthreads();
  for (int s = T / 2; s > 0; s >>= 1) {
    if (t < s) {
      sh[t] += sh[t + s];
      sh[T + t] = (u64)((int64_t)sh[T + t] + (int64_t)sh[T + t + s]);
    }
    __syncthreads();
  }
  const u64 total_half = sh[0];
  const int64_t total_hed = (int64_t)sh[T];
  __syncthreads();
  const u64 sum_halving = (u64)(total_hed / 2);
  const u64 half_case = 1ull << (64u - log_mod - 1u);
  return total_half - sum_halving - half_case;
}

// The sum of a column's level (k + 1) products without a carry chain per product: each term's four 32 x 32 partial
// products go straight into three 64-bit column accumulators (bits 0, 32 and 64 up) through v_mad_u64_u32's own
// addend, their carries out of the accumulator counted apart: 8 VALU per term instead of a 128-bit product (4 mads plus
// the limb assembly) and a 128-bit add (~19 VALU as compiled).  value() combines the columns and reduces once.
struct Acc128 {
  u64 a0 = 0, a32 = 0, a64 = 0;
  uint32_t n0 = 0, n32 = 0, n64 = 0;
  __device__ __forceinline__ void mac(u64 x, u64 w) {
    const uint32_t x0 = (uint32_t)x, x1 = (uint32_t)(x >> 32), w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
    uint64_t c0, c1, c2, c3, junk;
    // every carry is read >= 3 instructions after the mad that wrote it (VALU-written SGPR -> VALU read); not volatile:
    // the block has no side effect beyond its outputs, so the compiler may schedule the loads around it
    asm(
        "v_mad_u64_u32 %[a0], %[c0], %[x0], %[w0], %[a0]\n\t"
        "v_mad_u64_u32 %[a32], %[c1], %[x0], %[w1], %[a32]\n\t"
        "v_mad_u64_u32 %[a64], %[c3], %[x1], %[w1], %[a64]\n\t"
        "v_mad_u64_u32 %[a32], %[c2], %[x1], %[w0], %[a32]\n\t"
        "v_addc_co_u32_e64 %[n0], %[j], %[n0], 0, %[c0]\n\t"
        "v_addc_co_u32_e64 %[n32], %[j], %[n32], 0, %[c1]\n\t"
        "v_addc_co_u32_e64 %[n64], %[j], %[n64], 0, %[c3]\n\t"
        "v_addc_co_u32_e64 %[n32], %[j], %[n32], 0, %[c2]"
        : [a0] "+v"(a0), [a32] "+v"(a32), [a64] "+v"(a64), [n0] "+v"(n0), [n32] "+v"(n32), [n64] "+v"(n64),
          [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3), [j] "=&s"(junk)
        : [x0] "v"(x0), [x1] "v"(x1), [w0] "v"(w0), [w1] "v"(w1));
  }
  // a0 + a32 2^32 + (a64 + n0) 2^64 + n32 2^96 + n64 2^128, with 2^128 = -2^32 mod p
  __device__ __forceinline__ u64 value(u64 n_inv) const {
    const u64 lo = a0 + (a32 << 32);
    const u64 t = (a32 >> 32) + (lo < a0);
    u64 hi = a64 + t;
    uint32_t top = n64 + (hi < t);
    hi += n0;
    top += hi < (u64)n0;
    const u64 h32 = (u64)n32 << 32;
    hi += h32;
    top += hi < h32;
    const u64 v = Goldilocks::sub(Goldilocks::reduce128(lo, hi), (u64)top << 32);
    return n_inv ? Goldilocks::mul(v, n_inv) : v;
  }
};

}  // namespace pbs
}  // namespace mi
