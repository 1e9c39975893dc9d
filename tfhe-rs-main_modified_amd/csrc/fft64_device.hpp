// fft64_device.hpp — device helpers shared by the f64-FFT engines: the N = 2048 one-wave engine (fft64_pbs.hip) and
// the shape-generic engine (fft64_generic.hip).  Complex f64 arithmetic (FMA-contracted as the reference's pulp
// kernels' mul_add), the torus conversions of fft_impl/fft64/math/fft/mod.rs, the native decomposition and the
// modulus switch of the blind rotation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi {
namespace fft {

using u64 = uint64_t;

struct __align__(16) cplx {
  double re, im;
};

__device__ __forceinline__ cplx cadd(cplx a, cplx b) { return {a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cplx csub(cplx a, cplx b) { return {a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cplx cmul(cplx a, cplx b) {
  return {__fma_rn(a.re, b.re, -a.im * b.im), __fma_rn(a.re, b.im, a.im * b.re)};
}
// a * conj(b)
__device__ __forceinline__ cplx cmulc(cplx a, cplx b) {
  return {__fma_rn(a.re, b.re, a.im * b.im), __fma_rn(a.im, b.re, -a.re * b.im)};
}
// acc + a * b
__device__ __forceinline__ cplx cfma(cplx a, cplx b, cplx acc) {
  return {__fma_rn(a.re, b.re, __fma_rn(-a.im, b.im, acc.re)), __fma_rn(a.re, b.im, __fma_rn(a.im, b.re, acc.im))};
}
__device__ __forceinline__ cplx mul_neg_i(cplx a) { return {a.im, -a.re}; }  // -i a
__device__ __forceinline__ cplx mul_pos_i(cplx a) { return {-a.im, a.re}; }  // +i a

// ---- conversions (fft_impl/fft64/math/fft/mod.rs) -------------------------------------------------
// u64 -> i64 -> f64 (into_signed().cast_into()); exact int64 -> double rounding as Rust's `as f64`
__device__ __forceinline__ double s64_to_f64(u64 x) { return (double)(int64_t)x; }

// Scalar::from_torus (commons/math/torus/mod.rs:72-78) of x = y / 2^64, taking y = x 2^64 (an exact power-of-two
// scaling by the caller): round(fract(x) 2^64) mod 2^64 = round(y) mod 2^64.  All steps
// exact: r = rint(y); z = r - rint(r 2^-64) 2^64 in [-2^63, 2^63]; z = hi 2^32 + lo with lo in [0, 2^32); the
// words are read from the mantissas of hi + 1.5 2^52 and lo + 2^52.  round-half-even instead of half-away-from-
// zero: different only for an exact half-integer y, where the reference also saturates +2^63 (to i64::MAX; here
// it wraps to 2^63).
__device__ __forceinline__ void torus_words(double y, uint32_t& h, uint32_t& l) {
  const double r = __builtin_rint(y);
  const double z = __fma_rn(-__builtin_rint(r * 0x1p-64), 0x1p64, r);
  const double hi = __builtin_floor(z * 0x1p-32);
  const double lo = __fma_rn(-hi, 0x1p32, z);
  h = (uint32_t)__double_as_longlong(hi + 0x1.8p52);
  l = (uint32_t)__double_as_longlong(lo + 0x1p52);
}
__device__ __forceinline__ u64 from_torus_scaled(double y) {
  uint32_t h, l;
  torus_words(y, h, l);
  return ((u64)h << 32) | l;
}
// acc += from_torus(t) (t in torus units) as one 32-bit add with carry per word: f = fract(t) in [0, 1) is
// exact (t's bits below 2^0); s = f 2^32 exact; the high word is trunc(s), the low word fract(s) 2^32 rounded
// through the mantissa of fract(s) 2^32 + 2^52.  Differences from the exact from_torus, all far below the
// transform's own f64 error (>= 2^40 on these products): for |t| < 2^-12 the fraction rounds (and a low word that
// rounds up to 2^32 drops its carry), and fract of a tiny negative t clamps below 1.
__device__ __forceinline__ void add_torus(u64& acc, double t) {
  const double f = __builtin_amdgcn_fract(t);
  const double s = f * 0x1p32;
  const uint32_t h = (uint32_t)s;
  const uint32_t l = (uint32_t)__double_as_longlong(__fma_rn(__builtin_amdgcn_fract(s), 0x1p32, 0x1p52));
  const uint32_t alo = (uint32_t)acc, ahi = (uint32_t)(acc >> 32);
  const uint32_t nlo = alo + l;
  const uint32_t nhi = ahi + h + (nlo < alo ? 1u : 0u);
  acc = ((u64)nhi << 32) | nlo;
}

// ---- decomposition (commons/math/decomposition/decomposer.rs:156-185, iter.rs:131-151) ------------
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
__device__ __forceinline__ u64 decompose_one_level(int base_log, u64& state) {
  const u64 mask = (1ull << base_log) - 1;
  const u64 res = state & mask;
  state = (u64)((int64_t)state >> base_log);
  const u64 carry = (((res - 1) | state) & res) >> (base_log - 1);
  state += carry;
  return res - (carry << base_log);
}

// fft_impl/common.rs:10-23
__device__ __forceinline__ u64 modulus_switch(u64 input, unsigned log_modulus) {
  return (input + (1ull << (64u - log_modulus - 1u))) >> (64u - log_modulus);
}

// algorithms/modulus_switch.rs:60-104 centered_binary_ms_body_correction_to_add, reduced over the TG threads of
// one ciphertext (gt = index within them; sh = 2 TG u64 of that ciphertext's LDS).  Every thread of the
// workgroup calls it (barriers).
template <int TG>
__device__ u64 centered_body_correction(const u64* __restrict__ lwe, uint32_t n_lwe, unsigned log_mod, int gt,
                                        u64* sh) {
  u64 sum_half = 0;
  int64_t sum_hed = 0;
  for (uint32_t i = gt; i < n_lwe; i += TG) {
    const u64 a = lwe[i];
    const int64_t err = (int64_t)((modulus_switch(a, log_mod) << (64u - log_mod)) - a);
    const int64_t half = err / 2;
    sum_half += (u64)half;
    sum_hed += 2 * half - err;
  }
  sh[gt] = sum_half;
  sh[TG + gt] = (u64)sum_hed;
  __syncthreads();
  for (int s = TG / 2; s > 0; s >>= 1) {
    if (gt < s) {
      sh[gt] += sh[gt + s];
      sh[TG + gt] = (u64)((int64_t)sh[TG + gt] + (int64_t)sh[TG + gt + s]);
    }
    __syncthreads();
  }
  const u64 total_half = sh[0];
  const int64_t total_hed = (int64_t)sh[TG];
  __syncthreads();
  const u64 sum_halving = (u64)(total_hed / 2);
  const u64 half_case = 1ull << (64u - log_mod - 1u);
  return total_half - sum_halving - half_case;
}

}  // namespace fft
}  // namespace mi
