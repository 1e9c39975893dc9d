// mi_arith.hpp — device-side modular arithmetic for the MI355X NTT engine (gfx950).
//
// Two modulus policies with the same interface (add / sub / mul, canonical in [0,p)):
//
//  * Goldilocks  p = 2^64 - 2^32 + 1.  The reference reduces a 128-bit product with the
//    Solinas identity 2^64 = 2^32 - 1, 2^96 = -1 (tfhe-ntt/src/prime64/generic_solinas.rs:102-128).
//    gfx950 has no 64x64 multiply: the product is four v_mad_u64_u32 on 32-bit limbs, the
//    reduction is pure 32/64-bit VALU.  Multiplication by a power of two (the "friendly"
//    twiddles of prime64.rs:162-177, F6 in SURVEY.md) is a shift + the same reduction.
//
//  * Montgomery  any odd p < 2^64 (the generic prime64 path, prime64.rs:957-966): twiddles are
//    pre-scaled by R = 2^64 on the host, so a*w_mont*R^-1 = a*w (mod p), canonical out.
//
// Every op takes canonical inputs (< p) and returns the canonical residue, so any factorisation
// of the transform reproduces the reference bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi {

typedef uint64_t u64;
typedef uint32_t u32;

static constexpr u64 GL_P = 0xFFFFFFFF00000001ull;
static constexpr u64 GL_EPS = 0xFFFFFFFFull;  // 2^64 mod p = 2^32 - 1

__device__ __forceinline__ u32 lo32(u64 x) { return (u32)x; }
__device__ __forceinline__ u32 hi32(u64 x) { return (u32)(x >> 32); }

// 64x64 -> 128 with four 32x32+64 multiply-adds (v_mad_u64_u32).
__device__ __forceinline__ void mul64x64(u64 a, u64 b, u64 &lo, u64 &hi) {
  const u32 a0 = lo32(a), a1 = hi32(a), b0 = lo32(b), b1 = hi32(b);
  const u64 p00 = (u64)a0 * b0;
  const u64 p10 = (u64)a1 * b0 + (p00 >> 32);
  const u64 p01 = (u64)a0 * b1 + (u64)lo32(p10);
  const u64 p11 = (u64)a1 * b1 + (p10 >> 32) + (p01 >> 32);
  lo = (u64)lo32(p00) | ((u64)lo32(p01) << 32);
  hi = p11;
}

struct Goldilocks {
  static constexpr u64 P = GL_P;

  // a + b mod p.  If the 64-bit add carries, s + (2^32-1) is already canonical; otherwise
  // subtract p (= add 2^32-1 mod 2^64) when s >= p.
  __device__ __forceinline__ static u64 add(u64 a, u64 b) {
    const u64 s = a + b;
    const bool c = s < a;
    return (c || s >= P) ? s + GL_EPS : s;
  }
  // a - b mod p.  On borrow, d + p = d - (2^32-1) (mod 2^64) and cannot underflow.
  __device__ __forceinline__ static u64 sub(u64 a, u64 b) {
    const u64 d = a - b;
    return (a < b) ? d - GL_EPS : d;
  }
  // Lazy forms (r5) for butterfly chains whose values need only be congruent mod p (any 64-bit value) until a final
  // multiply or canonicalisation: a + t for a canonical t and any a (a carry folds as + EPS and cannot carry again:
  // a + t - 2^64 < a - EPS + 1), a - t for a canonical t (a borrow subtracts EPS: a - t + 2^64 > EPS, no wrap)
  __device__ __forceinline__ static u64 add_lazy(u64 a, u64 t) {
    unsigned long long c;
    const u64 s = __builtin_addcll(a, t, 0ull, &c);  // the add's own carry (not a 64-bit compare)
    return s + (c ? GL_EPS : 0);
  }
  __device__ __forceinline__ static u64 sub_lazy(u64 a, u64 t) {
    unsigned long long b;
    const u64 d = __builtin_subcll(a, t, 0ull, &b);
    return d - (b ? GL_EPS : 0);
  }
  __device__ __forceinline__ static u64 canon(u64 x) { return x >= P ? x - P : x; }
  // (hi:lo) mod p for any 128-bit value: hi = hh*2^32 + hl, 2^96 = -1, 2^64 = 2^32 - 1.
  __device__ __forceinline__ static u64 reduce128(u64 lo, u64 hi) {
    const u32 hh = hi32(hi), hl = lo32(hi);
    u64 t0 = lo - (u64)hh;
    t0 = (lo < (u64)hh) ? t0 - GL_EPS : t0;
    const u64 t1 = ((u64)hl << 32) - (u64)hl;
    const u64 r = t0 + t1;
    const bool c = r < t1;
    return (c || r >= P) ? r + GL_EPS : r;
  }
  __device__ __forceinline__ static u64 mul(u64 a, u64 b) {
    u64 lo, hi;
    mul64x64(a, b, lo, hi);
    return reduce128(lo, hi);
  }
  // |x 2^e| mod p for a twiddle 2^e (e < 192; 2^96 = -1), canonical, with the sign in `neg` (x 2^e = neg ? -t : t):
  // shifts and the 128-bit reduction instead of the four-limb product.  e must fold to a constant (unrolled stage
  // loops) so the branches disappear.  The friendly twiddles of prime64.rs:162-177.
  __device__ __forceinline__ static u64 mul_pow2(u64 x, int e, bool& neg) {
    neg = e >= 96;
    const int f = neg ? e - 96 : e;
    if (f == 0) return x >= P ? x - P : x;
    if (f < 64) return reduce128(x << f, x >> (64 - f));
    // 64 <= f < 96: with y = x 2^(f - 64) = hi 2^64 + lo (hi < 2^32), x 2^f = lo 2^64 + hi 2^128 = lo 2^64 - hi 2^32
    const int g = f - 64;
    const u64 lo = x << g, hi = g ? x >> (64 - g) : 0;
    return sub(reduce128(0, lo), hi << 32);
  }
};

// the power-of-two twiddles of the first five stages of every Goldilocks plan with the Solinas root tower
// (psi_N^(N / 32) = 8, prime64.rs:166-177): table entry 2^s + g (stage s, group g) is 2^(3 bitrev_5(2^s + g)), its
// inverse-table twin 2^(192 - that); checked against the plan's tables where a kernel relies on it (c_api.cpp)
__host__ __device__ constexpr int tower_exp(bool fwd, int s, int g) {
  int i = (1 << s) + g, r = 0;
  for (int b = 0; b < 5; ++b) r |= ((i >> b) & 1) << (4 - b);
  return fwd ? 3 * r : (192 - 3 * r) % 192;
}

// Generic odd modulus p < 2^64 in Montgomery form (R = 2^64).  `pinv` = -p^{-1} mod 2^64.
struct Montgomery {
  u64 p, pinv, r2;  // r2 = R^2 mod p (to enter Montgomery form on device)
  __device__ __forceinline__ u64 add(u64 a, u64 b) const {
    const u64 neg_b = p - b;
    return a >= neg_b ? a - neg_b : a + b;
  }
  __device__ __forceinline__ u64 sub(u64 a, u64 b) const {
    return a >= b ? a - b : a + (p - b);
  }
  // REDC(a*b): a < p, b < p  ->  a*b*R^-1 mod p, canonical.
  __device__ __forceinline__ u64 mul(u64 a, u64 b) const {
    u64 tlo, thi;
    mul64x64(a, b, tlo, thi);
    const u64 m = tlo * pinv;
    u64 mlo, mhi;
    mul64x64(m, p, mlo, mhi);
    // tlo + mlo == 0 mod 2^64; carry out iff tlo != 0
    const u64 c = (tlo != 0) ? 1 : 0;
    const u64 s = thi + mhi;
    const bool ov1 = s < thi;
    const u64 t = s + c;
    const bool ov = ov1 || (t < s);
    return (ov || t >= p) ? t - p : t;
  }
};

// Odd modulus p < 2^32 (r6: prime32 plans and the CRT primes of the native plans).  A twiddle table entry packs w in
// its low half and Shoup's quotient w' = floor(w 2^32 / p) in its high half: x w mod p = x w - floor(x w' / 2^32) p,
// which lies in [0, 2p), then one conditional subtraction (v_mul_hi_u32 + two v_mad_u64_u32 instead of Montgomery's
// two 64 x 64 products).  Values live in the low 32 bits of u64 registers, canonical, so the results are the same
// residues as the Montgomery form's (bit-exact).
struct Shoup32 {
  uint32_t p;
  __device__ __forceinline__ u64 add(u64 a, u64 b) const {
    const uint32_t x = (uint32_t)a, y = (uint32_t)b, neg_y = p - y;
    return x >= neg_y ? x - neg_y : x + y;
  }
  __device__ __forceinline__ u64 sub(u64 a, u64 b) const {
    const uint32_t x = (uint32_t)a, y = (uint32_t)b;
    return x >= y ? x - y : x + (p - y);
  }
  // x < 2^32, wv = w | w' << 32 with w < p
  __device__ __forceinline__ u64 mul(u64 a, u64 wv) const {
    const uint32_t x = (uint32_t)a, w = (uint32_t)wv, wq = (uint32_t)(wv >> 32);
    const uint32_t q = __umulhi(x, wq);
    const u64 r = (u64)x * w - (u64)q * p;
    return r >= p ? r - p : r;
  }
};

}  // namespace mi
