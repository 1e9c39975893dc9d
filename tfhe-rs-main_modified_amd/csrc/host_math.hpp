// host_math.hpp — host-side number theory for plan construction (product code).
//
// Restates what tfhe_ntt::prime64::Plan::try_new needs to build bit-identical twiddle tables:
//   is_prime64            tfhe-ntt/src/prime.rs:76-128   (deterministic Miller-Rabin, 12 bases)
//   exp_mod64             tfhe-ntt/src/prime.rs:32-50
//   find_primitive_root64 tfhe-ntt/src/roots.rs:6-91     (Tonelli-Shanks chain of square roots of -1)
//   find_root_solinas_64  tfhe-ntt/src/roots.rs:96-107
//   Solinas root table    tfhe-ntt/src/prime64.rs:162-177
// The chosen root fixes the output order of fwd/inv, so the exact root the reference would pick
// is reproduced, not just "a" primitive root.
#pragma once
#include <stdint.h>
#include <cstddef>
#include <optional>
#include <vector>

namespace mi {
namespace host {

using u64 = uint64_t;
using u128 = unsigned __int128;

static constexpr u64 SOLINAS_P = 0xFFFFFFFF00000001ull;

inline u64 mul_mod(u64 a, u64 b, u64 p) { return (u64)(((u128)a * b) % p); }

inline u64 exp_mod(u64 base, u64 pow, u64 p) {
  if (pow == 0) return 1;
  u64 y = 1, x = base;
  while (pow > 1) {
    if (pow & 1) y = mul_mod(x, y, p);
    x = mul_mod(x, x, p);
    pow >>= 1;
  }
  return mul_mod(x, y, p);
}

inline bool is_prime64(u64 n) {
  static const u64 small[12] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  for (u64 q : small)
    if (n % q == 0) return n == q;
  u64 s = 0, d = n - 1;
  while ((d & 1) == 0) { ++s; d >>= 1; }
  for (u64 a : small) {
    u64 x = exp_mod(a, d, n);
    if (x == 1 || x == n - 1) continue;
    bool witness = true;
    for (u64 c = 0; c + 1 < s; ++c) {
      x = mul_mod(x, x, n);
      if (x == n - 1) { witness = false; break; }
    }
    if (witness) return false;
  }
  return true;
}

inline std::optional<u64> tonelli_shanks(u64 p, u64 q, u64 s, u64 z, u64 n) {
  u64 m = s, c = exp_mod(z, q, p), t = exp_mod(n, q, p), r = exp_mod(n, (q + 1) / 2, p);
  for (;;) {
    if (t == 0) return u64(0);
    if (t == 1) return r;
    u64 i = 0, tp = t;
    while (i < m) {
      tp = mul_mod(tp, tp, p);
      ++i;
      if (tp == 1) break;
    }
    if (i == m) return std::nullopt;
    const u64 b = exp_mod(c, u64(1) << (m - i - 1), p);
    m = i;
    c = mul_mod(b, b, p);
    t = mul_mod(t, c, p);
    r = mul_mod(r, b, p);
  }
}

inline std::optional<u64> find_primitive_root64(u64 p, u64 degree) {
  if (degree < 2 || (degree & (degree - 1))) return std::nullopt;
  const unsigned lg = (unsigned)__builtin_ctzll(degree);
  u64 q = p - 1, s = 0;
  while ((q & 1) == 0) { q >>= 1; ++s; }
  std::optional<u64> z;
  for (u64 cand = 2; cand < p; ++cand)
    if (exp_mod(cand, (p - 1) / 2, p) == p - 1) { z = cand; break; }
  if (!z) return std::nullopt;
  u64 root = p - 1;
  for (unsigned i = 0; i + 1 < lg; ++i) {
    auto r = tonelli_shanks(p, q, s, *z, root);
    if (!r) return std::nullopt;
    root = *r;
  }
  return root;
}

inline std::optional<u64> solinas_root(u64 n) {
  switch (n) {
    case 32: return 8ull;
    case 64: return 2198989700608ull;
    case 128: return 14041890976876060974ull;
    case 256: return 14430643036723656017ull;
    case 512: return 4440654710286119610ull;
    case 1024: return 8816101479115663336ull;
    case 2048: return 10974926054405199669ull;
    case 4096: return 1206500561358145487ull;
    case 8192: return 10930245224889659871ull;
    case 16384: return 3333600369887534767ull;
    case 32768: return 15893793146607301539ull;
    default: {
      const u64 deg = 2 * n;
      if (deg == 0 || deg > (u64(1) << 32)) return std::nullopt;
      return exp_mod(16334397945464290598ull /* 2^32-th root */, (u64(1) << 32) / deg, SOLINAS_P);
    }
  }
}

inline unsigned bit_rev(unsigned nbits, u64 i) {
  return (unsigned)(__builtin_bitreverse64(i) >> (64 - nbits));
}

}  // namespace host
}  // namespace mi
