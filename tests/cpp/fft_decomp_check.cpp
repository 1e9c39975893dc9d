// Host check of mi::fft::decompose_l1_hi (csrc/fft64_decomp.hpp) against a plain restatement of the reference's
// native level-1 decomposition (commons/math/decomposition/decomposer.rs:156-185 init, iter.rs:131-151 one level),
// for every base_log 1..31 on the rounding corners (values around every multiple of 2^(63-B)) and random words.
// Build: hipcc -O2 -x hip fft_decomp_check.cpp -o fft_decomp_check (host code only, no GPU needed).
#include <stdio.h>
#include <stdint.h>
#include <random>

#include "../../tfhe-rs-main_modified_amd/csrc/fft64_decomp.hpp"

static uint64_t init_native(uint64_t input, int base_log, int level) {
  const unsigned rep = base_log * level, non_rep = 64u - rep;
  uint64_t res = input >> (non_rep - 1);
  const uint64_t rounding_bit = res & 1u;
  res += 1;
  res >>= 1;
  res &= (~0ull) >> (64u - rep);
  const uint64_t need_balance = (((res - 1) | (rounding_bit << (rep - 1))) & res) >> (rep - 1);
  return res - (need_balance << rep);
}
static int64_t one_level(int base_log, uint64_t& state) {
  const uint64_t mask = (1ull << base_log) - 1;
  const uint64_t res = state & mask;
  state = (uint64_t)((int64_t)state >> base_log);
  const uint64_t carry = (((res - 1) | state) & res) >> (base_log - 1);
  state += carry;
  return (int64_t)(res - (carry << base_log));
}

int main() {
  std::mt19937_64 rng(7);
  long checked = 0, bad = 0;
  for (int B = 1; B <= 31; ++B) {
    auto check = [&](uint64_t x) {
      uint64_t st = init_native(x, B, 1);
      const int64_t want = one_level(B, st);
      const int32_t got = mi::fft::decompose_l1_hi((uint32_t)(x >> 32), B);
      ++checked;
      if ((int64_t)got != want) {
        if (bad++ < 10) printf("B=%d x=%016llx want %lld got %d\n", B, (unsigned long long)x, (long long)want, got);
      }
    };
    const unsigned sh = 63 - B;  // rounding boundary granularity
    for (int i = 0; i < 20000; ++i) {
      const uint64_t base = (rng() >> sh) << sh;
      for (int d = -3; d <= 3; ++d) check(base + (uint64_t)(int64_t)d);
      check(base + (1ull << (sh > 0 ? sh - 1 : 0)));
      check(rng());
    }
    for (uint64_t x : {0ull, ~0ull, 1ull << 63, (1ull << 63) - 1, (1ull << 63) + 1}) check(x);
  }
  printf("%ld checked, %ld mismatches\n", checked, bad);
  return bad ? 1 : 0;
}
