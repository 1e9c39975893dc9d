// test_prime64.cpp — the reference's own prime64::Plan tests, restated against the C++ mirror
// (include/tfhe_ntt_amd.hpp) of the MI355X engine.  Reference: tfhe-ntt/src/prime64.rs (paths
// relative to /root/reference); each test names the reference test it restates.
//
//   ./test_prime64          every test (needs a HIP device)
//   ./test_prime64 --cpu    only the try_new None cases, which never touch the device
//
// The primes are the reference's largest_prime_in_arithmetic_progression64(1 << 16, 1, lo, hi) values
// (tests/test_cpp_mirror.py checks them against the oracle's restatement of prime.rs).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "tfhe_ntt_amd.hpp"

using tfhe_ntt_amd::prime64::Plan;
using u128 = unsigned __int128;

static int g_failures = 0;
#define EXPECT(cond)                                                              \
  do {                                                                            \
    if (!(cond)) {                                                                \
      std::fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                               \
    }                                                                             \
  } while (0)

static const uint64_t SOLINAS = 0xFFFFFFFF00000001ull;
// prime64.rs:1309-1314 (test_product) and :1459-1463 (test_mul_accumulate)
static const uint64_t PRODUCT_PRIMES[] = {1125899904679937ull, 2251799813554177ull, 4611686018427322369ull,
                                          9223372036853661697ull, SOLINAS, 18446744073707716609ull};
static const uint64_t MACC_PRIMES[] = {2251799813554177ull, 2305843009211662337ull, 4611686018427322369ull,
                                       9223372036853661697ull, 18446744073707716609ull};

static uint64_t mulm(uint64_t p, uint64_t a, uint64_t b) { return (uint64_t)((u128)a * b % p); }
static uint64_t addm(uint64_t p, uint64_t a, uint64_t b) { return (uint64_t)(((u128)a + b) % p); }
static uint64_t subm(uint64_t p, uint64_t a, uint64_t b) { return a >= b ? a - b : (uint64_t)((u128)a + p - b); }
static uint64_t powm(uint64_t p, uint64_t b, uint64_t e) {
  uint64_t r = 1;
  for (; e; e >>= 1, b = mulm(p, b, b))
    if (e & 1) r = mulm(p, r, b);
  return r;
}

static std::mt19937_64 g_rng(0x74666865);
static std::vector<uint64_t> random_poly(size_t n, uint64_t p) {
  std::vector<uint64_t> v(n);
  for (auto& x : v) x = g_rng() % p;
  return v;
}

// prime64.rs:1264-1276 negacyclic_convolution
static std::vector<uint64_t> negacyclic_convolution(size_t n, uint64_t p, const std::vector<uint64_t>& lhs,
                                                    const std::vector<uint64_t>& rhs) {
  std::vector<uint64_t> full(2 * n, 0), out(n);
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) full[i + j] = addm(p, full[i + j], mulm(p, lhs[i], rhs[j]));
  for (size_t i = 0; i < n; ++i) out[i] = subm(p, full[i], full[i + n]);
  return out;
}

// prime64.rs:1305-1361 test_product
static void test_product() {
  for (size_t n : {16, 32, 64, 128, 256, 512, 1024}) {
    for (uint64_t p : PRODUCT_PRIMES) {
      auto plan = Plan::try_new(n, p);
      EXPECT(plan.has_value());
      if (!plan) continue;
      const auto lhs = random_poly(n, p), rhs = random_poly(n, p);
      const auto conv = negacyclic_convolution(n, p, lhs, rhs);
      auto lf = lhs, rf = rhs;
      plan->fwd(lf.data(), lf.size());
      plan->fwd(rf.data(), rf.size());
      for (auto x : lf) EXPECT(x < p);
      for (auto x : rf) EXPECT(x < p);
      std::vector<uint64_t> prod(n);
      for (size_t i = 0; i < n; ++i) prod[i] = mulm(p, lf[i], rf[i]);
      plan->inv(prod.data(), prod.size());
      plan->mul_assign_normalize(lf.data(), lf.size(), rf.data(), rf.size());
      plan->inv(lf.data(), lf.size());
      for (size_t i = 0; i < n; ++i) {
        EXPECT(prod[i] < p);
        EXPECT(prod[i] == mulm(p, conv[i], n));
      }
      EXPECT(lf == conv);
    }
  }
}

// prime64.rs:1363-1385 / 1387-1423 (normalize, mul_assign_normalize vs u128 %)
static void test_normalize_and_mul_assign_normalize() {
  const uint64_t p = 9223372036853661697ull;  // largest_prime_in_arithmetic_progression64(1<<16, 1, 1<<50, 1<<63)
  const size_t n = 128;
  auto plan = Plan::try_new(n, p);
  EXPECT(plan.has_value());
  if (!plan) return;
  const uint64_t n_inv = powm(p, n, p - 2);
  auto val = random_poly(n, p), target = val;
  for (auto& x : target) x = mulm(p, x, n_inv);
  plan->normalize(val.data(), val.size());
  EXPECT(val == target);
  auto lhs = random_poly(n, p), rhs = random_poly(n, p), lt = lhs;
  for (size_t i = 0; i < n; ++i) lt[i] = mulm(p, mulm(p, lhs[i], rhs[i]), n_inv);
  plan->mul_assign_normalize(lhs.data(), lhs.size(), rhs.data(), rhs.size());
  EXPECT(lhs == lt);
}

// prime64.rs:1456-1490 test_mul_accumulate
static void test_mul_accumulate() {
  for (uint64_t p : MACC_PRIMES) {
    const size_t n = 128;
    auto plan = Plan::try_new(n, p);
    EXPECT(plan.has_value());
    if (!plan) continue;
    auto acc = random_poly(n, p), target = acc;
    const auto lhs = random_poly(n, p), rhs = random_poly(n, p);
    for (size_t i = 0; i < n; ++i) target[i] = addm(p, mulm(p, lhs[i], rhs[i]), target[i]);
    plan->mul_accumulate(acc.data(), acc.size(), lhs.data(), lhs.size(), rhs.data(), rhs.size());
    EXPECT(acc == target);
  }
}

// prime64.rs:1987-1990 (try_new(2048, 1024) is None) and the try_new validity rules (:769-775)
static void test_try_new_none() {
  EXPECT(!Plan::try_new(2048, 1024).has_value());                  // not prime
  EXPECT(!Plan::try_new(15, SOLINAS).has_value());                 // not a power of two
  EXPECT(!Plan::try_new(8, SOLINAS).has_value());                  // N < 16
  EXPECT(!Plan::try_new(1 << 10, 97).has_value());                 // prime without a 2N-th root
}

// slice length mismatches panic in the reference (assert_eq!, prime64.rs:898, 976)
static void test_length_mismatch_throws() {
  auto plan = Plan::try_new(32, SOLINAS);
  EXPECT(plan.has_value());
  if (!plan) return;
  std::vector<uint64_t> v(31, 0);
  bool threw = false;
  try {
    plan->fwd(v.data(), v.size());
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  EXPECT(threw);
}

// the host-slice pointwise ops run through the library's pooled staging slots: after the first call, a long run of
// calls allocates no device memory (hipMemGetInfo's free bytes do not move) and every result is exact
static void test_pointwise_host_no_allocation() {
  const size_t n = 2048;
  auto plan = Plan::try_new(n, SOLINAS);
  EXPECT(plan.has_value());
  if (!plan) return;
  const uint64_t p = SOLINAS, n_inv = powm(p, n, p - 2);
  auto acc = random_poly(n, p), lhs = random_poly(n, p), rhs = random_poly(n, p);
  plan->mul_accumulate(acc.data(), n, lhs.data(), n, rhs.data(), n);  // warm the slot
  plan->normalize(acc.data(), n);
  size_t free0 = 0, free1 = 0, total = 0;
  EXPECT(hipMemGetInfo(&free0, &total) == hipSuccess);
  bool exact = true;
  for (int it = 0; it < 300; ++it) {
    auto want = acc;
    for (size_t i = 0; i < n; ++i) want[i] = addm(p, mulm(p, lhs[i], rhs[i]), want[i]);
    plan->mul_accumulate(acc.data(), n, lhs.data(), n, rhs.data(), n);
    exact = exact && acc == want;
    for (size_t i = 0; i < n; ++i) want[i] = mulm(p, mulm(p, acc[i], rhs[i]), n_inv);
    plan->mul_assign_normalize(acc.data(), n, rhs.data(), n);
    exact = exact && acc == want;
    for (size_t i = 0; i < n; ++i) want[i] = mulm(p, acc[i], n_inv);
    plan->normalize(acc.data(), n);
    exact = exact && acc == want;
  }
  EXPECT(exact);
  EXPECT(hipMemGetInfo(&free1, &total) == hipSuccess);
  EXPECT(free1 == free0);
  if (free1 != free0) std::fprintf(stderr, "device free bytes moved: %zu -> %zu\n", free0, free1);
}

int main(int argc, char** argv) {
  const bool cpu_only = argc > 1 && std::string(argv[1]) == "--cpu";
  test_try_new_none();
  if (!cpu_only) {
    test_product();
    test_normalize_and_mul_assign_normalize();
    test_mul_accumulate();
    test_length_mismatch_throws();
    test_pointwise_host_no_allocation();
  }
  if (g_failures) {
    std::fprintf(stderr, "%d expectation(s) failed\n", g_failures);
    return 1;
  }
  std::printf("test_prime64: all %stests passed\n", cpu_only ? "CPU-only " : "");
  return 0;
}
