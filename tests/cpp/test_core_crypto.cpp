// test_core_crypto.cpp — the C++ core_crypto mirror (include/tfhe_ntt_amd.hpp, namespace core_crypto)
// against the CPU oracle (oracle/ks_oracle.c, pbs_oracle.c: restatements of the reference, linked
// here only as the checker), bit for bit, on seeded random keys and ciphertexts:
//   convert_standard_lwe_bootstrap_key_to_ntt64   lwe_bootstrap_key_conversion.rs:294-365 (Raw)
//   add_external_product_ntt64_assign (BNF)        ntt64_bnf_pbs.rs:541-681
//   programmable_bootstrap_ntt64_lwe_ciphertext    ntt64_bnf_pbs.rs:469-540 (standard modulus switch)
//   keyswitch_lwe_ciphertext                       lwe_keyswitch.rs:137-227 (2048 -> 918, B 2^4, L 4)
//   keyswitch_lwe_ciphertext_with_scalar_change    lwe_keyswitch.rs:331-447 (KS32: 2048 -> 879, B 2^2, L 8, 2^21)
//   lwe_ciphertext_centered_binary_modulus_switch  modulus_switch.rs:35-104 (u32 and u64 LWEs)
//   Ntt64View (all six helpers)                    commons/math/ntt/ntt64.rs:89-266
// and the f64-FFT mirror (namespace fft64) against exact integer arithmetic within the f64 error bound:
//   forward_as_torus -> backward_as_torus round trip, add_external_product_assign vs the exact negacyclic product
// Needs a HIP device.  Build: make -C tests/cpp.
#include <cmath>
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <vector>

#include "tfhe_ntt_amd.hpp"

extern "C" {
#include "../../oracle/ks_oracle.h"
#include "../../oracle/ntt_oracle.h"
#include "../../oracle/pbs_oracle.h"
}

namespace cc = tfhe_ntt_amd::core_crypto;
using tfhe_ntt_amd::prime64::Plan;

static int g_failures = 0;
#define EXPECT(cond)                                                                        \
  do {                                                                                      \
    if (!(cond)) {                                                                          \
      std::fprintf(stderr, "%s:%d: expectation failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                                         \
    }                                                                                       \
  } while (0)

static const uint64_t P = 0xFFFFFFFF00000001ull;
static const size_t N = 2048;

struct Dev {  // a device copy of a host vector
  uint64_t* p = nullptr;
  size_t n = 0;
  explicit Dev(const std::vector<uint64_t>& h) : n(h.size()) {
    if (hipMalloc(reinterpret_cast<void**>(&p), n * 8) != hipSuccess ||
        hipMemcpy(p, h.data(), n * 8, hipMemcpyHostToDevice) != hipSuccess)
      throw std::runtime_error("device copy failed");
  }
  explicit Dev(size_t count) : n(count) {
    if (hipMalloc(reinterpret_cast<void**>(&p), n * 8) != hipSuccess || hipMemset(p, 0, n * 8) != hipSuccess)
      throw std::runtime_error("device allocation failed");
  }
  ~Dev() { (void)hipFree(p); }
  std::vector<uint64_t> host() const {
    std::vector<uint64_t> h(n);
    if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(h.data(), p, n * 8, hipMemcpyDeviceToHost) != hipSuccess)
      throw std::runtime_error("device read failed");
    return h;
  }
};

static std::vector<uint64_t> uniform(uint64_t seed, uint64_t p, size_t count) {
  std::vector<uint64_t> v(count);
  ora_fill_uniform(seed, p, v.data(), count);
  return v;
}

int main() {
  std::vector<uint64_t> twid(N), itwid(N);
  uint64_t n_inv = 0;
  EXPECT(ora_plan_init(N, P, twid.data(), itwid.data(), &n_inv));
  const ora_ntt_tables tabs{N, P, twid.data(), itwid.data(), n_inv};
  auto plan = Plan::try_new(N, P);
  EXPECT(plan.has_value());
  if (!plan) return 1;

  // key conversion (Raw) of a native-modulus standard key, n_lwe = 16
  const size_t n_lwe = 16, polys = n_lwe * 4;
  const auto bsk_std = uniform(101, 0, polys * N);
  std::vector<uint64_t> bsk_ref(polys * N);
  ora_bsk_to_ntt(&tabs, bsk_std.data(), bsk_ref.data(), polys, 64, 0);
  Dev d_std(bsk_std), d_ntt(polys * N);
  cc::convert_standard_lwe_bootstrap_key_to_ntt64(*plan, d_std.p, d_ntt.p, polys, 64, false);
  EXPECT(d_ntt.host() == bsk_ref);

  // external product, BNF, level 1, base 2^23, batch 2
  {
    const size_t batch = 2;
    const auto ggsw = uniform(102, P, 4 * N), glwe = uniform(103, 0, batch * 2 * N), out = uniform(104, 0, batch * 2 * N);
    std::vector<uint64_t> want(out);
    for (size_t b = 0; b < batch; ++b)
      ora_ext_product_bnf(&tabs, 1, 23, 1, want.data() + b * 2 * N, ggsw.data(), glwe.data() + b * 2 * N);
    Dev d_g(ggsw), d_in(glwe), d_out(out);
    cc::add_external_product_ntt64_assign(*plan, d_out.p, d_in.p, d_g.p, 23, 1, batch, MI_NTT64_BNF);
    EXPECT(d_out.host() == want);
  }

  // PBS, BNF, level 1, base 2^23, batch 3, on the converted key
  {
    const size_t batch = 3;
    const auto lut = uniform(105, 0, 2 * N), lwe = uniform(106, 0, batch * (n_lwe + 1));
    std::vector<uint64_t> want(batch * (N + 1));
    for (size_t b = 0; b < batch; ++b)
      ora_pbs_bnf(&tabs, 1, 23, 1, want.data() + b * (N + 1), lwe.data() + b * (n_lwe + 1), lut.data(),
                  bsk_ref.data(), n_lwe);
    cc::NttBootstrapKey key(*plan, d_ntt.p, n_lwe, 23, 1, MI_NTT64_BNF);
    Dev d_lut(lut), d_lwe(lwe), d_out(batch * (N + 1));
    cc::programmable_bootstrap_ntt64_lwe_ciphertext(key, d_lwe.p, d_out.p, d_lut.p, batch);
    EXPECT(d_out.host() == want);
  }

  // keyswitch 2048 -> 918, base 2^4, 4 levels (PARAM_MESSAGE_2_CARRY_2), batch 5
  {
    const size_t in_dim = 2048, out_dim = 918, batch = 5;
    const int bl = 4, lv = 4;
    const auto ksk = uniform(107, 0, in_dim * lv * (out_dim + 1)), lwe = uniform(108, 0, batch * (in_dim + 1));
    std::vector<uint64_t> want(batch * (out_dim + 1));
    ora_lwe_keyswitch_batch(ksk.data(), in_dim, out_dim, bl, lv, lwe.data(), want.data(), batch, 4);
    Dev d_ksk(ksk), d_lwe(lwe), d_out(batch * (out_dim + 1));
    cc::LweKeyswitchKey key(d_ksk.p, in_dim, out_dim, bl, lv);
    cc::keyswitch_lwe_ciphertext(key, d_lwe.p, d_out.p, batch);
    EXPECT(d_out.host() == want);
  }

  // KS32: keyswitch_lwe_ciphertext_with_scalar_change 2048 -> 879, base 2^2, 8 levels, u32 output mod 2^21 (the HPU
  // KS32 parameters), then the centered binary modulus switch of the u32 LWEs to 2N = 4096, batch 6
  {
    const size_t in_dim = 2048, out_dim = 879, batch = 6;
    const int bl = 2, lv = 8, w = 21;
    const auto raw = uniform(109, 0, in_dim * lv * (out_dim + 1)), lwe = uniform(110, 0, batch * (in_dim + 1));
    std::vector<uint32_t> ksk(raw.size());
    for (size_t i = 0; i < raw.size(); ++i) ksk[i] = (uint32_t)raw[i] & ~((1u << (32 - w)) - 1);
    std::vector<uint32_t> want(batch * (out_dim + 1));
    ora_lwe_keyswitch32_batch(ksk.data(), in_dim, out_dim, bl, lv, w, lwe.data(), want.data(), batch, 4);
    uint32_t *d_ksk = nullptr, *d_out = nullptr;
    EXPECT(hipMalloc(reinterpret_cast<void**>(&d_ksk), ksk.size() * 4) == hipSuccess);
    EXPECT(hipMalloc(reinterpret_cast<void**>(&d_out), want.size() * 4) == hipSuccess);
    EXPECT(hipMemcpy(d_ksk, ksk.data(), ksk.size() * 4, hipMemcpyHostToDevice) == hipSuccess);
    Dev d_lwe(lwe), d_sw(batch * (out_dim + 1));
    cc::LweKeyswitchKey32 key(d_ksk, in_dim, out_dim, bl, lv, w);
    cc::keyswitch_lwe_ciphertext_with_scalar_change(key, d_lwe.p, d_out, batch);
    std::vector<uint32_t> got(want.size());
    EXPECT(hipDeviceSynchronize() == hipSuccess);
    EXPECT(hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost) == hipSuccess);
    EXPECT(got == want);
    cc::lwe_ciphertext_modulus_switch32(d_out, d_sw.p, out_dim, batch, 12, true);
    std::vector<uint64_t> want_sw(batch * (out_dim + 1));
    for (size_t b = 0; b < batch; ++b)
      ora_lwe_ms32(want.data() + b * (out_dim + 1), out_dim, 12, 1, want_sw.data() + b * (out_dim + 1));
    EXPECT(d_sw.host() == want_sw);
    (void)hipFree(d_ksk);
    (void)hipFree(d_out);
  }

  // Ntt64View (ntt64.rs:89-266) over a batch of 5: forward_normalized, forward_from_power_of_two_modulus (w = 21),
  // forward_from_decomp, add_backward, add_backward_on_power_of_two_modulus (w = 64); then the u64 centered switch
  {
    const size_t batch = 5;
    cc::Ntt64View view(*plan);
    EXPECT(view.polynomial_size() == N && view.custom_modulus() == P);
    const auto x = uniform(130, P, batch * N), w = uniform(131, 0, batch * N), st = uniform(132, 0, batch * N);
    std::vector<uint64_t> dg(batch * N);
    for (size_t i = 0; i < dg.size(); ++i) dg[i] = (uint64_t)((int64_t)(w[i] % (1u << 23)) - (1 << 22));
    std::vector<uint64_t> want(batch * N);
    Dev d_x(x), d_w(w), d_dg(dg), d_out(batch * N);
    ora_ntt64_view_forward_batch(&tabs, 0, 0, 1, want.data(), x.data(), batch, N, 4);
    view.forward_normalized(d_out.p, d_x.p, batch, N);
    EXPECT(d_out.host() == want);
    ora_ntt64_view_forward_batch(&tabs, 1, 21, 0, want.data(), w.data(), batch, N, 4);
    view.forward_from_power_of_two_modulus(21, d_out.p, d_w.p, batch, N);
    EXPECT(d_out.host() == want);
    ora_ntt64_view_forward_batch(&tabs, 2, 0, 0, want.data(), dg.data(), batch, N, 4);
    view.forward_from_decomp(d_out.p, d_dg.p, batch, N);
    EXPECT(d_out.host() == want);
    std::vector<uint64_t> want_st(x), want_y(x);  // add_backward: standard mod p, ntt = x
    ora_ntt64_view_add_backward_batch(&tabs, 0, want_st.data(), want_y.data(), batch, N, 4);
    Dev d_st(x), d_y(x);
    view.add_backward(d_st.p, d_y.p, batch, N);
    EXPECT(d_st.host() == want_st);
    EXPECT(d_y.host() == want_y);
    std::vector<uint64_t> want_st2(st), want_y2(x);
    ora_ntt64_view_add_backward_batch(&tabs, 64, want_st2.data(), want_y2.data(), batch, N, 4);
    Dev d_st2(st), d_y2(x);
    view.add_backward_on_power_of_two_modulus(64, d_st2.p, d_y2.p, batch, N);
    EXPECT(d_st2.host() == want_st2);
    EXPECT(d_y2.host() == want_y2);
    const size_t dim = 918;
    const auto lwe = uniform(133, 0, batch * (dim + 1));
    std::vector<uint64_t> want_sw(lwe.size());
    for (size_t b = 0; b < batch; ++b) ora_lwe_ms64(lwe.data() + b * (dim + 1), dim, 12, 1, want_sw.data() + b * (dim + 1));
    Dev d_lwe(lwe), d_sw(lwe.size());
    cc::lwe_ciphertext_modulus_switch(d_lwe.p, d_sw.p, dim, batch, 12, true);
    EXPECT(d_sw.host() == want_sw);
  }

  // errors surface as tfhe_ntt_amd::Error with the C status (base_log * level >= 64)
  {
    bool threw = false;
    try {
      Dev d(8 * 8 * 11);
      cc::LweKeyswitchKey bad(d.p, 8, 10, 8, 8);
    } catch (const tfhe_ntt_amd::Error& e) {
      threw = e.status() == MI_ERR_INVALID_ARG;
    }
    EXPECT(threw);
  }

  // GLWE-output blind rotation (BNF, in place, one accumulator per item) + many-sample extraction == the oracle's
  // blind_rotate_ntt64_bnf_assign + extract_lwe_sample_from_glwe_ciphertext at 0 and N/2; LUT-indexed PBS
  {
    const size_t batch = 3;
    const auto acc = uniform(120, 0, batch * 2 * N), lwe = uniform(121, 0, batch * (n_lwe + 1));
    std::vector<uint64_t> want_acc(acc), want_lwe(batch * 2 * (N + 1));
    const unsigned log_mod = 12;
    for (size_t b = 0; b < batch; ++b) {
      std::vector<uint64_t> ms(n_lwe);
      for (size_t i = 0; i < n_lwe; ++i) ms[i] = ora_modulus_switch(lwe[b * (n_lwe + 1) + i], log_mod);
      ora_blind_rotate_bnf(&tabs, 1, 23, 1, want_acc.data() + b * 2 * N, ms.data(),
                           ora_modulus_switch(lwe[b * (n_lwe + 1) + n_lwe], log_mod), bsk_ref.data(), n_lwe);
      for (size_t j = 0; j < 2; ++j)
        ora_sample_extract_nth(want_acc.data() + b * 2 * N, want_lwe.data() + (b * 2 + j) * (N + 1), N, 1, j * (N / 2), 0);
    }
    cc::NttBootstrapKey key(*plan, d_ntt.p, n_lwe, 23, 1, MI_NTT64_BNF);
    Dev d_acc(acc), d_lwe(lwe), d_out(batch * 2 * (N + 1));
    cc::blind_rotate_ntt64_assign(key, d_lwe.p, d_acc.p, batch);
    EXPECT(d_acc.host() == want_acc);
    cc::extract_lwe_sample_from_glwe_ciphertext(d_acc.p, d_out.p, N, 1, batch, 0, N / 2, 2);
    EXPECT(d_out.host() == want_lwe);
    // item b through LUT idx[b]: the rotated accumulators' first rows double as three LUTs
    const std::vector<uint64_t> luts = uniform(122, 0, 3 * 2 * N);
    const uint32_t idx_h[3] = {2, 0, 2};
    uint32_t* idx = nullptr;
    EXPECT(hipMalloc(reinterpret_cast<void**>(&idx), sizeof idx_h) == hipSuccess);
    EXPECT(hipMemcpy(idx, idx_h, sizeof idx_h, hipMemcpyHostToDevice) == hipSuccess);
    std::vector<uint64_t> want(batch * (N + 1));
    for (size_t b = 0; b < batch; ++b)
      ora_pbs_bnf(&tabs, 1, 23, 1, want.data() + b * (N + 1), lwe.data() + b * (n_lwe + 1),
                  luts.data() + idx_h[b] * 2 * N, bsk_ref.data(), n_lwe);
    Dev d_luts(luts), d_pbs(batch * (N + 1));
    cc::programmable_bootstrap_ntt64_lwe_ciphertext_lut_indexed(key, d_lwe.p, d_pbs.p, d_luts.p, idx, 3, batch);
    EXPECT(d_pbs.host() == want);
    (void)hipFree(idx);
  }

  // f64 FFT: round trip and an external product (k = 1, level 1, base 2^23) vs the exact product in Z_2^64[X]/(X^N+1),
  // at N = 2048 (the one-wave engine) and at 1024 / 8192 (the shape-generic engine), each on the legacy null stream and
  // on a created non-blocking stream (the r3 stale-scratch sequence: in-place reorder, N = 8192 external product)
  hipStream_t own = nullptr;
  EXPECT(hipStreamCreateWithFlags(&own, hipStreamNonBlocking) == hipSuccess);
  for (hipStream_t st : {(hipStream_t) nullptr, own})
  for (const size_t NF : {(size_t)2048, (size_t)1024, (size_t)8192}) {
    tfhe_ntt_amd::fft64::Fft fft(NF);
    const size_t batch = 2;
    const auto x = uniform(109, 0, batch * NF);
    Dev d_x(x), d_back(batch * NF);
    double* four = nullptr;
    EXPECT(hipMalloc(reinterpret_cast<void**>(&four), batch * NF * 8) == hipSuccess);
    fft.forward_as_torus(four, d_x.p, batch, st);
    EXPECT(hipStreamSynchronize(st) == hipSuccess);
    {  // serialised (natural) order and back: an exact permutation, out of place then in place
      double* nat = nullptr;
      EXPECT(hipMalloc(reinterpret_cast<void**>(&nat), batch * NF * 8) == hipSuccess);
      std::vector<double> h0(batch * NF), h1(batch * NF);
      EXPECT(hipMemcpy(h0.data(), four, batch * NF * 8, hipMemcpyDeviceToHost) == hipSuccess);
      fft.to_standard_order(nat, four, batch, st);
      fft.from_standard_order(nat, nat, batch, st);
      EXPECT(hipStreamSynchronize(st) == hipSuccess);
      EXPECT(hipMemcpy(h1.data(), nat, batch * NF * 8, hipMemcpyDeviceToHost) == hipSuccess);
      if (h0 != h1) {
        size_t bad = 0, first = 0;
        for (size_t i = 0; i < h0.size(); ++i)
          if (h0[i] != h1[i] && bad++ == 0) first = i;
        std::fprintf(stderr, "f64 standard-order round trip N = %zu (%s stream): %zu of %zu doubles differ, first at %zu\n",
                     NF, st ? "created" : "null", bad, h0.size(), first);
      }
      EXPECT(h0 == h1);
      (void)hipFree(nat);
    }
    fft.backward_as_torus(d_back.p, four, batch, false, st);
    const auto back = d_back.host();
    int64_t worst = 0;
    for (size_t i = 0; i < x.size(); ++i) {
      const int64_t d = (int64_t)(back[i] - x[i]);
      worst = std::max(worst, d < 0 ? -d : d);
    }
    EXPECT(worst < (int64_t(1) << 16));
    (void)hipFree(four);

    const int bl = 23;
    const auto ggsw = uniform(110, 0, 4 * NF), glwe = uniform(111, 0, 2 * NF), out0 = uniform(112, 0, 2 * NF);
    double* fg = nullptr;
    EXPECT(hipMalloc(reinterpret_cast<void**>(&fg), 4 * NF * 8) == hipSuccess);
    Dev d_g(ggsw), d_in(glwe), d_out(out0);
    tfhe_ntt_amd::fft64::convert_standard_lwe_bootstrap_key_to_fourier(fft, d_g.p, fg, 4, st);
    tfhe_ntt_amd::fft64::add_external_product_assign(fft, d_out.p, d_in.p, fg, bl, 1, 1, st);
    const auto got = d_out.host();
    // exact: decomposition digit (decomposer.rs, level 1) of each GLWE coefficient, negacyclic products mod 2^64
    std::vector<int64_t> dig(2 * NF);
    for (size_t i = 0; i < 2 * NF; ++i) {
      const uint64_t v = glwe[i];
      uint64_t res = v >> (64 - bl - 1);
      const uint64_t rb = res & 1;
      res = ((res + 1) >> 1) & ((1ull << bl) - 1);
      const uint64_t nb = (((res - 1) | (rb << (bl - 1))) & res) >> (bl - 1);
      const int64_t st = (int64_t)(res - (nb << bl));
      const uint64_t r = (uint64_t)st & ((1ull << bl) - 1);
      const uint64_t s2 = (uint64_t)(st >> bl);
      const uint64_t carry = (((r - 1) | s2) & r) >> (bl - 1);
      dig[i] = (int64_t)(r - (carry << bl));
    }
    worst = 0;
    for (int c = 0; c < 2; ++c)
      for (size_t e = 0; e < NF; ++e) {
        uint64_t acc = out0[c * NF + e];
        for (int r = 0; r < 2; ++r)
          for (size_t j = 0; j < NF; ++j) {  // coefficient e of X^j * G[r][c], times digit j of row r
            const size_t src = (e + NF - j) % NF;
            const uint64_t g = ggsw[(r * 2 + c) * NF + src];
            const uint64_t t = (uint64_t)dig[r * NF + j] * g;
            acc += (e >= j) ? t : (uint64_t)0 - t;
          }
        const int64_t d = (int64_t)(got[c * NF + e] - acc);
        worst = std::max(worst, d < 0 ? -d : d);
      }
    if (worst >= (int64_t(1) << (NF > 2048 ? 50 : 48)))
      std::fprintf(stderr, "f64 external product N = %zu (%s stream): worst |error| 2^%.2f\n", NF, st ? "created" : "null",
                   std::log2((double)worst));
    EXPECT(worst < (int64_t(1) << (NF > 2048 ? 50 : 48)));  // the f64 bound grows with sqrt(N log N)
    {  // the reference's FourierLweBootstrapKey bytes: write, load (a key owning its copy), write again: same bytes
      tfhe_ntt_amd::fft64::FourierBootstrapKey key(fft, fg, 1, bl, 1);
      for (const bool ver : {false, true}) {
        const auto bytes = key.serialize(ver);
        EXPECT(bytes.size() == (ver ? 8u : 0u) + 24 + 4 * (8 + 16 * (NF / 2)) + 32 + (ver ? 16u : 0u));
        const auto loaded = tfhe_ntt_amd::fft64::FourierBootstrapKey::load(fft, bytes.data(), bytes.size(), ver);
        EXPECT(loaded.input_lwe_dimension() == 1);
        EXPECT(loaded.serialize(ver) == bytes);
        bool threw = false;
        try {
          (void)tfhe_ntt_amd::fft64::FourierBootstrapKey::load(fft, bytes.data(), bytes.size() - 1, ver);
        } catch (const tfhe_ntt_amd::Error& e) {
          threw = e.status() == MI_ERR_INVALID_ARG;
        }
        EXPECT(threw);
      }
    }
    (void)hipFree(fg);
  }

  EXPECT(hipStreamDestroy(own) == hipSuccess);
  if (g_failures) {
    std::fprintf(stderr, "%d expectation(s) failed\n", g_failures);
    return 1;
  }
  std::printf("test_core_crypto: all tests passed\n");
  return 0;
}
