// tfhe_ntt_amd.hpp — header-only C++17 mirror of tfhe_ntt::prime64::Plan over the C ABI.
//
// The host-side surface a compiled caller binds (the reference is Rust; its toolchain is absent from
// this image, so the compiled host mirror is C++).  Names, argument meaning and error behaviour follow
// tfhe-ntt/src/prime64.rs (paths relative to /root/reference):
//   Plan::try_new(n, p)          prime64.rs:764-862  -> std::optional<Plan> (nullopt where the reference
//                                                       returns None; HIP failures throw tfhe_ntt_amd::Error)
//   ntt_size() / modulus()       prime64.rs:870-878
//   fwd / inv (&mut [u64])       prime64.rs:897-1046 -> host slices of exactly n values; a length mismatch
//                                                       throws std::invalid_argument where the reference
//                                                       panics on assert_eq! (prime64.rs:898, 976)
//   normalize / mul_assign_normalize / mul_accumulate   prime64.rs:1050-1222 (host slices, same rule)
// plus the batched device-pointer forms (`*_batch`, async on a hipStream_t passed as void*) that the
// GPU path is built for.  The plan is immutable and may be shared by threads and streams; it is
// move-only (the C handle is owned).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "tfhe_ntt_amd.h"

namespace tfhe_ntt_amd {

class Error : public std::runtime_error {
 public:
  Error(int status, const std::string& what) : std::runtime_error(what), status_(status) {}
  int status() const noexcept { return status_; }

 private:
  int status_;
};

inline void check(int status) {
  if (status != MI_OK)
    throw Error(status, std::string(mi_status_string(status)) + ": " + mi_last_error_message());
}

namespace prime64 {

class Plan {
 public:
  // prime64.rs:764-862: None for N < 16 / not a power of two / p not prime / no 2N-th root
  static std::optional<Plan> try_new(size_t polynomial_size, uint64_t modulus, int device = 0) {
    mi_ntt64_plan* raw = nullptr;
    const int st = mi_ntt64_plan_create(polynomial_size, modulus, device, &raw);
    if (st == MI_ERR_INVALID_ARG || st == MI_ERR_NOT_PRIME || st == MI_ERR_NO_ROOT) return std::nullopt;
    check(st);
    return Plan(raw, polynomial_size, modulus);
  }

  Plan(Plan&& o) noexcept : raw_(std::exchange(o.raw_, nullptr)), n_(o.n_), p_(o.p_) {}
  Plan& operator=(Plan&& o) noexcept {
    if (this != &o) {
      reset();
      raw_ = std::exchange(o.raw_, nullptr);
      n_ = o.n_;
      p_ = o.p_;
    }
    return *this;
  }
  Plan(const Plan&) = delete;
  Plan& operator=(const Plan&) = delete;
  ~Plan() { reset(); }

  size_t ntt_size() const noexcept { return n_; }
  uint64_t modulus() const noexcept { return p_; }
  const mi_ntt64_plan* raw() const noexcept { return raw_; }

  // ---- host slices (&mut [u64] of exactly ntt_size() values) ----------------------------------
  void fwd(uint64_t* buf, size_t len) const {
    require(len);
    check(mi_ntt64_fwd_host(raw_, buf, 1));
  }
  void inv(uint64_t* buf, size_t len) const {
    require(len);
    check(mi_ntt64_inv_host(raw_, buf, 1));
  }
  // the pointwise ops on host slices go through the library's pooled staging slots (mi_ntt64_*_host): no device
  // allocation and no device-wide synchronisation per call
  void normalize(uint64_t* buf, size_t len) const {
    require(len);
    check(mi_ntt64_normalize_host(raw_, buf, 1));
  }
  void mul_assign_normalize(uint64_t* lhs, size_t lhs_len, const uint64_t* rhs, size_t rhs_len) const {
    require(lhs_len);
    require(rhs_len);
    check(mi_ntt64_mul_assign_normalize_host(raw_, lhs, rhs, 1));
  }
  void mul_accumulate(uint64_t* acc, size_t acc_len, const uint64_t* lhs, size_t lhs_len, const uint64_t* rhs,
                      size_t rhs_len) const {
    require(acc_len);
    require(lhs_len);
    require(rhs_len);
    check(mi_ntt64_mul_accumulate_host(raw_, acc, lhs, rhs, 1));
  }

  // ---- device batches (batch polynomials, `stride` u64 apart), async on `stream` ---------------
  void fwd_batch(uint64_t* dev, size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_fwd_batch(raw_, dev, batch, stride, stream));
  }
  void inv_batch(uint64_t* dev, size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_inv_batch(raw_, dev, batch, stride, stream));
  }
  void normalize_batch(uint64_t* dev, size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_normalize_batch(raw_, dev, batch, stride, stream));
  }
  void mul_assign_normalize_batch(uint64_t* lhs, const uint64_t* rhs, size_t batch, size_t stride,
                                  void* stream = nullptr) const {
    check(mi_ntt64_mul_assign_normalize_batch(raw_, lhs, rhs, batch, stride, stream));
  }
  void mul_accumulate_batch(uint64_t* acc, const uint64_t* lhs, const uint64_t* rhs, size_t batch, size_t stride,
                            void* stream = nullptr) const {
    check(mi_ntt64_mul_accumulate_batch(raw_, acc, lhs, rhs, batch, stride, stream));
  }

 private:
  Plan(mi_ntt64_plan* raw, size_t n, uint64_t p) : raw_(raw), n_(n), p_(p) {}
  void reset() noexcept {
    if (raw_) (void)mi_ntt64_plan_destroy(raw_);
    raw_ = nullptr;
  }
  void require(size_t len) const {
    if (len != n_)
      throw std::invalid_argument("assertion `left == right` failed: slice length " + std::to_string(len) +
                                  " != ntt_size " + std::to_string(n_));
  }

  mi_ntt64_plan* raw_ = nullptr;
  size_t n_ = 0;
  uint64_t p_ = 0;
};

}  // namespace prime64

// ---- core_crypto consumers (tfhe/src/core_crypto, device pointers, async on `stream`) ----------
// The reference works on one ciphertext per call; every function here takes a leading batch.
// Layouts as in tfhe_ntt_amd.h.  Variants: MI_NTT64_SOLINAS / MI_NTT64_BNF.
namespace core_crypto {

// Ntt64View (commons/math/ntt/ntt64.rs:80-266): the per-polynomial helpers of every NTT consumer, over `batch`
// polynomials `stride` u64 apart in both operands (device pointers).  Argument order as the reference's; add_backward*
// leave `ntt` holding the inverse (switched for the power-of-two form), as Plan::inv in place does.
class Ntt64View {
 public:
  explicit Ntt64View(const prime64::Plan& plan) : plan_(plan.raw()), n_(plan.ntt_size()), p_(plan.modulus()) {}
  size_t polynomial_size() const noexcept { return n_; }
  uint64_t custom_modulus() const noexcept { return p_; }
  void forward(uint64_t* ntt, const uint64_t* standard, size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_forward_batch(plan_, ntt, standard, batch, stride, stream));
  }
  void forward_normalized(uint64_t* ntt, const uint64_t* standard, size_t batch, size_t stride,
                          void* stream = nullptr) const {
    check(mi_ntt64_forward_normalized_batch(plan_, ntt, standard, batch, stride, stream));
  }
  void add_backward(uint64_t* standard, uint64_t* ntt, size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_add_backward_batch(plan_, standard, ntt, batch, stride, stream));
  }
  void forward_from_power_of_two_modulus(unsigned input_modulus_width, uint64_t* ntt, const uint64_t* standard,
                                         size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_forward_from_power_of_two_modulus_batch(plan_, input_modulus_width, ntt, standard, batch, stride,
                                                           stream));
  }
  void forward_from_decomp(uint64_t* ntt, const uint64_t* decomp, size_t batch, size_t stride,
                           void* stream = nullptr) const {
    check(mi_ntt64_forward_from_decomp_batch(plan_, ntt, decomp, batch, stride, stream));
  }
  void add_backward_on_power_of_two_modulus(unsigned output_modulus_width, uint64_t* standard, uint64_t* ntt,
                                            size_t batch, size_t stride, void* stream = nullptr) const {
    check(mi_ntt64_add_backward_on_power_of_two_modulus_batch(plan_, output_modulus_width, standard, ntt, batch,
                                                              stride, stream));
  }

 private:
  const mi_ntt64_plan* plan_;
  size_t n_;
  uint64_t p_;
};

// algorithms/lwe_bootstrap_key_conversion.rs:294-365 (Raw: normalize = false)
inline void convert_standard_lwe_bootstrap_key_to_ntt64(const prime64::Plan& plan, const uint64_t* bsk_std,
                                                        uint64_t* bsk_ntt, size_t n_polys, unsigned in_modulus_width,
                                                        bool normalize, void* stream = nullptr) {
  check(mi_bsk_to_ntt64(plan.raw(), bsk_std, bsk_ntt, n_polys, in_modulus_width, normalize ? 1 : 0, stream));
}

// ntt64_pbs.rs:553-663 / ntt64_bnf_pbs.rs:541-681: out[b] += GGSW (.) glwe[b]; `glwe_dimension` = k
inline void add_external_product_ntt64_assign(const prime64::Plan& plan, uint64_t* out, const uint64_t* glwe,
                                              const uint64_t* ggsw_ntt, int base_log, int level, size_t batch,
                                              int variant, void* stream = nullptr, int glwe_dimension = 1) {
  check(mi_ext_product_ntt64_batch(plan.raw(), out, glwe, ggsw_ntt, glwe_dimension, base_log, level, batch, variant,
                                   stream));
}

// ntt64_pbs.rs:669-680 / ntt64_bnf_pbs.rs:683-705 (ct1 is left holding ct1 - ct0, as the reference)
inline void cmux_ntt64_assign(const prime64::Plan& plan, uint64_t* ct0, uint64_t* ct1, const uint64_t* ggsw_ntt,
                              int base_log, int level, size_t batch, int variant, void* stream = nullptr,
                              int glwe_dimension = 1) {
  check(mi_cmux_ntt64_batch(plan.raw(), ct0, ct1, ggsw_ntt, glwe_dimension, base_log, level, batch, variant, stream));
}

// An NTT-domain bootstrap key bound to a plan (entities/ntt_lwe_bootstrap_key.rs); move-only.
class NttBootstrapKey {
 public:
  // `stream`: the stream that produced bsk_ntt (the BNF preparation is ordered after it)
  NttBootstrapKey(const prime64::Plan& plan, const uint64_t* bsk_ntt, size_t n_lwe, int base_log, int level,
                  int variant, void* stream = nullptr, int glwe_dimension = 1)
      : n_lwe_(n_lwe), variant_(variant) {
    check(mi_pbs_ntt64_key_create(plan.raw(), bsk_ntt, n_lwe, glwe_dimension, base_log, level, variant, stream, &raw_));
  }
  // Serialised key bytes (MI_NTT_BSK_PLAIN / MI_NTT_BSK_VERSIONED) loaded straight into HBM
  // (mi_pbs_ntt64_key_load); `variant` is explicit: Raw (BNF) and Normalize (Solinas) keys store the same fields.
  static NttBootstrapKey load(const prime64::Plan& plan, const uint8_t* bytes, size_t len, int variant,
                              int format = MI_NTT_BSK_PLAIN, void* stream = nullptr) {
    mi_pbs_ntt64_key* raw = nullptr;
    check(mi_pbs_ntt64_key_load(plan.raw(), bytes, len, format, variant, stream, &raw));
    NttBootstrapKey key(raw, 0, variant);  // owns the upload before anything else can throw
    check(mi_pbs_ntt64_key_info(raw, &key.n_lwe_, nullptr, nullptr, nullptr, nullptr));
    return key;
  }
  NttBootstrapKey(NttBootstrapKey&& o) noexcept
      : raw_(std::exchange(o.raw_, nullptr)), n_lwe_(o.n_lwe_), variant_(o.variant_) {}
  NttBootstrapKey(const NttBootstrapKey&) = delete;
  NttBootstrapKey& operator=(const NttBootstrapKey&) = delete;
  ~NttBootstrapKey() {
    if (raw_) (void)mi_pbs_ntt64_key_destroy(raw_);
  }
  const mi_pbs_ntt64_key* raw() const noexcept { return raw_; }
  size_t input_lwe_dimension() const noexcept { return n_lwe_; }
  int variant() const noexcept { return variant_; }

 private:
  NttBootstrapKey(mi_pbs_ntt64_key* raw, size_t n_lwe, int variant) : raw_(raw), n_lwe_(n_lwe), variant_(variant) {}
  mi_pbs_ntt64_key* raw_ = nullptr;
  size_t n_lwe_;
  int variant_;
};

// programmable_bootstrap_ntt64[_bnf]_lwe_ciphertext_mem_optimized (ntt64_pbs.rs:482-538,
// ntt64_bnf_pbs.rs:469-540): lwe_out[b] (k N + 1) = PBS(lwe_in[b] (n + 1)) with the accumulator `lut`
inline void programmable_bootstrap_ntt64_lwe_ciphertext(const NttBootstrapKey& key, const uint64_t* lwe_in,
                                                        uint64_t* lwe_out, const uint64_t* lut, size_t batch,
                                                        int ms_mode = MI_MS_STANDARD, void* stream = nullptr) {
  check(mi_pbs_ntt64_batch(key.raw(), lwe_out, lwe_in, lut, batch, ms_mode, stream));
}

// the same with one LUT per item: item b uses GLWE lut_index[b] (device u32) of the n_lut in lut_list
inline void programmable_bootstrap_ntt64_lwe_ciphertext_lut_indexed(const NttBootstrapKey& key, const uint64_t* lwe_in,
                                                                    uint64_t* lwe_out, const uint64_t* lut_list,
                                                                    const uint32_t* lut_index, size_t n_lut,
                                                                    size_t batch, int ms_mode = MI_MS_STANDARD,
                                                                    void* stream = nullptr) {
  check(mi_pbs_ntt64_batch_lut_indexed(key.raw(), lwe_out, lwe_in, lut_list, lut_index, n_lut, batch, ms_mode,
                                       stream));
}

// blind_rotate_ntt64[_bnf]_assign (ntt64_pbs.rs:176-286 / ntt64_bnf_pbs.rs:174-266), batched and in place: every item
// rotates its own accumulator acc_glwe[b] ((k+1) N u64) by lwe_in[b]
inline void blind_rotate_ntt64_assign(const NttBootstrapKey& key, const uint64_t* lwe_in, uint64_t* acc_glwe,
                                      size_t batch, int ms_mode = MI_MS_STANDARD, void* stream = nullptr) {
  check(mi_blind_rotate_ntt64_batch(key.raw(), acc_glwe, lwe_in, batch, ms_mode, stream));
}

// extract_lwe_sample_from_glwe_ciphertext (glwe_sample_extraction.rs:89-160) at MonomialDegree(nth + j nth_stride),
// j < nth_count, of every GLWE in a batch; modulus 0 = native
inline void extract_lwe_sample_from_glwe_ciphertext(const uint64_t* glwe, uint64_t* lwe_out, size_t polynomial_size,
                                                    int glwe_dimension, size_t batch, size_t nth, size_t nth_stride = 0,
                                                    size_t nth_count = 1, uint64_t modulus = 0, int device = 0,
                                                    void* stream = nullptr) {
  check(mi_sample_extract_batch(lwe_out, glwe, polynomial_size, glwe_dimension, batch, nth, nth_stride, nth_count,
                                modulus, device, stream));
}

// entities/lwe_keyswitch_key.rs + algorithms/lwe_keyswitch.rs:103-227 (native modulus); move-only
class LweKeyswitchKey {
 public:
  LweKeyswitchKey(const uint64_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level, int device = 0,
                  void* stream = nullptr)
      : in_(in_dim), out_(out_dim) {
    check(mi_lwe_ksk_create(ksk, in_dim, out_dim, base_log, level, device, stream, &raw_));
  }
  LweKeyswitchKey(LweKeyswitchKey&& o) noexcept : raw_(std::exchange(o.raw_, nullptr)), in_(o.in_), out_(o.out_) {}
  LweKeyswitchKey(const LweKeyswitchKey&) = delete;
  LweKeyswitchKey& operator=(const LweKeyswitchKey&) = delete;
  ~LweKeyswitchKey() {
    if (raw_) (void)mi_lwe_ksk_destroy(raw_);
  }
  const mi_lwe_ksk* raw() const noexcept { return raw_; }
  size_t input_key_lwe_dimension() const noexcept { return in_; }
  size_t output_key_lwe_dimension() const noexcept { return out_; }

 private:
  mi_lwe_ksk* raw_ = nullptr;
  size_t in_, out_;
};

inline void keyswitch_lwe_ciphertext(const LweKeyswitchKey& key, const uint64_t* lwe_in, uint64_t* lwe_out,
                                     size_t batch, void* stream = nullptr) {
  check(mi_lwe_keyswitch_batch(key.raw(), lwe_out, lwe_in, batch, stream));
}

// LweKeyswitchKey<Vec<u32>> of the KS32 parameter sets (shortint/parameters/v1_5/hpu.rs:57-76); move-only
class LweKeyswitchKey32 {
 public:
  LweKeyswitchKey32(const uint32_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level, int out_modulus_log,
                    int device = 0, void* stream = nullptr)
      : in_(in_dim), out_(out_dim) {
    check(mi_lwe_ksk32_create(ksk, in_dim, out_dim, base_log, level, out_modulus_log, device, stream, &raw_));
  }
  LweKeyswitchKey32(LweKeyswitchKey32&& o) noexcept : raw_(std::exchange(o.raw_, nullptr)), in_(o.in_), out_(o.out_) {}
  LweKeyswitchKey32(const LweKeyswitchKey32&) = delete;
  LweKeyswitchKey32& operator=(const LweKeyswitchKey32&) = delete;
  ~LweKeyswitchKey32() {
    if (raw_) (void)mi_lwe_ksk32_destroy(raw_);
  }
  const mi_lwe_ksk32* raw() const noexcept { return raw_; }
  size_t input_key_lwe_dimension() const noexcept { return in_; }
  size_t output_key_lwe_dimension() const noexcept { return out_; }

 private:
  mi_lwe_ksk32* raw_ = nullptr;
  size_t in_, out_;
};

// keyswitch_lwe_ciphertext_with_scalar_change (lwe_keyswitch.rs:331-447) over a batch: u64 in, u32 out
inline void keyswitch_lwe_ciphertext_with_scalar_change(const LweKeyswitchKey32& key, const uint64_t* lwe_in,
                                                        uint32_t* lwe_out, size_t batch, void* stream = nullptr) {
  check(mi_lwe_keyswitch32_batch(key.raw(), lwe_out, lwe_in, batch, stream));
}

// lwe_ciphertext_[centered_binary_]modulus_switch of u32 LWEs (modulus_switch.rs:14-104), materialised into
// [0, 2^log_modulus) u64 values: the MI_MS_PRE_SWITCHED input of the blind rotation
inline void lwe_ciphertext_modulus_switch32(const uint32_t* lwe_in, uint64_t* switched, size_t lwe_dimension,
                                            size_t batch, int log_modulus, bool centered, int device = 0,
                                            void* stream = nullptr) {
  check(mi_lwe_modulus_switch32_batch(switched, lwe_in, lwe_dimension, batch, log_modulus,
                                      centered ? MI_MS_CENTERED : MI_MS_STANDARD, device, stream));
}

// the same switch of u64 LWEs (the native-modulus ciphertexts in front of every other blind rotation)
inline void lwe_ciphertext_modulus_switch(const uint64_t* lwe_in, uint64_t* switched, size_t lwe_dimension,
                                          size_t batch, int log_modulus, bool centered, int device = 0,
                                          void* stream = nullptr) {
  check(mi_lwe_modulus_switch_batch(switched, lwe_in, lwe_dimension, batch, log_modulus,
                                    centered ? MI_MS_CENTERED : MI_MS_STANDARD, device, stream));
}

// On-disk NTT bootstrap key (entities/ntt_lwe_bootstrap_key.rs:26-33): plain bincode or the versioned
// form, parsed and written by the library (mi_ntt_bsk_parse / mi_ntt_bsk_write, pure host code, no
// device needed); the layouts are documented in include/tfhe_ntt_amd.h.  Same bytes as
// tfhe_ntt_amd/ntt_bsk_format.py.
using NttBskFields = mi_ntt_bsk_header;

inline std::vector<uint8_t> serialize_ntt_bsk(const uint64_t* data, size_t count, NttBskFields f,
                                              int format = MI_NTT_BSK_PLAIN) {
  f.count = count;
  size_t len = 0;
  check(mi_ntt_bsk_serialized_size(&f, format, &len));
  std::vector<uint8_t> out(len);
  const int st = mi_ntt_bsk_write(&f, data, format, out.data(), out.size());
  if (st == MI_ERR_INVALID_ARG) throw std::invalid_argument(mi_last_error_message());
  check(st);
  return out;
}

// Throws std::invalid_argument on malformed bytes (see mi_ntt_bsk_parse).
inline NttBskFields deserialize_ntt_bsk(const uint8_t* buf, size_t len, std::vector<uint64_t>& data,
                                        int format = MI_NTT_BSK_PLAIN) {
  NttBskFields f{};
  const int st = mi_ntt_bsk_parse(buf, len, format, &f);
  if (st == MI_ERR_INVALID_ARG) throw std::invalid_argument(mi_last_error_message());
  check(st);
  data.resize(f.count);
  if (f.count) std::memcpy(data.data(), buf + f.data_offset, f.count * sizeof(uint64_t));
  return f;
}

}  // namespace core_crypto

// ---- the f64-FFT path (tfhe/src/core_crypto/fft_impl/fft64, algorithms/lwe_programmable_bootstrapping/
// fft64_pbs.rs): Fourier buffers are interleaved (re, im) doubles in the engine's frequency order ------------
namespace fft64 {

// Fft::new (fft_impl/fft64/math/fft/mod.rs:170-223): the process-wide plan of a polynomial size on a device.
class Fft {
 public:
  explicit Fft(size_t polynomial_size, int device = 0) { check(mi_fft64_plan_cached(polynomial_size, device, &raw_)); }
  const mi_fft64_plan* raw() const noexcept { return raw_; }
  // FftView::forward_as_torus / backward_as_torus / add_backward_as_torus over `batch` polynomials
  void forward_as_torus(double* fourier, const uint64_t* standard, size_t batch, void* stream = nullptr) const {
    check(mi_fft64_forward_torus_batch(raw_, fourier, standard, batch, stream));
  }
  void backward_as_torus(uint64_t* standard, const double* fourier, size_t batch, bool add = false,
                         void* stream = nullptr) const {
    check(mi_fft64_backward_torus_batch(raw_, standard, fourier, batch, add ? 1 : 0, stream));
  }
  // the reference's serialised natural order (tfhe-fft/src/unordered.rs:943-1020) <-> this engine's order
  void to_standard_order(double* standard_order, const double* fourier, size_t polys, void* stream = nullptr) const {
    check(mi_fft64_to_standard_order(raw_, standard_order, fourier, polys, stream));
  }
  void from_standard_order(double* fourier, const double* standard_order, size_t polys, void* stream = nullptr) const {
    check(mi_fft64_from_standard_order(raw_, fourier, standard_order, polys, stream));
  }

 private:
  const mi_fft64_plan* raw_ = nullptr;
};

// convert_standard_lwe_bootstrap_key_to_fourier (algorithms/lwe_bootstrap_key_conversion.rs:20-43)
inline void convert_standard_lwe_bootstrap_key_to_fourier(const Fft& fft, const uint64_t* bsk_std, double* bsk_fourier,
                                                          size_t n_polys, void* stream = nullptr) {
  check(mi_bsk_to_fourier64(fft.raw(), bsk_std, bsk_fourier, n_polys, stream));
}

// add_external_product_assign / cmux_assign (fft64_pbs.rs:270-330, 510-560)
inline void add_external_product_assign(const Fft& fft, uint64_t* out, const uint64_t* glwe, const double* ggsw_fourier,
                                        int base_log, int level, size_t batch, void* stream = nullptr,
                                        int glwe_dimension = 1) {
  check(mi_fft64_ext_product_batch(fft.raw(), out, glwe, ggsw_fourier, glwe_dimension, base_log, level, batch, stream));
}
inline void cmux_assign(const Fft& fft, uint64_t* ct0, uint64_t* ct1, const double* ggsw_fourier, int base_log,
                        int level, size_t batch, void* stream = nullptr, int glwe_dimension = 1) {
  check(mi_fft64_cmux_batch(fft.raw(), ct0, ct1, ggsw_fourier, glwe_dimension, base_log, level, batch, stream));
}

// FourierLweBootstrapKey bound to a plan (the Fourier key buffer is referenced; keep it alive); move-only
class FourierBootstrapKey {
 public:
  FourierBootstrapKey(const Fft& fft, const double* fbsk, size_t n_lwe, int base_log, int level,
                      int glwe_dimension = 1)
      : n_lwe_(n_lwe) {
    check(mi_fft64_plan_info(fft.raw(), &n_, nullptr));
    check(mi_fft64_pbs_key_create(fft.raw(), fbsk, n_lwe, glwe_dimension, base_log, level, &raw_));
  }
  FourierBootstrapKey(FourierBootstrapKey&& o) noexcept
      : raw_(std::exchange(o.raw_, nullptr)), n_lwe_(o.n_lwe_), n_(o.n_) {}
  FourierBootstrapKey(const FourierBootstrapKey&) = delete;
  FourierBootstrapKey& operator=(const FourierBootstrapKey&) = delete;
  ~FourierBootstrapKey() {
    if (raw_) (void)mi_fft64_pbs_key_destroy(raw_);
  }
  const mi_fft64_pbs_key* raw() const noexcept { return raw_; }
  size_t input_lwe_dimension() const noexcept { return n_lwe_; }

  // the reference's FourierLweBootstrapKey bytes (plain or versioned bincode) -> a key owning its device copy
  static FourierBootstrapKey load(const Fft& fft, const uint8_t* bytes, size_t len, bool versioned = false,
                                  void* stream = nullptr) {
    mi_fft64_pbs_key* k = nullptr;
    check(mi_fft64_pbs_key_load(fft.raw(), bytes, len, versioned ? MI_NTT_BSK_VERSIONED : MI_NTT_BSK_PLAIN, stream, &k));
    FourierBootstrapKey key(k, 0);  // owns the upload before anything else can throw
    check(mi_fft64_pbs_key_info(k, &key.n_lwe_, nullptr, nullptr, nullptr));
    check(mi_fft64_plan_info(fft.raw(), &key.n_, nullptr));
    return key;
  }
  // this key as the reference's bytes
  std::vector<uint8_t> serialize(bool versioned = false, void* stream = nullptr) const {
    const int fmt = versioned ? MI_NTT_BSK_VERSIONED : MI_NTT_BSK_PLAIN;
    int k = 0, level = 0;
    check(mi_fft64_pbs_key_info(raw_, nullptr, &k, nullptr, &level));
    size_t len = 0;
    check(mi_fft64_bsk_serialized_size(n_, n_lwe_, k, level, fmt, &len));
    std::vector<uint8_t> out(len);
    check(mi_fft64_pbs_key_write(raw_, fmt, out.data(), out.size(), stream));
    return out;
  }

 private:
  FourierBootstrapKey(mi_fft64_pbs_key* raw, size_t n_lwe) : raw_(raw), n_lwe_(n_lwe) {}
  mi_fft64_pbs_key* raw_ = nullptr;
  size_t n_lwe_;
  size_t n_ = 0;  // polynomial size of the plan
};

// programmable_bootstrap_lwe_ciphertext (fft64_pbs.rs:924-1060) over a batch
inline void programmable_bootstrap_lwe_ciphertext(const FourierBootstrapKey& key, const uint64_t* lwe_in,
                                                  uint64_t* lwe_out, const uint64_t* lut, size_t batch,
                                                  int ms_mode = MI_MS_STANDARD, void* stream = nullptr) {
  check(mi_fft64_pbs_batch(key.raw(), lwe_out, lwe_in, lut, batch, ms_mode, stream));
}

}  // namespace fft64
}  // namespace tfhe_ntt_amd
