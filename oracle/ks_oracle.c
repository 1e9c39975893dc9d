/*
 * ks_oracle.c — TEST INFRASTRUCTURE ONLY (see ks_oracle.h).
 * Restates the native-modulus LWE keyswitch of tfhe core_crypto
 * (reference paths relative to /root/reference/tfhe/src/core_crypto).
 */
#include "ks_oracle.h"

#include <string.h>

#include "pbs_oracle.h"

/* algorithms/lwe_keyswitch.rs:137-227 keyswitch_lwe_ciphertext_native_mod_compatible (native input
 * and output modulus): out = (0, ..., 0, b_in); for each input mask element a_i and each term of
 * SignedDecomposer::decompose(a_i) (decomposer.rs:219-227: init_decomposer_state, then iter.rs:103-119
 * yielding the least significant level first), out -= term * ksk_block_i[term index]
 * (slice_wrapping_sub_scalar_mul_assign, wrapping u64). */
void ora_lwe_keyswitch(const uint64_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                       const uint64_t *lwe_in, uint64_t *lwe_out) {
    const size_t out_size = out_dim + 1;
    memset(lwe_out, 0, out_size * sizeof(uint64_t));
    lwe_out[out_dim] = lwe_in[in_dim];
    for (size_t i = 0; i < in_dim; ++i) {
        uint64_t state = ora_decomp_init_native(lwe_in[i], base_log, level);
        const uint64_t *block = ksk + i * (size_t)level * out_size;
        for (int li = 0; li < level; ++li) {
            const uint64_t term = ora_decompose_one_level(base_log, &state);
            const uint64_t *row = block + (size_t)li * out_size;
            for (size_t j = 0; j < out_size; ++j) lwe_out[j] -= row[j] * term;
        }
    }
}

void ora_lwe_keyswitch_batch(const uint64_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                             const uint64_t *lwe_in, uint64_t *lwe_out, size_t batch, int threads) {
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
    for (size_t b = 0; b < batch; ++b)
        ora_lwe_keyswitch(ksk, in_dim, out_dim, base_log, level, lwe_in + b * (in_dim + 1),
                          lwe_out + b * (out_dim + 1));
}

/* decomposer.rs:25-49 native_closest_representable: round to the top level_count * base_log bits */
static uint64_t closest_representable64(uint64_t input, int level, int base_log) {
    const int shift = 64 - level * base_log - 1;
    uint64_t res = input >> shift;
    res += 1;
    res &= ~(uint64_t)1;
    return res << shift;
}

/* algorithms/lwe_keyswitch.rs:331-447 keyswitch_lwe_ciphertext_with_scalar_change.  The output is cleared, then its
 * body = SignedDecomposer::new(output_modulus_bits, 1).closest_representable(b) >> (64 - 32) (:417-426; the output
 * modulus bits are 32 for a native u32 modulus, log2 of the custom power of two otherwise, :406-412), and for each
 * input mask element and each term of the u64 SignedDecomposer (base_log, level) decomposition, out -= term.value()
 * cast to u32 * key row (slice_wrapping_sub_scalar_mul_assign: wrapping u32). */
void ora_lwe_keyswitch32(const uint32_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level, int out_mod_log,
                         const uint64_t *lwe_in, uint32_t *lwe_out) {
    const size_t out_size = out_dim + 1;
    memset(lwe_out, 0, out_size * sizeof(uint32_t));
    lwe_out[out_dim] = (uint32_t)(closest_representable64(lwe_in[in_dim], 1, out_mod_log) >> 32);
    for (size_t i = 0; i < in_dim; ++i) {
        uint64_t state = ora_decomp_init_native(lwe_in[i], base_log, level);
        const uint32_t *block = ksk + i * (size_t)level * out_size;
        for (int li = 0; li < level; ++li) {
            const uint32_t term = (uint32_t)ora_decompose_one_level(base_log, &state);
            const uint32_t *row = block + (size_t)li * out_size;
            for (size_t j = 0; j < out_size; ++j) lwe_out[j] -= row[j] * term;
        }
    }
}

void ora_lwe_keyswitch32_batch(const uint32_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                               int out_mod_log, const uint64_t *lwe_in, uint32_t *lwe_out, size_t batch, int threads) {
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
    for (size_t b = 0; b < batch; ++b)
        ora_lwe_keyswitch32(ksk, in_dim, out_dim, base_log, level, out_mod_log, lwe_in + b * (in_dim + 1),
                            lwe_out + b * (out_dim + 1));
}

/* fft_impl/common.rs:10-23 modulus_switch at Scalar = u32 */
static uint32_t modulus_switch32(uint32_t input, int log_mod) {
    if (log_mod == 32) return input;
    const uint32_t to_floor = input + (1u << (32 - log_mod - 1));
    return to_floor >> (32 - log_mod);
}

/* modulus_switch.rs:35-104 (centered_binary_ms_body_correction_to_add at Scalar = u32, Signed = i32: Rust's `/` on
 * i32 truncates toward zero, as C's) and the lazy switched ciphertext's body / mask (modulus_switched_lwe_ciphertext.rs
 * :150-172). */
void ora_lwe_ms32(const uint32_t *lwe, size_t dim, int log_mod, int centered, uint64_t *out) {
    uint32_t correction = 0;
    if (centered) {
        uint32_t sum_half_mask_round_errors = 0;
        int32_t sum_halving_errors_doubled = 0;
        for (size_t i = 0; i < dim; ++i) {
            const uint32_t a = lwe[i];
            const uint32_t round = log_mod == 32 ? modulus_switch32(a, log_mod)
                                                 : modulus_switch32(a, log_mod) << (32 - log_mod);
            const uint32_t error = round - a;
            const int32_t signed_error = (int32_t)error;
            const int32_t half_error = signed_error / 2;
            const int32_t halving_error_doubled = 2 * half_error - signed_error;
            sum_half_mask_round_errors += (uint32_t)half_error;
            sum_halving_errors_doubled += halving_error_doubled;
        }
        const uint32_t sum_halving_errors = (uint32_t)(sum_halving_errors_doubled / 2);
        sum_half_mask_round_errors -= sum_halving_errors;
        const uint32_t half_case = log_mod == 32 ? 0u : 1u << (32 - log_mod - 1);
        correction = sum_half_mask_round_errors - half_case;
    }
    for (size_t i = 0; i < dim; ++i) out[i] = modulus_switch32(lwe[i], log_mod);
    out[dim] = modulus_switch32(lwe[dim] + correction, log_mod);
}
