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
