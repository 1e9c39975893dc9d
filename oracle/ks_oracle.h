/*
 * ks_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the LWE keyswitch that precedes the PBS in the shortint KS-PBS order
 * (reference: /root/reference/tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs).  Only tests/,
 * smoke() and bench's CPU leg use it.
 *
 * Layouts (u64, native 2^64 modulus):
 *   LWE : dimension mask elements then the body
 *   KSK : in_dim blocks x level LWE ciphertexts of out_dim + 1 u64; within block i, ciphertext li
 *         encrypts s_in[i] * 2^(64 - base_log * (level - li))  (lwe_keyswitch_key_generation.rs:169-199:
 *         levels stored from level_count down to 1, the order SignedDecompositionIter yields them)
 */
#ifndef KS_ORACLE_H
#define KS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

void ora_lwe_keyswitch(const uint64_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                       const uint64_t *lwe_in, uint64_t *lwe_out);
/* OpenMP over `batch` ciphertexts (the reference's par_keyswitch_lwe_ciphertext splits one
 * ciphertext; here independent ciphertexts are spread, as the benchmark harness does). */
void ora_lwe_keyswitch_batch(const uint64_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                             const uint64_t *lwe_in, uint64_t *lwe_out, size_t batch, int threads);

/* KS32: algorithms/lwe_keyswitch.rs:331-447 keyswitch_lwe_ciphertext_with_scalar_change, InputScalar = u64 (native
 * modulus), OutputScalar = u32 with the power-of-two modulus 2^out_mod_log (values in the MSBs).  KSK: in_dim blocks x
 * level u32 LWE ciphertexts of out_dim + 1 words (levels as above).  Output: out_dim + 1 u32. */
void ora_lwe_keyswitch32(const uint32_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level, int out_mod_log,
                         const uint64_t *lwe_in, uint32_t *lwe_out);
void ora_lwe_keyswitch32_batch(const uint32_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                               int out_mod_log, const uint64_t *lwe_in, uint32_t *lwe_out, size_t batch, int threads);
/* algorithms/modulus_switch.rs:14-104 lwe_ciphertext_[centered_binary_]modulus_switch at Scalar = u32, read out as
 * entities/modulus_switched_lwe_ciphertext.rs:150-175 does: out[i] = modulus_switch(a_i) for the dim mask words and
 * out[dim] = modulus_switch(b + correction) (correction 0 unless centered), each in [0, 2^log_mod). */
void ora_lwe_ms32(const uint32_t *lwe, size_t dim, int log_mod, int centered, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
