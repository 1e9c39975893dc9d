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

#ifdef __cplusplus
}
#endif
#endif
