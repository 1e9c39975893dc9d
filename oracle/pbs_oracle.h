/*
 * pbs_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the core_crypto consumers of the NTT (reference paths relative to
 * /root/reference/tfhe/src/core_crypto): the GGSW x GLWE external product, CMUX, blind rotation
 * and programmable bootstrap in both NTT flavours —
 *   * "Solinas" : ciphertexts modulo the NTT prime  (algorithms/lwe_programmable_bootstrapping/ntt64_pbs.rs)
 *   * "BNF"     : native 2^64 ciphertexts, back-and-forth modulus switch to the prime
 *                 (algorithms/lwe_programmable_bootstrapping/ntt64_bnf_pbs.rs)
 * plus the modulus switches and BSK conversion around them (commons/math/ntt/ntt64.rs,
 * algorithms/lwe_bootstrap_key_conversion.rs).  Only tests/, smoke() and bench's CPU leg use it.
 *
 * Layouts (u64 everywhere, N = polynomial size, k = GLWE dimension, l = levels):
 *   GLWE      : (k+1) polynomials x N              (mask polys then body)
 *   NTT GGSW  : l levels (highest level first) x (k+1) rows x (k+1) polys x N  (ntt_ggsw_ciphertext.rs:176-192)
 *   NTT BSK   : n_lwe GGSWs back to back
 *   LWE       : n mask elements then the body
 * `plan` arguments are the oracle plan tables (twid, inv_twid, n_inv) for (N, p).
 */
#ifndef PBS_ORACLE_H
#define PBS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_ntt_tables {
    size_t n;
    uint64_t p;
    const uint64_t *twid;
    const uint64_t *inv_twid;
    uint64_t n_inv;
} ora_ntt_tables;

/* decomposer.rs:156-185 SignedDecomposer::init_decomposer_state (native u64) */
uint64_t ora_decomp_init_native(uint64_t input, int base_log, int level);
/* iter.rs:141-151 decompose_one_level; returns the term, updates *state */
uint64_t ora_decompose_one_level(int base_log, uint64_t *state);

/* ntt64.rs:166-178 / 184-197 */
uint64_t ora_modswitch_p2_to_prime(uint64_t v, unsigned width, uint64_t p);
uint64_t ora_modswitch_prime_to_p2(uint64_t v, unsigned width, uint64_t p);

/* the Ntt64View layer (ntt64.rs:89-266): kind 0 forward[_normalized], 1 forward_from_power_of_two_modulus(width),
 * 2 forward_from_decomp; add_backward (width 0) / add_backward_on_power_of_two_modulus(width) */
void ora_ntt64_view_forward_batch(const ora_ntt_tables *t, int kind, unsigned width, int normalize, uint64_t *ntt,
                                  const uint64_t *standard, size_t batch, size_t stride, int threads);
void ora_ntt64_view_add_backward_batch(const ora_ntt_tables *t, unsigned width, uint64_t *standard, uint64_t *ntt,
                                       size_t batch, size_t stride, int threads);
/* algorithms/modulus_switch.rs:14-104 at Scalar = u64, materialised (dim mask values, then the body) */
void ora_lwe_ms64(const uint64_t *lwe, size_t dim, unsigned log_mod, int centered, uint64_t *out);
uint64_t ora_centered_ms_body_correction(const uint64_t *mask, size_t n_lwe, unsigned log_modulus);
uint64_t ora_modulus_switch(uint64_t input, unsigned log_modulus);

/* ntt64_bnf_pbs.rs:541-681: out += GGSW (.) glwe  (native modulus) */
void ora_ext_product_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *out,
                         const uint64_t *ggsw, const uint64_t *glwe);
/* ntt64_pbs.rs:553-663: out += GGSW (.) glwe  (ciphertexts mod p) */
void ora_ext_product_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *out,
                             const uint64_t *ggsw, const uint64_t *glwe);

/* ntt64_bnf_pbs.rs:683-705 / ntt64_pbs.rs:669-680: ct0 <- ct0 + GGSW (.) (ct1 - ct0); ct1 is clobbered */
void ora_cmux_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *ct0, uint64_t *ct1,
                  const uint64_t *ggsw);
void ora_cmux_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *ct0, uint64_t *ct1,
                      const uint64_t *ggsw);

/* polynomial_algorithms.rs:395-507 monic monomial mul/div, native wrapping or custom modulus (q = 0: native) */
void ora_poly_monomial_mul(uint64_t *poly, size_t n, size_t degree, uint64_t q);
void ora_poly_monomial_div(uint64_t *poly, size_t n, size_t degree, uint64_t q);

/* fft_impl/common.rs:10-23 modulus_switch (native) and ntt64_pbs.rs:540-549 (non-native) */
uint64_t ora_modulus_switch(uint64_t input, unsigned log_modulus);
uint64_t ora_pbs_modulus_switch_non_native(uint64_t input, size_t n, uint64_t q);

/* ntt64_bnf_pbs.rs:208-266: blind rotation of `acc` by an already modulus-switched LWE
 * (mask values and body in [0, 2N]) */
void ora_blind_rotate_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                          const uint64_t *msed_mask, uint64_t msed_body, const uint64_t *bsk, size_t n_lwe);

/* glwe_sample_extraction.rs:89-160, nth = 0; q = 0 native else custom modulus */
void ora_sample_extract(const uint64_t *glwe, uint64_t *lwe_out, size_t n, int k, uint64_t q);

/* ntt64_bnf_pbs.rs:469-540: PBS of native ciphertexts (standard modulus switch, bsk Raw) */
void ora_pbs_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                 const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe);
/* same with the centered-binary modulus switch of the body when centered != 0
 * (algorithms/modulus_switch.rs:35-104) */
void ora_pbs_bnf_ms(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                    const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe, int centered);
uint64_t ora_centered_ms_body_correction(const uint64_t *mask, size_t n_lwe, unsigned log_modulus);
/* route the PBS restatement's transforms through the AVX-512 restatement (CPU baseline) */
void ora_pbs_set_fast_ntt(int on);

/* ntt64_pbs.rs:213-286 + 482-538: PBS of ciphertexts mod p (bsk pre-normalised) */
void ora_pbs_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                     const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe);

/* lwe_bootstrap_key_conversion.rs:294-365: standard BSK -> NTT domain.  `in_width` = 0: input
 * already mod p (plain forward), else power-of-two width (64 = native) modswitched first.
 * normalize != 0: NttLweBootstrapKeyOption::Normalize. */
void ora_bsk_to_ntt(const ora_ntt_tables *t, const uint64_t *bsk_std, uint64_t *bsk_ntt, size_t n_polys,
                    unsigned in_width, int normalize);

/* batched wrappers (OpenMP over independent items) */
void ora_pbs_bnf_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                       const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe,
                       size_t batch, int centered, int threads);
void ora_pbs_solinas_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                           const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe,
                           size_t batch, int threads);
void ora_ext_product_bnf_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *out,
                               const uint64_t *ggsw, const uint64_t *glwe, size_t batch, int threads);

/* ntt64_pbs.rs:213-286 blind_rotate_ntt64_assign_mem_optimized (acc in place; pre_switched: values in [0, 2N)) */
void ora_blind_rotate_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                              const uint64_t *lwe_in, const uint64_t *bsk, size_t n_lwe, int pre_switched);
/* glwe_sample_extraction.rs:89-160 at MonomialDegree(nth) (q = 0: native wrapping negation) */
void ora_sample_extract_nth(const uint64_t *glwe, uint64_t *lwe_out, size_t n, int k, size_t nth, uint64_t q);
/* batched in-place blind rotations, one accumulator per item (BNF ms_mode: 0 standard, 1 centered, 2 pre-switched) */
void ora_blind_rotate_bnf_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                                const uint64_t *lwe_in, const uint64_t *bsk, size_t n_lwe, size_t batch, int ms_mode,
                                int threads);
void ora_blind_rotate_solinas_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                                    const uint64_t *lwe_in, const uint64_t *bsk, size_t n_lwe, size_t batch,
                                    int pre_switched, int threads);

#ifdef __cplusplus
}
#endif
#endif
