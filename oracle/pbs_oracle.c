/*
 * pbs_oracle.c — TEST INFRASTRUCTURE ONLY (see pbs_oracle.h).
 * Restates the NTT external product / CMUX / blind rotation / PBS of tfhe core_crypto.
 * Reference paths are relative to /root/reference/tfhe/src/core_crypto.
 */
#include "pbs_oracle.h"

#include <stdlib.h>
#include <string.h>

#include "ntt_oracle.h"

typedef unsigned __int128 u128;

static inline uint64_t add_mod(uint64_t q, uint64_t a, uint64_t b) {
    uint64_t nb = q - b;
    return a >= nb ? a - nb : a + b;
}
/* commons/numeric/unsigned.rs:181-187 wrapping_sub_custom_mod */
static inline uint64_t sub_custom(uint64_t a, uint64_t b, uint64_t q) {
    return a >= b ? a - b : a - b + q;
}
/* unsigned.rs:219-225 wrapping_neg_custom_mod */
static inline uint64_t neg_custom(uint64_t a, uint64_t q) { return a == 0 ? 0 : q - a; }
/* unsigned.rs:174-179 wrapping_add_custom_mod = sub_custom(a, neg_custom(b)) */
static inline uint64_t add_custom(uint64_t a, uint64_t b, uint64_t q) { return sub_custom(a, neg_custom(b, q), q); }

static unsigned ceil_log2_u64(uint64_t x) { return x <= 1 ? 0 : 64u - (unsigned)__builtin_clzll(x - 1); }

/* decomposer.rs:64-71 balanced_rounding_condition_bit_trick + :156-185 init_decomposer_state */
uint64_t ora_decomp_init_native(uint64_t input, int base_log, int level) {
    const unsigned rep = (unsigned)(base_log * level), non_rep = 64u - rep;
    uint64_t res = input >> (non_rep - 1);
    const uint64_t rounding_bit = res & 1u;
    res += 1;
    res >>= 1;
    res &= (~0ull) >> (64u - rep);
    const uint64_t need_balance = (((res - 1) | (rounding_bit << (rep - 1))) & res) >> (rep - 1);
    return res - (need_balance << rep);
}

/* iter.rs:131-151 decomposition_bit_trick + decompose_one_level (arithmetic shift) */
uint64_t ora_decompose_one_level(int base_log, uint64_t *state) {
    const uint64_t mask = (1ull << base_log) - 1;
    const uint64_t res = *state & mask;
    *state = (uint64_t)((int64_t)*state >> base_log);
    const uint64_t carry = (((res - 1) | *state) & res) >> (base_log - 1);
    *state += carry;
    return res - (carry << base_log);
}

/* decomposer.rs:25-49 native_closest_representable */
static uint64_t native_closest_representable(uint64_t input, int level, int base_log) {
    const unsigned shift = 64u - (unsigned)(level * base_log) - 1u;
    uint64_t res = input >> shift;
    res += 1;
    res &= ~1ull;
    return res << shift;
}

/* decomposer.rs:521-548 SignedDecomposerNonNative::init_decomposer_state (abs part) */
static uint64_t nonnative_abs_closest(uint64_t abs_value, int level, int base_log, uint64_t q) {
    const unsigned shift_to_native = 64u - ceil_log2_u64(q);
    return native_closest_representable(abs_value << shift_to_native, level, base_log) >> shift_to_native;
}

/* ntt64.rs:166-178 */
uint64_t ora_modswitch_p2_to_prime(uint64_t v, unsigned width, uint64_t p) {
    u128 x = ((u128)v) >> (64u - width);
    return (uint64_t)(((x * (u128)p) + ((u128)1 << (width - 1))) >> width);
}

/* ntt64.rs:184-197 — note the OR (not an add) with p >> 1 */
uint64_t ora_modswitch_prime_to_p2(uint64_t v, unsigned width, uint64_t p) {
    u128 x = (((u128)v << width) | ((u128)p >> 1)) / (u128)p;
    return ((uint64_t)x) << (64u - width);
}

/* Plan::fwd / Plan::inv dispatch (prime64.rs:897-1046): the AVX-512 restatement when enabled and
 * available for the Solinas prime (as the reference's runtime dispatch), else the scalar restatement.
 * Both are bit-identical (tests/test_oracle.py); the fast one only serves the CPU baseline. */
static int g_fast_ntt = 0;
void ora_pbs_set_fast_ntt(int on) { g_fast_ntt = on; }
static void fwd_poly(const ora_ntt_tables *t, uint64_t *poly) {
    if (g_fast_ntt && t->p == 0xFFFFFFFF00000001ull && ora_fwd_avx512(t->n, t->twid, poly)) return;
    ora_fwd(t->n, t->p, t->twid, poly);
}
static void inv_poly(const ora_ntt_tables *t, uint64_t *poly) {
    if (g_fast_ntt && t->p == 0xFFFFFFFF00000001ull && ora_inv_avx512(t->n, t->inv_twid, poly)) return;
    ora_inv(t->n, t->p, t->inv_twid, poly);
}

/* ntt64_bnf_pbs.rs:541-681 add_external_product_ntt64_bnf_assign */
void ora_ext_product_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *out,
                         const uint64_t *ggsw, const uint64_t *glwe) {
    const size_t n = t->n, gs = (size_t)k + 1;
    const uint64_t p = t->p;
    uint64_t *states = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    uint64_t *acc = (uint64_t *)calloc(gs * n, sizeof(uint64_t));
    uint64_t *term = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    uint64_t *ntt_poly = (uint64_t *)malloc(n * sizeof(uint64_t));
    for (size_t i = 0; i < gs * n; ++i) states[i] = ora_decomp_init_native(glwe[i], base_log, level);
    for (int li = 0; li < level; ++li) { /* levels: highest first, as both iterators yield */
        for (size_t i = 0; i < gs * n; ++i) term[i] = ora_decompose_one_level(base_log, &states[i]);
        const uint64_t *mat = ggsw + (size_t)li * gs * gs * n;
        for (size_t r = 0; r < gs; ++r) {
            for (size_t j = 0; j < n; ++j) { /* ntt64.rs:221-240 forward_from_decomp */
                uint64_t x = term[r * n + j];
                ntt_poly[j] = ((int64_t)x < 0) ? x + p : x;
            }
            fwd_poly(t, ntt_poly);
            for (size_t c = 0; c < gs; ++c) /* update_with_fmadd_ntt64_bnf :707-726 */
                ora_mul_accumulate(n, p, acc + c * n, mat + (r * gs + c) * n, ntt_poly);
        }
    }
    for (size_t c = 0; c < gs; ++c) { /* normalize, inv, modswitch p -> 2^64, wrapping add */
        uint64_t *a = acc + c * n;
        ora_normalize(n, p, t->n_inv, a);
        inv_poly(t, a);
        for (size_t j = 0; j < n; ++j) out[c * n + j] += ora_modswitch_prime_to_p2(a[j], 64, p);
    }
    free(states); free(acc); free(term); free(ntt_poly);
}

/* ntt64_pbs.rs:553-663 add_external_product_ntt64_assign (decomposition iter.rs:623-745) */
void ora_ext_product_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *out,
                             const uint64_t *ggsw, const uint64_t *glwe) {
    const size_t n = t->n, gs = (size_t)k + 1;
    const uint64_t q = t->p;
    const unsigned shift = ceil_log2_u64(q) - (unsigned)(base_log * level);
    const uint64_t half = q / 2 + (q % 2); /* div_ceil(2) */
    uint64_t *states = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    unsigned char *signs = (unsigned char *)malloc(gs * n);
    uint64_t *acc = (uint64_t *)calloc(gs * n, sizeof(uint64_t));
    uint64_t *ntt_poly = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    for (size_t i = 0; i < gs * n; ++i) {
        const uint64_t x = glwe[i];
        if (x < half) { states[i] = nonnative_abs_closest(x, level, base_log, q) >> shift; signs[i] = 0; }
        else { states[i] = nonnative_abs_closest(q - x, level, base_log, q) >> shift; signs[i] = 1; }
    }
    for (int li = 0; li < level; ++li) {
        for (size_t i = 0; i < gs * n; ++i) {
            uint64_t term = ora_decompose_one_level(base_log, &states[i]);
            if (signs[i]) term = (uint64_t)0 - term;
            ntt_poly[i] = ((int64_t)term >= 0) ? term : q + term;
        }
        const uint64_t *mat = ggsw + (size_t)li * gs * gs * n;
        for (size_t r = 0; r < gs; ++r) {
            uint64_t *np = ntt_poly + r * n;
            fwd_poly(t, np);
            for (size_t c = 0; c < gs; ++c) ora_mul_accumulate(n, q, acc + c * n, mat + (r * gs + c) * n, np);
        }
    }
    for (size_t c = 0; c < gs; ++c) { /* ntt64.rs:110-137 add_backward */
        uint64_t *a = acc + c * n;
        inv_poly(t, a);
        for (size_t j = 0; j < n; ++j) out[c * n + j] = add_custom(out[c * n + j], a[j], q);
    }
    free(states); free(signs); free(acc); free(ntt_poly);
}

void ora_cmux_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *ct0, uint64_t *ct1,
                  const uint64_t *ggsw) {
    const size_t len = ((size_t)k + 1) * t->n;
    for (size_t i = 0; i < len; ++i) ct1[i] -= ct0[i];
    ora_ext_product_bnf(t, k, base_log, level, ct0, ggsw, ct1);
}

void ora_cmux_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *ct0, uint64_t *ct1,
                      const uint64_t *ggsw) {
    const size_t len = ((size_t)k + 1) * t->n;
    for (size_t i = 0; i < len; ++i) ct1[i] = sub_custom(ct1[i], ct0[i], t->p);
    ora_ext_product_solinas(t, k, base_log, level, ct0, ggsw, ct1);
}

static inline uint64_t neg_q(uint64_t x, uint64_t q) { return q ? neg_custom(x, q) : (uint64_t)0 - x; }

static void rotate_right(uint64_t *a, size_t n, size_t r, uint64_t *tmp) {
    for (size_t i = 0; i < n; ++i) tmp[(i + r) % n] = a[i];
    memcpy(a, tmp, n * sizeof(uint64_t));
}

/* polynomial_algorithms.rs:462-507 */
void ora_poly_monomial_mul(uint64_t *poly, size_t n, size_t degree, uint64_t q) {
    uint64_t *tmp = (uint64_t *)malloc(n * sizeof(uint64_t));
    if ((degree / n) % 2 == 1)
        for (size_t i = 0; i < n; ++i) poly[i] = neg_q(poly[i], q);
    const size_t rem = degree % n;
    rotate_right(poly, n, rem, tmp);
    for (size_t i = 0; i < rem; ++i) poly[i] = neg_q(poly[i], q);
    free(tmp);
}

/* polynomial_algorithms.rs:395-442 */
void ora_poly_monomial_div(uint64_t *poly, size_t n, size_t degree, uint64_t q) {
    uint64_t *tmp = (uint64_t *)malloc(n * sizeof(uint64_t));
    if ((degree / n) % 2 == 1)
        for (size_t i = 0; i < n; ++i) poly[i] = neg_q(poly[i], q);
    const size_t rem = degree % n;
    rotate_right(poly, n, (n - rem) % n, tmp); /* rotate_left(rem) */
    for (size_t i = n - rem; i < n; ++i) poly[i] = neg_q(poly[i], q);
    free(tmp);
}

/* fft_impl/common.rs:10-23 */
uint64_t ora_modulus_switch(uint64_t input, unsigned log_modulus) {
    if (log_modulus == 64) return input;
    const uint64_t r = input + (1ull << (64u - log_modulus - 1u));
    return r >> (64u - log_modulus);
}

/* ntt64_pbs.rs:540-549 with misc.rs:6-18 divide_round */
uint64_t ora_pbs_modulus_switch_non_native(uint64_t input, size_t n, uint64_t q) {
    const unsigned lg = (unsigned)__builtin_ctzll(n) + 1u;
    const u128 num = ((u128)input) << lg;
    const u128 div = num / q, rem = num % q;
    return (uint64_t)(div + (rem >= ((u128)q >> 1) ? 1 : 0));
}

void ora_blind_rotate_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                          const uint64_t *msed_mask, uint64_t msed_body, const uint64_t *bsk, size_t n_lwe) {
    const size_t n = t->n, gs = (size_t)k + 1, ggsw_len = (size_t)level * gs * gs * n;
    uint64_t *ct1 = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    for (size_t i = 0; i < n_lwe; ++i) {
        if (msed_mask[i] == 0) continue; /* ntt64_bnf_pbs.rs:241 */
        memcpy(ct1, acc, gs * n * sizeof(uint64_t));
        for (size_t c = 0; c < gs; ++c) ora_poly_monomial_mul(ct1 + c * n, n, (size_t)msed_mask[i], 0);
        ora_cmux_bnf(t, k, base_log, level, acc, ct1, bsk + i * ggsw_len);
    }
    for (size_t c = 0; c < gs; ++c) ora_poly_monomial_div(acc + c * n, n, (size_t)msed_body, 0);
    free(ct1);
}

void ora_sample_extract(const uint64_t *glwe, uint64_t *lwe_out, size_t n, int k, uint64_t q) {
    for (int c = 0; c < k; ++c) {
        const uint64_t *a = glwe + (size_t)c * n;
        uint64_t *m = lwe_out + (size_t)c * n;
        m[0] = a[0];
        for (size_t j = 1; j < n; ++j) m[j] = neg_q(a[n - j], q);
    }
    lwe_out[(size_t)k * n] = glwe[(size_t)k * n];
}

/* algorithms/modulus_switch.rs:60-104 centered_binary_ms_body_correction_to_add */
uint64_t ora_centered_ms_body_correction(const uint64_t *mask, size_t n_lwe, unsigned log_modulus) {
    uint64_t sum_half = 0;
    int64_t sum_halving_doubled = 0;
    for (size_t i = 0; i < n_lwe; ++i) {
        const uint64_t rounded = ora_modulus_switch(mask[i], log_modulus) << (64u - log_modulus);
        const int64_t err = (int64_t)(rounded - mask[i]);
        const int64_t half = err / 2; /* truncating signed division, as Rust */
        sum_halving_doubled += 2 * half - err;
        sum_half += (uint64_t)half;
    }
    const uint64_t sum_halving = (uint64_t)(sum_halving_doubled / 2);
    const uint64_t half_case = 1ull << (64u - log_modulus - 1u);
    return sum_half - sum_halving - half_case;
}

void ora_pbs_bnf(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                 const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe) {
    ora_pbs_bnf_ms(t, k, base_log, level, lwe_out, lwe_in, lut, bsk, n_lwe, 0);
}

void ora_pbs_bnf_ms(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                    const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe, int centered) {
    const size_t n = t->n, gs = (size_t)k + 1;
    const unsigned log_mod = (unsigned)__builtin_ctzll(n) + 1u; /* to_blind_rotation_input_modulus_log */
    uint64_t *acc = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    uint64_t *ms = (uint64_t *)malloc((n_lwe + 1) * sizeof(uint64_t));
    memcpy(acc, lut, gs * n * sizeof(uint64_t));
    for (size_t i = 0; i < n_lwe; ++i) ms[i] = ora_modulus_switch(lwe_in[i], log_mod);
    const uint64_t corr = centered ? ora_centered_ms_body_correction(lwe_in, n_lwe, log_mod) : 0;
    const uint64_t body = ora_modulus_switch(lwe_in[n_lwe] + corr, log_mod); /* modulus_switched_lwe_ciphertext.rs:155-162 */
    ora_blind_rotate_bnf(t, k, base_log, level, acc, ms, body, bsk, n_lwe);
    ora_sample_extract(acc, lwe_out, n, k, 0);
    free(acc); free(ms);
}

/* blind_rotate_ntt64_assign_mem_optimized (ntt64_pbs.rs:213-286): acc (the LUT, modulo p) is divided by X^ms(body)
 * first, then the CMUX loop over the mask.  pre_switched: lwe_in holds the switched values in [0, 2N) (a value of 0
 * skips the step like a raw 0 does: X^0 and X^2N leave ct1 - ct0 = 0). */
void ora_blind_rotate_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                              const uint64_t *lwe_in, const uint64_t *bsk, size_t n_lwe, int pre_switched) {
    const size_t n = t->n, gs = (size_t)k + 1, ggsw_len = (size_t)level * gs * gs * n;
    const uint64_t q = t->p;
    uint64_t *ct1 = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    const size_t deg_b = pre_switched ? (size_t)lwe_in[n_lwe]
                                      : (size_t)ora_pbs_modulus_switch_non_native(lwe_in[n_lwe], n, q);
    for (size_t c = 0; c < gs; ++c) ora_poly_monomial_div(acc + c * n, n, deg_b, q);
    for (size_t i = 0; i < n_lwe; ++i) {
        if (lwe_in[i] == 0) continue; /* ntt64_pbs.rs:257 */
        memcpy(ct1, acc, gs * n * sizeof(uint64_t));
        const size_t deg = pre_switched ? (size_t)lwe_in[i]
                                        : (size_t)ora_pbs_modulus_switch_non_native(lwe_in[i], n, q);
        for (size_t c = 0; c < gs; ++c) ora_poly_monomial_mul(ct1 + c * n, n, deg, q);
        ora_cmux_solinas(t, k, base_log, level, acc, ct1, bsk + i * ggsw_len);
    }
    free(ct1);
}

void ora_pbs_solinas(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                     const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe) {
    const size_t n = t->n, gs = (size_t)k + 1;
    uint64_t *acc = (uint64_t *)malloc(gs * n * sizeof(uint64_t));
    memcpy(acc, lut, gs * n * sizeof(uint64_t));
    ora_blind_rotate_solinas(t, k, base_log, level, acc, lwe_in, bsk, n_lwe, 0);
    ora_sample_extract(acc, lwe_out, n, k, t->p);
    free(acc);
}

/* extract_lwe_sample_from_glwe_ciphertext (glwe_sample_extraction.rs:89-160) at MonomialDegree(nth), restated step by
 * step: body = B[nth]; each mask polynomial copied, reversed, its first N - nth - 1 entries negated (wrapping, or
 * modulo q), then rotated left by that count. */
void ora_sample_extract_nth(const uint64_t *glwe, uint64_t *lwe_out, size_t n, int k, size_t nth, uint64_t q) {
    const size_t opposite = n - nth - 1;
    uint64_t *tmp = (uint64_t *)malloc(n * sizeof(uint64_t));
    lwe_out[(size_t)k * n] = glwe[(size_t)k * n + nth];
    for (int c = 0; c < k; ++c) {
        uint64_t *m = lwe_out + (size_t)c * n;
        for (size_t j = 0; j < n; ++j) m[j] = glwe[(size_t)c * n + (n - 1 - j)]; /* copy + reverse */
        for (size_t j = 0; j < opposite; ++j) m[j] = neg_q(m[j], q);
        for (size_t j = 0; j < n; ++j) tmp[j] = m[(j + opposite) % n];          /* rotate_left(opposite) */
        memcpy(m, tmp, n * sizeof(uint64_t));
    }
    free(tmp);
}

/* the batched GLWE-output blind rotations (one accumulator per item, in place), one item per thread.
 * BNF ms_mode: 0 standard switch of the native LWE, 1 centered (body corrected), 2 pre-switched values. */
void ora_blind_rotate_bnf_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                                const uint64_t *lwe_in, const uint64_t *bsk, size_t n_lwe, size_t batch, int ms_mode,
                                int threads) {
    const size_t glwe = ((size_t)k + 1) * t->n, in_len = n_lwe + 1;
    const unsigned log_mod = (unsigned)__builtin_ctzll(t->n) + 1u;
    long long b;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b) {
        const uint64_t *in = lwe_in + (size_t)b * in_len;
        uint64_t *ms = (uint64_t *)malloc(in_len * sizeof(uint64_t));
        for (size_t i = 0; i < n_lwe; ++i) ms[i] = ms_mode == 2 ? in[i] : ora_modulus_switch(in[i], log_mod);
        uint64_t body;
        if (ms_mode == 2) body = in[n_lwe];
        else {
            const uint64_t corr = ms_mode == 1 ? ora_centered_ms_body_correction(in, n_lwe, log_mod) : 0;
            body = ora_modulus_switch(in[n_lwe] + corr, log_mod);
        }
        ora_blind_rotate_bnf(t, k, base_log, level, acc + (size_t)b * glwe, ms, body, bsk, n_lwe);
        free(ms);
    }
}

void ora_blind_rotate_solinas_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *acc,
                                    const uint64_t *lwe_in, const uint64_t *bsk, size_t n_lwe, size_t batch,
                                    int pre_switched, int threads) {
    const size_t glwe = ((size_t)k + 1) * t->n;
    long long b;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b)
        ora_blind_rotate_solinas(t, k, base_log, level, acc + (size_t)b * glwe, lwe_in + (size_t)b * (n_lwe + 1), bsk,
                                 n_lwe, pre_switched);
}

void ora_bsk_to_ntt(const ora_ntt_tables *t, const uint64_t *bsk_std, uint64_t *bsk_ntt, size_t n_polys,
                    unsigned in_width, int normalize) {
    const size_t n = t->n;
    for (size_t pi = 0; pi < n_polys; ++pi) {
        const uint64_t *src = bsk_std + pi * n;
        uint64_t *dst = bsk_ntt + pi * n;
        for (size_t j = 0; j < n; ++j) dst[j] = in_width ? ora_modswitch_p2_to_prime(src[j], in_width, t->p) : src[j];
        fwd_poly(t, dst);
        if (normalize) ora_normalize(n, t->p, t->n_inv, dst);
    }
}

void ora_pbs_bnf_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                       const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe,
                       size_t batch, int centered, int threads) {
    const size_t out_len = (size_t)k * t->n + 1, in_len = n_lwe + 1;
    long long b;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b)
        ora_pbs_bnf_ms(t, k, base_log, level, lwe_out + (size_t)b * out_len, lwe_in + (size_t)b * in_len, lut, bsk,
                       n_lwe, centered);
}

/* programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized (ntt64_pbs.rs:482-538) over a batch, one PBS per
 * thread as the reference's rayon throughput harness (pbs_bench.rs:865-886) */
void ora_pbs_solinas_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *lwe_out,
                           const uint64_t *lwe_in, const uint64_t *lut, const uint64_t *bsk, size_t n_lwe,
                           size_t batch, int threads) {
    const size_t out_len = (size_t)k * t->n + 1, in_len = n_lwe + 1;
    long long b;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b)
        ora_pbs_solinas(t, k, base_log, level, lwe_out + (size_t)b * out_len, lwe_in + (size_t)b * in_len, lut, bsk,
                        n_lwe);
}

void ora_ext_product_bnf_batch(const ora_ntt_tables *t, int k, int base_log, int level, uint64_t *out,
                               const uint64_t *ggsw, const uint64_t *glwe, size_t batch, int threads) {
    const size_t len = ((size_t)k + 1) * t->n;
    long long b;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b)
        ora_ext_product_bnf(t, k, base_log, level, out + (size_t)b * len, ggsw, glwe + (size_t)b * len);
}

/* ---- the Ntt64View layer (commons/math/ntt/ntt64.rs:89-266), one polynomial per call, batched with OpenMP ---- */
/* u64::wrapping_add_custom_mod (commons/numeric/unsigned.rs:174-187) = self.wrapping_sub_custom_mod(
 * other.wrapping_neg_custom_mod(m)) with wrapping_neg_custom_mod (:219-225) and wrapping_sub_custom_mod (:181-187) */
static uint64_t wrapping_add_custom_mod(uint64_t a, uint64_t b, uint64_t m) {
    const uint64_t nb = b == 0 ? 0 : m - b;
    return a >= nb ? a - nb : a - nb + m;
}

/* kind 0 forward (:89-95) / forward_normalized (:97-108, normalize != 0), 1 forward_from_power_of_two_modulus
 * (:201-214, modswitch_from_power_of_two_to_ntt_prime :166-177), 2 forward_from_decomp (:221-240) */
void ora_ntt64_view_forward_batch(const ora_ntt_tables *t, int kind, unsigned width, int normalize, uint64_t *ntt,
                                  const uint64_t *standard, size_t batch, size_t stride, int threads) {
    const size_t n = t->n;
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
    for (size_t b = 0; b < batch; ++b) {
        uint64_t *dst = ntt + b * stride;
        const uint64_t *src = standard + b * stride;
        for (size_t j = 0; j < n; ++j) {
            uint64_t x = src[j]; /* ntt.copy_from_slice(standard) */
            if (kind == 1) x = ora_modswitch_p2_to_prime(x, width, t->p);
            else if (kind == 2) x = (int64_t)x < 0 ? x + t->p : x; /* x.wrapping_add(custom_modulus) */
            dst[j] = x;
        }
        ora_fwd(n, t->p, t->twid, dst);
        if (normalize) ora_normalize(n, t->p, t->n_inv, dst);
    }
}

/* width 0: add_backward (:110-131); else add_backward_on_power_of_two_modulus (:244-266) with
 * modswitch_from_ntt_prime_to_power_of_two (:184-196).  ntt is left as the reference leaves it. */
void ora_ntt64_view_add_backward_batch(const ora_ntt_tables *t, unsigned width, uint64_t *standard, uint64_t *ntt,
                                       size_t batch, size_t stride, int threads) {
    const size_t n = t->n;
#pragma omp parallel for num_threads(threads > 0 ? threads : 1) schedule(static)
    for (size_t b = 0; b < batch; ++b) {
        uint64_t *y = ntt + b * stride, *out = standard + b * stride;
        ora_inv(n, t->p, t->inv_twid, y);
        if (width) {
            for (size_t j = 0; j < n; ++j) y[j] = ora_modswitch_prime_to_p2(y[j], width, t->p);
            for (size_t j = 0; j < n; ++j) out[j] += y[j];
        } else {
            for (size_t j = 0; j < n; ++j) out[j] = wrapping_add_custom_mod(out[j], y[j], t->p);
        }
    }
}

/* lwe_ciphertext_[centered_binary_]modulus_switch at Scalar = u64 (algorithms/modulus_switch.rs:14-104), read out as
 * the lazy switched ciphertext does (entities/modulus_switched_lwe_ciphertext.rs:150-172): out[i] = ms(a_i), out[dim]
 * = ms(b + correction) */
void ora_lwe_ms64(const uint64_t *lwe, size_t dim, unsigned log_mod, int centered, uint64_t *out) {
    const uint64_t corr = centered ? ora_centered_ms_body_correction(lwe, dim, log_mod) : 0;
    for (size_t i = 0; i < dim; ++i) out[i] = ora_modulus_switch(lwe[i], log_mod);
    out[dim] = ora_modulus_switch(lwe[dim] + corr, log_mod);
}
