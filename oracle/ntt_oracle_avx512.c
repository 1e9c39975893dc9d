/*
 * ntt_oracle_avx512.c — TEST INFRASTRUCTURE / CPU BASELINE ONLY.
 *
 * Restatement of the reference's AVX-512 Solinas fast path, the path
 * `prime64::Plan::fwd/inv` dispatches to on an AVX-512 host (prime64.rs:943-956,
 * 1021-1034).  It is what bench.py times as the `cpu_baseline` ("port").
 *
 *   widening_mul_u64x8            lib.rs:175-207 (4 x vpmuludq emulation)
 *   Solinas::mul (V4)             generic_solinas.rs:414-446
 *   u64 add/sub (V4)              generic_solinas.rs:298-318
 *   fwd_breadth_first_avx512      generic_solinas.rs:801-927
 *   fwd_depth_first_avx512        generic_solinas.rs:931-1032 (RECURSION_THRESHOLD = 1024, prime64.rs:7)
 *   inv_breadth_first_avx512      generic_solinas.rs:1444-1560
 *   inv_depth_first_avx512        generic_solinas.rs:1036-1140
 *   permute/interleave helpers    prime64.rs:83-157
 */
#include "ntt_oracle.h"

#include <immintrin.h>

#define TGT __attribute__((target("avx512f")))
#define RECURSION_THRESHOLD 1024

int ora_have_avx512(void) {
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") ? 1 : 0;
}

TGT static inline void widening_mul(__m512i x, __m512i y, __m512i *lo, __m512i *hi) {
    const __m512i lo_mask = _mm512_set1_epi64(0x00000000FFFFFFFFll);
    __m512i x_hi = _mm512_shuffle_epi32(x, (_MM_PERM_ENUM)0xB1);
    __m512i y_hi = _mm512_shuffle_epi32(y, (_MM_PERM_ENUM)0xB1);
    __m512i z_lo_lo = _mm512_mul_epu32(x, y);
    __m512i z_lo_hi = _mm512_mul_epu32(x, y_hi);
    __m512i z_hi_lo = _mm512_mul_epu32(x_hi, y);
    __m512i z_hi_hi = _mm512_mul_epu32(x_hi, y_hi);
    __m512i z_lo_lo_shift = _mm512_srli_epi64(z_lo_lo, 32);
    __m512i sum_tmp = _mm512_add_epi64(z_lo_hi, z_lo_lo_shift);
    __m512i sum_lo = _mm512_and_si512(sum_tmp, lo_mask);
    __m512i sum_mid = _mm512_srli_epi64(sum_tmp, 32);
    __m512i sum_mid2 = _mm512_add_epi64(z_hi_lo, sum_lo);
    __m512i sum_mid2_hi = _mm512_srli_epi64(sum_mid2, 32);
    __m512i sum_hi = _mm512_add_epi64(z_hi_hi, sum_mid);
    *hi = _mm512_add_epi64(sum_hi, sum_mid2_hi);
    *lo = _mm512_add_epi64(_mm512_slli_epi64(_mm512_add_epi64(z_lo_hi, z_hi_lo), 32), z_lo_lo);
}

TGT static inline __m512i v_add(__m512i a, __m512i b) {
    const __m512i p = _mm512_set1_epi64((long long)ORA_SOLINAS_P);
    __m512i neg_b = _mm512_sub_epi64(p, b);
    __mmask8 ge = _mm512_cmpge_epu64_mask(a, neg_b);
    return _mm512_mask_blend_epi64(ge, _mm512_add_epi64(a, b), _mm512_sub_epi64(a, neg_b));
}

TGT static inline __m512i v_sub(__m512i a, __m512i b) {
    const __m512i p = _mm512_set1_epi64((long long)ORA_SOLINAS_P);
    __m512i neg_b = _mm512_sub_epi64(p, b);
    __mmask8 ge = _mm512_cmpge_epu64_mask(a, b);
    return _mm512_mask_blend_epi64(ge, _mm512_add_epi64(a, neg_b), _mm512_sub_epi64(a, b));
}

TGT static inline __m512i v_mul(__m512i a, __m512i b) {
    const __m512i p = _mm512_set1_epi64((long long)ORA_SOLINAS_P);
    __m512i lo, hi;
    widening_mul(a, b, &lo, &hi);
    __m512i mid = _mm512_and_si512(hi, _mm512_set1_epi64(0x00000000FFFFFFFFll));
    __m512i hh = _mm512_srli_epi64(_mm512_and_si512(hi, _mm512_set1_epi64((long long)0xFFFFFFFF00000000ull)), 32);
    __m512i low2 = _mm512_sub_epi64(lo, hh);
    __mmask8 gt = _mm512_cmpgt_epu64_mask(hh, lo);
    low2 = _mm512_mask_blend_epi64(gt, low2, _mm512_add_epi64(low2, p));
    __m512i product = _mm512_sub_epi64(_mm512_slli_epi64(mid, 32), mid);
    __m512i result = _mm512_add_epi64(low2, product);
    __mmask8 product_gt_result = _mm512_cmpgt_epu64_mask(product, result);
    __mmask8 p_gt_result = _mm512_cmpgt_epu64_mask(p, result);
    __mmask8 not_cond = (__mmask8)(~product_gt_result & p_gt_result);
    return _mm512_mask_blend_epi64(not_cond, _mm512_sub_epi64(result, p), result);
}

/* prime64.rs:85-157 lane shuffles */
TGT static inline void interleave4(__m512i a, __m512i b, __m512i *o0, __m512i *o1) {
    const __m512i i0 = _mm512_setr_epi64(0x0, 0x1, 0x2, 0x3, 0x8, 0x9, 0xa, 0xb);
    const __m512i i1 = _mm512_setr_epi64(0x4, 0x5, 0x6, 0x7, 0xc, 0xd, 0xe, 0xf);
    *o0 = _mm512_permutex2var_epi64(a, i0, b);
    *o1 = _mm512_permutex2var_epi64(a, i1, b);
}
TGT static inline __m512i permute4(const uint64_t *w) {
    __m512i w01 = _mm512_castsi128_si512(_mm_loadu_si128((const __m128i *)w));
    return _mm512_permutexvar_epi64(_mm512_setr_epi64(0, 0, 0, 0, 1, 1, 1, 1), w01);
}
TGT static inline void interleave2(__m512i a, __m512i b, __m512i *o0, __m512i *o1) {
    const __m512i i0 = _mm512_setr_epi64(0x0, 0x1, 0x8, 0x9, 0x4, 0x5, 0xc, 0xd);
    const __m512i i1 = _mm512_setr_epi64(0x2, 0x3, 0xa, 0xb, 0x6, 0x7, 0xe, 0xf);
    *o0 = _mm512_permutex2var_epi64(a, i0, b);
    *o1 = _mm512_permutex2var_epi64(a, i1, b);
}
TGT static inline __m512i permute2(const uint64_t *w) {
    __m512i w0123 = _mm512_castsi256_si512(_mm256_loadu_si256((const __m256i *)w));
    return _mm512_permutexvar_epi64(_mm512_setr_epi64(0, 0, 2, 2, 1, 1, 3, 3), w0123);
}
TGT static inline void interleave1(__m512i a, __m512i b, __m512i *o0, __m512i *o1) {
    *o0 = _mm512_unpacklo_epi64(a, b);
    *o1 = _mm512_unpackhi_epi64(a, b);
}
TGT static inline __m512i permute1(const uint64_t *w) {
    __m512i w8 = _mm512_loadu_si512((const void *)w);
    return _mm512_permutexvar_epi64(_mm512_setr_epi64(0, 4, 1, 5, 2, 6, 3, 7), w8);
}

/* one radix-2 CT stage over chunks of 2t (t >= 8) with a splatted twiddle */
TGT static void fwd_stage_splat(uint64_t *data, size_t n, size_t t, const uint64_t *w) {
    for (size_t c = 0; c < n / (2 * t); ++c) {
        __m512i w1 = _mm512_set1_epi64((long long)w[c]);
        uint64_t *z0 = data + 2 * t * c, *z1 = z0 + t;
        for (size_t j = 0; j < t; j += 8) {
            __m512i a = _mm512_loadu_si512(z0 + j), b = _mm512_loadu_si512(z1 + j);
            __m512i z1w = v_mul(b, w1);
            _mm512_storeu_si512(z0 + j, v_add(a, z1w));
            _mm512_storeu_si512(z1 + j, v_sub(a, z1w));
        }
    }
}

/* generic_solinas.rs:801-927 */
TGT static void fwd_breadth_first(uint64_t *data, size_t n, const uint64_t *twid, size_t depth, size_t half) {
    size_t t = n / 2, m = 1, w_idx = (m << depth) + half * m;
    while (m < n / 8) {
        fwd_stage_splat(data, n, t, twid + w_idx);
        t /= 2; m *= 2; w_idx *= 2;
    }
    /* t = 4 */
    for (size_t c = 0; c < n / 16; ++c) {
        __m512i w1 = permute4(twid + w_idx + 2 * c);
        __m512i x0 = _mm512_loadu_si512(data + 16 * c), x1 = _mm512_loadu_si512(data + 16 * c + 8), z0, z1;
        interleave4(x0, x1, &z0, &z1);
        __m512i z1w = v_mul(z1, w1);
        interleave4(v_add(z0, z1w), v_sub(z0, z1w), &x0, &x1);
        _mm512_storeu_si512(data + 16 * c, x0);
        _mm512_storeu_si512(data + 16 * c + 8, x1);
    }
    w_idx *= 2;
    /* t = 2 */
    for (size_t c = 0; c < n / 16; ++c) {
        __m512i w1 = permute2(twid + w_idx + 4 * c);
        __m512i x0 = _mm512_loadu_si512(data + 16 * c), x1 = _mm512_loadu_si512(data + 16 * c + 8), z0, z1;
        interleave2(x0, x1, &z0, &z1);
        __m512i z1w = v_mul(z1, w1);
        interleave2(v_add(z0, z1w), v_sub(z0, z1w), &x0, &x1);
        _mm512_storeu_si512(data + 16 * c, x0);
        _mm512_storeu_si512(data + 16 * c + 8, x1);
    }
    w_idx *= 2;
    /* t = 1 */
    for (size_t c = 0; c < n / 16; ++c) {
        __m512i w1 = permute1(twid + w_idx + 8 * c);
        __m512i x0 = _mm512_loadu_si512(data + 16 * c), x1 = _mm512_loadu_si512(data + 16 * c + 8), z0, z1;
        interleave1(x0, x1, &z0, &z1);
        __m512i z1w = v_mul(z1, w1);
        interleave1(v_add(z0, z1w), v_sub(z0, z1w), &x0, &x1);
        _mm512_storeu_si512(data + 16 * c, x0);
        _mm512_storeu_si512(data + 16 * c + 8, x1);
    }
}

/* generic_solinas.rs:931-1032 */
TGT static void fwd_depth_first(uint64_t *data, size_t n, const uint64_t *twid, size_t depth, size_t half) {
    if (n <= RECURSION_THRESHOLD) {
        fwd_breadth_first(data, n, twid, depth, half);
        return;
    }
    fwd_stage_splat(data, n, n / 2, twid + ((size_t)1 << depth) + half);
    fwd_depth_first(data, n / 2, twid, depth + 1, half * 2);
    fwd_depth_first(data + n / 2, n / 2, twid, depth + 1, half * 2 + 1);
}

TGT static void inv_stage_splat(uint64_t *data, size_t n, size_t t, const uint64_t *w) {
    for (size_t c = 0; c < n / (2 * t); ++c) {
        __m512i w1 = _mm512_set1_epi64((long long)w[c]);
        uint64_t *z0 = data + 2 * t * c, *z1 = z0 + t;
        for (size_t j = 0; j < t; j += 8) {
            __m512i a = _mm512_loadu_si512(z0 + j), b = _mm512_loadu_si512(z1 + j);
            _mm512_storeu_si512(z0 + j, v_add(a, b));
            _mm512_storeu_si512(z1 + j, v_mul(v_sub(a, b), w1));
        }
    }
}

/* generic_solinas.rs:1444-1560 */
TGT static void inv_breadth_first(uint64_t *data, size_t n, const uint64_t *inv_twid, size_t depth, size_t half) {
    size_t t = 1, m = n, w_idx = (m << depth) + half * m;
    m /= 2; w_idx /= 2; /* t = 1 */
    for (size_t c = 0; c < n / 16; ++c) {
        __m512i w1 = permute1(inv_twid + w_idx + 8 * c);
        __m512i x0 = _mm512_loadu_si512(data + 16 * c), x1 = _mm512_loadu_si512(data + 16 * c + 8), z0, z1;
        interleave1(x0, x1, &z0, &z1);
        interleave1(v_add(z0, z1), v_mul(v_sub(z0, z1), w1), &x0, &x1);
        _mm512_storeu_si512(data + 16 * c, x0);
        _mm512_storeu_si512(data + 16 * c + 8, x1);
    }
    t *= 2;
    m /= 2; w_idx /= 2; /* t = 2 */
    for (size_t c = 0; c < n / 16; ++c) {
        __m512i w1 = permute2(inv_twid + w_idx + 4 * c);
        __m512i x0 = _mm512_loadu_si512(data + 16 * c), x1 = _mm512_loadu_si512(data + 16 * c + 8), z0, z1;
        interleave2(x0, x1, &z0, &z1);
        interleave2(v_add(z0, z1), v_mul(v_sub(z0, z1), w1), &x0, &x1);
        _mm512_storeu_si512(data + 16 * c, x0);
        _mm512_storeu_si512(data + 16 * c + 8, x1);
    }
    t *= 2;
    m /= 2; w_idx /= 2; /* t = 4 */
    for (size_t c = 0; c < n / 16; ++c) {
        __m512i w1 = permute4(inv_twid + w_idx + 2 * c);
        __m512i x0 = _mm512_loadu_si512(data + 16 * c), x1 = _mm512_loadu_si512(data + 16 * c + 8), z0, z1;
        interleave4(x0, x1, &z0, &z1);
        interleave4(v_add(z0, z1), v_mul(v_sub(z0, z1), w1), &x0, &x1);
        _mm512_storeu_si512(data + 16 * c, x0);
        _mm512_storeu_si512(data + 16 * c + 8, x1);
    }
    t *= 2;
    while (m > 1) {
        m /= 2; w_idx /= 2;
        inv_stage_splat(data, n, t, inv_twid + w_idx);
        t *= 2;
    }
}

/* generic_solinas.rs:1036-1140 */
TGT static void inv_depth_first(uint64_t *data, size_t n, const uint64_t *inv_twid, size_t depth, size_t half) {
    if (n <= RECURSION_THRESHOLD) {
        inv_breadth_first(data, n, inv_twid, depth, half);
        return;
    }
    inv_depth_first(data, n / 2, inv_twid, depth + 1, half * 2);
    inv_depth_first(data + n / 2, n / 2, inv_twid, depth + 1, half * 2 + 1);
    inv_stage_splat(data, n, n / 2, inv_twid + ((size_t)1 << depth) + half);
}

int ora_fwd_batch_avx512(size_t n, const uint64_t *twid, uint64_t *data, size_t batch, size_t stride, int threads) {
    if (!ora_have_avx512() || n < 16) return 0;
    long long b;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b) fwd_depth_first(data + (size_t)b * stride, n, twid, 0, 0);
    return 1;
}

int ora_inv_batch_avx512(size_t n, const uint64_t *inv_twid, uint64_t *data, size_t batch, size_t stride, int threads) {
    if (!ora_have_avx512() || n < 16) return 0;
    long long b;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b) inv_depth_first(data + (size_t)b * stride, n, inv_twid, 0, 0);
    return 1;
}

/* single polynomial, no threading (used inside the batched PBS restatement) */
int ora_fwd_avx512(size_t n, const uint64_t *twid, uint64_t *data) {
    if (!ora_have_avx512() || n < 16) return 0;
    fwd_depth_first(data, n, twid, 0, 0);
    return 1;
}

int ora_inv_avx512(size_t n, const uint64_t *inv_twid, uint64_t *data) {
    if (!ora_have_avx512() || n < 16) return 0;
    inv_depth_first(data, n, inv_twid, 0, 0);
    return 1;
}
