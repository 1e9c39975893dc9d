/*
 * ntt_oracle.c — TEST INFRASTRUCTURE ONLY (see ntt_oracle.h).
 *
 * A plain-C restatement of tfhe-ntt's prime64 negacyclic NTT.  Every function
 * cites the reference file:line it follows (paths relative to
 * /root/reference/tfhe-ntt/src).  This is the parity checker for the HIP
 * product path and the CPU baseline timed by bench.py; it is never linked into
 * the product library.
 */
#include "ntt_oracle.h"

#include <string.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* prime.rs:9-11 mul_mod64 (Div64::rem_u128 is an exact remainder, fastdiv.rs:140) */
uint64_t ora_mul_mod(uint64_t a, uint64_t b, uint64_t p) {
    return (uint64_t)(((u128)a * (u128)b) % (u128)p);
}

/* prime.rs:32-50 exp_mod64: note pow==0 -> 1, else square-and-multiply with a final mul */
uint64_t ora_exp_mod(uint64_t base, uint64_t pow, uint64_t p) {
    if (pow == 0) return 1;
    uint64_t y = 1, x = base;
    while (pow > 1) {
        if (pow % 2 == 1) y = ora_mul_mod(x, y, p);
        x = ora_mul_mod(x, x, p);
        pow /= 2;
    }
    return ora_mul_mod(x, y, p);
}

/* prime.rs:52-67 is_prime_miller_rabin_iter */
static int mr_iter(uint64_t n, uint64_t s, uint64_t d, uint64_t a) {
    uint64_t x = ora_exp_mod(a, d, n);
    uint64_t nm1 = n - 1;
    if (x == 1 || x == nm1) return 1;
    for (uint64_t count = 0; count + 1 < s; ++count) {
        x = ora_mul_mod(x, x, n);
        if (x == nm1) return 1;
    }
    return 0;
}

/* prime.rs:76-128 is_prime64 (small-prime sieve then deterministic Miller–Rabin) */
int ora_is_prime64(uint64_t n) {
    static const uint64_t small[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (n < 2) return 0;
    for (int i = 0; i < 12; ++i)
        if (n % small[i] == 0) return n == small[i];
    uint64_t s = 0, d = n - 1;
    while (d % 2 == 0) { s++; d /= 2; }
    for (int i = 0; i < 12; ++i)
        if (!mr_iter(n, s, d, small[i])) return 0;
    return 1;
}

/* prime.rs:130-179 largest_prime_in_arithmetic_progression64 */
int ora_largest_prime_in_ap(uint64_t a, uint64_t b, uint64_t lo, uint64_t hi, uint64_t *out) {
    if (lo > hi) return 0;
    if (b > hi) return 0;
    if (a == 0) {
        if (lo <= b && b <= hi && ora_is_prime64(b)) { *out = b; return 1; }
        return 0;
    }
    uint64_t m = lo > b ? lo : b;
    uint64_t x_lo = (m - b) / a;
    if ((m - b) % a != 0) x_lo += 1;
    uint64_t x_hi = (hi - b) / a;
    uint64_t x = x_hi;
    for (;;) {
        uint64_t val = a * x + b;
        if (ora_is_prime64(val)) { *out = val; return 1; }
        if (x == x_lo) break;
        x -= 1;
    }
    return 0;
}

/* roots.rs:6-15 get_q_s64 */
static void get_q_s(uint64_t p, uint64_t *q, uint64_t *s) {
    uint64_t qq = p - 1, ss = 0;
    while (qq % 2 == 0) { qq /= 2; ss++; }
    *q = qq; *s = ss;
}

/* roots.rs:17-28 get_z64 (first quadratic non-residue >= 2) */
static int get_z(uint64_t p, uint64_t *z) {
    for (uint64_t n = 2; n < p; ++n) {
        if (ora_exp_mod(n, (p - 1) / 2, p) == p - 1) { *z = n; return 1; }
    }
    return 0;
}

/* roots.rs:31-66 sqrt_mod_ex64 (Tonelli–Shanks) */
static int sqrt_mod_ex(uint64_t p, uint64_t q, uint64_t s, uint64_t z, uint64_t n, uint64_t *out) {
    uint64_t m = s;
    uint64_t c = ora_exp_mod(z, q, p);
    uint64_t t = ora_exp_mod(n, q, p);
    uint64_t r = ora_exp_mod(n, q / 2 + (q % 2), p); /* q.div_ceil(2) */
    for (;;) {
        if (t == 0) { *out = 0; return 1; }
        if (t == 1) { *out = r; return 1; }
        uint64_t i = 0, t_pow = t;
        while (i < m) {
            t_pow = ora_mul_mod(t_pow, t_pow, p);
            i++;
            if (t_pow == 1) break;
        }
        if (i == m) return 0;
        uint64_t b = ora_exp_mod(c, (uint64_t)1 << (m - i - 1), p);
        m = i;
        c = ora_mul_mod(b, b, p);
        t = ora_mul_mod(t, c, p);
        r = ora_mul_mod(r, b, p);
    }
}

/* roots.rs:68-91 find_primitive_root64: n-1 successive square roots starting at p-1 */
int ora_find_primitive_root64(uint64_t p, uint64_t degree, uint64_t *out) {
    if (degree < 2 || (degree & (degree - 1))) return 0; /* reference asserts */
    unsigned n = (unsigned)__builtin_ctzll(degree);
    uint64_t root = p - 1, q, s, z;
    get_q_s(p, &q, &s);
    if (!get_z(p, &z)) return 0;
    for (unsigned i = 0; i + 1 < n; ++i) {
        if (!sqrt_mod_ex(p, q, s, z, root, &root)) return 0;
    }
    *out = root;
    return 1;
}

/* roots.rs:96-107 find_root_solinas_64 */
int ora_find_root_solinas64(uint64_t degree, uint64_t *out) {
    const uint64_t OMG_2_32 = 16334397945464290598ull;
    if (degree == 0 || degree > ((uint64_t)1 << 32)) return 0;
    *out = ora_exp_mod(OMG_2_32, ((uint64_t)1 << 32) / degree, ORA_SOLINAS_P);
    return 1;
}

/* lib.rs:123-125 bit_rev */
static size_t bit_rev(unsigned nbits, size_t i) {
    size_t r = 0;
    for (unsigned b = 0; b < nbits; ++b) r |= ((i >> b) & 1u) << (nbits - 1 - b);
    return r;
}

/* prime64.rs:159-204 init_negacyclic_twiddles (and, for p < 2^63, the twid/inv_twid halves of
 * init_negacyclic_twiddles_shoup prime64.rs:206-241, which use the same root and indexing). */
static void init_twiddles(uint64_t p, size_t n, uint64_t w, uint64_t *twid, uint64_t *inv_twid) {
    unsigned nbits = (unsigned)__builtin_ctzll(n);
    uint64_t wk = 1;
    for (size_t k = 0; k < n; ++k) {
        twid[bit_rev(nbits, k)] = wk;
        size_t inv_idx = bit_rev(nbits, (n - k) % n);
        inv_twid[inv_idx] = (k == 0) ? wk : p - wk;
        wk = ora_mul_mod(wk, w, p);
    }
}

/* prime64.rs:764-862 Plan::try_new (twiddle / n_inv part; Barrett & Shoup constants are
 * implementation detail of the CPU reduction and do not change any output) */
int ora_plan_init(size_t n, uint64_t p, uint64_t *twid, uint64_t *inv_twid, uint64_t *n_inv) {
    uint64_t root;
    if (n < 16 || (n & (n - 1)) || !ora_is_prime64(p) ||
        !ora_find_primitive_root64(p, 2 * (uint64_t)n, &root))
        return 0;
    uint64_t w;
    if (p == ORA_SOLINAS_P) {
        /* prime64.rs:162-179 hard-coded friendly roots */
        switch (n) {
        case 32: w = 8ull; break;
        case 64: w = 2198989700608ull; break;
        case 128: w = 14041890976876060974ull; break;
        case 256: w = 14430643036723656017ull; break;
        case 512: w = 4440654710286119610ull; break;
        case 1024: w = 8816101479115663336ull; break;
        case 2048: w = 10974926054405199669ull; break;
        case 4096: w = 1206500561358145487ull; break;
        case 8192: w = 10930245224889659871ull; break;
        case 16384: w = 3333600369887534767ull; break;
        case 32768: w = 15893793146607301539ull; break;
        default:
            if (!ora_find_root_solinas64(2 * (uint64_t)n, &w)) return 0;
        }
    } else {
        w = root; /* prime64.rs:181 / 216 */
    }
    init_twiddles(p, n, w, twid, inv_twid);
    *n_inv = ora_exp_mod((uint64_t)n, p - 2, p); /* prime64.rs:844 */
    return 1;
}

/* generic_solinas.rs:81-100 add/sub (canonical), and the Solinas reduction generic_solinas.rs:102-128 */
static inline uint64_t add_mod(uint64_t p, uint64_t a, uint64_t b) {
    uint64_t neg_b = p - b;
    return a >= neg_b ? a - neg_b : a + b;
}
static inline uint64_t sub_mod(uint64_t p, uint64_t a, uint64_t b) {
    uint64_t neg_b = p - b;
    return a >= b ? a - b : a + neg_b;
}
static inline uint64_t solinas_mul(uint64_t a, uint64_t b) {
    const uint64_t p = ORA_SOLINAS_P;
    u128 wide = (u128)a * b;
    uint64_t lo = (uint64_t)wide, hi = (uint64_t)(wide >> 64);
    uint64_t mid = hi & 0xFFFFFFFFull;
    hi = (hi & 0xFFFFFFFF00000000ull) >> 32;
    uint64_t low2 = lo - hi;
    if (hi > lo) low2 += p;
    uint64_t product = (mid << 32) - mid;
    uint64_t result = low2 + product;
    if (result < product || result >= p) result -= p;
    return result;
}
static inline uint64_t mul_mod_p(uint64_t p, uint64_t a, uint64_t b) {
    return p == ORA_SOLINAS_P ? solinas_mul(a, b) : ora_mul_mod(a, b, p);
}

/* generic_solinas.rs:449-481 fwd_breadth_first_scalar (the depth-first wrapper
 * generic_solinas.rs:1338-1386 runs the same butterflies in another order) */
void ora_fwd(size_t n, uint64_t p, const uint64_t *twid, uint64_t *data) {
    size_t t = n / 2, m = 1, w_idx = 1;
    while (m < n) {
        for (size_t i = 0; i < m; ++i) {
            uint64_t w1 = twid[w_idx + i];
            uint64_t *z0 = data + 2 * t * i, *z1 = z0 + t;
            for (size_t j = 0; j < t; ++j) {
                uint64_t z1w = mul_mod_p(p, z1[j], w1);
                uint64_t a = z0[j];
                z0[j] = add_mod(p, a, z1w);
                z1[j] = sub_mod(p, a, z1w);
            }
        }
        t /= 2; m *= 2; w_idx *= 2;
    }
}

/* generic_solinas.rs:483-514 inv_breadth_first_scalar (GS butterflies, unnormalized) */
void ora_inv(size_t n, uint64_t p, const uint64_t *inv_twid, uint64_t *data) {
    size_t t = 1, m = n, w_idx = n;
    while (m > 1) {
        m /= 2; w_idx /= 2;
        for (size_t i = 0; i < m; ++i) {
            uint64_t w1 = inv_twid[w_idx + i];
            uint64_t *z0 = data + 2 * t * i, *z1 = z0 + t;
            for (size_t j = 0; j < t; ++j) {
                uint64_t a = z0[j], b = z1[j];
                z0[j] = add_mod(p, a, b);
                z1[j] = mul_mod_p(p, sub_mod(p, a, b), w1);
            }
        }
        t *= 2;
    }
}

void ora_fwd_batch(size_t n, uint64_t p, const uint64_t *twid, uint64_t *data, size_t batch, size_t stride, int threads) {
    long long b;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b) ora_fwd(n, p, twid, data + (size_t)b * stride);
}

void ora_inv_batch(size_t n, uint64_t p, const uint64_t *inv_twid, uint64_t *data, size_t batch, size_t stride, int threads) {
    long long b;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (b = 0; b < (long long)batch; ++b) ora_inv(n, p, inv_twid, data + (size_t)b * stride);
}

/* prime64.rs:1210-1214 (Solinas) / 1216-1220 (generic): acc = acc + lhs*rhs mod p */
void ora_mul_accumulate(size_t n, uint64_t p, uint64_t *acc, const uint64_t *lhs, const uint64_t *rhs) {
    for (size_t i = 0; i < n; ++i) acc[i] = add_mod(p, acc[i], mul_mod_p(p, lhs[i], rhs[i]));
}

/* prime64.rs:1165-1170: x = x * n_inv mod p */
void ora_normalize(size_t n, uint64_t p, uint64_t n_inv, uint64_t *x) {
    for (size_t i = 0; i < n; ++i) x[i] = mul_mod_p(p, x[i], n_inv);
}

/* prime64.rs:1113-1121: lhs = (lhs*rhs)*n_inv mod p */
void ora_mul_assign_normalize(size_t n, uint64_t p, uint64_t n_inv, uint64_t *lhs, const uint64_t *rhs) {
    for (size_t i = 0; i < n; ++i) lhs[i] = mul_mod_p(p, mul_mod_p(p, lhs[i], rhs[i]), n_inv);
}

/* prime64.rs:1264-1276 negacyclic_convolution (test helper of the reference) */
void ora_negacyclic_convolution(size_t n, uint64_t p, const uint64_t *lhs, const uint64_t *rhs, uint64_t *out) {
    uint64_t *full = (uint64_t *)calloc(2 * n, sizeof(uint64_t));
    for (size_t i = 0; i < n; ++i)
        for (size_t j = 0; j < n; ++j)
            full[i + j] = add_mod(p, full[i + j], ora_mul_mod(lhs[i], rhs[j], p));
    for (size_t i = 0; i < n; ++i) out[i] = sub_mod(p, full[i], full[i + n]);
    free(full);
}

/* Counter-based generator (SURVEY.md §8d input recipe: splitmix64, uniform in [0,p) by
 * rejection).  Element i, attempt k hashes seed + (i+1)*G + k*H with the splitmix64 finalizer,
 * so the GPU bench can generate the identical batch in parallel on device.  Only the low
 * bitlen(p) bits are kept before the rejection test. */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
void ora_fill_uniform(uint64_t seed, uint64_t p, uint64_t *out, size_t count) {
    const int shift = p ? __builtin_clzll(p) : 0; /* draw bitlen(p) bits: acceptance >= 1/2 */
    for (size_t i = 0; i < count; ++i) {
        uint64_t v, k = 0;
        do {
            v = mix64(seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull + k * 0xD1B54A32D192ED03ull) >> shift;
            k++;
        } while (p != 0 && v >= p);
        out[i] = v;
    }
}
