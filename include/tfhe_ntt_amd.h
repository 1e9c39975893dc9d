/*
 * tfhe_ntt_amd.h — C ABI of the MI355X-native negacyclic NTT engine.
 *
 * Drop-in boundary for the tfhe-ntt `prime64::Plan` hot path (reference paths relative to
 * /root/reference).  Every entry point is `extern "C"`, takes plain pointers and sizes, never
 * aborts, and returns an `mi_status` (0 = OK).  Buffers are caller-owned; device pointers are
 * HIP device allocations on the plan's device; `stream` is a `hipStream_t` passed as `void*`
 * (NULL = the legacy default stream).  All `_batch` calls are asynchronous on `stream`.
 *
 * Batch layout: `batch` polynomials of `n` u64 coefficients, polynomial b starting at
 * `buf + b * stride` (stride >= n, in u64 units).  Values must be canonical (< p): inputs >= p
 * are outside the reference's domain (the reference test asserts it, prime64.rs:1328-1333).
 */
#ifndef TFHE_NTT_AMD_H
#define TFHE_NTT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum mi_status {
    MI_OK = 0,
    MI_ERR_INVALID_ARG = 1, /* N not a power of two / N < 16 / bad pointer or stride  */
    MI_ERR_NOT_PRIME = 2,   /* modulus fails is_prime64 (prime.rs:76-128)             */
    MI_ERR_NO_ROOT = 3,     /* no primitive 2N-th root of unity mod p (roots.rs:68-91) */
    MI_ERR_HIP = 4,         /* a HIP runtime call failed (see mi_last_error_message)  */
    MI_ERR_OOM = 5,         /* device allocation failed                               */
    MI_ERR_UNSUPPORTED = 6  /* valid request outside what this build implements       */
} mi_status;

typedef struct mi_ntt64_plan mi_ntt64_plan;

/* Human-readable text for a status code, and the detail of the last error on this thread. */
const char *mi_status_string(int status);
const char *mi_last_error_message(void);

/* ---- Plan -------------------------------------------------------------------------------
 * Replaces tfhe_ntt::prime64::Plan::try_new (tfhe-ntt/src/prime64.rs:764-862): the reference
 * returns None for N < 16, N not a power of two, p not prime, or no 2N-th root; here those are
 * MI_ERR_INVALID_ARG / MI_ERR_NOT_PRIME / MI_ERR_NO_ROOT.  Twiddles are built on the host exactly
 * as init_negacyclic_twiddles (prime64.rs:159-204) and uploaded to `device`.  A plan is immutable
 * after creation and may be shared by any number of streams / host threads. */
int mi_ntt64_plan_create(size_t n, uint64_t p, int device, mi_ntt64_plan **out_plan);
int mi_ntt64_plan_destroy(mi_ntt64_plan *plan);

/* Plan::ntt_size / Plan::modulus (prime64.rs:870-878); also the device the plan lives on. */
int mi_ntt64_plan_info(const mi_ntt64_plan *plan, size_t *n, uint64_t *p, int *device);

/* Host copies of the canonical twiddle tables (twid[bitrev(k)] = w^k, inv_twid as prime64.rs:193-199)
 * and N^{-1} mod p (prime64.rs:844).  Each table has n entries.  Any pointer may be NULL. */
int mi_ntt64_plan_twiddles(const mi_ntt64_plan *plan, uint64_t *twid, uint64_t *inv_twid, uint64_t *n_inv);

/* ---- Transforms (device pointers, async) -----------------------------------------------
 * Plan::fwd (prime64.rs:897-968): natural order in, bit-reversed NTT order out, in place.
 * Plan::inv (prime64.rs:975-1046): bit-reversed in, natural order out, unnormalised (x N). */
int mi_ntt64_fwd_batch(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch, size_t stride, void *stream);
int mi_ntt64_inv_batch(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch, size_t stride, void *stream);

/* ---- Pointwise ops (device pointers, async), all in the NTT domain -----------------------
 * Plan::normalize            (prime64.rs:1137-1179): x   = x * N^{-1}             mod p
 * Plan::mul_assign_normalize (prime64.rs:1050-1133): lhs = lhs * rhs * N^{-1}     mod p
 * Plan::mul_accumulate       (prime64.rs:1182-1222): acc = acc + lhs * rhs        mod p
 * The three operands of a call share one `stride`. */
int mi_ntt64_normalize_batch(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch, size_t stride, void *stream);
int mi_ntt64_mul_assign_normalize_batch(const mi_ntt64_plan *plan, uint64_t *lhs, const uint64_t *rhs,
                                        size_t batch, size_t stride, void *stream);
int mi_ntt64_mul_accumulate_batch(const mi_ntt64_plan *plan, uint64_t *acc, const uint64_t *lhs,
                                  const uint64_t *rhs, size_t batch, size_t stride, void *stream);

/* ---- Host-pointer convenience (copy in, run, copy out, synchronise) ---------------------
 * The single-polynomial `&mut [u64]` form of Plan::fwd / Plan::inv, batched; used by config 1
 * plumbing and the tests.  `buf` holds batch * n contiguous u64 on the host. */
int mi_ntt64_fwd_host(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch);
int mi_ntt64_inv_host(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch);

/* ---- Synthetic input (device, async) ----------------------------------------------------
 * Fills `count` u64 with the counter-based generator of SURVEY.md §8d (splitmix64 finaliser over
 * seed + (i+1)*G + k*H, top bits dropped to bitlen(p), rejection to [0,p); p = 0: full u64 range).  Identical stream to
 * the oracle's ora_fill_uniform, so GPU-generated batches can be checked on the host. */
int mi_fill_uniform(uint64_t *buf, size_t count, uint64_t seed, uint64_t p, int device, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* TFHE_NTT_AMD_H */
