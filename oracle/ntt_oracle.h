/*
 * ntt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's `tfhe_ntt::prime64` negacyclic NTT path
 * (reference: /root/reference/tfhe-ntt/src/{prime64.rs,prime64/generic_solinas.rs,
 * roots.rs,prime.rs}).  It is the *checker* for the HIP product path: only
 * tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may load it.
 * Nothing under tfhe-rs-main_modified_amd/ links or calls this code.
 *
 * Parity pinning: the reference is Rust and cannot be compiled in this image
 * (no cargo/rustc), and has no Python/C implementation of the path, so this
 * restatement is pinned by the reference's own known-answer tests (Solinas
 * root table roots.rs:150-172, prime search prime.rs:199-213, is_prime
 * prime.rs:184-196, Plan::try_new(2048,1024)=None prime64.rs:1988-1990, the
 * prime32 doc round trip lib.rs:25-49) and by its property tests (negacyclic
 * convolution prime64.rs:1264-1361) — see tests/test_oracle.py.
 */
#ifndef NTT_ORACLE_H
#define NTT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORA_SOLINAS_P 0xFFFFFFFF00000001ull

/* ---- scalar number theory (prime.rs / roots.rs) ---- */
uint64_t ora_mul_mod(uint64_t a, uint64_t b, uint64_t p);
uint64_t ora_exp_mod(uint64_t base, uint64_t pow, uint64_t p);
int ora_is_prime64(uint64_t n);
/* returns 1 and writes *out on success, 0 for None */
int ora_largest_prime_in_ap(uint64_t factor, uint64_t offset, uint64_t lo, uint64_t hi, uint64_t *out);
int ora_find_primitive_root64(uint64_t p, uint64_t degree, uint64_t *out);
int ora_find_root_solinas64(uint64_t degree, uint64_t *out);

/* ---- Plan (prime64.rs:159-204, 764-862) ----
 * returns 1 on success (Some(plan)), 0 when the reference returns None. */
int ora_plan_init(size_t n, uint64_t p, uint64_t *twid, uint64_t *inv_twid, uint64_t *n_inv);

/* ---- transforms (generic_solinas.rs:449-561, 1338-1440) ---- */
void ora_fwd(size_t n, uint64_t p, const uint64_t *twid, uint64_t *data);
void ora_inv(size_t n, uint64_t p, const uint64_t *inv_twid, uint64_t *data);
/* batched, `batch` polys at `stride` u64 apart, OpenMP over the batch with `threads` threads */
void ora_fwd_batch(size_t n, uint64_t p, const uint64_t *twid, uint64_t *data, size_t batch, size_t stride, int threads);
void ora_inv_batch(size_t n, uint64_t p, const uint64_t *inv_twid, uint64_t *data, size_t batch, size_t stride, int threads);

/* ---- pointwise ops (prime64.rs:1050-1222) ---- */
void ora_mul_accumulate(size_t n, uint64_t p, uint64_t *acc, const uint64_t *lhs, const uint64_t *rhs);
void ora_normalize(size_t n, uint64_t p, uint64_t n_inv, uint64_t *x);
void ora_mul_assign_normalize(size_t n, uint64_t p, uint64_t n_inv, uint64_t *lhs, const uint64_t *rhs);

/* ---- schoolbook negacyclic product mod p (prime64.rs:1264-1276), for property checks ---- */
void ora_negacyclic_convolution(size_t n, uint64_t p, const uint64_t *lhs, const uint64_t *rhs, uint64_t *out);

/* ---- AVX-512 restatement of the reference's fast path (CPU baseline only) ----
 * fwd_depth_first_avx512/inv_depth_first_avx512 (generic_solinas.rs:801-1032, 1036, 1444)
 * with the 4-multiply widening emulation (lib.rs:175-207).  Returns 0 if the CPU lacks AVX-512F. */
int ora_have_avx512(void);
int ora_fwd_batch_avx512(size_t n, const uint64_t *twid, uint64_t *data, size_t batch, size_t stride, int threads);
int ora_inv_batch_avx512(size_t n, const uint64_t *inv_twid, uint64_t *data, size_t batch, size_t stride, int threads);
int ora_fwd_avx512(size_t n, const uint64_t *twid, uint64_t *data);
int ora_inv_avx512(size_t n, const uint64_t *inv_twid, uint64_t *data);

/* deterministic input generator shared with the GPU tests/bench (splitmix64 -> uniform in [0,p) by rejection) */
void ora_fill_uniform(uint64_t seed, uint64_t p, uint64_t *out, size_t count);

#ifdef __cplusplus
}
#endif
#endif
