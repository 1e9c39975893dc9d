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
/* Build provenance (no reference counterpart): sha256 of the sources this library was built from
 * (tools/source_hash.py: csrc sources and headers, the asm-body generators, this header, the Makefile), so a
 * caller can tell whether the loaded library matches the tree beside it. */
const char *mi_build_source_hash(void);

/* ---- Plan -------------------------------------------------------------------------------
 * Replaces tfhe_ntt::prime64::Plan::try_new (tfhe-ntt/src/prime64.rs:764-862): the reference
 * returns None for N < 16, N not a power of two, p not prime, or no 2N-th root; here those are
 * MI_ERR_INVALID_ARG / MI_ERR_NOT_PRIME / MI_ERR_NO_ROOT.  Twiddles are built on the host exactly
 * as init_negacyclic_twiddles (prime64.rs:159-204) and uploaded to `device`.  A plan is immutable
 * after creation and may be shared by any number of streams / host threads.  Sizes 16 <= N <= 2^31
 * (the Solinas field's 2N-th roots end at 2N = 2^32, roots.rs:96-107); N > 2^14 runs as passes of
 * top stages through HBM plus 2^14-element blocks. */
int mi_ntt64_plan_create(size_t n, uint64_t p, int device, mi_ntt64_plan **out_plan);
int mi_ntt64_plan_destroy(mi_ntt64_plan *plan);

/* The process-wide plan cache of Ntt64::new (tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:27-79):
 * one immutable plan per (n, p, device), built on first use (concurrent first callers build it once)
 * and shared by every later caller and thread; later lookups are a read-locked map probe.  Cached
 * plans live until process exit, as the reference's static PLANS map; mi_ntt64_plan_destroy on one
 * is a no-op.  Same status codes as mi_ntt64_plan_create (the reference panics where it is None). */
int mi_ntt64_plan_cached(size_t n, uint64_t p, int device, const mi_ntt64_plan **out_plan);

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

/* ---- The Ntt64View layer (tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:81-266), batched -------------------
 * The per-polynomial helpers every tfhe-rs NTT consumer calls (ntt64_pbs.rs:600-663, ntt64_bnf_pbs.rs:596-681,
 * lwe_bootstrap_key_conversion.rs:294-365), over `batch` polynomials of the plan's size `stride` u64 apart in both
 * operands (device pointers, async on `stream`).  Any plan; the Solinas N = 2048 plan runs them as one fused launch
 * each.  Results equal the reference's bit for bit, including what it leaves in its buffers.
 *   forward             Ntt64View::forward (:89-95):            ntt = fwd(standard)
 *   forward_normalized  Ntt64View::forward_normalized (:97-108): ntt = normalize(fwd(standard))
 *   forward_from_power_of_two_modulus (:201-214): ntt = fwd(switch(standard)), switch x -> ((x >> (64 - w)) p
 *                       + 2^(w-1)) >> w (modswitch_from_power_of_two_to_ntt_prime, :166-177), w in [1, 64]
 *   forward_from_decomp (:221-240): ntt = fwd(d), d = x + p (wrapping) where x < 0 as an i64, else x
 * For these four `ntt` may equal the input buffer (in place) or be disjoint from it.
 *   add_backward (:110-131): ntt = inv(ntt) (in place, as Plan::inv), standard = wrapping_add_custom_mod(standard,
 *                       ntt, p) (commons/numeric/unsigned.rs:174-187); standard canonical (< p)
 *   add_backward_on_power_of_two_modulus (:244-266): ntt = switch(inv(ntt)) with switch v -> (((v << w) | p >> 1) / p)
 *                       << (64 - w) (modswitch_from_ntt_prime_to_power_of_two, :184-196: an OR, not an add), then
 *                       standard += ntt (wrapping), w in [1, 64]
 * For these two `standard` and `ntt` must be disjoint.  A width outside [1, 64] (the reference's shifts overflow there)
 * or overlapping operands are MI_ERR_INVALID_ARG. */
int mi_ntt64_forward_batch(const mi_ntt64_plan *plan, uint64_t *ntt, const uint64_t *standard, size_t batch,
                           size_t stride, void *stream);
int mi_ntt64_forward_normalized_batch(const mi_ntt64_plan *plan, uint64_t *ntt, const uint64_t *standard, size_t batch,
                                      size_t stride, void *stream);
int mi_ntt64_forward_from_power_of_two_modulus_batch(const mi_ntt64_plan *plan, unsigned input_modulus_width,
                                                     uint64_t *ntt, const uint64_t *standard, size_t batch,
                                                     size_t stride, void *stream);
int mi_ntt64_forward_from_decomp_batch(const mi_ntt64_plan *plan, uint64_t *ntt, const uint64_t *decomp, size_t batch,
                                       size_t stride, void *stream);
int mi_ntt64_add_backward_batch(const mi_ntt64_plan *plan, uint64_t *standard, uint64_t *ntt, size_t batch,
                                size_t stride, void *stream);
int mi_ntt64_add_backward_on_power_of_two_modulus_batch(const mi_ntt64_plan *plan, unsigned output_modulus_width,
                                                        uint64_t *standard, uint64_t *ntt, size_t batch, size_t stride,
                                                        void *stream);

/* ---- Host-pointer convenience (copy in, run, copy out, synchronise) ---------------------
 * The single-polynomial `&mut [u64]` form of Plan::fwd / Plan::inv, batched; used by config 1
 * plumbing and the tests.  `buf` holds batch * n contiguous u64 on the host. */
int mi_ntt64_fwd_host(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch);
int mi_ntt64_inv_host(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch);
/* The same host form of the pointwise ops, on `batch` contiguous polynomials per operand, through the pooled
 * staging slots of mi_ntt64_fwd_host (no allocation, no device synchronisation in the steady state):
 * Plan::normalize (prime64.rs:1137-1179), Plan::mul_assign_normalize (prime64.rs:1050-1133),
 * Plan::mul_accumulate (prime64.rs:1182-1222) — what Ntt64View's update_with_fmadd reaches per polynomial
 * (ntt64_pbs.rs:683-702). */
int mi_ntt64_normalize_host(const mi_ntt64_plan *plan, uint64_t *buf, size_t batch);
int mi_ntt64_mul_assign_normalize_host(const mi_ntt64_plan *plan, uint64_t *lhs, const uint64_t *rhs, size_t batch);
int mi_ntt64_mul_accumulate_host(const mi_ntt64_plan *plan, uint64_t *acc, const uint64_t *lhs, const uint64_t *rhs,
                                 size_t batch);

/* ---- Synthetic input (device, async) ----------------------------------------------------
 * Fills `count` u64 with the counter-based generator of SURVEY.md §8d (splitmix64 finaliser over
 * seed + (i+1)*G + k*H, top bits dropped to bitlen(p), rejection to [0,p); p = 0: full u64 range).  Identical stream to
 * the oracle's ora_fill_uniform, so GPU-generated batches can be checked on the host. */
int mi_fill_uniform(uint64_t *buf, size_t count, uint64_t seed, uint64_t p, int device, void *stream);

/* ---- External product / CMUX / PBS (core_crypto consumers of the plan) -------------------
 * Reference paths below are relative to /root/reference/tfhe/src/core_crypto.  These run for the
 * Solinas plan (p = 2^64 - 2^32 + 1), any decomposition with base_log * level < 64, at the shapes
 *   N in {1024, 2048, 4096} with GLWE dimension k in {1, 2};
 *   N = 512 with k in {1, 4}        (shortint PARAM_MESSAGE_1_CARRY_1: N 512, k 4);
 *   N in {8192, ..., 131072} with k in {1, 2} (PARAM_MESSAGE_3_CARRY_3: N 8192, 4_4: N 65536; the accumulators of
 *                                    a chunk of ciphertexts live in HBM and each CMUX step is a sequence of
 *                                    device-wide passes);
 * other plans / shapes return MI_ERR_UNSUPPORTED.  The N = 2048, k = 1, level-1 shapes run on the hand-scheduled
 * engine, N <= 4096 on the fused one-workgroup-per-ciphertext kernels.
 * Layouts are the reference's entity layouts, contiguous:
 *   GLWE       : (k+1) polynomials of N u64 (mask then body)
 *   GGSW (NTT) : level-major, highest level first; per level (k+1) rows x (k+1) columns of N u64,
 *                each polynomial in the plan's forward (bit-reversed) NTT order
 *   BSK  (NTT) : n_lwe GGSWs back to back ((k+1)^2 * level * N u64 each)
 *   LWE        : mask (dimension u64) then body
 * Variant MI_NTT64_SOLINAS works modulo p (algorithms/lwe_programmable_bootstrapping/ntt64_pbs.rs);
 * MI_NTT64_BNF works on native 2^64 ciphertexts with the back-and-forth modulus switch
 * (ntt64_bnf_pbs.rs). */
typedef enum mi_ntt64_variant { MI_NTT64_SOLINAS = 0, MI_NTT64_BNF = 1 } mi_ntt64_variant;

/* Modulus switch of the PBS input: standard rounding (fft_impl/common.rs:10-23, as
 * ntt64_bnf_pbs.rs:512; ntt64_pbs.rs:540-549 for Solinas), the centered-binary variant the shortint
 * parameters use (BNF only, algorithms/modulus_switch.rs:35-104), or PRE_SWITCHED: lwe_in already
 * holds the switched values in [0, 2N) (the ModulusSwitchedLweCiphertext input of
 * blind_rotate_ntt64[_bnf]_assign_mem_optimized, ntt64_bnf_pbs.rs:208-266 / ntt64_pbs.rs:213-286). */
typedef enum mi_ms_mode { MI_MS_STANDARD = 0, MI_MS_CENTERED = 1, MI_MS_PRE_SWITCHED = 2 } mi_ms_mode;

/* convert_standard_lwe_bootstrap_key_to_ntt64 (algorithms/lwe_bootstrap_key_conversion.rs:294-365)
 * over `n_polys` polynomials (= n_lwe * (k+1)^2 * level): bsk_ntt = fwd(switch(bsk_std)) [* N^{-1}],
 * where switch = forward_from_power_of_two_modulus (commons/math/ntt/ntt64.rs:166-178) from a
 * 2^in_modulus_width modulus when in_modulus_width > 0, identity when 0 (Solinas-modulus keys).
 * normalize != 0 is NttLweBootstrapKeyOption::Normalize.  Device pointers, may not alias. */
int mi_bsk_to_ntt64(const mi_ntt64_plan *plan, const uint64_t *bsk_std, uint64_t *bsk_ntt, size_t n_polys,
                    unsigned in_modulus_width, int normalize, void *stream);

/* out_glwe[b] += GGSW (.) in_glwe[b] for b < batch, one shared NTT-domain GGSW:
 * add_external_product_ntt64_assign (ntt64_pbs.rs:553-663) or, for MI_NTT64_BNF,
 * add_external_product_ntt64_bnf_assign (ntt64_bnf_pbs.rs:541-681; GGSW converted Raw). */
int mi_ext_product_ntt64_batch(const mi_ntt64_plan *plan, uint64_t *out_glwe, const uint64_t *in_glwe,
                               const uint64_t *ggsw_ntt, int k, int base_log, int level, size_t batch, int variant,
                               void *stream);

/* CMUX, per item: ct1[b] -= ct0[b]; ct0[b] += GGSW (.) ct1[b] — cmux_ntt64_assign (ntt64_pbs.rs:669-680)
 * / cmux_ntt64_bnf_assign (ntt64_bnf_pbs.rs:683-705); like the reference, ct1 is left holding ct1 - ct0. */
int mi_cmux_ntt64_batch(const mi_ntt64_plan *plan, uint64_t *ct0, uint64_t *ct1, const uint64_t *ggsw_ntt, int k,
                        int base_log, int level, size_t batch, int variant, void *stream);
/* The same with one GGSW per item ("one shared GGSW or a per-item GGSW index array"): item b uses
 * GGSW ggsw_index[b] of the n_ggsw GGSWs stored back to back in ggsw_list (device u32 array of `batch` entries);
 * an item whose index is >= n_ggsw is left untouched (both its GLWEs), so a bad index never reads outside the
 * list.  Useful for batched CMUX trees and per-ciphertext selectors. */
int mi_ext_product_ntt64_batch_indexed(const mi_ntt64_plan *plan, uint64_t *out_glwe, const uint64_t *in_glwe,
                                       const uint64_t *ggsw_list, const uint32_t *ggsw_index, size_t n_ggsw, int k,
                                       int base_log, int level, size_t batch, int variant, void *stream);
int mi_cmux_ntt64_batch_indexed(const mi_ntt64_plan *plan, uint64_t *ct0, uint64_t *ct1, const uint64_t *ggsw_list,
                                const uint32_t *ggsw_index, size_t n_ggsw, int k, int base_log, int level,
                                size_t batch, int variant, void *stream);

/* A GGSW list made ready for repeated external products / CMUXes (the reference's NttGgswCiphertext[List] kept in the
 * NTT domain, entities/ntt_ggsw_ciphertext_list.rs): n_ggsw GGSWs back to back (layout above) on the plan's device.
 * The fused N = 2048, k = 1, level-1 bodies read their GGSW in their own coefficient order (pbs_tw.hip), so for that
 * shape the list is permuted once into a private copy (on `stream`, synchronised before returning; the caller's
 * buffer may then be freed); every other shape references the caller's list (keep it alive).  The raw-pointer calls
 * above permute a twisted-shape GGSW on every call. */
typedef struct mi_ntt64_ggsw mi_ntt64_ggsw;
int mi_ntt64_ggsw_create(const mi_ntt64_plan *plan, const uint64_t *ggsw_list, size_t n_ggsw, int k, int base_log,
                         int level, int variant, void *stream, mi_ntt64_ggsw **out);
int mi_ntt64_ggsw_destroy(mi_ntt64_ggsw *ggsw);
int mi_ntt64_ggsw_info(const mi_ntt64_ggsw *ggsw, size_t *n_ggsw, int *k, int *base_log, int *level, int *variant);
/* mi_ext_product_ntt64_batch / mi_cmux_ntt64_batch on a prepared list: ggsw_index NULL = GGSW 0 for every item, else
 * item b uses GGSW ggsw_index[b] (an index >= n_ggsw leaves the item untouched, as the _indexed calls). */
int mi_ext_product_ntt64_prepared_batch(const mi_ntt64_ggsw *ggsw, uint64_t *out_glwe, const uint64_t *in_glwe,
                                        const uint32_t *ggsw_index, size_t batch, void *stream);
int mi_cmux_ntt64_prepared_batch(const mi_ntt64_ggsw *ggsw, uint64_t *ct0, uint64_t *ct1, const uint32_t *ggsw_index,
                                 size_t batch, void *stream);

/* A bootstrap key made ready for mi_pbs_ntt64_batch on the plan's device.  MI_NTT64_BNF keys
 * (converted Raw, as ntt64_bnf_pbs.rs tests do) are copied once with N^{-1} folded in — the
 * reference normalises each product at run time (ntt64_bnf_pbs.rs:670); in exact mod-p arithmetic
 * both orders give identical values.  Keys of the fused N = 2048, k = 1, level-1 engine (either variant) are
 * copied once in the order its blind rotation reads (pbs_tw.hip prepare_tw_key_kernel); other
 * MI_NTT64_SOLINAS keys are referenced, not copied (the caller keeps `bsk_ntt` alive).  Replaces the
 * reference's PodStack scratch (ntt64_pbs.rs:705-751). */
typedef struct mi_pbs_ntt64_key mi_pbs_ntt64_key;
/* The copy runs on `stream` (the stream that produced bsk_ntt) and synchronises it before returning. */
int mi_pbs_ntt64_key_create(const mi_ntt64_plan *plan, const uint64_t *bsk_ntt, size_t n_lwe, int k, int base_log,
                            int level, int variant, void *stream, mi_pbs_ntt64_key **out_key);
int mi_pbs_ntt64_key_destroy(mi_pbs_ntt64_key *key);
/* n_lwe, k, base_log, level, variant of a key (any pointer may be NULL). */
int mi_pbs_ntt64_key_info(const mi_pbs_ntt64_key *key, size_t *n_lwe, int *k, int *base_log, int *level,
                          int *variant);

/* ---- On-disk NTT bootstrap key (entities/ntt_lwe_bootstrap_key.rs:26-33) -----------------------
 * MI_NTT_BSK_PLAIN     = bincode::serialize(&NttLweBootstrapKey<ABox<[u64]>>) (bincode 1.3, fixint,
 *                        little-endian): u64 count, count u64 (n_lwe, level, k+1, k+1, N NTT-domain
 *                        coefficients), polynomial_size, glwe_size, level, base_log as u64, the
 *                        SerializableCiphertextModulus (u128 modulus, u64 scalar_bits = 64).
 * MI_NTT_BSK_VERSIONED = bincode of key.versionize() (tfhe-versionable; the type has no `Named` impl,
 *                        so this is its whole versioned form): u32 1 (NttLweBootstrapKeyVersions::V1),
 *                        u32 1 (NttGgswCiphertextListVersions::V1), the data sequence, then every scalar
 *                        field behind its own u32 version tag 0 (PolynomialSizeVersions::V0, ...,
 *                        SerializableCiphertextModulusVersions::V0).
 * An NTT key's modulus is the NTT prime for both PBS variants (ntt64_bnf_pbs.rs:44-94; Ntt64::new
 * asserts a custom modulus, ntt64.rs:38); whether the values are Raw (BNF) or Normalize (Solinas) is not
 * stored, so loaders take the variant explicitly. */
typedef enum mi_ntt_bsk_format { MI_NTT_BSK_PLAIN = 0, MI_NTT_BSK_VERSIONED = 1 } mi_ntt_bsk_format;
typedef struct mi_ntt_bsk_header {
    uint64_t polynomial_size, glwe_size, level, base_log;
    uint64_t modulus_lo, modulus_hi; /* u128 ciphertext modulus (0 = native 2^64)                   */
    uint64_t input_lwe_dimension;    /* count / (level * glwe_size^2 * polynomial_size)              */
    uint64_t count;                  /* u64 elements of the key data                                 */
    uint64_t data_offset;            /* byte offset of the first element in the serialised buffer    */
} mi_ntt_bsk_header;
/* Parses and validates `len` bytes (truncated / trailing bytes, unknown version tags, scalar_bits != 64
 * as the reference's TryFrom<SerializableCiphertextModulus>, a modulus above 2^64, data that is not a
 * whole number of GGSWs, size fields whose product overflows): MI_ERR_INVALID_ARG with the reason in
 * mi_last_error_message.  A modulus of 2^64 is canonicalised to 0 (native), as TryFrom does. */
int mi_ntt_bsk_parse(const uint8_t *bytes, size_t len, int format, mi_ntt_bsk_header *out);
/* Bytes `mi_ntt_bsk_write` produces for header `h` (h->count elements; data_offset ignored). */
int mi_ntt_bsk_serialized_size(const mi_ntt_bsk_header *h, int format, size_t *out_len);
/* Serialises host `data` (h->count u64) into `out` (exactly the serialized size). */
int mi_ntt_bsk_write(const mi_ntt_bsk_header *h, const uint64_t *data, int format, uint8_t *out, size_t out_len);
/* Loads serialised key bytes (host memory) straight into HBM on the plan's device (one host-to-device
 * copy on `stream`, no re-layout) and makes a PBS key of `variant` that owns the upload: the stored
 * polynomial size must equal the plan's, glwe_size 2, and the modulus the plan's prime. */
int mi_pbs_ntt64_key_load(const mi_ntt64_plan *plan, const uint8_t *bytes, size_t len, int format, int variant,
                          void *stream, mi_pbs_ntt64_key **out_key);

/* Batched programmable bootstrap: lwe_out[b] = SampleExtract_0(BlindRotate(lut, lwe_in[b])).
 * programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized (ntt64_bnf_pbs.rs:469-540) or
 * programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized (ntt64_pbs.rs:482-538).
 * lwe_in: batch x (n_lwe + 1) u64; lut: one GLWE shared by the batch; lwe_out: batch x (k*N + 1). */
int mi_pbs_ntt64_batch(const mi_pbs_ntt64_key *key, uint64_t *lwe_out, const uint64_t *lwe_in, const uint64_t *lut,
                       size_t batch, int ms_mode, void *stream);

/* The same bootstrap with one LUT per item (the CUDA backend's lut_indexes, backends/tfhe-cuda-backend/cuda/include/
 * pbs/programmable_bootstrap.h:41; the shortint many-LUT / per-block LUT batches): lut_list holds n_lut GLWEs
 * ((k+1) N u64 each), item b uses GLWE lut_index[b] (device u32 array of `batch` entries).  An item whose index is
 * >= n_lut is left untouched (lwe_out[b] not written).  lut_index NULL: item b uses GLWE b (n_lut >= batch). */
int mi_pbs_ntt64_batch_lut_indexed(const mi_pbs_ntt64_key *key, uint64_t *lwe_out, const uint64_t *lwe_in,
                                   const uint64_t *lut_list, const uint32_t *lut_index, size_t n_lut, size_t batch,
                                   int ms_mode, void *stream);

/* Batched GLWE-output blind rotation, in place: acc_glwe[b] <- BlindRotate(acc_glwe[b], lwe_in[b]) for b < batch,
 * every item rotating its own accumulator (one LUT per ciphertext).
 *   MI_NTT64_BNF     : blind_rotate_ntt64_bnf_assign[_mem_optimized] (ntt64_bnf_pbs.rs:174-266): the CMUX loop over
 *                      the switched mask, then the division by X^ms(body).  The reference takes a
 *                      ModulusSwitchedLweCiphertext; here lwe_in is the native LWE switched inside the kernel
 *                      (MI_MS_STANDARD = lwe_ciphertext_modulus_switch, MI_MS_CENTERED = the centered binary switch,
 *                      algorithms/modulus_switch.rs) or already switched (MI_MS_PRE_SWITCHED, values in [0, 2N)).
 *   MI_NTT64_SOLINAS : blind_rotate_ntt64_assign[_mem_optimized] (ntt64_pbs.rs:176-286): the division by
 *                      X^ms(body) first, then the loop; lwe_in modulo p (MI_MS_STANDARD) or PRE_SWITCHED.
 * acc_glwe: batch x (k+1) x N u64 on the key's device.  Same shapes as mi_pbs_ntt64_batch. */
int mi_blind_rotate_ntt64_batch(const mi_pbs_ntt64_key *key, uint64_t *acc_glwe, const uint64_t *lwe_in, size_t batch,
                                int ms_mode, void *stream);

/* extract_lwe_sample_from_glwe_ciphertext (algorithms/glwe_sample_extraction.rs:89-160) at
 * MonomialDegree(nth_first + j * nth_stride) for j < nth_count, over a batch of GLWEs (k+1 polynomials of
 * polynomial_size u64): lwe_out[b * nth_count + j] (k * polynomial_size + 1 u64).  The many-LUT extraction of a
 * rotated accumulator is one call (e.g. mockups/tfhe-hpu-mockup/src/lib.rs:736-761: nth_stride = fn_stride,
 * nth_count = lut_nb).  modulus 0 = native 2^64 (wrapping opposite), else the custom modulus q.  Every degree must be
 * < polynomial_size (MI_ERR_INVALID_ARG otherwise).  Device pointers on `device`, async on `stream`. */
int mi_sample_extract_batch(uint64_t *lwe_out, const uint64_t *glwe, size_t polynomial_size, int k, size_t batch,
                            size_t nth_first, size_t nth_stride, size_t nth_count, uint64_t modulus, int device,
                            void *stream);

/* ---- Scratch pool (no reference counterpart: the reference's PodStack / ComputationBuffers) -----------------------
 * Batched entry points that need temporary device memory take it from a per-device pool of blocks kept for reuse,
 * ordered by events (a block is reissued only behind the last kernel that used it, on any stream; no call blocks the
 * host).  _trim frees the idle blocks of `device` (-1: every device) once their last users retired; _bytes reports
 * what the pool holds. */
int mi_scratch_trim(int device, size_t *released);
int mi_scratch_bytes(int device, size_t *bytes);

/* ---- Multi-GPU helpers (single process, several devices) ----------------------------------------
 * The analogue of the CUDA backend's helper_multi_gpu (backends/tfhe-cuda-backend/cuda/src/utils/
 * helper_multi_gpu.cu:10-98, helper_multi_gpu.cuh:150-265) for a host that drives several GPUs from one
 * process (as tfhe-rs's CudaStreams do).  Bootstraps and transforms are independent, so the data path has
 * no collective: batches are split contiguously (the first total % count devices take one more; with
 * fewer units than devices the first `total` take one each), read-only state is broadcast once and LWE
 * batches are scattered from / gathered to the first device with peer-to-peer copies (xGMI links on
 * MI355X).  A device may appear more than once in a set (e.g. {0, 0} rehearses the split on one GPU).
 * All copies are asynchronous: ordered after `stream` (on devices[0]) and, for gather / PBS, `stream`
 * is ordered after them. */
typedef struct mi_multi_gpu mi_multi_gpu;
/* cuda_setup_multi_gpu (helper_multi_gpu.cu:11-40): enables peer access between devices[0] and every other
 * device of the set, and creates one non-blocking stream per entry. */
int mi_multi_gpu_create(const int *devices, int count, mi_multi_gpu **out);
int mi_multi_gpu_destroy(mi_multi_gpu *m);
int mi_multi_gpu_count(const mi_multi_gpu *m, int *count);
/* device and stream (hipStream_t as void*) of entry `index` (either pointer may be NULL) */
int mi_multi_gpu_info(const mi_multi_gpu *m, int index, int *device, void **stream);
int mi_multi_gpu_synchronize(const mi_multi_gpu *m);
/* get_active_gpu_count (helper_multi_gpu.cu:42-49): min(ceil(num_inputs / 12), gpu_count), at least 1 */
int mi_multi_gpu_active_count(uint32_t num_inputs, uint32_t gpu_count, uint32_t *out);
/* get_gpu_offset / get_num_inputs_on_gpu (helper_multi_gpu.cu:51-98): entry `index`'s [offset, offset + n) */
int mi_multi_gpu_shard(size_t total, int index, int count, size_t *offset, size_t *n);
/* dsts[i] (on devices[i]) <- `bytes` at src (devices[0]); an entry equal to src is skipped */
int mi_multi_gpu_broadcast(mi_multi_gpu *m, const void *src, void *const *dsts, size_t bytes, void *stream);
/* multi_gpu_scatter_lwe_async, trivial index: dsts[i] <- shard i of `total` units of unit_bytes at src */
int mi_multi_gpu_scatter(mi_multi_gpu *m, const void *src, void *const *dsts, size_t total, size_t unit_bytes,
                         void *stream);
/* multi_gpu_gather_lwe_async, trivial index: shard i of dst (devices[0]) <- srcs[i] */
int mi_multi_gpu_gather(mi_multi_gpu *m, void *dst, const void *const *srcs, size_t total, size_t unit_bytes,
                        void *stream);
/* Batched PBS over the device set: scatter lwe_in (devices[0]), mi_pbs_ntt64_batch on every active device
 * with keys[i] / luts[i] (bound to devices[i], same shape), gather into lwe_out (devices[0]).  Only the first
 * get_active_gpu_count(batch, count) entries are active (helper_multi_gpu.cu:42-49, min(ceil(batch / 12),
 * count), as the reference's CudaStreams::active_gpu_subset, helper_multi_gpu.h:74-79); the keys / LUTs of
 * inactive entries are not read and may be NULL.  Shard 0 runs in place on `stream`; the others use
 * stream-ordered scratch on their device.
 * _ordered: producer_streams[i] is the stream of devices[i] that produced keys[i] / luts[i] (NULL array or
 * entry: that device's legacy null stream).  Shard i starts after the work queued on it and it is ordered
 * after shard i's last read, so the caller may release / reuse the LUT on that stream right away.
 * mi_pbs_ntt64_multi_gpu is _ordered with producer_streams = NULL. */
int mi_pbs_ntt64_multi_gpu(mi_multi_gpu *m, const mi_pbs_ntt64_key *const *keys, uint64_t *lwe_out,
                           const uint64_t *lwe_in, const uint64_t *const *luts, size_t batch, int ms_mode,
                           void *stream);
int mi_pbs_ntt64_multi_gpu_ordered(mi_multi_gpu *m, const mi_pbs_ntt64_key *const *keys, uint64_t *lwe_out,
                                   const uint64_t *lwe_in, const uint64_t *const *luts, size_t batch, int ms_mode,
                                   void *stream, void *const *producer_streams);

/* ---- f64-FFT PBS (the default shortint PBS path) ----------------------------
 * Reference paths relative to /root/reference/tfhe/src/core_crypto.  The negacyclic f64 FFT of
 * fft_impl/fft64/math/fft/mod.rs (Twisties :58-76, forward_as_torus / forward_as_integer / backward_as_torus
 * :406-511): N real u64 coefficients -> N/2 complex values x[n] + i x[n + N/2], twisted by exp(i pi n / N),
 * transformed with an N/2-point DFT (exp(-2 pi i / (N/2)) kernel).  Fourier buffers hold interleaved
 * (re, im) doubles, N/2 complex per polynomial, in this engine's order: position p holds frequency
 * freq[p] (mi_fft64_fourier_order).  The reference's tfhe-fft "unordered" in-memory order is implementation
 * defined, but its serialised order is the natural one: mi_fft64_to/from_standard_order convert to and from
 * it.  Results are f64 computations: parity with the reference is decryption-exact and within the FFT error bound,
 * not bit-exact.  This build: 32 <= N <= 2^18; N = 2048 runs the one-wave engine (GLWE dimension k in {1, 2}), every
 * other N the shape-generic engine (1 <= k <= 16; multi-kernel, accumulators in HBM); any decomposition with
 * base_log * level < 64. */
typedef struct mi_fft64_plan mi_fft64_plan;
/* Fft::new (fft_impl/fft64/math/fft/mod.rs:170-223): MI_ERR_INVALID_ARG if n is not a power of two,
 * MI_ERR_UNSUPPORTED for sizes this build does not compile.  _cached: one plan per (n, device), kept until
 * process exit as the reference's PLANS map (destroy is a no-op on it). */
int mi_fft64_plan_create(size_t n, int device, mi_fft64_plan **out_plan);
int mi_fft64_plan_cached(size_t n, int device, const mi_fft64_plan **out_plan);
int mi_fft64_plan_destroy(mi_fft64_plan *plan);
int mi_fft64_plan_info(const mi_fft64_plan *plan, size_t *n, int *device);
/* freq[p] for p < n/2: the DFT frequency stored at Fourier position p (host call) */
int mi_fft64_fourier_order(const mi_fft64_plan *plan, uint32_t *freq);
/* The reference's serialised Fourier order (FourierPolynomialList's serde, fft_impl/fft64/math/fft/mod.rs:642-690,
 * through tfhe-fft's Plan::serialize_fourier_buffer / deserialize_fourier_buffer, tfhe-fft/src/unordered.rs:943-1020):
 * element i of a serialised polynomial is DFT frequency i, whatever the plan's internal order.  These convert
 * `polys` polynomials of n/2 complex between that natural order and this engine's (device pointers, async; in place
 * when the two pointers are equal), so a FourierLweBootstrapKey / FourierGgswCiphertext deserialised by the
 * reference's own serde loads with one call, and a key converted here serialises as the reference expects. */
int mi_fft64_to_standard_order(const mi_fft64_plan *plan, double *standard_order, const double *fourier, size_t polys,
                               void *stream);
int mi_fft64_from_standard_order(const mi_fft64_plan *plan, double *fourier, const double *standard_order,
                                 size_t polys, void *stream);
/* FftView::forward_as_torus / backward_as_torus (add != 0: add_backward_as_torus), per polynomial over a
 * batch of contiguous polynomials (device pointers, async): fourier = batch x n/2 x 2 doubles. */
int mi_fft64_forward_torus_batch(const mi_fft64_plan *plan, double *fourier, const uint64_t *standard, size_t batch,
                                 void *stream);
int mi_fft64_backward_torus_batch(const mi_fft64_plan *plan, uint64_t *standard, const double *fourier, size_t batch,
                                  int add, void *stream);
/* convert_standard_lwe_bootstrap_key_to_fourier (algorithms/lwe_bootstrap_key_conversion.rs:20-43): every
 * polynomial of the standard key (n_polys = n_lwe (k+1)^2 level) through forward_as_torus. */
int mi_bsk_to_fourier64(const mi_fft64_plan *plan, const uint64_t *bsk_std, double *bsk_fourier, size_t n_polys,
                        void *stream);
/* add_external_product_assign / cmux_assign (algorithms/lwe_programmable_bootstrapping/fft64_pbs.rs:270-330,
 * 510-560; fft_impl/fft64/crypto/ggsw.rs:483-603): native 2^64 GLWEs, one shared Fourier GGSW (level x (k+1)
 * x (k+1) x n/2 complex, highest level first).  CMUX leaves ct1 holding ct1 - ct0, as the reference. */
int mi_fft64_ext_product_batch(const mi_fft64_plan *plan, uint64_t *out_glwe, const uint64_t *in_glwe,
                               const double *ggsw_fourier, int k, int base_log, int level, size_t batch, void *stream);
int mi_fft64_cmux_batch(const mi_fft64_plan *plan, uint64_t *ct0, uint64_t *ct1, const double *ggsw_fourier, int k,
                        int base_log, int level, size_t batch, void *stream);
/* A Fourier bootstrap key (FourierLweBootstrapKey, referenced: the caller keeps `fbsk` alive) and the batched
 * programmable_bootstrap_lwe_ciphertext (fft64_pbs.rs:924-1060; blind rotation fft_impl/fft64/crypto/
 * bootstrap.rs:294-381, 481-521).  ms_mode as mi_pbs_ntt64_batch. */
typedef struct mi_fft64_pbs_key mi_fft64_pbs_key;
int mi_fft64_pbs_key_create(const mi_fft64_plan *plan, const double *fbsk, size_t n_lwe, int k, int base_log,
                            int level, mi_fft64_pbs_key **out_key);
int mi_fft64_pbs_key_destroy(mi_fft64_pbs_key *key);
int mi_fft64_pbs_key_info(const mi_fft64_pbs_key *key, size_t *n_lwe, int *k, int *base_log, int *level);
int mi_fft64_pbs_batch(const mi_fft64_pbs_key *key, uint64_t *lwe_out, const uint64_t *lwe_in, const uint64_t *lut,
                       size_t batch, int ms_mode, void *stream);
/* One accumulator per item: lut_index NULL = batch_programmable_bootstrap_lwe_ciphertext_mem_optimized
 * (fft64_pbs.rs:1055-1127: item b bootstraps through GLWE b of lut_list, n_lut >= batch); otherwise item b uses GLWE
 * lut_index[b] (device u32) and an index >= n_lut leaves lwe_out[b] untouched. */
int mi_fft64_pbs_batch_lut_indexed(const mi_fft64_pbs_key *key, uint64_t *lwe_out, const uint64_t *lwe_in,
                                   const uint64_t *lut_list, const uint32_t *lut_index, size_t n_lut, size_t batch,
                                   int ms_mode, void *stream);
/* blind_rotate_assign[_mem_optimized] (fft64_pbs.rs:186-250; FourierLweBootstrapKey::blind_rotate_assign,
 * fft_impl/fft64/crypto/bootstrap.rs:294-381), batched and in place: acc_glwe[b] ((k+1) N u64) is divided by
 * X^ms(body) and rotated through the CMUX loop over lwe_in[b].  ms_mode as mi_pbs_ntt64_batch (the reference's
 * ModulusSwitchedLweCiphertext input: MI_MS_PRE_SWITCHED, or the native LWE switched on the device). */
int mi_fft64_blind_rotate_batch(const mi_fft64_pbs_key *key, uint64_t *acc_glwe, const uint64_t *lwe_in, size_t batch,
                                int ms_mode, void *stream);
/* The multi-GPU bootstrap of mi_pbs_ntt64_multi_gpu[_ordered] (same sharding, active-GPU count, scatter / gather and
 * producer-stream ordering) on the f64-FFT path: keys[i] (bound to a plan of devices[i], same shape) and luts[i] on
 * devices[i], lwe_in / lwe_out on devices[0]. */
int mi_fft64_pbs_multi_gpu(mi_multi_gpu *m, const mi_fft64_pbs_key *const *keys, uint64_t *lwe_out,
                           const uint64_t *lwe_in, const uint64_t *const *luts, size_t batch, int ms_mode,
                           void *stream);
int mi_fft64_pbs_multi_gpu_ordered(mi_multi_gpu *m, const mi_fft64_pbs_key *const *keys, uint64_t *lwe_out,
                                   const uint64_t *lwe_in, const uint64_t *const *luts, size_t batch, int ms_mode,
                                   void *stream, void *const *producer_streams);
/* The reference's serialised FourierLweBootstrapKey (fft_impl/fft64/crypto/bootstrap.rs:30-39, the list's custom
 * Serialize fft_impl/fft64/math/fft/mod.rs:642-690, bincode 1.3 defaults as for the NTT key): format
 * MI_NTT_BSK_PLAIN = bincode::serialize(&key): u64 (2 + P), u64 polynomial_size, u64 P, then P polynomials each as
 * u64 (N/2) and N/2 (re, im) f64 pairs in the natural DFT order (tfhe-fft/src/unordered.rs:943-964), then
 * input_lwe_dimension, glwe_size, decomposition_base_log, decomposition_level_count as u64;
 * MI_NTT_BSK_VERSIONED = bincode of key.versionize(): u32 1 (FourierLweBootstrapKeyVersions::V1), u32 0
 * (FourierPolynomialListVersioned::V0), the same list, a u32 0 before each scalar field
 * (backward_compatibility/fft_impl/mod.rs:14-70).  _load validates the bytes (length, tags, per-polynomial length,
 * P = n_lwe level glwe_size^2, the plan's polynomial size), uploads them with one strided copy and reorders them
 * into this engine's order on `stream` (synchronised before returning); the key owns that device copy.  _write
 * produces exactly mi_fft64_bsk_serialized_size bytes from any key (a loaded one or one over a caller tensor). */
int mi_fft64_bsk_serialized_size(size_t polynomial_size, size_t n_lwe, int k, int level, int format,
                                 size_t *out_len);
int mi_fft64_pbs_key_load(const mi_fft64_plan *plan, const uint8_t *bytes, size_t len, int format, void *stream,
                          mi_fft64_pbs_key **out_key);
int mi_fft64_pbs_key_write(const mi_fft64_pbs_key *key, int format, uint8_t *out, size_t out_len, void *stream);

/* ---- prime32::Plan (tfhe-ntt/src/prime32.rs:632-1025) ----------------------------------------
 * The same negacyclic transform and pointwise ops on u32 buffers for a prime p < 2^32.  try_new
 * (prime32.rs:662-671) returns None for N < 32, N not a power of two, p not prime, no 2N-th root:
 * here MI_ERR_INVALID_ARG / MI_ERR_NOT_PRIME / MI_ERR_NO_ROOT.  Twiddles follow
 * init_negacyclic_twiddles (prime32.rs:223-246), outputs are canonical (< p) as the reference's
 * tests assert (prime32.rs:1114-1133). */
typedef struct mi_ntt32_plan mi_ntt32_plan;
int mi_ntt32_plan_create(size_t n, uint32_t p, int device, mi_ntt32_plan **out_plan);
int mi_ntt32_plan_destroy(mi_ntt32_plan *plan);
int mi_ntt32_plan_info(const mi_ntt32_plan *plan, size_t *n, uint32_t *p, int *device);
/* Plan::fwd / Plan::inv (prime32.rs:797-898) */
int mi_ntt32_fwd_batch(const mi_ntt32_plan *plan, uint32_t *buf, size_t batch, size_t stride, void *stream);
int mi_ntt32_inv_batch(const mi_ntt32_plan *plan, uint32_t *buf, size_t batch, size_t stride, void *stream);
/* Plan::normalize / mul_assign_normalize / mul_accumulate (prime32.rs:900-1025) */
int mi_ntt32_normalize_batch(const mi_ntt32_plan *plan, uint32_t *buf, size_t batch, size_t stride, void *stream);
int mi_ntt32_mul_assign_normalize_batch(const mi_ntt32_plan *plan, uint32_t *lhs, const uint32_t *rhs,
                                        size_t batch, size_t stride, void *stream);
int mi_ntt32_mul_accumulate_batch(const mi_ntt32_plan *plan, uint32_t *acc, const uint32_t *lhs,
                                  const uint32_t *rhs, size_t batch, size_t stride, void *stream);

/* ---- Exact native-modulus negacyclic products over a CRT of NTT primes ----------------------
 * negacyclic_polymul of native32.rs:410-500, native64.rs:1041-1160, native128.rs:297-320 and the
 * binary-RHS plans native_binary{32,64,128}.rs (rhs coefficients in {0,1}): prod = lhs * rhs in
 * Z_{2^W}[X]/(X^N + 1), W = 32 / 64 / 128 (u128 = two little-endian u64 words).  The prime sets are
 * the reference's (lib.rs primes32 / primes52).  Plan52 kinds exist in the reference only on CPUs
 * with AVX-512 IFMA (their try_new returns None otherwise); here they always exist. */
typedef enum mi_native_kind {
    MI_NATIVE32_PLAN32 = 0,        /* native32::Plan32           P0..P2 (32-bit)  */
    MI_NATIVE32_PLAN52 = 1,        /* native32::Plan52           P0..P1 (52-bit)  */
    MI_NATIVE64_PLAN32 = 2,        /* native64::Plan32           P0..P4 (32-bit)  */
    MI_NATIVE64_PLAN52 = 3,        /* native64::Plan52           P0..P2 (52-bit)  */
    MI_NATIVE128_PLAN32 = 4,       /* native128::Plan32          P0..P9 (32-bit)  */
    MI_NATIVE_BINARY32_PLAN32 = 5, /* native_binary32::Plan32    P0..P1 (32-bit)  */
    MI_NATIVE_BINARY32_PLAN52 = 6, /* native_binary32::Plan52    P0     (52-bit)  */
    MI_NATIVE_BINARY64_PLAN32 = 7, /* native_binary64::Plan32    P0..P2 (32-bit)  */
    MI_NATIVE_BINARY64_PLAN52 = 8, /* native_binary64::Plan52    P0..P1 (52-bit)  */
    MI_NATIVE_BINARY128_PLAN32 = 9 /* native_binary128::Plan32   P0..P4 (32-bit)  */
} mi_native_kind;
typedef struct mi_native_plan mi_native_plan;
/* Plan32/Plan52::try_new(n) (e.g. native64.rs:932-941): None when a component prime plan is. */
int mi_native_plan_create(int kind, size_t n, int device, mi_native_plan **out_plan);
int mi_native_plan_destroy(mi_native_plan *plan);
int mi_native_plan_info(const mi_native_plan *plan, size_t *n, int *width_bits, int *num_primes);
/* Batched negacyclic_polymul: `batch` contiguous polynomials of n words each in prod/lhs/rhs
 * (device pointers, async on `stream`; scratch is stream-ordered and freed before return). */
int mi_native_polymul_batch(const mi_native_plan *plan, void *prod, const void *lhs, const void *rhs, size_t batch,
                            void *stream);

/* ---- LWE keyswitch (tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs) ---------------------------
 * The keyswitch in front of the PBS in the shortint KS-PBS order (PARAM_MESSAGE_2_CARRY_2:
 * 2048 -> 918, base 2^4, 4 levels; shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/ks_pbs.rs:29-47).
 * mi_lwe_ksk_create takes the reference's LweKeyswitchKey layout as a device pointer: in_dim blocks of
 * `level` LWE ciphertexts of out_dim + 1 u64, levels stored as generate_lwe_keyswitch_key writes them
 * (lwe_keyswitch_key_generation.rs:169-199), and prepares a private device copy (the caller's buffer
 * may be freed afterwards; the preparation runs on `stream`, the stream that produced `ksk`, and synchronises
 * it).  MI_ERR_INVALID_ARG where SignedDecomposer::new would assert
 * (base_log * level >= 64); MI_ERR_UNSUPPORTED when in_dim * level * ceil((base_log + 1) / 8) >= 2^17
 * (beyond the exact int32 accumulation of the int8 matrix-core path). */
typedef struct mi_lwe_ksk mi_lwe_ksk;
int mi_lwe_ksk_create(const uint64_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level, int device,
                      void *stream, mi_lwe_ksk **out_key);
int mi_lwe_ksk_destroy(mi_lwe_ksk *key);
int mi_lwe_ksk_info(const mi_lwe_ksk *key, size_t *in_dim, size_t *out_dim, int *base_log, int *level);
/* keyswitch_lwe_ciphertext_native_mod_compatible (lwe_keyswitch.rs:137-227) over a batch:
 * lwe_out[b] (out_dim + 1 u64) = keyswitch(lwe_in[b] (in_dim + 1 u64)), native 2^64 modulus, bit-exact.
 * Device pointers, async on `stream` (stream-ordered scratch, freed before return). */
int mi_lwe_keyswitch_batch(const mi_lwe_ksk *key, uint64_t *lwe_out, const uint64_t *lwe_in, size_t batch,
                           void *stream);

/* ---- KS32: the keyswitch with a scalar change of the HPU KS32 parameter sets ----------------------------------
 * keyswitch_lwe_ciphertext_with_scalar_change (lwe_keyswitch.rs:331-447), as V1_5_HPU_PARAM_MESSAGE_2_CARRY_2_KS32_
 * PBS_TUNIFORM_2M128 runs it (shortint/parameters/v1_5/hpu.rs:57-76: 2048 -> 879, ks base 2^2, 8 levels,
 * post_keyswitch_ciphertext_modulus 2^21; mockups/tfhe-hpu-mockup/src/lib.rs:720-736): u64 input LWEs (native
 * modulus) -> u32 output LWEs of modulus 2^out_modulus_log, power-of-two encoded in the MSBs of the u32 words, as the
 * reference stores non-native power-of-two moduli.  The key: in_dim blocks of `level` u32 LWE ciphertexts of
 * out_dim + 1 words (the LweKeyswitchKey<Vec<u32>> layout, levels as generate_lwe_keyswitch_key writes them).
 * The body is closest_representable(b) at out_modulus_log bits, shifted down by 32; every mask digit of the u64
 * SignedDecomposer (base_log, level) times its key row is subtracted with wrapping u32 arithmetic.
 * MI_ERR_INVALID_ARG where the reference asserts (base_log * level > 32) or out_modulus_log is outside [1, 32];
 * the same 2^17 GEMM-depth bound as mi_lwe_ksk_create.  Bit-exact. */
typedef struct mi_lwe_ksk32 mi_lwe_ksk32;
int mi_lwe_ksk32_create(const uint32_t *ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                        int out_modulus_log, int device, void *stream, mi_lwe_ksk32 **out_key);
int mi_lwe_ksk32_destroy(mi_lwe_ksk32 *key);
int mi_lwe_ksk32_info(const mi_lwe_ksk32 *key, size_t *in_dim, size_t *out_dim, int *base_log, int *level,
                      int *out_modulus_log);
int mi_lwe_keyswitch32_batch(const mi_lwe_ksk32 *key, uint32_t *lwe_out, const uint64_t *lwe_in, size_t batch,
                             void *stream);
/* The modulus switch of u32 LWEs (lwe_dim mask words + body) to [0, 2^log_modulus): MI_MS_STANDARD =
 * lwe_ciphertext_modulus_switch, MI_MS_CENTERED = lwe_ciphertext_centered_binary_modulus_switch
 * (algorithms/modulus_switch.rs:14-104, at Scalar = u32), materialised as the ModulusSwitchedLweCiphertext values
 * (entities/modulus_switched_lwe_ciphertext.rs:150-175): switched[b] = lwe_dim + 1 u64 in [0, 2^log_modulus), the
 * MI_MS_PRE_SWITCHED input of mi_blind_rotate_ntt64_batch / mi_pbs_ntt64_batch (log_modulus = log2(2N)). */
int mi_lwe_modulus_switch32_batch(uint64_t *switched, const uint32_t *lwe_in, size_t lwe_dim, size_t batch,
                                  int log_modulus, int ms_mode, int device, void *stream);
/* The same switch of u64 LWEs (the native 2^64 ciphertexts in front of every other blind rotation):
 * lwe_ciphertext_modulus_switch / lwe_ciphertext_centered_binary_modulus_switch (algorithms/modulus_switch.rs:14-104)
 * at Scalar = u64, materialised as the LazyStandardModulusSwitchedLweCiphertext reads them
 * (entities/modulus_switched_lwe_ciphertext.rs:150-175) — what the HPU mockup runs before blind_rotate_ntt64_bnf_assign
 * (mockups/tfhe-hpu-mockup/src/lib.rs:725-736).  Both forms: log_modulus in [1, BITS] for MI_MS_STANDARD (identity at
 * BITS, fft_impl/common.rs:10-23) and [1, BITS - 1] for MI_MS_CENTERED, whose half_case shift (modulus_switch.rs:95)
 * underflows at BITS in the reference; anything else is MI_ERR_INVALID_ARG.  BITS = 32 for the u32 call above. */
int mi_lwe_modulus_switch_batch(uint64_t *switched, const uint64_t *lwe_in, size_t lwe_dim, size_t batch,
                                int log_modulus, int ms_mode, int device, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* TFHE_NTT_AMD_H */
