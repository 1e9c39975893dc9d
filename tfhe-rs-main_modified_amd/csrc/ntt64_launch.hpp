// ntt64_launch.hpp — host-side launchers exported by ntt64_kernels.hip to the C ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pbs_io.hpp"

namespace mi {

// Montgomery parameters for a generic odd prime (R = 2^64).
struct MontParams {
  uint64_t p = 0, pinv = 0, r2 = 0;
};

// Register-window transform kernels (ntt64_kernels.hip).  `tw` points at the plan's device table
// (forward or inverse).
hipError_t launch_ntt(bool fwd, int logn, bool goldilocks, const MontParams& mp, uint64_t* data,
                      size_t batch, size_t stride, const uint64_t* tw, hipStream_t s);

// p < 2^32 plans (Shoup32 tables): u64 buffers (data64) or the prime32 plans' u32 buffers (data32); prime32 pointwise ops
// (u32 buffers, Montgomery constants)
hipError_t launch_ntt_shoup32(bool fwd, int logn, uint32_t p, uint64_t* data64, uint32_t* data32, size_t batch,
                              size_t stride, const uint64_t* tw, hipStream_t s);
hipError_t launch_pointwise_u32(int op, const MontParams& mp, uint32_t* out, const uint32_t* a, const uint32_t* b,
                                size_t n, size_t batch, size_t stride, uint64_t c, hipStream_t s);

// Twisted shift-twiddle transform (ntt64_tw.hip): Solinas prime, N = 2048 only.  `twist` = the
// plan's rho_i^j table (forward) or rho_i^-j table (inverse), 2048 u64 each.
// key conversion of native-modulus polynomials (N = 2048 Solinas plan): dst = fwd(modswitch_{2^64 -> p}(src))
hipError_t launch_ntt_tw_ms64(uint64_t* dst, const uint64_t* src, size_t n_polys, const uint64_t* twist,
                              hipStream_t s);
// The Ntt64View layer (ntt64_view.hip, ntt64.rs:89-266).  Generic passes for any plan: view_pre writes
// ntt = conv(standard) (kind 0 copy, 1 switch 2^width -> p, 2 negative decomposition digits + p) ahead of the plan's
// forward; view_post follows its inverse (width > 0: ntt = switch p -> 2^width, standard += ntt wrapping; width 0:
// standard = wrapping_add_custom_mod(standard, ntt, p)).  The fused twisted N = 2048 forms: view_fwd_tw (same kinds,
// any width for kind 1; twist = the forward table or its N^-1 copy) and view_inv_tw (pow2_64: the width-64 switch;
// else the custom-modulus add).
hipError_t launch_view_pre(int kind, uint64_t* ntt, const uint64_t* standard, size_t n, size_t batch, size_t stride,
                           unsigned width, uint64_t p, hipStream_t s);
hipError_t launch_view_post(uint64_t* standard, uint64_t* ntt, size_t n, size_t batch, size_t stride, unsigned width,
                            uint64_t p, hipStream_t s);
hipError_t launch_view_fwd_tw(int kind, uint64_t* ntt, const uint64_t* standard, size_t batch, size_t stride,
                              unsigned width, const uint64_t* twist, hipStream_t s);
hipError_t launch_view_inv_tw(bool pow2_64, uint64_t* standard, uint64_t* ntt, size_t batch, size_t stride,
                              const uint64_t* twist, hipStream_t s);
hipError_t launch_ntt_tw(bool fwd, uint64_t* data, size_t batch, size_t stride, const uint64_t* twist,
                         hipStream_t s, int sub_log = 0);
// The MAC-fused inverse bodies of the large-N blind rotation (ntt64_tw.hip): for n_items ciphertexts, every 2048-block
// of the k + 1 products y[b][c] = sum_{li, r} digits[b][li][r] . ggsw[li][r][c] (NTT domain, the step's GGSW with any
// normalisation folded in) formed on load and run through the inverse body (the split inverse's first phase);
// twist = the 2048 plan's inverse body table (SplitTw body_inv).  l (k + 1) in {2, 3, 4, 6, 8} (inv_mac_supported).
bool inv_mac_supported(int level, int kp1);
hipError_t launch_ntt_tw_inv_mac(uint64_t* y, const uint64_t* digits, const uint64_t* ggsw, size_t n_items, int kp1,
                                 int level, int logn, const uint64_t* twist, hipStream_t s);

// The split transform of a Solinas plan with 2^12 <= N <= 2^MI_SPLIT_MAX_LOGN = 2^20 (ntt64_kernels.hip; GPU parity:
// tests/test_ntt_gpu.py test_fwd_inv_all_sizes_solinas 2^12 .. 2^18, test_fwd_inv_beyond_2_18 2^19 / 2^20 — the
// two-pass tops t = 7 .. 9 —, test_large_n_strided_batch up to 2^19): the reference's first
// t = log2 N - 11 stages as passes over strided columns, the block twist (element j of 2048-block b times alpha_b^j,
// alpha_b = psi_N^(2 bitrev_t(b) + 1 - 2^t)) fused into the last forward / first inverse pass, and every 2048-block
// through the twisted N = 2048 body (ntt64_tw.hip) of the cached 2048-point Solinas plan.  Device tables:
struct SplitTw {
  const uint64_t* blk_fwd = nullptr;   // N: alpha_b^j at b 2048 + j
  const uint64_t* blk_inv = nullptr;   // N: alpha_b^-j
  const uint64_t* body_fwd = nullptr;  // the 2048 plan's d_twist_f (forward body tables)
  const uint64_t* body_inv = nullptr;  // the 2048 plan's d_twist_i (inverse body tables)
};
// tw = the N plan's forward (fwd) or inverse (inv) twiddle table; data: batch polynomials `stride` u64 apart
// acc (inverse only): the last top pass accumulates its output into acc (same layout as data) instead of storing it,
// acc_mode 1 = BNF (acc += modswitch p -> 2^64), 2 = Solinas (acc = acc + x mod p); data then holds an intermediate
// skip_first: the transform's first phase already ran — the forward's first top pass (fused into the blind rotation's
// rotation + decomposition pass) or the inverse's 2048-block bodies (launch_ntt_tw_inv_mac)
// the split transform of N = 2^(11 + t), t <= 3, as one launch (ntt64_tw.hip ntt_tw_fused_kernel): blk = the block
// twist (SplitTw blk_fwd / blk_inv), body_tab = the 2048 body's table (body_fwd / body_inv)
hipError_t launch_ntt_split_fused(bool fwd, int t, uint64_t* data, size_t batch, size_t stride, const uint64_t* blk,
                                  const uint64_t* body_tab, hipStream_t s);
hipError_t launch_ntt_split(bool fwd, int logn, uint64_t* data, size_t batch, size_t stride, const uint64_t* tw,
                            const SplitTw& st, hipStream_t s, uint64_t* acc = nullptr, int acc_mode = 0,
                            bool skip_first = false);
// how launch_ntt_split cuts the t = log2 N - 11 top stages into passes: the first pass's stage count (the forward's
// first pass, s0 = 0) and whether it is the only one (then it carries the block twist)
inline void split_first_pass(int logn, int* k0, bool* only) {
  const int t = logn - 11, passes = (t + 4) / 5;
  *k0 = (t + passes - 1) / passes;
  *only = passes == 1;
}

// op: 0 normalize (out *= c), 1 mul_assign_normalize (out = out*b*c), 2 mul_accumulate (out += a*b[*c])
hipError_t launch_pointwise(int op, bool goldilocks, const MontParams& mp, uint64_t* out, const uint64_t* a,
                            const uint64_t* b, size_t n, size_t batch, size_t stride, uint64_t c, hipStream_t s);

// native-modulus CRT products (native_crt.hip): up to 10 primes; prefix = prod_{l<k} p_l mod 2^128,
// inv_prefix[k] = (prod_{l<k} p_l)^-1 mod p_k, m = prod of all primes mod 2^128
constexpr int MI_CRT_MAX = 10;
struct CrtConst {
  int k = 0, prime_bits = 32;
  uint64_t p[MI_CRT_MAX] = {}, inv_prefix[MI_CRT_MAX] = {}, prefix_lo[MI_CRT_MAX] = {}, prefix_hi[MI_CRT_MAX] = {};
  uint64_t m_lo = 0, m_hi = 0;
  // Montgomery constants per prime (R = 2^64; r6: the residue split and the Garner steps without 128-bit division):
  // pinv = -p^-1 mod R, r1 = R mod p, r2 = R^2 mod p, inv_prefix_m = inv_prefix R mod p, pjk_m[j][k] = (p_j mod p_k) R mod p_k
  uint64_t pinv[MI_CRT_MAX] = {}, r1[MI_CRT_MAX] = {}, r2[MI_CRT_MAX] = {}, inv_prefix_m[MI_CRT_MAX] = {};
  uint64_t pjk_m[MI_CRT_MAX][MI_CRT_MAX] = {};
};
hipError_t launch_crt_residues(uint64_t* planes, const void* in, size_t count, int width, int binary,
                               const CrtConst& c, hipStream_t s);
hipError_t launch_crt_reconstruct(void* out, const uint64_t* planes, size_t count, int width, const CrtConst& c,
                                  hipStream_t s);

hipError_t launch_fill_uniform(uint64_t* out, size_t count, uint64_t seed, uint64_t p, hipStream_t s);

}  // namespace mi

namespace mi {

// pbs_kernels.hip — Goldilocks, the shapes of mi::capi::check_pbs_shape up to N = 8192, any level count (callers
// validate the shape; other shapes return hipErrorInvalidValue).
hipError_t launch_lift_switched(uint64_t* dst, const uint64_t* src, size_t count, bool bnf, int logn, hipStream_t s);
hipError_t launch_bsk_to_ntt(int logn, uint64_t* dst, const uint64_t* src, size_t n_polys, unsigned in_width,
                             int normalize, uint64_t n_inv, const uint64_t* tw, hipStream_t s);
hipError_t launch_scale(uint64_t* dst, const uint64_t* src, size_t count, uint64_t c, hipStream_t s);
// cmux: glwe -= out first (written back), then out += GGSW (.) glwe
// gidx (device, may be NULL): item b uses GGSW gidx[b] of the n_ggsw in `ggsw` (an index >= n_ggsw leaves the item
// untouched); NULL: every item uses the one GGSW (n_ggsw must then be >= 1)
hipError_t launch_ext_product(int logn, int k, bool bnf, bool cmux, int level, uint64_t* out, uint64_t* glwe,
                              const uint64_t* ggsw, size_t batch, int base_log, const uint64_t* tw,
                              const uint64_t* itw, uint64_t n_inv, hipStream_t s, const uint32_t* gidx = nullptr,
                              uint32_t n_ggsw = 1);
hipError_t launch_pbs(int logn, int k, bool bnf, int level, uint64_t* out, const uint64_t* lwe_in, const PbsIo& io,
                      const uint64_t* bsk, size_t n_lwe, size_t batch, int base_log, const uint64_t* tw,
                      const uint64_t* itw, int centered, hipStream_t s);
// extract_lwe_sample_from_glwe_ciphertext (glwe_sample_extraction.rs:89-160) at MonomialDegree(nth_first + j nth_stride)
// for j < nth_count of every GLWE: out[b nth_count + j] (k N + 1 u64); modulus 0 = native 2^64
hipError_t launch_sample_extract(uint64_t* out, const uint64_t* glwe, int logn, int k, size_t batch, size_t nth_first,
                                 size_t nth_stride, size_t nth_count, uint64_t modulus, hipStream_t s);
// pbs_large.hip — N = 2^14 ... 2^17 (beyond one workgroup): the blind rotation / external product as device-wide
// passes per CMUX step over chunks of ciphertexts whose accumulators live in HBM; same arguments as above
hipError_t launch_pbs_large(int logn, int k, bool bnf, int level, uint64_t* out, const uint64_t* lwe_in,
                            const PbsIo& io, const uint64_t* bsk, size_t n_lwe, size_t batch, int base_log,
                            const uint64_t* tw, const uint64_t* itw, int centered, hipStream_t s,
                            const SplitTw* split = nullptr);
hipError_t launch_ext_product_large(int logn, int k, bool bnf, bool cmux, int level, uint64_t* out, uint64_t* glwe,
                                    const uint64_t* ggsw, size_t batch, int base_log, const uint64_t* tw,
                                    const uint64_t* itw, uint64_t n_inv, hipStream_t s, const uint32_t* gidx,
                                    uint32_t n_ggsw, const SplitTw* split = nullptr);
hipError_t launch_bsk_to_ntt_large(int logn, uint64_t* dst, const uint64_t* src, size_t n_polys, unsigned in_width,
                                   int normalize, uint64_t n_inv, const uint64_t* tw, hipStream_t s,
                                   const SplitTw* split = nullptr);
// BNF, level 1, base_log <= 31, on the twisted transform; tab = plan twist tables [fwd | inverse]
// BNF level-1 external product (cmux=false: out += GGSW . glwe) / CMUX (cmux=true: ct0 = out,
// ct1 = glwe) on the twisted transform; the GGSW is the Raw NTT key (N^-1 via the third table)
// prepared: the GGSWs are already in the bodies' read order (ext_tw_reads_w1p(): mi_ntt64_ggsw_create permuted them)
hipError_t launch_ext_tw(bool cmux, bool sol, uint64_t* out, uint64_t* glwe, const uint64_t* ggsw, size_t batch,
                         int base_log, const uint64_t* tab, hipStream_t s, const uint32_t* gidx = nullptr,
                         uint32_t n_ggsw = 1, bool prepared = false);
// whether the external-product / CMUX bodies read their GGSW in the W1' order (a prepared list is permuted once)
bool ext_tw_reads_w1p();
// Solinas PBS on the twisted engine: switched = pre-switched mask + body values in [0, 2N)
// the twisted bodies' key order (pbs_tw.hip): per N = 2048 polynomial, positions permuted to the W1' step layout
// when the blind-rotation (ext: external-product) body reads that order, times c when scale (dst may equal src)
hipError_t launch_prepare_tw_key(uint64_t* dst, const uint64_t* src, size_t n_polys, uint64_t c, int scale,
                                 hipStream_t s, bool ext = false);
hipError_t launch_ms_non_native(uint64_t* dst, const uint64_t* src, size_t count, hipStream_t s);
hipError_t launch_pbs_tw_sol(uint64_t* out, const uint64_t* switched, const PbsIo& io, const uint64_t* bsk,
                             size_t n_lwe, size_t batch, int base_log, const uint64_t* tab, hipStream_t s);
hipError_t launch_pbs_tw(uint64_t* out, const uint64_t* lwe_in, const PbsIo& io, const uint64_t* bsk, size_t n_lwe,
                         size_t batch, int base_log, const uint64_t* tab, int centered, hipStream_t s);

}  // namespace mi
// (keyswitch.hip's entry points: keyswitch_launch.hpp)
