// pbs_kernels.hip — NTT-domain GGSW x GLWE external product, CMUX / blind rotation and programmable
// bootstrap for MI355X, in both NTT flavours of tfhe core_crypto (reference paths relative to
// /root/reference/tfhe/src/core_crypto):
//   BNF     : native 2^64 ciphertexts, back-and-forth modulus switch to the Goldilocks prime
//             (algorithms/lwe_programmable_bootstrapping/ntt64_bnf_pbs.rs:208-726)
//   SOLINAS : ciphertexts modulo the prime (algorithms/lwe_programmable_bootstrapping/ntt64_pbs.rs:213-702)
// for every shape the twisted engine (pbs_tw.hip: N = 2048, k = 1, level 1) does not cover: polynomial
// sizes N = 2^LOGN (1024, 2048, 4096), GLWE dimension k = K (1, 2), any decomposition level count
// (a runtime loop), as the reference's shape-generic code (ntt64_bnf_pbs.rs:541-681, ntt64_pbs.rs:553-663).
//
// MI355X design: one workgroup (T = N / 8 lanes) owns one ciphertext for the WHOLE blind rotation.  The
// GLWE accumulator (k+1 polynomials) lives in VGPRs across all n CMUX steps, so the only per-step global
// traffic is the step's NTT GGSW (shared by every workgroup of the launch, hence L2/MALL-resident: all
// workgroups walk the key in the same order).  Each step rotates through LDS, decomposes in registers,
// runs (k+1) forward + (k+1) inverse NTTs per level with the register-window engine of ntt64_regs.hpp,
// multiply-accumulates against the GGSW in the NTT domain and switches the result back — the
// reference's host-side passes per CMUX fused into one loop body.
//
// Bit-exactness: every step restates the reference arithmetic exactly; the only reordering is the
// BNF N^{-1} normalisation, which is folded into a private copy of the key (exact: Goldilocks
// arithmetic is canonical, (sum a*g) * N^-1 == sum a*(g*N^-1) mod p).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_regs.hpp"
#include "pbs_device.hpp"

namespace mi {
namespace pbs {

// Coefficients per lane: 8, or 4 for the wide GLWEs (k >= 3, e.g. N = 512, k = 4 of PARAM_MESSAGE_1_CARRY_1,
// shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/ks_pbs.rs:8-27), whose (k + 1) polynomials of
// accumulator, digits and products must stay in the registers of one lane.
template <int K>
constexpr int loge_for() { return K >= 3 ? 2 : 3; }

// Waves per SIMD the level-1 kernels are compiled for (amdgpu_waves_per_eu): 2 fits N = 512, k = 4 in 254 VGPRs
// without spilling; the k = 1 shapes that fit 168 VGPRs without spilling get 3 (hipcc -Rpass-analysis=
// kernel-resource-usage).  The runtime-level kernels keep the decomposition state live and stay at the compiler's
// choice (1 wave per SIMD).
template <int LOGN, int K, bool L1, bool PBS>
constexpr int shape_waves() {
  if (!L1) return 1;
  if (K == 1 && (PBS ? LOGN == 9 : LOGN <= 11)) return 3;
  return 2;
}

template <int LOGN, int K>
struct Shape {
  static constexpr int LOGE = loge_for<K>();
  using G = Geo<LOGN, LOGE>;
  static constexpr int N = G::N;
  static constexpr int T = G::T;  // lanes per polynomial = workgroup size
  static constexpr int E = G::E;
  static constexpr int LO_COL = G::LOGN - G::LOGE;                  // column layout e = r * T + t
  static constexpr int LO_NTT = win_lo<G, true>(G::NWIN - 1);       // forward exit / inverse entry layout
  static constexpr unsigned LOG_MOD = LOGN + 1;  // PolynomialSize::to_blind_rotation_input_modulus_log
};

// ---- one external product on registers ------------------------------------------------------
// in: ct1[K+1][E] (column layout, the GLWE to decompose); out: y[K+1][E] (column layout, the GLWE
// contribution out += GGSW (.) ct1 in the ciphertext domain).  `ggsw` = level x (K+1) x (K+1) x N (NTT
// domain, highest level first; row r = the decomposition of GLWE polynomial r); BNF keys are expected
// pre-normalised unless `normalize`.  L1: the level count is 1 at compile time (the shortint shapes' 1_1 / 2_2),
// so no decomposition state stays live beside the digits (the register budget of 2 waves per SIMD); else the levels
// are a runtime loop.
template <int LOGN, int K, bool BNF, bool L1, bool SB = false>
__device__ __forceinline__ void ext_product_regs(const u64 (&ct1)[K + 1][Shape<LOGN, K>::E],
                                                 u64 (&y)[K + 1][Shape<LOGN, K>::E], const u64* __restrict__ ggsw,
                                                 int base_log, int level, int t, u64* sh,
                                                 const u64* __restrict__ tw, const u64* __restrict__ itw,
                                                 bool normalize, u64 n_inv) {
  using S = Shape<LOGN, K>;
  using G = typename S::G;
  constexpr int E = S::E, N = S::N;
  const Goldilocks gl;
  if constexpr (L1) level = 1;
  // digit li of every coefficient: decomposer.rs:156-185 + iter.rs:131-151 (BNF) / iter.rs:623-745 (Solinas), mapped
  // into [0, p) as ntt64.rs:231-238; the state arrays exist only for the runtime-level form
  u64 state[L1 ? 1 : K + 1][L1 ? 1 : E];
  bool sign[L1 ? 1 : K + 1][L1 ? 1 : E];
  auto init = [&](u64 v, u64& st, bool& sg) {
    if (BNF) {
      st = decomp_init_native(v, base_log, level);
      sg = false;
    } else {
      const unsigned shift = 64u - (unsigned)(base_log * level);
      sg = v >= P / 2 + 1;  // div_ceil(2)
      st = closest_abs_nonnative(sg ? P - v : v, base_log, level) >> shift;
    }
  };
  auto digit = [&](u64& st, bool sg) -> u64 {
    u64 term = decompose_one_level(base_log, st);
    if (!BNF && sg) term = (u64)0 - term;  // iter.rs:722-731
    return ((int64_t)term < 0) ? term + P : term;  // ntt64.rs:231-238 / iter.rs:724-730
  };
  if constexpr (!L1) {
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) init(ct1[c][r], state[c][r], sign[c][r]);
  }
#pragma unroll
  for (int c = 0; c <= K; ++c)
#pragma unroll
    for (int r = 0; r < E; ++r) y[c][r] = 0;

#pragma unroll 1
  for (int li = 0; li < level; ++li) {
    u64 x[K + 1][E];
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) {
        if constexpr (L1) {
          u64 st;
          bool sg;
          init(ct1[c][r], st, sg);
          x[c][r] = digit(st, sg);
        } else {
          x[c][r] = digit(state[c][r], sign[c][r]);
        }
      }
    ntt_regs<G, true, K + 1, Goldilocks, true>(x, t, sh, tw, gl);  // lazy: the MAC below reduces its sums anyway
    // the iterator yields DecompositionLevel(level_count) first (the least significant digit), the
    // GGSW stores that level first too (ggsw_encryption.rs:318-375): GGSW block li pairs with term li
    const u64* mat = ggsw + (size_t)li * (K + 1) * (K + 1) * N;
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int pos = elem<G>(t, r, S::LO_NTT);
      // update_with_fmadd (ntt64_pbs.rs:683-702 / ntt64_bnf_pbs.rs:707-726): row rr times column c
#pragma unroll
      for (int c = 0; c <= K; ++c) {
        // r5: the K + 1 products summed as 128-bit values with one reduction (pbs::Acc128, 8 VALU per term) instead
        // of a canonical multiply and add per term (~33 VALU as compiled)
        pbs::Acc128 acc;
#pragma unroll
        for (int rr = 0; rr <= K; ++rr) acc.mac(x[rr][r], mat[(rr * (K + 1) + c) * N + pos]);
        y[c][r] = L1 ? acc.value(0) : gl.add(y[c][r], acc.value(0));
        // SB (r5, the N = 512, k = 4 level-1 PBS): one column's key loads at a time, so fewer loaded values are live
        // at once — 248 VGPRs and no spill instead of 256 + 18 spilled inside the step loop, +4 % PBS/s (session 41)
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if (BNF && normalize) {
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) y[c][r] = gl.mul(y[c][r], n_inv);
  }
  ntt_regs<G, false, K + 1>(y, t, sh, itw, gl);
  if (BNF) {
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) y[c][r] = modswitch_prime_to_native(y[c][r]);
  }
}

// ---- external product / CMUX batch (config 3) ----------------------------------------------------
// EXT : out[b] += GGSW (.) glwe[b]                          (add_external_product_ntt64[_bnf]_assign)
// CMUX: glwe[b] -= out[b]; out[b] += GGSW (.) glwe[b]       (cmux_ntt64[_bnf]_assign, ct0 = out, ct1 = glwe)
template <int LOGN, int K, bool BNF, bool CMUX, bool L1>
__global__ __launch_bounds__((Shape<LOGN, K>::T)) __attribute__((amdgpu_waves_per_eu(shape_waves<LOGN, K, L1, false>())))
void ext_product_kernel(u64* __restrict__ out, u64* __restrict__ glwe,
                                                                     const u64* __restrict__ ggsw_list, uint32_t batch,
                                                                     int base_log, int level,
                                                                     const u64* __restrict__ tw,
                                                                     const u64* __restrict__ itw, u64 n_inv,
                                                                     const uint32_t* __restrict__ gidx,
                                                                     uint32_t n_ggsw) {
  using S = Shape<LOGN, K>;
  using G = typename S::G;
  constexpr int E = S::E, N = S::N;
  __shared__ u64 sh[(K + 1) * G::PADDED];
  const int t = threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;  // uniform per workgroup
  // per-item GGSW (gidx[b] < n_ggsw; an out-of-range index leaves the item untouched) or one shared GGSW
  const uint32_t gi = gidx ? __builtin_amdgcn_readfirstlane(gidx[b]) : 0u;
  if (gi >= n_ggsw) return;
  const u64* ggsw = ggsw_list + (size_t)gi * level * (K + 1) * (K + 1) * N;
  u64* in = glwe + (size_t)b * (K + 1) * N;
  u64* o = out + (size_t)b * (K + 1) * N;
  u64 ct[K + 1][E], y[K + 1][E], acc[K + 1][E];
#pragma unroll
  for (int c = 0; c <= K; ++c)
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int e = c * N + elem<G>(t, r, S::LO_COL);
      ct[c][r] = in[e];
      acc[c][r] = o[e];
      if (CMUX) {  // ntt64_pbs.rs:669-680 / ntt64_bnf_pbs.rs:683-705: ct1 -= ct0
        ct[c][r] = BNF ? ct[c][r] - acc[c][r] : sub_custom(ct[c][r], acc[c][r]);
        in[e] = ct[c][r];
      }
    }
  ext_product_regs<LOGN, K, BNF, L1>(ct, y, ggsw, base_log, level, t, sh, tw, itw, true, n_inv);
#pragma unroll
  for (int c = 0; c <= K; ++c)
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int e = c * N + elem<G>(t, r, S::LO_COL);
      o[e] = BNF ? acc[c][r] + y[c][r] : add_custom(acc[c][r], y[c][r]);  // ntt64.rs:110-137 / 244-266
    }
}

// ---- programmable bootstrap batch (configs 4/5) -----------------------------------------------
// lwe_in: batch x (n+1); lut: (K+1) x N shared; bsk: n x level x (K+1) x (K+1) x N (BNF: pre-normalised
// copy); lwe_out: batch x (K N + 1).  Structure = programmable_bootstrap_ntt64[_bnf]_lwe_ciphertext_mem_optimized.
template <int LOGN, int K, bool BNF, bool L1, bool SB = false>
__global__ __launch_bounds__((Shape<LOGN, K>::T)) __attribute__((amdgpu_waves_per_eu(shape_waves<LOGN, K, L1, true>())))
void pbs_kernel(u64* __restrict__ lwe_out, const u64* __restrict__ lwe_in,
                                                             PbsIo io, const u64* __restrict__ bsk,
                                                             uint32_t n_lwe, uint32_t batch, int base_log, int level,
                                                             const u64* __restrict__ tw, const u64* __restrict__ itw,
                                                             int centered) {
  using S = Shape<LOGN, K>;
  using G = typename S::G;
  constexpr int E = S::E, N = S::N, T = S::T;
  __shared__ u64 sh[(K + 1) * G::PADDED];
  const int t = threadIdx.x;
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;
  const u64* lut = io.lut_for(b, (uint64_t)(K + 1) * N);
  if (!lut) return;  // LUT index out of range: the item is left untouched
  const u64* lwe = lwe_in + (size_t)b * (n_lwe + 1);
  const size_t ggsw_len = (size_t)level * (K + 1) * (K + 1) * N;
  const unsigned log_mod = S::LOG_MOD;

  u64 body_corr = 0;
  if (BNF && centered) body_corr = centered_body_correction<T>(lwe, n_lwe, log_mod, t, sh);

  u64 acc[K + 1][E];
#pragma unroll
  for (int c = 0; c <= K; ++c)
#pragma unroll
    for (int r = 0; r < E; ++r) acc[c][r] = lut[c * N + elem<G>(t, r, S::LO_COL)];

  if (!BNF) {  // ntt64_pbs.rs:237-249: rotate the LUT by -ms(b) first (custom modulus)
    const u64 body = ms_non_native(lwe[n_lwe], log_mod);
    const int full = (int)(body / N) & 1, rem = (int)(body % N);
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) sh[c * N + elem<G>(t, r, S::LO_COL)] = acc[c][r];
    __syncthreads();
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const int m = elem<G>(t, r, S::LO_COL);  // div_assign: new[m] = old[(m + rem) % N], neg for m >= N - rem
        u64 v = sh[c * N + ((m + rem) & (N - 1))];
        if (full ^ (m >= N - rem)) v = neg_custom(v);
        acc[c][r] = v;
      }
    __syncthreads();
  }

  for (uint32_t i = 0; i < n_lwe; ++i) {
    const u64 a_raw = lwe[i];
    u64 a;
    if (BNF) {
      a = modulus_switch(a_raw, log_mod);
      if (a == 0) continue;  // ntt64_bnf_pbs.rs:241
    } else {
      if (a_raw == 0) continue;  // ntt64_pbs.rs:257
      a = ms_non_native(a_raw, log_mod);
    }
    const int full = (int)(a / N) & 1, rem = (int)(a % N);
    // ct1 = acc * X^a (polynomial_wrapping_monic_monomial_mul_assign[_custom_mod]) ; ct1 -= acc
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) sh[c * N + elem<G>(t, r, S::LO_COL)] = acc[c][r];
    __syncthreads();
    u64 ct1[K + 1][E], y[K + 1][E];
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const int e = elem<G>(t, r, S::LO_COL);  // mul_assign: new[e] = old[(e - rem) % N], neg for e < rem
        u64 v = sh[c * N + ((e - rem) & (N - 1))];
        if (full ^ (e < rem)) v = neg_q<BNF>(v);
        ct1[c][r] = BNF ? v - acc[c][r] : sub_custom(v, acc[c][r]);  // cmux: ct1 - ct0
      }
    __syncthreads();
    ext_product_regs<LOGN, K, BNF, L1, SB>(ct1, y, bsk + (size_t)i * ggsw_len, base_log, level, t, sh, tw, itw, false, 0);
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) acc[c][r] = BNF ? acc[c][r] + y[c][r] : add_custom(acc[c][r], y[c][r]);
  }

  // BNF: final rotation by -ms(b) (ntt64_bnf_pbs.rs:262-270); then sample extract (nth = 0)
#pragma unroll
  for (int c = 0; c <= K; ++c)
#pragma unroll
    for (int r = 0; r < E; ++r) sh[c * N + elem<G>(t, r, S::LO_COL)] = acc[c][r];
  __syncthreads();
  int full = 0, rem = 0;
  if (BNF) {
    const u64 body = modulus_switch(lwe[n_lwe] + body_corr, log_mod);
    full = (int)(body / N) & 1;
    rem = (int)(body % N);
  }
  if (io.glwe_out) {  // blind_rotate_ntt64[_bnf]_assign: the rotated GLWE itself
    u64* g = io.glwe_out + (size_t)b * (K + 1) * N;
#pragma unroll
    for (int c = 0; c <= K; ++c)
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const int m = elem<G>(t, r, S::LO_COL);
        u64 v = sh[c * N + ((m + rem) & (N - 1))];
        if (full ^ (m >= N - rem)) v = neg_q<BNF>(v);
        g[c * N + m] = v;
      }
    return;
  }
  // rotated[c][m] = sign * acc[c][(m + rem) % N]; glwe_sample_extraction.rs:89-160: mask polynomial c
  // gives out[c N + 0] = A_c[0], out[c N + j] = -A_c[N - j]; the body coefficient 0 gives out[K N]
  u64* out = lwe_out + (size_t)b * (K * N + 1);
#pragma unroll
  for (int c = 0; c < K; ++c)
#pragma unroll
    for (int r = 0; r < E; ++r) {
      const int j = elem<G>(t, r, S::LO_COL);
      const int m = (j == 0) ? 0 : N - j;
      u64 v = sh[c * N + ((m + rem) & (N - 1))];
      if (full ^ (m >= N - rem)) v = neg_q<BNF>(v);
      out[c * N + j] = (j == 0) ? v : neg_q<BNF>(v);
    }
  if (t == 0) {
    u64 v = sh[K * N + (rem & (N - 1))];
    if (full ^ (0 >= N - rem)) v = neg_q<BNF>(v);
    out[K * N] = v;
  }
}

// ---- key conversion (lwe_bootstrap_key_conversion.rs:294-365) + normalisation ---------------------
// bsk_ntt[pi] = fwd(modswitch_{2^w -> p}(bsk_std[pi])) [* N^-1]; also used to prepare the BNF copy.
template <int LOGN>
__global__ __launch_bounds__((Shape<LOGN, 1>::T)) void bsk_to_ntt_kernel(u64* __restrict__ dst, const u64* __restrict__ src,
                                                                    uint64_t n_polys, unsigned in_width, int normalize,
                                                                    u64 n_inv, const u64* __restrict__ tw) {
  using S = Shape<LOGN, 1>;
  using G = typename S::G;
  constexpr int E = S::E, N = S::N;
  __shared__ u64 sh[G::PADDED];
  const Goldilocks gl;
  const int t = threadIdx.x;
  const uint64_t pi = blockIdx.x;
  if (pi >= n_polys) return;
  u64 x[1][E];
#pragma unroll
  for (int r = 0; r < E; ++r) {
    u64 v = src[pi * N + elem<G>(t, r, S::LO_COL)];
    if (in_width) {  // ntt64.rs:166-178
      const unsigned __int128 w = ((unsigned __int128)(v >> (64u - in_width))) * P + ((unsigned __int128)1 << (in_width - 1));
      v = (u64)(w >> in_width);
    }
    x[0][r] = v;
  }
  ntt_regs<G, true, 1>(x, t, sh, tw, gl);
#pragma unroll
  for (int r = 0; r < E; ++r) {
    u64 v = x[0][r];
    if (normalize) v = gl.mul(v, n_inv);
    dst[pi * N + elem<G>(t, r, S::LO_NTT)] = v;
  }
}

__global__ __launch_bounds__(256) void scale_kernel(u64* __restrict__ dst, const u64* __restrict__ src, uint64_t count,
                                                    u64 c) {
  const Goldilocks gl;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = gl.mul(src[i], c);
}

// PRE_SWITCHED inputs: lift each switched value v in [0, 2N) to a representative whose standard
// switch is v again — BNF: v << (64 - log 2N) ((v 2^s + 2^(s-1)) >> s = v); Solinas: round(v p / 2N),
// whose ms_non_native is v (the rounding error is < 2N / p) and which is 0 iff v is 0 (same skip).
__global__ __launch_bounds__(256) void lift_switched_kernel(u64* __restrict__ dst, const u64* __restrict__ src,
                                                            uint64_t count, int bnf, unsigned log2n) {
  const u64 n2 = 1ull << log2n;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    const u64 v = src[i] & (n2 - 1);
    dst[i] = bnf ? v << (64 - log2n) : (u64)(((unsigned __int128)v * P + (n2 >> 1)) >> log2n);
  }
}

// extract_lwe_sample_from_glwe_ciphertext (glwe_sample_extraction.rs:89-160) at nth = nth_first + j nth_stride:
// mask polynomial c of the output is reverse(A_c), its first N - nth - 1 entries negated, rotated left by that count,
// i.e. out[c N + i] = A_c[nth - i] for i <= nth and -A_c[N + nth - i] above; the body is B[nth].  Negation is
// wrapping (native modulus, q = 0) or modulo the custom modulus q (slice_wrapping_opposite_assign_custom_mod).
__global__ __launch_bounds__(256) void sample_extract_kernel(u64* __restrict__ out, const u64* __restrict__ glwe,
                                                             uint32_t logn, uint32_t k, uint64_t batch,
                                                             uint64_t nth_first, uint64_t nth_stride,
                                                             uint64_t nth_count, u64 q) {
  const uint64_t n = 1ull << logn, per_out = (uint64_t)k * n + 1, per_in = (uint64_t)(k + 1) * n;
  const uint64_t total = batch * nth_count * per_out;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t item = i / per_out, o = i % per_out;
    const uint64_t b = item / nth_count, nth = nth_first + (item % nth_count) * nth_stride;
    const uint64_t c = o >> logn, j = o & (n - 1);  // o = k N: the body (c = k, j = 0)
    const u64* a = glwe + b * per_in + c * n;
    u64 v;
    if (c == k) v = a[nth];
    else if (j <= nth) v = a[nth - j];
    else {
      v = a[n + nth - j];
      v = q ? (v == 0 ? 0 : q - v) : (u64)0 - v;
    }
    out[i] = v;
  }
}

}  // namespace pbs

hipError_t launch_sample_extract(uint64_t* out, const uint64_t* glwe, int logn, int k, size_t batch, size_t nth_first,
                                 size_t nth_stride, size_t nth_count, uint64_t modulus, hipStream_t s) {
  const uint64_t total = (uint64_t)batch * nth_count * (((uint64_t)k << logn) + 1);
  if (total == 0) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(pbs::sample_extract_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, glwe, (uint32_t)logn,
                     (uint32_t)k, (uint64_t)batch, (uint64_t)nth_first, (uint64_t)nth_stride, (uint64_t)nth_count,
                     (u64)modulus);
  return hipGetLastError();
}

// ---- dispatch ------------------------------------------------------------------------------------
// Shapes compiled (callers validate, c_api.cpp mi::capi::check_pbs_shape): N = 1024 / 2048 / 4096 with K in {1, 2};
// N = 512 with K in {1, 4} (PARAM_MESSAGE_1_CARRY_1).  N >= 8192 (PARAM_MESSAGE_3_CARRY_3, 4_4) runs the multi-kernel
// blind rotation of pbs_large.hip (measured faster from N = 8192 on: profiles/r3/fused_vs_large_pbs.txt).

hipError_t launch_lift_switched(uint64_t* dst, const uint64_t* src, size_t count, bool bnf, int logn, hipStream_t s) {
  if (count == 0) return hipSuccess;
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pbs::lift_switched_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, (uint64_t)count,
                     bnf ? 1 : 0, (unsigned)(logn + 1));
  return hipGetLastError();
}

template <int LOGN>
static hipError_t bsk_launch(uint64_t* dst, const uint64_t* src, size_t n_polys, unsigned in_width, int normalize,
                             uint64_t n_inv, const uint64_t* tw, hipStream_t s) {
  hipLaunchKernelGGL((pbs::bsk_to_ntt_kernel<LOGN>), dim3((unsigned)n_polys), dim3(pbs::Shape<LOGN, 1>::T), 0, s, dst, src,
                     (uint64_t)n_polys, in_width, normalize, n_inv, tw);
  return hipGetLastError();
}

hipError_t launch_bsk_to_ntt(int logn, uint64_t* dst, const uint64_t* src, size_t n_polys, unsigned in_width,
                             int normalize, uint64_t n_inv, const uint64_t* tw, hipStream_t s) {
  if (n_polys == 0) return hipSuccess;
  switch (logn) {
    case 9: return bsk_launch<9>(dst, src, n_polys, in_width, normalize, n_inv, tw, s);
    case 10: return bsk_launch<10>(dst, src, n_polys, in_width, normalize, n_inv, tw, s);
    case 11: return bsk_launch<11>(dst, src, n_polys, in_width, normalize, n_inv, tw, s);
    case 12: return bsk_launch<12>(dst, src, n_polys, in_width, normalize, n_inv, tw, s);
    case 13: return bsk_launch<13>(dst, src, n_polys, in_width, normalize, n_inv, tw, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_scale(uint64_t* dst, const uint64_t* src, size_t count, uint64_t c, hipStream_t s) {
  if (count == 0) return hipSuccess;
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(pbs::scale_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, (uint64_t)count, c);
  return hipGetLastError();
}

template <int LOGN, int K, bool BNF, bool CMUX>
static hipError_t ext_launch(int level, uint64_t* out, uint64_t* glwe, const uint64_t* ggsw, size_t batch,
                             int base_log, const uint64_t* tw, const uint64_t* itw, uint64_t n_inv, hipStream_t s,
                             const uint32_t* gidx, uint32_t n_ggsw) {
  if (level == 1)
    hipLaunchKernelGGL((pbs::ext_product_kernel<LOGN, K, BNF, CMUX, true>), dim3((unsigned)batch),
                       dim3(pbs::Shape<LOGN, K>::T), 0, s, out, glwe, ggsw, (uint32_t)batch, base_log, level, tw, itw,
                       n_inv, gidx, n_ggsw);
  else
    hipLaunchKernelGGL((pbs::ext_product_kernel<LOGN, K, BNF, CMUX, false>), dim3((unsigned)batch),
                       dim3(pbs::Shape<LOGN, K>::T), 0, s, out, glwe, ggsw, (uint32_t)batch, base_log, level, tw, itw,
                       n_inv, gidx, n_ggsw);
  return hipGetLastError();
}

template <int LOGN, int K>
static hipError_t ext_shape(bool bnf, bool cmux, int level, uint64_t* out, uint64_t* glwe, const uint64_t* ggsw,
                            size_t batch, int base_log, const uint64_t* tw, const uint64_t* itw, uint64_t n_inv,
                            hipStream_t s, const uint32_t* gi, uint32_t ng) {
  if (bnf)
    return cmux ? ext_launch<LOGN, K, true, true>(level, out, glwe, ggsw, batch, base_log, tw, itw, n_inv, s, gi, ng)
                : ext_launch<LOGN, K, true, false>(level, out, glwe, ggsw, batch, base_log, tw, itw, n_inv, s, gi, ng);
  return cmux ? ext_launch<LOGN, K, false, true>(level, out, glwe, ggsw, batch, base_log, tw, itw, n_inv, s, gi, ng)
              : ext_launch<LOGN, K, false, false>(level, out, glwe, ggsw, batch, base_log, tw, itw, n_inv, s, gi, ng);
}

hipError_t launch_ext_product(int logn, int k, bool bnf, bool cmux, int level, uint64_t* out, uint64_t* glwe,
                              const uint64_t* ggsw, size_t batch, int base_log, const uint64_t* tw,
                              const uint64_t* itw, uint64_t n_inv, hipStream_t s, const uint32_t* gidx,
                              uint32_t n_ggsw) {
  if (batch == 0) return hipSuccess;
#define MI_EXT_SHAPE(L, KK)                                                                      \
  if (logn == L && k == KK)                                                                      \
    return ext_shape<L, KK>(bnf, cmux, level, out, glwe, ggsw, batch, base_log, tw, itw, n_inv, s, gidx, n_ggsw);
  MI_EXT_SHAPE(9, 1) MI_EXT_SHAPE(9, 4) MI_EXT_SHAPE(10, 1) MI_EXT_SHAPE(10, 2) MI_EXT_SHAPE(11, 1) MI_EXT_SHAPE(11, 2)
  MI_EXT_SHAPE(12, 1) MI_EXT_SHAPE(12, 2)
#undef MI_EXT_SHAPE
  return hipErrorInvalidValue;
}

template <int LOGN, int K>
static hipError_t pbs_shape(bool bnf, int level, uint64_t* out, const uint64_t* lwe_in, const PbsIo& lut,
                            const uint64_t* bsk, size_t n_lwe, size_t batch, int base_log, const uint64_t* tw,
                            const uint64_t* itw, int centered, hipStream_t s) {
  const dim3 grid((unsigned)batch), block(pbs::Shape<LOGN, K>::T);
  if constexpr (LOGN == 9 && K == 4) {  // r5, the measured shape (1_1): the MAC's key loads one column at a time
    if (level == 1) {
      if (bnf)
        hipLaunchKernelGGL((pbs::pbs_kernel<LOGN, K, true, true, true>), grid, block, 0, s, out, lwe_in, lut, bsk,
                           (uint32_t)n_lwe, (uint32_t)batch, base_log, level, tw, itw, centered);
      else
        hipLaunchKernelGGL((pbs::pbs_kernel<LOGN, K, false, true, true>), grid, block, 0, s, out, lwe_in, lut, bsk,
                           (uint32_t)n_lwe, (uint32_t)batch, base_log, level, tw, itw, centered);
      return hipGetLastError();
    }
  }
#define MI_PBS_K(B, L)                                                                                             \
  hipLaunchKernelGGL((pbs::pbs_kernel<LOGN, K, B, L>), grid, block, 0, s, out, lwe_in, lut, bsk, (uint32_t)n_lwe, \
                     (uint32_t)batch, base_log, level, tw, itw, centered)
  if (bnf) {
    if (level == 1) MI_PBS_K(true, true);
    else MI_PBS_K(true, false);
  } else {
    if (level == 1) MI_PBS_K(false, true);
    else MI_PBS_K(false, false);
  }
#undef MI_PBS_K
  return hipGetLastError();
}

hipError_t launch_pbs(int logn, int k, bool bnf, int level, uint64_t* out, const uint64_t* lwe_in, const PbsIo& lut,
                      const uint64_t* bsk, size_t n_lwe, size_t batch, int base_log, const uint64_t* tw,
                      const uint64_t* itw, int centered, hipStream_t s) {
  if (batch == 0) return hipSuccess;
#define MI_PBS_SHAPE(L, KK)                                                                                     \
  if (logn == L && k == KK)                                                                                     \
    return pbs_shape<L, KK>(bnf, level, out, lwe_in, lut, bsk, n_lwe, batch, base_log, tw, itw, centered, s);
  MI_PBS_SHAPE(9, 1) MI_PBS_SHAPE(9, 4) MI_PBS_SHAPE(10, 1) MI_PBS_SHAPE(10, 2) MI_PBS_SHAPE(11, 1) MI_PBS_SHAPE(11, 2)
  MI_PBS_SHAPE(12, 1) MI_PBS_SHAPE(12, 2)
#undef MI_PBS_SHAPE
  return hipErrorInvalidValue;
}

}  // namespace mi
