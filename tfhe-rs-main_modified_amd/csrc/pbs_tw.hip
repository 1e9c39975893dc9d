// pbs_tw.hip — programmable bootstrap, BNF and Solinas flavours, decomposition level 1, on the twisted
// N = 2048 Goldilocks transform (reference: tfhe/src/core_crypto/algorithms/lwe_programmable_bootstrapping/
// ntt64_bnf_pbs.rs:208-726, programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized; ntt64_pbs.rs:
// 213-702, programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized).
//
// MI355X design: one 128-lane workgroup (2 waves) per LWE ciphertext.  Each wave keeps one GLWE
// polynomial of the accumulator in VGPRs (v128..v191) for the whole blind rotation and runs the
// complete CMUX step — rotation, decomposition, forward transform, GGSW multiply-accumulate (the
// partner's transformed polynomial comes through LDS), inverse transform, exact prime -> 2^64
// modulus switch — as one generated asm body (tools/gen_pbs_kernel.py -> pbs_tw_body.hpp).  256
// VGPRs and 33.5 KiB of LDS per workgroup (two 16.5 KiB wave buffers + tables): 2 waves per SIMD.  This wrapper computes the centered body
// correction (if asked) before the loop and does the final rotation by -ms(b) + sample extraction.
// Bit-exactness: the same restatement as pbs_kernels.hip (N^-1 folded into the key copy).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "scratch.hpp"
#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "pbs_tw_body.hpp"

namespace mi {
namespace pbstw {

static constexpr int N = 2048;
// per-wave LDS buffer of the blind-rotation kernels (u64): N, padded to a 32 x 66 tile when the bodies run one-pass
// transposes (tools/gen_pbs_kernel.py PBS_FULL_T); 2 x 16.5 KiB + the 512 B table per workgroup keeps 4 per CU
static constexpr int NPW = MI_PBS_LDS_STRIDE;
static_assert(NPW >= N, "a wave buffer holds at least one polynomial");
static constexpr unsigned LOG_MOD = 12;  // PolynomialSize::to_blind_rotation_input_modulus_log

__device__ __forceinline__ u64 modulus_switch(u64 input, unsigned log_modulus) {  // fft_impl/common.rs:10-23
  return (input + (1ull << (64u - log_modulus - 1u))) >> (64u - log_modulus);
}

// algorithms/modulus_switch.rs:60-104 centered_binary_ms_body_correction_to_add (128-lane reduction)
__device__ u64 centered_body_correction(const u64* __restrict__ lwe, uint32_t n_lwe, int t, u64* sh) {
  u64 sum_half = 0;
  int64_t sum_hed = 0;
  for (uint32_t i = t; i < n_lwe; i += 128) {
    const u64 a = lwe[i];
    const int64_t err = (int64_t)((modulus_switch(a, LOG_MOD) << (64u - LOG_MOD)) - a);
    const int64_t half = err / 2;  // truncating, as Rust's signed division
    sum_half += (u64)half;
    sum_hed += 2 * half - err;
  }
  sh[t] = sum_half;
  sh[128 + t] = (u64)sum_hed;
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (t < s) {
      sh[t] += sh[t + s];
      sh[128 + t] = (u64)((int64_t)sh[128 + t] + (int64_t)sh[128 + t + s]);
    }
    __syncthreads();
  }
  const u64 total_half = sh[0];
  const int64_t total_hed = (int64_t)sh[128];
  __syncthreads();
  return total_half - (u64)(total_hed / 2) - (1ull << (64u - LOG_MOD - 1u));
}

// The forward's lane-pair twiddles (tab[N..N+31]) and the W1'' inverse's last-DIT-stage twiddles (tab[3 (N+32)..],
// powers of two: the same for the plain and the N^-1-folded untwist) into LDS, read by the bodies' pair stages.
__device__ __forceinline__ void load_lane_pair_tables(u64* lwtab, const u64* __restrict__ tab, int t) {
  if (t < 64) lwtab[t] = t < 32 ? tab[N + t] : tab[3 * (N + 32) + (t - 32)];
  __syncthreads();
}

// lwe_in: batch x (n+1); io: the accumulator's LUT (2 x N per GLWE) and the output form (PbsIo); bsk: n x 2 x 2 x N
// (NTT domain, N^-1 folded in); tab: [fwd twist (N) | fwd lane-pair twiddles (32) | inverse twist (N) | inverse
// lane-pair (32) | ...].
__global__ __launch_bounds__(128) void pbs_tw_kernel(u64* __restrict__ lwe_out, const u64* __restrict__ lwe_in,
                                                     PbsIo io, const u64* __restrict__ bsk,
                                                     uint32_t n_lwe, uint32_t batch, int base_log,
                                                     const u64* __restrict__ tab, int centered) {
  __shared__ u64 buf[2 * NPW];
  __shared__ u64 lwtab[64];
  const int t = threadIdx.x;
  const uint32_t lane = t & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;  // uniform per workgroup
  const u64* lut = io.lut_for(b, 2 * N);
  if (!lut) return;  // LUT index out of range: the item is left untouched
  const u64* lwe = lwe_in + (size_t)b * (n_lwe + 1);
  load_lane_pair_tables(lwtab, tab, t);  // ends with a workgroup barrier
  u64 body_corr = 0;
  if (centered) body_corr = centered_body_correction(lwe, n_lwe, t, buf);

  const uint32_t S = (uint32_t)(uintptr_t)(buf + w * NPW), SP = (uint32_t)(uintptr_t)(buf + (1 - w) * NPW);
  const u64* lutw = lut + (size_t)w * N;
  const u64* gown = bsk + (size_t)3 * w * N;
  const u64* gpar = bsk + (size_t)(2 - w) * N;
  const uint32_t lut_lo = (uint32_t)(uintptr_t)lutw, lut_hi = (uint32_t)((uintptr_t)lutw >> 32);
  const uint32_t gown_lo = (uint32_t)(uintptr_t)gown, gown_hi = (uint32_t)((uintptr_t)gown >> 32);
  const uint32_t gpar_lo = (uint32_t)(uintptr_t)gpar, gpar_hi = (uint32_t)((uintptr_t)gpar >> 32);
  const uint32_t lwe_lo = (uint32_t)(uintptr_t)lwe, lwe_hi = (uint32_t)((uintptr_t)lwe >> 32);
  const uint32_t tab_lo = (uint32_t)(uintptr_t)tab, tab_hi = (uint32_t)((uintptr_t)tab >> 32);
  MI_PBS_BODY_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [lut_lo] "s"(lut_lo), [lut_hi] "s"(lut_hi),
                     [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi), [gpar_lo] "s"(gpar_lo),
                     [gpar_hi] "s"(gpar_hi), [lwe_lo] "s"(lwe_lo), [lwe_hi] "s"(lwe_hi), [n] "s"(n_lwe),
                     [tab_lo] "s"(tab_lo), [tab_hi] "s"(tab_hi), [bl] "s"(base_log),
                     [LW] "s"((uint32_t)(uintptr_t)lwtab));
  // buf[w NPW + e] = acc_w[e].  Final rotation by -ms(b) (ntt64_bnf_pbs.rs:262-270), then sample
  // extraction at nth = 0 (glwe_sample_extraction.rs:89-160): out[0] = A'[0], out[j] = -A'[N - j].
  const u64* acc = buf + w * NPW;
  const u64 body = modulus_switch(lwe[n_lwe] + body_corr, LOG_MOD);
  const int full = (int)(body / N) & 1, rem = (int)(body % N);
  if (io.glwe_out) {  // blind_rotate_ntt64_bnf_assign: the rotated GLWE itself (new[m] = old[(m + rem) % N], signed)
    u64* g = io.glwe_out + ((size_t)b * 2 + w) * N;
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const int m = 64 * r + (int)lane;
      u64 v = acc[(m + rem) & (N - 1)];
      if (full ^ (m >= N - rem)) v = (u64)0 - v;
      g[m] = v;
    }
    return;
  }
  u64* out = lwe_out + (size_t)b * (N + 1);
  if (w == 0) {
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const int j = 64 * r + (int)lane;
      const int m = (j == 0) ? 0 : N - j;
      u64 v = acc[(m + rem) & (N - 1)];
      if (full ^ (m >= N - rem)) v = (u64)0 - v;
      out[j] = (j == 0) ? v : (u64)0 - v;
    }
  } else if (lane == 0) {
    u64 v = acc[rem & (N - 1)];
    if (full) v = (u64)0 - v;
    out[N] = v;
  }
}

// ---- Solinas-modulus PBS (ntt64_pbs.rs:213-286, 482-538) on the same engine ---------------------------
static constexpr u64 P = GL_P;
__device__ __forceinline__ u64 neg_custom(u64 a) { return a == 0 ? 0 : P - a; }

// ntt64_pbs.rs:540-549 pbs_modulus_switch_non_native (divide_round(a 2N, p), misc.rs:6-18), reduced mod
// 2N: X^(2N) = 1, so a value that rounds to 2N rotates like 0 (and 0 skips the step, whose CMUX
// difference would be 0 anyway)
__device__ __forceinline__ u64 ms_non_native(u64 input) {
  const unsigned __int128 num = ((unsigned __int128)input) << (LOG_MOD);
  const u64 nh = (u64)(num >> 64), nl = (u64)num;
  unsigned __int128 r = (unsigned __int128)nh * GL_EPS + nl;  // num = nh p + r
  u64 q = nh;
  while (r >= P) { r -= P; ++q; }
  return (q + (r >= (P >> 1) ? 1 : 0)) & (2 * N - 1);
}

__global__ __launch_bounds__(256) void ms_non_native_kernel(u64* __restrict__ dst, const u64* __restrict__ src,
                                                            uint64_t count) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += (uint64_t)gridDim.x * 256)
    dst[i] = ms_non_native(src[i]);
}

// switched: batch x (n+1) switched values in [0, 2N) (mask, then body); lut: 2 x N mod p;
// bsk: n x 2 x 2 x N Normalize NTT key.  The LUT is rotated by -ms(b) into LDS first
// (polynomial_wrapping_monic_monomial_div_assign_custom_mod, ntt64_pbs.rs:237-249); the body runs the
// loop; sample extraction at nth = 0 negates modulo p (glwe_sample_extraction.rs:89-160).
__global__ __launch_bounds__(128) void pbs_tw_sol_kernel(u64* __restrict__ lwe_out, const u64* __restrict__ switched,
                                                         PbsIo io, const u64* __restrict__ bsk,
                                                         uint32_t n_lwe, uint32_t batch, int base_log,
                                                         const u64* __restrict__ tab) {
  __shared__ u64 buf[2 * NPW];
  __shared__ u64 lwtab[64];
  const int t = threadIdx.x;
  const uint32_t lane = t & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;
  const u64* lut = io.lut_for(b, 2 * N);
  if (!lut) return;  // LUT index out of range: the item is left untouched
  const u64* msw = switched + (size_t)b * (n_lwe + 1);
  load_lane_pair_tables(lwtab, tab, t);
  {
    const u64 body = msw[n_lwe] & (2 * N - 1);
    const int full = (int)(body / N) & 1, rem = (int)(body % N);
    const u64* l = lut + (size_t)w * N;
    for (int r = 0; r < 32; ++r) {
      const int m = 64 * r + (int)lane;  // new[m] = old[(m + rem) % N], negated for m >= N - rem
      u64 v = l[(m + rem) & (N - 1)];
      if (full ^ (m >= N - rem)) v = neg_custom(v);
      buf[w * NPW + m] = v;
    }
  }
  __syncthreads();
  const uint32_t S = (uint32_t)(uintptr_t)(buf + w * NPW), SP = (uint32_t)(uintptr_t)(buf + (1 - w) * NPW);
  const u64* gown = bsk + (size_t)3 * w * N;
  const u64* gpar = bsk + (size_t)(2 - w) * N;
  const uint32_t gown_lo = (uint32_t)(uintptr_t)gown, gown_hi = (uint32_t)((uintptr_t)gown >> 32);
  const uint32_t gpar_lo = (uint32_t)(uintptr_t)gpar, gpar_hi = (uint32_t)((uintptr_t)gpar >> 32);
  const uint32_t lwe_lo = (uint32_t)(uintptr_t)msw, lwe_hi = (uint32_t)((uintptr_t)msw >> 32);
  const uint32_t tab_lo = (uint32_t)(uintptr_t)tab, tab_hi = (uint32_t)((uintptr_t)tab >> 32);
  MI_PBS_BODY_SOL_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                     [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [lwe_lo] "s"(lwe_lo), [lwe_hi] "s"(lwe_hi),
                     [n] "s"(n_lwe), [tab_lo] "s"(tab_lo), [tab_hi] "s"(tab_hi), [bl] "s"(base_log),
                     [LW] "s"((uint32_t)(uintptr_t)lwtab));
  const u64* acc = buf + w * NPW;
  if (io.glwe_out) {  // blind_rotate_ntt64_assign: the accumulator (rotated by -ms(b) before the loop)
    u64* g = io.glwe_out + ((size_t)b * 2 + w) * N;
#pragma unroll 4
    for (int r = 0; r < 32; ++r) g[64 * r + lane] = acc[64 * r + lane];
    return;
  }
  u64* out = lwe_out + (size_t)b * (N + 1);
  if (w == 0) {
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const int j = 64 * r + (int)lane;
      out[j] = (j == 0) ? acc[0] : neg_custom(acc[N - j]);
    }
  } else if (lane == 0) {
    out[N] = acc[0];
  }
}

// external product / CMUX batch (config 3): one workgroup per GLWE pair, wave w on polynomial w;
// SOL: GLWEs modulo p with a Normalize GGSW (ntt64_pbs.rs:553-702), else BNF (native GLWEs, Raw GGSW).
// r6: the bodies use v0..v167 (MI_EXT_VGPRS) and 8.5 KiB of LDS per wave (the half-wave transposes, the partner
// exchange in two 16-row halves), so three waves fit per SIMD instead of the blind-rotation bodies' two
// (tools/gen_pbs_kernel.py set_regmap / mac_ext).
template <bool CMUX, bool SOL>
__device__ __forceinline__ void ext_tw_item(u64* __restrict__ out, u64* __restrict__ glwe, const u64* __restrict__ ggsw,
                                            uint32_t b, int base_log, const u64* __restrict__ tab, u64* buf,
                                            u64* lwtab, uint32_t lane, uint32_t w) {
  const uint32_t S = (uint32_t)(uintptr_t)(buf + w * MI_EXT_LDS_STRIDE),
                 SP = (uint32_t)(uintptr_t)(buf + (1 - w) * MI_EXT_LDS_STRIDE);
  u64* o = out + ((size_t)b * 2 + w) * N;
  u64* g = glwe + ((size_t)b * 2 + w) * N;
  const u64* gown = ggsw + (size_t)3 * w * N;
  const u64* gpar = ggsw + (size_t)(2 - w) * N;
  const uint32_t o_lo = (uint32_t)(uintptr_t)o, o_hi = (uint32_t)((uintptr_t)o >> 32);
  const uint32_t g_lo = (uint32_t)(uintptr_t)g, g_hi = (uint32_t)((uintptr_t)g >> 32);
  const uint32_t gown_lo = (uint32_t)(uintptr_t)gown, gown_hi = (uint32_t)((uintptr_t)gown >> 32);
  const uint32_t gpar_lo = (uint32_t)(uintptr_t)gpar, gpar_hi = (uint32_t)((uintptr_t)gpar >> 32);
  const uint32_t tab_lo = (uint32_t)(uintptr_t)tab, tab_hi = (uint32_t)((uintptr_t)tab >> 32);
  if constexpr (SOL && CMUX)
    MI_PBS_BODY_CMUX_SOL_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [glwe_lo] "s"(g_lo), [glwe_hi] "s"(g_hi),
                            [out_lo] "s"(o_lo), [out_hi] "s"(o_hi), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                            [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [tab_lo] "s"(tab_lo),
                            [tab_hi] "s"(tab_hi), [bl] "s"(base_log), [LW] "s"((uint32_t)(uintptr_t)lwtab));
  else if constexpr (SOL)
    MI_PBS_BODY_EXT_SOL_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [glwe_lo] "s"(g_lo), [glwe_hi] "s"(g_hi),
                           [out_lo] "s"(o_lo), [out_hi] "s"(o_hi), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                           [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [tab_lo] "s"(tab_lo),
                           [tab_hi] "s"(tab_hi), [bl] "s"(base_log), [LW] "s"((uint32_t)(uintptr_t)lwtab));
  else if constexpr (CMUX)
    MI_PBS_BODY_CMUX_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [glwe_lo] "s"(g_lo), [glwe_hi] "s"(g_hi),
                            [out_lo] "s"(o_lo), [out_hi] "s"(o_hi), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                            [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [tab_lo] "s"(tab_lo),
                            [tab_hi] "s"(tab_hi), [bl] "s"(base_log), [LW] "s"((uint32_t)(uintptr_t)lwtab));
  else
    MI_PBS_BODY_EXT_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [glwe_lo] "s"(g_lo), [glwe_hi] "s"(g_hi),
                           [out_lo] "s"(o_lo), [out_hi] "s"(o_hi), [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi),
                           [gpar_lo] "s"(gpar_lo), [gpar_hi] "s"(gpar_hi), [tab_lo] "s"(tab_lo),
                           [tab_hi] "s"(tab_hi), [bl] "s"(base_log), [LW] "s"((uint32_t)(uintptr_t)lwtab));
}

template <bool CMUX, bool SOL = false>
__global__ __launch_bounds__(128) void ext_tw_kernel(u64* __restrict__ out, u64* __restrict__ glwe,
                                                     const u64* __restrict__ ggsw_list, uint32_t batch, int base_log,
                                                     const u64* __restrict__ tab, const uint32_t* __restrict__ gidx,
                                                     uint32_t n_ggsw) {
  __shared__ u64 buf[2 * MI_EXT_LDS_STRIDE];
  __shared__ u64 lwtab[64];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (blockIdx.x >= batch) return;
  load_lane_pair_tables(lwtab, tab, threadIdx.x);
  // one item per workgroup; per-item GGSW (gidx[b] < n_ggsw; an out-of-range index leaves the item untouched) or one
  // shared GGSW
  const uint32_t b = blockIdx.x;
  const uint32_t gi = gidx ? __builtin_amdgcn_readfirstlane(gidx[b]) : 0u;
  if (gi >= n_ggsw) return;  // uniform per workgroup
  ext_tw_item<CMUX, SOL>(out, glwe, ggsw_list + (size_t)gi * 4 * N, b, base_log, tab, buf, lwtab, lane, w);
}

// The blind-rotation body keeps the NTT-domain data in the forward's W1' register layout through the MAC
// (tools/gen_pbs_kernel.py PBS_W1P / tw_key_index), so it reads its key in that order: position 64 R + L of each
// polynomial holds NTT-domain coefficient 64 (L >> 1) + 32 (L & 1) + 2 (R & 15) + (R >> 4).  One workgroup per
// polynomial stages it in LDS (so dst may equal src) and optionally multiplies by c (BNF: N^-1 folded in, exact).
__global__ __launch_bounds__(256) void prepare_tw_key_kernel(u64* dst, const u64* src, size_t n_polys, u64 c, int scale,
                                                             int permute) {
  __shared__ u64 poly[N];
  for (size_t q = blockIdx.x; q < n_polys; q += gridDim.x) {
    const u64* in = src + q * N;
    for (int e = threadIdx.x; e < N; e += 256) poly[e] = in[e];
    __syncthreads();
    u64* out = dst + q * N;
    for (int pos = threadIdx.x; pos < N; pos += 256) {
      const int R = pos >> 6, L = pos & 63;
      const u64 v = poly[permute ? 64 * (L >> 1) + 32 * (L & 1) + 2 * (R & 15) + (R >> 4) : pos];
      out[pos] = scale ? Goldilocks().mul(v, c) : v;
    }
    __syncthreads();
  }
}

}  // namespace pbstw

hipError_t launch_prepare_tw_key(uint64_t* dst, const uint64_t* src, size_t n_polys, uint64_t c, int scale,
                                 hipStream_t s, bool ext) {
  if (n_polys == 0) return hipSuccess;
  const unsigned blocks = (unsigned)(n_polys < 65535 ? n_polys : 65535);
  hipLaunchKernelGGL(pbstw::prepare_tw_key_kernel, dim3(blocks), dim3(256), 0, s, dst, src, n_polys, c, scale,
                     ext ? MI_EXT_W1P : MI_PBS_W1P);
  return hipGetLastError();
}

bool ext_tw_reads_w1p() { return MI_EXT_W1P != 0; }

hipError_t launch_ext_tw(bool cmux, bool sol, uint64_t* out, uint64_t* glwe, const uint64_t* ggsw, size_t batch,
                         int base_log, const uint64_t* tab, hipStream_t s, const uint32_t* gidx, uint32_t n_ggsw,
                         bool prepared) {
  if (batch == 0) return hipSuccess;
  if (base_log < 1 || base_log > 31) return hipErrorInvalidValue;
  u64* perm = nullptr;  // MI_EXT_W1P on a raw list: the caller's GGSWs in the body's W1' order, in pooled scratch
  if (MI_EXT_W1P && !prepared) {
    hipError_t e = mi::scratch_alloc((void**)&perm, (size_t)n_ggsw * 4 * pbstw::N * sizeof(u64), s);
    if (e != hipSuccess) return e;
    e = launch_prepare_tw_key(perm, ggsw, (size_t)n_ggsw * 4, 0, 0, s, true);
    if (e != hipSuccess) {
      (void)mi::scratch_free(perm, s);
      return e;
    }
    ggsw = perm;
  }
  const dim3 g((unsigned)batch), blk(128);  // one workgroup per item (a looping persistent grid measured slower, r5)
  if (sol && cmux)
    hipLaunchKernelGGL((pbstw::ext_tw_kernel<true, true>), g, blk, 0, s, out, glwe, ggsw, (uint32_t)batch, base_log, tab, gidx, n_ggsw);
  else if (sol)
    hipLaunchKernelGGL((pbstw::ext_tw_kernel<false, true>), g, blk, 0, s, out, glwe, ggsw, (uint32_t)batch, base_log, tab, gidx, n_ggsw);
  else if (cmux)
    hipLaunchKernelGGL((pbstw::ext_tw_kernel<true>), g, blk, 0, s, out, glwe, ggsw, (uint32_t)batch, base_log, tab, gidx, n_ggsw);
  else
    hipLaunchKernelGGL((pbstw::ext_tw_kernel<false>), g, blk, 0, s, out, glwe, ggsw, (uint32_t)batch, base_log, tab, gidx, n_ggsw);
  const hipError_t e = hipGetLastError();
  if (perm) (void)mi::scratch_free(perm, s);
  return e;
}

hipError_t launch_ms_non_native(uint64_t* dst, const uint64_t* src, size_t count, hipStream_t s) {
  if (count == 0) return hipSuccess;
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 65535) blocks = 65535;
  hipLaunchKernelGGL(pbstw::ms_non_native_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, (uint64_t)count);
  return hipGetLastError();
}

hipError_t launch_pbs_tw_sol(uint64_t* out, const uint64_t* switched, const PbsIo& io, const uint64_t* bsk,
                             size_t n_lwe, size_t batch, int base_log, const uint64_t* tab, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (base_log < 1 || base_log > 31) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pbstw::pbs_tw_sol_kernel, dim3((unsigned)batch), dim3(128), 0, s, out, switched, io, bsk,
                     (uint32_t)n_lwe, (uint32_t)batch, base_log, tab);
  return hipGetLastError();
}

hipError_t launch_pbs_tw(uint64_t* out, const uint64_t* lwe_in, const PbsIo& io, const uint64_t* bsk, size_t n_lwe,
                         size_t batch, int base_log, const uint64_t* tab, int centered, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (base_log < 1 || base_log > 31) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pbstw::pbs_tw_kernel, dim3((unsigned)batch), dim3(128), 0, s, out, lwe_in, io, bsk,
                     (uint32_t)n_lwe, (uint32_t)batch, base_log, tab, centered);
  return hipGetLastError();
}

}  // namespace mi
