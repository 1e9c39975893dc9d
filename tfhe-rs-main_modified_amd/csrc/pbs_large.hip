// pbs_large.hip — blind rotation, PBS, external product and CMUX for polynomial sizes beyond one workgroup
// (N = 2^14 ... 2^17; the shortint PARAM_MESSAGE_4_CARRY_4 shape is N = 65536, k = 1, n = 1117, B = 2^11, l = 3,
// shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/ks_pbs.rs:71-90), both NTT variants (reference paths
// relative to /root/reference/tfhe/src/core_crypto):
//   BNF     : algorithms/lwe_programmable_bootstrapping/ntt64_bnf_pbs.rs:208-726
//   SOLINAS : algorithms/lwe_programmable_bootstrapping/ntt64_pbs.rs:213-702
//
// MI355X design.  An N = 65536 GLWE accumulator (k + 1 polynomials, 1 MiB at k = 1) cannot live in one workgroup, so
// the accumulators of a chunk of ciphertexts live in HBM and every CMUX step is a short sequence of device-wide
// kernels over the whole chunk, each one a streaming pass:
//   decompose : ct1 = X^a acc - acc (the monomial rotation read straight from acc), signed decomposition into `level`
//               digit polynomials per GLWE polynomial (mod p)           -> digits [b][level][k+1][N]
//   forward   : the plan's large-N transform over all chunk x level x (k+1) digit polynomials (ntt64_kernels.hip:
//               top stages on strided columns + 2^14 register-window blocks, the reference's depth-first split)
//   mac       : y[b][c] = sum_{li, r} digits[b][li][r] . GGSW_i[li][r][c]   (the step's GGSW is shared by the whole
//               chunk: read once per chunk, L2/MALL-resident across the ciphertexts)
//   inverse   : large-N inverse transform of the chunk x (k+1) products
//   accumulate: acc += modswitch_{p -> 2^64}(y) (BNF) / acc += y mod p (Solinas)
// Masks that switch to 0 give ct1 = 0 and an exactly-zero contribution (decomposition of 0 is 0 at every level), so
// every ciphertext runs every step and no per-ciphertext control flow reaches the kernels; the reference's skip
// (ntt64_bnf_pbs.rs:241, ntt64_pbs.rs:257) changes no value.  The elementwise kernels are HBM-bound (coalesced,
// grid-stride); the transforms are the engine's large-N kernels.  Bit-exact: every pass restates the reference
// arithmetic exactly (canonical residues), as the fused kernels of pbs_kernels.hip do.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "scratch.hpp"
#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_tile.hpp"
#include "ntt64_tile_asm.hpp"
#include "pbs_device.hpp"

namespace mi {
namespace pbs {

struct LargeShape {
  uint32_t logn, n, k, level;
  int base_log;
};

__device__ __forceinline__ uint64_t grid_stride_start() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t grid_stride() { return (uint64_t)gridDim.x * blockDim.x; }

// signed decomposition of one GLWE coefficient into `level` digits mod p, least significant level first (the
// order the reference's iterator yields them and the GGSW stores its blocks): BNF = decomposer.rs:156-185 +
// iter.rs:131-151 (digits mapped into [0, p) as ntt64.rs:231-238); Solinas = iter.rs:623-745 (sign-magnitude)
template <bool BNF>
__device__ __forceinline__ void decompose_store(u64 x, u64* __restrict__ dst, uint64_t level_stride, int base_log,
                                                int level) {
  u64 state;
  bool sign = false;
  if (BNF) {
    state = decomp_init_native(x, base_log, level);
  } else {
    const unsigned shift = 64u - (unsigned)(base_log * level);
    sign = x >= P / 2 + 1;
    state = closest_abs_nonnative(sign ? P - x : x, base_log, level) >> shift;
  }
  for (int li = 0; li < level; ++li) {
    u64 term = decompose_one_level(base_log, state);
    if (!BNF && sign) term = (u64)0 - term;
    dst[(uint64_t)li * level_stride] = ((int64_t)term < 0) ? term + P : term;
  }
}

// acc[b] = the item's LUT (BNF), or the LUT rotated by -ms(body) (Solinas, ntt64_pbs.rs:237-249); item b of the chunk
// is item b0 + b of the caller's batch (PbsIo); a skipped item (LUT index out of range) gets a zero accumulator
template <bool BNF>
__global__ __launch_bounds__(256) void large_init_acc(u64* __restrict__ acc, PbsIo io, uint64_t b0,
                                                      const u64* __restrict__ lwe_in, uint32_t n_lwe, uint32_t batch,
                                                      LargeShape sh) {
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n, total = per * batch;
  for (uint64_t i = grid_stride_start(); i < total; i += grid_stride()) {
    const uint64_t b = i / per, ce = i % per;
    const uint32_t c = (uint32_t)(ce >> sh.logn), m = (uint32_t)(ce & (sh.n - 1));
    const u64* lut = io.lut_for(b0 + b, per);
    if (!lut) {
      acc[i] = 0;
    } else if (BNF) {
      acc[i] = lut[ce];
    } else {
      const u64 body = ms_non_native(lwe_in[b * (n_lwe + 1) + n_lwe], sh.logn + 1);
      const uint32_t full = (uint32_t)(body >> sh.logn) & 1u, rem = (uint32_t)(body & (sh.n - 1));
      u64 v = lut[(uint64_t)c * sh.n + ((m + rem) & (sh.n - 1))];  // div_assign by X^body
      if (full ^ (m >= sh.n - rem)) v = neg_custom(v);
      acc[i] = v;
    }
  }
}

// step i of the blind rotation: ct1 = X^a acc - acc (polynomial_wrapping_monic_monomial_mul_assign[_custom_mod],
// then the CMUX difference), decomposed into digits[b][li][c][N]
template <bool BNF>
__global__ __launch_bounds__(256) void large_rotate_decompose(u64* __restrict__ digits, const u64* __restrict__ acc,
                                                              const u64* __restrict__ lwe_in, uint32_t n_lwe,
                                                              uint32_t step, uint32_t batch, LargeShape sh) {
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n, total = per * batch;
  const unsigned log_mod = sh.logn + 1;
  for (uint64_t i = grid_stride_start(); i < total; i += grid_stride()) {
    const uint64_t b = i / per, ce = i % per;
    const uint32_t c = (uint32_t)(ce >> sh.logn), e = (uint32_t)(ce & (sh.n - 1));
    const u64 a_raw = lwe_in[b * (n_lwe + 1) + step];
    u64 a = 0;
    if (BNF) a = modulus_switch(a_raw, log_mod);
    else if (a_raw != 0) a = ms_non_native(a_raw, log_mod);
    const uint32_t full = (uint32_t)(a >> sh.logn) & 1u, rem = (uint32_t)(a & (sh.n - 1));
    const u64* ap = acc + b * per + (uint64_t)c * sh.n;
    u64 v = ap[(e - rem) & (sh.n - 1)];  // mul_assign by X^a: new[e] = old[(e - rem) % N], negated for e < rem
    if (full ^ (e < rem)) v = neg_q<BNF>(v);
    const u64 ct1 = BNF ? v - ap[e] : sub_custom(v, ap[e]);
    decompose_store<BNF>(ct1, digits + b * sh.level * per + (uint64_t)c * sh.n + e, per, sh.base_log, (int)sh.level);
  }
}

// Step i of the blind rotation fused with the forward's first pass of the split transform (launch_ntt_split): thread j
// of GLWE polynomial (b, c) forms ct1 = X^a acc - acc at the 2^K coefficients e = j + r cols (cols = N / 2^K), decomposes
// them, and for each level li runs the first K top CT stages of the transform (s0 = 0: twiddle tw[m + g]) on the
// digits in registers (ONLY: the pass is the last one, so the block twist follows), storing digit polynomial (b, li, c)
// (stage 0's twiddles are the tower's powers of two, Goldilocks::mul_pow2; the split tables exist only when they are)
// in the layout of large_rotate_decompose.  Replaces that pass plus the transform's first pass: acc is read once and
// the digits written once (not written, read and written again).
template <int K, bool BNF, bool ONLY>
__global__ __launch_bounds__(256) void large_rotdec_top(u64* __restrict__ digits, const u64* __restrict__ acc,
                                                        const u64* __restrict__ lwe_in, uint32_t n_lwe, uint32_t step,
                                                        LargeShape sh, const u64* __restrict__ tw,
                                                        const u64* __restrict__ twist) {
  constexpr int R = 1 << K;
  const Goldilocks gl;
  const uint64_t cols = (uint64_t)sh.n >> K;
  const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= cols) return;
  const uint32_t bc = blockIdx.y, b = bc / (sh.k + 1), c = bc % (sh.k + 1);
  const unsigned log_mod = sh.logn + 1;
  const u64 a_raw = lwe_in[(uint64_t)b * (n_lwe + 1) + step];
  u64 a = 0;
  if (BNF) a = modulus_switch(a_raw, log_mod);
  else if (a_raw != 0) a = ms_non_native(a_raw, log_mod);
  const uint32_t full = (uint32_t)(a >> sh.logn) & 1u, rem = (uint32_t)(a & (sh.n - 1));
  const u64* ap = acc + (uint64_t)bc * sh.n;
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n;
  u64* dp = digits + (uint64_t)b * sh.level * per + (uint64_t)c * sh.n + j;
  u64 st[R];
  bool sg[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t e = (uint32_t)(j + r * cols);
    u64 v = ap[(e - rem) & (sh.n - 1)];  // X^a acc: new[e] = old[(e - rem) % N], negated for e < rem
    if (full ^ (e < rem)) v = neg_q<BNF>(v);
    const u64 x = BNF ? v - ap[e] : sub_custom(v, ap[e]);
    if (BNF) {
      st[r] = decomp_init_native(x, sh.base_log, (int)sh.level);
      sg[r] = false;
    } else {  // iter.rs:623-745, as decompose_store
      const unsigned shift = 64u - (unsigned)(sh.base_log * (int)sh.level);
      sg[r] = x >= P / 2 + 1;
      st[r] = closest_abs_nonnative(sg[r] ? P - x : x, sh.base_log, (int)sh.level) >> shift;
    }
  }
  for (uint32_t li = 0; li < sh.level; ++li) {
    u64 x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      u64 term = decompose_one_level(sh.base_log, st[r]);
      if (!BNF && sg[r]) term = (u64)0 - term;
      x[r] = ((int64_t)term < 0) ? term + P : term;
    }
#pragma unroll
    for (int s = 0; s < K; ++s) {  // stage s: m = 2^s groups, pair distance 2^(K-1-s) in r; twiddle tw[m + g] = 2^e
      const int d = 1 << (K - 1 - s);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r & d) continue;
        bool ng;
        const u64 z = Goldilocks::mul_pow2(x[r + d], tower_exp(true, s, r >> (K - s)), ng);  // canonical, any input
        const u64 u = x[r];
        if (ONLY) {  // r5: any 64-bit representatives until the block twist's multiply (as the K = 5 tile)
          x[r] = ng ? Goldilocks::sub_lazy(u, z) : Goldilocks::add_lazy(u, z);
          x[r + d] = ng ? Goldilocks::add_lazy(u, z) : Goldilocks::sub_lazy(u, z);
        } else {
          x[r] = ng ? gl.sub(u, z) : gl.add(u, z);
          x[r + d] = ng ? gl.add(u, z) : gl.sub(u, z);
        }
      }
    }
    u64* o = dp + (uint64_t)li * per;
    // the block twist per level: an opaque base keeps its loads inside the level loop (hoisted, the 2^K values would
    // stay live across the loop beside the digits and the decomposition state)
    const u64* tws = twist;
    if (ONLY) asm volatile("" : "+s"(tws));
#pragma unroll
    for (int r = 0; r < R; ++r) {
      u64 v = x[r];
      if (ONLY) v = gl.mul(v, tws[j + r * cols]);
      __builtin_nontemporal_store(v, o + r * cols);  // the digits are read once, by the next pass
    }
  }
}

// the generated K = 5 blocks by wave index (tools/gen_tile_asm.py -> ntt64_tile_asm.hpp)
template <int W>
__device__ __forceinline__ void tile5_fwd_a(u64 (&x)[8]) {
  if constexpr (W == 0) tile_asm::k5_fwd_a_w0(x);
  else if constexpr (W == 1) tile_asm::k5_fwd_a_w1(x);
  else if constexpr (W == 2) tile_asm::k5_fwd_a_w2(x);
  else tile_asm::k5_fwd_a_w3(x);
}
template <int W>
__device__ __forceinline__ void tile5_fwd_b_tw(u64 (&x)[8], const u64 (&tw)[8]) {
  if constexpr (W == 0) tile_asm::k5_fwd_b_tw_w0(x, tw);
  else if constexpr (W == 1) tile_asm::k5_fwd_b_tw_w1(x, tw);
  else if constexpr (W == 2) tile_asm::k5_fwd_b_tw_w2(x, tw);
  else tile_asm::k5_fwd_b_tw_w3(x, tw);
}

// The same step at K = 4 / 5 as a cooperative tile (ntt64_tile.hpp): lane (wave W, column c) forms ct1 and the
// decomposition state of its phase-A rows, then per level runs the phase-A stages, the LDS exchange and the phase-B
// stages and stores the digit polynomial from its phase-B rows.  Grid: x = column tiles of 64, y = GLWE polynomials.
template <int K, bool BNF, bool ONLY, int W>
__device__ __forceinline__ void rotdec_tile_body(u64* __restrict__ dp, const u64* __restrict__ ap, uint32_t full,
                                                 uint32_t rem, uint64_t cols, uint64_t col, uint32_t c, uint64_t per,
                                                 const LargeShape& sh, const u64* __restrict__ twist, u64* lds) {
  using Rw = tile::Rows<K>;
  constexpr int RPT = Rw::RPT;
  u64 st[RPT];
  bool sg[RPT];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const uint32_t e = (uint32_t)(Rw::a(W, k) * cols + col);
    u64 v = ap[(e - rem) & (sh.n - 1)];  // X^a acc: new[e] = old[(e - rem) % N], negated for e < rem
    if (full ^ (e < rem)) v = neg_q<BNF>(v);
    const u64 x = BNF ? v - ap[e] : sub_custom(v, ap[e]);
    if (BNF) {
      st[k] = decomp_init_native(x, sh.base_log, (int)sh.level);
      sg[k] = false;
    } else {
      const unsigned shift = 64u - (unsigned)(sh.base_log * (int)sh.level);
      sg[k] = x >= P / 2 + 1;
      st[k] = closest_abs_nonnative(sg[k] ? P - x : x, sh.base_log, (int)sh.level) >> shift;
    }
  }
  u64 tv[ONLY ? RPT : 1];  // the block twist of the lane's phase-B rows: the same for every level
  if constexpr (ONLY) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) tv[k] = twist[Rw::b(W, k) * cols + col];
  }
#pragma unroll 1
  for (uint32_t li = 0; li < sh.level; ++li) {
    u64 x[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      u64 term = decompose_one_level(sh.base_log, st[k]);
      if (!BNF && sg[k]) term = (u64)0 - term;
      x[k] = ((int64_t)term < 0) ? term + P : term;
    }
    u64* o = dp + (uint64_t)li * per;
    if constexpr (K == 5 && ONLY) {  // r5: phase A, phase B and the block twist as generated asm (gen_tile_asm.py)
      tile5_fwd_a<W>(x);
      tile::exchange<K, W, true>(x, lds, c);
      tile5_fwd_b_tw<W>(x, tv);
#pragma unroll
      for (int k = 0; k < RPT; ++k) __builtin_nontemporal_store(x[k], o + Rw::b(W, k) * cols + col);
      continue;
    }
    tile::phase_a<K, true, W>(x);
    tile::exchange<K, W, true>(x, lds, c);
    tile::phase_b<K, true, W>(x);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const uint64_t e = Rw::b(W, k) * cols + col;
      // the digits are read once, by the next pass: non-temporal
      if constexpr (ONLY) __builtin_nontemporal_store(Goldilocks::mul(x[k], tv[k]), o + e);
      else __builtin_nontemporal_store(Goldilocks::canon(x[k]), o + e);  // the lazy tile stages
    }
  }
}

template <int K, bool BNF, bool ONLY>
__global__ __launch_bounds__(256) void large_rotdec_tile(u64* __restrict__ digits, const u64* __restrict__ acc,
                                                         const u64* __restrict__ lwe_in, uint32_t n_lwe, uint32_t step,
                                                         LargeShape sh, const u64* __restrict__ twist) {
  __shared__ u64 lds[(1 << K) * 64];
  const uint64_t cols = (uint64_t)sh.n >> K;
  const uint32_t c = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t col = (uint64_t)blockIdx.x * 64 + c;
  const uint32_t bc = blockIdx.y, b = bc / (sh.k + 1), cc = bc % (sh.k + 1);
  const unsigned log_mod = sh.logn + 1;
  const u64 a_raw = lwe_in[(uint64_t)b * (n_lwe + 1) + step];
  u64 a = 0;
  if (BNF) a = modulus_switch(a_raw, log_mod);
  else if (a_raw != 0) a = ms_non_native(a_raw, log_mod);
  const uint32_t full = (uint32_t)(a >> sh.logn) & 1u, rem = (uint32_t)(a & (sh.n - 1));
  const u64* ap = acc + (uint64_t)bc * sh.n;
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n;
  u64* dp = digits + (uint64_t)b * sh.level * per + (uint64_t)cc * sh.n;
  switch (w) {
    case 0: rotdec_tile_body<K, BNF, ONLY, 0>(dp, ap, full, rem, cols, col, c, per, sh, twist, lds); break;
    case 1: rotdec_tile_body<K, BNF, ONLY, 1>(dp, ap, full, rem, cols, col, c, per, sh, twist, lds); break;
    case 2: rotdec_tile_body<K, BNF, ONLY, 2>(dp, ap, full, rem, cols, col, c, per, sh, twist, lds); break;
    default: rotdec_tile_body<K, BNF, ONLY, 3>(dp, ap, full, rem, cols, col, c, per, sh, twist, lds); break;
  }
}

template <int K, bool BNF>
static hipError_t rotdec_top_launch(bool only, u64* digits, const u64* acc, const u64* lwe_in, uint32_t n_lwe,
                                    uint32_t step, uint32_t nb, const LargeShape& sh, const u64* tw, const u64* twist,
                                    hipStream_t s) {
  if constexpr (K >= 4) {
    if ((sh.n >> K) >= 64) {  // the cooperative tile (>= one 64-column tile)
      const dim3 tgrid((unsigned)(((uint64_t)sh.n >> K) / 64), nb * (sh.k + 1));
      if (only)
        hipLaunchKernelGGL((large_rotdec_tile<K, BNF, true>), tgrid, dim3(256), 0, s, digits, acc, lwe_in, n_lwe, step,
                           sh, twist);
      else
        hipLaunchKernelGGL((large_rotdec_tile<K, BNF, false>), tgrid, dim3(256), 0, s, digits, acc, lwe_in, n_lwe, step,
                           sh, twist);
      return hipGetLastError();
    }
  }
  const dim3 grid((unsigned)((((uint64_t)sh.n >> K) + 255) / 256), nb * (sh.k + 1));
  if (only)
    hipLaunchKernelGGL((large_rotdec_top<K, BNF, true>), grid, dim3(256), 0, s, digits, acc, lwe_in, n_lwe, step, sh,
                       tw, twist);
  else
    hipLaunchKernelGGL((large_rotdec_top<K, BNF, false>), grid, dim3(256), 0, s, digits, acc, lwe_in, n_lwe, step, sh,
                       tw, twist);
  return hipGetLastError();
}

template <bool BNF>
static hipError_t rotdec_top(int k0, bool only, u64* digits, const u64* acc, const u64* lwe_in, uint32_t n_lwe,
                             uint32_t step, uint32_t nb, const LargeShape& sh, const u64* tw, const u64* twist,
                             hipStream_t s) {
  switch (k0) {
    case 1: return rotdec_top_launch<1, BNF>(only, digits, acc, lwe_in, n_lwe, step, nb, sh, tw, twist, s);
    case 2: return rotdec_top_launch<2, BNF>(only, digits, acc, lwe_in, n_lwe, step, nb, sh, tw, twist, s);
    case 3: return rotdec_top_launch<3, BNF>(only, digits, acc, lwe_in, n_lwe, step, nb, sh, tw, twist, s);
    case 4: return rotdec_top_launch<4, BNF>(only, digits, acc, lwe_in, n_lwe, step, nb, sh, tw, twist, s);
    case 5: return rotdec_top_launch<5, BNF>(only, digits, acc, lwe_in, n_lwe, step, nb, sh, tw, twist, s);
    default: return hipErrorInvalidValue;
  }
}

// external product / CMUX input: CMUX first writes glwe -= out back (ct1 = ct1 - ct0), then both decompose glwe.
// gidx: item b is skipped (nothing written anywhere) when gidx[b] >= n_ggsw
template <bool BNF, bool CMUX>
__global__ __launch_bounds__(256) void large_glwe_decompose(u64* __restrict__ digits, u64* __restrict__ glwe,
                                                            const u64* __restrict__ out, uint32_t batch, LargeShape sh,
                                                            const uint32_t* __restrict__ gidx, uint32_t n_ggsw) {
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n, total = per * batch;
  for (uint64_t i = grid_stride_start(); i < total; i += grid_stride()) {
    const uint64_t b = i / per, ce = i % per;
    if (gidx && gidx[b] >= n_ggsw) continue;
    u64 x = glwe[i];
    if (CMUX) {
      x = BNF ? x - out[i] : sub_custom(x, out[i]);
      glwe[i] = x;
    }
    decompose_store<BNF>(x, digits + b * sh.level * per + ce, per, sh.base_log, (int)sh.level);
  }
}

// y[b][c][e] = sum over levels li and rows r of digits[b][li][r][e] * G[li][r][c][e] (update_with_fmadd,
// ntt64_pbs.rs:683-702 / ntt64_bnf_pbs.rs:707-726), times N^-1 when `n_inv` != 0 (the external product on a Raw
// BNF GGSW; the PBS's BNF key copy has N^-1 folded in already).  ggsw = the GGSW of item b: ggsw_list + gidx[b] (or
// the one GGSW when gidx is NULL)
__global__ __launch_bounds__(256) void large_mac(u64* __restrict__ y, const u64* __restrict__ digits,
                                                 const u64* __restrict__ ggsw_list, uint32_t batch, LargeShape sh,
                                                 u64 n_inv, const uint32_t* __restrict__ gidx, uint32_t n_ggsw) {
  const Goldilocks gl;
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n, total = per * batch;
  const uint64_t ggsw_len = (uint64_t)sh.level * (sh.k + 1) * per;
  for (uint64_t i = grid_stride_start(); i < total; i += grid_stride()) {
    const uint64_t b = i / per, ce = i % per;
    const uint32_t c = (uint32_t)(ce >> sh.logn), e = (uint32_t)(ce & (sh.n - 1));
    uint32_t g = 0;
    if (gidx) {
      g = gidx[b];
      if (g >= n_ggsw) continue;
    }
    const u64* G = ggsw_list + (uint64_t)g * ggsw_len;
    const u64* d = digits + b * sh.level * per + e;
    u64 acc = 0;
    for (uint32_t li = 0; li < sh.level; ++li)
      for (uint32_t r = 0; r <= sh.k; ++r)
        acc = gl.add(acc, gl.mul(d[(uint64_t)li * per + (uint64_t)r * sh.n],
                                 G[((uint64_t)li * (sh.k + 1) * (sh.k + 1) + (uint64_t)r * (sh.k + 1) + c) * sh.n + e]));
    y[i] = n_inv ? gl.mul(acc, n_inv) : acc;
  }
}

// The same product with every output column of an item in one thread (k + 1 = KP1 columns): each digit is read once
// instead of k + 1 times (the digits are (level + 1) / 2 of the step's HBM bytes at k = 1), and the level (k + 1)
// terms of a column are summed as 128-bit products with one reduction at the end (2^128 = -2^32 mod p).  A thread
// takes two adjacent coefficients (16-byte accesses).  Grid: x over coefficient pairs, y over the items.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// Acc128: the sum of a column's products with one reduction at the end (pbs_device.hpp)

// LEVEL > 0: the level count is compile-time (the shortint shapes' 1 - 3), so the level loop unrolls and every load of
// the item is issued before the first product; LEVEL = 0 reads it from sh
template <int KP1, int LEVEL>
__global__ __launch_bounds__(256) void large_mac_cols(u64* __restrict__ y, const u64* __restrict__ digits,
                                                      const u64* __restrict__ ggsw_list, uint32_t batch,
                                                      LargeShape sh, u64 n_inv, const uint32_t* __restrict__ gidx,
                                                      uint32_t n_ggsw) {
  const uint32_t e = (blockIdx.x * 256 + threadIdx.x) * 2;
  const uint32_t level = LEVEL ? (uint32_t)LEVEL : sh.level;
  const uint64_t n = sh.n, per = KP1 * n;
  const uint64_t ggsw_len = (uint64_t)level * KP1 * per;
  for (uint32_t b = blockIdx.y; b < batch; b += gridDim.y) {
    const u64* G = ggsw_list + e;
    if (gidx) {
      const uint32_t g = gidx[b];
      if (g >= n_ggsw) continue;
      G += (uint64_t)g * ggsw_len;
    }
    const u64* d = digits + (uint64_t)b * level * per + e;
    Acc128 acc[KP1][2];
    if constexpr (LEVEL > 0) {
      // all of the item's digit pairs first (the HBM loads in flight together), then the products with the GGSW
      // rows (L2)
      u64x2 x[LEVEL][KP1];
#pragma unroll
      for (int li = 0; li < LEVEL; ++li)
#pragma unroll
        for (int r = 0; r < KP1; ++r)
          // digits are read once: non-temporal, so the stream does not evict the GGSW rows every item re-reads
          x[li][r] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(d + ((uint64_t)li * KP1 + r) * n));
#pragma unroll
      for (int li = 0; li < LEVEL; ++li)
#pragma unroll
        for (int r = 0; r < KP1; ++r)
#pragma unroll
          for (int c = 0; c < KP1; ++c) {
            const ulonglong2 w = *reinterpret_cast<const ulonglong2*>(G + (((uint64_t)li * KP1 + r) * KP1 + c) * n);
            acc[c][0].mac(x[li][r].x, w.x);
            acc[c][1].mac(x[li][r].y, w.y);
          }
    } else {
      for (uint32_t li = 0; li < level; ++li) {
#pragma unroll
        for (int r = 0; r < KP1; ++r) {
          const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(d + ((uint64_t)li * KP1 + r) * n));
#pragma unroll
          for (int c = 0; c < KP1; ++c) {
            const ulonglong2 w = *reinterpret_cast<const ulonglong2*>(G + (((uint64_t)li * KP1 + r) * KP1 + c) * n);
            acc[c][0].mac(x.x, w.x);
            acc[c][1].mac(x.y, w.y);
          }
        }
      }
    }
    u64* out = y + (uint64_t)b * per + e;
#pragma unroll
    for (int c = 0; c < KP1; ++c) {
      const u64x2 v = {acc[c][0].value(n_inv), acc[c][1].value(n_inv)};
      __builtin_nontemporal_store(v, reinterpret_cast<u64x2*>(out + (uint64_t)c * n));
    }
  }
}

// large_mac_cols for k + 1 <= 4 (every shortint shape) and 16-byte aligned operands, large_mac otherwise
inline hipError_t launch_large_mac(u64* y, const u64* digits, const u64* ggsw_list, uint32_t batch,
                                   const LargeShape& sh, u64 n_inv, const uint32_t* gidx, uint32_t n_ggsw,
                                   hipStream_t s) {
  const bool aligned = (((uintptr_t)y | (uintptr_t)digits | (uintptr_t)ggsw_list) & 15) == 0;
  if (sh.k <= 3 && sh.n >= 512 && aligned) {
    const dim3 grid(sh.n / 512, std::min<uint32_t>(batch, 65535));
#define MI_MAC_COLS(KP, L) \
  hipLaunchKernelGGL((large_mac_cols<KP, L>), grid, dim3(256), 0, s, y, digits, ggsw_list, batch, sh, n_inv, gidx, n_ggsw)
#define MI_MAC_K(KP)                                  \
  switch (sh.level) {                                 \
    case 1: MI_MAC_COLS(KP, 1); break;                \
    case 2: MI_MAC_COLS(KP, 2); break;                \
    case 3: MI_MAC_COLS(KP, 3); break;                \
    default: MI_MAC_COLS(KP, 0); break;               \
  }
    switch (sh.k) {
      case 0: MI_MAC_K(1); break;
      case 1: MI_MAC_K(2); break;
      case 2: MI_MAC_K(3); break;
      default: MI_MAC_K(4); break;
    }
#undef MI_MAC_K
#undef MI_MAC_COLS
  } else {
    const uint64_t elems = (uint64_t)batch * (sh.k + 1) * sh.n;
    hipLaunchKernelGGL(large_mac, dim3((unsigned)std::min<uint64_t>((elems + 255) / 256, 65536)), dim3(256), 0, s, y,
                       digits, ggsw_list, batch, sh, n_inv, gidx, n_ggsw);
  }
  return hipGetLastError();
}

// acc += modswitch_{p -> 2^64}(y) (ntt64.rs:184-197 + wrapping add) / acc += y mod p (ntt64.rs:244-266)
template <bool BNF>
__global__ __launch_bounds__(256) void large_accumulate(u64* __restrict__ acc, const u64* __restrict__ y, uint32_t batch,
                                                        LargeShape sh, const uint32_t* __restrict__ gidx,
                                                        uint32_t n_ggsw) {
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n, total = per * batch;
  for (uint64_t i = grid_stride_start(); i < total; i += grid_stride()) {
    if (gidx && gidx[i / per] >= n_ggsw) continue;
    acc[i] = BNF ? acc[i] + modswitch_prime_to_native(y[i]) : add_custom(acc[i], y[i]);
  }
}

// centered_binary_ms_body_correction_to_add (algorithms/modulus_switch.rs:60-104), one workgroup per ciphertext
__global__ __launch_bounds__(256) void large_body_correction(u64* __restrict__ corr, const u64* __restrict__ lwe_in,
                                                             uint32_t n_lwe, unsigned log_mod) {
  __shared__ u64 sh[512];
  const u64 v = centered_body_correction<256>(lwe_in + (uint64_t)blockIdx.x * (n_lwe + 1), n_lwe, log_mod,
                                              (int)threadIdx.x, sh);
  if (threadIdx.x == 0) corr[blockIdx.x] = v;
}

// BNF: rotate by -ms(body [+ centered correction]) (ntt64_bnf_pbs.rs:262-270); Solinas: the LUT was pre-rotated;
// then sample extraction of coefficient 0 (glwe_sample_extraction.rs:89-160): out[c N] = A_c[0],
// out[c N + j] = -A_c[N - j], out[k N] = B[0]
// With io.glwe_out the rotated accumulator itself is stored (blind_rotate_ntt64[_bnf]_assign); skipped items
// (io.lut_for == NULL) are not written.  lwe_out / glwe_out point at the chunk's first item; b0 is its global index.
template <bool BNF, bool GLWE>
__global__ __launch_bounds__(256) void large_extract(u64* __restrict__ lwe_out, const u64* __restrict__ acc,
                                                     const u64* __restrict__ lwe_in, const u64* __restrict__ corr,
                                                     uint32_t n_lwe, uint32_t batch, LargeShape sh, PbsIo io,
                                                     uint64_t b0) {
  const uint64_t per = (uint64_t)(sh.k + 1) * sh.n;
  const uint64_t per_out = GLWE ? per : (uint64_t)sh.k * sh.n + 1, total = per_out * batch;
  for (uint64_t i = grid_stride_start(); i < total; i += grid_stride()) {
    const uint64_t b = i / per_out, o = i % per_out;
    if ((io.lut_idx || GLWE) && !io.lut_for(b0 + b, per)) continue;
    uint32_t full = 0, rem = 0;
    if (BNF) {
      const u64 body = modulus_switch(lwe_in[b * (n_lwe + 1) + n_lwe] + (corr ? corr[b] : 0), sh.logn + 1);
      full = (uint32_t)(body >> sh.logn) & 1u;
      rem = (uint32_t)(body & (sh.n - 1));
    }
    const uint32_t c = (uint32_t)(o >> sh.logn), j = (uint32_t)(o & (sh.n - 1));  // o = k N gives c = k, j = 0
    if (GLWE) {  // new[j] = old[(j + rem) % N], negated for j >= N - rem
      u64 v = acc[b * per + (uint64_t)c * sh.n + ((j + rem) & (sh.n - 1))];
      if (full ^ (j >= sh.n - rem)) v = neg_q<BNF>(v);
      lwe_out[i] = v;
      continue;
    }
    const uint32_t m = (j == 0) ? 0 : sh.n - j;
    u64 v = acc[b * per + (uint64_t)c * sh.n + ((m + rem) & (sh.n - 1))];
    if (full ^ (m >= sh.n - rem)) v = neg_q<BNF>(v);
    lwe_out[i] = (c == sh.k || j == 0) ? v : neg_q<BNF>(v);
  }
}

// forward_from_power_of_two_modulus (ntt64.rs:166-178): x -> round(x p / 2^w) of the key conversion
__global__ __launch_bounds__(256) void large_modswitch_to_prime(u64* __restrict__ dst, const u64* __restrict__ src,
                                                                uint64_t count, unsigned in_width) {
  for (uint64_t i = grid_stride_start(); i < count; i += grid_stride()) {
    u64 v = src[i];
    if (in_width) {
      const unsigned __int128 w =
          ((unsigned __int128)(v >> (64u - in_width))) * P + ((unsigned __int128)1 << (in_width - 1));
      v = (u64)(w >> in_width);
    }
    dst[i] = v;
  }
}

inline unsigned blocks_for(uint64_t total) {
  const uint64_t b = (total + 255) / 256;
  return (unsigned)std::min<uint64_t>(b, 65536);
}

// the plan's transform: the split engine (launch_ntt_split) when the plan has one, else the register-window passes
inline hipError_t ntt_large(bool fwd, int logn, u64* d, size_t batch, size_t stride, const u64* tw,
                            const SplitTw* split, hipStream_t s) {
  if (split) return launch_ntt_split(fwd, logn, d, batch, stride, tw, *split, s);
  return launch_ntt(fwd, logn, true, MontParams{}, d, batch, stride, tw, s);
}

// ciphertexts per chunk: the digits, products and accumulators of one chunk stay below ~4 GiB of scratch (of 288 GB)
inline size_t chunk_for(const LargeShape& sh, size_t batch) {
  const size_t per_item = ((size_t)sh.level + 2) * (sh.k + 1) * sh.n * sizeof(u64);
  return std::max<size_t>(1, std::min(batch, ((size_t)4 << 30) / per_item));
}

}  // namespace pbs

// Lanes: a chunk of >= PBS_LANE_MIN ciphertexts is split into mi::pbs_lane_count() parts (default 2, >= 16 ciphertexts
// each), the first on the caller's stream and the others on pooled side streams (mi::StreamFork), their launches
// interleaved step by step.  Each ciphertext's blind rotation is independent, so the parts share nothing but the key,
// and the GPU overlaps one part's memory-bound launches (the rotation + decomposition pass, the MAC, the accumulating
// inverse pass) with another's issue-bound transform bodies.
static constexpr uint32_t PBS_LANE_MIN = 64;


hipError_t launch_pbs_large(int logn, int k, bool bnf, int level, uint64_t* out, const uint64_t* lwe_in,
                            const PbsIo& io, const uint64_t* bsk, size_t n_lwe, size_t batch, int base_log,
                            const uint64_t* tw, const uint64_t* itw, int centered, hipStream_t s,
                            const SplitTw* split) {
  using namespace pbs;
  if (batch == 0) return hipSuccess;
  const LargeShape sh{(uint32_t)logn, 1u << logn, (uint32_t)k, (uint32_t)level, base_log};
  const size_t per = (size_t)(k + 1) * sh.n, chunk = chunk_for(sh, batch);
  const size_t ggsw_len = (size_t)level * (k + 1) * per;
  u64 *scratch = nullptr;
  hipError_t e = mi::scratch_alloc((void**)&scratch, (chunk * ((size_t)level + 2) * per + chunk) * sizeof(u64), s);
  if (e != hipSuccess) return e;
  int k0 = 0;
  bool only = false;
  if (split) split_first_pass(logn, &k0, &only);
  // r5: the MAC fused into the inverse's bodies (ntt64_tw.hip ntt_tw_inv_mac_kernel) where generated (l (k + 1) in
  // {2, 3, 4, 6, 8}); other shapes run the separate MAC pass
  const bool mac_fused = split && inv_mac_supported(level, k + 1);
  // one lane's share of a chunk: ciphertexts [b0, b0 + nb) of the batch, its scratch slices, its stream
  struct Lane {
    size_t b0;
    uint32_t nb;
    hipStream_t st;
    const u64* in;
    u64 *digits, *y, *acc, *corr;
  };
  auto init = [&](const Lane& L) -> hipError_t {
    const uint64_t elems = (uint64_t)L.nb * per;
    if (bnf)
      hipLaunchKernelGGL(large_init_acc<true>, dim3(blocks_for(elems)), dim3(256), 0, L.st, L.acc, io,
                         (uint64_t)L.b0, L.in, (uint32_t)n_lwe, L.nb, sh);
    else
      hipLaunchKernelGGL(large_init_acc<false>, dim3(blocks_for(elems)), dim3(256), 0, L.st, L.acc, io,
                         (uint64_t)L.b0, L.in, (uint32_t)n_lwe, L.nb, sh);
    return hipGetLastError();
  };
  auto step = [&](const Lane& L, uint32_t i) -> hipError_t {  // CMUX step i of the lane's blind rotations
    const uint32_t nb = L.nb;
    const uint64_t elems = (uint64_t)nb * per;
    hipError_t e;
    if (split) {  // rotation + decomposition + the transform's first pass in one kernel, then the rest of the transform
      e = bnf ? rotdec_top<true>(k0, only, L.digits, L.acc, L.in, (uint32_t)n_lwe, i, nb, sh, tw, split->blk_fwd, L.st)
              : rotdec_top<false>(k0, only, L.digits, L.acc, L.in, (uint32_t)n_lwe, i, nb, sh, tw, split->blk_fwd, L.st);
      if (e == hipSuccess)
        e = launch_ntt_split(true, logn, L.digits, (size_t)nb * level * (k + 1), sh.n, tw, *split, L.st, nullptr, 0,
                             true);
    } else {
      if (bnf)
        hipLaunchKernelGGL(large_rotate_decompose<true>, dim3(blocks_for(elems)), dim3(256), 0, L.st, L.digits, L.acc,
                           L.in, (uint32_t)n_lwe, i, nb, sh);
      else
        hipLaunchKernelGGL(large_rotate_decompose<false>, dim3(blocks_for(elems)), dim3(256), 0, L.st, L.digits, L.acc,
                           L.in, (uint32_t)n_lwe, i, nb, sh);
      e = ntt_large(true, logn, L.digits, (size_t)nb * level * (k + 1), sh.n, tw, split, L.st);
    }
    if (e != hipSuccess) return e;
    if (mac_fused)  // the MAC formed on load by the inverse's 2048-block bodies, then the inverse's top passes
      return (e = launch_ntt_tw_inv_mac(L.y, L.digits, bsk + (size_t)i * ggsw_len, nb, k + 1, level, logn,
                                         split->body_inv, L.st)) != hipSuccess
                 ? e
                 : launch_ntt_split(false, logn, L.y, (size_t)nb * (k + 1), sh.n, itw, *split, L.st, L.acc,
                                    bnf ? 1 : 2, true);
    e = launch_large_mac(L.y, L.digits, bsk + (size_t)i * ggsw_len, nb, sh, (u64)0, nullptr, 1u, L.st);
    if (e != hipSuccess) return e;
    if (split)  // the inverse's last pass accumulates into acc itself (launch_ntt_split acc_mode)
      return launch_ntt_split(false, logn, L.y, (size_t)nb * (k + 1), sh.n, itw, *split, L.st, L.acc, bnf ? 1 : 2);
    e = ntt_large(false, logn, L.y, (size_t)nb * (k + 1), sh.n, itw, split, L.st);
    if (e != hipSuccess) return e;
    if (bnf)
      hipLaunchKernelGGL(large_accumulate<true>, dim3(blocks_for(elems)), dim3(256), 0, L.st, L.acc, L.y, nb, sh,
                         (const uint32_t*)nullptr, 1u);
    else
      hipLaunchKernelGGL(large_accumulate<false>, dim3(blocks_for(elems)), dim3(256), 0, L.st, L.acc, L.y, nb, sh,
                         (const uint32_t*)nullptr, 1u);
    return hipGetLastError();
  };
  auto finish = [&](const Lane& L) -> hipError_t {  // body correction, final rotation + extraction
    const uint32_t nb = L.nb;
    const bool corr_on = bnf && centered;
    if (corr_on)
      hipLaunchKernelGGL(large_body_correction, dim3(nb), dim3(256), 0, L.st, L.corr, L.in, (uint32_t)n_lwe,
                         (unsigned)(logn + 1));
    const u64* cr = corr_on ? L.corr : (const u64*)nullptr;
    if (io.glwe_out) {
      const uint64_t outs = (uint64_t)nb * per;
      u64* o = io.glwe_out + L.b0 * per;
      if (bnf)
        hipLaunchKernelGGL((large_extract<true, true>), dim3(blocks_for(outs)), dim3(256), 0, L.st, o, L.acc, L.in, cr,
                           (uint32_t)n_lwe, nb, sh, io, (uint64_t)L.b0);
      else
        hipLaunchKernelGGL((large_extract<false, true>), dim3(blocks_for(outs)), dim3(256), 0, L.st, o, L.acc, L.in,
                           cr, (uint32_t)n_lwe, nb, sh, io, (uint64_t)L.b0);
    } else {
      const uint64_t outs = (uint64_t)nb * ((uint64_t)k * sh.n + 1);
      u64* o = out + L.b0 * ((size_t)k * sh.n + 1);
      if (bnf)
        hipLaunchKernelGGL((large_extract<true, false>), dim3(blocks_for(outs)), dim3(256), 0, L.st, o, L.acc, L.in,
                           cr, (uint32_t)n_lwe, nb, sh, io, (uint64_t)L.b0);
      else
        hipLaunchKernelGGL((large_extract<false, false>), dim3(blocks_for(outs)), dim3(256), 0, L.st, o, L.acc, L.in,
                           cr, (uint32_t)n_lwe, nb, sh, io, (uint64_t)L.b0);
    }
    return hipGetLastError();
  };
  for (size_t c0 = 0; c0 < batch && e == hipSuccess; c0 += chunk) {
    const uint32_t nb = (uint32_t)std::min(chunk, batch - c0);
    mi::StreamFork fork;
    const int want = nb >= PBS_LANE_MIN ? std::min<int>(mi::pbs_lane_count(2), (int)(nb / 16)) : 1;
    if (want > 1) (void)fork.fork(s, want - 1);  // fewer lanes when a side stream cannot be had
    const int lanes = 1 + fork.sides();
    Lane L[1 + mi::StreamFork::MAX_SIDE];
    for (int j = 0, off = 0; j < lanes; ++j) {
      const uint32_t n = nb / lanes + ((uint32_t)j < nb % lanes ? 1u : 0u);
      L[j] = Lane{c0 + off, n, j == 0 ? s : fork.side(j - 1), lwe_in + (c0 + off) * (n_lwe + 1),
                  scratch + (size_t)off * level * per, scratch + chunk * level * per + (size_t)off * per,
                  scratch + chunk * (level + 1) * per + (size_t)off * per, scratch + chunk * (level + 2) * per + off};
      off += (int)n;
    }
    for (int j = 0; j < lanes && e == hipSuccess; ++j) e = init(L[j]);
    for (uint32_t i = 0; i < n_lwe && e == hipSuccess; ++i)
      for (int j = 0; j < lanes && e == hipSuccess; ++j) e = step(L[j], i);
    for (int j = 0; j < lanes && e == hipSuccess; ++j) e = finish(L[j]);
    const hipError_t ej = fork.join();  // the caller's stream after the side lane (also on error: scratch ordering)
    if (e == hipSuccess) e = ej;
  }
  const hipError_t ef = mi::scratch_free(scratch, s);
  return e != hipSuccess ? e : ef;
}

// convert_standard_lwe_bootstrap_key_to_ntt64 (lwe_bootstrap_key_conversion.rs:294-365) at large N: modulus switch
// into dst, the large-N forward transform in place, optional normalisation (NttLweBootstrapKeyOption::Normalize)
hipError_t launch_bsk_to_ntt_large(int logn, uint64_t* dst, const uint64_t* src, size_t n_polys, unsigned in_width,
                                   int normalize, uint64_t n_inv, const uint64_t* tw, hipStream_t s,
                                   const SplitTw* split) {
  using namespace pbs;
  if (n_polys == 0) return hipSuccess;
  const uint64_t count = (uint64_t)n_polys << logn;
  hipLaunchKernelGGL(large_modswitch_to_prime, dim3(blocks_for(count)), dim3(256), 0, s, dst, src, count, in_width);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = ntt_large(true, logn, dst, n_polys, (size_t)1 << logn, tw, split, s);
  if (e == hipSuccess && normalize) e = launch_scale(dst, dst, count, n_inv, s);
  return e;
}

hipError_t launch_ext_product_large(int logn, int k, bool bnf, bool cmux, int level, uint64_t* out, uint64_t* glwe,
                                    const uint64_t* ggsw, size_t batch, int base_log, const uint64_t* tw,
                                    const uint64_t* itw, uint64_t n_inv, hipStream_t s, const uint32_t* gidx,
                                    uint32_t n_ggsw, const SplitTw* split) {
  using namespace pbs;
  if (batch == 0) return hipSuccess;
  const LargeShape sh{(uint32_t)logn, 1u << logn, (uint32_t)k, (uint32_t)level, base_log};
  const size_t per = (size_t)(k + 1) * sh.n, chunk = chunk_for(sh, batch);
  u64* scratch = nullptr;
  hipError_t e = mi::scratch_alloc((void**)&scratch, chunk * ((size_t)level + 1) * per * sizeof(u64), s);
  if (e != hipSuccess) return e;
  u64* digits = scratch;
  u64* y = digits + chunk * level * per;
  for (size_t b0 = 0; b0 < batch && e == hipSuccess; b0 += chunk) {
    const uint32_t nb = (uint32_t)std::min(chunk, batch - b0);
    const uint64_t elems = (uint64_t)nb * per;
    u64* o = out + b0 * per;
    u64* g = glwe + b0 * per;
    const uint32_t* gi = gidx ? gidx + b0 : nullptr;
#define MI_LARGE_DEC(B, C)                                                                                          \
  hipLaunchKernelGGL((large_glwe_decompose<B, C>), dim3(blocks_for(elems)), dim3(256), 0, s, digits, g, o, nb, sh, gi, \
                     n_ggsw)
    if (bnf) {
      if (cmux) MI_LARGE_DEC(true, true); else MI_LARGE_DEC(true, false);
    } else {
      if (cmux) MI_LARGE_DEC(false, true); else MI_LARGE_DEC(false, false);
    }
#undef MI_LARGE_DEC
    e = ntt_large(true, logn, digits, (size_t)nb * level * (k + 1), sh.n, tw, split, s);
    if (e != hipSuccess) break;
    // BNF GGSWs are the reference's Raw NTT keys: the product is normalised here (ntt64_bnf_pbs.rs:670)
    e = launch_large_mac(y, digits, ggsw, nb, sh, bnf ? (u64)n_inv : (u64)0, gi, gi ? n_ggsw : 1u, s);
    if (e != hipSuccess) break;
    e = ntt_large(false, logn, y, (size_t)nb * (k + 1), sh.n, itw, split, s);
    if (e != hipSuccess) break;
    if (bnf)
      hipLaunchKernelGGL(large_accumulate<true>, dim3(blocks_for(elems)), dim3(256), 0, s, o, y, nb, sh, gi, n_ggsw);
    else
      hipLaunchKernelGGL(large_accumulate<false>, dim3(blocks_for(elems)), dim3(256), 0, s, o, y, nb, sh, gi, n_ggsw);
    e = hipGetLastError();
  }
  const hipError_t ef = mi::scratch_free(scratch, s);
  return e != hipSuccess ? e : ef;
}

}  // namespace mi
