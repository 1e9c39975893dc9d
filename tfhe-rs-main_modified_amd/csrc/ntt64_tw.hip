// ntt64_tw.hip — "twisted" N = 2048 Goldilocks transform: shift-only butterflies.
//
// Same transform as Plan::fwd / Plan::inv of the Solinas plan (reference:
// tfhe-ntt/src/prime64/generic_solinas.rs:449-514, twiddles prime64.rs:159-204), bit-identical
// because every value it writes is the canonical residue, computed through an
// algebraically equivalent factorisation that trades general 64x64 modular multiplies for shifts:
//
//   forward = the reference's first 5 merged-CT stages (m = 1..16): their twiddles twid[m+i] are
//             powers of two in the Solinas root tower (psi^64 = 8), so b*w is a shift + fold;
//           -> twist: element 64 i + j (block i, 0 <= j < 64) times rho_i^j, rho_i = psi^(2 rev5(i) + 1)
//              (the only general multiplies left: 2048 per transform instead of 11264);
//           -> per 64-element block a cyclic CT DFT with omega = psi^64 = 8 (natural in, bit-reversed
//              out): every twiddle is 2^(3k).
//   inverse = the mirror (GS stages with the inverse exponents, untwist by rho_i^-j), unnormalised.
// tools/gen_tw_tables.py derives the exponent tables from the plan's twiddles and checks the
// factorisation against the oracle; tests/test_ntt_gpu.py checks this kernel bit-exactly.
//
// MI355X mapping: one wave (64 lanes) per polynomial, 32 coefficients per lane in VGPRs.
//   W0 layout (lane = j, register = i): the 5 twisted-out stages act on register bits, all
//      exponents compile-time; loads/stores are 512-B coalesced rows.
//   one in-wave LDS transpose (two 8 KiB halves, row stride 34 u64: conflict-free both ways),
//   W1 layout (lane = 2 i + j0, register = j >> 1): cyclic stages on register bits, compile-time.
//   last cyclic stage (bit j0, across lane pairs): one DPP quad_perm swap regroups the pairs so each
//      lane owns 16 whole butterflies (lane-variable twiddle, one multiply each) and 16-B outputs.
// No __syncthreads: every wave owns its LDS slice.  The data path is one generated asm body per
// direction (tools/gen_tw_kernel.py -> ntt64_tw_body.hpp); DESIGN.md §4 has the layouts and costs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_tw_tables.hpp"
#include "ntt64_tw_device.hpp"

namespace mi {
namespace tw {

// ---- whole-body asm kernel (tools/gen_tw_kernel.py) ----------------------------------------------
// The generated body owns v8..v127 / s20..s99 and performs load -> all stages -> store itself; the wrappers
// (ntt64_tw_device.hpp tw_body) only derive the wave's polynomial and the per-lane LDS / global addresses.

// Waves per workgroup, measured (tools/variant_probe.hip: same process, rotated order, identical-body controls):
// the forward runs best with one wave per group (a finished wave frees its slot and its 8.5 KiB of LDS at once:
// 57.5 vs 59.8 us per 8192-poly launch with 4-wave groups); the inverse, whose W1'' transposes read with half
// the lanes, with four (60.5 vs 62.4 us with one).
template <bool FWD>
constexpr uint32_t tw_waves() { return FWD ? 1u : 4u; }

// sub_log > 0 (the split transform of N = 2^(11 + sub_log), ntt64_kernels.hip launch_ntt_split): unit `poly` is block
// poly & (2^sub_log - 1) of polynomial poly >> sub_log, 2048 contiguous coefficients at that block's offset
template <bool FWD>
__global__ __launch_bounds__(64 * tw_waves<FWD>()) void ntt_tw_body_kernel(u64* __restrict__ data, uint32_t batch,
                                                                          uint64_t stride,
                                                                          const u64* __restrict__ twist,
                                                                          uint32_t sub_log) {
  constexpr uint32_t W = tw_waves<FWD>();
  __shared__ u64 lds[W * WAVE_LDS2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = W == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t poly = blockIdx.x * W + wv;
  if (poly >= batch) return;
  u64* p = data + (uint64_t)(poly >> sub_log) * stride + (uint64_t)(poly & ((1u << sub_log) - 1)) * 2048;
  tw_body<FWD>(p, twist, (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2), lane);
}

// ---- the split transform of N = 2^(11 + T), T <= 3, in one launch ------------------------------------------------
// One workgroup of 2^T waves per polynomial.  Forward: the T top stages (stage 0 on: the Solinas tower's powers of
// two, Goldilocks::mul_pow2) on the 2048 columns of 2^T rows and the block twist (element e times blk[e]), stored;
// a workgroup barrier; then wave w runs the 2048 body on block w.  Inverse: the bodies, a barrier, then the block
// untwist and the T stages (GS, reverse order) on the columns, stored.  The same arithmetic as
// ntt_top_kernel<T, FWD, Goldilocks, u64, TWIST, 0, true> at s0 = 0 followed / preceded by ntt_tw_body_kernel with
// sub_log = T (bit-exact), but the polynomial crosses HBM once: the intermediate is written and re-read by the same
// workgroup, from L2 / the memory-side cache.  A lane holds 32 / 2^T columns x 2^T rows = 32 values (T = 3: two
// calls of 2 columns, within 128 VGPRs).
template <int T, bool FWD>
__device__ __forceinline__ void fused_columns(u64* __restrict__ poly, const u64* __restrict__ blk, uint32_t tid,
                                              int c0) {
  constexpr int R = 1 << T, CPL = T == 3 ? 2 : 32 >> T, THREADS = 64 << T;  // CPL: columns of this call
  u64 x[CPL][R];
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint32_t e = (uint32_t)(i * 2048 + (c0 + c) * THREADS) + tid;
      x[c][i] = FWD ? poly[e] : Goldilocks::mul(poly[e], blk[e]);
    }
#pragma unroll
  for (int st = 0; st < T; ++st) {
    const int s = FWD ? st : T - 1 - st;  // stage s: 2^s groups, pair distance 2^(T-1-s) in i
    const int d = 1 << (T - 1 - s);
#pragma unroll
    for (int c = 0; c < CPL; ++c)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if (i & d) continue;
        const int ex = tower_exp(FWD, s, i >> (T - s));
        bool ng;
        if (FWD) {
          const u64 z = Goldilocks::mul_pow2(x[c][i + d], ex, ng);
          const u64 a = x[c][i];
          x[c][i] = ng ? Goldilocks::sub(a, z) : Goldilocks::add(a, z);
          x[c][i + d] = ng ? Goldilocks::add(a, z) : Goldilocks::sub(a, z);
        } else {  // (a - b) w = (b - a) |w| for a negative w
          const u64 a = x[c][i], b = x[c][i + d];
          x[c][i] = Goldilocks::add(a, b);
          x[c][i + d] = Goldilocks::mul_pow2(ex >= 96 ? Goldilocks::sub(b, a) : Goldilocks::sub(a, b), ex, ng);
        }
      }
  }
#pragma unroll
  for (int c = 0; c < CPL; ++c)
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const uint32_t e = (uint32_t)(i * 2048 + (c0 + c) * THREADS) + tid;
      poly[e] = FWD ? Goldilocks::mul(x[c][i], blk[e]) : x[c][i];
    }
}

template <int T, bool FWD>
__global__ __launch_bounds__(64 << T) __attribute__((amdgpu_waves_per_eu(4))) void ntt_tw_fused_kernel(
    u64* __restrict__ data, uint64_t stride, const u64* __restrict__ blk, const u64* __restrict__ body_tab) {
  __shared__ u64 lds[(1 << T) * WAVE_LDS2];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  u64* poly = data + (uint64_t)blockIdx.x * stride;
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  if constexpr (FWD) {
    fused_columns<T, true>(poly, blk, tid, 0);
    if constexpr (T == 3) fused_columns<T, true>(poly, blk, tid, 2);  // two calls: 2 x 16 values (VGPRs)
    __syncthreads();  // the workgroup's stores are visible to its waves (one CU, one L1)
    tw_body<true>(poly + wv * 2048, body_tab, S, lane);
  } else {
    tw_body<false>(poly + wv * 2048, body_tab, S, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the body's stores (inline asm: not tracked by the compiler)
    __syncthreads();
    fused_columns<T, false>(poly, blk, tid, 0);
    if constexpr (T == 3) fused_columns<T, false>(poly, blk, tid, 2);
  }
}

// Key conversion, native 2^64 input (convert_standard_lwe_bootstrap_key_to_ntt64,
// lwe_bootstrap_key_conversion.rs:294-365 with ntt64.rs:166-178): each wave loads one standard-domain polynomial,
// switches it into Z_p, runs the forward body and writes the NTT-domain polynomial to `dst` (may equal `src`: a
// wave reads its whole polynomial before writing).  `twist` = the plan's forward table, or its N^-1-scaled copy for
// the Normalize variant (the twist multiplies every element exactly once, so the output is fwd(x) N^-1).
__global__ __launch_bounds__(64) void ntt_tw_ms64_kernel(u64* dst, const u64* src, uint32_t n_polys,
                                                         const u64* __restrict__ twist) {
  __shared__ u64 lds[WAVE_LDS2];
  const uint32_t lane = threadIdx.x;
  const uint32_t poly = blockIdx.x;
  if (poly >= n_polys) return;
  const u64* p = src + (uint64_t)poly * 2048;
  u64* q = dst + (uint64_t)poly * 2048;
  const uint32_t S = (uint32_t)(uintptr_t)lds;
  const uint32_t l8 = lane * 8;
  const FwdAddrs a(S, lane);
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t olo = (uint32_t)(uintptr_t)q, ohi = (uint32_t)((uintptr_t)q >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2048;
  MI_TW_BODY_FWD_MS64([g_lo] "s"(glo), [g_hi] "s"(ghi), [o_lo] "s"(olo), [o_hi] "s"(ohi), [tw_lo] "s"(twlo),
                      [tw_hi] "s"(twhi), [lw] "s"(lw), [l8] "v"(l8), [t1w] "v"(a.t1w), [t1r] "v"(a.t1r),
                      [t2wl] "v"(a.t2wl), [t2wh] "v"(a.t2wh), [t2r] "v"(a.t2r), [lwo] "v"(a.lwo));
}


// ---- the MAC-fused inverse bodies of the large-N blind rotation (pbs_large.hip, tools/gen_tw_kernel.py gen_inv_mac) ---
// Unit u = (blk n_items + b) (k + 1) + c: output column c of item b, 2048-block blk.  The body forms the block of
// y_c = sum over the L = l (k + 1) terms q = li (k + 1) + r of digits[b][li][r] . GGSW[li][r][c] on load (digit q at
// digits + b L N + q N, GGSW row q at ggsw + (q (k + 1) + c) N, both + blk 2048), runs the inverse body on it and
// stores y (the products' [b][c][N] layout).  Four waves per workgroup, as the inverse.  The unit order puts the k + 1
// columns of one (item, block) in adjacent waves of a workgroup (the second reads the item's digit rows from L1 / L2,
// not HBM: each digit row is read from HBM once, as large_mac_cols does) and walks the items of one block before the
// next block (the step's GGSW rows of a block stay L2-resident across the items).
template <int L>
__device__ __forceinline__ void inv_mac_unit(u64* __restrict__ y, const u64* __restrict__ digits,
                                             const u64* __restrict__ ggsw, uint32_t u, uint32_t n_items,
                                             uint32_t sub_log, uint32_t kp1, const u64* __restrict__ twist, u64* wl,
                                             uint32_t lane) {
  const uint32_t c = u % kp1, ib = u / kp1, b = ib % n_items, blk = ib / n_items;
  const uint64_t n = (uint64_t)2048 << sub_log;
  u64* p = y + ((uint64_t)b * kp1 + c) * n + (uint64_t)blk * 2048;
  const u64* d = digits + (uint64_t)b * L * n + (uint64_t)blk * 2048;
  const u64* g = ggsw + (uint64_t)c * n + (uint64_t)blk * 2048;
  const uint32_t S = (uint32_t)(uintptr_t)wl;
  const uint32_t l8 = lane * 8;
  const tw::InvAddrs a(S, lane);
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2 * (2048 + 32);  // the last-DIT-stage table (tw_body<false>)
  const uint32_t dlo = (uint32_t)(uintptr_t)d, dhi = (uint32_t)((uintptr_t)d >> 32);
  const uint32_t gglo = (uint32_t)(uintptr_t)g, gghi = (uint32_t)((uintptr_t)g >> 32);
  const uint32_t dstep = (uint32_t)(n * 8), gstep = (uint32_t)(kp1 * n * 8);
#define MI_INV_MAC_OPS                                                                                             \
  [g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw), [l8] "v"(l8), [t4w] "v"(a.t4w), \
      [t1x] "v"(a.t1x), [t1y] "v"(a.t1y), [lwo] "v"(a.lwo), [d_lo] "s"(dlo), [d_hi] "s"(dhi), [dstep] "s"(dstep),           \
      [gg_lo] "s"(gglo), [gg_hi] "s"(gghi), [gstep] "s"(gstep)
  if constexpr (L == 2) MI_TW_BODY_INV_MAC2(MI_INV_MAC_OPS);
  else if constexpr (L == 3) MI_TW_BODY_INV_MAC3(MI_INV_MAC_OPS);
  else if constexpr (L == 4) MI_TW_BODY_INV_MAC4(MI_INV_MAC_OPS);
  else if constexpr (L == 6) MI_TW_BODY_INV_MAC6(MI_INV_MAC_OPS);
  else MI_TW_BODY_INV_MAC8(MI_INV_MAC_OPS);
#undef MI_INV_MAC_OPS
}

template <int L>
__global__ __launch_bounds__(256) void ntt_tw_inv_mac_kernel(u64* __restrict__ y, const u64* __restrict__ digits,
                                                             const u64* __restrict__ ggsw, uint32_t units,
                                                             uint32_t n_items, uint32_t sub_log, uint32_t kp1,
                                                             const u64* __restrict__ twist) {
  constexpr uint32_t W = 4;
  __shared__ u64 lds[W * WAVE_LDS2];
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t u = blockIdx.x * W + wv;
  if (u < units) inv_mac_unit<L>(y, digits, ggsw, u, n_items, sub_log, kp1, twist, lds + wv * WAVE_LDS2, lane);
}

}  // namespace tw

hipError_t launch_ntt_tw_ms64(uint64_t* dst, const uint64_t* src, size_t n_polys, const uint64_t* twist,
                              hipStream_t s) {
  constexpr size_t CHUNK = size_t(1) << 30;
  for (size_t off = 0; off < n_polys; off += CHUNK) {
    const uint32_t n = (uint32_t)std::min(CHUNK, n_polys - off);
    hipLaunchKernelGGL(tw::ntt_tw_ms64_kernel, dim3(n), dim3(64), 0, s, dst + off * 2048, src + off * 2048, n, twist);
  }
  return hipGetLastError();
}

template <int T>
static void fused_launch(bool fwd, uint64_t* d, uint32_t n, size_t stride, const uint64_t* blk, const uint64_t* body_tab,
                         hipStream_t s) {
  if (fwd)
    hipLaunchKernelGGL((tw::ntt_tw_fused_kernel<T, true>), dim3(n), dim3(64 << T), 0, s, d, (uint64_t)stride, blk,
                       body_tab);
  else
    hipLaunchKernelGGL((tw::ntt_tw_fused_kernel<T, false>), dim3(n), dim3(64 << T), 0, s, d, (uint64_t)stride, blk,
                       body_tab);
}

hipError_t launch_ntt_split_fused(bool fwd, int t, uint64_t* data, size_t batch, size_t stride, const uint64_t* blk,
                                  const uint64_t* body_tab, hipStream_t s) {
  if (t < 1 || t > 3) return hipErrorInvalidValue;
  constexpr size_t CHUNK = size_t(1) << 30;
  for (size_t off = 0; off < batch; off += CHUNK) {
    const uint32_t n = (uint32_t)std::min(CHUNK, batch - off);
    uint64_t* d = data + off * stride;
    switch (t) {
      case 1: fused_launch<1>(fwd, d, n, stride, blk, body_tab, s); break;
      case 2: fused_launch<2>(fwd, d, n, stride, blk, body_tab, s); break;
      default: fused_launch<3>(fwd, d, n, stride, blk, body_tab, s); break;
    }
  }
  return hipGetLastError();
}

bool inv_mac_supported(int level, int kp1) {
  const int L = level * kp1;
  return L == 2 || L == 3 || L == 4 || L == 6 || L == 8;
}

hipError_t launch_ntt_tw_inv_mac(uint64_t* y, const uint64_t* digits, const uint64_t* ggsw, size_t n_items, int kp1,
                                 int level, int logn, const uint64_t* twist, hipStream_t s) {
  const int sub_log = logn - 11;
  if (sub_log < 1 || !inv_mac_supported(level, kp1)) return hipErrorInvalidValue;
  if (n_items == 0) return hipSuccess;
  const uint64_t units = (uint64_t)n_items * kp1 << sub_log;
  if (units > 0xffffffffull - 4 * 65536) return hipErrorInvalidValue;  // uint32 unit indices (the callers' chunks are far below)
  const dim3 grid((unsigned)((units + 3) / 4)), block(256);
  const uint32_t un = (uint32_t)units, ni = (uint32_t)n_items, sl = (uint32_t)sub_log, kp = (uint32_t)kp1;
  switch (level * kp1) {
    case 2: hipLaunchKernelGGL(tw::ntt_tw_inv_mac_kernel<2>, grid, block, 0, s, y, digits, ggsw, un, ni, sl, kp, twist); break;
    case 3: hipLaunchKernelGGL(tw::ntt_tw_inv_mac_kernel<3>, grid, block, 0, s, y, digits, ggsw, un, ni, sl, kp, twist); break;
    case 4: hipLaunchKernelGGL(tw::ntt_tw_inv_mac_kernel<4>, grid, block, 0, s, y, digits, ggsw, un, ni, sl, kp, twist); break;
    case 6: hipLaunchKernelGGL(tw::ntt_tw_inv_mac_kernel<6>, grid, block, 0, s, y, digits, ggsw, un, ni, sl, kp, twist); break;
    default: hipLaunchKernelGGL(tw::ntt_tw_inv_mac_kernel<8>, grid, block, 0, s, y, digits, ggsw, un, ni, sl, kp, twist); break;
  }
  return hipGetLastError();
}

hipError_t launch_ntt_tw(bool fwd, uint64_t* data, size_t batch, size_t stride, const uint64_t* twist, hipStream_t s,
                         int sub_log) {
  if (batch == 0) return hipSuccess;
  // grid.x limit 2^31 - 1 (a whole chunk is 16 TiB of polynomials); a chunk of units holds whole polynomials
  const size_t CHUNK = (size_t(1) << 30) >> sub_log << sub_log;
  const size_t units = batch << sub_log;
  for (size_t off = 0; off < units; off += CHUNK) {
    const uint32_t n = (uint32_t)std::min(CHUNK, units - off);
    uint64_t* d = data + (off >> sub_log) * stride;
    if (fwd) {
      constexpr uint32_t W = tw::tw_waves<true>();
      hipLaunchKernelGGL((tw::ntt_tw_body_kernel<true>), dim3((n + W - 1) / W), dim3(64 * W), 0, s, d, n,
                         (uint64_t)stride, twist, (uint32_t)sub_log);
    } else {
      constexpr uint32_t W = tw::tw_waves<false>();
      hipLaunchKernelGGL((tw::ntt_tw_body_kernel<false>), dim3((n + W - 1) / W), dim3(64 * W), 0, s, d, n,
                         (uint64_t)stride, twist, (uint32_t)sub_log);
    }
  }
  return hipGetLastError();
}

}  // namespace mi
