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

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_tw_tables.hpp"
#include "ntt64_tw_body.hpp"

namespace mi {
namespace tw {

// ---- whole-body asm kernel (tools/gen_tw_kernel.py) ----------------------------------------------
// The generated body owns v8..v127 / s20..s99 and performs load -> all stages -> store itself; this
// wrapper only derives the wave's polynomial and the per-lane LDS / global addresses.
static constexpr int WAVE_LDS2 = 1088;  // u64: max(32 x 34, 16 x 66)

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
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8;
  const uint32_t t1w = S + (lane & 31) * 8;
  const uint32_t t1r = S + (i * 34 + par) * 8;
  const uint32_t lwo = par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  // forward: the lane-pair twiddles follow the twist rows; inverse: the last-DIT-stage table, two regions on
  // (the plan's allocation: [fwd + 32 | inverse + 32 | inverse N^-1 + 32 | 32], `twist` = the inverse region)
  const u64* lw = FWD ? twist + 2048 : twist + 2 * (2048 + 32);
  if constexpr (FWD) {
    const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8;
    const uint32_t t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
    const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
    MI_TW_BODY_FWD([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r), [t2wl] "v"(t2wl), [t2wh] "v"(t2wh),
                   [t2r] "v"(t2r), [lwo] "v"(lwo));
  } else {
    const uint32_t t4w = S + ((i & 15) * 66 + par) * 8;
    const uint32_t t1x = S + (lane + (lane >> 5)) * 8;        // W0 side of the W1'' transposes
    const uint32_t t1y = S + ((i & 15) * 66 + 33 * par) * 8;  // W1'' side
    MI_TW_BODY_INV([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t4w] "v"(t4w), [t1x] "v"(t1x), [t1y] "v"(t1y), [lwo] "v"(lwo));
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
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8;
  const uint32_t t1w = S + (lane & 31) * 8;
  const uint32_t t1r = S + (i * 34 + par) * 8;
  const uint32_t lwo = par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t olo = (uint32_t)(uintptr_t)q, ohi = (uint32_t)((uintptr_t)q >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2048;
  const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8;
  const uint32_t t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
  const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
  MI_TW_BODY_FWD_MS64([g_lo] "s"(glo), [g_hi] "s"(ghi), [o_lo] "s"(olo), [o_hi] "s"(ohi), [tw_lo] "s"(twlo),
                      [tw_hi] "s"(twhi), [lw] "s"(lw), [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r),
                      [t2wl] "v"(t2wl), [t2wh] "v"(t2wh), [t2r] "v"(t2r), [lwo] "v"(lwo));
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
