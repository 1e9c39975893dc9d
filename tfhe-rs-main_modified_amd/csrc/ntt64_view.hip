// ntt64_view.hip — the Ntt64View layer of tfhe-rs as batched device operations.
//
// Reference: tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:81-266 — the six per-polynomial helpers every tfhe-rs NTT
// consumer calls (ntt64_pbs.rs:600-663, ntt64_bnf_pbs.rs:596-681, lwe_bootstrap_key_conversion.rs:294-365):
//   forward                               copy + Plan::fwd                                   (:89-95)
//   forward_normalized                    copy + Plan::fwd + Plan::normalize                 (:97-108)
//   forward_from_power_of_two_modulus     switch 2^w -> p (:166-177), then Plan::fwd          (:201-214)
//   forward_from_decomp                   negative (as i64) x -> x + p wrapping, Plan::fwd    (:221-240)
//   add_backward                          Plan::inv in place, standard = wrapping_add_custom_mod(standard, ntt, p)
//                                                                                             (:110-131)
//   add_backward_on_power_of_two_modulus  Plan::inv in place, ntt = switch p -> 2^w (:184-196, the OR rounding),
//                                         standard += ntt wrapping                             (:244-266)
// Two implementations, one result:
//   * the Solinas N = 2048 plan: the conversions fused into the twisted asm bodies (tools/gen_view_kernel.py ->
//     ntt64_view_body.hpp): one launch, the polynomial crosses HBM once each way; add_backward at w < 64 runs the
//     inverse body in place followed by the generic epilogue below;
//   * every other plan (any N, any NTT prime): an elementwise HBM pass (prologue or epilogue) around the plan's own
//     transform (launch_transform), with the switches in exact 128-bit arithmetic.
// Every output equals the reference's on the same inputs, including the buffer the reference leaves behind: `ntt`
// holds inv(ntt) (switched to 2^w for the power-of-two form) after an add_backward call, as Plan::inv in place.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_tw_device.hpp"
#include "ntt64_view_body.hpp"

namespace mi {
namespace view {

typedef unsigned __int128 u128;

// ---- generic elementwise passes (any plan) --------------------------------------------------------------------

// modswitch_from_power_of_two_to_ntt_prime (ntt64.rs:166-177): the top w bits of x (MSB-aligned), rounded into Z_p
__device__ __forceinline__ u64 pow2_to_p(u64 x, uint32_t w, u64 p) {
  const u128 v = (u128)(x >> (64u - w));
  return (u64)((v * p + ((u128)1 << (w - 1u))) >> w);
}

// modswitch_from_ntt_prime_to_power_of_two (ntt64.rs:184-196): ((v << w) | p >> 1) / p, MSB-aligned (the OR is the
// reference's, not an add: for w < 63 it merges with v's low bits)
__device__ __forceinline__ u64 p_to_pow2(u64 v, uint32_t w, u64 p) {
  const u128 q = (((u128)v << w) | (u128)(p >> 1)) / p;
  return (u64)q << (64u - w);
}

// u64::wrapping_add_custom_mod (commons/numeric/unsigned.rs:174-187, 219-225): a.wrapping_sub_custom_mod(b.neg)
__device__ __forceinline__ u64 add_custom_mod(u64 a, u64 b, u64 p) {
  const u64 nb = b == 0 ? 0 : p - b;
  return a >= nb ? a - nb : a - nb + p;
}

enum : int { PRE_COPY = 0, PRE_POW2 = 1, PRE_DECOMP = 2 };

// ntt[b][i] = conv(standard[b][i]) for the `n` coefficients of each of `batch` polynomials `stride` apart (ntt may
// equal standard)
__global__ void view_pre_kernel(u64* ntt, const u64* standard, size_t n, size_t batch, size_t stride, int kind,
                                uint32_t w, u64 p) {
  const size_t total = n * batch;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const size_t off = (e / n) * stride + e % n;
    u64 x = standard[off];
    if (kind == PRE_POW2) x = pow2_to_p(x, w, p);
    else if (kind == PRE_DECOMP) x = (int64_t)x < 0 ? x + p : x;
    ntt[off] = x;
  }
}

// the add_backward epilogue on the inverse's output: w > 0: ntt = p_to_pow2(ntt), standard += ntt (wrapping);
// w = 0: standard = wrapping_add_custom_mod(standard, ntt, p)
__global__ void view_post_kernel(u64* standard, u64* ntt, size_t n, size_t batch, size_t stride, uint32_t w, u64 p) {
  const size_t total = n * batch;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const size_t off = (e / n) * stride + e % n;
    u64 v = ntt[off];
    if (w) {
      v = p_to_pow2(v, w, p);
      ntt[off] = v;
      standard[off] += v;
    } else {
      standard[off] = add_custom_mod(standard[off], v, p);
    }
  }
}

static unsigned elementwise_grid(size_t total) {
  return (unsigned)std::min<size_t>((total + 255) / 256, (size_t)256 * 64);
}

// ---- the fused twisted N = 2048 bodies ----------------------------------------------------------------------------
// forward: one wave per workgroup (the forward body's measured best, ntt64_tw.hip tw_waves); `twist` = the plan's
// forward table (or its N^-1 rows for forward_normalized), the lane-pair twiddles 2048 entries on
template <int KIND>
__global__ __launch_bounds__(64) void view_fwd_kernel(u64* ntt, const u64* standard, uint32_t batch, uint64_t stride,
                                                      const u64* __restrict__ twist, uint32_t m_lo, uint32_t m_hi) {
  __shared__ u64 lds[tw::WAVE_LDS2];
  const uint32_t lane = threadIdx.x, poly = blockIdx.x;
  if (poly >= batch) return;
  const u64* p = standard + (uint64_t)poly * stride;
  u64* q = ntt + (uint64_t)poly * stride;
  const uint32_t S = (uint32_t)(uintptr_t)lds;
  const uint32_t l8 = lane * 8;
  const tw::FwdAddrs a(S, lane);  // the forward body's W1x transposes (ntt64_tw_device.hpp)
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t olo = (uint32_t)(uintptr_t)q, ohi = (uint32_t)((uintptr_t)q >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2048;
#define MI_VIEW_FWD_OPS                                                                                           \
  [g_lo] "s"(glo), [g_hi] "s"(ghi), [o_lo] "s"(olo), [o_hi] "s"(ohi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi),    \
      [lw] "s"(lw), [l8] "v"(l8), [t1w] "v"(a.t1w), [t1r] "v"(a.t1r), [t2wl] "v"(a.t2wl), [t2wh] "v"(a.t2wh),  \
      [t2r] "v"(a.t2r), [lwo] "v"(a.lwo)
  if constexpr (KIND == PRE_COPY) {
    MI_TW_BODY_FWD_COPY(MI_VIEW_FWD_OPS);
  } else if constexpr (KIND == PRE_POW2) {
    MI_TW_BODY_FWD_POW2(MI_VIEW_FWD_OPS, [m_lo] "s"(m_lo), [m_hi] "s"(m_hi));
  } else {
    MI_TW_BODY_FWD_DECOMP(MI_VIEW_FWD_OPS);
  }
#undef MI_VIEW_FWD_OPS
}

// inverse + add: four waves per workgroup (the inverse body's measured best); `twist` = the plan's inverse table
template <bool POW2_64>
__global__ __launch_bounds__(256) void view_inv_kernel(u64* standard, u64* ntt, uint32_t batch, uint64_t stride,
                                                       const u64* __restrict__ twist) {
  constexpr uint32_t W = 4;
  __shared__ u64 lds[W * tw::WAVE_LDS2];
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t poly = blockIdx.x * W + wv;
  if (poly >= batch) return;
  u64* p = ntt + (uint64_t)poly * stride;
  u64* q = standard + (uint64_t)poly * stride;
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * tw::WAVE_LDS2);
  const uint32_t l8 = lane * 8;
  const tw::InvAddrs a(S, lane);
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t olo = (uint32_t)(uintptr_t)q, ohi = (uint32_t)((uintptr_t)q >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2 * (2048 + 32);  // the last-DIT-stage table (tw_body<false>)
#define MI_VIEW_INV_OPS                                                                                          \
  [g_lo] "s"(glo), [g_hi] "s"(ghi), [o_lo] "s"(olo), [o_hi] "s"(ohi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi),   \
      [lw] "s"(lw), [l8] "v"(l8), [t4w] "v"(a.t4w), [t1x] "v"(a.t1x), [t1y] "v"(a.t1y), [lwo] "v"(a.lwo)
  if constexpr (POW2_64) {
    MI_TW_BODY_INV_ADD64(MI_VIEW_INV_OPS);
  } else {
    MI_TW_BODY_INV_ADDP(MI_VIEW_INV_OPS);
  }
#undef MI_VIEW_INV_OPS
}

}  // namespace view

hipError_t launch_view_pre(int kind, uint64_t* ntt, const uint64_t* standard, size_t n, size_t batch, size_t stride,
                           unsigned width, uint64_t p, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  hipLaunchKernelGGL(view::view_pre_kernel, dim3(view::elementwise_grid(n * batch)), dim3(256), 0, s, ntt, standard, n,
                     batch, stride, kind, (uint32_t)width, p);
  return hipGetLastError();
}

hipError_t launch_view_post(uint64_t* standard, uint64_t* ntt, size_t n, size_t batch, size_t stride, unsigned width,
                            uint64_t p, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  hipLaunchKernelGGL(view::view_post_kernel, dim3(view::elementwise_grid(n * batch)), dim3(256), 0, s, standard, ntt, n,
                     batch, stride, (uint32_t)width, p);
  return hipGetLastError();
}

hipError_t launch_view_fwd_tw(int kind, uint64_t* ntt, const uint64_t* standard, size_t batch, size_t stride,
                              unsigned width, const uint64_t* twist, hipStream_t s) {
  // the mask that clears the low 64 - w bits (forward_from_power_of_two_modulus; all ones at w = 64)
  const uint64_t mask = width >= 64 ? ~0ull : ~((1ull << (64 - width)) - 1);
  constexpr size_t CHUNK = size_t(1) << 30;
  for (size_t off = 0; off < batch; off += CHUNK) {
    const uint32_t n = (uint32_t)std::min(CHUNK, batch - off);
    u64* d = ntt + off * stride;
    const u64* src = standard + off * stride;
    const uint32_t lo = (uint32_t)mask, hi = (uint32_t)(mask >> 32);
    if (kind == view::PRE_COPY)
      hipLaunchKernelGGL(view::view_fwd_kernel<view::PRE_COPY>, dim3(n), dim3(64), 0, s, d, src, n, (uint64_t)stride,
                         twist, lo, hi);
    else if (kind == view::PRE_POW2)
      hipLaunchKernelGGL(view::view_fwd_kernel<view::PRE_POW2>, dim3(n), dim3(64), 0, s, d, src, n, (uint64_t)stride,
                         twist, lo, hi);
    else
      hipLaunchKernelGGL(view::view_fwd_kernel<view::PRE_DECOMP>, dim3(n), dim3(64), 0, s, d, src, n,
                         (uint64_t)stride, twist, lo, hi);
  }
  return hipGetLastError();
}

hipError_t launch_view_inv_tw(bool pow2_64, uint64_t* standard, uint64_t* ntt, size_t batch, size_t stride,
                              const uint64_t* twist, hipStream_t s) {
  constexpr size_t CHUNK = size_t(1) << 30;
  for (size_t off = 0; off < batch; off += CHUNK) {
    const uint32_t n = (uint32_t)std::min(CHUNK, batch - off);
    u64* st = standard + off * stride;
    u64* d = ntt + off * stride;
    if (pow2_64)
      hipLaunchKernelGGL(view::view_inv_kernel<true>, dim3((n + 3) / 4), dim3(256), 0, s, st, d, n, (uint64_t)stride,
                         twist);
    else
      hipLaunchKernelGGL(view::view_inv_kernel<false>, dim3((n + 3) / 4), dim3(256), 0, s, st, d, n,
                         (uint64_t)stride, twist);
  }
  return hipGetLastError();
}

}  // namespace mi
