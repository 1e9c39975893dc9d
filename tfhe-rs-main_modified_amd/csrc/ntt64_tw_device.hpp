// ntt64_tw_device.hpp — one wave's twisted N = 2048 Goldilocks body (tools/gen_tw_kernel.py -> ntt64_tw_body.hpp) as a
// device function, for the kernels that run it (ntt64_tw.hip: the transform, the key conversion and the one-launch
// split transform, whose bodies run on blocks the same workgroup just wrote).
// The body owns v8..v127 / s20..s99 and does load -> all stages -> store in place at p; the caller gives it the
// wave's LDS slice (WAVE_LDS2 u64) and the plan's twist table.  ntt64_tw.hip's header comment has the layouts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"
#include "ntt64_tw_body.hpp"

namespace mi {
namespace tw {

static constexpr int WAVE_LDS2 = 1088;  // u64: max(32 x 34, 16 x 66)

// One wave's 2048-coefficient body (load -> all stages -> store, in place at p) on its LDS slice S.
template <bool FWD>
__device__ __forceinline__ void tw_body(u64* p, const u64* __restrict__ twist, uint32_t S, uint32_t lane) {
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

}  // namespace tw
}  // namespace mi
