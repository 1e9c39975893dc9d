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

// Per-lane addresses of the forward body's transposes in its W1x layout (tools/gen_tw_kernel.py FWD_W1X: the lane pair
// of block i is lanes i and i + 32): T1 rows of 33 u64, T2 rows of 65 u64 with the column swizzle c ^ (c >> 5), the
// lane-pair twiddles 16 entries on for the upper half-wave.
struct FwdAddrs {
  uint32_t t1w, t1r, lwo, t2wl, t2wh, t2r;
  __device__ __forceinline__ FwdAddrs(uint32_t S, uint32_t lane) {
    const uint32_t par = lane >> 5, i = lane & 31;
    t1w = S + (lane & 31) * 8;
    t1r = S + (i * 33 + par) * 8;
    lwo = par * 128;
    t2wl = S + ((i & 15) * 65 + 33 * par) * 8;
    t2wh = S + ((i & 15) * 65 + 31 * par + 1) * 8;
    t2r = S + (lane ^ (lane >> 5)) * 8;
  }
};

// Per-lane addresses of the inverse bodies' W1'' transposes in the same W1x lane map (INV_W1X: the pair bit j5 on
// lane bit 5): t1x the W0 side, t1y / t4w the W1'' side (rows of 66 / 65 u64), the last-DIT-stage table 16 entries on
// for the upper half-wave.
struct InvAddrs {
  uint32_t lwo, t4w, t1x, t1y;
  __device__ __forceinline__ InvAddrs(uint32_t S, uint32_t lane) {
    const uint32_t par = lane >> 5, i = lane & 31;
    lwo = par * 128;
    t4w = S + ((i & 15) * 65 + par) * 8;
    t1x = S + (lane + (lane >> 5)) * 8;
    t1y = S + ((i & 15) * 66 + 33 * par) * 8;
  }
};

// One wave's 2048-coefficient body (load -> all stages -> store, in place at p) on its LDS slice S.
template <bool FWD>
__device__ __forceinline__ void tw_body(u64* p, const u64* __restrict__ twist, uint32_t S, uint32_t lane) {
  const uint32_t l8 = lane * 8;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  // forward: the lane-pair twiddles follow the twist rows; inverse: the last-DIT-stage table, two regions on
  // (the plan's allocation: [fwd + 32 | inverse + 32 | inverse N^-1 + 32 | 32], `twist` = the inverse region)
  const u64* lw = FWD ? twist + 2048 : twist + 2 * (2048 + 32);
  if constexpr (FWD) {
    const FwdAddrs a(S, lane);
    MI_TW_BODY_FWD([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(a.t1w), [t1r] "v"(a.t1r), [t2wl] "v"(a.t2wl), [t2wh] "v"(a.t2wh),
                   [t2r] "v"(a.t2r), [lwo] "v"(a.lwo));
  } else {
    const InvAddrs a(S, lane);
    MI_TW_BODY_INV([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t4w] "v"(a.t4w), [t1x] "v"(a.t1x), [t1y] "v"(a.t1y), [lwo] "v"(a.lwo));
  }
}

}  // namespace tw
}  // namespace mi
