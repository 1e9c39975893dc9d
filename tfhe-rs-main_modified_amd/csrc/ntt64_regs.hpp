// ntt64_regs.hpp — device building blocks: an N-point negacyclic NTT held in the registers of one
// workgroup (E = 2^LOGE coefficients per lane), transposed through LDS between register windows.
//
// Semantics (reference paths relative to /root/reference/tfhe-ntt/src):
//   forward = generic_solinas.rs:449-481 (CT, twid[m + i], natural in / bit-reversed out)
//   inverse = generic_solinas.rs:483-514 (GS, inv_twid[m + i], bit-reversed in / natural out)
// Layout contract (element index e of the polynomial, lane t, register r):
//   fwd entry / inv exit :  e = elem(t, r, LOGN - LOGE)   ("column" layout: e = r * T + t)
//   fwd exit  / inv entry :  e = elem(t, r, 0) for LOGN % LOGE == 0, else the last window's layout
// so a forward transform's output can feed an inverse transform without any data movement.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "mi_arith.hpp"

namespace mi {

template <int LOGN_, int LOGE_>
struct Geo {
  static constexpr int LOGN = LOGN_;
  static constexpr int LOGE = LOGE_;
  static constexpr int N = 1 << LOGN;
  static constexpr int E = 1 << LOGE;
  static constexpr int LOGT = LOGN - LOGE;  // lanes per polynomial = 2^LOGT
  static constexpr int T = 1 << LOGT;
  static constexpr int PPW = T >= 64 ? 1 : 64 / T;  // polynomials per workgroup
  static constexpr int THREADS = T * PPW;
  static constexpr int NFULL = LOGN / LOGE;
  static constexpr int REM = LOGN % LOGE;
  static constexpr int NWIN = NFULL + (REM ? 1 : 0);
  // LDS image: 4 u64 of padding per 32 (keeps the strided window reads off shared banks)
  static constexpr int PADDED = N + (N >> 3);
  static_assert(LOGN >= LOGE, "window wider than the transform");
  static_assert(THREADS <= 1024, "workgroup too large");
};

__device__ __forceinline__ int lds_addr(int e) { return e + ((e >> 5) << 2); }

template <class G>
__device__ __forceinline__ int elem(int t, int r, int lo) {
  return ((t >> lo) << (lo + G::LOGE)) | (r << lo) | (t & ((1 << lo) - 1));
}

// low bit of register window w
template <class G, bool FWD>
__host__ __device__ __forceinline__ constexpr int win_lo(int w) {
  if (FWD) return (w < G::NFULL) ? G::LOGN - G::LOGE * (w + 1) : 0;
  return (w < G::NFULL) ? G::LOGE * w : G::LOGN - G::LOGE;
}

// `twc` (SUB only): the transform is block b of 2^k blocks left by k top stages of a larger one
// (large-N plans): its stage with m groups reads the big table at m * twc + g, twc = 2^k + b, because
// the big stage has m 2^k groups and block b owns groups [b m, (b + 1) m).
// Solinas prime (Mod = Goldilocks): the reference's stages with m < 32 groups use the tower's power-of-two twiddles
// (entry m + g = 2^tower_exp(log2 m, g), every Goldilocks plan, prime64.rs:166-177); where the window also leaves the
// group index compile-time (the lanes' bits lie below the window: lo >= LOGT, the first forward / last inverse
// window) the multiply is a shift (Goldilocks::mul_pow2) instead of a table load and a four-limb product.
// LAZY (forward, Goldilocks only, r5): the butterflies' outputs are any 64-bit representatives (Goldilocks::add_lazy /
// sub_lazy against the canonical product), for consumers that reduce anyway (the shape kernels' MAC, pbs::Acc128)
template <class G, bool FWD, class Mod, bool SUB = false, bool LAZY = false>
__device__ __forceinline__ void window_butterflies(u64 (&x)[G::E], int t, int w, const u64* __restrict__ tw,
                                                   const Mod& mod, uint32_t twc = 1) {
  constexpr bool lazy = LAZY && FWD && std::is_same<Mod, Goldilocks>::value;
  const int lo = win_lo<G, FWD>(w);
  int rb_first, rb_last;  // r-bits of this window that still need a stage
  if (w < G::NFULL) { rb_first = 0; rb_last = G::LOGE - 1; }
  else if (FWD) { rb_first = 0; rb_last = G::REM - 1; }
  else { rb_first = G::LOGE - G::REM; rb_last = G::LOGE - 1; }

#pragma unroll
  for (int s = 0; s < G::LOGE; ++s) {
    const int rb = FWD ? (G::LOGE - 1 - s) : s;
    if (rb < rb_first || rb > rb_last) continue;
    const int b = lo + rb;                 // butterfly bit of the element index
    const int m = 1 << (G::LOGN - 1 - b);  // reference's `m` for this stage
    const int half = 1 << rb;
    const int tpart = (t >> lo) << (G::LOGE - rb - 1);
#pragma unroll
    for (int r0 = 0; r0 < G::E; ++r0) {
      if (r0 & half) continue;
      const int r1 = r0 | half;
      if (std::is_same<Mod, Goldilocks>::value && !SUB && m < 32 && lo >= G::LOGT) {
        const int s_ref = G::LOGN - 1 - b, ex = tower_exp(FWD, s_ref, r0 >> (rb + 1));  // (t >> lo) == 0 here
        bool ng;
        if (FWD && lazy) {
          const u64 z = Goldilocks::mul_pow2(x[r1], ex, ng);
          const u64 a = x[r0];
          x[r0] = ng ? Goldilocks::sub_lazy(a, z) : Goldilocks::add_lazy(a, z);
          x[r1] = ng ? Goldilocks::add_lazy(a, z) : Goldilocks::sub_lazy(a, z);
        } else if (FWD) {
          const u64 z = Goldilocks::mul_pow2(x[r1], ex, ng);
          const u64 a = x[r0];
          x[r0] = ng ? Goldilocks::sub(a, z) : Goldilocks::add(a, z);
          x[r1] = ng ? Goldilocks::add(a, z) : Goldilocks::sub(a, z);
        } else {  // (a - b) w = (b - a) |w| for a negative w
          const u64 a = x[r0], bb = x[r1];
          x[r0] = Goldilocks::add(a, bb);
          x[r1] = Goldilocks::mul_pow2(ex >= 96 ? Goldilocks::sub(bb, a) : Goldilocks::sub(a, bb), ex, ng);
        }
        continue;
      }
      const u64 wv = tw[(SUB ? m * twc : m) + (tpart | (r0 >> (rb + 1)))];
      if constexpr (lazy) {
        const u64 z1w = Goldilocks::mul(x[r1], wv);  // any x: a canonical product
        const u64 a = x[r0];
        x[r0] = Goldilocks::add_lazy(a, z1w);
        x[r1] = Goldilocks::sub_lazy(a, z1w);
      } else if (FWD) {
        const u64 z1w = mod.mul(x[r1], wv);
        const u64 a = x[r0];
        x[r0] = mod.add(a, z1w);
        x[r1] = mod.sub(a, z1w);
      } else {
        const u64 a = x[r0], bb = x[r1];
        x[r0] = mod.add(a, bb);
        x[r1] = mod.mul(mod.sub(a, bb), wv);
      }
    }
  }
}

// LDS transpose between windows w-1 and w.  `sh` = PADDED u64 of this polynomial's scratch.
// Barriers are the caller's responsibility when several polynomials share barriers.
template <class G, bool FWD>
__device__ __forceinline__ void window_store(const u64 (&x)[G::E], int t, int w, u64* sh) {
  const int lo = win_lo<G, FWD>(w);
#pragma unroll
  for (int r = 0; r < G::E; ++r) sh[lds_addr(elem<G>(t, r, lo))] = x[r];
}
template <class G, bool FWD>
__device__ __forceinline__ void window_load(u64 (&x)[G::E], int t, int w, const u64* sh) {
  const int lo = win_lo<G, FWD>(w);
#pragma unroll
  for (int r = 0; r < G::E; ++r) x[r] = sh[lds_addr(elem<G>(t, r, lo))];
}

// Whole transform of NP polynomials (registers x[p]) sharing barriers; sh has NP * PADDED u64.
// Entry: layout of window 0; exit: layout of the last window.  Contains __syncthreads().
template <class G, bool FWD, int NP, class Mod, bool LAZY = false>
__device__ __forceinline__ void ntt_regs(u64 (&x)[NP][G::E], int t, u64* sh, const u64* __restrict__ tw,
                                         const Mod& mod) {
#pragma unroll
  for (int w = 0; w < G::NWIN; ++w) {
    if (w > 0) {
#pragma unroll
      for (int p = 0; p < NP; ++p) window_store<G, FWD>(x[p], t, w - 1, sh + p * G::PADDED);
      __syncthreads();
#pragma unroll
      for (int p = 0; p < NP; ++p) window_load<G, FWD>(x[p], t, w, sh + p * G::PADDED);
      __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) window_butterflies<G, FWD, Mod, false, LAZY>(x[p], t, w, tw, mod);
  }
}

}  // namespace mi
