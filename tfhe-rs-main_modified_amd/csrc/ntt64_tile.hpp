// ntt64_tile.hpp — the first top pass of the split transform (stage 0 .. K - 1, K = 4 or 5, Solinas prime) as a
// cooperative tile: a 256-lane workgroup owns 64 columns x 2^K rows of one polynomial (a row is N / 2^K coefficients
// apart), each lane 2^K / 4 rows of its column.  The one-column-per-lane form (ntt_top_kernel, large_rotdec_top)
// holds all 2^K rows of a column in one lane: 32 u64 at K = 5, 90 - 160 VGPRs, and one long load -> compute -> store
// sequence per wave; measured at 2.3 - 3.1 TB/s in the 4_4 blind rotation (profiles/r4/session6/).  Here a lane holds
// 8 (K = 5) or 4 (K = 4) rows and the pass exchanges them once through LDS:
//   phase A: lane (wave w, column c) holds rows w + 4 k: the stages whose butterflies are >= 4 rows apart
//            (s <= K - 3) pair registers k and k + d / 4 of the same lane;
//   phase B: rows 2^(K-2) w + k: the last two stages (2 and 1 rows apart) pair registers k, k + d.
// Forward stages are lazy (Goldilocks::add_lazy / sub_lazy: any 64-bit representative, r5): the callers multiply by
// the block twist (canonical product) or canonicalise before storing.
// The forward runs A, LDS transpose (16 KiB: rows x 64 columns, a wave writes / reads whole 512-B rows: conflict-free),
// B; the inverse B, transpose, A.  Every twiddle of stages 0 .. 4 is a power of two by the Solinas tower
// (tower_exp, Goldilocks::mul_pow2), compile-time in each register because the wave index is a template parameter
// (the kernels switch on it once).  Same values as the column form: bit-exact.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"

namespace mi {
namespace tile {

template <int K>
struct Rows {
  static constexpr int RPT = (1 << K) / 4;                        // rows per lane
  static constexpr int a(int w, int k) { return w + 4 * k; }      // phase A row of register k
  static constexpr int b(int w, int k) { return RPT * w + k; }    // phase B row of register k
};

// stage S of the pass on the lane's registers (row r of register k: phase A or B mapping, wave W)
template <int K, bool FWD, int S, int W, bool PB>
__device__ __forceinline__ void stage(u64 (&x)[Rows<K>::RPT]) {
  constexpr int RPT = Rows<K>::RPT, d = 1 << (K - 1 - S), dk = PB ? d : d / 4;
  static_assert(PB ? (d <= 2) : (d >= 4), "stage in the wrong phase");
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    if (k & dk) continue;
    const int row = PB ? Rows<K>::b(W, k) : Rows<K>::a(W, k);
    const int ex = tower_exp(FWD, S, row >> (K - S));
    bool ng;
    if (FWD) {  // lazy: outputs congruent mod p, any 64-bit value (z canonical; the callers canonicalise or multiply)
      const u64 z = Goldilocks::mul_pow2(x[k + dk], ex, ng);
      const u64 u = x[k];
      x[k] = ng ? Goldilocks::sub_lazy(u, z) : Goldilocks::add_lazy(u, z);
      x[k + dk] = ng ? Goldilocks::add_lazy(u, z) : Goldilocks::sub_lazy(u, z);
    } else {  // (a - b) w = (b - a) |w| for a negative w
      const u64 u = x[k], v = x[k + dk];
      x[k] = Goldilocks::add(u, v);
      x[k + dk] = Goldilocks::mul_pow2(ex >= 96 ? Goldilocks::sub(v, u) : Goldilocks::sub(u, v), ex, ng);
    }
  }
}

// the phase-A stages (0 .. K - 3) in order (FWD) or reverse (inverse), then the phase-B ones likewise
template <int K, bool FWD, int W>
__device__ __forceinline__ void phase_a(u64 (&x)[Rows<K>::RPT]) {
  if constexpr (FWD) {
    stage<K, true, 0, W, false>(x);
    stage<K, true, 1, W, false>(x);
    if constexpr (K == 5) stage<K, true, 2, W, false>(x);
  } else {
    if constexpr (K == 5) stage<K, false, 2, W, false>(x);
    stage<K, false, 1, W, false>(x);
    stage<K, false, 0, W, false>(x);
  }
}

template <int K, bool FWD, int W>
__device__ __forceinline__ void phase_b(u64 (&x)[Rows<K>::RPT]) {
  if constexpr (FWD) {
    stage<K, true, K - 2, W, true>(x);
    stage<K, true, K - 1, W, true>(x);
  } else {
    stage<K, false, K - 1, W, true>(x);
    stage<K, false, K - 2, W, true>(x);
  }
}

// registers of phase `from` -> registers of the other phase through the workgroup's 2^K x 64 LDS tile
// (barrier before the writes too: the tile may still be read by the previous use)
template <int K, int W, bool A_TO_B>
__device__ __forceinline__ void exchange(u64 (&x)[Rows<K>::RPT], u64* lds, uint32_t c) {
  constexpr int RPT = Rows<K>::RPT;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RPT; ++k) lds[(A_TO_B ? Rows<K>::a(W, k) : Rows<K>::b(W, k)) * 64 + c] = x[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < RPT; ++k) x[k] = lds[(A_TO_B ? Rows<K>::b(W, k) : Rows<K>::a(W, k)) * 64 + c];
}

}  // namespace tile
}  // namespace mi
