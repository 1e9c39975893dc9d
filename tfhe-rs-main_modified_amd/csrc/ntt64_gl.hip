// ntt64_gl.hip — persistent, software-pipelined Goldilocks NTT (p = 2^64 - 2^32 + 1) for MI355X.
//
// Same transform as ntt64_kernels.hip (reference: tfhe-ntt/src/prime64/generic_solinas.rs
// fwd 449-481 / inv 483-514, twiddle tables prime64.rs:159-204), restructured for throughput:
//
//  * persistent grid (a few workgroups per CU) walking the batch; the plan's twiddle table is
//    staged into LDS once per workgroup and read from there by every polynomial;
//  * software pipelining: the next polynomial's coefficients are loaded into a second register
//    set while the current one is transformed, so HBM traffic overlaps the VALU-bound butterflies
//    (measured v1 ran memory and compute phases back to back);
//  * register windows of E = 2^LOGE coefficients per lane, LDS transposes between windows
//    (XOR-swizzled image, no padding);
//  * all arithmetic canonical, so the result is bit-identical to the reference.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"

namespace mi {
namespace gl {

template <int LOGN_, int LOGE_>
struct Geo {
  static constexpr int LOGN = LOGN_;
  static constexpr int LOGE = LOGE_;
  static constexpr int N = 1 << LOGN;
  static constexpr int E = 1 << LOGE;
  static constexpr int LOGT = LOGN - LOGE;
  static constexpr int T = 1 << LOGT;  // lanes per polynomial
  static constexpr int NFULL = LOGN / LOGE;
  static constexpr int REM = LOGN % LOGE;
  static constexpr int NWIN = NFULL + (REM ? 1 : 0);
  static_assert(T >= 64 && T <= 1024, "one polynomial per workgroup, whole waves");
};

// LDS image of one polynomial: element e at u64 slot e ^ (((e >> SA) & 15) << 1), a bijection.
// Chosen by an exhaustive search over XOR swizzles (bank model of MI355X_MICROARCH.md §LDS:
// ds_read_b64 = 2 groups of 32 lanes over 32 u64 slots, ds_write_b64 = 4 groups of 16 over 16):
// 1.11x the conflict-free cycle count for E = 8 (SA = 4), 1.17x for E = 16 (SA = 5), vs 3.2x/4.3x
// for the plain layout.
template <int SA>
__device__ __forceinline__ int lds_slot(int e) { return e ^ (((e >> SA) & 15) << 1); }

template <class G>
__device__ __forceinline__ int elem(int t, int r, int lo) {
  return ((t >> lo) << (lo + G::LOGE)) | (r << lo) | (t & ((1 << lo) - 1));
}

template <class G, bool FWD>
__device__ __forceinline__ constexpr int win_lo(int w) {
  if (FWD) return (w < G::NFULL) ? G::LOGN - G::LOGE * (w + 1) : 0;
  return (w < G::NFULL) ? G::LOGE * w : G::LOGN - G::LOGE;
}

template <class G, bool FWD>
__device__ __forceinline__ void butterflies(u64 (&x)[G::E], int t, int w, const u64* __restrict__ tw_lds) {
  const int lo = win_lo<G, FWD>(w);
  int rb_first, rb_last;
  if (w < G::NFULL) { rb_first = 0; rb_last = G::LOGE - 1; }
  else if (FWD) { rb_first = 0; rb_last = G::REM - 1; }
  else { rb_first = G::LOGE - G::REM; rb_last = G::LOGE - 1; }
#pragma unroll
  for (int s = 0; s < G::LOGE; ++s) {
    const int rb = FWD ? (G::LOGE - 1 - s) : s;
    if (rb < rb_first || rb > rb_last) continue;
    const int b = lo + rb;
    const int m = 1 << (G::LOGN - 1 - b);
    const int half = 1 << rb;
    const int tpart = (t >> lo) << (G::LOGE - rb - 1);
    u64 wv[G::E / 2];
#pragma unroll
    for (int j = 0; j < (G::E >> (rb + 1)); ++j) wv[j] = tw_lds[m + (tpart | j)];
#pragma unroll
    for (int r0 = 0; r0 < G::E; ++r0) {
      if (r0 & half) continue;
      const int r1 = r0 | half;
      const u64 w1 = wv[r0 >> (rb + 1)];
      if (FWD) {
        const u64 z1w = Goldilocks::mul(x[r1], w1);
        const u64 a = x[r0];
        x[r0] = Goldilocks::add(a, z1w);
        x[r1] = Goldilocks::sub(a, z1w);
      } else {
        const u64 a = x[r0], bb = x[r1];
        x[r0] = Goldilocks::add(a, bb);
        x[r1] = Goldilocks::mul(Goldilocks::sub(a, bb), w1);
      }
    }
  }
}

template <class G, bool FWD>
__global__ __launch_bounds__(G::T) void ntt_gl_persistent(u64* __restrict__ data, uint32_t batch, uint64_t stride,
                                                         const u64* __restrict__ tw) {
  __shared__ u64 tw_lds[G::N];
  __shared__ u64 xch[G::N];
  const int t = threadIdx.x;
  for (int i = t; i < G::N; i += G::T) tw_lds[i] = tw[i];

  const int lo0 = win_lo<G, FWD>(0);
  const int loL = win_lo<G, FWD>(G::NWIN - 1);
  uint32_t poly = blockIdx.x;
  u64 x[G::E], y[G::E];
  if (poly < batch) {
    const u64* src = data + (uint64_t)poly * stride;
#pragma unroll
    for (int r = 0; r < G::E; ++r) y[r] = src[elem<G>(t, r, lo0)];
  }
  __syncthreads();  // twiddles staged

  for (; poly < batch; poly += gridDim.x) {
#pragma unroll
    for (int r = 0; r < G::E; ++r) x[r] = y[r];
    const uint32_t next = poly + gridDim.x;
    if (next < batch) {  // prefetch the next polynomial while this one is transformed
      const u64* src = data + (uint64_t)next * stride;
#pragma unroll
      for (int r = 0; r < G::E; ++r) y[r] = src[elem<G>(t, r, lo0)];
    }
#pragma unroll
    for (int w = 0; w < G::NWIN; ++w) {
      if (w > 0) {
        const int lo_prev = win_lo<G, FWD>(w - 1), lo = win_lo<G, FWD>(w);
#pragma unroll
        for (int r = 0; r < G::E; ++r) xch[lds_slot<G::LOGE + 1>(elem<G>(t, r, lo_prev))] = x[r];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < G::E; ++r) x[r] = xch[lds_slot<G::LOGE + 1>(elem<G>(t, r, lo))];
        __syncthreads();
      }
      butterflies<G, FWD>(x, t, w, tw_lds);
    }
    u64* dst = data + (uint64_t)poly * stride;
#pragma unroll
    for (int r = 0; r < G::E; ++r) dst[elem<G>(t, r, loL)] = x[r];
  }
}

template <int LOGN, int LOGE, bool FWD>
static hipError_t launch(u64* data, size_t batch, size_t stride, const u64* tw, hipStream_t s, int wg_per_cu) {
  using G = Geo<LOGN, LOGE>;
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  size_t grid = (size_t)cus * wg_per_cu;
  if (grid > batch) grid = batch;
  hipLaunchKernelGGL((ntt_gl_persistent<G, FWD>), dim3((unsigned)grid), dim3(G::T), 0, s, data, (uint32_t)batch,
                     (uint64_t)stride, tw);
  return hipGetLastError();
}

}  // namespace gl

// Goldilocks persistent path; returns hipErrorInvalidValue for sizes it does not cover.
hipError_t launch_ntt_gl(bool fwd, int logn, int variant, uint64_t* data, size_t batch, size_t stride,
                         const uint64_t* tw, hipStream_t s) {
  const int wg = 4;
  if (logn == 11) {
    if (variant == 3) return fwd ? gl::launch<11, 4, true>(data, batch, stride, tw, s, wg)
                                 : gl::launch<11, 4, false>(data, batch, stride, tw, s, wg);
    return fwd ? gl::launch<11, 3, true>(data, batch, stride, tw, s, wg)
               : gl::launch<11, 3, false>(data, batch, stride, tw, s, wg);
  }
  return hipErrorInvalidValue;
}

}  // namespace mi
