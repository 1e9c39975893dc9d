// native_crt.hip — residue split and CRT reconstruction for the exact native-modulus negacyclic
// products of tfhe-ntt (reference paths relative to /root/reference/tfhe-ntt/src):
//   native32.rs:337-500, native64.rs:929-1160, native128.rs:120-320 (Plan32 / Plan52) and the
//   binary-RHS twins native_binary{32,64,128}.rs: value mod p_k per prime, K prime NTTs, pointwise
//   product x N^-1, K inverse NTTs, then a mixed-radix (Garner) reconstruction whose top digit
//   decides the sign (`sign = v_top > p_top / 2`, e.g. native64.rs:66), reduced mod 2^W.
// The transforms themselves run through the prime plans' window kernels (ntt64_kernels.hip); the two
// kernels here are elementwise and HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"

namespace mi {
namespace crt {

// the Montgomery form of prime k (REDC(a b) for any a < 2^64 and b < p_k is canonical: a b < R p_k)
__device__ __forceinline__ Montgomery mont(const CrtConst& c, int k) { return Montgomery{c.p[k], c.pinv[k], c.r2[k]}; }

// x mod p for x < 3p (the CRT primes of one plan lie within a factor of two of each other)
__device__ __forceinline__ u64 fold3(u64 x, u64 p) {
  x = x >= p ? x - p : x;
  return x >= p ? x - p : x;
}

// one coefficient of a width-bit word array (u128 = two little-endian u64 words)
__device__ __forceinline__ unsigned __int128 load_value(const void* in, size_t i, int width) {
  if (width == 32) return ((const uint32_t*)in)[i];
  if (width == 64) return ((const u64*)in)[i];
  const u64* w = (const u64*)in + 2 * i;
  return ((unsigned __int128)w[1] << 64) | w[0];
}

// planes[k * count + i] = value_i mod p_k; `binary`: the binary-RHS split (fwd_binary, e.g.
// native_binary64.rs:371-389) keeps the value truncated to the prime word (u32 for 32-bit primes)
__global__ __launch_bounds__(256) void residue_kernel(u64* __restrict__ planes, const void* __restrict__ in,
                                                      uint64_t count, int width, int binary, CrtConst c) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned __int128 v = load_value(in, i, width);
    if (binary) v = c.prime_bits == 32 ? (unsigned __int128)(uint32_t)v : (unsigned __int128)(u64)v;
    const u64 lo = (u64)v, hi = (u64)(v >> 64);
    for (int k = 0; k < c.k; ++k) {
      const Montgomery m = mont(c, k);
      u64 r = m.mul(lo, c.r1[k]);                       // REDC(lo (R mod p)) = lo mod p
      if (width == 128) r = m.add(r, m.mul(hi, c.r2[k]));  // + REDC(hi R^2) = hi 2^64 mod p
      planes[(uint64_t)k * count + i] = r;
    }
  }
}

__global__ __launch_bounds__(256) void reconstruct_kernel(void* __restrict__ out, const u64* __restrict__ planes,
                                                          uint64_t count, int width, CrtConst c) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    u64 v[MI_CRT_MAX];
    for (int k = 0; k < c.k; ++k) {
      const u64 r = planes[(uint64_t)k * count + i];
      if (k == 0) {
        v[0] = r;
        continue;
      }
      // s = sum_{j<k} v_j prod_{l<j} p_l  mod p_k (Horner from the top digit), in Montgomery products by constants
      const Montgomery m = mont(c, k);
      const u64 pk = c.p[k];
      u64 s = fold3(v[k - 1], pk);
      for (int j = k - 2; j >= 0; --j) s = m.add(m.mul(s, c.pjk_m[j][k]), fold3(v[j], pk));
      const u64 d = r >= s ? r - s : r + pk - s;
      v[k] = m.mul(d, c.inv_prefix_m[k]);
    }
    unsigned __int128 acc = 0;  // sum v_k * prod_{l<k} p_l  mod 2^128
    for (int k = 0; k < c.k; ++k) {
      const unsigned __int128 pre = ((unsigned __int128)c.prefix_hi[k] << 64) | c.prefix_lo[k];
      acc += (unsigned __int128)v[k] * pre;
    }
    if (v[c.k - 1] > c.p[c.k - 1] / 2) acc -= ((unsigned __int128)c.m_hi << 64) | c.m_lo;
    if (width == 32) ((uint32_t*)out)[i] = (uint32_t)acc;
    else if (width == 64) ((u64*)out)[i] = (u64)acc;
    else {
      ((u64*)out)[2 * i] = (u64)acc;
      ((u64*)out)[2 * i + 1] = (u64)(acc >> 64);
    }
  }
}

static unsigned grid_for(uint64_t count) {
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  return (unsigned)(blocks ? blocks : 1);
}

}  // namespace crt

hipError_t launch_crt_residues(uint64_t* planes, const void* in, size_t count, int width, int binary,
                               const CrtConst& c, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(crt::residue_kernel, dim3(crt::grid_for(count)), dim3(256), 0, s, planes, in, (uint64_t)count,
                     width, binary, c);
  return hipGetLastError();
}

hipError_t launch_crt_reconstruct(void* out, const uint64_t* planes, size_t count, int width, const CrtConst& c,
                                  hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(crt::reconstruct_kernel, dim3(crt::grid_for(count)), dim3(256), 0, s, out, planes,
                     (uint64_t)count, width, c);
  return hipGetLastError();
}

}  // namespace mi
