// fft64_decomp.hpp — the level-1 decomposition digit of the f64-FFT PBS (fft64_pbs.hip), callable from host
// code so that tests/cpp/fft_decomp_check.cpp can check it exhaustively on the rounding corners.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi {
namespace fft {

// Level-1 signed digit of a native u64 for base_log B <= 31, from the high word alone: the same value as
// decomp_init_native + decompose_one_level in fft64_pbs.hip (decomposer.rs:156-185, iter.rs:131-151), restated on the
// top B + 1 bits t: res = ((t + 1) >> 1) mod 2^B, then digit = res - 2^B when res > 2^(B-1), or res = 2^(B-1)
// with the rounding bit set (the reference's need_balance / carry), else res.  Checked against a host
// restatement of the 64-bit functions on the rounding corners by tests/cpp/fft_decomp_check.cpp.
__host__ __device__ __forceinline__ int32_t decompose_l1_hi(uint32_t hi, int base_log) {
  const uint32_t t = hi >> (31 - base_log);
  const uint32_t res = ((t + 1u) >> 1) & ((1u << base_log) - 1u);
  const uint32_t half = 1u << (base_log - 1);
  const bool neg = res + (t & 1u) > half;
  return (int32_t)(neg ? res - (1u << base_log) : res);
}

}  // namespace fft
}  // namespace mi
