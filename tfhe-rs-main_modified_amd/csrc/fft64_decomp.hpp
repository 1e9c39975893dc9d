// fft64_decomp.hpp — the level-1 decomposition digit of the f64-FFT PBS (fft64_pbs.hip), callable from host
// code so that tests/cpp/fft_decomp_check.cpp can check it exhaustively on the rounding corners.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi {
namespace fft {

// Level-1 signed digit of a native u64 for base_log B <= 31, from the high word alone: the same value as
// decomp_init_native + decompose_one_level in fft64_pbs.hip (decomposer.rs:156-185, iter.rs:131-151).
// With t = the top B + 1 bits (x >> (63 - B)), the reference's digit is the B-bit value ((t + 1) >> 1) mod 2^B
// read as signed (two's complement), except for the one unbalanced tie t = 2^B (binary 10...0), whose digit is
// +2^(B-1) instead of -2^(B-1) (its rounding bit is 0, so need_balance stays 0).  With s = 31 - B:
// (t + 1) >> 1 = (hi + 2^s) >> (s + 1) (a wrap of the 32-bit sum only drops bit B, which the mod 2^B drops too),
// so the digit is one arithmetic shift of hi + 2^s plus the tie select.  Checked against a host restatement
// of the 64-bit functions on the rounding corners by tests/cpp/fft_decomp_check.cpp.
__host__ __device__ __forceinline__ int32_t decompose_l1_hi(uint32_t hi, int base_log) {
  const int s = 31 - base_log;
  const uint32_t f = hi + (1u << s);
  const int32_t d = (int32_t)f >> (s + 1);  // bits [s + 1, 31] of f: the B-bit field, sign-extended
  const bool tie = (hi >> s) == (1u << base_log);
  return tie ? (int32_t)(1u << (base_log - 1)) : d;
}

}  // namespace fft
}  // namespace mi
