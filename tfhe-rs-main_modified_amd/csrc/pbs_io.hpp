// pbs_io.hpp — where a bootstrap's accumulator starts and what it leaves, shared by every PBS engine (NTT: pbs_tw.hip,
// pbs_kernels.hip, pbs_large.hip; f64: fft64_pbs.hip, fft64_generic.hip) and the C ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mi {

// The accumulator of item b starts as GLWE `lut_for(b)` of the list `lut` (glwe_len u64 each):
//   lut_idx != NULL : GLWE lut_idx[b]; an index >= n_lut skips the item (nothing read, nothing written)
//   per_item != 0   : GLWE b (blind_rotate_*_assign: every item rotates its own accumulator; the f64 path's
//                     batch_programmable_bootstrap_lwe_ciphertext_mem_optimized, fft64_pbs.rs:1055-1127)
//   otherwise       : GLWE 0, shared by the batch (programmable_bootstrap_*_lwe_ciphertext)
// glwe_out != NULL: the rotated accumulator of item b is stored to glwe_out[b] ((k+1) N u64; it may be the LUT list
// itself, in place) instead of extracting sample 0 into lwe_out[b].  Item indices are global to the caller's batch.
struct PbsIo {
  const uint64_t* lut = nullptr;
  const uint32_t* lut_idx = nullptr;
  uint32_t n_lut = 1;
  uint32_t per_item = 0;
  uint64_t* glwe_out = nullptr;
  __host__ __device__ const uint64_t* lut_for(uint64_t b, uint64_t glwe_len) const {
    uint64_t i = per_item ? b : 0;
    if (lut_idx) {
      i = lut_idx[b];
      if (i >= n_lut) return nullptr;
    }
    return lut + i * glwe_len;
  }
};

}  // namespace mi
