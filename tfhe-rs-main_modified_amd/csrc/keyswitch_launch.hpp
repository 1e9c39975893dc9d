// keyswitch_launch.hpp — host entry points of keyswitch.hip (kept out of ntt64_launch.hpp, which every kernel
// source includes).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mi {

// keyswitch.hip — native-modulus LWE keyswitch on the int8 matrix cores.
size_t ks_key_bytes(size_t in_dim, size_t out_dim, int base_log, int level);
size_t ks32_key_bytes(size_t in_dim, size_t out_dim, int base_log, int level);  // the 4-plane KS32 layout
int ks_digit_bytes_per_term(int base_log);  // signed bytes per decomposition digit
size_t ks_digit_bytes(size_t in_dim, int base_log, int level, size_t batch);
hipError_t launch_ksk_prepare(void* frag, const uint64_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                              hipStream_t s);
hipError_t launch_keyswitch(uint64_t* out, const uint64_t* lwe_in, const void* frag, void* digits, size_t batch,
                            size_t in_dim, size_t out_dim, int base_log, int level, hipStream_t s);
// KS32 (keyswitch_lwe_ciphertext_with_scalar_change, lwe_keyswitch.rs:331-447): u32 key words, u32 outputs of modulus
// 2^out_log (1 <= out_log <= 32), the same digit / GEMM path as the native keyswitch
hipError_t launch_ksk32_prepare(void* frag, const uint32_t* ksk, size_t in_dim, size_t out_dim, int base_log,
                                int level, hipStream_t st);
hipError_t launch_keyswitch32(uint32_t* out, const uint64_t* lwe_in, const void* frag, void* digits, size_t batch,
                              size_t in_dim, size_t out_dim, int base_log, int level, int out_log, hipStream_t st);
// the (centered binary) modulus switch of u32 LWEs of dimension dim to [0, 2^log_mod): (dim + 1) u64 per ciphertext
hipError_t launch_lwe_ms32(uint64_t* out, const uint32_t* in, size_t dim, size_t batch, int log_mod, bool centered,
                           hipStream_t st);
// the same for u64 LWEs (the native-modulus ciphertexts): (dim + 1) u64 per ciphertext in [0, 2^log_mod)
hipError_t launch_lwe_ms64(uint64_t* out, const uint64_t* in, size_t dim, size_t batch, int log_mod, bool centered,
                           hipStream_t st);

}  // namespace mi
