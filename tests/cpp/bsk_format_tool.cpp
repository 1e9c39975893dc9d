// CPU-only check of the library's NTT-BSK parser / writer (mi_ntt_bsk_*, through the C++ mirror in
// include/tfhe_ntt_amd.hpp) against the Python one: reads a serialised key on stdin (argv[1] = "1" for
// the versioned form), deserialises it, re-serialises it and writes the bytes to stdout; prints the
// fields on stderr.  No GPU needed (the format calls are host-only).
#include <cstdio>
#include <iostream>
#include <iterator>
#include <vector>

#include "tfhe_ntt_amd.hpp"

int main(int argc, char** argv) {
  const int format = argc > 1 && argv[1][0] == '1' ? MI_NTT_BSK_VERSIONED : MI_NTT_BSK_PLAIN;
  std::vector<uint8_t> in((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
  std::vector<uint64_t> data;
  try {
    const auto f = tfhe_ntt_amd::core_crypto::deserialize_ntt_bsk(in.data(), in.size(), data, format);
    std::fprintf(stderr, "%llu %llu %llu %llu %llu\n", (unsigned long long)f.polynomial_size,
                 (unsigned long long)f.glwe_size, (unsigned long long)f.level, (unsigned long long)f.base_log,
                 (unsigned long long)f.input_lwe_dimension);
    const auto out = tfhe_ntt_amd::core_crypto::serialize_ntt_bsk(data.data(), data.size(), f, format);
    std::fwrite(out.data(), 1, out.size(), stdout);
  } catch (const std::invalid_argument& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 3;
  }
  return 0;
}
