// CPU-only check of the C++ mirror's NTT-BSK serialiser (include/tfhe_ntt_amd.hpp) against the Python
// one: reads a serialised key on stdin, deserialises it, re-serialises it and writes the bytes to
// stdout; prints the fields on stderr.  No GPU and no engine library needed.
#include <cstdio>
#include <iostream>
#include <iterator>
#include <vector>

#include "tfhe_ntt_amd.hpp"

int main() {
  std::vector<uint8_t> in((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
  std::vector<uint64_t> data;
  try {
    const auto f = tfhe_ntt_amd::core_crypto::deserialize_ntt_bsk(in.data(), in.size(), data);
    std::fprintf(stderr, "%llu %llu %llu %llu %llu\n", (unsigned long long)f.polynomial_size,
                 (unsigned long long)f.glwe_size, (unsigned long long)f.level, (unsigned long long)f.base_log,
                 (unsigned long long)f.input_lwe_dimension);
    const auto out = tfhe_ntt_amd::core_crypto::serialize_ntt_bsk(data.data(), data.size(), f);
    std::fwrite(out.data(), 1, out.size(), stdout);
  } catch (const std::invalid_argument& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 3;
  }
  return 0;
}
