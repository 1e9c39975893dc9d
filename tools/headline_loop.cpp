// headline_loop.cpp — the bench headline's transform launches without Python or torch, for rocprofv3 --pmc passes
// (the profiler's counter passes crash the host inside the python bench process on this image; this loop runs the
// same library entry points: mi_ntt64_fwd_batch / mi_ntt64_inv_batch on a resident 8192 x 2048 batch, config 2).
//   g++ -O2 -std=c++17 -I include tools/headline_loop.cpp -o tools/headline_loop \
//       -L tfhe-rs-main_modified_amd/tfhe_ntt_amd -ltfhe_ntt_amd -Wl,-rpath,'$ORIGIN/../tfhe-rs-main_modified_amd/tfhe_ntt_amd' \
//       -I /opt/rocm/include -L /opt/rocm/lib -lamdhip64 -D__HIP_PLATFORM_AMD__
//   tools/headline_loop [steps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "tfhe_ntt_amd.h"

#define CK(x)                                                                 \
  do {                                                                        \
    int e_ = (int)(x);                                                        \
    if (e_ != 0) {                                                            \
      std::fprintf(stderr, "%s:%d status %d\n", __FILE__, __LINE__, e_);      \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int steps = argc > 1 ? std::atoi(argv[1]) : 20;
  const size_t n = 2048, batch = 8192;
  const uint64_t p = 0xFFFFFFFF00000001ull;
  mi_ntt64_plan* plan = nullptr;
  CK(mi_ntt64_plan_create(n, p, 0, &plan));
  uint64_t* buf = nullptr;
  CK(hipMalloc(&buf, n * batch * sizeof(uint64_t)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(mi_fill_uniform(buf, n * batch, 0x74666867ull, p, 0, s));
  for (int i = 0; i < steps; ++i) {
    CK(mi_ntt64_fwd_batch(plan, buf, batch, n, s));
    CK(mi_ntt64_inv_batch(plan, buf, batch, n, s));
  }
  CK(hipStreamSynchronize(s));
  std::printf("headline_loop: %d fwd+inv steps over %zu x %zu done\n", steps, batch, n);
  CK(hipFree(buf));
  CK(hipStreamDestroy(s));
  CK(mi_ntt64_plan_destroy(plan));
  return 0;
}
