// Diagnostic (GPU box): the C++ mirror's f64 sequence at one N through the C ABI on the legacy null stream, each stage
// checked on its own: forward_as_torus (vs a second run), to_standard_order (a permutation of it), from_standard_order
// out of place and in place (== the forward output).  ./fftg_rt_probe N reps [keep]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>
#include "tfhe_ntt_amd.h"

static std::vector<double> d2h(const double* p, size_t n) {
  std::vector<double> h(n);
  (void)hipMemcpy(h.data(), p, n * 8, hipMemcpyDeviceToHost);
  return h;
}

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? (size_t)atoll(argv[1]) : 8192, batch = 2, reps = argc > 2 ? (size_t)atoll(argv[2]) : 5;
  // argv[3] == "keep": the default memory pool never releases memory (release threshold UINT64_MAX), so a
  // stream-ordered block is never returned to the runtime's VM heap between reps
  if (argc > 3 && std::string(argv[3]) == "keep") {
    hipMemPool_t mp;
    uint64_t thr = ~0ull;
    if (hipDeviceGetDefaultMemPool(&mp, 0) != hipSuccess || hipMemPoolSetAttribute(mp, hipMemPoolAttrReleaseThreshold, &thr) != hipSuccess)
      std::printf("cannot set the pool's release threshold\n");
  }
  mi_fft64_plan* plan = nullptr;
  if (mi_fft64_plan_create(n, 0, &plan) != 0) { std::printf("plan failed\n"); return 1; }
  std::vector<uint64_t> x(batch * n);
  for (size_t i = 0; i < x.size(); ++i) x[i] = (i + 1) * 0x9E3779B97F4A7C15ull;
  uint64_t* dx = nullptr;
  (void)hipMalloc((void**)&dx, x.size() * 8);
  (void)hipMemcpy(dx, x.data(), x.size() * 8, hipMemcpyHostToDevice);
  int bad_fwd = 0, bad_oop = 0, bad_inp = 0, bad_nan = 0;
  std::vector<double> ref;
  for (size_t r = 0; r < reps; ++r) {
    double *four = nullptr, *nat = nullptr, *back = nullptr;
    (void)hipMalloc((void**)&four, batch * n * 8);
    (void)hipMalloc((void**)&nat, batch * n * 8);
    (void)hipMalloc((void**)&back, batch * n * 8);
    if (mi_fft64_forward_torus_batch(plan, four, dx, batch, nullptr) != 0) std::printf("fwd error\n");
    const auto h0 = d2h(four, batch * n);
    for (double v : h0) bad_nan += std::isnan(v);
    if (ref.empty()) ref = h0; else bad_fwd += h0 != ref;
    if (mi_fft64_to_standard_order(plan, nat, four, batch, nullptr) != 0) std::printf("to_std error\n");
    if (mi_fft64_from_standard_order(plan, back, nat, batch, nullptr) != 0) std::printf("from_std error\n");
    bad_oop += d2h(back, batch * n) != h0;
    if (mi_fft64_from_standard_order(plan, nat, nat, batch, nullptr) != 0) std::printf("from_std in place error\n");
    const bool inp_bad = d2h(nat, batch * n) != h0;
    if (inp_bad) std::fprintf(stderr, "PROBE rep %zu: in-place round trip WRONG\n", r);
    bad_inp += inp_bad;
    (void)hipFree(four); (void)hipFree(nat); (void)hipFree(back);
  }
  std::printf("N=%zu reps=%zu: forward differs %d, out-of-place round trip %d, in-place round trip %d, NaN %d\n", n, reps,
              bad_fwd, bad_oop, bad_inp, bad_nan);
  return 0;
}
