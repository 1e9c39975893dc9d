// key_alias_probe.hip — diagnostic build (not part of the library); see tools/key_alias_probe.py.
// Times the BNF level-1 NTT PBS body walking a real 918-step key against the same body with the key
// advance set to 0 (every step reads one 64 KiB GGSW), batch 4096, random inputs.  One JSON line.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "mi_arith.hpp"
#include "pbs_tw_body.hpp"
#include "_pbs_alias_body.hpp"

using mi::u64;
static constexpr int N = 2048;

template <bool ALIAS>
__global__ __launch_bounds__(128) void probe_pbs(const u64* __restrict__ lwe_in, const u64* __restrict__ lut,
                                                 const u64* __restrict__ bsk, uint32_t n_lwe, uint32_t batch,
                                                 int base_log, const u64* __restrict__ tab, u64* __restrict__ sink) {
  __shared__ u64 buf[2 * N];
  __shared__ u64 lwtab[64];
  const int t = threadIdx.x;
  const uint32_t lane = t & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(t >> 6);
  const uint32_t b = blockIdx.x;
  if (b >= batch) return;
  const u64* lwe = lwe_in + (size_t)b * (n_lwe + 1);
  if (t < 64) lwtab[t] = t < 32 ? tab[N + t] : tab[2 * N + 32 + (t - 32)];
  __syncthreads();
  const uint32_t S = (uint32_t)(uintptr_t)(buf + w * N), SP = (uint32_t)(uintptr_t)(buf + (1 - w) * N);
  const u64* lutw = lut + (size_t)w * N;
  const u64* gown = bsk + (size_t)3 * w * N;
  const u64* gpar = bsk + (size_t)(2 - w) * N;
  const uint32_t lut_lo = (uint32_t)(uintptr_t)lutw, lut_hi = (uint32_t)((uintptr_t)lutw >> 32);
  const uint32_t gown_lo = (uint32_t)(uintptr_t)gown, gown_hi = (uint32_t)((uintptr_t)gown >> 32);
  const uint32_t gpar_lo = (uint32_t)(uintptr_t)gpar, gpar_hi = (uint32_t)((uintptr_t)gpar >> 32);
  const uint32_t lwe_lo = (uint32_t)(uintptr_t)lwe, lwe_hi = (uint32_t)((uintptr_t)lwe >> 32);
  const uint32_t tab_lo = (uint32_t)(uintptr_t)tab, tab_hi = (uint32_t)((uintptr_t)tab >> 32);
  if constexpr (ALIAS) {
    MI_PBS_BODY_ALIAS_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [lut_lo] "s"(lut_lo), [lut_hi] "s"(lut_hi),
                         [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi), [gpar_lo] "s"(gpar_lo),
                         [gpar_hi] "s"(gpar_hi), [lwe_lo] "s"(lwe_lo), [lwe_hi] "s"(lwe_hi), [n] "s"(n_lwe),
                         [tab_lo] "s"(tab_lo), [tab_hi] "s"(tab_hi), [bl] "s"(base_log),
                         [LW] "s"((uint32_t)(uintptr_t)lwtab));
  } else {
    MI_PBS_BODY_BNF_L1([lane] "v"(lane), [S] "s"(S), [SP] "s"(SP), [lut_lo] "s"(lut_lo), [lut_hi] "s"(lut_hi),
                       [gown_lo] "s"(gown_lo), [gown_hi] "s"(gown_hi), [gpar_lo] "s"(gpar_lo),
                       [gpar_hi] "s"(gpar_hi), [lwe_lo] "s"(lwe_lo), [lwe_hi] "s"(lwe_hi), [n] "s"(n_lwe),
                       [tab_lo] "s"(tab_lo), [tab_hi] "s"(tab_hi), [bl] "s"(base_log),
                       [LW] "s"((uint32_t)(uintptr_t)lwtab));
  }
  sink[(size_t)b * 128 + t] = buf[w * N + lane];  // keep the result live (vector store)
}

__global__ void fill(u64* d, size_t n, u64 seed, u64 mod) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) {
    u64 x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    d[i] = mod ? x % mod : x;
  }
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

int main() {
  const uint32_t n_lwe = 918, batch = 4096;
  const u64 P = 0xFFFFFFFF00000001ull;
  u64 *lwe, *lut, *bsk, *tab, *sink;
  const size_t bsk_n = (size_t)n_lwe * 4 * N;
  CK(hipMalloc(&lwe, (size_t)batch * (n_lwe + 1) * 8));
  CK(hipMalloc(&lut, 2 * N * 8));
  CK(hipMalloc(&bsk, bsk_n * 8));
  CK(hipMalloc(&tab, 4 * 2080 * 8));
  CK(hipMalloc(&sink, (size_t)batch * 128 * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto fl = [&](u64* d, size_t n, u64 seed, u64 mod) {
    hipLaunchKernelGGL(fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, n, seed, mod);
  };
  fl(lwe, (size_t)batch * (n_lwe + 1), 1, 0);
  fl(lut, 2 * N, 2, 0);
  fl(bsk, bsk_n, 3, P);
  fl(tab, 4 * 2080, 4, P);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  double ms[2][3];
  for (int rep = 0; rep < 3; ++rep)
    for (int a = 0; a < 2; ++a) {
      CK(hipEventRecord(e0, s));
      if (a)
        hipLaunchKernelGGL(probe_pbs<true>, dim3(batch), dim3(128), 0, s, lwe, lut, bsk, n_lwe, batch, 23, tab, sink);
      else
        hipLaunchKernelGGL(probe_pbs<false>, dim3(batch), dim3(128), 0, s, lwe, lut, bsk, n_lwe, batch, 23, tab, sink);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float m = 0;
      CK(hipEventElapsedTime(&m, e0, e1));
      ms[a][rep] = m;
    }
  printf("{\"pbs_ms_real_key\": [%.2f, %.2f, %.2f], \"pbs_ms_aliased_64KiB_key\": [%.2f, %.2f, %.2f], \"batch\": %u, "
         "\"n_lwe\": %u}\n",
         ms[0][0], ms[0][1], ms[0][2], ms[1][0], ms[1][1], ms[1][2], batch, n_lwe);
  return 0;
}
