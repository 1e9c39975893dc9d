// bfly_bench.hip — throughput of Goldilocks butterfly implementations on gfx950, register-only
// (no memory in the loop): compiler-generated (mi_arith.hpp) vs the generated asm (gl_asm.hpp).
// Each lane holds 8 u64 and runs 3 CT stages (4 butterflies each) per iteration, twiddles in VGPRs.
// Build+run:  hipcc --offload-arch=gfx950 -O3 -I tfhe-rs-main_modified_amd/csrc tools/bfly_bench.hip -o tools/bfly_bench && tools/bfly_bench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mi_arith.hpp"
#include "gl_asm.hpp"

using namespace mi;
typedef uint32_t u32;

#define NX 8

__device__ __forceinline__ void ct_cpp(u64& a, u64& b, u64 w) {
  const u64 t = Goldilocks::mul(b, w);
  const u64 a0 = a;
  a = Goldilocks::add(a0, t);
  b = Goldilocks::sub(a0, t);
}
__device__ __forceinline__ void gs_cpp(u64& a, u64& b, u64 w) {
  const u64 a0 = a, b0 = b;
  a = Goldilocks::add(a0, b0);
  b = Goldilocks::mul(Goldilocks::sub(a0, b0), w);
}

template <int MODE, int OCC>
__global__ __launch_bounds__(256, OCC) void kbench(u64* io, const u64* tw, int iters) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  u64 x[NX];
  for (int i = 0; i < NX; ++i) x[i] = io[(size_t)gid * NX + i];
  u64 w[4];
  for (int i = 0; i < 4; ++i) w[i] = tw[(threadIdx.x + i) & 63];
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int h = 4 >> s;  // butterfly distance
      int j = 0;
      u32 lo[NX], hi[NX];
      if (MODE >= 1) {
#pragma unroll
        for (int i = 0; i < NX; ++i) { lo[i] = (u32)x[i]; hi[i] = (u32)(x[i] >> 32); }
      }
      int ia[4], ib[4];
#pragma unroll
      for (int r = 0; r < NX; ++r)
        if (!(r & h)) { ia[j] = r; ib[j] = r | h; ++j; }
      if (MODE == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ct_cpp(x[ia[q]], x[ib[q]], w[q]);
      } else if (MODE == 3) {
#pragma unroll
        for (int q = 0; q < 4; ++q) gs_cpp(x[ia[q]], x[ib[q]], w[q]);
      } else {
        u32 w0[4], w1[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) { w0[q] = (u32)w[q]; w1[q] = (u32)(w[q] >> 32); }
        if (MODE == 1) {
          glasm::ct4(lo[ia[0]], hi[ia[0]], lo[ib[0]], hi[ib[0]], lo[ia[1]], hi[ia[1]], lo[ib[1]], hi[ib[1]],
                     lo[ia[2]], hi[ia[2]], lo[ib[2]], hi[ib[2]], lo[ia[3]], hi[ia[3]], lo[ib[3]], hi[ib[3]],
                     w0[0], w1[0], w0[1], w1[1], w0[2], w1[2], w0[3], w1[3]);
        } else if (MODE == 2) {
#pragma unroll
          for (int q = 0; q < 4; ++q) glasm::ct1(lo[ia[q]], hi[ia[q]], lo[ib[q]], hi[ib[q]], w0[q], w1[q]);
        } else if (MODE == 4) {
          glasm::gs4(lo[ia[0]], hi[ia[0]], lo[ib[0]], hi[ib[0]], lo[ia[1]], hi[ia[1]], lo[ib[1]], hi[ib[1]],
                     lo[ia[2]], hi[ia[2]], lo[ib[2]], hi[ib[2]], lo[ia[3]], hi[ia[3]], lo[ib[3]], hi[ib[3]],
                     w0[0], w1[0], w0[1], w1[1], w0[2], w1[2], w0[3], w1[3]);
        } else if (MODE == 5) {
#pragma unroll
          for (int q = 0; q < 2; ++q)
            glasm::ct2(lo[ia[2 * q]], hi[ia[2 * q]], lo[ib[2 * q]], hi[ib[2 * q]], lo[ia[2 * q + 1]], hi[ia[2 * q + 1]],
                       lo[ib[2 * q + 1]], hi[ib[2 * q + 1]], w0[2 * q], w1[2 * q], w0[2 * q + 1], w1[2 * q + 1]);
        }
#pragma unroll
        for (int i = 0; i < NX; ++i) x[i] = ((u64)hi[i] << 32) | lo[i];
      }
    }
  }
  for (int i = 0; i < NX; ++i) io[(size_t)gid * NX + i] = x[i];
}

static u64 mulmod(u64 a, u64 b) { return (u64)(((unsigned __int128)a * b) % 0xFFFFFFFF00000001ull); }

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  const int blocks = 256 * 16;
  const size_t n = (size_t)blocks * 256 * NX;
  const u64 P = 0xFFFFFFFF00000001ull;
  u64* h = (u64*)malloc(n * 8);
  u64* ref = (u64*)malloc(n * 8);
  u64* got = (u64*)malloc(n * 8);
  u64* ref2 = (u64*)malloc(n * 8);
  u64 htw[64];
  u64 s = 12345;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
  for (size_t i = 0; i < n; ++i) { u64 v; do v = rnd(); while (v >= P); h[i] = v; }
  // edge values
  h[0] = 0; h[1] = P - 1; h[2] = 1; h[3] = P - 1; h[4] = 0xFFFFFFFFull; h[5] = 1ull << 32; h[6] = P - 1; h[7] = P - 2;
  for (int i = 0; i < 64; ++i) { u64 v; do v = rnd(); while (v >= P); htw[i] = v; }
  htw[0] = P - 1; htw[1] = 1; htw[2] = 0;
  u64 *dio, *dtw;
  hipMalloc(&dio, n * 8);
  hipMalloc(&dtw, 64 * 8);
  hipMemcpy(dtw, htw, 64 * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct { const char* name; void (*f)(u64*, const u64*, int); } ks[] = {
      {"ct c++ occ4", kbench<0, 4>}, {"ct asm x4 occ4", kbench<1, 4>}, {"ct asm x1 occ4", kbench<2, 4>},
      {"ct asm x2 occ4", kbench<5, 4>},
      {"gs c++ occ4", kbench<3, 4>}, {"gs asm x4 occ4", kbench<4, 4>},
      {"ct c++ occ2", kbench<0, 2>}, {"ct asm x4 occ2", kbench<1, 2>}, {"ct asm x1 occ2", kbench<2, 2>},
      {"ct asm x2 occ2", kbench<5, 2>},
  };
  // correctness: 1 iteration each, compare with the C++ version (CT and GS separately)
  for (int k = 0; k < 10; ++k) {
    hipMemcpy(dio, h, n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ks[k].f, dim3(blocks), dim3(256), 0, 0, dio, dtw, 3);
    hipMemcpy(got, dio, n * 8, hipMemcpyDeviceToHost);
    const bool gs = (k == 4 || k == 5);
    u64* r = gs ? ref2 : ref;
    if (k == 0 || k == 4) memcpy(r, got, n * 8);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += (got[i] != r[i]) || got[i] >= P;
    printf("%-18s check vs c++: %s (%zu bad)\n", ks[k].name, bad ? "FAIL" : "ok", bad);
  }
  (void)mulmod;
  const int iters = 200;
  for (auto& k : ks) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipMemcpy(dio, h, n * 8, hipMemcpyHostToDevice);
      hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, dio, dtw, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double bf = (double)blocks * 256 * iters * 12;
    printf("%-18s %8.3f ms  %7.1f G butterflies/s  %6.1f cycles/butterfly/SIMD @2.4GHz\n", k.name, best, bf / best / 1e6,
           best * 1e-3 * 2.4e9 * 1024 / (bf / 64));
  }
  return 0;
}
