// fft64_launch.hpp — host-side launchers of the f64-FFT PBS kernels: the one-wave N = 2048 engine (fft64_pbs.hip)
// and the shape-generic engine (fft64_generic.hip, every other N).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "pbs_io.hpp"

namespace mi {

// Device twiddle tables of an N = 2048 plan (complex values as interleaved re, im doubles):
//   t1  [16][64]  w^j omega^(j k1), w = exp(i pi / 2M), omega = exp(-2 pi i / M), M = 1024
//   t2  [3][16]   W64^(jl q1) = exp(-2 pi i jl q1 / 64), q1 = 1..3
//   cm  [16]      exp(i pi m / 32)
//   cmi [16]      exp(-i pi m / 32) / M  (torus units; the API backward applies the 2^64)
struct FftTables {
  const double* t1;
  const double* t2;
  const double* cm;
  const double* cmi;
};

hipError_t launch_fft64_fwd_torus(double* fourier, const uint64_t* std_, size_t batch, const FftTables& t,
                                  hipStream_t s);
hipError_t launch_fft64_bwd_torus(uint64_t* std_, const double* fourier, size_t batch, bool add, const FftTables& t,
                                  hipStream_t s);
hipError_t launch_fft64_ext_product(int k, bool cmux, uint64_t* out, uint64_t* glwe, const double* ggsw, size_t batch,
                                    int base_log, int level, const FftTables& t, hipStream_t s);
hipError_t launch_fft64_pbs(int k, uint64_t* out, const uint64_t* lwe_in, const PbsIo& io, const double* fbsk,
                            size_t n_lwe, size_t batch, int base_log, int level, int ms_mode, const FftTables& t,
                            hipStream_t s);
// Fourier order interchange of `polys` polynomials (N / 2 complex each; in place allowed): to_standard = engine
// order -> the reference's serialised natural order (tfhe-fft/src/unordered.rs:943-964), else the reverse (:974-1020)
hipError_t launch_fft64_reorder(double* out, const double* in, size_t polys, bool to_standard, hipStream_t s);

// Device tables of a generic plan (N = 2^logn, M = N / 2; complex values as interleaved re, im doubles):
//   tw   [M]  exp(i pi n / 2M)        (Twisties::new(M), fft/mod.rs:64-75)
//   untw [M]  exp(-i pi n / 2M) / M   (torus units)
//   wm   [M]  exp(-2 pi i t / M)
struct FftGenTables {
  const double* tw;
  const double* untw;
  const double* wm;
  int logn;
};

hipError_t launch_fftg_fwd_torus(double* fourier, const uint64_t* std_, size_t batch, const FftGenTables& t,
                                 hipStream_t s);
hipError_t launch_fftg_bwd_torus(uint64_t* std_, const double* fourier, size_t batch, bool add, const FftGenTables& t,
                                 hipStream_t s);
hipError_t launch_fftg_reorder(double* out, const double* in, size_t polys, bool to_standard, const FftGenTables& t,
                               hipStream_t s);
hipError_t launch_fftg_ext_product(int k, bool cmux, uint64_t* out, uint64_t* glwe, const double* ggsw, size_t batch,
                                   int base_log, int level, const FftGenTables& t, hipStream_t s);
hipError_t launch_fftg_pbs(int k, uint64_t* out, const uint64_t* lwe_in, const PbsIo& io, const double* fbsk,
                           size_t n_lwe, size_t batch, int base_log, int level, int ms_mode, const FftGenTables& t,
                           hipStream_t s);
// engine position -> frequency of a generic plan (fft64_generic.hip: k1 C + p holds k1 + R bitrev_C(p))
uint32_t fftg_frequency(int logn, uint32_t pos);

// position (register r, lane l) of the Fourier layout -> frequency index (see fft64_pbs.hip)
inline uint32_t fft64_frequency(int r, int l) {
  const int k1 = (l & 3) | (((l >> 4) & 3) << 2), q1 = ((l >> 3) & 1) | (((l >> 2) & 1) << 1);
  return (uint32_t)(k1 + 16 * q1 + 64 * r);
}

}  // namespace mi
