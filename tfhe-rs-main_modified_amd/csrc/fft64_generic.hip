// fft64_generic.hip — the shape-generic f64-FFT engine: every polynomial size 32 <= N <= 2^18 other than the
// one-wave N = 2048 engine's (fft64_pbs.hip), with the same operator surface: forward_as_torus /
// backward_as_torus, the Fourier-order interchange, the external product / CMUX and the programmable bootstrap
// for any GLWE dimension k and decomposition.  Reference paths relative to /root/reference/tfhe/src/core_crypto:
//   Fft::new + Twisties       fft_impl/fft64/math/fft/mod.rs:58-76, 170-223 (any power-of-two polynomial size)
//   conversions               fft_impl/fft64/math/fft/mod.rs:227-356, 524-586
//   external product          fft_impl/fft64/crypto/ggsw.rs:483-603 (+ update_with_fmadd :617-698)
//   blind rotate / PBS        fft_impl/fft64/crypto/bootstrap.rs:294-381, 481-521
//   sample extraction         algorithms/glwe_sample_extraction.rs:89-160
// The shortint parameter sets next to PARAM_MESSAGE_2_CARRY_2 run here: MESSAGE_1_CARRY_1 (N = 512, k = 4),
// MESSAGE_3_CARRY_3 (N = 8192) and MESSAGE_4_CARRY_4 (N = 65536).
//
// Transform.  As the reference: N real coefficients fold into M = N / 2 complex values u[n] = x[n] + i x[n + M],
// twisted by exp(i pi n / 2M) and transformed by an M-point DFT with the exp(-2 pi i / M) kernel.  M = R x C with
// C = min(M, 8192) (one row fits the LDS of one workgroup: 128 KiB) and R = M / C <= 16:
//   columns  (R > 1 only) a radix-R DFT over n1 of x[n1 C + n2] per column n2, in registers, times the four-step
//            twiddle W_M^(n2 k1), stored as row k1 (coalesced over n2); the element producer (twist, folding,
//            digit extraction, the CMUX difference) is fused into its loads
//   rows     one C-point DFT per row in LDS: decimation in frequency, radix-8 steps (a closed group of 8
//            elements at stride L / 8 per thread, W_L twiddles from the plan's table) and one radix-2 / radix-4
//            step for the remaining bits; rows are read and written coalesced through LDS
// The inverse runs the conjugate passes in reverse (decimation in time), the MAC of the external product fused
// into its row loads and the untwist + torus accumulation into its last stores.  The Fourier-domain order is this
// engine's own: position k1 C + p holds frequency k1 + R bitrev_C(p) (mi_fft64_fourier_order); the reference
// serialises the natural order, which fftg_reorder converts to and from.
//
// The blind rotation keeps the chunk's accumulators in HBM; one CMUX step is the forward pass over all
// chunk x level x (k + 1) digit polynomials (digits computed on the fly from the accumulator and the rotation), and
// the inverse pass over the chunk x (k + 1) products (MAC in, acc += from_torus out).  Masks that switch to 0 give an
// exactly-zero difference, digits, transform and product, so every ciphertext runs every step (bit-identical to the
// reference's skip, bootstrap.rs:336).  Results are f64 computations, not bit-identical to the reference's
// (parity is decryption + an error bound against the numpy restatement).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "scratch.hpp"
#include "fft64_device.hpp"
#include "fft64_launch.hpp"

namespace mi {
namespace fft {
namespace gen {

constexpr int MAX_LOGC = 13;  // one LDS row: 8192 complex = 128 KiB

__host__ __device__ __forceinline__ uint32_t brev(uint32_t x, int bits) {
  return bits == 0 ? 0u : (__builtin_bitreverse32(x) >> (32 - bits));
}

// x * W16^e, W16 = exp(-2 pi i / 16) (INV: the conjugate), e in [0, 8) (compile-time after unrolling)
template <bool INV>
__device__ __forceinline__ cplx w16(cplx x, int e) {
  constexpr double C8 = 0.92387953251128673848, S8 = 0.38268343236508978178, R2 = 0.70710678118654752440;
  double c, s;  // W16^e = c - i s
  switch (e) {
    case 0: return x;
    case 4: return INV ? mul_pos_i(x) : mul_neg_i(x);
    case 1: c = C8, s = S8; break;
    case 2: c = R2, s = R2; break;
    case 3: c = S8, s = C8; break;
    case 5: c = -S8, s = C8; break;
    case 6: c = -R2, s = R2; break;
    default: c = -C8, s = S8; break;
  }
  return cmul(x, cplx{c, INV ? s : -s});
}

// R-point DFT in registers (R <= 16).  Forward: decimation in frequency, natural order in, bit-reversed out
// (register t holds X[bitrev(t)]).  INV: decimation in time with the conjugate kernel, bit-reversed in, natural
// out (unnormalised).
template <int R, bool INV>
__device__ __forceinline__ void small_dft(cplx (&a)[R]) {
  if constexpr (!INV) {
#pragma unroll
    for (int h = R / 2; h >= 1; h >>= 1)
#pragma unroll
      for (int s = 0; s < R; s += 2 * h)
#pragma unroll
        for (int t = 0; t < h; ++t) {
          const cplx u = a[s + t], v = a[s + t + h];
          a[s + t] = cadd(u, v);
          a[s + t + h] = w16<false>(csub(u, v), t * (8 / h));  // W_2h^t
        }
  } else {
#pragma unroll
    for (int h = 1; h < R; h <<= 1)
#pragma unroll
      for (int s = 0; s < R; s += 2 * h)
#pragma unroll
        for (int t = 0; t < h; ++t) {
          const cplx u = a[s + t], v = w16<true>(a[s + t + h], t * (8 / h));
          a[s + t] = cadd(u, v);
          a[s + t + h] = csub(u, v);
        }
  }
}

template <int LOGC>
struct RowGeom {
  static constexpr int C = 1 << LOGC;
  static constexpr int TPR = C / 8;                          // threads per row (one radix-8 group each)
  static constexpr int RPW = TPR >= 256 ? 1 : 256 / TPR;     // rows per workgroup
  static constexpr int T = TPR * RPW;
  static constexpr int S8 = LOGC / 3, REM = LOGC % 3;        // radix-8 steps, then one radix-2^REM step
};

// ---- element producers / consumers -----------------------------------------------------------------------
// A source gives element x of row `row` (load); a sink takes it (store).  Rows are C elements; for R = 1 a row is
// one polynomial and x its folded index n.

struct PlainIO {  // rows of C complex, row-major
  cplx* ptr;
  uint32_t logc;
  __device__ __forceinline__ cplx load(uint64_t row, uint32_t x) const { return ptr[(row << logc) + x]; }
  __device__ __forceinline__ void store(uint64_t row, uint32_t x, cplx v) const { ptr[(row << logc) + x] = v; }
};

// forward_as_torus: (x[n] + i x[n + M]) 2^-64, twisted (convert_forward_torus, fft/mod.rs:524-543)
struct TorusSrc {
  const u64* std_;
  const cplx* tw;
  uint32_t logn;
  __device__ __forceinline__ cplx load(uint64_t p, uint32_t n) const {
    const u64* x = std_ + (p << logn);
    const uint32_t m = 1u << (logn - 1);
    constexpr double NORM = 0x1p-64;
    return cmul(cplx{s64_to_f64(x[n]) * NORM, s64_to_f64(x[n + m]) * NORM}, tw[n]);
  }
};

// digit li of the signed decomposition (least significant level first, as the iterator yields them)
__device__ __forceinline__ u64 digit(u64 x, int base_log, int level, int li) {
  u64 st = decomp_init_native(x, base_log, level), d = 0;
  for (int i = 0; i <= li; ++i) d = decompose_one_level(base_log, st);
  return d;
}

// Digit polynomials of the external product, p = (b level + li)(k + 1) + c: digit li of glwe[b][c], as
// convert_forward_integer (fft/mod.rs:250-269), twisted
struct GlweDigitSrc {
  const u64* glwe;
  const cplx* tw;
  uint32_t logn, kp1, level;
  int base_log;
  __device__ __forceinline__ cplx load(uint64_t p, uint32_t n) const {
    const uint32_t c = (uint32_t)(p % kp1), li = (uint32_t)((p / kp1) % level);
    const uint64_t b = p / ((uint64_t)kp1 * level);
    const u64* x = glwe + ((b * kp1 + c) << logn);
    const uint32_t m = 1u << (logn - 1);
    const u64 d0 = digit(x[n], base_log, (int)level, (int)li), d1 = digit(x[n + m], base_log, (int)level, (int)li);
    return cmul(cplx{s64_to_f64(d0), s64_to_f64(d1)}, tw[n]);
  }
};

// Digit polynomials of blind-rotation step `step`: ct1 = X^a acc - acc (polynomial_wrapping_monic_monomial_mul
// and the CMUX difference, bootstrap.rs:336-360), a = the switched mask element of ciphertext b
struct RotDigitSrc {
  const u64* acc;
  const u64* lwe;
  const cplx* tw;
  uint32_t logn, kp1, level, n_lwe, step;
  int base_log, ms_mode;
  __device__ __forceinline__ cplx load(uint64_t p, uint32_t n) const {
    const uint32_t c = (uint32_t)(p % kp1), li = (uint32_t)((p / kp1) % level);
    const uint64_t b = p / ((uint64_t)kp1 * level);
    const uint32_t nn = 1u << logn, m = nn >> 1;
    const u64 a_raw = lwe[b * (n_lwe + 1) + step];
    const uint32_t a = (uint32_t)(ms_mode == 2 ? (a_raw & (2 * nn - 1)) : modulus_switch(a_raw, logn + 1));
    const uint32_t full = (a >> logn) & 1u, rem = a & (nn - 1);
    const u64* ap = acc + ((b * kp1 + c) << logn);
    u64 ct[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t e = n + (h ? m : 0u);
      u64 v = ap[(e - rem) & (nn - 1)];  // new[e] = old[(e - rem) mod N], negated for e < rem (and when full)
      if (full ^ (e < rem ? 1u : 0u)) v = (u64)0 - v;
      ct[h] = digit(v - ap[e], base_log, (int)level, (int)li);
    }
    return cmul(cplx{s64_to_f64(ct[0]), s64_to_f64(ct[1])}, tw[n]);
  }
};

// update_with_fmadd (ggsw.rs:617-698): y[b][w] = sum over levels li and rows c of D[b][li][c] . G[li][c][w];
// a row of the inverse pass is (b (k + 1) + w) R + k1
struct MacSrc {
  const cplx* d;
  const cplx* g;
  uint32_t logm, logc, logr, kp1, level;
  __device__ __forceinline__ cplx load(uint64_t row, uint32_t x) const {
    const uint64_t q = row >> logr;
    const uint64_t pos = ((row & ((1u << logr) - 1)) << logc) + x;
    const uint32_t w = (uint32_t)(q % kp1);
    const uint64_t b = q / kp1;
    cplx acc = {0.0, 0.0};
    for (uint32_t li = 0; li < level; ++li)
      for (uint32_t c = 0; c < kp1; ++c)
        acc = cfma(d[(((b * level + li) * kp1 + c) << logm) + pos], g[(((uint64_t)(li * kp1 + c) * kp1 + w) << logm) + pos],
                   acc);
    return acc;
  }
};

// backward_as_torus (convert_[add_]backward_torus, fft/mod.rs:545-565): untwist (x 1/M folded into untw), exact
// from_torus of both halves, stored or added
struct TorusSink {
  u64* std_;
  const cplx* untw;
  uint32_t logn;
  int add;
  __device__ __forceinline__ void store(uint64_t p, uint32_t n, cplx v) const {
    const cplx y = cmul(v, untw[n]);
    u64* x = std_ + (p << logn);
    const uint32_t m = 1u << (logn - 1);
    const u64 re = from_torus_scaled(y.re * 0x1p64), im = from_torus_scaled(y.im * 0x1p64);
    x[n] = add ? x[n] + re : re;
    x[n + m] = add ? x[n + m] + im : im;
  }
};

// the external product's accumulation: acc += from_torus(untwisted product) (add_torus, as the N = 2048 engine)
struct AccSink {
  u64* acc;
  const cplx* untw;
  uint32_t logn;
  __device__ __forceinline__ void store(uint64_t p, uint32_t n, cplx v) const {
    const cplx y = cmul(v, untw[n]);
    u64* x = acc + (p << logn);
    const uint32_t m = 1u << (logn - 1);
    add_torus(x[n], y.re);
    add_torus(x[n + m], y.im);
  }
};

// ---- row pass: one C-point DFT per row in LDS ---------------------------------------------------------------
// Register t of a radix-8 group needs W_L^(j0 bitrev(t)): all seven from the one table value W_L^j0 (six products,
// a few ulps, far below the transform's own f64 error), instead of seven table reads.
__device__ __forceinline__ void r8_twiddles(cplx (&w)[8], cplx w1) {
  const cplx w2 = cmul(w1, w1), w3 = cmul(w1, w2), w4 = cmul(w2, w2);
  w[1] = w4, w[2] = w2, w[3] = cmul(w2, w4), w[4] = w1, w[5] = cmul(w1, w4), w[6] = w3, w[7] = cmul(w3, w4);
}

// radix-8 butterfly of a group on block size L = 2^LOGL (forward: DFT8 then twiddles; INV: the conjugate transpose)
template <int LOGL, bool INV>
__device__ __forceinline__ void r8_core(cplx (&a)[8], uint32_t j0, const cplx* __restrict__ wm, uint32_t logm) {
  cplx w[8];
  r8_twiddles(w, wm[j0 << (logm - LOGL)]);
  if constexpr (!INV) {
    small_dft<8, false>(a);
#pragma unroll
    for (int t = 1; t < 8; ++t) a[t] = cmul(a[t], w[t]);
  } else {
#pragma unroll
    for (int t = 1; t < 8; ++t) a[t] = cmulc(a[t], w[t]);
    small_dft<8, true>(a);
  }
}

// radix-8 step in LDS: group g = (block, j0), elements block L + j0 + t L/8
template <int LOGL, bool INV>
__device__ __forceinline__ void radix8_step(cplx* buf, int g, const cplx* __restrict__ wm, uint32_t logm) {
  constexpr int SL = LOGL - 3;
  const uint32_t j0 = (uint32_t)g & ((1u << SL) - 1u);
  const uint32_t base = (((uint32_t)g >> SL) << LOGL) + j0;
  cplx a[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) a[t] = buf[base + ((uint32_t)t << SL)];
  r8_core<LOGL, INV>(a, j0, wm, logm);
#pragma unroll
  for (int t = 0; t < 8; ++t) buf[base + ((uint32_t)t << SL)] = a[t];
}

// the last (forward) / first (inverse) radix-2^REM step: L = 2^REM, j0 = 0, no twiddles; 8 / 2^REM groups a thread
template <int LOGC, bool INV>
__device__ __forceinline__ void rem_step(cplx* buf, int g) {
  using G = RowGeom<LOGC>;
  constexpr int R = 1 << G::REM;
#pragma unroll
  for (int j = 0; j < 8 / R; ++j) {
    const uint32_t base = (uint32_t)(g + j * G::TPR) * R;
    cplx a[R];
#pragma unroll
    for (int t = 0; t < R; ++t) a[t] = buf[base + t];
    small_dft<R, INV>(a);
#pragma unroll
    for (int t = 0; t < R; ++t) buf[base + t] = a[t];
  }
}

// steps I = FIRST .. END - 1 of the S8 radix-8 steps, each followed by a barrier; step I runs at LOGL = LOGC - 3 I
// (forward) or at LOGL = LOGC - 3 (S8 - 1 - I) (inverse: the same steps in reverse order)
template <int LOGC, int I, int END, bool INV>
__device__ __forceinline__ void radix8_steps(cplx* buf, int g, const cplx* __restrict__ wm, uint32_t logm) {
  using G = RowGeom<LOGC>;
  if constexpr (I < END) {
    constexpr int STEP = INV ? (G::S8 - 1 - I) : I;
    radix8_step<LOGC - 3 * STEP, INV>(buf, g, wm, logm);
    __syncthreads();
    radix8_steps<LOGC, I + 1, END, INV>(buf, g, wm, logm);
  }
}

// One row per TPR threads.  The radix-8 step on the whole row (L = C) touches g + t C/8, t < 8 — the coalesced
// pattern of a row copy — so the forward takes its first step straight from the source and the inverse stores its
// last step straight to the sink; the other steps run in LDS, and the forward's result (bit-reversed) and the
// inverse's input are copied out / in coalesced.
template <int LOGC, bool INV, class Src, class Dst>
__global__ __launch_bounds__(RowGeom<LOGC>::T) void rows_kernel(Src src, Dst dst, uint64_t rows,
                                                               const cplx* __restrict__ wm, uint32_t logm) {
  using G = RowGeom<LOGC>;
  __shared__ cplx lds[G::RPW * G::C];
  const int rl = (int)threadIdx.x / G::TPR, g = (int)threadIdx.x % G::TPR;
  const uint64_t row = (uint64_t)blockIdx.x * G::RPW + rl;
  const bool ok = row < rows;  // every thread takes part in the barriers
  cplx* buf = lds + rl * G::C;
  if constexpr (!INV) {
    cplx a[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) a[t] = ok ? src.load(row, (uint32_t)(g + t * G::TPR)) : cplx{0.0, 0.0};
    r8_core<LOGC, false>(a, (uint32_t)g, wm, logm);
#pragma unroll
    for (int t = 0; t < 8; ++t) buf[g + t * G::TPR] = a[t];
    __syncthreads();
    radix8_steps<LOGC, 1, G::S8, false>(buf, g, wm, logm);
    if constexpr (G::REM) {
      rem_step<LOGC, false>(buf, g);
      __syncthreads();
    }
    if (ok) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t x = (uint32_t)(g + j * G::TPR);
        dst.store(row, x, buf[x]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t x = (uint32_t)(g + j * G::TPR);
      buf[x] = ok ? src.load(row, x) : cplx{0.0, 0.0};
    }
    __syncthreads();
    if constexpr (G::REM) {
      rem_step<LOGC, true>(buf, g);
      __syncthreads();
    }
    radix8_steps<LOGC, 0, G::S8 - 1, true>(buf, g, wm, logm);
    cplx a[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) a[t] = buf[g + t * G::TPR];
    r8_core<LOGC, true>(a, (uint32_t)g, wm, logm);
    if (ok) {
#pragma unroll
      for (int t = 0; t < 8; ++t) dst.store(row, (uint32_t)(g + t * G::TPR), a[t]);
    }
  }
}

// ---- column pass (R > 1): radix-R DFT over n1 of x[n1 C + n2], four-step twiddle W_M^(n2 k1) ----------------
__device__ __forceinline__ uint64_t gs_start() { return (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ uint64_t gs_stride() { return (uint64_t)gridDim.x * blockDim.x; }

template <int LOGR, class Src>
__global__ __launch_bounds__(256) void cols_fwd_kernel(Src src, cplx* __restrict__ out, uint64_t polys, uint32_t logc,
                                                       const cplx* __restrict__ wm) {
  constexpr int R = 1 << LOGR;
  const uint32_t cmask = (1u << logc) - 1u;
  for (uint64_t i = gs_start(); i < (polys << logc); i += gs_stride()) {
    const uint64_t p = i >> logc;
    const uint32_t n2 = (uint32_t)i & cmask;
    cplx a[R];
#pragma unroll
    for (int n1 = 0; n1 < R; ++n1) a[n1] = src.load(p, ((uint32_t)n1 << logc) + n2);
    small_dft<R, false>(a);
    cplx* o = out + (p << (logc + LOGR));
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const uint32_t k1 = brev((uint32_t)t, LOGR);
      o[((uint64_t)k1 << logc) + n2] = t ? cmul(a[t], wm[n2 * k1]) : a[t];
    }
  }
}

template <int LOGR, class Sink>
__global__ __launch_bounds__(256) void cols_inv_kernel(Sink sink, const cplx* __restrict__ in, uint64_t polys,
                                                       uint32_t logc, const cplx* __restrict__ wm) {
  constexpr int R = 1 << LOGR;
  const uint32_t cmask = (1u << logc) - 1u;
  for (uint64_t i = gs_start(); i < (polys << logc); i += gs_stride()) {
    const uint64_t p = i >> logc;
    const uint32_t n2 = (uint32_t)i & cmask;
    const cplx* src = in + (p << (logc + LOGR));
    cplx a[R];
#pragma unroll
    for (int t = 0; t < R; ++t) {
      const uint32_t k1 = brev((uint32_t)t, LOGR);
      const cplx v = src[((uint64_t)k1 << logc) + n2];
      a[t] = t ? cmulc(v, wm[n2 * k1]) : v;
    }
    small_dft<R, true>(a);
#pragma unroll
    for (int n1 = 0; n1 < R; ++n1) sink.store(p, ((uint32_t)n1 << logc) + n2, a[n1]);
  }
}

// ---- engine order <-> natural order (tfhe-fft/src/unordered.rs:943-1020: the serialised order is natural) -----
__host__ __device__ __forceinline__ uint32_t position_of(uint32_t f, uint32_t logc, uint32_t logr) {
  return ((f & ((1u << logr) - 1u)) << logc) | brev(f >> logr, (int)logc);
}
__host__ __device__ __forceinline__ uint32_t frequency_at(uint32_t pos, uint32_t logc, uint32_t logr) {
  return (pos >> logc) | (brev(pos & ((1u << logc) - 1u), (int)logc) << logr);
}

// the in-place reorder's staging copy (a kernel, not an SDMA copy: ordered on the stream like every other launch)
__global__ __launch_bounds__(256) void copy_cplx_kernel(cplx* __restrict__ out, const cplx* __restrict__ in, uint64_t n) {
  for (uint64_t i = gs_start(); i < n; i += gs_stride()) out[i] = in[i];
}

template <bool TO_STD>
__global__ __launch_bounds__(256) void reorder_kernel(cplx* __restrict__ out, const cplx* __restrict__ in,
                                                      uint64_t polys, uint32_t logc, uint32_t logr) {
  const uint32_t logm = logc + logr, mmask = (1u << logm) - 1u;
  for (uint64_t i = gs_start(); i < (polys << logm); i += gs_stride()) {
    const uint64_t base = i & ~(uint64_t)mmask;
    const uint32_t j = (uint32_t)i & mmask;
    out[i] = in[base + (TO_STD ? position_of(j, logc, logr) : frequency_at(j, logc, logr))];
  }
}

// ---- blind-rotation bookkeeping ----------------------------------------------------------------------------
// acc[b] = LUT / X^body (polynomial_wrapping_monic_monomial_div, bootstrap.rs:499-507)
// acc[b] = the item's LUT / X^body (io: pbs_io.hpp; item b of the chunk is item b0 + b of the batch; a skipped item,
// LUT index out of range, gets a zero accumulator and is not written back)
__global__ __launch_bounds__(256) void init_acc_kernel(u64* __restrict__ acc, PbsIo io, uint64_t b0,
                                                       const u64* __restrict__ lwe, const u64* __restrict__ corr,
                                                       uint32_t n_lwe, uint32_t batch, uint32_t logn, uint32_t kp1,
                                                       int ms_mode) {
  const uint32_t nn = 1u << logn;
  const uint64_t per = (uint64_t)kp1 << logn;
  for (uint64_t i = gs_start(); i < per * batch; i += gs_stride()) {
    const uint64_t b = i / per, ce = i % per;
    const uint32_t c = (uint32_t)(ce >> logn), m = (uint32_t)ce & (nn - 1);
    const u64* lut = io.lut_for(b0 + b, per);
    if (!lut) {
      acc[i] = 0;
      continue;
    }
    const u64 bv = lwe[b * (n_lwe + 1) + n_lwe];
    const u64 body = ms_mode == 2 ? (bv & (2 * nn - 1)) : modulus_switch(bv + (corr ? corr[b] : 0), logn + 1);
    const uint32_t full = (uint32_t)(body >> logn) & 1u, rem = (uint32_t)body & (nn - 1);
    u64 v = lut[((uint64_t)c << logn) + ((m + rem) & (nn - 1))];
    if (full ^ (m >= nn - rem ? 1u : 0u)) v = (u64)0 - v;
    acc[i] = v;
  }
}

// centered_binary_ms_body_correction_to_add (algorithms/modulus_switch.rs:60-104), one workgroup per ciphertext
__global__ __launch_bounds__(256) void body_correction_kernel(u64* __restrict__ corr, const u64* __restrict__ lwe,
                                                              uint32_t n_lwe, unsigned log_mod) {
  __shared__ u64 sh[512];
  const u64 v = centered_body_correction<256>(lwe + (uint64_t)blockIdx.x * (n_lwe + 1), n_lwe, log_mod,
                                              (int)threadIdx.x, sh);
  if (threadIdx.x == 0) corr[blockIdx.x] = v;
}

// extract_lwe_sample_from_glwe_ciphertext, nth = 0: out[c N] = A_c[0], out[c N + j] = -A_c[N - j], out[k N] = B[0];
// items whose LUT index is out of range (io.lut_idx) are not written
__global__ __launch_bounds__(256) void extract_kernel(u64* __restrict__ out, const u64* __restrict__ acc,
                                                      uint32_t batch, uint32_t logn, uint32_t k, PbsIo io, uint64_t b0) {
  const uint32_t nn = 1u << logn;
  const uint64_t per_out = ((uint64_t)k << logn) + 1, per = (uint64_t)(k + 1) << logn;
  for (uint64_t i = gs_start(); i < per_out * batch; i += gs_stride()) {
    const uint64_t b = i / per_out, o = i % per_out;
    if (io.lut_idx && !io.lut_for(b0 + b, per)) continue;
    const uint32_t c = (uint32_t)(o >> logn), j = (uint32_t)o & (nn - 1);
    const u64 v = acc[b * per + ((uint64_t)c << logn) + (j ? nn - j : 0u)];
    out[i] = (c == k || j == 0) ? v : (u64)0 - v;
  }
}

// blind_rotate_assign (fft64_pbs.rs:186-250): the rotated accumulators of a chunk into io.glwe_out (skipped items kept)
__global__ __launch_bounds__(256) void store_glwe_kernel(const u64* __restrict__ acc, uint32_t batch, uint64_t per,
                                                         PbsIo io, uint64_t b0) {
  for (uint64_t i = gs_start(); i < per * batch; i += gs_stride()) {
    const uint64_t b = i / per;
    if (!io.lut_for(b0 + b, per)) continue;
    io.glwe_out[b0 * per + i] = acc[i];
  }
}

// CMUX input: ct1 -= ct0 (cmux, fft64_pbs.rs:510-560), elementwise
__global__ __launch_bounds__(256) void sub_assign_kernel(u64* __restrict__ a, const u64* __restrict__ b, uint64_t count) {
  for (uint64_t i = gs_start(); i < count; i += gs_stride()) a[i] -= b[i];
}

inline unsigned blocks_for(uint64_t total) { return (unsigned)std::min<uint64_t>((total + 255) / 256, 65536); }

// ---- launch helpers ---------------------------------------------------------------------------------------
template <int LOGC, bool INV, class Src, class Dst>
hipError_t rows_at(Src src, Dst dst, uint64_t rows, const cplx* wm, uint32_t logm, hipStream_t s) {
  using G = RowGeom<LOGC>;
  const uint64_t grid = (rows + G::RPW - 1) / G::RPW;
  if (grid > 0xFFFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL((rows_kernel<LOGC, INV, Src, Dst>), dim3((unsigned)grid), dim3(G::T), 0, s, src, dst, rows, wm,
                     logm);
  return hipGetLastError();
}

template <bool INV, class Src, class Dst>
hipError_t rows(uint32_t logc, Src src, Dst dst, uint64_t n_rows, const cplx* wm, uint32_t logm, hipStream_t s) {
  if (n_rows == 0) return hipSuccess;
  switch (logc) {
    case 4: return rows_at<4, INV>(src, dst, n_rows, wm, logm, s);
    case 5: return rows_at<5, INV>(src, dst, n_rows, wm, logm, s);
    case 6: return rows_at<6, INV>(src, dst, n_rows, wm, logm, s);
    case 7: return rows_at<7, INV>(src, dst, n_rows, wm, logm, s);
    case 8: return rows_at<8, INV>(src, dst, n_rows, wm, logm, s);
    case 9: return rows_at<9, INV>(src, dst, n_rows, wm, logm, s);
    case 10: return rows_at<10, INV>(src, dst, n_rows, wm, logm, s);
    case 11: return rows_at<11, INV>(src, dst, n_rows, wm, logm, s);
    case 12: return rows_at<12, INV>(src, dst, n_rows, wm, logm, s);
    case 13: return rows_at<13, INV>(src, dst, n_rows, wm, logm, s);
    default: return hipErrorInvalidValue;
  }
}

template <class Src>
hipError_t cols_fwd(uint32_t logr, Src src, cplx* out, uint64_t polys, uint32_t logc, const cplx* wm, hipStream_t s) {
  const unsigned grid = blocks_for(polys << logc);
  switch (logr) {
    case 1: hipLaunchKernelGGL((cols_fwd_kernel<1, Src>), dim3(grid), dim3(256), 0, s, src, out, polys, logc, wm); break;
    case 2: hipLaunchKernelGGL((cols_fwd_kernel<2, Src>), dim3(grid), dim3(256), 0, s, src, out, polys, logc, wm); break;
    case 3: hipLaunchKernelGGL((cols_fwd_kernel<3, Src>), dim3(grid), dim3(256), 0, s, src, out, polys, logc, wm); break;
    case 4: hipLaunchKernelGGL((cols_fwd_kernel<4, Src>), dim3(grid), dim3(256), 0, s, src, out, polys, logc, wm); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <class Sink>
hipError_t cols_inv(uint32_t logr, Sink sink, const cplx* in, uint64_t polys, uint32_t logc, const cplx* wm,
                    hipStream_t s) {
  const unsigned grid = blocks_for(polys << logc);
  switch (logr) {
    case 1: hipLaunchKernelGGL((cols_inv_kernel<1, Sink>), dim3(grid), dim3(256), 0, s, sink, in, polys, logc, wm); break;
    case 2: hipLaunchKernelGGL((cols_inv_kernel<2, Sink>), dim3(grid), dim3(256), 0, s, sink, in, polys, logc, wm); break;
    case 3: hipLaunchKernelGGL((cols_inv_kernel<3, Sink>), dim3(grid), dim3(256), 0, s, sink, in, polys, logc, wm); break;
    case 4: hipLaunchKernelGGL((cols_inv_kernel<4, Sink>), dim3(grid), dim3(256), 0, s, sink, in, polys, logc, wm); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

struct Geo {
  uint32_t logn, logm, logr, logc;
  const cplx *tw, *untw, *wm;
};
inline Geo geo(const FftGenTables& t) {
  Geo g;
  g.logn = (uint32_t)t.logn;
  g.logm = g.logn - 1;
  g.logr = g.logm > (uint32_t)MAX_LOGC ? g.logm - (uint32_t)MAX_LOGC : 0u;
  g.logc = g.logm - g.logr;
  g.tw = reinterpret_cast<const cplx*>(t.tw);
  g.untw = reinterpret_cast<const cplx*>(t.untw);
  g.wm = reinterpret_cast<const cplx*>(t.wm);
  return g;
}

// forward transform of `polys` polynomials produced by `src` into `out` (engine order)
template <class Src>
hipError_t forward(const Geo& g, Src src, cplx* out, uint64_t polys, hipStream_t s) {
  if (g.logr == 0) return rows<false>(g.logc, src, PlainIO{out, g.logc}, polys, g.wm, g.logm, s);
  hipError_t e = cols_fwd(g.logr, src, out, polys, g.logc, g.wm, s);
  if (e != hipSuccess) return e;
  return rows<false>(g.logc, PlainIO{out, g.logc}, PlainIO{out, g.logc}, polys << g.logr, g.wm, g.logm, s);
}

// inverse transform of `polys` rows-sources into `sink`; `tmp` holds polys x M complex when R > 1
template <class Src, class Sink>
hipError_t inverse(const Geo& g, Src src, Sink sink, cplx* tmp, uint64_t polys, hipStream_t s) {
  if (g.logr == 0) return rows<true>(g.logc, src, sink, polys, g.wm, g.logm, s);
  hipError_t e = rows<true>(g.logc, src, PlainIO{tmp, g.logc}, polys << g.logr, g.wm, g.logm, s);
  if (e != hipSuccess) return e;
  return cols_inv(g.logr, sink, tmp, polys, g.logc, g.wm, s);
}

// items per chunk: digits (level (k + 1) M complex), products (R > 1: (k + 1) M complex) and accumulators stay
// below ~4 GiB of scratch (of 288 GB)
inline size_t chunk_for(const Geo& g, uint32_t kp1, uint32_t level, size_t batch) {
  const size_t per_item = ((size_t)level + 2) * kp1 * ((size_t)8 << g.logn);
  return std::max<size_t>(1, std::min(batch, ((size_t)4 << 30) / per_item));
}

}  // namespace gen
}  // namespace fft

using fft::cplx;

uint32_t fftg_frequency(int logn, uint32_t pos) {
  const uint32_t logm = (uint32_t)logn - 1;
  const uint32_t logr = logm > (uint32_t)fft::gen::MAX_LOGC ? logm - (uint32_t)fft::gen::MAX_LOGC : 0u;
  return fft::gen::frequency_at(pos, logm - logr, logr);
}

hipError_t launch_fftg_fwd_torus(double* fourier, const uint64_t* std_, size_t batch, const FftGenTables& t,
                                 hipStream_t s) {
  using namespace fft::gen;
  if (batch == 0) return hipSuccess;
  const Geo g = geo(t);
  return forward(g, TorusSrc{std_, g.tw, g.logn}, reinterpret_cast<cplx*>(fourier), batch, s);
}

hipError_t launch_fftg_bwd_torus(uint64_t* std_, const double* fourier, size_t batch, bool add, const FftGenTables& t,
                                 hipStream_t s) {
  using namespace fft::gen;
  if (batch == 0) return hipSuccess;
  const Geo g = geo(t);
  const PlainIO in{const_cast<cplx*>(reinterpret_cast<const cplx*>(fourier)), g.logc};  // read only
  const TorusSink sink{std_, g.untw, g.logn, add ? 1 : 0};
  if (g.logr == 0) return inverse(g, in, sink, nullptr, batch, s);
  cplx* tmp = nullptr;
  hipError_t e = mi::scratch_alloc((void**)&tmp, (batch << g.logm) * sizeof(cplx), s);
  if (e != hipSuccess) return e;
  e = inverse(g, in, sink, tmp, batch, s);
  const hipError_t ef = mi::scratch_free(tmp, s);
  return e != hipSuccess ? e : ef;
}

hipError_t launch_fftg_reorder(double* out, const double* in, size_t polys, bool to_standard, const FftGenTables& t,
                               hipStream_t s) {
  using namespace fft::gen;
  if (polys == 0) return hipSuccess;
  const Geo g = geo(t);
  const size_t bytes = (polys << g.logm) * sizeof(cplx);
  const cplx* src = reinterpret_cast<const cplx*>(in);
  cplx* tmp = nullptr;
  hipError_t e = hipSuccess;
  if (out == in) {  // a permutation in place: stage the input
    if ((e = mi::scratch_alloc((void**)&tmp, bytes, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(copy_cplx_kernel, dim3(blocks_for(polys << g.logm)), dim3(256), 0, s, tmp, src, (uint64_t)(polys << g.logm));
    if ((e = hipGetLastError()) != hipSuccess) {
      (void)mi::scratch_free(tmp, s);
      return e;
    }
    src = tmp;
  }
  const unsigned grid = blocks_for(polys << g.logm);
  if (to_standard)
    hipLaunchKernelGGL(reorder_kernel<true>, dim3(grid), dim3(256), 0, s, reinterpret_cast<cplx*>(out), src,
                       (uint64_t)polys, g.logc, g.logr);
  else
    hipLaunchKernelGGL(reorder_kernel<false>, dim3(grid), dim3(256), 0, s, reinterpret_cast<cplx*>(out), src,
                       (uint64_t)polys, g.logc, g.logr);
  e = hipGetLastError();
  if (tmp) {
    const hipError_t ef = mi::scratch_free(tmp, s);
    if (e == hipSuccess) e = ef;
  }
  return e;
}

hipError_t launch_fftg_ext_product(int k, bool cmux, uint64_t* out, uint64_t* glwe, const double* ggsw, size_t batch,
                                   int base_log, int level, const FftGenTables& t, hipStream_t s) {
  using namespace fft::gen;
  if (batch == 0) return hipSuccess;
  const Geo g = geo(t);
  const uint32_t kp1 = (uint32_t)k + 1, lv = (uint32_t)level;
  const size_t per = (size_t)kp1 << g.logn;  // u64 per GLWE
  const size_t chunk = chunk_for(g, kp1, lv, batch);
  const size_t dig = ((chunk * lv * kp1) << g.logm), prod = g.logr ? ((chunk * kp1) << g.logm) : 0;
  cplx* scratch = nullptr;
  hipError_t e = mi::scratch_alloc((void**)&scratch, (dig + prod) * sizeof(cplx), s);
  if (e != hipSuccess) return e;
  cplx* d = scratch;
  cplx* y = g.logr ? scratch + dig : nullptr;
  const cplx* gg = reinterpret_cast<const cplx*>(ggsw);
  for (size_t b0 = 0; b0 < batch && e == hipSuccess; b0 += chunk) {
    const uint64_t nb = std::min(chunk, batch - b0);
    uint64_t* o = out + b0 * per;
    uint64_t* in = glwe + b0 * per;
    if (cmux) {
      hipLaunchKernelGGL(sub_assign_kernel, dim3(blocks_for(nb * per)), dim3(256), 0, s, in, (const uint64_t*)o,
                         (uint64_t)(nb * per));
      if ((e = hipGetLastError()) != hipSuccess) break;
    }
    e = forward(g, GlweDigitSrc{in, g.tw, g.logn, kp1, lv, base_log}, d, nb * lv * kp1, s);
    if (e != hipSuccess) break;
    e = inverse(g, MacSrc{d, gg, g.logm, g.logc, g.logr, kp1, lv}, AccSink{o, g.untw, g.logn}, y, nb * kp1, s);
  }
  const hipError_t ef = mi::scratch_free(scratch, s);
  return e != hipSuccess ? e : ef;
}

// Lanes, as launch_pbs_large (pbs_large.hip): a chunk of >= FFTG_LANE_MIN ciphertexts is split into
// mi::pbs_lane_count(fftg_default_lanes(logn)) parts on the caller's stream and pooled side streams (mi::StreamFork), launches interleaved step
// by step, so one part's memory-bound passes overlap another's transform rows.
static constexpr uint32_t FFTG_LANE_MIN = 64;
// default lane count per N, from the one-box sweep of profiles/r4/session24/lane_sweep.txt (PBS/s at 1 / 2 / 3 / 4
// lanes: 1_1 (N 512) 35.6 / 41.9 / 41.4 / 34.8 k, 3_3 (N 8192) 2.36 / 2.55 / 2.53 / 2.67 k, 4_4 (N 65536) 176 / 184 /
// 187 / 181) and the next boxes (4_4: 184.4 at 2 lanes, 180.1 at 3; 3_3: 2.67 k at 4 again, profiles/r4/session27/)
static int fftg_default_lanes(uint32_t logn) { return logn >= 16 ? 2 : logn >= 13 ? 4 : 2; }


hipError_t launch_fftg_pbs(int k, uint64_t* out, const uint64_t* lwe_in, const PbsIo& io, const double* fbsk,
                           size_t n_lwe, size_t batch, int base_log, int level, int ms_mode, const FftGenTables& t,
                           hipStream_t s) {
  using namespace fft::gen;
  if (batch == 0) return hipSuccess;
  const Geo g = geo(t);
  const uint32_t kp1 = (uint32_t)k + 1, lv = (uint32_t)level;
  const size_t per = (size_t)kp1 << g.logn;
  const size_t chunk = chunk_for(g, kp1, lv, batch);
  const size_t dig = ((chunk * lv * kp1) << g.logm), prod = g.logr ? ((chunk * kp1) << g.logm) : 0;
  const size_t acc_u64 = chunk * per;
  cplx* scratch = nullptr;
  hipError_t e = mi::scratch_alloc((void**)&scratch, (dig + prod) * sizeof(cplx) + (acc_u64 + chunk) * sizeof(uint64_t), s);
  if (e != hipSuccess) return e;
  cplx* d_all = scratch;
  cplx* y_all = g.logr ? scratch + dig : nullptr;
  uint64_t* acc_all = reinterpret_cast<uint64_t*>(scratch + dig + prod);
  uint64_t* corr_all = acc_all + acc_u64;
  const cplx* key = reinterpret_cast<const cplx*>(fbsk);
  const size_t ggsw_len = ((size_t)lv * kp1 * kp1) << g.logm;  // complex per GGSW
  struct Lane {  // ciphertexts [b0, b0 + nb) of the batch, their scratch slices, their stream
    size_t b0;
    uint32_t nb;
    hipStream_t st;
    const uint64_t* in;
    cplx *d, *y;
    uint64_t *acc, *corr;
  };
  for (size_t c0 = 0; c0 < batch && e == hipSuccess; c0 += chunk) {
    const uint32_t nb_all = (uint32_t)std::min(chunk, batch - c0);
    mi::StreamFork fork;
    const int want = nb_all >= FFTG_LANE_MIN ? std::min<int>(mi::pbs_lane_count(fftg_default_lanes(g.logn)), (int)(nb_all / 16)) : 1;
    if (want > 1) (void)fork.fork(s, want - 1);  // fewer lanes when a side stream cannot be had
    const int lanes = 1 + fork.sides();
    Lane L[1 + mi::StreamFork::MAX_SIDE];
    for (int j = 0, off = 0; j < lanes; ++j) {
      const uint32_t n = nb_all / lanes + ((uint32_t)j < nb_all % lanes ? 1u : 0u);
      L[j] = Lane{c0 + off, n, j == 0 ? s : fork.side(j - 1), lwe_in + (c0 + off) * (n_lwe + 1),
                  d_all + (((size_t)off * lv * kp1) << g.logm), y_all ? y_all + (((size_t)off * kp1) << g.logm) : nullptr,
                  acc_all + (size_t)off * per, corr_all + off};
      off += (int)n;
    }
    for (int j = 0; j < lanes && e == hipSuccess; ++j) {
      const Lane& l = L[j];
      if (ms_mode == 1)
        hipLaunchKernelGGL(body_correction_kernel, dim3(l.nb), dim3(256), 0, l.st, l.corr, l.in, (uint32_t)n_lwe,
                           g.logn + 1);
      hipLaunchKernelGGL(init_acc_kernel, dim3(blocks_for((uint64_t)l.nb * per)), dim3(256), 0, l.st, l.acc, io,
                         (uint64_t)l.b0, l.in, ms_mode == 1 ? (const uint64_t*)l.corr : nullptr, (uint32_t)n_lwe, l.nb,
                         g.logn, kp1, ms_mode);
      e = hipGetLastError();
    }
    for (uint32_t i = 0; i < (uint32_t)n_lwe && e == hipSuccess; ++i)
      for (int j = 0; j < lanes && e == hipSuccess; ++j) {
        const Lane& l = L[j];
        e = forward(g, RotDigitSrc{l.acc, l.in, g.tw, g.logn, kp1, lv, (uint32_t)n_lwe, i, base_log, ms_mode}, l.d,
                    (uint64_t)l.nb * lv * kp1, l.st);
        if (e == hipSuccess)
          e = inverse(g, MacSrc{l.d, key + i * ggsw_len, g.logm, g.logc, g.logr, kp1, lv},
                      AccSink{l.acc, g.untw, g.logn}, l.y, (uint64_t)l.nb * kp1, l.st);
      }
    for (int j = 0; j < lanes && e == hipSuccess; ++j) {
      const Lane& l = L[j];
      if (io.glwe_out) {
        hipLaunchKernelGGL(store_glwe_kernel, dim3(blocks_for((uint64_t)l.nb * per)), dim3(256), 0, l.st,
                           (const uint64_t*)l.acc, l.nb, (uint64_t)per, io, (uint64_t)l.b0);
      } else {
        const uint64_t outs = (uint64_t)l.nb * (((uint64_t)k << g.logn) + 1);
        hipLaunchKernelGGL(extract_kernel, dim3(blocks_for(outs)), dim3(256), 0, l.st,
                           out + l.b0 * (((size_t)k << g.logn) + 1), (const uint64_t*)l.acc, l.nb, g.logn,
                           (uint32_t)k, io, (uint64_t)l.b0);
      }
      e = hipGetLastError();
    }
    const hipError_t ej = fork.join();  // the caller's stream after the side lane (also on error: scratch ordering)
    if (e == hipSuccess) e = ej;
  }
  const hipError_t ef = mi::scratch_free(scratch, s);
  return e != hipSuccess ? e : ef;
}

}  // namespace mi
