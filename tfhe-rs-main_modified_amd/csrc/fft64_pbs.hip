// fft64_pbs.hip — the f64-FFT programmable bootstrap of tfhe core_crypto (the default shortint PBS path)
// on MI355X.  Reference paths relative to /root/reference/tfhe/src/core_crypto:
//   negacyclic FFT          fft_impl/fft64/math/fft/mod.rs:30-76 (Twisties), 227-356 (conversions),
//                           524-586 (forward_with_conv / backward_with_conv)
//   external product        fft_impl/fft64/crypto/ggsw.rs:483-603 (+ update_with_fmadd :617-698)
//   blind rotate / PBS      fft_impl/fft64/crypto/bootstrap.rs:294-381, 481-521
//   key conversion          fft_impl/fft64/crypto/bootstrap.rs:199-225 (forward_as_torus per polynomial)
//
// The transform: a real negacyclic polynomial of N = 2048 u64 coefficients is folded into M = 1024 complex
// values u[n] = x[n] + i x[n + M] (forward_with_conv's split), twisted by w^n = exp(i pi n / 2M)
// (Twisties::new(M)), and transformed with an M-point complex DFT (exp(-2 pi i / M) kernel).  The reference
// runs tfhe-fft's measured "unordered" plan, whose Fourier-domain order is implementation defined; here the
// order is this engine's own (documented below, exported by mi_fft64_fourier_order); the reference serialises the
// natural order, which fourier_reorder_kernel converts to and from.  Results are f64 computations, not bit-identical to the reference's
// (parity is decryption + an error bound against a numpy restatement).
//
// MI355X mapping: one wave per polynomial, 16 complex values per lane in VGPRs (lane j holds u[j + 64 m],
// m < 16), M = 16 x 64 split into three radix passes (fft_fwd below): an in-lane DFT16 over m; a DFT4 over the
// two top lane bits done in registers with gfx950's half-lane swaps (v_permlane32_swap / v_permlane16_swap);
// one LDS transpose (rows of 17, conflict-free) and an in-lane DFT16 over the low four lane bits.  The inverse
// runs the conjugate passes in reverse.  All f64 arithmetic is FMA-contracted by hand where the reference's pulp
// kernels use mul_add.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fft64_decomp.hpp"
#include "fft64_device.hpp"
#include "fft64_launch.hpp"

namespace mi {
namespace fft {

constexpr double C8 = 0.92387953251128673848;   // cos(pi / 8)
constexpr double S8 = 0.38268343236508978178;   // sin(pi / 8)
constexpr double R2 = 0.70710678118654752440;   // sqrt(1/2)

// DFT4 in place on a[o], a[o + s], a[o + 2s], a[o + 3s]; INV: exp(+2 pi i / 4) kernel
template <bool INV>
__device__ __forceinline__ void dft4(cplx* a, int o, int s) {
  const cplx a0 = a[o], a1 = a[o + s], a2 = a[o + 2 * s], a3 = a[o + 3 * s];
  const cplx s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
  const cplx r = INV ? mul_pos_i(d13) : mul_neg_i(d13);
  a[o] = cadd(s02, s13);
  a[o + 2 * s] = csub(s02, s13);
  a[o + s] = cadd(d02, r);
  a[o + 3 * s] = csub(d02, r);
}

// x * W16^e (forward: exp(-2 pi i e / 16); INV: conjugate), e in 1..9
template <bool INV>
__device__ __forceinline__ cplx tw16(cplx x, int e) {
  double c, s;  // W = c - i s (forward)
  switch (e) {
    case 1: c = C8, s = S8; break;
    case 2: c = R2, s = R2; break;
    case 3: c = S8, s = C8; break;
    case 4: return INV ? mul_pos_i(x) : mul_neg_i(x);
    case 6: c = -R2, s = R2; break;
    case 9: c = -C8, s = -S8; break;  // exp(-2 pi i 9/16) = -cos(pi/8) + i sin(pi/8)
    default: return x;
  }
  if (e == 2 || e == 6) {  // (c - i s) with |c| = |s| = R2: 2 adds + 2 muls
    const double sgn_c = (e == 2) ? 1.0 : -1.0;
    if (!INV) {  // (re + i im)(sgn R2 - i R2)
      const double re = sgn_c * x.re + x.im, im = sgn_c * x.im - x.re;
      return {re * R2, im * R2};
    } else {  // (re + i im)(sgn R2 + i R2)
      const double re = sgn_c * x.re - x.im, im = sgn_c * x.im + x.re;
      return {re * R2, im * R2};
    }
  }
  const cplx w = {c, INV ? s : -s};
  return cmul(x, w);
}

// DFT16 of a[0..16) in place, natural order in and out: X[k1 + 4 k2] = sum_m a[m] W16^(m k)
template <bool INV>
__device__ __forceinline__ void dft16(cplx (&a)[16]) {
#pragma unroll
  for (int m1 = 0; m1 < 4; ++m1) dft4<INV>(a, m1, 4);  // over m2: a[m1 + 4 k1] = b[m1][k1]
#pragma unroll
  for (int m1 = 1; m1 < 4; ++m1)
#pragma unroll
    for (int k1 = 1; k1 < 4; ++k1) a[m1 + 4 * k1] = tw16<INV>(a[m1 + 4 * k1], m1 * k1);
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) dft4<INV>(a, 4 * k1, 1);  // over m1: a[4 k1 + k2] = X[k1 + 4 k2]
  cplx t[16];
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1)
#pragma unroll
    for (int k2 = 0; k2 < 4; ++k2) t[k1 + 4 * k2] = a[4 * k1 + k2];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = t[i];
}

constexpr int ROW = 17;                // transpose row stride (complex): conflict-free both ways
constexpr int BUF = 64 * ROW;          // per-wave LDS buffer (complex): 17 KiB
constexpr int TB = 48;                 // pass-3 twiddle table: [q1 - 1][jl], q1 = 1..3

// In-register exchanges across the lane halves (gfx950 v_permlane32_swap / v_permlane16_swap): lanes 32..63
// of `a` trade places with lanes 0..31 of `b` (X = 32), or lanes 16..31 / 48..63 of `a` with lanes 0..15 /
// 32..47 of `b` (X = 16).  For a pair of registers holding elements (r, r') this turns the lane bit into the
// register bit: afterwards the low lanes hold (r: bit 0, r: bit 1) and the high lanes (r': bit 0, r': bit 1).
template <int X>
__device__ __forceinline__ void swap_dw(double& a, double& b) {
  const u64 x = __double_as_longlong(a), y = __double_as_longlong(b);
  uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32), yl = (uint32_t)y, yh = (uint32_t)(y >> 32);
  if constexpr (X == 32) {
    const auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    xl = l[0], yl = l[1], xh = h[0], yh = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    xl = l[0], yl = l[1], xh = h[0], yh = h[1];
  }
  a = __longlong_as_double((long long)(((u64)xh << 32) | xl));
  b = __longlong_as_double((long long)(((u64)yh << 32) | yl));
}
template <int X>
__device__ __forceinline__ void swap_c(cplx& a, cplx& b) {
  swap_dw<X>(a.re, b.re);
  swap_dw<X>(a.im, b.im);
}

// The per-m twist factor exp(i pi m / 32) (the host table's cm, rounded the same way from long double): built in SGPRs
// right at its use by volatile scalar moves (volatile: not hoisted out of the blind-rotation loop, where 30 live
// constants would spill), so the pass-1 twist and the inverse's untwist read no table (16 serialised LDS loads per
// transform otherwise, each a full LDS latency in front of 4 FMAs)
__device__ __forceinline__ double sconst(u64 bits) {
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)bits));
  asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(bits >> 32)));
  return __longlong_as_double((long long)(((u64)hi << 32) | lo));
}
template <bool CONJ_SCALED>  // false: exp(i pi m / 32); true: exp(-i pi m / 32) / M (the host table's cmi)
__device__ __forceinline__ cplx cm_const(int m) {
  constexpr u64 T[16][2] = {
      {0x3ff0000000000000ull, 0x0000000000000000ull},
      {0x3fefd88da3d12526ull, 0x3fb917a6bc29b42cull},
      {0x3fef6297cff75cb0ull, 0x3fc8f8b83c69a60bull},
      {0x3fee9f4156c62ddaull, 0x3fd294062ed59f06ull},
      {0x3fed906bcf328d46ull, 0x3fd87de2a6aea963ull},
      {0x3fec38b2f180bdb1ull, 0x3fde2b5d3806f63bull},
      {0x3fea9b66290ea1a3ull, 0x3fe1c73b39ae68c8ull},
      {0x3fe8bc806b151741ull, 0x3fe44cf325091dd6ull},
      {0x3fe6a09e667f3bcdull, 0x3fe6a09e667f3bcdull},
      {0x3fe44cf325091dd6ull, 0x3fe8bc806b151741ull},
      {0x3fe1c73b39ae68c8ull, 0x3fea9b66290ea1a3ull},
      {0x3fde2b5d3806f63bull, 0x3fec38b2f180bdb1ull},
      {0x3fd87de2a6aea963ull, 0x3fed906bcf328d46ull},
      {0x3fd294062ed59f06ull, 0x3fee9f4156c62ddaull},
      {0x3fc8f8b83c69a60bull, 0x3fef6297cff75cb0ull},
      {0x3fb917a6bc29b42cull, 0x3fefd88da3d12526ull}};
  const cplx c = {sconst(T[m][0]), sconst(T[m][1])};
  if (CONJ_SCALED) return {c.re * (1.0 / 1024.0), -c.im * (1.0 / 1024.0)};  // 1 / M: a power of two, exact
  return c;
}

// Forward: u[m] = folded value at n = lane + 64 m (untwisted); out: the Fourier layout.  M = 16 x 64 with
// n = j + 64 m, j = jl + 16 jh (jl = lane & 15, jh = lane >> 4), frequency f = k1 + 16 q1 + 64 q2:
//   pass 1  in-lane DFT16 over m -> k1 (register), twiddle T1[k1][j] = w^j omega^(j k1) (`t1`, twist folded in;
//           the per-m twist factor `cm` = exp(i pi m / 32) goes before the DFT16)
//   pass 2  DFT4 over jh (lane bits 5, 4) in registers: two radix-2 stages, each one half-lane swap of the
//           register pairs (r, r + 8) / (r, r + 4) and a butterfly (the W4 twiddle -i is per register)
//           -> q1 = q10 + 2 q11 in register bits 3, 2; lane bits 5, 4 now hold k1 bits 3, 2
//   pass 3  twiddle W64^(jl q1) (`t2` = [q1 - 1][jl]), LDS transpose of lane bits 0..3 <-> register bits
//           (rows of 17: conflict-free), in-lane DFT16 over jl -> q2
// Position (lane L, register R) holds f = k1 + 16 q1 + 64 R with k1 = (L & 3) | ((L >> 4) & 3) << 2,
// q1 = ((L >> 3) & 1) | ((L >> 2) & 1) << 1.
__device__ __forceinline__ void fft_fwd(cplx (&u)[16], cplx* buf, const cplx* __restrict__ t1, const cplx* t2,
                                        const cplx* __restrict__ cm, int lane) {
  (void)cm;  // the table's values are cm_const<false>'s
#pragma unroll
  for (int m = 1; m < 16; ++m) u[m] = cmul(u[m], cm_const<false>(m));
  dft16<false>(u);
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) u[k1] = cmul(u[k1], t1[k1 * 64 + lane]);
  // radix 2 over jh1 (lane bit 5): (r, r + 8) = (jh1 = 0, jh1 = 1) -> (q10 = 0, q10 = 1)
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    swap_c<32>(u[r], u[r + 8]);
    const cplx a = u[r], b = u[r + 8];
    u[r] = cadd(a, b);
    u[r + 8] = csub(a, b);
  }
  // radix 2 over jh0 (lane bit 4) with W4^(jh0 q10): (r, r + 4) = (jh0 = 0, jh0 = 1) -> (q11 = 0, q11 = 1)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (r & 4) continue;
    swap_c<16>(u[r], u[r + 4]);
    const cplx a = u[r], b = (r & 8) ? mul_neg_i(u[r + 4]) : u[r + 4];
    u[r] = cadd(a, b);
    u[r + 4] = csub(a, b);
  }
  const int jl = lane & 15;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int q1 = ((r >> 3) & 1) | (((r >> 2) & 1) << 1);
    if (q1) u[r] = cmul(u[r], t2[(q1 - 1) * 16 + jl]);
    buf[ROW * lane + r] = u[r];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int row = (lane & 48) * ROW + (lane & 15);  // element (lane' = 16 h + jl, r = lane & 15)
#pragma unroll
  for (int j = 0; j < 16; ++j) u[j] = buf[row + ROW * j];
  dft16<false>(u);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inverse of fft_fwd (the conjugate transpose of every pass in reverse order), including the 1/M normalisation
// and the untwist (`cmi` = exp(-i pi m / 32) / M: the output is the torus value, ready for add_torus /
// from_torus).
__device__ __forceinline__ void fft_inv(cplx (&u)[16], cplx* buf, const cplx* __restrict__ t1, const cplx* t2,
                                        const cplx* __restrict__ cmi, int lane) {
  dft16<true>(u);
  const int row = (lane & 48) * ROW + (lane & 15);
#pragma unroll
  for (int j = 0; j < 16; ++j) buf[row + ROW * j] = u[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int jl = lane & 15;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    u[r] = buf[ROW * lane + r];
    const int q1 = ((r >> 3) & 1) | (((r >> 2) & 1) << 1);
    if (q1) u[r] = cmulc(u[r], t2[(q1 - 1) * 16 + jl]);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if (r & 4) continue;
    const cplx a = u[r], b = u[r + 4];
    u[r] = cadd(a, b);
    u[r + 4] = (r & 8) ? mul_pos_i(csub(a, b)) : csub(a, b);
    swap_c<16>(u[r], u[r + 4]);
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const cplx a = u[r], b = u[r + 8];
    u[r] = cadd(a, b);
    u[r + 8] = csub(a, b);
    swap_c<32>(u[r], u[r + 8]);
  }
#pragma unroll
  for (int k1 = 0; k1 < 16; ++k1) u[k1] = cmulc(u[k1], t1[k1 * 64 + lane]);
  dft16<true>(u);
  (void)cmi;  // the table's values are cm_const<true>'s
#pragma unroll
  for (int m = 0; m < 16; ++m) u[m] = cmul(u[m], cm_const<true>(m));
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct Tables {
  const cplx* t1;   // [16][64] forward pass-1 twiddles (twist folded in)
  const cplx* t2;   // [3][16] W64^(jl q1), q1 = 1..3
  const cplx* cm;   // [16] exp(i pi m / 32)
  const cplx* cmi;  // [16] exp(-i pi m / 32) / M
};

constexpr int N = 2048, M = 1024, NPL = N / 64;  // 32 coefficients per lane

// ---- forward_as_torus / backward_as_torus over a batch of polynomials (key conversion, tests) ------
// one wave per polynomial; `fourier`: batch x 1024 complex in the Fourier layout (position reg * 64 + lane)
__global__ __launch_bounds__(64) void fwd_torus_kernel(cplx* __restrict__ fourier, const u64* __restrict__ std_,
                                                       uint64_t batch, Tables tb) {
  __shared__ cplx buf[BUF];
  __shared__ cplx t2[TB];
  const int lane = threadIdx.x;
  if (lane < TB) t2[lane] = tb.t2[lane];
  __syncthreads();
  const uint64_t b = blockIdx.x;
  if (b >= batch) return;
  const u64* x = std_ + b * N;
  constexpr double NORM = 1.0 / 18446744073709551616.0;  // 2^-64 (convert_forward_torus)
  cplx u[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) u[m] = {s64_to_f64(x[lane + 64 * m]) * NORM, s64_to_f64(x[M + lane + 64 * m]) * NORM};
  fft_fwd(u, buf, tb.t1, t2, tb.cm, lane);
  cplx* out = fourier + b * M;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[r * 64 + lane] = u[r];
}

__global__ __launch_bounds__(64) void bwd_torus_kernel(u64* __restrict__ std_, const cplx* __restrict__ fourier,
                                                       uint64_t batch, int add, Tables tb) {
  __shared__ cplx buf[BUF];
  __shared__ cplx t2[TB];
  const int lane = threadIdx.x;
  if (lane < TB) t2[lane] = tb.t2[lane];
  __syncthreads();
  const uint64_t b = blockIdx.x;
  if (b >= batch) return;
  const cplx* in = fourier + b * M;
  cplx u[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) u[r] = in[r * 64 + lane];
  fft_inv(u, buf, tb.t1, t2, tb.cmi, lane);
  u64* x = std_ + b * N;
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const u64 re = from_torus_scaled(u[m].re * 0x1p64), im = from_torus_scaled(u[m].im * 0x1p64);
    x[lane + 64 * m] = add ? x[lane + 64 * m] + re : re;
    x[M + lane + 64 * m] = add ? x[M + lane + 64 * m] + im : im;
  }
}

// ---- Fourier order interchange (tfhe-fft/src/unordered.rs:943-1020, serialize / deserialize_fourier_buffer) ----
// The reference serialises a Fourier polynomial in the natural DFT order (element i = frequency i), whatever its
// plan's internal order.  Engine position p = 64 r + l holds frequency fft64_frequency(r, l) = 64 r + f(l), a
// permutation of the low six bits only.  One 256-lane workgroup per polynomial stages it in LDS (coalesced 16-B
// reads), then writes the other order coalesced; in place is safe (every read lands before the barrier).
__device__ __forceinline__ int low6_frequency(int l) {  // f(l): see fft64_frequency (fft64_launch.hpp)
  return (l & 3) | (((l >> 4) & 3) << 2) | (((l >> 3) & 1) << 4) | (((l >> 2) & 1) << 5);
}
__device__ __forceinline__ int low6_position(int k) {  // f^-1
  return (k & 3) | (((k >> 5) & 1) << 2) | (((k >> 4) & 1) << 3) | (((k >> 2) & 3) << 4);
}
template <bool TO_STD>
__global__ __launch_bounds__(256) void fourier_reorder_kernel(cplx* out, const cplx* in, uint64_t polys) {
  __shared__ cplx buf[M];
  const uint64_t b = blockIdx.x;
  if (b >= polys) return;
  const cplx* src = in + b * M;
#pragma unroll
  for (int i = 0; i < M / 256; ++i) buf[threadIdx.x + 256 * i] = src[threadIdx.x + 256 * i];
  __syncthreads();
  cplx* dst = out + b * M;
#pragma unroll
  for (int i = 0; i < M / 256; ++i) {
    const int j = threadIdx.x + 256 * i, hi = j & ~63, lo = j & 63;
    dst[j] = buf[hi | (TO_STD ? low6_position(lo) : low6_frequency(lo))];
  }
}

// Synchronisation of the (K + 1) waves of one ciphertext.  A workgroup holding one ciphertext uses its barrier;
// with several ciphertexts per workgroup each wave publishes a step counter in LDS and waits for its partners'
// (s_sleep between polls), so the ciphertexts of a workgroup do not have to run in lockstep.
template <int K, bool WG_BARRIER>
struct PairSync {
  uint32_t* flags;  // this ciphertext's K + 1 counters (LDS)
  int w;
  uint32_t count;
  __device__ __forceinline__ void sync() {
    if (WG_BARRIER) {
      __syncthreads();
      return;
    }
    ++count;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    *reinterpret_cast<volatile uint32_t*>(flags + w) = count;
    // wait (in one asm block, so the register allocator sees straight-line code) until every partner's counter
    // has reached ours: poll with ds_read_b32, the decision on the first lane's value (all lanes read the same
    // address), s_sleep between polls
#pragma unroll
    for (int o = 0; o < K; ++o) {
      const int rr = o + (o >= w ? 1 : 0);
      const uint32_t lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(flags + rr);
      uint32_t v, sv;
      asm volatile(
          "s_waitcnt lgkmcnt(0)\n"
          "1:\n\t"
          "ds_read_b32 %0, %2\n\t"
          "s_waitcnt lgkmcnt(0)\n\t"
          "v_readfirstlane_b32 %1, %0\n\t"
          "s_cmp_ge_u32 %1, %3\n\t"
          "s_cbranch_scc1 2f\n\t"
          "s_sleep 1\n\t"
          "s_branch 1b\n"
          "2:"
          : "=&v"(v), "=&s"(sv)
          : "v"(lds), "s"(count)
          : "memory", "scc");
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
};

// ---- external product on registers ----------------------------------------------------------------
// Wave w (< K + 1, wave-uniform) owns GLWE polynomial w.  in: ct1[NPL] = this wave's polynomial of the GLWE
// to decompose (coefficient lane + 64 r); acc[r] += from_torus(the product's polynomial w).  `ggsw`: level x
// (K+1) rows x (K+1) cols x M complex (Fourier layout), highest level first, as the reference's
// FourierGgswCiphertext.  `pair` = this ciphertext's (K+1) per-wave LDS buffers; t1 / t2 the twiddle tables
// (LDS copies in the PBS / external-product kernels).
template <int K, bool L1, bool WGB>
__device__ __forceinline__ void ext_product_add(u64 (&acc)[NPL], const u64 (&ct1)[NPL], const cplx* __restrict__ ggsw,
                                                int base_log, int level, cplx* pair, const cplx* t1, const cplx* t2,
                                                const cplx* cm, const cplx* cmi, int w, int lane,
                                                PairSync<K, WGB>& ps) {
  cplx* buf = pair + w * BUF;
  cplx y[16];
  if (L1) {
    cplx u[16];
    if (base_log <= 31) {  // uniform: digits from the high words, exact in int32
#pragma unroll
      for (int m = 0; m < 16; ++m)
        u[m] = {(double)decompose_l1_hi((uint32_t)(ct1[m] >> 32), base_log),
                (double)decompose_l1_hi((uint32_t)(ct1[m + 16] >> 32), base_log)};
    } else {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        u64 s0 = decomp_init_native(ct1[m], base_log, 1), s1 = decomp_init_native(ct1[m + 16], base_log, 1);
        const u64 d0 = decompose_one_level(base_log, s0), d1 = decompose_one_level(base_log, s1);
        u[m] = {s64_to_f64(d0), s64_to_f64(d1)};  // convert_forward_integer: into_signed as f64
      }
    }
    fft_fwd(u, buf, t1, t2, cm, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) buf[r * 64 + lane] = u[r];
    // update_with_fmadd: y_w = sum_rr X_rr * G[rr][w] (own transform from registers, the other K from LDS).
    // Branch-free (the other rows are rr = o + (o >= w), o < K); the key rows are loaded in batches of HB positions,
    // each issued one batch ahead (the first before the exchange barrier, so its latency overlaps the wait).  One-box
    // A/Bs: in the 4-ciphertext PBS workgroups HB = 4 is 0.9 % faster than 2 and HB = 8 1.9 % slower than 4
    // (profiles/r3/fft_hb*_ab); the one-ciphertext external-product workgroups (WGB) lost 10 % with 4, so they keep 2.
    const cplx* gw = ggsw + (size_t)(w * (K + 1) + w) * M + lane;
    const cplx* go[K];
    const cplx* xo[K];
#pragma unroll
    for (int o = 0; o < K; ++o) {
      const int rr = o + (o >= w ? 1 : 0);
      go[o] = ggsw + (size_t)(rr * (K + 1) + w) * M + lane;
      xo[o] = pair + rr * BUF + lane;
    }
    constexpr int HB = WGB ? 2 : 4;
    cplx kw[HB], ko[K][HB];
#pragma unroll
    for (int j = 0; j < HB; ++j) {
      kw[j] = gw[j * 64];
#pragma unroll
      for (int o = 0; o < K; ++o) ko[o][j] = go[o][j * 64];
    }
    ps.sync();
#pragma unroll
    for (int h = 0; h < 16 / HB; ++h) {
#pragma unroll
      for (int j = 0; j < HB; ++j) {
        const int r = h * HB + j;
        cplx a = cmul(u[r], kw[j]);
#pragma unroll
        for (int o = 0; o < K; ++o) a = cfma(xo[o][r * 64], ko[o][j], a);
        y[r] = a;
      }
      if (h + 1 < 16 / HB) {
#pragma unroll
        for (int j = 0; j < HB; ++j) {
          const int r = (h + 1) * HB + j;
          kw[j] = gw[r * 64];
#pragma unroll
          for (int o = 0; o < K; ++o) ko[o][j] = go[o][r * 64];
        }
      }
    }
    ps.sync();
  } else {
    u64 st[NPL];
#pragma unroll
    for (int r = 0; r < NPL; ++r) st[r] = decomp_init_native(ct1[r], base_log, level);
#pragma unroll
    for (int r = 0; r < 16; ++r) y[r] = {0.0, 0.0};
#pragma unroll 1
    for (int li = 0; li < level; ++li) {
      cplx u[16];
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        const u64 d0 = decompose_one_level(base_log, st[m]), d1 = decompose_one_level(base_log, st[m + 16]);
        u[m] = {s64_to_f64(d0), s64_to_f64(d1)};
      }
      fft_fwd(u, buf, t1, t2, cm, lane);
#pragma unroll
      for (int r = 0; r < 16; ++r) buf[r * 64 + lane] = u[r];
      ps.sync();
      // the decomposition iterator yields the least significant level first, which the GGSW stores first
      const cplx* mat = ggsw + (size_t)li * (K + 1) * (K + 1) * M;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        cplx a = y[r];
#pragma unroll
        for (int rr = 0; rr <= K; ++rr)
          a = cfma(pair[rr * BUF + r * 64 + lane], mat[(size_t)(rr * (K + 1) + w) * M + r * 64 + lane], a);
        y[r] = a;
      }
      ps.sync();
    }
  }
  fft_inv(y, buf, t1, t2, cmi, lane);
#pragma unroll
  for (int m = 0; m < 16; ++m) {  // convert_add_backward_torus
    add_torus(acc[m], y[m].re);
    add_torus(acc[m + 16], y[m].im);
  }
}

// Workgroup layout of the batched kernels: CT ciphertexts x (K + 1) waves; LDS = CT (K + 1) transpose /
// exchange buffers + the two twiddle tables, copied once per workgroup.
template <int K, int CT>
struct Wg {
  static constexpr int WAVES = CT * (K + 1), THREADS = 64 * WAVES;
  cplx bufs[WAVES * BUF];
  cplx t1[16 * 64];
  cplx t2[TB];
  cplx cm[16], cmi[16];
  uint32_t flags[WAVES];
};

template <int K, int CT>
__device__ __forceinline__ void load_tables(Wg<K, CT>& wg, const Tables& tb) {
  for (int i = threadIdx.x; i < 16 * 64; i += Wg<K, CT>::THREADS) wg.t1[i] = tb.t1[i];
  if (threadIdx.x < TB) wg.t2[threadIdx.x] = tb.t2[threadIdx.x];
  if (threadIdx.x < 16) {
    wg.cm[threadIdx.x] = tb.cm[threadIdx.x];
    wg.cmi[threadIdx.x] = tb.cmi[threadIdx.x];
  }
  if (threadIdx.x < Wg<K, CT>::WAVES) wg.flags[threadIdx.x] = 0;
  __syncthreads();
}

// EXT : out[b] += GGSW (.) glwe[b]                       (add_external_product_assign)
// CMUX: glwe[b] -= out[b]; out[b] += GGSW (.) glwe[b]    (cmux: ct1 -= ct0; ct0 += ext(ct1))
template <int K, bool CMUX, bool L1, int CT>
__device__ __forceinline__ void ext_product_body(u64* __restrict__ out, u64* __restrict__ glwe,
                                                 const cplx* __restrict__ ggsw, uint32_t batch, int base_log,
                                                 int level, const Tables& tb, Wg<K, CT>& wg) {
  load_tables(wg, tb);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ct = wave / (K + 1), w = wave % (K + 1);
  const uint32_t b0 = blockIdx.x * CT + ct;
  const bool valid = b0 < batch;  // every wave takes part in the barriers
  const uint32_t b = valid ? b0 : batch - 1;
  u64* in = glwe + ((size_t)b * (K + 1) + w) * N;
  u64* o = out + ((size_t)b * (K + 1) + w) * N;
  u64 ct1[NPL], acc[NPL];
#pragma unroll
  for (int r = 0; r < NPL; ++r) {
    ct1[r] = in[lane + 64 * r];
    acc[r] = o[lane + 64 * r];
    if (CMUX) {
      ct1[r] -= acc[r];
      if (valid) in[lane + 64 * r] = ct1[r];
    }
  }
  PairSync<K, CT == 1> ps{wg.flags + ct * (K + 1), w, 0u};
  ext_product_add<K, L1>(acc, ct1, ggsw, base_log, level, wg.bufs + ct * (K + 1) * BUF, wg.t1, wg.t2, wg.cm, wg.cmi, w,
                         lane, ps);
  if (valid) {
#pragma unroll
    for (int r = 0; r < NPL; ++r) o[lane + 64 * r] = acc[r];
  }
}

// One GLWE per workgroup (the external product / CMUX entry points; the PBS kernel below batches 4 ciphertexts
// per workgroup for the shortint shape).
template <int K, bool CMUX, bool L1>
__global__ __launch_bounds__(64 * (K + 1)) void ext_product_kernel(u64* __restrict__ out, u64* __restrict__ glwe,
                                                                   const cplx* __restrict__ ggsw, uint32_t batch,
                                                                   int base_log, int level, Tables tb) {
  __shared__ Wg<K, 1> wg;
  ext_product_body<K, CMUX, L1, 1>(out, glwe, ggsw, batch, base_log, level, tb, wg);
}
constexpr int CT_FAST = 4;
// ---- programmable bootstrap (bootstrap.rs:481-521 + blind_rotate_assign :294-381) -------------------
// lwe_in: batch x (n + 1); lut: (K+1) x N shared; fbsk: n x level x (K+1) x (K+1) x M complex;
// lwe_out: batch x (K N + 1).  ms_mode: 0 standard, 1 centered, 2 pre-switched (values in [0, 2N)).
// With several ciphertexts per workgroup a mask element that switches to 0 is not skipped (the reference
// skips it, bootstrap.rs:336): its CMUX difference is the zero polynomial, whose digits, transforms and
// products are exactly 0, so the accumulator is unchanged bit for bit either way.
// io (pbs_io.hpp): the item's LUT (shared, per item or indexed) and the output form (LWE of sample 0, or the rotated
// GLWE itself: blind_rotate_assign, fft64_pbs.rs:186-250).  An item whose LUT index is out of range runs on LUT 0 like a
// padding item and writes nothing.
template <int K, bool L1, int CT>
__device__ __forceinline__ void pbs_body(u64* __restrict__ lwe_out, const u64* __restrict__ lwe_in, const PbsIo& io,
                                         const cplx* __restrict__ fbsk, uint32_t n_lwe,
                                         uint32_t batch, int base_log, int level, int ms_mode, const Tables& tb,
                                         Wg<K, CT>& wg) {
  constexpr int TG = 64 * (K + 1);
  constexpr unsigned LOG_MOD = 12;  // PolynomialSize(2048)::to_blind_rotation_input_modulus_log
  load_tables(wg, tb);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int ct = wave / (K + 1), w = wave % (K + 1);
  const uint32_t b0 = blockIdx.x * CT + ct;
  const uint32_t b = b0 < batch ? b0 : batch - 1;
  const u64* lut = io.lut_for(b, (uint64_t)(K + 1) * N);
  const bool valid = b0 < batch && lut;  // every wave takes part in the barriers
  if (!lut) lut = io.lut;
  const u64* lwe = lwe_in + (size_t)b * (n_lwe + 1);
  const size_t ggsw_len = (size_t)level * (K + 1) * (K + 1) * M;
  cplx* pair = wg.bufs + ct * (K + 1) * BUF;
  u64* mine = reinterpret_cast<u64*>(pair + w * BUF);  // this wave's rotation buffer (2048 u64 = 16 KiB)

  u64 body_corr = 0;
  if (ms_mode == 1)
    body_corr = centered_body_correction<TG>(lwe, n_lwe, LOG_MOD, w * 64 + lane, reinterpret_cast<u64*>(pair));
  const u64 body = (ms_mode == 2) ? (lwe[n_lwe] & (2 * N - 1)) : modulus_switch(lwe[n_lwe] + body_corr, LOG_MOD);

  // local accumulator = LUT / X^body (polynomial_wrapping_monic_monomial_div)
  u64 acc[NPL];
  {
    const u64* lp = lut + (size_t)w * N;
    const int full = (int)(body / N) & 1, rem = (int)(body % N);
#pragma unroll
    for (int r = 0; r < NPL; ++r) {
      const int m = lane + 64 * r;  // div: new[m] = old[(m + rem) % N], negated for m >= N - rem
      u64 v = lp[(m + rem) & (N - 1)];
      if (full ^ (m >= N - rem)) v = (u64)0 - v;
      acc[r] = v;
    }
  }

  const uint32_t lane_bytes = (uint32_t)lane * 8u;
  PairSync<K, CT == 1> ps{wg.flags + ct * (K + 1), w, 0u};

  for (uint32_t i = 0; i < n_lwe; ++i) {
    const uint32_t a = (uint32_t)((ms_mode == 2) ? (lwe[i] & (2 * N - 1)) : modulus_switch(lwe[i], LOG_MOD));
    if (CT == 1 && a == 0) continue;  // bootstrap.rs:336 (uniform per workgroup)
    const bool full = (a >> 11) & 1u;
    const int rem = (int)(a & (N - 1));
#pragma unroll
    for (int r = 0; r < NPL; ++r) mine[lane + 64 * r] = acc[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // polynomial_wrapping_monic_monomial_mul_and_subtract: ct1[e] = s_e acc[(e - rem) mod N] - acc[e], s_e = -1 iff
    // full ^ (e < rem).  With m = s_e < 0 ? ~0 : 0:  s_e v - acc = (v ^ m) - (acc + m).
    // Source of e = lane + 64 r: (e - rem) mod N at byte rot + 512 r (no wrap: e >= rem) or that minus 16 KiB.
    // Lanes >= rem never wrap; below rem, e < rem holds exactly for the wrapped sources, which are the
    // in-range ones — so one per-lane base (A or A - 16 KiB) selected by the same compare as the sign, and the
    // 512 r in the instruction's offset field.
    const uint32_t rot = (lane_bytes - (uint32_t)rem * 8u) & (8u * N - 1u);
    const char* base_a = reinterpret_cast<const char*>(mine) + rot;
    const char* base_b = lane >= rem ? base_a : base_a - 8 * N;
    u64 ct1[NPL];
#pragma unroll
    for (int r = 0; r < NPL; ++r) {
      const bool wrapped = lane < rem - 64 * r;
      const u64 v = *reinterpret_cast<const u64*>((wrapped ? base_a : base_b) + 512 * r);
      const uint32_t m = (wrapped != full) ? ~0u : 0u;
      const u64 mm = ((u64)m << 32) | m;
      ct1[r] = (v ^ mm) - (acc[r] + mm);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    ext_product_add<K, L1>(acc, ct1, fbsk + (size_t)i * ggsw_len, base_log, level, pair, wg.t1, wg.t2, wg.cm, wg.cmi, w,
                           lane, ps);
  }

  if (io.glwe_out) {  // the rotated accumulator (the LUT was divided by X^body before the loop)
    if (valid) {
      u64* g = io.glwe_out + ((size_t)b * (K + 1) + w) * N;
#pragma unroll
      for (int r = 0; r < NPL; ++r) g[lane + 64 * r] = acc[r];
    }
    return;
  }
  // extract_lwe_sample_from_glwe_ciphertext (glwe_sample_extraction.rs:89-160), nth = 0
  u64* out = lwe_out + (size_t)b * (K * N + 1);
  if (w < K) {
#pragma unroll
    for (int r = 0; r < NPL; ++r) mine[lane + 64 * r] = acc[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (valid) {
#pragma unroll
      for (int r = 0; r < NPL; ++r) {
        const int j = lane + 64 * r;
        out[(size_t)w * N + j] = (j == 0) ? mine[0] : (u64)0 - mine[N - j];
      }
    }
  } else if (lane == 0 && valid) {
    out[(size_t)K * N] = acc[0];
  }
}

template <int K, bool L1>
__global__ __launch_bounds__(64 * (K + 1)) void pbs_kernel(u64* __restrict__ lwe_out, const u64* __restrict__ lwe_in,
                                                           PbsIo io, const cplx* __restrict__ fbsk,
                                                           uint32_t n_lwe, uint32_t batch, int base_log, int level,
                                                           int ms_mode, Tables tb) {
  __shared__ Wg<K, 1> wg;
  pbs_body<K, L1, 1>(lwe_out, lwe_in, io, fbsk, n_lwe, batch, base_log, level, ms_mode, tb, wg);
}
__global__ __launch_bounds__(128 * CT_FAST) __attribute__((amdgpu_waves_per_eu(2))) void pbs_kernel_k1l1(
    u64* __restrict__ lwe_out, const u64* __restrict__ lwe_in, PbsIo io,
    const cplx* __restrict__ fbsk, uint32_t n_lwe, uint32_t batch, int base_log, int level, int ms_mode, Tables tb) {
  __shared__ Wg<1, CT_FAST> wg;
  pbs_body<1, true, CT_FAST>(lwe_out, lwe_in, io, fbsk, n_lwe, batch, base_log, level, ms_mode, tb, wg);
}

}  // namespace fft

// ---- launchers ----------------------------------------------------------------------------------
static fft::Tables tables(const FftTables& t) {
  return {reinterpret_cast<const fft::cplx*>(t.t1), reinterpret_cast<const fft::cplx*>(t.t2),
          reinterpret_cast<const fft::cplx*>(t.cm), reinterpret_cast<const fft::cplx*>(t.cmi)};
}

hipError_t launch_fft64_fwd_torus(double* fourier, const uint64_t* std_, size_t batch, const FftTables& t,
                                  hipStream_t s) {
  if (batch == 0) return hipSuccess;
  hipLaunchKernelGGL(fft::fwd_torus_kernel, dim3((unsigned)batch), dim3(64), 0, s,
                     reinterpret_cast<fft::cplx*>(fourier), std_, (uint64_t)batch, tables(t));
  return hipGetLastError();
}

hipError_t launch_fft64_bwd_torus(uint64_t* std_, const double* fourier, size_t batch, bool add, const FftTables& t,
                                  hipStream_t s) {
  if (batch == 0) return hipSuccess;
  hipLaunchKernelGGL(fft::bwd_torus_kernel, dim3((unsigned)batch), dim3(64), 0, s, std_,
                     reinterpret_cast<const fft::cplx*>(fourier), (uint64_t)batch, add ? 1 : 0, tables(t));
  return hipGetLastError();
}

hipError_t launch_fft64_reorder(double* out, const double* in, size_t polys, bool to_standard, hipStream_t s) {
  if (polys == 0) return hipSuccess;
  auto* o = reinterpret_cast<fft::cplx*>(out);
  const auto* i = reinterpret_cast<const fft::cplx*>(in);
  if (to_standard)
    hipLaunchKernelGGL(fft::fourier_reorder_kernel<true>, dim3((unsigned)polys), dim3(256), 0, s, o, i, (uint64_t)polys);
  else
    hipLaunchKernelGGL(fft::fourier_reorder_kernel<false>, dim3((unsigned)polys), dim3(256), 0, s, o, i, (uint64_t)polys);
  return hipGetLastError();
}

template <int K, bool CMUX, bool L1>
static hipError_t ext_one(uint64_t* out, uint64_t* glwe, const fft::cplx* g, size_t batch, int base_log, int level,
                          const FftTables& t, hipStream_t s) {
  hipLaunchKernelGGL((fft::ext_product_kernel<K, CMUX, L1>), dim3((unsigned)batch), dim3(64 * (K + 1)), 0, s, out, glwe,
                     g, (uint32_t)batch, base_log, level, tables(t));
  return hipGetLastError();
}

template <int K>
static hipError_t ext_k(bool cmux, uint64_t* out, uint64_t* glwe, const double* ggsw, size_t batch, int base_log,
                        int level, const FftTables& t, hipStream_t s) {
  const auto* g = reinterpret_cast<const fft::cplx*>(ggsw);
  if (level == 1)
    return cmux ? ext_one<K, true, true>(out, glwe, g, batch, base_log, level, t, s)
                : ext_one<K, false, true>(out, glwe, g, batch, base_log, level, t, s);
  return cmux ? ext_one<K, true, false>(out, glwe, g, batch, base_log, level, t, s)
              : ext_one<K, false, false>(out, glwe, g, batch, base_log, level, t, s);
}

hipError_t launch_fft64_ext_product(int k, bool cmux, uint64_t* out, uint64_t* glwe, const double* ggsw, size_t batch,
                                    int base_log, int level, const FftTables& t, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (k == 1) return ext_k<1>(cmux, out, glwe, ggsw, batch, base_log, level, t, s);
  if (k == 2) return ext_k<2>(cmux, out, glwe, ggsw, batch, base_log, level, t, s);
  return hipErrorInvalidValue;
}

template <int K, bool L1>
static hipError_t pbs_one(uint64_t* out, const uint64_t* lwe_in, const PbsIo& lut, const fft::cplx* g, size_t n_lwe,
                          size_t batch, int base_log, int level, int ms_mode, const FftTables& t, hipStream_t s) {
  if (K == 1 && L1)
    hipLaunchKernelGGL(fft::pbs_kernel_k1l1, dim3((unsigned)((batch + fft::CT_FAST - 1) / fft::CT_FAST)),
                       dim3(128 * fft::CT_FAST), 0, s, out, lwe_in, lut, g, (uint32_t)n_lwe, (uint32_t)batch, base_log,
                       level, ms_mode, tables(t));
  else
    hipLaunchKernelGGL((fft::pbs_kernel<K, L1>), dim3((unsigned)batch), dim3(64 * (K + 1)), 0, s, out, lwe_in, lut, g,
                       (uint32_t)n_lwe, (uint32_t)batch, base_log, level, ms_mode, tables(t));
  return hipGetLastError();
}

hipError_t launch_fft64_pbs(int k, uint64_t* out, const uint64_t* lwe_in, const PbsIo& lut, const double* fbsk,
                            size_t n_lwe, size_t batch, int base_log, int level, int ms_mode, const FftTables& t,
                            hipStream_t s) {
  if (batch == 0) return hipSuccess;
  const auto* g = reinterpret_cast<const fft::cplx*>(fbsk);
  const bool l1 = level == 1;
  if (k == 1)
    return l1 ? pbs_one<1, true>(out, lwe_in, lut, g, n_lwe, batch, base_log, level, ms_mode, t, s)
              : pbs_one<1, false>(out, lwe_in, lut, g, n_lwe, batch, base_log, level, ms_mode, t, s);
  if (k == 2)
    return l1 ? pbs_one<2, true>(out, lwe_in, lut, g, n_lwe, batch, base_log, level, ms_mode, t, s)
              : pbs_one<2, false>(out, lwe_in, lut, g, n_lwe, batch, base_log, level, ms_mode, t, s);
  return hipErrorInvalidValue;
}

}  // namespace mi
