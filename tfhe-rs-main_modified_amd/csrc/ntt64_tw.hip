// ntt64_tw.hip — "twisted" N = 2048 Goldilocks transform: shift-only butterflies.
//
// Same transform as Plan::fwd / Plan::inv of the Solinas plan (reference:
// tfhe-ntt/src/prime64/generic_solinas.rs:449-514, twiddles prime64.rs:159-204), bit-identical
// because every value it writes is the canonical residue, computed through an
// algebraically equivalent factorisation that trades general 64x64 modular multiplies for shifts:
//
//   forward = the reference's first 5 merged-CT stages (m = 1..16): their twiddles twid[m+i] are
//             powers of two in the Solinas root tower (psi^64 = 8), so b*w is a shift + fold;
//           -> twist: element 64 i + j (block i, 0 <= j < 64) times rho_i^j, rho_i = psi^(2 rev5(i) + 1)
//              (the only general multiplies left: 2048 per transform instead of 11264);
//           -> per 64-element block a cyclic CT DFT with omega = psi^64 = 8 (natural in, bit-reversed
//              out): every twiddle is 2^(3k).
//   inverse = the mirror (GS stages with the inverse exponents, untwist by rho_i^-j), unnormalised.
// tools/gen_tw_tables.py derives the exponent tables from the plan's twiddles and checks the
// factorisation against the oracle; tests/test_ntt_gpu.py checks this kernel bit-exactly.
//
// MI355X mapping: one wave (64 lanes) per polynomial, 32 coefficients per lane in VGPRs.
//   W0 layout (lane = j, register = i): the 5 twisted-out stages act on register bits, all
//      exponents compile-time; loads/stores are 512-B coalesced rows.
//   one in-wave LDS transpose (two 8 KiB halves, row stride 34 u64: conflict-free both ways),
//   W1 layout (lane = 2 i + j0, register = j >> 1): cyclic stages on register bits, compile-time.
//   last cyclic stage (bit j0, across lane pairs): one DPP quad_perm swap regroups the pairs so each
//      lane owns 16 whole butterflies (lane-variable twiddle, one multiply each) and 16-B outputs.
// No __syncthreads: every wave owns its LDS slice.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_tw_tables.hpp"
#include "ntt64_tw_asm.hpp"
#include "ntt64_tw_body.hpp"

namespace mi {
namespace tw {

static constexpr u64 P = GL_P;
static constexpr u64 EPS = GL_EPS;
static constexpr int ROW = 34;  // LDS row stride (u64) of the 32 x 32 transpose half
static constexpr int WAVE_LDS = 32 * ROW;

template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- arithmetic on "semi" values (any u64, representing x mod p) ----------------------------
__device__ __forceinline__ u64 canon(u64 x) {
  const u64 y = x + EPS;
  return (y < x) ? y : x;  // y wrapped <=> x >= p
}
// a semi + t canonical -> semi (a + t - 2^64 < p, so one fold suffices)
__device__ __forceinline__ u64 add_sc(u64 a, u64 t) {
  const u64 s = a + t;
  return (s < a) ? s + EPS : s;
}
// a semi - t canonical -> semi (a - t + 2^64 > EPS when it borrows)
__device__ __forceinline__ u64 sub_sc(u64 a, u64 t) {
  const u64 d = a - t;
  return (a < t) ? d - EPS : d;
}
// both semi
__device__ __forceinline__ u64 add_ff(u64 a, u64 b) {
  u64 s = a + b;
  if (s < a) {
    const u64 s2 = s + EPS;
    s = (s2 < s) ? s2 + EPS : s2;
  }
  return s;
}
__device__ __forceinline__ u64 sub_ff(u64 a, u64 b) {
  u64 d = a - b;
  if (a < b) {
    const u64 d2 = d - EPS;
    d = (d2 > d) ? d2 - EPS : d2;
  }
  return d;
}

// x * 2^S mod p for a compile-time S < 192, returned as a canonical magnitude m with
// x * 2^S = (neg<S>() ? -m : m).  2^96 = -1, and for 64 <= S % 96 < 96, 2^S = -2^-(96 - S % 96).
template <int S>
__device__ __forceinline__ constexpr bool neg() {
  return (S >= 96) != ((S % 96) >= 64);
}
template <int S>
__device__ __forceinline__ u64 tmul(u64 x) {
  constexpr int E = S % 96;
  if constexpr (E == 0) {
    return canon(x);
  } else if constexpr (E < 64) {
    return Goldilocks::reduce128(x << E, x >> (64 - E));  // 128-bit x * 2^E, hi < 2^E
  } else {
    constexpr int K = 96 - E;  // x * 2^-K = (x >> K) + u - u * 2^32, u = low K bits of x moved to the top of a word
    const u64 bh = x >> K;
    const u64 u = (u64)(uint32_t)(x << (32 - K));
    const u64 X = bh + u;
    const u64 U = u << 32;
    const u64 d = X - U;
    return (X < U) ? d - EPS : d;
  }
}

// CT butterfly (a, b) -> (a + b w, a - b w), w = 2^S
template <int S>
__device__ __forceinline__ void ct(u64& a, u64& b) {
  const u64 t = tmul<S>(b);
  const u64 a0 = a;
  if constexpr (neg<S>()) {
    a = sub_sc(a0, t);
    b = add_sc(a0, t);
  } else {
    a = add_sc(a0, t);
    b = sub_sc(a0, t);
  }
}
// GS butterfly (a, b) -> (a + b, (a - b) w), w = 2^S
template <int S>
__device__ __forceinline__ void gs(u64& a, u64& b) {
  const u64 a0 = a, b0 = b;
  a = add_ff(a0, b0);
  b = tmul<S>(neg<S>() ? sub_ff(b0, a0) : sub_ff(a0, b0));
}

__device__ __forceinline__ u64 swap_pair_lanes(u64 v) {  // value of lane ^ 1 (DPP quad_perm [1,0,3,2])
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), 0xB1, 0xF, 0xF, false);
  return ((u64)(uint32_t)hi << 32) | (uint32_t)lo;
}

__host__ __device__ constexpr u64 pow2mod(int e) {
  u64 v = 1;
  for (int i = 0; i < e; ++i) {
    const u64 d = v + v;
    v = (d < v || d >= P) ? d - P : d;  // d < v: wrapped, true value d + 2^64 - p = d + EPS
  }
  return v;
}

// ---- layouts ---------------------------------------------------------------------------------
// W0: x[r] = element 64 r + lane.   W1: x[r] = element 64 (lane >> 1) + 2 r + (lane & 1).
// Both transposes run in two 8 KiB halves so that only 16 extra values per lane are live.
// Forward halves split by j (LDS slot (i, j - 32h) = i * ROW + j - 32h, ROW = 34); inverse halves
// split by i (slot (i - 16h, j) = (i - 16h) * ROWI + j, ROWI = 66).  Both row strides make every
// ds_write_b64 / ds_read_b64 of the pattern bank-conflict free (MI355X_MICROARCH.md §LDS).
static constexpr int ROWI = 66;
static_assert(16 * ROWI <= WAVE_LDS, "inverse half must fit the wave's LDS slice");

__device__ __forceinline__ void lds_fence() {
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void w0_to_w1(u64 (&x)[32], u64* sh, int lane) {
  u64 y[16];
  const int rbase = (lane >> 1) * ROW + (lane & 1);
  // half 0: lanes with j < 32 publish their column, every lane takes W1 registers 0..15
  if (lane < 32) {
#pragma unroll
    for (int r = 0; r < 32; ++r) sh[r * ROW + lane] = x[r];
  }
  lds_fence();
#pragma unroll
  for (int q = 0; q < 16; ++q) y[q] = sh[rbase + 2 * q];
  lds_fence();
  // half 1: lanes with j >= 32, W1 registers 16..31
  if (lane >= 32) {
#pragma unroll
    for (int r = 0; r < 32; ++r) sh[r * ROW + lane - 32] = x[r];
  }
  lds_fence();
#pragma unroll
  for (int q = 0; q < 16; ++q) x[16 + q] = sh[rbase + 2 * q];
  lds_fence();
#pragma unroll
  for (int q = 0; q < 16; ++q) x[q] = y[q];
}

__device__ __forceinline__ void w1_to_w0(u64 (&x)[32], u64* sh, int lane) {
  u64 y[16];
  const int wbase = ((lane >> 1) & 15) * ROWI + (lane & 1);
  // half 0: lanes with i < 16 publish their block, every lane takes W0 registers 0..15
  if (lane < 32) {
#pragma unroll
    for (int q = 0; q < 32; ++q) sh[wbase + 2 * q] = x[q];
  }
  lds_fence();
#pragma unroll
  for (int r = 0; r < 16; ++r) y[r] = sh[r * ROWI + lane];
  lds_fence();
  if (lane >= 32) {
#pragma unroll
    for (int q = 0; q < 32; ++q) sh[wbase + 2 * q] = x[q];
  }
  lds_fence();
#pragma unroll
  for (int r = 0; r < 16; ++r) x[16 + r] = sh[r * ROWI + lane];
  lds_fence();
#pragma unroll
  for (int r = 0; r < 16; ++r) x[r] = y[r];
}

// ---- stage groups ----------------------------------------------------------------------------
// group 1 (W0, register bits = i): stage s has 2^s groups, pair distance 16 >> s registers
__device__ __forceinline__ void g1_fwd(u64 (&x)[32]) {
  sfor<5>([&](auto s_) {
    constexpr int s = decltype(s_)::value;
    constexpr int d = 16 >> s;
    sfor<16>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      constexpr int r = ((k / d) * 2 * d) + (k % d);  // k-th register with bit d clear
      ct<G1_FWD[s][r >> (5 - s)]>(x[r], x[r + d]);
    });
  });
}
__device__ __forceinline__ void g1_inv(u64 (&x)[32]) {
  sfor<5>([&](auto s_) {
    constexpr int s = 4 - decltype(s_)::value;
    constexpr int d = 16 >> s;
    sfor<16>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      constexpr int r = ((k / d) * 2 * d) + (k % d);
      gs<G1_INV[s][r >> (5 - s)]>(x[r], x[r + d]);
    });
  });
}
// cyclic stages q = 0..4 (W1, register bits = j >> 1): pair distance 16 >> q registers
__device__ __forceinline__ void cyc_fwd(u64 (&x)[32]) {
  sfor<5>([&](auto q_) {
    constexpr int q = decltype(q_)::value;
    constexpr int d = 16 >> q;
    sfor<16>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      constexpr int r = ((k / d) * 2 * d) + (k % d);
      ct<CYC_FWD[q][r >> (5 - q)]>(x[r], x[r + d]);
    });
  });
}
__device__ __forceinline__ void cyc_inv(u64 (&x)[32]) {
  sfor<5>([&](auto q_) {
    constexpr int q = 4 - decltype(q_)::value;
    constexpr int d = 16 >> q;
    sfor<16>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      constexpr int r = ((k / d) * 2 * d) + (k % d);
      gs<CYC_INV[q][r >> (5 - q)]>(x[r], x[r + d]);
    });
  });
}

// ---- kernels ---------------------------------------------------------------------------------
template <bool FWD, bool ASM>
__global__ __launch_bounds__(256, 4) void ntt_tw_kernel(u64* __restrict__ data, uint32_t batch, uint64_t stride,
                                                     const u64* __restrict__ twist) {
  __shared__ u64 lds[4 * WAVE_LDS];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const uint32_t poly = blockIdx.x * 4 + wv;
  if (poly >= batch) return;  // whole wave: no workgroup barriers in this kernel
  u64* __restrict__ p = data + (uint64_t)poly * stride;
  u64* sh = lds + wv * WAVE_LDS;
  const int par = lane & 1;
  const int i = lane >> 1;
  u64 x[32];
  if constexpr (FWD) {
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = p[64 * r + lane];
    if constexpr (ASM) {
      twasm::g1_fwd_0(x); twasm::g1_fwd_1(x); twasm::g1_fwd_2(x); twasm::g1_fwd_3(x); twasm::g1_fwd_4(x);
    } else {
      g1_fwd(x);
    }
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = Goldilocks::mul(x[r], twist[64 * r + lane]);
    w0_to_w1(x, sh, lane);
    if constexpr (ASM) {
      twasm::cyc_fwd_0(x); twasm::cyc_fwd_1(x); twasm::cyc_fwd_2(x); twasm::cyc_fwd_3(x); twasm::cyc_fwd_4(x);
    } else {
      cyc_fwd(x);
    }
    // last cyclic stage (pairs across lanes 2i, 2i+1): even lane takes pairs k, odd lane pairs k + 16
    sfor<16>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      const u64 send = par ? x[k] : x[k + 16];
      const u64 recv = swap_pair_lanes(send);
      const u64 a = par ? recv : x[k];
      const u64 b = par ? x[k + 16] : recv;
      constexpr u64 w_even = pow2mod(CYC_FWD[5][k]), w_odd = pow2mod(CYC_FWD[5][k + 16]);
      const u64 w = par ? w_odd : w_even;
      const u64 t = Goldilocks::mul(b, w);
      const u64 o0 = canon(add_sc(a, t)), o1 = canon(sub_sc(a, t));
      u64* dst = p + 64 * i + 2 * k + 32 * par;
      dst[0] = o0;
      dst[1] = o1;
    });
  } else {
    // first inverse stage on the lane-pair layout, then regroup to W1
    sfor<16>([&](auto k_) {
      constexpr int k = decltype(k_)::value;
      const u64* src = p + 64 * i + 2 * k + 32 * par;
      const u64 a = src[0], b = src[1];
      constexpr u64 w_even = pow2mod(CYC_INV[5][k]), w_odd = pow2mod(CYC_INV[5][k + 16]);
      const u64 w = par ? w_odd : w_even;
      const u64 a2 = add_ff(a, b);
      const u64 b2 = Goldilocks::mul(sub_ff(a, b), w);
      const u64 send = par ? a2 : b2;
      const u64 recv = swap_pair_lanes(send);
      x[k] = par ? recv : a2;
      x[k + 16] = par ? b2 : recv;
    });
    if constexpr (ASM) {
      twasm::cyc_inv_4(x); twasm::cyc_inv_3(x); twasm::cyc_inv_2(x); twasm::cyc_inv_1(x); twasm::cyc_inv_0(x);
    } else {
      cyc_inv(x);
    }
    w1_to_w0(x, sh, lane);
#pragma unroll
    for (int r = 0; r < 32; ++r) x[r] = Goldilocks::mul(x[r], twist[64 * r + lane]);
    if constexpr (ASM) {
      twasm::g1_inv_4(x); twasm::g1_inv_3(x); twasm::g1_inv_2(x); twasm::g1_inv_1(x); twasm::g1_inv_0(x);
    } else {
      g1_inv(x);
    }
#pragma unroll
    for (int r = 0; r < 32; ++r) p[64 * r + lane] = canon(x[r]);
  }
}

// ---- whole-body asm kernel (tools/gen_tw_kernel.py) ----------------------------------------------
// The generated body owns v8..v127 / s20..s99 and performs load -> all stages -> store itself; this
// wrapper only derives the wave's polynomial and the per-lane LDS / global addresses.
static constexpr int WAVE_LDS2 = 1088;  // u64: max(32 x 34, 16 x 66)

template <bool FWD>
__global__ __launch_bounds__(256, 4) void ntt_tw_body_kernel(u64* __restrict__ data, uint32_t batch, uint64_t stride,
                                                             const u64* __restrict__ twist) {
  __shared__ u64 lds[4 * WAVE_LDS2];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t poly = blockIdx.x * 4 + wv;
  if (poly >= batch) return;
  u64* p = data + (uint64_t)poly * stride;
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8;
  const uint32_t t1w = S + (lane & 31) * 8;
  const uint32_t t1r = S + (i * 34 + par) * 8;
  const uint32_t lwo = par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)p, ghi = (uint32_t)((uintptr_t)p >> 32);
  const uint32_t twlo = (uint32_t)(uintptr_t)twist, twhi = (uint32_t)((uintptr_t)twist >> 32);
  const u64* lw = twist + 2048;
  if constexpr (FWD) {
    const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8;
    const uint32_t t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
    const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
    MI_TW_BODY_FWD([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r), [t2wl] "v"(t2wl), [t2wh] "v"(t2wh),
                   [t2r] "v"(t2r), [lwo] "v"(lwo));
  } else {
    const uint32_t t4w = S + ((i & 15) * 66 + par) * 8;
    const uint32_t t4r = S + lane * 8;
    MI_TW_BODY_INV([g_lo] "s"(glo), [g_hi] "s"(ghi), [tw_lo] "s"(twlo), [tw_hi] "s"(twhi), [lw] "s"(lw),
                   [l8] "v"(l8), [t1w] "v"(t1w), [t1r] "v"(t1r), [t4w] "v"(t4w), [t4r] "v"(t4r),
                   [lwo] "v"(lwo));
  }
}

// ---- persistent software-pipelined kernel (tools/gen_tw_kernel.py gen_pipe) ------------------------
// One 8-wave workgroup per CU (192 VGPRs per wave: 2 waves per SIMD).  The workgroup copies the
// direction's twist + pair-stage tables (N + 32 u64) into LDS once; each wave then walks the
// polynomials poly0, poly0 + step, ... with the next one's rows prefetched into v128..v191 while the
// current one is transformed.  HBM load latency is exposed once per wave, not once per polynomial.
static constexpr int PIPE_WAVES = 8;
static constexpr int TAB = 2048 + 32;

template <bool FWD>
__global__ __launch_bounds__(64 * PIPE_WAVES, 1) void ntt_tw_pipe_kernel(u64* __restrict__ data, uint32_t batch,
                                                                          uint32_t stride_bytes,
                                                                          const u64* __restrict__ twist) {
  __shared__ u64 lds[PIPE_WAVES * WAVE_LDS2];
  __shared__ u64 tab[TAB];
  for (int t = threadIdx.x; t < TAB; t += 64 * PIPE_WAVES) tab[t] = twist[t];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t poly0 = blockIdx.x * PIPE_WAVES + wv;
  const uint32_t step = gridDim.x * PIPE_WAVES;
  if (poly0 >= batch) return;  // whole wave; no barrier follows
  const uint32_t S = (uint32_t)(uintptr_t)(lds + wv * WAVE_LDS2);
  const uint32_t par = lane & 1, i = lane >> 1;
  const uint32_t l8 = lane * 8;
  const uint32_t t1w = S + (lane & 31) * 8;
  const uint32_t t1r = S + (i * 34 + par) * 8;
  const uint32_t twl = (uint32_t)(uintptr_t)tab + lane * 8;
  const uint32_t lwl = (uint32_t)(uintptr_t)(tab + 2048) + par * 128;
  const uint32_t glo = (uint32_t)(uintptr_t)data, ghi = (uint32_t)((uintptr_t)data >> 32);
  if constexpr (FWD) {
    const uint32_t t2wl = S + ((i & 15) * 66 + 33 * par) * 8;
    const uint32_t t2wh = S + ((i & 15) * 66 + 31 * par + 1) * 8;
    const uint32_t t2r = S + (lane ^ (lane >> 5)) * 8;
    MI_TW_PIPE_FWD([g_lo] "s"(glo), [g_hi] "s"(ghi), [p0] "s"(poly0), [batch] "s"(batch), [step] "s"(step),
                   [sb] "s"(stride_bytes), [l8] "v"(l8), [twl] "v"(twl), [lwl] "v"(lwl), [t1w] "v"(t1w),
                   [t1r] "v"(t1r), [t2wl] "v"(t2wl), [t2wh] "v"(t2wh), [t2r] "v"(t2r));
  } else {
    const uint32_t t4w = S + ((i & 15) * 66 + par) * 8;
    const uint32_t t4r = S + lane * 8;
    MI_TW_PIPE_INV([g_lo] "s"(glo), [g_hi] "s"(ghi), [p0] "s"(poly0), [batch] "s"(batch), [step] "s"(step),
                   [sb] "s"(stride_bytes), [l8] "v"(l8), [twl] "v"(twl), [lwl] "v"(lwl), [t1w] "v"(t1w),
                   [t1r] "v"(t1r), [t4w] "v"(t4w), [t4r] "v"(t4r));
  }
}

}  // namespace tw

static int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    cus = 256;
  return cus;
}

hipError_t launch_ntt_tw(bool fwd, int variant, uint64_t* data, size_t batch, size_t stride, const uint64_t* twist,
                         hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (variant == 7) {  // persistent pipelined asm body: one 8-wave workgroup per CU
    if (batch > 0xFFFFFFFFull || stride * 8 > 0xFFFFFFFFull) return hipErrorInvalidValue;
    static const int cus = device_cus();
    const size_t wgs = (batch + tw::PIPE_WAVES - 1) / tw::PIPE_WAVES;
    const unsigned grid = (unsigned)(wgs < (size_t)cus ? wgs : (size_t)cus);
    if (fwd)
      hipLaunchKernelGGL((tw::ntt_tw_pipe_kernel<true>), dim3(grid), dim3(64 * tw::PIPE_WAVES), 0, s, data,
                         (uint32_t)batch, (uint32_t)(stride * 8), twist);
    else
      hipLaunchKernelGGL((tw::ntt_tw_pipe_kernel<false>), dim3(grid), dim3(64 * tw::PIPE_WAVES), 0, s, data,
                         (uint32_t)batch, (uint32_t)(stride * 8), twist);
    return hipGetLastError();
  }
  const unsigned grid = (unsigned)((batch + 3) / 4);
  if (variant == 4) {  // whole-body asm
    if (fwd)
      hipLaunchKernelGGL((tw::ntt_tw_body_kernel<true>), dim3(grid), dim3(256), 0, s, data, (uint32_t)batch,
                         (uint64_t)stride, twist);
    else
      hipLaunchKernelGGL((tw::ntt_tw_body_kernel<false>), dim3(grid), dim3(256), 0, s, data, (uint32_t)batch,
                         (uint64_t)stride, twist);
    return hipGetLastError();
  }
  const bool asm_stages = variant == 5;  // 5: asm stage blocks, 6: compiler-generated stages
#define MI_TW_LAUNCH(F, A)                                                                              \
  hipLaunchKernelGGL((tw::ntt_tw_kernel<F, A>), dim3(grid), dim3(256), 0, s, data, (uint32_t)batch,  \
                     (uint64_t)stride, twist)
  if (fwd) {
    if (asm_stages) MI_TW_LAUNCH(true, true); else MI_TW_LAUNCH(true, false);
  } else {
    if (asm_stages) MI_TW_LAUNCH(false, true); else MI_TW_LAUNCH(false, false);
  }
#undef MI_TW_LAUNCH
  return hipGetLastError();
}

}  // namespace mi
