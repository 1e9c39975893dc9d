// ntt64_kernels.hip — batched negacyclic NTT over u64 primes for MI355X (gfx950).
//
// Reference semantics (paths relative to /root/reference/tfhe-ntt/src):
//   forward  = prime64.rs:897-968 -> generic_solinas.rs:449-481/931-1032 (radix-2 Cooley-Tukey,
//              twiddle twid[m + i] for block i at stage m, natural order in, bit-reversed out)
//   inverse  = prime64.rs:975-1046 -> generic_solinas.rs:483-561/1036 (Gentleman-Sande with
//              inv_twid[m + i], bit-reversed in, natural order out, unnormalised)
//
// MI355X design (not a translation of the CPU schedule):
//   * one workgroup owns PPW whole polynomials; each lane keeps E = 2^LOGE coefficients in
//     VGPRs and runs LOGE radix-2 stages on them with no data movement ("register window");
//   * between windows the polynomial is transposed through LDS (padded layout), so the N-point
//     transform costs ceil(LOGN / LOGE) - 1 LDS round trips and exactly one HBM read + write;
//   * twiddles come from a plan-owned device table (16 KiB at N = 2048, L2/L1 resident);
//   * Goldilocks arithmetic is 32-bit-limb VALU (no MFMA: integer modular arithmetic).
// Bit-exactness follows from canonical arithmetic: any schedule of the same
// butterflies with the same twiddles returns the same residues.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "mi_arith.hpp"
#include "ntt64_launch.hpp"
#include "ntt64_regs.hpp"
#include "ntt64_tile.hpp"
#include "ntt64_tile_asm.hpp"
#include "pbs_device.hpp"

namespace mi {

// IO = u64 (prime64 plans) or uint32_t (prime32 plans, prime32.rs:797-898: the same transform on
// u32 buffers; arithmetic stays 64-bit Montgomery, exact for any odd prime)
// SUB: large-N plans; the launch covers batch * 2^sub_log blocks of N = 2^G::LOGN, block b of
// polynomial q at data + q * stride + b * N, with the block's twiddle multiplier 2^sub_log + b.
template <class G, bool FWD, class Mod, class IO, bool SUB = false>
__global__ __launch_bounds__(G::THREADS) void ntt_window_kernel(IO* __restrict__ data, uint32_t batch, uint64_t stride,
                                                                const u64* __restrict__ tw, Mod mod,
                                                                uint32_t sub_log = 0) {
  __shared__ u64 lds[G::PPW * G::PADDED];
  const int tid = threadIdx.x;
  const int pw = tid >> G::LOGT;     // polynomial within the workgroup
  const int t = tid & (G::T - 1);    // lane within the polynomial
  const uint64_t unit = (uint64_t)blockIdx.x * G::PPW + pw;
  const uint64_t poly = SUB ? unit >> sub_log : unit;
  const uint32_t blk = SUB ? (uint32_t)(unit & ((1u << sub_log) - 1)) : 0;
  const uint32_t twc = SUB ? (1u << sub_log) + blk : 1;
  const bool valid = poly < batch;
  IO* __restrict__ src = data + poly * stride + (SUB ? (uint64_t)blk * G::N : 0);
  u64* sh = lds + pw * G::PADDED;

  u64 x[G::E];
  {
    const int lo = win_lo<G, FWD>(0);
#pragma unroll
    for (int r = 0; r < G::E; ++r) x[r] = valid ? (u64)src[elem<G>(t, r, lo)] : 0;
  }
#pragma unroll
  for (int w = 0; w < G::NWIN; ++w) {
    if (w > 0) {
      const int lo_prev = win_lo<G, FWD>(w - 1), lo = win_lo<G, FWD>(w);
#pragma unroll
      for (int r = 0; r < G::E; ++r) sh[lds_addr(elem<G>(t, r, lo_prev))] = x[r];
      __syncthreads();
#pragma unroll
      for (int r = 0; r < G::E; ++r) x[r] = sh[lds_addr(elem<G>(t, r, lo))];
      __syncthreads();
    }
    window_butterflies<G, FWD, Mod, SUB>(x, t, w, tw, mod, twc);
  }
  if (valid) {
    const int lo = win_lo<G, FWD>(G::NWIN - 1);
#pragma unroll
    for (int r = 0; r < G::E; ++r) src[elem<G>(t, r, lo)] = (IO)x[r];
  }
}

// ---------------------------------------------------------------------------------------------
// Large-N plans (N > 2^14, beyond one workgroup's registers): the transform is split into passes through memory, the
// decomposition the reference's depth-first recursion also uses (generic_solinas.rs:931-1032: top stages on the whole
// polynomial, then independent halves).
//   forward = the k = logn - 14 top CT stages in passes of at most 4 stages on strided columns (this kernel), then
//             2^k independent blocks of 2^14 with the remaining stages (ntt_window_kernel<SUB>, multiplier 2^k + b);
//   inverse = the blocks' GS stages first, then the top GS passes in reverse order.
// A pass that starts after S0 stages works inside each of the 2^S0 blocks of 2^(logn - S0) elements the stages above
// left independent: thread j of block b owns the 2^K elements b 2^(logn - S0) + j + i cols (i < 2^K, cols =
// 2^(logn - S0 - K), coalesced across j), and its local stage s (m = 2^s local groups) reads the table at
// (2^S0 + b) 2^s + g, the global stage S0 + s's twiddle of the block's group.
// TWIST (the split transform, launch_ntt_split): 1 = the forward's last pass multiplies each output element e (index
// within the polynomial) by twist[e] after its stages; 2 = the inverse's first pass multiplies each input by twist[e]
// before them.
// ACC (the inverse's last pass inside the large-N blind rotation, pbs_large.hip): instead of storing the output x,
// acc[e] += modswitch_{p -> 2^64}(x) (1, BNF, ntt64.rs:184-197 + wrapping add) or acc[e] = acc[e] + x mod p (2,
// Solinas, ntt64.rs:244-266), acc laid out like data (stride apart per polynomial)
// P2 (a pass that starts at stage 0 of a Goldilocks plan with the Solinas tower): the twiddles are the powers of two
// 2^tower_exp(s, g), multiplied by shifts (Goldilocks::mul_pow2) instead of table loads and four-limb products.
template <int K, bool FWD, class Mod, class IO, int TWIST = 0, int ACC = 0, bool P2 = false>
__global__ __launch_bounds__(256) void ntt_top_kernel(IO* __restrict__ data, uint64_t stride, uint32_t logn, uint32_t s0,
                                                      const u64* __restrict__ tw, Mod mod,
                                                      const u64* __restrict__ twist = nullptr,
                                                      u64* __restrict__ acc = nullptr) {
  constexpr int R = 1 << K;
  const uint32_t logc = logn - s0 - K;
  const uint64_t cols = (uint64_t)1 << logc;
  const uint64_t jg = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (jg >= ((uint64_t)1 << (logn - K))) return;
  const uint64_t blk = jg >> logc, j = jg & (cols - 1);
  const uint64_t twc = ((uint64_t)1 << s0) + blk;
  const uint64_t e0 = (blk << (logn - s0)) + j;  // element index of register 0 within the polynomial
  IO* __restrict__ src = data + (uint64_t)blockIdx.y * stride + e0;
  u64 x[R];
#pragma unroll
  for (int i = 0; i < R; ++i) x[i] = (u64)src[i * cols];
  if constexpr (TWIST == 2) {
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = mod.mul(x[i], twist[e0 + i * cols]);
  }
#pragma unroll
  for (int st = 0; st < K; ++st) {
    const int s = FWD ? st : K - 1 - st;  // stage s has m = 2^s groups, pair distance 2^(K-1-s) in i
    const int m = 1 << s, d = 1 << (K - 1 - s);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i & d) continue;
      if constexpr (P2) {
        const int g = i >> (K - s), ex = tower_exp(FWD, s, g);
        bool ng;
        if (FWD) {
          const u64 z = Goldilocks::mul_pow2(x[i + d], ex, ng);
          const u64 a = x[i];
          x[i] = ng ? Goldilocks::sub(a, z) : Goldilocks::add(a, z);
          x[i + d] = ng ? Goldilocks::add(a, z) : Goldilocks::sub(a, z);
        } else {  // (a - b) w = (b - a) |w| for a negative w
          const u64 a = x[i], b = x[i + d];
          x[i] = Goldilocks::add(a, b);
          x[i + d] = Goldilocks::mul_pow2(ex >= 96 ? Goldilocks::sub(b, a) : Goldilocks::sub(a, b), ex, ng);
        }
        continue;
      }
      const u64 wv = tw[twc * m + (uint64_t)(i >> (K - s))];
      if (FWD) {
        const u64 z = mod.mul(x[i + d], wv);
        const u64 a = x[i];
        x[i] = mod.add(a, z);
        x[i + d] = mod.sub(a, z);
      } else {
        const u64 a = x[i], b = x[i + d];
        x[i] = mod.add(a, b);
        x[i + d] = mod.mul(mod.sub(a, b), wv);
      }
    }
  }
  if constexpr (TWIST == 1) {
#pragma unroll
    for (int i = 0; i < R; ++i) x[i] = mod.mul(x[i], twist[e0 + i * cols]);
  }
  if constexpr (ACC != 0) {
    u64* __restrict__ a = acc + (uint64_t)blockIdx.y * stride + e0;
#pragma unroll
    for (int i = 0; i < R; ++i)
      a[i * cols] = ACC == 1 ? a[i * cols] + pbs::modswitch_prime_to_native(x[i]) : pbs::add_custom(a[i * cols], x[i]);
    return;
  }
#pragma unroll
  for (int i = 0; i < R; ++i) src[i * cols] = (IO)x[i];
}

// The stage-0 pass of the split transform at K = 4 / 5 as a cooperative tile (ntt64_tile.hpp): the same function as
// ntt_top_kernel<K, FWD, Goldilocks, u64, TWIST, ACC, true> at s0 = 0.  Grid: x = column tiles of 64, y = polynomials.
template <int K, bool FWD, int TWIST, int ACC, int W>
__device__ __forceinline__ void top_tile_body(u64* __restrict__ poly, uint64_t cols, uint64_t col, uint32_t c,
                                              const u64* __restrict__ twist, u64* __restrict__ accp, u64* lds) {
  using Rw = tile::Rows<K>;
  constexpr int RPT = Rw::RPT;
  u64 x[RPT];
  if constexpr (FWD) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) x[k] = poly[Rw::a(W, k) * cols + col];
    tile::phase_a<K, true, W>(x);
    tile::exchange<K, W, true>(x, lds, c);
    tile::phase_b<K, true, W>(x);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const uint64_t e = Rw::b(W, k) * cols + col;
      poly[e] = TWIST == 1 ? Goldilocks::mul(x[k], twist[e]) : Goldilocks::canon(x[k]);  // lazy stages
    }
  } else {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const uint64_t e = Rw::b(W, k) * cols + col;
      x[k] = TWIST == 2 ? Goldilocks::mul(poly[e], twist[e]) : poly[e];
    }
    tile::phase_b<K, false, W>(x);
    tile::exchange<K, W, false>(x, lds, c);
    tile::phase_a<K, false, W>(x);
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      const uint64_t e = Rw::a(W, k) * cols + col;
      if constexpr (ACC == 1) accp[e] = accp[e] + pbs::modswitch_prime_to_native(x[k]);
      else if constexpr (ACC == 2) accp[e] = pbs::add_custom(accp[e], x[k]);
      else poly[e] = x[k];
    }
  }
}

template <int K, bool FWD, int TWIST, int ACC>
__global__ __launch_bounds__(256) void ntt_top_tile_kernel(u64* __restrict__ data, uint64_t stride, uint32_t logn,
                                                           const u64* __restrict__ twist, u64* __restrict__ acc) {
  __shared__ u64 lds[(1 << K) * 64];
  const uint64_t cols = (uint64_t)1 << (logn - K);
  const uint32_t c = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t col = (uint64_t)blockIdx.x * 64 + c;
  u64* poly = data + (uint64_t)blockIdx.y * stride;
  u64* accp = ACC ? acc + (uint64_t)blockIdx.y * stride : nullptr;
  switch (w) {
    case 0: top_tile_body<K, FWD, TWIST, ACC, 0>(poly, cols, col, c, twist, accp, lds); break;
    case 1: top_tile_body<K, FWD, TWIST, ACC, 1>(poly, cols, col, c, twist, accp, lds); break;
    case 2: top_tile_body<K, FWD, TWIST, ACC, 2>(poly, cols, col, c, twist, accp, lds); break;
    default: top_tile_body<K, FWD, TWIST, ACC, 3>(poly, cols, col, c, twist, accp, lds); break;
  }
}

// ---------------------------------------------------------------------------------------------
// launch dispatch

template <int LOGN, int LOGE, bool FWD, class Mod, class IO>
static hipError_t launch_window(IO* data, size_t batch, size_t stride, const u64* tw, const Mod& mod,
                                hipStream_t stream) {
  using G = Geo<LOGN, LOGE>;
  const unsigned grid = (unsigned)((batch + G::PPW - 1) / G::PPW);
  hipLaunchKernelGGL((ntt_window_kernel<G, FWD, Mod, IO>), dim3(grid), dim3(G::THREADS), 0, stream, data,
                     (uint32_t)batch, (uint64_t)stride, tw, mod);
  return hipGetLastError();
}

constexpr int SUB_LOGN = 14;  // block size of the large-N second pass
constexpr int MAX_LOGN = 31;  // 2N-th roots of unity exist in the Solinas field up to 2N = 2^32

template <int K, bool FWD, class Mod, class IO>
static hipError_t launch_top(IO* data, size_t batch, size_t stride, int logn, int s0, const u64* tw, const Mod& mod,
                             hipStream_t s) {
  const uint64_t threads = (uint64_t)1 << (logn - K);
  const dim3 grid((unsigned)((threads + 255) / 256), (unsigned)batch);
  hipLaunchKernelGGL((ntt_top_kernel<K, FWD, Mod, IO>), grid, dim3(256), 0, s, data, (uint64_t)stride, (uint32_t)logn,
                     (uint32_t)s0, tw, mod);
  return hipGetLastError();
}

template <bool FWD, class Mod, class IO>
static hipError_t dispatch_large(int logn, IO* data, size_t batch, size_t stride, const u64* tw, const Mod& mod,
                                 hipStream_t s) {
  const int k = logn - SUB_LOGN;
  if (k < 1 || logn > MAX_LOGN) return hipErrorInvalidValue;
  // the top passes put polynomials on grid.y, the blocks pass batch x 2^k workgroups on grid.x
  const size_t max_batch = std::min<size_t>(65535, ((size_t)1 << 31) >> k);
  if (batch > max_batch) {
    for (size_t b0 = 0; b0 < batch; b0 += max_batch) {
      const size_t nb = batch - b0 < max_batch ? batch - b0 : max_batch;
      const hipError_t e = dispatch_large<FWD>(logn, data + b0 * stride, nb, stride, tw, mod, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  auto top = [&](int s0, int kk) -> hipError_t {
    switch (kk) {
      case 1: return launch_top<1, FWD>(data, batch, stride, logn, s0, tw, mod, s);
      case 2: return launch_top<2, FWD>(data, batch, stride, logn, s0, tw, mod, s);
      case 3: return launch_top<3, FWD>(data, batch, stride, logn, s0, tw, mod, s);
      default: return launch_top<4, FWD>(data, batch, stride, logn, s0, tw, mod, s);
    }
  };
  auto tops = [&]() -> hipError_t {  // passes of <= 4 stages: s0 = 0, 4, 8, ...; the inverse runs them in reverse
    const int passes = (k + 3) / 4;
    for (int q = 0; q < passes; ++q) {
      const int pi = FWD ? q : passes - 1 - q;
      const int s0 = 4 * pi, kk = std::min(4, k - s0);
      const hipError_t e = top(s0, kk);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto blocks = [&]() -> hipError_t {
    using G = Geo<SUB_LOGN, 4>;
    const uint64_t units = (uint64_t)batch << k;
    hipLaunchKernelGGL((ntt_window_kernel<G, FWD, Mod, IO, true>), dim3((unsigned)units), dim3(G::THREADS), 0, s, data,
                       (uint32_t)batch, (uint64_t)stride, tw, mod, (uint32_t)k);
    return hipGetLastError();
  };
  hipError_t e = FWD ? tops() : blocks();
  if (e == hipSuccess) e = FWD ? blocks() : tops();
  return e;
}

template <bool FWD, class Mod, class IO>
static hipError_t dispatch(int logn, IO* data, size_t batch, size_t stride, const u64* tw,
                           const Mod& mod, hipStream_t s) {
  if (logn > SUB_LOGN) return dispatch_large<FWD>(logn, data, batch, stride, tw, mod, s);
  switch (logn) {
    case 4: return launch_window<4, 3, FWD>(data, batch, stride, tw, mod, s);
    case 5: return launch_window<5, 3, FWD>(data, batch, stride, tw, mod, s);
    case 6: return launch_window<6, 3, FWD>(data, batch, stride, tw, mod, s);
    case 7: return launch_window<7, 3, FWD>(data, batch, stride, tw, mod, s);
    case 8: return launch_window<8, 3, FWD>(data, batch, stride, tw, mod, s);
    case 9: return launch_window<9, 3, FWD>(data, batch, stride, tw, mod, s);
    case 10: return launch_window<10, 3, FWD>(data, batch, stride, tw, mod, s);
    case 11: return launch_window<11, 3, FWD>(data, batch, stride, tw, mod, s);
    case 12: return launch_window<12, 3, FWD>(data, batch, stride, tw, mod, s);
    case 13: return launch_window<13, 3, FWD>(data, batch, stride, tw, mod, s);
    case 14: return launch_window<14, 4, FWD>(data, batch, stride, tw, mod, s);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------------------------
// The split transform (ntt64_launch.hpp SplitTw): t = logn - 11 top stages on strided columns with the block twist
// fused into the forward's last / the inverse's first pass, and the 2048-blocks through the twisted N = 2048 body.
// Factorisation (checked against the oracle on the CPU for N = 2^12 ... 2^17, fwd and inv:
// tools/check_split_factorisation.py; on the GPU for every N = 2^12 ... 2^20 the split engine serves: tests/test_ntt_gpu.py): after the reference's first t stages, block b of 2048 coefficients holds the
// residue mod X^2048 - zeta_b; with alpha_b = psi_N^(2 bitrev_t(b) + 1 - 2^t) (alpha_b^2048 = -zeta_b) the substitution
// X = alpha_b Y makes it the negacyclic (mod Y^2048 + 1) transform of the 2048 plan, whose root is psi_N^(N / 2048)
// (the Solinas root tower), in the same bit-reversed output order.
template <int K, bool FWD, int TWIST, int ACC>
static hipError_t launch_top_tw(u64* data, size_t batch, size_t stride, int logn, int s0, const u64* tw,
                                const u64* twist, u64* acc, hipStream_t s) {
  const uint64_t threads = (uint64_t)1 << (logn - K);
  const dim3 grid((unsigned)((threads + 255) / 256), (unsigned)batch);
  // the pass at stage 0 has the tower's power-of-two twiddles (the split tables are only built when the plan's
  // tables agree, c_api.cpp); at K = 4 / 5 it runs as the cooperative tile (>= 64 columns: logn >= K + 6)
  if constexpr (K >= 4) {
    if (s0 == 0 && logn >= K + 6) {
      const dim3 tgrid((unsigned)(((uint64_t)1 << (logn - K)) / 64), (unsigned)batch);
      // the compiled stages: the inverse's K = 5 untwist + stages as generated asm measured slower (r5, a block that
      // waits for all its row loads loses the overlap the compiled code keeps)
      hipLaunchKernelGGL((ntt_top_tile_kernel<K, FWD, TWIST, ACC>), tgrid, dim3(256), 0, s, data, (uint64_t)stride,
                         (uint32_t)logn, twist, acc);
      return hipGetLastError();
    }
  }
  if (s0 == 0)
    hipLaunchKernelGGL((ntt_top_kernel<K, FWD, Goldilocks, u64, TWIST, ACC, true>), grid, dim3(256), 0, s, data,
                       (uint64_t)stride, (uint32_t)logn, (uint32_t)s0, tw, Goldilocks{}, twist, acc);
  else
    hipLaunchKernelGGL((ntt_top_kernel<K, FWD, Goldilocks, u64, TWIST, ACC>), grid, dim3(256), 0, s, data,
                       (uint64_t)stride, (uint32_t)logn, (uint32_t)s0, tw, Goldilocks{}, twist, acc);
  return hipGetLastError();
}

template <bool FWD, int TWIST, int ACC = 0>
static hipError_t top_tw(int kk, u64* data, size_t batch, size_t stride, int logn, int s0, const u64* tw,
                         const u64* twist, hipStream_t s, u64* acc = nullptr) {
  switch (kk) {
    case 1: return launch_top_tw<1, FWD, TWIST, ACC>(data, batch, stride, logn, s0, tw, twist, acc, s);
    case 2: return launch_top_tw<2, FWD, TWIST, ACC>(data, batch, stride, logn, s0, tw, twist, acc, s);
    case 3: return launch_top_tw<3, FWD, TWIST, ACC>(data, batch, stride, logn, s0, tw, twist, acc, s);
    case 4: return launch_top_tw<4, FWD, TWIST, ACC>(data, batch, stride, logn, s0, tw, twist, acc, s);
    case 5: return launch_top_tw<5, FWD, TWIST, ACC>(data, batch, stride, logn, s0, tw, twist, acc, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_ntt_split(bool fwd, int logn, u64* data, size_t batch, size_t stride, const u64* tw,
                            const SplitTw& st, hipStream_t s, u64* acc, int acc_mode, bool skip_first) {
  if (acc && fwd) return hipErrorInvalidValue;  // acc: inverse only
  const int t = logn - 11;
  if (t < 1 || t > 10) return hipErrorInvalidValue;
  if (batch == 0) return hipSuccess;
  // t <= 3, the whole transform, no accumulation: top stages and bodies in one launch, one workgroup per polynomial.
  // Not inside the blind rotation (skip_first / acc): at its batch (one or two generations of workgroups) the fused
  // form's memory phase and body phase do not overlap across workgroups and measured slower.
  if (t <= 3 && !skip_first && !acc)
    return launch_ntt_split_fused(fwd, t, data, batch, stride, fwd ? st.blk_fwd : st.blk_inv,
                                  fwd ? st.body_fwd : st.body_inv, s);
  // the top passes put polynomials on grid.y (<= 65535 per launch); passes of <= 5 stages, balanced
  const int passes = (t + 4) / 5;
  int ks[2] = {(t + passes - 1) / passes, t - (t + passes - 1) / passes};
  auto tops = [&](u64* d, size_t nb) -> hipError_t {
    for (int q = skip_first && fwd ? 1 : 0; q < passes; ++q) {
      const int pi = fwd ? q : passes - 1 - q;
      const int s0 = pi == 0 ? 0 : ks[0], kk = ks[pi];
      const bool twist_here = fwd ? (pi == passes - 1) : (q == 0);
      // the inverse's last pass (q = passes - 1) accumulates into acc instead of storing, when asked
      u64* a = (!fwd && acc && q == passes - 1) ? acc + (d - data) : nullptr;
      hipError_t e;
      if (a && twist_here)
        e = acc_mode == 1 ? top_tw<false, 2, 1>(kk, d, nb, stride, logn, s0, tw, st.blk_inv, s, a)
                          : top_tw<false, 2, 2>(kk, d, nb, stride, logn, s0, tw, st.blk_inv, s, a);
      else if (a)
        e = acc_mode == 1 ? top_tw<false, 0, 1>(kk, d, nb, stride, logn, s0, tw, nullptr, s, a)
                          : top_tw<false, 0, 2>(kk, d, nb, stride, logn, s0, tw, nullptr, s, a);
      else if (!twist_here) e = fwd ? top_tw<true, 0>(kk, d, nb, stride, logn, s0, tw, nullptr, s)
                                    : top_tw<false, 0>(kk, d, nb, stride, logn, s0, tw, nullptr, s);
      else e = fwd ? top_tw<true, 1>(kk, d, nb, stride, logn, s0, tw, st.blk_fwd, s)
                   : top_tw<false, 2>(kk, d, nb, stride, logn, s0, tw, st.blk_inv, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  auto all_tops = [&]() -> hipError_t {
    for (size_t b0 = 0; b0 < batch; b0 += 65535) {
      const hipError_t e = tops(data + b0 * stride, std::min<size_t>(65535, batch - b0));
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  hipError_t e = fwd ? all_tops()
                     : (skip_first ? hipSuccess : launch_ntt_tw(false, data, batch, stride, st.body_inv, s, t));
  if (e == hipSuccess) e = fwd ? launch_ntt_tw(true, data, batch, stride, st.body_fwd, s, t) : all_tops();
  return e;
}

hipError_t launch_ntt(bool fwd, int logn, bool goldilocks, const MontParams& mp, u64* data, size_t batch,
                      size_t stride, const u64* tw, hipStream_t s) {
  if (goldilocks) {
    Goldilocks g;
    return fwd ? dispatch<true>(logn, data, batch, stride, tw, g, s) : dispatch<false>(logn, data, batch, stride, tw, g, s);
  }
  Montgomery m{mp.p, mp.pinv, mp.r2};
  return fwd ? dispatch<true>(logn, data, batch, stride, tw, m, s) : dispatch<false>(logn, data, batch, stride, tw, m, s);
}

// p < 2^32 (Shoup32 tables, c_api.cpp plan_create): u64 buffers (data64) or u32 buffers (data32, prime32 plans)
hipError_t launch_ntt_shoup32(bool fwd, int logn, uint32_t p, u64* data64, uint32_t* data32, size_t batch,
                              size_t stride, const uint64_t* tw, hipStream_t s) {
  const Shoup32 m{p};
  if (data32)
    return fwd ? dispatch<true>(logn, data32, batch, stride, tw, m, s) : dispatch<false>(logn, data32, batch, stride, tw, m, s);
  return fwd ? dispatch<true>(logn, data64, batch, stride, tw, m, s) : dispatch<false>(logn, data64, batch, stride, tw, m, s);
}

// ---------------------------------------------------------------------------------------------
// pointwise ops (prime64.rs:1050-1222), 2 u64 per lane per iteration, grid-stride

enum PwOp { PW_NORMALIZE = 0, PW_MUL_ASSIGN_NORMALIZE = 1, PW_MUL_ACCUMULATE = 2 };

template <int OP, class Mod>
__device__ __forceinline__ u64 pw_one(u64 o, u64 a, u64 b, u64 c, const Mod& mod) {
  if (OP == PW_NORMALIZE) return mod.mul(o, c);
  if (OP == PW_MUL_ASSIGN_NORMALIZE) return mod.mul(mod.mul(o, b), c);
  u64 prod = mod.mul(a, b);
  if (c != 0) prod = mod.mul(prod, c);  // Montgomery: c = R^2 mod p restores the plain product
  return mod.add(o, prod);
}

// VW = values per lane per iteration (2 -> 16-byte accesses, needs even stride + 16-B alignment); CONTIG: stride == n,
// the batch is one flat array (no per-element row division)
template <int OP, int VW, class Mod, class IO = u64, bool CONTIG = false>
__global__ __launch_bounds__(256) void pointwise_kernel(IO* __restrict__ out, const IO* __restrict__ a,
                                                        const IO* __restrict__ b, uint32_t n, uint32_t batch,
                                                        uint64_t stride, u64 c, Mod mod) {
  const uint64_t per_poly = n / VW;
  const uint64_t total = per_poly * batch;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t off;
    if constexpr (CONTIG) {
      off = VW * i;
    } else {
      const uint64_t poly = i / per_poly;
      off = poly * stride + VW * (i - poly * per_poly);
    }
    if constexpr (VW == 2) {
      const ulonglong2 ov = *reinterpret_cast<const ulonglong2*>(out + off);
      ulonglong2 av = make_ulonglong2(0, 0), bv = make_ulonglong2(0, 0);
      if (OP == PW_MUL_ACCUMULATE) av = *reinterpret_cast<const ulonglong2*>(a + off);
      if (OP != PW_NORMALIZE) bv = *reinterpret_cast<const ulonglong2*>(b + off);
      *reinterpret_cast<ulonglong2*>(out + off) =
          make_ulonglong2(pw_one<OP>(ov.x, av.x, bv.x, c, mod), pw_one<OP>(ov.y, av.y, bv.y, c, mod));
    } else {
      const u64 av = (OP == PW_MUL_ACCUMULATE) ? (u64)a[off] : 0;
      const u64 bv = (OP != PW_NORMALIZE) ? (u64)b[off] : 0;
      out[off] = (IO)pw_one<OP>((u64)out[off], av, bv, c, mod);
    }
  }
}

template <int OP, class Mod>
static hipError_t launch_pw(u64* out, const u64* a, const u64* b, size_t n, size_t batch, size_t stride, u64 c,
                            const Mod& mod, hipStream_t s) {
  const bool vec = (stride % 2 == 0) && ((uintptr_t)out % 16 == 0) && ((uintptr_t)a % 16 == 0) &&
                   ((uintptr_t)b % 16 == 0);
  const uint64_t total = (uint64_t)(vec ? n / 2 : n) * batch;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
  if (vec && stride == n)
    hipLaunchKernelGGL((pointwise_kernel<OP, 2, Mod, u64, true>), dim3((unsigned)blocks), dim3(256), 0, s, out, a, b,
                       (uint32_t)n, (uint32_t)batch, (uint64_t)stride, c, mod);
  else if (vec)
    hipLaunchKernelGGL((pointwise_kernel<OP, 2, Mod>), dim3((unsigned)blocks), dim3(256), 0, s, out, a, b,
                       (uint32_t)n, (uint32_t)batch, (uint64_t)stride, c, mod);
  else
    hipLaunchKernelGGL((pointwise_kernel<OP, 1, Mod>), dim3((unsigned)blocks), dim3(256), 0, s, out, a, b,
                       (uint32_t)n, (uint32_t)batch, (uint64_t)stride, c, mod);
  return hipGetLastError();
}

hipError_t launch_pointwise(int op, bool goldilocks, const MontParams& mp, u64* out, const u64* a, const u64* b,
                            size_t n, size_t batch, size_t stride, u64 c, hipStream_t s) {
  if (goldilocks) {
    Goldilocks g;
    if (op == PW_NORMALIZE) return launch_pw<PW_NORMALIZE>(out, a, b, n, batch, stride, c, g, s);
    if (op == PW_MUL_ASSIGN_NORMALIZE) return launch_pw<PW_MUL_ASSIGN_NORMALIZE>(out, a, b, n, batch, stride, c, g, s);
    return launch_pw<PW_MUL_ACCUMULATE>(out, a, b, n, batch, stride, c, g, s);
  }
  Montgomery m{mp.p, mp.pinv, mp.r2};
  if (op == PW_NORMALIZE) return launch_pw<PW_NORMALIZE>(out, a, b, n, batch, stride, c, m, s);
  if (op == PW_MUL_ASSIGN_NORMALIZE) return launch_pw<PW_MUL_ASSIGN_NORMALIZE>(out, a, b, n, batch, stride, c, m, s);
  return launch_pw<PW_MUL_ACCUMULATE>(out, a, b, n, batch, stride, c, m, s);
}

hipError_t launch_pointwise_u32(int op, const MontParams& mp, uint32_t* out, const uint32_t* a, const uint32_t* b,
                                size_t n, size_t batch, size_t stride, uint64_t c, hipStream_t s) {
  Montgomery m{mp.p, mp.pinv, mp.r2};
  uint64_t blocks = ((uint64_t)n * batch + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
#define MI_PW32(OP)                                                                                         \
  hipLaunchKernelGGL((pointwise_kernel<OP, 1, Montgomery, uint32_t>), dim3((unsigned)blocks), dim3(256), 0, s, \
                     out, a, b, (uint32_t)n, (uint32_t)batch, (uint64_t)stride, c, m)
  if (op == PW_NORMALIZE) MI_PW32(PW_NORMALIZE);
  else if (op == PW_MUL_ASSIGN_NORMALIZE) MI_PW32(PW_MUL_ASSIGN_NORMALIZE);
  else MI_PW32(PW_MUL_ACCUMULATE);
#undef MI_PW32
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// synthetic input, identical stream to oracle/ntt_oracle.c:ora_fill_uniform

__device__ __forceinline__ u64 mix64(u64 z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// `shift` = clz(p) computed on the host (0 for p = 0): keep bitlen(p) bits, then reject >= p.
__global__ __launch_bounds__(256) void fill_uniform_kernel(u64* __restrict__ out, uint64_t count, u64 seed, u64 p,
                                                           uint32_t shift) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    u64 v, k = 0;
    do {
      v = mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull + k * 0xD1B54A32D192ED03ull) >> shift;
      ++k;
    } while (p != 0 && v >= p);
    out[i] = v;
  }
}

hipError_t launch_fill_uniform(u64* out, size_t count, u64 seed, u64 p, hipStream_t s) {
  uint64_t blocks = (count + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (blocks == 0) return hipSuccess;
  const uint32_t shift = p ? (uint32_t)__builtin_clzll(p) : 0u;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, (uint64_t)count, seed, p, shift);
  return hipGetLastError();
}

}  // namespace mi
