// keyswitch.hip — batched native-modulus LWE keyswitch on the int8 matrix cores.
//
// Reference: tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs:137-227
// (keyswitch_lwe_ciphertext_native_mod_compatible): out = (0, .., 0, b) - sum_i sum_l d_{i,l} * KSK[i][l],
// d_{i,l} the balanced signed digits of a_i (decomposer.rs:156-185, iter.rs:103-151), all mod 2^64.
//
// MI355X design.  Over a batch the keyswitch is a GEMM: rows = ciphertexts, K = in_dim * level digit
// columns, N = out_dim + 1 key columns, mod 2^64.  Digits lie in [-2^(B-1), 2^(B-1)], so it runs
// exactly on v_mfma_i32_16x16x64_i8: every 64-bit key word is recoded once into 8 signed bytes
// s_t in [-128, 127] with x = sum_t s_t 2^(8t) mod 2^64, the 8 byte planes are 8 int8 GEMMs sharing
// the digit operand, and the epilogue folds the exact int32 sums as sum_t S_t << 8t mod 2^64.
// Digits wider than a signed byte (base_log > 7) are split the same way into nd = ceil((B+1)/8)
// signed bytes e_s (d = sum_s e_s 256^s) against key rows pre-shifted by 8s, so the GEMM depth is
// K = in_dim * level * nd and |S_t| <= K * 128 * 128 < 2^31 for K < 2^17 (checked at key creation).
//   * ksk_prepare_kernel (once per key): u64 key -> byte planes in MFMA B-fragment order
//     [col tile][k block][plane][lane] x 16 B, zero-padded to 16-column / 64-digit tiles;
//   * ks_digits_kernel (per batch): decomposition of every mask element into int8 digits in A-fragment
//     order [row tile][k block][lane] x 16 B (padded rows and digits are 0);
//   * ks_gemm_kernel: one wave = 4 row tiles x 1 column tile x 8 planes = 32 accumulators of 16x16 i32;
//     operands stream straight from global memory in fragment order (1 KiB coalesced per fragment),
//     the 4 waves of a workgroup share the digit fragments through L1/L2; epilogue writes u64 outputs.
// Fragment maps (gfx950): lane l holds row/column (l & 15) of the tile and the 16 consecutive k of
// group l >> 4 — the same k map for A and B, so the k order inside a block does not matter; C/D:
// col = l & 15, row = 4 (l >> 4) + reg (cdna_hip_programming.md §3).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ntt64_launch.hpp"

namespace mi {
namespace ks {

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
using u64 = uint64_t;

// decomposer.rs:64-71 + :156-185 init_decomposer_state (native u64, closest representable)
__device__ __forceinline__ u64 decomp_init(u64 input, int base_log, int level) {
  const unsigned rep = (unsigned)(base_log * level), non_rep = 64u - rep;
  u64 res = input >> (non_rep - 1);
  const u64 rounding_bit = res & 1u;
  res += 1;
  res >>= 1;
  res &= (~0ull) >> (64u - rep);
  const u64 need_balance = (((res - 1) | (rounding_bit << (rep - 1))) & res) >> (rep - 1);
  return res - (need_balance << rep);
}

// iter.rs:131-151 decompose_one_level (arithmetic shift); the digit as a signed integer
__device__ __forceinline__ int decompose_one(int base_log, u64& state) {
  const u64 mask = (1ull << base_log) - 1;
  const u64 res = state & mask;
  state = (u64)((int64_t)state >> base_log);
  const u64 carry = (((res - 1) | state) & res) >> (base_log - 1);
  state += carry;
  return (int)(int64_t)(res - (carry << base_log));
}

// signed byte t of x: x = sum_t s_t 2^(8t) mod 2^64, s_t in [-128, 127]
__device__ __forceinline__ int8_t signed_byte(u64 x, int t) {
  unsigned carry = 0;
  int s = 0;
  for (int u = 0; u <= t; ++u) {
    const unsigned v = (unsigned)((x >> (8 * u)) & 255u) + carry;
    carry = v >= 128u;
    s = (int)v - (carry ? 256 : 0);
  }
  return (int8_t)s;
}

struct Shape {
  uint32_t in_dim, out_size, level, base_log, nd, K, KB, CT;
};

__device__ __forceinline__ uint4 pack16(const int8_t (&b)[16]) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    w[q] = (uint32_t)(uint8_t)b[4 * q] | ((uint32_t)(uint8_t)b[4 * q + 1] << 8) |
           ((uint32_t)(uint8_t)b[4 * q + 2] << 16) | ((uint32_t)(uint8_t)b[4 * q + 3] << 24);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// frag[((ct * KB + kb) * 8 + t) * 64 + lane] = plane t of GEMM rows k = 64 kb + 16 (lane >> 4) + j,
// column 16 ct + (lane & 15); GEMM row k = (i * level + li) * nd + s holds KSK row i * level + li
// (in_dim blocks of `level` LWEs) shifted left by 8 s.
__global__ __launch_bounds__(256) void ksk_prepare_kernel(uint4* __restrict__ frag, const u64* __restrict__ ksk,
                                                          Shape s) {
  const uint64_t total = (uint64_t)s.CT * s.KB * 8 * 64;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t lane = idx & 63, t = (idx >> 6) & 7;
    const uint64_t rest = idx >> 9;
    const uint32_t kb = rest % s.KB, ct = rest / s.KB;
    const uint32_t col = ct * 16 + (lane & 15);
    int8_t b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t k = kb * 64 + 16 * (lane >> 4) + j;
      const uint32_t row = k / s.nd, sh = 8 * (k % s.nd);
      const u64 x = (k < s.K && col < s.out_size) ? ksk[(uint64_t)row * s.out_size + col] << sh : 0;
      b[j] = signed_byte(x, (int)t);
    }
    frag[idx] = pack16(b);
  }
}

// afrag[(mt * KB + kb) * 64 + lane] = digits k = 64 kb + 16 (lane >> 4) + j of ciphertext
// 16 mt + (lane & 15); rows >= batch and k >= K are zero.
__global__ __launch_bounds__(256) void ks_digits_kernel(uint4* __restrict__ afrag, const u64* __restrict__ lwe_in,
                                                        uint32_t batch, uint32_t rows, Shape s) {
  const uint64_t total = (uint64_t)rows * s.KB * 4;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = idx & 3;
    const uint32_t kb = (idx >> 2) % s.KB;
    const uint32_t row = (uint32_t)((idx >> 2) / s.KB);
    int8_t b[16];
    const u64* x = lwe_in + (uint64_t)row * (s.in_dim + 1);
    uint32_t cur_i = 0xFFFFFFFFu, cur_li = 0;
    u64 state = 0;
    int d = 0;
    for (int j = 0; j < 16; ++j) {
      const uint32_t k = kb * 64 + 16 * g + j;
      int8_t e = 0;
      if (row < batch && k < s.K) {
        const uint32_t kd = k / s.nd, i = kd / s.level, li = kd % s.level;
        if (i != cur_i) {
          state = decomp_init(x[i], (int)s.base_log, (int)s.level);
          cur_i = i;
          cur_li = 0;
        }
        while (cur_li <= li) {  // terms come least significant first (iter.rs:103-119)
          d = decompose_one((int)s.base_log, state);
          ++cur_li;
        }
        e = signed_byte((u64)(int64_t)d, (int)(k % s.nd));
      }
      b[j] = e;
    }
    const uint32_t mt = row >> 4, lane = (row & 15) + 16 * g;
    afrag[((uint64_t)mt * s.KB + kb) * 64 + lane] = pack16(b);
  }
}

static constexpr int MT_W = 4;  // row tiles per wave
static constexpr int WAVES = 4;  // column tiles per workgroup

__global__ __launch_bounds__(64 * WAVES) void ks_gemm_kernel(u64* __restrict__ out, const u64* __restrict__ lwe_in,
                                                             const uint4* __restrict__ afrag,
                                                             const uint4* __restrict__ bfrag, uint32_t batch,
                                                             Shape s) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t ct = blockIdx.x * WAVES + (threadIdx.x >> 6);
  if (ct >= s.CT) return;  // whole wave; no barriers in this kernel
  const uint32_t mt0 = blockIdx.y * MT_W;
  const uint4* A = afrag + (uint64_t)mt0 * s.KB * 64 + lane;
  const uint4* B = bfrag + (uint64_t)ct * s.KB * 8 * 64 + lane;
  i32x4 acc[MT_W][8];
#pragma unroll
  for (int m = 0; m < MT_W; ++m)
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[m][t] = i32x4{0, 0, 0, 0};
  for (uint32_t kb = 0; kb < s.KB; ++kb) {
    uint4 a[MT_W], b[8];
#pragma unroll
    for (int m = 0; m < MT_W; ++m) a[m] = A[((uint64_t)m * s.KB + kb) * 64];
#pragma unroll
    for (int t = 0; t < 8; ++t) b[t] = B[((uint64_t)kb * 8 + t) * 64];
#pragma unroll
    for (int m = 0; m < MT_W; ++m) {
      const i32x4 av = {(int)a[m].x, (int)a[m].y, (int)a[m].z, (int)a[m].w};
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const i32x4 bv = {(int)b[t].x, (int)b[t].y, (int)b[t].z, (int)b[t].w};
        acc[m][t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc[m][t], 0, 0, 0);
      }
    }
  }
  const uint32_t col = ct * 16 + (lane & 15);
  if (col >= s.out_size) return;
  const bool is_body = col == s.out_size - 1;
#pragma unroll
  for (int m = 0; m < MT_W; ++m) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t row = (mt0 + m) * 16 + 4 * (lane >> 4) + r;
      if (row >= batch) continue;
      u64 v = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) v += (u64)(int64_t)acc[m][t][r] << (8 * t);
      const u64 base = is_body ? lwe_in[(uint64_t)row * (s.in_dim + 1) + s.in_dim] : 0;
      out[(uint64_t)row * s.out_size + col] = base - v;
    }
  }
}

}  // namespace ks

int ks_digit_bytes_per_term(int base_log) { return (base_log + 1 + 7) / 8; }

static ks::Shape ks_shape(size_t in_dim, size_t out_dim, int base_log, int level) {
  ks::Shape s;
  s.in_dim = (uint32_t)in_dim;
  s.out_size = (uint32_t)(out_dim + 1);
  s.level = (uint32_t)level;
  s.base_log = (uint32_t)base_log;
  s.nd = (uint32_t)ks_digit_bytes_per_term(base_log);
  s.K = (uint32_t)(in_dim * (size_t)level * s.nd);
  s.KB = (s.K + 63) / 64;
  s.CT = (s.out_size + 15) / 16;
  return s;
}

size_t ks_key_bytes(size_t in_dim, size_t out_dim, int base_log, int level) {
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level);
  return (size_t)s.CT * s.KB * 8 * 64 * 16;
}

size_t ks_digit_bytes(size_t in_dim, int base_log, int level, size_t batch) {
  const size_t kb = (in_dim * (size_t)level * (size_t)ks_digit_bytes_per_term(base_log) + 63) / 64;
  const size_t rows = (batch + 16 * ks::MT_W - 1) / (16 * ks::MT_W) * 16 * ks::MT_W;
  return rows * kb * 64;
}

hipError_t launch_ksk_prepare(void* frag, const uint64_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                              hipStream_t st) {
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level);
  const uint64_t total = (uint64_t)s.CT * s.KB * 8 * 64;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65535 * 4 ? (total + 255) / 256 : 65535 * 4);
  hipLaunchKernelGGL(ks::ksk_prepare_kernel, dim3(grid), dim3(256), 0, st, (uint4*)frag, ksk, s);
  return hipGetLastError();
}

hipError_t launch_keyswitch(uint64_t* out, const uint64_t* lwe_in, const void* frag, void* digits, size_t batch,
                            size_t in_dim, size_t out_dim, int base_log, int level, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level);
  const uint32_t rows = (uint32_t)((batch + 16 * ks::MT_W - 1) / (16 * ks::MT_W) * 16 * ks::MT_W);
  const uint64_t total = (uint64_t)rows * s.KB * 4;
  const unsigned dgrid = (unsigned)((total + 255) / 256 < 65535 * 4 ? (total + 255) / 256 : 65535 * 4);
  hipLaunchKernelGGL(ks::ks_digits_kernel, dim3(dgrid), dim3(256), 0, st, (uint4*)digits, lwe_in, (uint32_t)batch,
                     rows, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const dim3 grid((s.CT + ks::WAVES - 1) / ks::WAVES, rows / (16 * ks::MT_W));
  hipLaunchKernelGGL(ks::ks_gemm_kernel, grid, dim3(64 * ks::WAVES), 0, st, out, lwe_in, (const uint4*)digits,
                     (const uint4*)frag, (uint32_t)batch, s);
  return hipGetLastError();
}

}  // namespace mi
