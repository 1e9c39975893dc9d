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
//     [column group of GN tiles][k block][tile][plane][lane] x 16 B (one contiguous block per k step),
//     zero-padded to whole column groups / 64-digit blocks;
//   * ks_digits_kernel (per batch): decomposition of every mask element into int8 digits in A-fragment
//     order [row group of GM tiles][k block][tile][lane] x 16 B (padded rows and digits are 0); for one byte per
//     digit at 1 / 2 / 4 / 8 levels, ks_digits_l_kernel (r6) builds each 16 KiB (row group, k block) in LDS from
//     coalesced row reads;
//   * ks_gemm_kernel: one 8-wave workgroup per CU computes a 256-row x 32-column block (x 8 planes):
//     each k step's 16 + 16 KiB of fragments are copied global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4) into a 3-buffer ring two steps ahead of the MFMAs (counted vmcnt + raw
//     s_barrier, so the copies stay in flight across barriers); fragment reads are inline-asm
//     ds_read_b128 so the compiler does not drain the ring before them.  Each wave owns 4 row tiles x 1
//     column tile x 8 planes = 32 accumulators of 16x16 i32 (128 AGPRs, two waves per SIMD).  Blocks
//     are mapped XCD-aware: the workgroups one XCD runs together cover 8 row groups x 4 column groups,
//     so the fragments they share are re-read from that XCD's L2.
// Fragment maps (gfx950): lane l holds row/column (l & 15) of the tile and the 16 consecutive k of
// group l >> 4 — the same k map for A and B, so the k order inside a block does not matter; C/D:
// col = l & 15, row = 4 (l >> 4) + reg (cdna_hip_programming.md §3).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ntt64_launch.hpp"
#include "keyswitch_launch.hpp"

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
  uint32_t body_log;  // KS32 (keyswitch_lwe_ciphertext_with_scalar_change): the output modulus 2^body_log
};

__device__ __forceinline__ uint4 pack16(const int8_t (&b)[16]) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    w[q] = (uint32_t)(uint8_t)b[4 * q] | ((uint32_t)(uint8_t)b[4 * q + 1] << 8) |
           ((uint32_t)(uint8_t)b[4 * q + 2] << 16) | ((uint32_t)(uint8_t)b[4 * q + 3] << 24);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Workgroup block = 256 rows x 32 columns (x 8 planes): 32 KiB per k step for 256 MFMAs (a 128 x 64 block moves
// 40 KiB: the B side carries 8 planes, so tall blocks stage fewer bytes per MFMA).  r6: the block is split over
// WAVE_R x WAVE_C = 8 waves, two per SIMD, each owning 4 row tiles x 8 plane fragments (32 accumulators, 128
// AGPRs): an LDS-DMA piece stalls its wave's issue for 100+ cycles among MFMAs and ds_reads (MI355X_MICROARCH.md,
// 'LDS-DMA piece issue cost'), and with one wave per SIMD those stalls were the kernel's time (MFMA busy ~0.5);
// the second wave issues its MFMAs through them.
static constexpr int WAVE_R = 4, WAVE_C = 2, NW = WAVE_R * WAVE_C;
static constexpr int NFR = 8;          // plane fragments (column tiles x planes) per wave and k step
static constexpr int GM = 4 * WAVE_R;  // row tiles (of 16) per workgroup block
static constexpr int A_STEP = GM * 64;  // uint4 per k step of a row group
static constexpr int A_PIECES = GM / NW;  // 1 KiB LDS-DMA pieces per wave and k step
// B side, per key word type: the native u64 key needs all 8 byte planes of 2 column tiles per wave; the KS32 u32 key
// (sums mod 2^32) only planes 0..3 (the signed-byte recoding of the low 4 bytes does not depend on the high ones), so
// its workgroups cover 4 column tiles x 4 planes with the same accumulators, 16 B fragments and LDS step (r6).
template <bool K32>
struct Geo {
  static constexpr int GN = K32 ? 4 : 2;        // column tiles (of 16) per workgroup block
  static constexpr int NPL = K32 ? 4 : 8;       // byte planes
  static constexpr int CW = GN / WAVE_C;        // column tiles per wave
  static constexpr int B_STEP = GN * NPL * 64;  // uint4 per k step of a column group
  static constexpr int B_PIECES = GN * NPL / NW;
  static_assert(CW * NPL == NFR, "NFR plane fragments per wave");
};
static_assert(Geo<false>::B_STEP == Geo<true>::B_STEP && Geo<false>::B_PIECES == Geo<true>::B_PIECES,
              "one LDS ring shape and DMA split for both key types");
static constexpr int B_STEP = Geo<false>::B_STEP, B_PIECES = Geo<false>::B_PIECES;
static constexpr int PIECES = A_PIECES + B_PIECES;
static constexpr uint32_t NBUF = 3;  // LDS stage buffers (NBUF x 32 KiB); 4 and 5 measured no faster (r6 s17)

// frag[(((cg * KB + kb) * GN + ci) * NPL + t) * 64 + lane] = plane t of GEMM rows k = 64 kb + 16 (lane >> 4) + j,
// column 16 (GN cg + ci) + (lane & 15); GEMM row k = (i * level + li) * nd + s holds KSK row i * level + li
// (in_dim blocks of `level` LWEs) shifted left by 8 s.
// W = u64 (native keyswitch) or uint32_t (KS32: the u32 key words zero-extended; planes 0..3 stored)
template <typename W>
__global__ __launch_bounds__(256) void ksk_prepare_kernel(uint4* __restrict__ frag, const W* __restrict__ ksk,
                                                          Shape s) {
  using G = Geo<sizeof(W) == 4>;
  constexpr int GN = G::GN, NPL = G::NPL;
  const uint64_t total = (uint64_t)s.CT * s.KB * NPL * 64;  // CT is a multiple of GN
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t lane = idx & 63, t = (idx >> 6) % NPL, ci = (idx / (64 * NPL)) % GN;
    const uint64_t rest = idx / (64 * NPL * GN);
    const uint32_t kb = rest % s.KB, cg = rest / s.KB;
    const uint32_t col = (cg * GN + ci) * 16 + (lane & 15);
    int8_t b[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint32_t k = kb * 64 + 16 * (lane >> 4) + j;
      const uint32_t row = k / s.nd, sh = 8 * (k % s.nd);
      const u64 x = (k < s.K && col < s.out_size) ? (u64)ksk[(uint64_t)row * s.out_size + col] << sh : 0;
      b[j] = signed_byte(x, (int)t);
    }
    frag[idx] = pack16(b);
  }
}

// afrag[((mg * KB + kb) * GM + mi) * 64 + lane] = digits k = 64 kb + 16 (lane >> 4) + j of ciphertext
// 16 (GM mg + mi) + (lane & 15); rows >= batch and k >= K are zero.
__global__ __launch_bounds__(256) void ks_digits_kernel(uint4* __restrict__ afrag, const u64* __restrict__ lwe_in,
                                                        uint32_t batch, uint32_t rows, Shape s) {
  const uint64_t total = (uint64_t)rows * s.KB * 4;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (uint64_t)gridDim.x * blockDim.x) {
    // idx walks afrag in storage order (coalesced 1 KiB stores per wave); a wave reads 16 rows x 128 B
    const uint32_t lane = idx & 63, g = lane >> 4;
    const uint64_t piece = idx >> 6;  // (mg * KB + kb) * GM + mi
    const uint32_t mi = piece % GM, kb = (piece / GM) % s.KB, mg = (uint32_t)(piece / GM / s.KB);
    const uint32_t row = (mg * GM + mi) * 16 + (lane & 15);
    int8_t b[16];
    const u64* x = lwe_in + (uint64_t)row * (s.in_dim + 1);
    const int bl = (int)s.base_log, lv = (int)s.level;
    // digit column k = (i * level + li) * nd + sb, walked incrementally: 3 divisions per thread, not 3 per
    // digit; terms come least significant first (iter.rs:103-119)
    const uint32_t k0 = kb * 64 + 16 * g, kd0 = k0 / s.nd;
    uint32_t sb = k0 - kd0 * s.nd, i = kd0 / s.level, li = kd0 - i * s.level;
    const bool live = row < batch;
    u64 state = 0;
    int d = 0;
    if (live && k0 < s.K) {  // the state after terms 0..li of coefficient i
      state = decomp_init(x[i], bl, lv);
      for (uint32_t u = 0; u <= li; ++u) d = decompose_one(bl, state);
    }
    for (int j = 0; j < 16; ++j) {
      const uint32_t k = k0 + j;
      const bool on = live && k + 1 < s.K;
      b[j] = (live && k < s.K) ? signed_byte((u64)(int64_t)d, (int)sb) : 0;
      if (++sb == s.nd) {  // next decomposition term
        sb = 0;
        if (++li == s.level) {  // next mask coefficient
          li = 0;
          ++i;
          if (on) state = decomp_init(x[i], bl, lv);
        }
        if (on) d = decompose_one(bl, state);
      }
    }
    afrag[idx] = pack16(b);
  }
}

// r6: the common digit shapes (one signed byte per term, nd = 1, and a level count that divides 16: 1, 2, 4, 8), one
// workgroup per (row group mg, KBW consecutive k blocks) = KBW 16 KiB blocks of afrag.  ks_digits_kernel's lanes each
// read 4 coefficients of 16 different rows per load (16 KiB-strided); here the workgroup reads its 256 rows x 16
// coefficients (KBW = 1 block of 64 / LEVEL coefficients at LEVEL <= 4, two blocks of 8 at LEVEL 8) with 16
// consecutive lanes on consecutive coefficients of one row (whole 128-byte lines: at LEVEL 8 one block's 64-byte half
// line left the other half to another workgroup, often on another XCD), decomposes each coefficient into its LEVEL
// digits (unrolled), places them in the fragment order in LDS (one LEVEL-byte write), and stores the blocks with
// coalesced 16-byte stores.  Same bytes as ks_digits_kernel.
template <int LEVEL>
__global__ __launch_bounds__(256) void ks_digits_l_kernel(uint4* __restrict__ afrag, const u64* __restrict__ lwe_in,
                                                          uint32_t batch, uint32_t rows, Shape s) {
  static_assert(16 % LEVEL == 0, "a coefficient's digits stay inside one 16-byte fragment");
  constexpr int CPB = 64 / LEVEL;                // coefficients per k block
  constexpr int KBW = LEVEL > 4 ? LEVEL / 4 : 1;  // k blocks per workgroup: 16 coefficients (128 B) per row
  constexpr int CPW = CPB * KBW;
  using W = std::conditional_t<LEVEL == 1, uint8_t,
                               std::conditional_t<LEVEL == 2, uint16_t, std::conditional_t<LEVEL == 4, uint32_t, u64>>>;
  __shared__ uint4 blk[KBW * GM * 64];  // KBW x 16 KiB: the (mg, kb) blocks in storage order
  const uint32_t nkw = (s.KB + KBW - 1) / KBW;
  const uint32_t kb0 = (blockIdx.x % nkw) * KBW, mg = blockIdx.x / nkw;
  const uint32_t t = threadIdx.x;
  const int bl = (int)s.base_log;
  uint8_t* bytes = reinterpret_cast<uint8_t*>(blk);
#pragma unroll 4
  for (uint32_t q = 0; q < (GM * 16 * CPW) / 256; ++q) {
    const uint32_t pidx = q * 256 + t, R = pidx / CPW, cw = pidx % CPW;  // row in the group, coefficient in the span
    const uint32_t kbi = cw / CPB, c = cw % CPB;
    const uint32_t row = mg * GM * 16 + R, i = kb0 * CPB + cw;
    const u64 x = (row < batch && i < s.in_dim) ? lwe_in[(uint64_t)row * (s.in_dim + 1) + i] : 0;
    u64 state = decomp_init(x, bl, LEVEL);  // 0 decomposes to 0 at every level (padding rows / columns)
    W w = 0;
#pragma unroll
    for (int l = 0; l < LEVEL; ++l) w |= (W)(uint8_t)(int8_t)decompose_one(bl, state) << (8 * l);
    const uint32_t kk = LEVEL * c, lane = (kk >> 4) * 16 + (R & 15);
    *reinterpret_cast<W*>(bytes + ((kbi * GM + (R >> 4)) * 64 + lane) * 16 + (kk & 15)) = w;
  }
  __syncthreads();
#pragma unroll
  for (int kbi = 0; kbi < KBW; ++kbi) {
    if (kb0 + kbi >= s.KB) break;  // uniform: a ragged last span
    uint4* dst = afrag + ((uint64_t)mg * s.KB + kb0 + kbi) * (GM * 64);
#pragma unroll
    for (uint32_t q = 0; q < GM * 64 / 256; ++q) dst[q * 256 + t] = blk[kbi * GM * 64 + q * 256 + t];
  }
}

// Block t of the launch order -> (row group, column group): XCD x (workgroups x, x + 8, ... are dispatched
// to the same XCD) takes the contiguous range [x * per, (x + 1) * per) of an order that walks 8 row groups
// inside each column group, so the ~32 blocks an XCD holds at once share 4 column groups' key fragments.
__device__ __forceinline__ bool ks_block(uint32_t bid, uint32_t n_mg, uint32_t n_cg, uint32_t& mg, uint32_t& cg) {
  const uint32_t n_rb = (n_mg + 7) / 8, tiles = n_rb * 8 * n_cg, per = (tiles + 7) / 8;
  const uint32_t t = (bid & 7) * per + (bid >> 3);
  if (t >= tiles) return false;
  const uint32_t rb = t / (8 * n_cg), w = t % (8 * n_cg);
  cg = w / 8;
  mg = rb * 8 + w % 8;
  return mg < n_mg;
}

__device__ __forceinline__ i32x4 frag(const uint4* p) {
  const uint4 x = *p;
  return i32x4{(int)x.x, (int)x.y, (int)x.z, (int)x.w};
}

// native_closest_representable (decomposer.rs:25-49) of a u64 at one level of `bits` bits
__device__ __forceinline__ u64 closest_representable(u64 x, uint32_t bits) {
  const uint32_t shift = 64u - bits - 1u;
  return (((x >> shift) + 1u) & ~(u64)1) << shift;
}

// OUT32: keyswitch_lwe_ciphertext_with_scalar_change (lwe_keyswitch.rs:331-447): the body is the input body rounded
// to the output modulus' 2^body_log and scaled down by 2^32, the sums wrap mod 2^32, and u32 words are stored
template <bool OUT32>
__global__ __launch_bounds__(64 * NW, 1) void ks_gemm_kernel(void* __restrict__ out_v, const u64* __restrict__ lwe_in,
                                                         const uint4* __restrict__ afrag,
                                                         const uint4* __restrict__ bfrag, uint32_t batch,
                                                         uint32_t n_mg, Shape s) {
  // NBUF stage buffers (A pieces, then B pieces) of 32 KiB: while step kb multiplies, step kb + 1 is
  // read into registers and steps kb + 2 .. kb + NBUF are in flight (deep enough to cover the L2 /
  // MALL latency at the per-CU byte rate one step of MFMAs needs)
  constexpr int GN = Geo<OUT32>::GN, NPL = Geo<OUT32>::NPL, CW = Geo<OUT32>::CW;  // CW column tiles per wave
  __shared__ uint4 lds[NBUF][A_STEP + B_STEP];
  uint32_t mg, cg;
  if (!ks_block(blockIdx.x, n_mg, s.CT / GN, mg, cg)) return;  // whole workgroup, before any barrier
  const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w / WAVE_C, wc = w % WAVE_C;
  // LDS-DMA staging: wave w copies A pieces [A_PIECES w, A_PIECES (w + 1)) and the same share of the B
  // pieces of each k step (a piece = one tile-plane's 64 lanes x 16 B, written lane-linearly, which is
  // the fragment order).
  const uint4* ga = afrag + (uint64_t)mg * s.KB * A_STEP + (A_PIECES * w) * 64 + lane;
  const uint4* gb = bfrag + (uint64_t)cg * s.KB * B_STEP + (B_PIECES * w) * 64 + lane;
  // quarter `part` of this wave's pieces of step kb into stage buffer `buf`
  static_assert(PIECES % 4 == 0, "pieces are issued in quarters");
  auto dma = [&](uint32_t kb, uint32_t buf, int part) {
#pragma unroll
    for (int u = 0; u < PIECES / 4; ++u) {
      const int q = part * (PIECES / 4) + u;
      if (q < A_PIECES)
        __builtin_amdgcn_global_load_lds(ga + (uint64_t)kb * A_STEP + q * 64, &lds[buf][(A_PIECES * w + q) * 64],
                                         16, 0, 0);
      else
        __builtin_amdgcn_global_load_lds(gb + (uint64_t)kb * B_STEP + (q - A_PIECES) * 64,
                                         &lds[buf][A_STEP + (B_PIECES * w + q - A_PIECES) * 64], 16, 0, 0);
    }
  };
  i32x4 acc[4][CW][NPL];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int c = 0; c < CW; ++c)
#pragma unroll
      for (int t = 0; t < NPL; ++t) acc[m][c][t] = i32x4{0, 0, 0, 0};
  // this lane's fragment addresses in buffer 0 (buffer b adds b * BUF_BYTES)
  const uint32_t lds0 = (uint32_t)(uintptr_t)&lds[0][0];
  const uint32_t a_addr = lds0 + ((wr * 4) * 64 + lane) * 16;
  const uint32_t b_addr = lds0 + (A_STEP + (wc * CW * NPL) * 64 + lane) * 16;
  constexpr uint32_t BUF_BYTES = (A_STEP + B_STEP) * 16;
  // Fragment reads are inline asm: the compiler cannot tell the stage buffers apart and would drain
  // every LDS-DMA in flight (vmcnt(0)) before its own ds_reads; lgkm_wait retires them.
  auto rd_a = [&](uint32_t buf, i32x4(&A)[4]) {
    const uint32_t ao = a_addr + buf * BUF_BYTES;
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\tds_read_b128 %2, %4 offset:2048\n\t"
        "ds_read_b128 %3, %4 offset:3072"
        : "=&v"(A[0]), "=&v"(A[1]), "=&v"(A[2]), "=&v"(A[3])
        : "v"(ao));
  };
  auto rd_b = [&](uint32_t buf, int j, i32x4& Bj) {  // plane t of column tile c, j = NPL c + t
    const uint32_t bo = b_addr + buf * BUF_BYTES + 1024 * j;
    asm volatile("ds_read_b128 %0, %1" : "=&v"(Bj) : "v"(bo));
  };
  static_assert(NFR == 8, "lgkm_wait names 8 plane fragments");
  auto lgkm_wait = [&](i32x4(&A)[4], i32x4(&Bf)[NFR]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(Bf[0]), "+v"(Bf[1]), "+v"(Bf[2]),
                   "+v"(Bf[3]), "+v"(Bf[4]), "+v"(Bf[5]), "+v"(Bf[6]), "+v"(Bf[7]));
  };
  // prologue: steps 0..2 in flight; steps 0 and 1 landed; step 0's fragments in (A, Bf); a barrier so
  // that nobody's step-NBUF DMA overwrites buffer 0 before every wave has read it
  // (a copy of a step past the end is clamped to the last step: redundant but harmless, and it keeps
  // exactly PIECES copies per step in flight, so every wait below is the same counted vmcnt)
  const uint32_t last = s.KB - 1;
#pragma unroll
  for (int p = 0; p < 4; ++p) dma(0, 0, p);
#pragma unroll
  for (uint32_t b = 1; b < NBUF; ++b) {
#pragma unroll
    for (int p = 0; p < 4; ++p) dma(b < last ? b : last, b, p);
  }
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * PIECES) : "memory");  // steps 0 and 1 landed
  __builtin_amdgcn_s_barrier();
  i32x4 A[4], NA[4], Bf[NFR];
  rd_a(0, A);
#pragma unroll
  for (int j = 0; j < NFR; ++j) rd_b(0, j, Bf[j]);
  lgkm_wait(A, Bf);
  __builtin_amdgcn_s_barrier();
  // Step kb: NFR groups of 4 MFMAs, group j on plane fragment Bf[j] (j = NPL c + t) and the 4 row tiles A.
  // Behind group j the wave refills Bf[j] with step kb + 1's fragment (just freed), reads step kb + 1's
  // A into NA behind group 0, and issues a quarter of step kb + NBUF's LDS-DMA into the buffer step kb
  // occupied behind groups 1, 3, 5, 7 (an MFMA leaves half its cycles to other issue).  Step kb + 2's
  // copy is in flight throughout; the closing wait retires it and the barrier publishes it.
  uint32_t buf = 0;
  for (uint32_t kb = 0; kb < s.KB; ++kb) {
    const uint32_t nbuf = (buf + 1) % NBUF, src = kb + NBUF < last ? kb + NBUF : last;
#pragma unroll
    for (int j = 0; j < NFR; ++j) {
      const int c = j / NPL, t = j % NPL;
#pragma unroll
      for (int m = 0; m < 4; ++m) {  // accumulators pinned to AGPRs ("+a"): fragments keep the VGPRs
        if (j == 0 && m == 0)  // A was just copied by VALU: 2 wait states before an MFMA reads it
          asm("s_nop 1\n\tv_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc[m][c][t]) : "v"(A[m]), "v"(Bf[j]));
        else
          asm("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(acc[m][c][t]) : "v"(A[m]), "v"(Bf[j]));
      }
      __builtin_amdgcn_sched_barrier(0);
      if (j == 0) rd_a(nbuf, NA);  // in the last step these read a stale buffer: unused
      rd_b(nbuf, j, Bf[j]);
      if ((j & 1) && j < 8) dma(src, buf, j >> 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    lgkm_wait(NA, Bf);
#pragma unroll
    for (int m = 0; m < 4; ++m) A[m] = NA[m];
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NBUF - 2) * PIECES) : "memory");  // step kb + 2 landed
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    buf = nbuf;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA may outlive the workgroup
  // the compiler does not know the asm above holds MFMAs: 12 wait states before it reads their results
  asm volatile("s_nop 7\n\ts_nop 3" ::: "memory");
#pragma unroll
  for (int c = 0; c < CW; ++c) {
    const uint32_t col = (cg * GN + wc * CW + c) * 16 + (lane & 15);
    if (col >= s.out_size) continue;
    const bool is_body = col == s.out_size - 1;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t row = (mg * GM + wr * 4 + m) * 16 + 4 * (lane >> 4) + r;
        if (row >= batch) continue;
        u64 v = 0;
#pragma unroll
        for (int t = 0; t < NPL; ++t) v += (u64)(int64_t)acc[m][c][t][r] << (8 * t);
        u64 base = is_body ? lwe_in[(uint64_t)row * (s.in_dim + 1) + s.in_dim] : 0;
        if constexpr (OUT32) {
          if (is_body) base = closest_representable(base, s.body_log) >> 32;
          static_cast<uint32_t*>(out_v)[(uint64_t)row * s.out_size + col] = (uint32_t)(base - v);
        } else {
          static_cast<u64*>(out_v)[(uint64_t)row * s.out_size + col] = base - v;
        }
      }
    }
  }
}

// ---- the modulus switch of an LWE (lwe_ciphertext_modulus_switch / lwe_ciphertext_centered_binary_modulus_switch,
// algorithms/modulus_switch.rs:14-104): u32 words for the KS32 bootstrap's input (mockups/tfhe-hpu-mockup/src/lib.rs:
// 720-736), u64 words for the native-modulus ciphertexts of every other PBS ----
// modulus_switch (fft_impl/common.rs:10-23) at Scalar = T: identity at log_mod == BITS
template <typename T>
__device__ __forceinline__ T ms_word(T x, uint32_t log_mod) {
  constexpr uint32_t BITS = 8 * sizeof(T);
  return log_mod >= BITS ? x : (T)(x + ((T)1 << (BITS - log_mod - 1u))) >> (BITS - log_mod);
}

// One wave per ciphertext: the switched mask (LazyStandardModulusSwitchedLweCiphertext::mask,
// modulus_switched_lwe_ciphertext.rs:164-172) and, when `centered`, the body correction of
// lwe_ciphertext_centered_binary_modulus_switch (modulus_switch.rs:56-102) at Scalar = T / Signed: the wrapping
// sum of the halved rounding errors and the exact sum of the halving errors are order-free, so the lanes' partial
// sums combine by a butterfly reduction; then body = modulus_switch(b + correction) (:150-162).  out: (dim + 1) u64 per
// ciphertext, every value in [0, 2^log_mod) (the blind rotation's MI_MS_PRE_SWITCHED input).  The centered form is
// called with log_mod < BITS only (the reference's half_case shift underflows at BITS).  The halving errors are each
// in {-1, 0, 1}, so their sum fits an int32 for any dimension the callers accept (< 2^24).
template <typename T>
__global__ __launch_bounds__(256) void lwe_ms_kernel(u64* __restrict__ out, const T* __restrict__ in, uint32_t dim,
                                                     uint32_t batch, uint32_t log_mod, int centered) {
  using S = typename std::conditional<sizeof(T) == 4, int32_t, int64_t>::type;
  constexpr uint32_t BITS = 8 * sizeof(T);
  const uint32_t lane = threadIdx.x & 63, item = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (item >= batch) return;
  const T* x = in + (uint64_t)item * (dim + 1);
  u64* y = out + (uint64_t)item * (dim + 1);
  T sum_half = 0;
  int32_t sum_hed = 0;
  for (uint32_t i = lane; i < dim; i += 64) {
    const T a = x[i], sw = ms_word<T>(a, log_mod);
    y[i] = sw;
    if (centered) {
      const T round = log_mod >= BITS ? sw : (T)(sw << (BITS - log_mod));
      const S err = (S)(T)(round - a), half = err / 2;  // signed division truncates toward zero, as Rust's
      sum_half += (T)half;
      sum_hed += (int32_t)(2 * half - err);
    }
  }
  if (centered) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      if constexpr (sizeof(T) == 4) {
        sum_half += (T)__shfl_xor((int)sum_half, off, 64);
      } else {
        sum_half += (T)__shfl_xor((long long)sum_half, off, 64);
      }
      sum_hed += __shfl_xor(sum_hed, off, 64);
    }
  }
  if (lane == 0) {
    T corr = 0;
    if (centered) {
      const T half_case = (T)1 << (BITS - log_mod - 1u);
      corr = (T)(sum_half - (T)(S)(sum_hed / 2)) - half_case;
    }
    y[dim] = ms_word<T>((T)(x[dim] + corr), log_mod);
  }
}

}  // namespace ks

int ks_digit_bytes_per_term(int base_log) { return (base_log + 1 + 7) / 8; }

// k32: the KS32 key geometry (ks::Geo<true>)
static ks::Shape ks_shape(size_t in_dim, size_t out_dim, int base_log, int level, bool k32 = false) {
  const uint32_t gn = k32 ? ks::Geo<true>::GN : ks::Geo<false>::GN;
  ks::Shape s;
  s.in_dim = (uint32_t)in_dim;
  s.out_size = (uint32_t)(out_dim + 1);
  s.level = (uint32_t)level;
  s.base_log = (uint32_t)base_log;
  s.nd = (uint32_t)ks_digit_bytes_per_term(base_log);
  s.K = (uint32_t)(in_dim * (size_t)level * s.nd);
  s.KB = (s.K + 63) / 64;
  s.CT = (s.out_size + 16 * gn - 1) / (16 * gn) * gn;  // whole column groups
  s.body_log = 64;
  return s;
}

size_t ks_key_bytes(size_t in_dim, size_t out_dim, int base_log, int level) {
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level);
  return (size_t)s.CT * s.KB * ks::Geo<false>::NPL * 64 * 16;
}

size_t ks32_key_bytes(size_t in_dim, size_t out_dim, int base_log, int level) {
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level, true);
  return (size_t)s.CT * s.KB * ks::Geo<true>::NPL * 64 * 16;
}

size_t ks_digit_bytes(size_t in_dim, int base_log, int level, size_t batch) {
  const size_t kb = (in_dim * (size_t)level * (size_t)ks_digit_bytes_per_term(base_log) + 63) / 64;
  const size_t rows = (batch + 16 * ks::GM - 1) / (16 * ks::GM) * 16 * ks::GM;
  return rows * kb * 64;
}

hipError_t launch_ksk_prepare(void* frag, const uint64_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                              hipStream_t st) {
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level);
  const uint64_t total = (uint64_t)s.CT * s.KB * ks::Geo<false>::NPL * 64;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65535 * 4 ? (total + 255) / 256 : 65535 * 4);
  hipLaunchKernelGGL(ks::ksk_prepare_kernel<uint64_t>, dim3(grid), dim3(256), 0, st, (uint4*)frag, ksk, s);
  return hipGetLastError();
}

hipError_t launch_ksk32_prepare(void* frag, const uint32_t* ksk, size_t in_dim, size_t out_dim, int base_log,
                                int level, hipStream_t st) {
  const ks::Shape s = ks_shape(in_dim, out_dim, base_log, level, true);
  const uint64_t total = (uint64_t)s.CT * s.KB * ks::Geo<true>::NPL * 64;
  const unsigned grid = (unsigned)((total + 255) / 256 < 65535 * 4 ? (total + 255) / 256 : 65535 * 4);
  hipLaunchKernelGGL(ks::ksk_prepare_kernel<uint32_t>, dim3(grid), dim3(256), 0, st, (uint4*)frag, ksk, s);
  return hipGetLastError();
}

hipError_t launch_lwe_ms32(uint64_t* out, const uint32_t* in, size_t dim, size_t batch, int log_mod, bool centered,
                           hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const unsigned grid = (unsigned)((batch + 3) / 4);
  hipLaunchKernelGGL(ks::lwe_ms_kernel<uint32_t>, dim3(grid), dim3(256), 0, st, out, in, (uint32_t)dim,
                     (uint32_t)batch, (uint32_t)log_mod, centered ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_lwe_ms64(uint64_t* out, const uint64_t* in, size_t dim, size_t batch, int log_mod, bool centered,
                           hipStream_t st) {
  if (batch == 0) return hipSuccess;
  const unsigned grid = (unsigned)((batch + 3) / 4);
  hipLaunchKernelGGL(ks::lwe_ms_kernel<uint64_t>, dim3(grid), dim3(256), 0, st, out, in, (uint32_t)dim,
                     (uint32_t)batch, (uint32_t)log_mod, centered ? 1 : 0);
  return hipGetLastError();
}

// out_log 0: the native u64 keyswitch into `out` (u64); else KS32 into u32 words with output modulus 2^out_log
static hipError_t keyswitch_launch(void* out, const uint64_t* lwe_in, const void* frag, void* digits, size_t batch,
                                   size_t in_dim, size_t out_dim, int base_log, int level, int out_log, hipStream_t st) {
  if (batch == 0) return hipSuccess;
  ks::Shape s = ks_shape(in_dim, out_dim, base_log, level, out_log != 0);
  if (out_log) s.body_log = (uint32_t)out_log;
  const uint32_t rows = (uint32_t)((batch + 16 * ks::GM - 1) / (16 * ks::GM) * 16 * ks::GM);
  const uint64_t total = (uint64_t)rows * s.KB * 4;
  const unsigned dgrid = (unsigned)((total + 255) / 256 < 65535 * 4 ? (total + 255) / 256 : 65535 * 4);
  if (s.nd == 1 && (level == 1 || level == 2 || level == 4 || level == 8)) {
    auto kern = level == 1 ? ks::ks_digits_l_kernel<1> : level == 2 ? ks::ks_digits_l_kernel<2>
                : level == 4 ? ks::ks_digits_l_kernel<4> : ks::ks_digits_l_kernel<8>;
    const uint32_t kbw = level > 4 ? (uint32_t)level / 4 : 1;  // the kernel's KBW
    // one workgroup per row group and span of kbw k blocks (16 KiB each)
    const unsigned blocks = (unsigned)(rows / (16 * ks::GM) * ((s.KB + kbw - 1) / kbw));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, st, (uint4*)digits, lwe_in, (uint32_t)batch, rows, s);
  } else {
    hipLaunchKernelGGL(ks::ks_digits_kernel, dim3(dgrid), dim3(256), 0, st, (uint4*)digits, lwe_in, (uint32_t)batch,
                       rows, s);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t n_mg = rows / (16 * ks::GM), n_cg = s.CT / (out_log ? ks::Geo<true>::GN : ks::Geo<false>::GN);
  const uint32_t tiles = (n_mg + 7) / 8 * 8 * n_cg;
  const unsigned grid = 8 * ((tiles + 7) / 8);
  if (out_log)
    hipLaunchKernelGGL(ks::ks_gemm_kernel<true>, dim3(grid), dim3(64 * ks::NW), 0, st, out, lwe_in, (const uint4*)digits,
                       (const uint4*)frag, (uint32_t)batch, n_mg, s);
  else
    hipLaunchKernelGGL(ks::ks_gemm_kernel<false>, dim3(grid), dim3(64 * ks::NW), 0, st, out, lwe_in, (const uint4*)digits,
                       (const uint4*)frag, (uint32_t)batch, n_mg, s);
  return hipGetLastError();
}

hipError_t launch_keyswitch(uint64_t* out, const uint64_t* lwe_in, const void* frag, void* digits, size_t batch,
                            size_t in_dim, size_t out_dim, int base_log, int level, hipStream_t st) {
  return keyswitch_launch(out, lwe_in, frag, digits, batch, in_dim, out_dim, base_log, level, 0, st);
}

hipError_t launch_keyswitch32(uint32_t* out, const uint64_t* lwe_in, const void* frag, void* digits, size_t batch,
                              size_t in_dim, size_t out_dim, int base_log, int level, int out_log, hipStream_t st) {
  return keyswitch_launch(out, lwe_in, frag, digits, batch, in_dim, out_dim, base_log, level, out_log, st);
}

}  // namespace mi
