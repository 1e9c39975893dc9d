// c_api_internal.hpp — state shared by the C-ABI translation units (c_api*.cpp): the opaque handle
// structs of include/tfhe_ntt_amd.h and the error / device helpers.  Not part of the public surface.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/tfhe_ntt_amd.h"
#include "host_math.hpp"
#include "fft64_launch.hpp"
#include "ntt64_launch.hpp"

using mi::host::u128;
using mi::host::u64;

// largest log2 N of the split transform (launch_ntt_split): its block-twist tables hold 2 N u64
constexpr int MI_SPLIT_MAX_LOGN = 20;

struct mi_ntt64_plan {
  size_t n = 0;
  int logn = 0;
  u64 p = 0;
  int device = 0;
  bool goldilocks = false;
  bool twisted = false;  // N = 2048 Solinas: the twisted shift-twiddle kernel (ntt64_tw.hip)
  bool cached = false;   // owned by the process-wide plan cache (mi_ntt64_plan_cached); destroy is a no-op
  std::vector<u64> twid, inv_twid;  // canonical host tables (reference layout)
  u64 n_inv = 0;
  mi::MontParams mp;
  u64 c_normalize = 0, c_man = 0, c_macc = 0;  // device constants of the pointwise ops
  u64* d_twid = nullptr;
  u64* d_inv_twid = nullptr;
  // p < 2^32 (not Solinas): the transforms' Shoup32 tables, w | floor(w 2^32 / p) << 32, forward then inverse (2 N)
  u64* d_tw32 = nullptr;
  u64* d_itw32 = nullptr;
  // twisted N = 2048 Solinas transform (ntt64_tw.hip): rho_i^j and rho_i^-j, 64 i + j
  u64* d_twist_f = nullptr;
  u64* d_twist_i = nullptr;
  u64* d_twist_fn = nullptr;  // forward twist rows x N^-1 + the forward lane-pair twiddles (normalising key conversion)
  // Solinas 2^12 <= N <= 2^MI_SPLIT_MAX_LOGN: the split transform (ntt64_kernels.hip launch_ntt_split): d_split holds
  // the block twist alpha_b^j then alpha_b^-j (2 N u64); sub2048 is the cached 2048 plan whose body tables it uses
  u64* d_split = nullptr;
  const mi_ntt64_plan* sub2048 = nullptr;
  mi::SplitTw split_tables() const {
    mi::SplitTw t;
    t.blk_fwd = d_split;
    t.blk_inv = d_split + n;
    t.body_fwd = sub2048->d_twist_f;
    t.body_inv = sub2048->d_twist_i;
    return t;
  }
};

struct mi_fft64_plan {
  size_t n = 0;
  int device = 0;
  bool cached = false;
  bool generic = false;        // the shape-generic engine (N != 2048)
  double* d_tables = nullptr;  // N = 2048: t1 (2048) | t2 (96, padded to 128) | cm (32) | cmi (32) doubles;
                               // generic: tw | untw | wm (M complex each)
  mi::FftTables tables{};
  mi::FftGenTables gtables{};
};

struct mi_fft64_pbs_key {
  const mi_fft64_plan* plan = nullptr;
  const double* fbsk = nullptr;  // caller-owned Fourier key, or `owned`
  double* owned = nullptr;       // device copy made by mi_fft64_pbs_key_load
  size_t n_lwe = 0;
  int k = 1, base_log = 0, level = 0;
};

// a GGSW list made ready for the external product / CMUX (mi_ntt64_ggsw_create): the fused N = 2048 level-1 bodies read
// their GGSW in the W1' order (pbs_tw.hip), so for that shape the list is permuted once into a private copy instead of
// per call; every other shape references the caller's list
struct mi_ntt64_ggsw {
  const mi_ntt64_plan* plan = nullptr;
  size_t n_ggsw = 0;
  int k = 1, base_log = 0, level = 0, variant = 0;
  const u64* ggsw = nullptr;  // what the kernels read
  u64* owned = nullptr;       // the W1'-ordered private copy (or nullptr)
};

struct mi_pbs_ntt64_key {
  const mi_ntt64_plan* plan = nullptr;
  size_t n_lwe = 0;
  int k = 1, base_log = 0, level = 0, variant = 0;
  const u64* bsk = nullptr;  // what the kernel reads
  u64* owned = nullptr;      // private copy (prepare_pbs_key: BNF N^{-1} folded in; twisted engine: W1' order); loaded keys
};

namespace mi {
namespace capi {

std::string& last_error();

inline int fail(int status, const std::string& msg) {
  last_error() = msg;
  return status;
}

inline int hip_fail(hipError_t e, const char* what) {
  return fail(MI_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// shared by mi_pbs_ntt64_key_create and mi_pbs_ntt64_key_load
int check_pbs_shape(const mi_ntt64_plan* plan, int k, int base_log, int level, int variant);
// whether a consumer shape runs on the twisted N = 2048 engine (pbs_tw.hip: k = 1, level 1)
bool twisted_ext_applies(const mi_ntt64_plan* plan, int variant, int k, int base_log, int level);
// whether a PBS key of this shape needs a private device copy: BNF keys (N^{-1} folded in) and every key of the
// twisted engine (its blind rotation reads the key in its W1' register order)
bool pbs_key_needs_copy(const mi_ntt64_plan* plan, int variant, int k, int base_log, int level);
// fill that copy from src (dst may equal src; a no-op for a key that needs no copy when dst == src); synchronises
// `stream`
int prepare_pbs_key(const mi_ntt64_plan* plan, int variant, int k, int base_log, int level, u64* dst, const u64* src,
                    size_t count, hipStream_t stream);

}  // namespace capi
}  // namespace mi
