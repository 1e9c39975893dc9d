// c_api.cpp — the extern "C" boundary declared in include/tfhe_ntt_amd.h.
//
// Owns plan construction (host twiddles exactly as tfhe-ntt/src/prime64.rs:159-204 + 764-862,
// uploaded once to the plan's device) and argument validation; never aborts, every failure is
// a status code plus a thread-local message.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <tuple>
#include <vector>

#include "scratch.hpp"
#include "build_info.hpp"  // build/ (Makefile): MI_SOURCE_HASH
#include "keyswitch_launch.hpp"
#include "c_api_internal.hpp"
#include "mi_arith.hpp"
#include "ntt64_tw_tables.hpp"

namespace mi {
namespace capi {
std::string& last_error() {
  thread_local std::string msg;
  return msg;
}
}  // namespace capi
}  // namespace mi

using namespace mi::capi;

namespace {

u64 mont_form(u64 x, u64 p) { return (u64)(((u128)x << 64) % p); }

}  // namespace

extern "C" {

const char* mi_status_string(int status) {
  switch (status) {
    case MI_OK: return "ok";
    case MI_ERR_INVALID_ARG: return "invalid argument";
    case MI_ERR_NOT_PRIME: return "modulus is not prime";
    case MI_ERR_NO_ROOT: return "no primitive 2N-th root of unity for this modulus";
    case MI_ERR_HIP: return "HIP runtime error";
    case MI_ERR_OOM: return "device out of memory";
    case MI_ERR_UNSUPPORTED: return "unsupported by this build";
    default: return "unknown status";
  }
}

const char* mi_last_error_message(void) { return last_error().c_str(); }

const char* mi_build_source_hash(void) { return MI_SOURCE_HASH; }

static int plan_create(size_t n, uint64_t p, int device, mi_ntt64_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  // prime64.rs:769-775 — same order of checks as the reference
  if (n < 16 || (n & (n - 1)) != 0) return fail(MI_ERR_INVALID_ARG, "polynomial size must be a power of two >= 16");
  if (!mi::host::is_prime64(p)) return fail(MI_ERR_NOT_PRIME, "modulus is not prime");
  auto root = mi::host::find_primitive_root64(p, 2 * (u64)n);
  if (!root) return fail(MI_ERR_NO_ROOT, "no primitive 2N-th root of unity");
  const int logn = __builtin_ctzll(n);
  // N > 2^14 runs as passes of <= 4 top stages + 2^(logn - 14) blocks (ntt64_kernels.hip dispatch_large); the
  // reference's Solinas root exists up to 2N = 2^32 (roots.rs:96-107), other primes need 2N | p - 1 (checked above)
  if (logn > 31) return fail(MI_ERR_UNSUPPORTED, "this build runs N <= 2^31 on device");

  std::unique_ptr<mi_ntt64_plan> plan(new (std::nothrow) mi_ntt64_plan);
  if (!plan) return fail(MI_ERR_OOM, "host allocation failed");
  plan->n = n;
  plan->logn = logn;
  plan->p = p;
  plan->device = device;
  plan->goldilocks = (p == mi::host::SOLINAS_P);

  // prime64.rs:162-182: Solinas uses the hard-coded friendly root tower, other primes the
  // Tonelli-Shanks root.
  u64 w;
  if (plan->goldilocks) {
    auto r = mi::host::solinas_root(n);
    if (!r) { return fail(MI_ERR_NO_ROOT, "no Solinas root for this size"); }
    w = *r;
  } else {
    w = *root;
  }
  plan->twid.assign(n, 0);
  plan->inv_twid.assign(n, 0);
  u64 wk = 1;
  for (size_t k = 0; k < n; ++k) {  // prime64.rs:184-203
    plan->twid[mi::host::bit_rev(logn, k)] = wk;
    const unsigned inv_idx = mi::host::bit_rev(logn, (n - k) % n);
    plan->inv_twid[inv_idx] = (k == 0) ? wk : p - wk;
    wk = mi::host::mul_mod(wk, w, p);
  }
  plan->n_inv = mi::host::exp_mod((u64)n, p - 2, p);  // prime64.rs:844

  std::vector<u64> dev_tw(plan->twid), dev_itw(plan->inv_twid);
  if (plan->goldilocks) {
    plan->c_normalize = plan->n_inv;
    plan->c_man = plan->n_inv;
    plan->c_macc = 0;
  } else {
    u64 inv = p;  // Newton: p * inv == 1 mod 2^64
    for (int i = 0; i < 6; ++i) inv *= 2 - p * inv;
    plan->mp.p = p;
    plan->mp.pinv = (u64)0 - inv;
    const u64 r1 = (u64)(((u128)1 << 64) % p);
    plan->mp.r2 = mi::host::mul_mod(r1, r1, p);
    for (size_t k = 0; k < n; ++k) {
      dev_tw[k] = mont_form(dev_tw[k], p);
      dev_itw[k] = mont_form(dev_itw[k], p);
    }
    plan->c_normalize = mont_form(plan->n_inv, p);
    plan->c_man = mont_form(mont_form(plan->n_inv, p), p);
    plan->c_macc = plan->mp.r2;
  }

  DeviceGuard g(device);
  if (!g.ok) { return fail(MI_ERR_HIP, "hipSetDevice failed"); }
  if (hipMalloc(&plan->d_twid, n * sizeof(u64)) != hipSuccess ||
      hipMalloc(&plan->d_inv_twid, n * sizeof(u64)) != hipSuccess) {
    if (plan->d_twid) (void)hipFree(plan->d_twid);
    return fail(MI_ERR_OOM, "twiddle allocation failed");
  }
  hipError_t e = hipMemcpy(plan->d_twid, dev_tw.data(), n * sizeof(u64), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(plan->d_inv_twid, dev_itw.data(), n * sizeof(u64), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(plan->d_twid);
    (void)hipFree(plan->d_inv_twid);
    return hip_fail(e, "twiddle upload");
  }
  if (!plan->goldilocks && p < ((u64)1 << 32)) {  // the Shoup32 transform tables (mi_arith.hpp Shoup32)
    std::vector<u64> t32(2 * n);
    for (size_t k = 0; k < n; ++k) {
      t32[k] = plan->twid[k] | ((u64)(((u128)plan->twid[k] << 32) / p) << 32);
      t32[n + k] = plan->inv_twid[k] | ((u64)(((u128)plan->inv_twid[k] << 32) / p) << 32);
    }
    e = hipMalloc(&plan->d_tw32, 2 * n * sizeof(u64));
    if (e == hipSuccess) e = hipMemcpy(plan->d_tw32, t32.data(), 2 * n * sizeof(u64), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      if (plan->d_tw32) (void)hipFree(plan->d_tw32);
      (void)hipFree(plan->d_twid);
      (void)hipFree(plan->d_inv_twid);
      return hip_fail(e, "twiddle upload");
    }
    plan->d_itw32 = plan->d_tw32 + n;
  }
  if (plan->goldilocks && n == 2048) {
    // The twisted factorisation needs the reference's first five stages to use power-of-two
    // twiddles (the Solinas root tower, psi^64 = 8); check it against the tables it was built from.
    bool tower_ok = true;
    for (int st = 0; st < 5 && tower_ok; ++st)
      for (int g = 0; g < (1 << st); ++g)
        if (plan->twid[(1u << st) + g] != mi::host::exp_mod(2, (u64)mi::tw::G1_FWD[st][g], p)) tower_ok = false;
    if (tower_ok) {
      const u64 psi = plan->twid[mi::host::bit_rev(logn, 1)];
      std::vector<u64> tf(n + 32), ti(n + 32);
      for (int g = 0; g < 32; ++g) {  // twiddles of the lane-pair stage (ntt64_tw.hip)
        tf[n + g] = mi::host::exp_mod(2, (u64)mi::tw::CYC_FWD[5][g], p);
        ti[n + g] = mi::host::exp_mod(2, (u64)mi::tw::CYC_INV[5][g], p);
      }
      for (unsigned i = 0; i < 32; ++i) {
        const u64 rho = mi::host::exp_mod(psi, 2 * (u64)mi::host::bit_rev(5, i) + 1, p);
        const u64 rho_inv = mi::host::exp_mod(rho, p - 2, p);
        u64 f = 1, b = 1;
        for (unsigned j = 0; j < 64; ++j) {
          // the forward bodies' scale plan (ntt64_tw_tables.hpp, tools/tw_scale_plan.py): the five G1 stages leave
          // block i scaled by 2^TW_G1_OUT_SCALE[i], the cyclic stages take element j scaled by 2^TW_CYC_IN_SCALE[j >> 1]
          const int sc = (mi::tw::TW_CYC_IN_SCALE[0][j >> 1] - mi::tw::TW_G1_OUT_SCALE[0][i] + 192) % 192;
          tf[64 * i + j] = sc ? mi::host::mul_mod(f, mi::host::exp_mod(2, (u64)sc, p), p) : f;
          ti[64 * i + j] = b;
          f = mi::host::mul_mod(f, rho, p);
          b = mi::host::mul_mod(b, rho_inv, p);
        }
      }
      // one allocation [fwd | inverse | inverse with N^-1 folded into the untwist rows | the inverse's
      // last-DIT-stage twiddles | fwd with N^-1 folded into the twist rows]; the PBS / external-product bodies
      // address the first three from one base (pbs_tw.hip), the standalone inverse its untwist rows and the
      // fourth region, the normalising key conversion the last (ntt64_tw.hip)
      std::vector<u64> tn(ti);
      for (unsigned e = 0; e < n; ++e) tn[e] = mi::host::mul_mod(ti[e], plan->n_inv, p);
      // the standalone inverse's last DIT stage (joins j and j + 32 across a lane pair): entry m + 16 par is
      // 2^e with e = -3 (2 m + par) mod 192 = omega^-(2 m + par) (tools/gen_tw_kernel.py inv_last_exp)
      std::vector<u64> tl(32);
      for (unsigned m = 0; m < 16; ++m)
        for (unsigned par = 0; par < 2; ++par)
          tl[m + 16 * par] = mi::host::exp_mod(2, (u64)((192 - 3 * (2 * m + par) % 192) % 192), p);
      std::vector<u64> tfn(tf);  // the normalising key conversion's forward twist (lane-pair twiddles unscaled)
      for (unsigned e = 0; e < n; ++e) tfn[e] = mi::host::mul_mod(tf[e], plan->n_inv, p);
      if (hipMalloc(&plan->d_twist_f, (4 * (n + 32) + 32) * sizeof(u64)) == hipSuccess &&
          hipMemcpy(plan->d_twist_f + 3 * (n + 32), tl.data(), 32 * sizeof(u64), hipMemcpyHostToDevice) ==
              hipSuccess &&
          hipMemcpy(plan->d_twist_f + 3 * (n + 32) + 32, tfn.data(), (n + 32) * sizeof(u64),
                    hipMemcpyHostToDevice) == hipSuccess &&
          hipMemcpy(plan->d_twist_f, tf.data(), (n + 32) * sizeof(u64), hipMemcpyHostToDevice) == hipSuccess &&
          hipMemcpy(plan->d_twist_f + n + 32, ti.data(), (n + 32) * sizeof(u64), hipMemcpyHostToDevice) ==
              hipSuccess &&
          hipMemcpy(plan->d_twist_f + 2 * (n + 32), tn.data(), (n + 32) * sizeof(u64), hipMemcpyHostToDevice) ==
              hipSuccess) {
        plan->d_twist_i = plan->d_twist_f + n + 32;
        plan->d_twist_fn = plan->d_twist_f + 3 * (n + 32) + 32;
      } else {
        if (plan->d_twist_f) (void)hipFree(plan->d_twist_f);
        plan->d_twist_f = plan->d_twist_i = nullptr;
        (void)hipFree(plan->d_twid);
        (void)hipFree(plan->d_inv_twid);
            return fail(MI_ERR_OOM, "twist table allocation failed");
      }
    }
  }
  plan->twisted = plan->d_twist_f != nullptr;
  if (plan->goldilocks && logn >= 12 && logn <= MI_SPLIT_MAX_LOGN) {
    // the split transform (launch_ntt_split): needs the 2048 plan's twisted body and the root tower
    // psi_N^(N / 2048) = psi_2048 (prime64.rs:166-177), checked here against the tables both plans were built from
    const mi_ntt64_plan* sub = nullptr;
    const u64 psi = plan->twid[mi::host::bit_rev(logn, 1)];
    // the top passes at stage 0 multiply by shifts (Goldilocks::mul_pow2): entries 1 .. 31 of both tables must be
    // the powers of two tower_exp names
    bool pow2_ok = true;
    for (int st = 0; st < 5; ++st)
      for (int g = 0; g < (1 << st); ++g) {
        const size_t i = ((size_t)1 << st) + g;
        pow2_ok = pow2_ok && plan->twid[i] == mi::host::exp_mod(2, (u64)mi::tower_exp(true, st, g), p) &&
                  plan->inv_twid[i] == mi::host::exp_mod(2, (u64)mi::tower_exp(false, st, g), p);
      }
    // a failure to build the cached 2048 sub-plan (e.g. a transient OOM) fails this plan too, with the sub-plan's
    // status and message, instead of quietly leaving it on the slower window kernels for its lifetime
    if (pow2_ok) {
      const int rc = mi_ntt64_plan_cached(2048, p, device, &sub);
      if (rc != MI_OK) {
        (void)hipFree(plan->d_twid);
        (void)hipFree(plan->d_inv_twid);
        return rc;
      }
    }
    if (pow2_ok && sub->twisted &&
        mi::host::exp_mod(psi, (u64)(n / 2048), p) == sub->twid[mi::host::bit_rev(11, 1)]) {
      const int t = logn - 11;
      std::vector<u64> blk(2 * n);
      for (size_t b = 0; b < ((size_t)1 << t); ++b) {
        // alpha_b = psi^(2 bitrev_t(b) + 1 - 2^t mod 2N)
        const u64 e = (2 * (u64)mi::host::bit_rev(t, (unsigned)b) + 1 + 2 * (u64)n - ((u64)1 << t)) % (2 * (u64)n);
        const u64 a = mi::host::exp_mod(psi, e, p), ai = mi::host::exp_mod(a, p - 2, p);
        u64 f = 1, g = 1;
        for (size_t j = 0; j < 2048; ++j) {
          blk[b * 2048 + j] = f;
          blk[n + b * 2048 + j] = g;
          f = mi::host::mul_mod(f, a, p);
          g = mi::host::mul_mod(g, ai, p);
        }
      }
      if (hipMalloc(&plan->d_split, 2 * n * sizeof(u64)) != hipSuccess) {
        (void)hipFree(plan->d_twid);
        (void)hipFree(plan->d_inv_twid);
        return fail(MI_ERR_OOM, "split-transform table allocation failed");
      }
      if (hipMemcpy(plan->d_split, blk.data(), 2 * n * sizeof(u64), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(plan->d_split);
        (void)hipFree(plan->d_twid);
        (void)hipFree(plan->d_inv_twid);
        return fail(MI_ERR_HIP, "split-transform table upload failed");
      }
      plan->sub2048 = sub;
    }
  }
  *out_plan = plan.release();
  return MI_OK;
}

// the host tables (2 x N u64 plus their device-form copies: ~64 GiB at N = 2^31) are std::vectors: an allocation
// failure is returned as MI_ERR_OOM instead of unwinding through the C ABI (plan_create holds the plan in a
// unique_ptr, and every device allocation comes after the large host tables)
int mi_ntt64_plan_create(size_t n, uint64_t p, int device, mi_ntt64_plan** out_plan) {
  try {
    return plan_create(n, p, device, out_plan);
  } catch (const std::bad_alloc&) {
    if (out_plan) *out_plan = nullptr;
    return fail(MI_ERR_OOM, "host allocation of the twiddle tables failed");
  }
}

int mi_ntt64_plan_destroy(mi_ntt64_plan* plan) {
  if (!plan || plan->cached) return MI_OK;
  {
    DeviceGuard g(plan->device);
    if (plan->d_twid) (void)hipFree(plan->d_twid);
    if (plan->d_inv_twid) (void)hipFree(plan->d_inv_twid);
    if (plan->d_twist_f) (void)hipFree(plan->d_twist_f);  // d_twist_i points into the same allocation
    if (plan->d_split) (void)hipFree(plan->d_split);
    if (plan->d_tw32) (void)hipFree(plan->d_tw32);  // d_itw32 points into the same allocation
  }
  delete plan;
  return MI_OK;
}

// Ntt64::new's PLANS map (ntt64.rs:27-79): a read-locked probe, then one slot per key whose plan is built under
// that slot's own mutex, so concurrent first users of one (n, p, device) build it once and other keys are not
// blocked behind that build.  A failed build is not cached (the reference's map only ever holds built plans):
// the slot stays empty and the next caller retries, so a transient failure (e.g. an OOM while uploading the
// tables) does not make the key unusable for the rest of the process.
int mi_ntt64_plan_cached(size_t n, uint64_t p, int device, const mi_ntt64_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  struct Slot {
    std::mutex build;
    std::atomic<mi_ntt64_plan*> plan{nullptr};
  };
  static std::shared_mutex mu;
  static std::map<std::tuple<size_t, uint64_t, int>, std::unique_ptr<Slot>>* plans =
      new std::map<std::tuple<size_t, uint64_t, int>, std::unique_ptr<Slot>>;  // never destroyed, like PLANS
  const auto key = std::make_tuple(n, p, device);
  Slot* slot = nullptr;
  {
    std::shared_lock<std::shared_mutex> rd(mu);
    auto it = plans->find(key);
    if (it != plans->end()) slot = it->second.get();
  }
  if (!slot) {
    std::unique_lock<std::shared_mutex> wr(mu);
    auto& ent = (*plans)[key];
    if (!ent) ent.reset(new Slot);
    slot = ent.get();
  }
  mi_ntt64_plan* built = slot->plan.load(std::memory_order_acquire);
  if (!built) {
    std::lock_guard<std::mutex> lk(slot->build);
    built = slot->plan.load(std::memory_order_acquire);
    if (!built) {
      const int st = mi_ntt64_plan_create(n, p, device, &built);
      if (st != MI_OK) return st;  // last_error() already holds the reason; nothing is cached
      built->cached = true;
      slot->plan.store(built, std::memory_order_release);
    }
  }
  *out_plan = built;
  return MI_OK;
}

int mi_ntt64_plan_info(const mi_ntt64_plan* plan, size_t* n, uint64_t* p, int* device) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (n) *n = plan->n;
  if (p) *p = plan->p;
  if (device) *device = plan->device;
  return MI_OK;
}

int mi_ntt64_plan_twiddles(const mi_ntt64_plan* plan, uint64_t* twid, uint64_t* inv_twid, uint64_t* n_inv) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (twid) std::memcpy(twid, plan->twid.data(), plan->n * sizeof(u64));
  if (inv_twid) std::memcpy(inv_twid, plan->inv_twid.data(), plan->n * sizeof(u64));
  if (n_inv) *n_inv = plan->n_inv;
  return MI_OK;
}

static int check_batch(const mi_ntt64_plan* plan, const void* buf, size_t batch, size_t stride) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (batch == 0) return MI_OK;
  if (!buf) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (stride < plan->n) return fail(MI_ERR_INVALID_ARG, "stride < ntt size");
  if (batch > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  return MI_OK;
}

// Kernel routing: the twisted shift-twiddle kernel for the Solinas N = 2048 plan, the split transform (top passes +
// that kernel on 2048-blocks) for Solinas 2^12 <= N <= 2^MI_SPLIT_MAX_LOGN, else the register-window kernels (Shoup32
// arithmetic for p < 2^32, Montgomery above).  One kernel per plan shape; nothing in the environment changes it.
static hipError_t launch_transform(bool fwd, const mi_ntt64_plan* plan, uint64_t* buf, size_t batch, size_t stride,
                                   hipStream_t s) {
  if (plan->twisted)
    return mi::launch_ntt_tw(fwd, buf, batch, stride, fwd ? plan->d_twist_f : plan->d_twist_i, s);
  if (plan->d_split)
    return mi::launch_ntt_split(fwd, plan->logn, buf, batch, stride, fwd ? plan->d_twid : plan->d_inv_twid,
                                plan->split_tables(), s);
  if (plan->d_tw32)
    return mi::launch_ntt_shoup32(fwd, plan->logn, (uint32_t)plan->p, buf, nullptr, batch, stride,
                                  fwd ? plan->d_tw32 : plan->d_itw32, s);
  return mi::launch_ntt(fwd, plan->logn, plan->goldilocks, plan->mp, buf, batch, stride,
                        fwd ? plan->d_twid : plan->d_inv_twid, s);
}

static int run_ntt(bool fwd, const mi_ntt64_plan* plan, uint64_t* buf, size_t batch, size_t stride, void* stream) {
  int st = check_batch(plan, buf, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  DeviceGuard g(plan->device);
  hipError_t e = launch_transform(fwd, plan, buf, batch, stride, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, fwd ? "fwd launch" : "inv launch");
}

int mi_ntt64_fwd_batch(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch, size_t stride, void* stream) {
  return run_ntt(true, plan, buf, batch, stride, stream);
}

int mi_ntt64_inv_batch(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch, size_t stride, void* stream) {
  return run_ntt(false, plan, buf, batch, stride, stream);
}

static int run_pw(int op, const mi_ntt64_plan* plan, uint64_t* out, const uint64_t* a, const uint64_t* b,
                  size_t batch, size_t stride, void* stream) {
  int st = check_batch(plan, out, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  if (op >= 1 && !b) return fail(MI_ERR_INVALID_ARG, "rhs is NULL");
  if (op == 2 && !a) return fail(MI_ERR_INVALID_ARG, "lhs is NULL");
  const u64 c = op == 0 ? plan->c_normalize : (op == 1 ? plan->c_man : plan->c_macc);
  DeviceGuard g(plan->device);
  hipError_t e = mi::launch_pointwise(op, plan->goldilocks, plan->mp, out, a, b, plan->n, batch, stride, c,
                                      (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "pointwise launch");
}

int mi_ntt64_normalize_batch(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch, size_t stride, void* stream) {
  return run_pw(0, plan, buf, nullptr, nullptr, batch, stride, stream);
}

int mi_ntt64_mul_assign_normalize_batch(const mi_ntt64_plan* plan, uint64_t* lhs, const uint64_t* rhs, size_t batch,
                                        size_t stride, void* stream) {
  return run_pw(1, plan, lhs, nullptr, rhs, batch, stride, stream);
}

int mi_ntt64_mul_accumulate_batch(const mi_ntt64_plan* plan, uint64_t* acc, const uint64_t* lhs, const uint64_t* rhs,
                                  size_t batch, size_t stride, void* stream) {
  return run_pw(2, plan, acc, lhs, rhs, batch, stride, stream);
}

// ---- the Ntt64View layer (tfhe/src/core_crypto/commons/math/ntt/ntt64.rs:89-266), batched ------------------------
// The Solinas N = 2048 plan runs the fused twisted bodies (ntt64_view.hip: one launch, conversions at load / store);
// every other plan an elementwise pass around its own transform.  Two operands of one call are either the same buffer
// (forward forms only) or disjoint.
static bool view_overlap(const uint64_t* a, const uint64_t* b, size_t n, size_t batch, size_t stride) {
  const size_t span = (batch - 1) * stride + n;
  return a < b + span && b < a + span;
}

static int run_view_fwd(const mi_ntt64_plan* plan, int kind, unsigned width, bool normalized, uint64_t* ntt,
                        const uint64_t* standard, size_t batch, size_t stride, void* stream) {
  int st = check_batch(plan, ntt, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  if (!standard) return fail(MI_ERR_INVALID_ARG, "standard buffer is NULL");
  if (kind == 1 && (width < 1 || width > 64))
    return fail(MI_ERR_INVALID_ARG, "input_modulus_width must be in [1, 64]");
  if (ntt != standard && view_overlap(ntt, standard, plan->n, batch, stride))
    return fail(MI_ERR_INVALID_ARG, "ntt and standard must be the same buffer or disjoint");
  DeviceGuard g(plan->device);
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (plan->twisted) {
    e = mi::launch_view_fwd_tw(kind, ntt, standard, batch, stride, width,
                               normalized ? plan->d_twist_fn : plan->d_twist_f, s);
  } else {
    if (kind != 0 || ntt != standard)
      e = mi::launch_view_pre(kind, ntt, standard, plan->n, batch, stride, width, plan->p, s);
    if (e == hipSuccess) e = launch_transform(true, plan, ntt, batch, stride, s);
    if (e == hipSuccess && normalized)
      e = mi::launch_pointwise(0, plan->goldilocks, plan->mp, ntt, nullptr, nullptr, plan->n, batch, stride,
                               plan->c_normalize, s);
  }
  return e == hipSuccess ? MI_OK : hip_fail(e, "Ntt64View forward launch");
}

int mi_ntt64_forward_batch(const mi_ntt64_plan* plan, uint64_t* ntt, const uint64_t* standard, size_t batch,
                           size_t stride, void* stream) {
  return run_view_fwd(plan, 0, 0, false, ntt, standard, batch, stride, stream);
}

int mi_ntt64_forward_normalized_batch(const mi_ntt64_plan* plan, uint64_t* ntt, const uint64_t* standard, size_t batch,
                                      size_t stride, void* stream) {
  return run_view_fwd(plan, 0, 0, true, ntt, standard, batch, stride, stream);
}

int mi_ntt64_forward_from_power_of_two_modulus_batch(const mi_ntt64_plan* plan, unsigned input_modulus_width,
                                                     uint64_t* ntt, const uint64_t* standard, size_t batch,
                                                     size_t stride, void* stream) {
  return run_view_fwd(plan, 1, input_modulus_width, false, ntt, standard, batch, stride, stream);
}

int mi_ntt64_forward_from_decomp_batch(const mi_ntt64_plan* plan, uint64_t* ntt, const uint64_t* decomp, size_t batch,
                                       size_t stride, void* stream) {
  return run_view_fwd(plan, 2, 0, false, ntt, decomp, batch, stride, stream);
}

// width 0: add_backward (custom modulus); else add_backward_on_power_of_two_modulus with that output width
static int run_view_add(const mi_ntt64_plan* plan, unsigned width, uint64_t* standard, uint64_t* ntt, size_t batch,
                        size_t stride, void* stream) {
  int st = check_batch(plan, ntt, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  if (!standard) return fail(MI_ERR_INVALID_ARG, "standard buffer is NULL");
  if (view_overlap(ntt, standard, plan->n, batch, stride))
    return fail(MI_ERR_INVALID_ARG, "standard and ntt must be disjoint");
  DeviceGuard g(plan->device);
  const hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  if (plan->twisted && (width == 0 || width == 64)) {
    e = mi::launch_view_inv_tw(width == 64, standard, ntt, batch, stride, plan->d_twist_i, s);
  } else {
    e = launch_transform(false, plan, ntt, batch, stride, s);
    if (e == hipSuccess) e = mi::launch_view_post(standard, ntt, plan->n, batch, stride, width, plan->p, s);
  }
  return e == hipSuccess ? MI_OK : hip_fail(e, "Ntt64View add_backward launch");
}

int mi_ntt64_add_backward_batch(const mi_ntt64_plan* plan, uint64_t* standard, uint64_t* ntt, size_t batch,
                                size_t stride, void* stream) {
  return run_view_add(plan, 0, standard, ntt, batch, stride, stream);
}

int mi_ntt64_add_backward_on_power_of_two_modulus_batch(const mi_ntt64_plan* plan, unsigned output_modulus_width,
                                                        uint64_t* standard, uint64_t* ntt, size_t batch, size_t stride,
                                                        void* stream) {
  if (output_modulus_width < 1 || output_modulus_width > 64)
    return fail(MI_ERR_INVALID_ARG, "output_modulus_width must be in [1, 64]");
  return run_view_add(plan, output_modulus_width, standard, ntt, batch, stride, stream);
}

// The `&mut [u64]` host form (Plan::fwd / Plan::inv on a caller slice, as Ntt64View::forward / add_backward call
// it per polynomial, ntt64.rs:89-137).  Each call borrows a staging slot of the plan's device from a process-wide
// pool: a private non-blocking stream of the highest priority, a device buffer and a mapped, coherent pinned host buffer, all grown on
// demand and reused.  Up to ZERO_COPY_BYTES the transform runs in place on the pinned buffer itself (the kernel
// reads and writes host memory over PCIe: one launch and one wait per call instead of two copies around the
// launch); above it a call is memcpy -> async H2D -> transform -> async D2H -> wait -> memcpy.  No allocation in the
// steady state, and nothing else of the process is synchronised (no hipDeviceSynchronize), so concurrent callers
// (rayon workers) each run on their own slot and stream.
}  // extern "C"

namespace {
struct HostSlot {
  int device = 0;
  hipStream_t stream = nullptr;
  u64* dbuf = nullptr;
  u64* hbuf = nullptr;   // pinned, mapped, coherent
  u64* hdev = nullptr;   // hbuf's device address
  size_t cap = 0;        // u64 elements of both buffers
};

// in-place transform on the mapped host buffer up to this size (profiles/r3/host_path_zero_copy.json against the
// staged rows of profiles/r3/bench_line_driver_cmd.json: faster up to 2 MiB per call — 39.8 vs 46.8 us for one
// N = 1024 round trip, 51.6 vs 87.5 us at 16 polynomials — and level with the staged call at 4 MiB)
constexpr size_t ZERO_COPY_BYTES = (size_t)2 << 20;

struct HostSlotPool {
  std::mutex mu;
  std::vector<HostSlot*> free;  // slots are never destroyed: the pool lives until process exit, as PLANS does
};

HostSlotPool& host_pool() {
  static HostSlotPool* p = new HostSlotPool;
  return *p;
}

HostSlot* acquire_slot(int device) {
  HostSlotPool& pool = host_pool();
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    for (size_t i = 0; i < pool.free.size(); ++i)
      if (pool.free[i]->device == device) {
        HostSlot* s = pool.free[i];
        pool.free[i] = pool.free.back();
        pool.free.pop_back();
        return s;
      }
  }
  HostSlot* s = new (std::nothrow) HostSlot;
  if (!s) return nullptr;
  s->device = device;
  // the highest stream priority: a per-polynomial host call is latency-bound, and a high-priority stream gets
  // hardware queues of its own, so it is never queued behind bulk work of the process's normal-priority streams
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
  if (hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, greatest) != hipSuccess) {
    delete s;
    return nullptr;
  }
  return s;
}

void release_slot(HostSlot* s) {
  HostSlotPool& pool = host_pool();
  std::lock_guard<std::mutex> lk(pool.mu);
  pool.free.push_back(s);
}

hipError_t slot_reserve(HostSlot* s, size_t elems) {
  if (elems <= s->cap) return hipSuccess;
  hipError_t e = hipStreamSynchronize(s->stream);
  if (s->dbuf) (void)hipFree(s->dbuf);
  if (s->hbuf) (void)hipHostFree(s->hbuf);
  s->dbuf = s->hbuf = s->hdev = nullptr;
  s->cap = 0;
  if (e == hipSuccess) e = hipMalloc(&s->dbuf, elems * sizeof(u64));
  if (e == hipSuccess)
    e = hipHostMalloc(&s->hbuf, elems * sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable);
  if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&s->hdev, s->hbuf, 0);
  if (e == hipSuccess) s->cap = elems;
  return e;
}
}  // namespace

extern "C" {

static int run_host(bool fwd, const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) {
  int st = check_batch(plan, buf, batch, plan ? plan->n : 0);
  if (st != MI_OK || batch == 0) return st;
  DeviceGuard g(plan->device);
  if (!g.ok) return fail(MI_ERR_HIP, "hipSetDevice failed");
  HostSlot* slot = acquire_slot(plan->device);
  if (!slot) return fail(MI_ERR_HIP, "staging stream creation failed");
  const size_t elems = batch * plan->n, bytes = elems * sizeof(u64);
  hipError_t e = slot_reserve(slot, elems);
  if (e != hipSuccess) {
    release_slot(slot);
    return fail(MI_ERR_OOM, std::string("staging buffer allocation failed: ") + hipGetErrorString(e));
  }
  std::memcpy(slot->hbuf, buf, bytes);
  if (bytes <= ZERO_COPY_BYTES) {
    e = launch_transform(fwd, plan, slot->hdev, batch, plan->n, slot->stream);
  } else {
    e = hipMemcpyAsync(slot->dbuf, slot->hbuf, bytes, hipMemcpyHostToDevice, slot->stream);
    if (e == hipSuccess) e = launch_transform(fwd, plan, slot->dbuf, batch, plan->n, slot->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(slot->hbuf, slot->dbuf, bytes, hipMemcpyDeviceToHost, slot->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(slot->stream);
  if (e == hipSuccess) std::memcpy(buf, slot->hbuf, bytes);
  release_slot(slot);
  return e == hipSuccess ? MI_OK : hip_fail(e, "host transform");
}

int mi_ntt64_fwd_host(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) { return run_host(true, plan, buf, batch); }

// The host form of the pointwise ops (Plan::normalize / mul_assign_normalize / mul_accumulate on `&mut [u64]`,
// prime64.rs:1050-1222; update_with_fmadd's per-polynomial calls, ntt64_pbs.rs:683-702): the operands go into one
// pooled staging slot (operand k at k * batch * n), the kernel runs on the slot's stream — in place on the mapped
// pinned buffer up to ZERO_COPY_BYTES, staged through the slot's device buffer above — and the result comes back.
// Same slot pool as run_host: no allocation and no device-wide synchronisation in the steady state.
static int run_host_pw(int op, const mi_ntt64_plan* plan, uint64_t* out, const uint64_t* a, const uint64_t* b,
                       size_t batch) {
  int st = check_batch(plan, out, batch, plan ? plan->n : 0);
  if (st != MI_OK || batch == 0) return st;
  if (op >= 1 && !b) return fail(MI_ERR_INVALID_ARG, "rhs is NULL");
  if (op == 2 && !a) return fail(MI_ERR_INVALID_ARG, "lhs is NULL");
  DeviceGuard g(plan->device);
  if (!g.ok) return fail(MI_ERR_HIP, "hipSetDevice failed");
  HostSlot* slot = acquire_slot(plan->device);
  if (!slot) return fail(MI_ERR_HIP, "staging stream creation failed");
  const size_t elems = batch * plan->n, bytes = elems * sizeof(u64);
  const size_t nops = op == 0 ? 1 : (op == 1 ? 2 : 3);
  hipError_t e = slot_reserve(slot, nops * elems);
  if (e != hipSuccess) {
    release_slot(slot);
    return fail(MI_ERR_OOM, std::string("staging buffer allocation failed: ") + hipGetErrorString(e));
  }
  // operand order in the slot: out, then a (mul_accumulate's lhs), then b (the rhs)
  std::memcpy(slot->hbuf, out, bytes);
  if (op == 2) std::memcpy(slot->hbuf + elems, a, bytes);
  if (op >= 1) std::memcpy(slot->hbuf + (nops - 1) * elems, b, bytes);
  const bool zero_copy = nops * bytes <= ZERO_COPY_BYTES;
  u64* base = zero_copy ? slot->hdev : slot->dbuf;
  if (!zero_copy) e = hipMemcpyAsync(slot->dbuf, slot->hbuf, nops * bytes, hipMemcpyHostToDevice, slot->stream);
  const u64 c = op == 0 ? plan->c_normalize : (op == 1 ? plan->c_man : plan->c_macc);
  if (e == hipSuccess)
    e = mi::launch_pointwise(op, plan->goldilocks, plan->mp, base, op == 2 ? base + elems : nullptr,
                             op >= 1 ? base + (nops - 1) * elems : nullptr, plan->n, batch, plan->n, c, slot->stream);
  if (e == hipSuccess && !zero_copy) e = hipMemcpyAsync(slot->hbuf, slot->dbuf, bytes, hipMemcpyDeviceToHost, slot->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(slot->stream);
  if (e == hipSuccess) std::memcpy(out, slot->hbuf, bytes);
  release_slot(slot);
  return e == hipSuccess ? MI_OK : hip_fail(e, "host pointwise op");
}

int mi_ntt64_normalize_host(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) {
  return run_host_pw(0, plan, buf, nullptr, nullptr, batch);
}

int mi_ntt64_mul_assign_normalize_host(const mi_ntt64_plan* plan, uint64_t* lhs, const uint64_t* rhs, size_t batch) {
  return run_host_pw(1, plan, lhs, nullptr, rhs, batch);
}

int mi_ntt64_mul_accumulate_host(const mi_ntt64_plan* plan, uint64_t* acc, const uint64_t* lhs, const uint64_t* rhs,
                                 size_t batch) {
  return run_host_pw(2, plan, acc, lhs, rhs, batch);
}

int mi_ntt64_inv_host(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) { return run_host(false, plan, buf, batch); }

int mi_fill_uniform(uint64_t* buf, size_t count, uint64_t seed, uint64_t p, int device, void* stream) {
  if (count == 0) return MI_OK;
  if (!buf) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  DeviceGuard g(device);
  hipError_t e = mi::launch_fill_uniform(buf, count, seed, p, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fill launch");
}

// ---- external product / PBS ------------------------------------------------------------------

}  // extern "C"

// polynomial sizes from which the PBS / external product run as device-wide passes with the accumulators in HBM
// (pbs_large.hip) instead of one fused workgroup per ciphertext (pbs_kernels.hip): at N = 8192 the fused kernel (1024
// lanes, 128 VGPRs, spilling) takes 994.5 ms per 1024 PBS of the 3_3 shape, the passes 786.7 ms; below it the fused
// kernels win (profiles/r3/fused_vs_large_pbs.txt)
static constexpr int LARGE_PATH_MIN_LOGN = 13;

int mi::capi::check_pbs_shape(const mi_ntt64_plan* plan, int k, int base_log, int level, int variant) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (variant != MI_NTT64_SOLINAS && variant != MI_NTT64_BNF) return fail(MI_ERR_INVALID_ARG, "unknown variant");
  if (level < 1 || base_log < 1 || base_log * level > 63)
    return fail(MI_ERR_INVALID_ARG, "decomposition must satisfy level >= 1, base_log >= 1, base_log*level < 64");
  // the compiled shapes (pbs_kernels.hip): N in {1024, 2048, 4096} with k in {1, 2}, N = 512 with k in {1, 4}
  // (PARAM_MESSAGE_1_CARRY_1), N = 8192 with k = 1 (PARAM_MESSAGE_3_CARRY_3)
  const int ln = plan->logn;
  // (PARAM_MESSAGE_1_CARRY_1); and N = 2^13 ... 2^17 with k in {1, 2} on the multi-kernel path of pbs_large.hip
  // (PARAM_MESSAGE_3_CARRY_3: N = 8192, 4_4: N = 65536)
  const bool shape_ok = plan->goldilocks && ((ln >= 10 && ln <= 12 && (k == 1 || k == 2)) ||
                                             (ln == 9 && (k == 1 || k == 4)) ||
                                             (ln >= LARGE_PATH_MIN_LOGN && ln <= 17 && (k == 1 || k == 2)));
  if (!shape_ok)
    return fail(MI_ERR_UNSUPPORTED,
                "external product / PBS run for the Solinas plan at N in {1024, 2048, 4096} with k in {1, 2}, "
                "N = 512 with k in {1, 4}, N in {8192, ..., 131072} with k in {1, 2}");
  return MI_OK;
}

// the split-transform tables of a plan (launch_ntt_split), or NULL: the large-N passes then run the window kernels.
// Returns a pointer to thread-local storage, valid until the next call on this thread.
static const mi::SplitTw* split_of(const mi_ntt64_plan* plan) {
  thread_local mi::SplitTw t;
  if (!plan->d_split) return nullptr;
  t = plan->split_tables();
  return &t;
}

// the twisted-transform bodies (pbs_tw.hip) cover level 1, base_log <= 31 (BNF and Solinas) on the
// Solinas N = 2048 plan; every other shape runs the generic kernels (pbs_kernels.hip)
bool mi::capi::twisted_ext_applies(const mi_ntt64_plan* plan, int variant, int k, int base_log, int level) {
  (void)variant;
  return k == 1 && level == 1 && base_log <= 31 && plan->twisted;
}

extern "C" {

int mi_bsk_to_ntt64(const mi_ntt64_plan* plan, const uint64_t* bsk_std, uint64_t* bsk_ntt, size_t n_polys,
                    unsigned in_modulus_width, int normalize, void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (n_polys == 0) return MI_OK;
  if (!bsk_std || !bsk_ntt) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (in_modulus_width > 64) return fail(MI_ERR_INVALID_ARG, "in_modulus_width > 64");
  if (!plan->goldilocks || plan->logn < 9 || plan->logn > 17)
    return fail(MI_ERR_UNSUPPORTED, "key conversion runs for the Solinas plan at N in {512, ..., 131072}");
  if (n_polys > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "too many polynomials");
  DeviceGuard g(plan->device);
  if (plan->twisted && in_modulus_width == 64) {  // the fused twisted-body conversion (ntt64_tw.hip)
    hipError_t e = mi::launch_ntt_tw_ms64(bsk_ntt, bsk_std, n_polys, normalize ? plan->d_twist_fn : plan->d_twist_f,
                                          (hipStream_t)stream);
    return e == hipSuccess ? MI_OK : hip_fail(e, "bsk conversion launch");
  }
  hipError_t e = plan->logn > 13  // the fused conversion kernel covers N <= 8192
                     ? mi::launch_bsk_to_ntt_large(plan->logn, bsk_ntt, bsk_std, n_polys, in_modulus_width,
                                                   normalize ? 1 : 0, plan->n_inv, plan->d_twid, (hipStream_t)stream,
                                                   split_of(plan))
                     : mi::launch_bsk_to_ntt(plan->logn, bsk_ntt, bsk_std, n_polys, in_modulus_width, normalize ? 1 : 0,
                                             plan->n_inv, plan->d_twid, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "bsk conversion launch");
}

static int ext_common(const mi_ntt64_plan* plan, bool cmux, uint64_t* out, uint64_t* in, const uint64_t* ggsw,
                      const uint32_t* gidx, size_t n_ggsw, int k, int base_log, int level, size_t batch, int variant,
                      void* stream, bool prepared = false) {
  int st = check_pbs_shape(plan, k, base_log, level, variant);
  if (st != MI_OK) return st;
  if (batch == 0) return MI_OK;
  if (!out || !in || !ggsw) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  if (n_ggsw == 0 || n_ggsw > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "GGSW count out of range");
  DeviceGuard g(plan->device);
  hipError_t e;
  if (twisted_ext_applies(plan, variant, k, base_log, level))
    e = mi::launch_ext_tw(cmux, variant == MI_NTT64_SOLINAS, out, in, ggsw, batch, base_log, plan->d_twist_f,
                          (hipStream_t)stream, gidx, (uint32_t)n_ggsw, prepared);
  else if (plan->logn >= LARGE_PATH_MIN_LOGN)
    e = mi::launch_ext_product_large(plan->logn, k, variant == MI_NTT64_BNF, cmux, level, out, in, ggsw, batch,
                                     base_log, plan->d_twid, plan->d_inv_twid, plan->n_inv, (hipStream_t)stream, gidx,
                                     (uint32_t)n_ggsw, split_of(plan));
  else
    e = mi::launch_ext_product(plan->logn, k, variant == MI_NTT64_BNF, cmux, level, out, in, ggsw, batch, base_log,
                               plan->d_twid, plan->d_inv_twid, plan->n_inv, (hipStream_t)stream, gidx,
                               (uint32_t)n_ggsw);
  return e == hipSuccess ? MI_OK : hip_fail(e, cmux ? "cmux launch" : "external product launch");
}

int mi_ntt64_ggsw_create(const mi_ntt64_plan* plan, const uint64_t* ggsw_list, size_t n_ggsw, int k, int base_log,
                         int level, int variant, void* stream, mi_ntt64_ggsw** out) {
  if (!out) return fail(MI_ERR_INVALID_ARG, "out is NULL");
  *out = nullptr;
  int st = check_pbs_shape(plan, k, base_log, level, variant);
  if (st != MI_OK) return st;
  if (!ggsw_list) return fail(MI_ERR_INVALID_ARG, "ggsw_list is NULL");
  if (n_ggsw == 0 || n_ggsw > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "GGSW count out of range");
  std::unique_ptr<mi_ntt64_ggsw> g(new (std::nothrow) mi_ntt64_ggsw);
  if (!g) return fail(MI_ERR_OOM, "host allocation failed");
  g->plan = plan;
  g->n_ggsw = n_ggsw;
  g->k = k;
  g->base_log = base_log;
  g->level = level;
  g->variant = variant;
  g->ggsw = ggsw_list;
  if (twisted_ext_applies(plan, variant, k, base_log, level) && mi::ext_tw_reads_w1p()) {
    const size_t polys = n_ggsw * 4;  // k = 1, level 1: (k + 1)^2 polynomials per GGSW
    DeviceGuard dg(plan->device);
    if (hipMalloc(&g->owned, polys * plan->n * sizeof(u64)) != hipSuccess)
      return fail(MI_ERR_OOM, "GGSW copy allocation failed");
    hipError_t e = mi::launch_prepare_tw_key(g->owned, ggsw_list, polys, 0, 0, (hipStream_t)stream, true);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) {
      (void)hipFree(g->owned);
      return hip_fail(e, "GGSW preparation");
    }
    g->ggsw = g->owned;
  }
  *out = g.release();
  return MI_OK;
}

int mi_ntt64_ggsw_destroy(mi_ntt64_ggsw* g) {
  if (!g) return MI_OK;
  if (g->owned) {
    DeviceGuard dg(g->plan->device);
    (void)hipFree(g->owned);
  }
  delete g;
  return MI_OK;
}

int mi_ntt64_ggsw_info(const mi_ntt64_ggsw* g, size_t* n_ggsw, int* k, int* base_log, int* level, int* variant) {
  if (!g) return fail(MI_ERR_INVALID_ARG, "ggsw is NULL");
  if (n_ggsw) *n_ggsw = g->n_ggsw;
  if (k) *k = g->k;
  if (base_log) *base_log = g->base_log;
  if (level) *level = g->level;
  if (variant) *variant = g->variant;
  return MI_OK;
}

int mi_ext_product_ntt64_prepared_batch(const mi_ntt64_ggsw* g, uint64_t* out_glwe, const uint64_t* in_glwe,
                                        const uint32_t* ggsw_index, size_t batch, void* stream) {
  if (!g) return fail(MI_ERR_INVALID_ARG, "ggsw is NULL");
  return ext_common(g->plan, false, out_glwe, const_cast<uint64_t*>(in_glwe), g->ggsw, ggsw_index,
                    ggsw_index ? g->n_ggsw : 1, g->k, g->base_log, g->level, batch, g->variant, stream, g->owned != nullptr);
}

int mi_cmux_ntt64_prepared_batch(const mi_ntt64_ggsw* g, uint64_t* ct0, uint64_t* ct1, const uint32_t* ggsw_index,
                                 size_t batch, void* stream) {
  if (!g) return fail(MI_ERR_INVALID_ARG, "ggsw is NULL");
  return ext_common(g->plan, true, ct0, ct1, g->ggsw, ggsw_index, ggsw_index ? g->n_ggsw : 1, g->k, g->base_log,
                    g->level, batch, g->variant, stream, g->owned != nullptr);
}

int mi_ext_product_ntt64_batch(const mi_ntt64_plan* plan, uint64_t* out_glwe, const uint64_t* in_glwe,
                               const uint64_t* ggsw_ntt, int k, int base_log, int level, size_t batch, int variant,
                               void* stream) {
  return ext_common(plan, false, out_glwe, const_cast<uint64_t*>(in_glwe), ggsw_ntt, nullptr, 1, k, base_log, level,
                    batch, variant, stream);
}

int mi_cmux_ntt64_batch(const mi_ntt64_plan* plan, uint64_t* ct0, uint64_t* ct1, const uint64_t* ggsw_ntt, int k,
                        int base_log, int level, size_t batch, int variant, void* stream) {
  return ext_common(plan, true, ct0, ct1, ggsw_ntt, nullptr, 1, k, base_log, level, batch, variant, stream);
}

int mi_ext_product_ntt64_batch_indexed(const mi_ntt64_plan* plan, uint64_t* out_glwe, const uint64_t* in_glwe,
                                       const uint64_t* ggsw_list, const uint32_t* ggsw_index, size_t n_ggsw, int k,
                                       int base_log, int level, size_t batch, int variant, void* stream) {
  if (!ggsw_index && batch) return fail(MI_ERR_INVALID_ARG, "ggsw_index is NULL");
  return ext_common(plan, false, out_glwe, const_cast<uint64_t*>(in_glwe), ggsw_list, ggsw_index, n_ggsw, k, base_log,
                    level, batch, variant, stream);
}

int mi_cmux_ntt64_batch_indexed(const mi_ntt64_plan* plan, uint64_t* ct0, uint64_t* ct1, const uint64_t* ggsw_list,
                                const uint32_t* ggsw_index, size_t n_ggsw, int k, int base_log, int level,
                                size_t batch, int variant, void* stream) {
  if (!ggsw_index && batch) return fail(MI_ERR_INVALID_ARG, "ggsw_index is NULL");
  return ext_common(plan, true, ct0, ct1, ggsw_list, ggsw_index, n_ggsw, k, base_log, level, batch, variant, stream);
}

}  // extern "C"

bool mi::capi::pbs_key_needs_copy(const mi_ntt64_plan* plan, int variant, int k, int base_log, int level) {
  return variant == MI_NTT64_BNF || twisted_ext_applies(plan, variant, k, base_log, level);
}

int mi::capi::prepare_pbs_key(const mi_ntt64_plan* plan, int variant, int k, int base_log, int level, u64* dst,
                              const u64* src, size_t count, hipStream_t stream) {
  const bool bnf = variant == MI_NTT64_BNF;
  hipError_t e = hipSuccess;
  if (twisted_ext_applies(plan, variant, k, base_log, level))
    e = mi::launch_prepare_tw_key(dst, src, count / plan->n, plan->n_inv, bnf ? 1 : 0, stream);
  else if (bnf)
    e = mi::launch_scale(dst, src, count, plan->n_inv, stream);
  else if (dst != src)
    e = hipMemcpyAsync(dst, src, count * sizeof(u64), hipMemcpyDeviceToDevice, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "bootstrap key preparation");
}

extern "C" {

int mi_pbs_ntt64_key_create(const mi_ntt64_plan* plan, const uint64_t* bsk_ntt, size_t n_lwe, int k, int base_log,
                            int level, int variant, void* stream, mi_pbs_ntt64_key** out_key) {
  if (!out_key) return fail(MI_ERR_INVALID_ARG, "out_key is NULL");
  *out_key = nullptr;
  int st = check_pbs_shape(plan, k, base_log, level, variant);
  if (st != MI_OK) return st;
  if (n_lwe == 0 || n_lwe > 0xFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "n_lwe out of range");
  if (!bsk_ntt) return fail(MI_ERR_INVALID_ARG, "bsk is NULL");
  mi_pbs_ntt64_key* key = new (std::nothrow) mi_pbs_ntt64_key;
  if (!key) return fail(MI_ERR_OOM, "host allocation failed");
  key->plan = plan;
  key->n_lwe = n_lwe;
  key->k = k;
  key->base_log = base_log;
  key->level = level;
  key->variant = variant;
  key->bsk = bsk_ntt;
  if (pbs_key_needs_copy(plan, variant, k, base_log, level)) {
    const size_t count = n_lwe * (size_t)(k + 1) * (k + 1) * level * plan->n;
    DeviceGuard g(plan->device);
    if (hipMalloc(&key->owned, count * sizeof(u64)) != hipSuccess) {
      delete key;
      return fail(MI_ERR_OOM, "bootstrap key copy allocation failed");
    }
    // ordered after the work that produced bsk_ntt on `stream` (the caller's stream)
    st = prepare_pbs_key(plan, variant, k, base_log, level, key->owned, bsk_ntt, count, (hipStream_t)stream);
    if (st != MI_OK) {
      (void)hipFree(key->owned);
      delete key;
      return st;
    }
    key->bsk = key->owned;
  }
  *out_key = key;
  return MI_OK;
}

int mi_pbs_ntt64_key_destroy(mi_pbs_ntt64_key* key) {
  if (!key) return MI_OK;
  if (key->owned) {
    DeviceGuard g(key->plan->device);
    (void)hipFree(key->owned);
  }
  delete key;
  return MI_OK;
}

}  // extern "C"

// every NTT bootstrap entry point: the accumulator's start and the output form come in `io` (ntt64_launch.hpp PbsIo);
// lwe_out is ignored when io.glwe_out is set
static int pbs_common(const mi_pbs_ntt64_key* key, uint64_t* lwe_out, const uint64_t* lwe_in, mi::PbsIo io,
                      size_t batch, int ms_mode, void* stream) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (ms_mode != MI_MS_STANDARD && ms_mode != MI_MS_CENTERED && ms_mode != MI_MS_PRE_SWITCHED)
    return fail(MI_ERR_INVALID_ARG, "unknown ms_mode");
  if (ms_mode == MI_MS_CENTERED && key->variant != MI_NTT64_BNF)
    return fail(MI_ERR_INVALID_ARG, "centered modulus switch applies to native-modulus (BNF) inputs");
  if (batch == 0) return MI_OK;
  if ((!lwe_out && !io.glwe_out) || !lwe_in || !io.lut) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  const mi_ntt64_plan* plan = key->plan;
  const hipStream_t s = (hipStream_t)stream;
  DeviceGuard g(plan->device);
  if (key->variant == MI_NTT64_SOLINAS && twisted_ext_applies(plan, key->variant, key->k, key->base_log, key->level)) {
    // Solinas on the twisted engine: the body reads switched values (the caller's, or switched here
    // into stream-ordered scratch by ms_non_native)
    const size_t count = batch * (key->n_lwe + 1);
    u64* sw = nullptr;
    if (ms_mode != MI_MS_PRE_SWITCHED) {
      if (mi::scratch_alloc((void**)&sw, count * sizeof(u64), s) != hipSuccess)
        return fail(MI_ERR_OOM, "scratch allocation failed");
      hipError_t e = mi::launch_ms_non_native(sw, lwe_in, count, s);
      if (e != hipSuccess) {
        (void)mi::scratch_free(sw, s);
        return hip_fail(e, "modulus switch launch");
      }
    }
    hipError_t e = mi::launch_pbs_tw_sol(lwe_out, sw ? sw : lwe_in, io, key->bsk, key->n_lwe, batch, key->base_log,
                                         plan->d_twist_f, s);
    if (sw) (void)mi::scratch_free(sw, s);
    return e == hipSuccess ? MI_OK : hip_fail(e, "pbs launch");
  }
  u64* lifted = nullptr;  // PRE_SWITCHED: stream-ordered copy lifted back to the standard switch
  if (ms_mode == MI_MS_PRE_SWITCHED) {
    const size_t count = batch * (key->n_lwe + 1);
    if (mi::scratch_alloc((void**)&lifted, count * sizeof(u64), s) != hipSuccess)
      return fail(MI_ERR_OOM, "scratch allocation failed");
    hipError_t e = mi::launch_lift_switched(lifted, lwe_in, count, key->variant == MI_NTT64_BNF, plan->logn, s);
    if (e != hipSuccess) {
      (void)mi::scratch_free(lifted, s);
      return hip_fail(e, "lift launch");
    }
    lwe_in = lifted;
    ms_mode = MI_MS_STANDARD;
  }
  hipError_t e;
  if (twisted_ext_applies(plan, key->variant, key->k, key->base_log, key->level))
    e = mi::launch_pbs_tw(lwe_out, lwe_in, io, key->bsk, key->n_lwe, batch, key->base_log, plan->d_twist_f,
                          ms_mode == MI_MS_CENTERED, s);
  else if (plan->logn >= LARGE_PATH_MIN_LOGN)
    e = mi::launch_pbs_large(plan->logn, key->k, key->variant == MI_NTT64_BNF, key->level, lwe_out, lwe_in, io,
                             key->bsk, key->n_lwe, batch, key->base_log, plan->d_twid, plan->d_inv_twid,
                             ms_mode == MI_MS_CENTERED, s, split_of(plan));
  else
    e = mi::launch_pbs(plan->logn, key->k, key->variant == MI_NTT64_BNF, key->level, lwe_out, lwe_in, io, key->bsk, key->n_lwe, batch,
                       key->base_log, plan->d_twid, plan->d_inv_twid, ms_mode == MI_MS_CENTERED, s);
  if (lifted) (void)mi::scratch_free(lifted, s);
  return e == hipSuccess ? MI_OK : hip_fail(e, "pbs launch");
}

extern "C" {

int mi_pbs_ntt64_batch(const mi_pbs_ntt64_key* key, uint64_t* lwe_out, const uint64_t* lwe_in, const uint64_t* lut,
                       size_t batch, int ms_mode, void* stream) {
  mi::PbsIo io;
  io.lut = lut;
  if (!lwe_out && batch) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  return pbs_common(key, lwe_out, lwe_in, io, batch, ms_mode, stream);
}

int mi_pbs_ntt64_batch_lut_indexed(const mi_pbs_ntt64_key* key, uint64_t* lwe_out, const uint64_t* lwe_in,
                                   const uint64_t* lut_list, const uint32_t* lut_index, size_t n_lut, size_t batch,
                                   int ms_mode, void* stream) {
  if (batch && !lwe_out) return fail(MI_ERR_INVALID_ARG, "lwe_out is NULL");
  if (n_lut == 0 || n_lut > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "n_lut out of range");
  if (!lut_index && n_lut < batch) return fail(MI_ERR_INVALID_ARG, "per-item LUTs: n_lut < batch");
  mi::PbsIo io;
  io.lut = lut_list;
  io.lut_idx = lut_index;
  io.n_lut = (uint32_t)n_lut;
  io.per_item = lut_index ? 0 : 1;  // no index array: item b uses GLWE b
  return pbs_common(key, lwe_out, lwe_in, io, batch, ms_mode, stream);
}

int mi_blind_rotate_ntt64_batch(const mi_pbs_ntt64_key* key, uint64_t* acc_glwe, const uint64_t* lwe_in, size_t batch,
                                int ms_mode, void* stream) {
  if (batch && !acc_glwe) return fail(MI_ERR_INVALID_ARG, "acc_glwe is NULL");
  mi::PbsIo io;
  io.lut = acc_glwe;
  io.per_item = 1;
  io.glwe_out = acc_glwe;
  return pbs_common(key, nullptr, lwe_in, io, batch, ms_mode, stream);
}

int mi_sample_extract_batch(uint64_t* lwe_out, const uint64_t* glwe, size_t polynomial_size, int k, size_t batch,
                            size_t nth_first, size_t nth_stride, size_t nth_count, uint64_t modulus, int device,
                            void* stream) {
  if (polynomial_size < 2 || (polynomial_size & (polynomial_size - 1)) != 0 || polynomial_size > ((size_t)1 << 31))
    return fail(MI_ERR_INVALID_ARG, "polynomial size must be a power of two in [2, 2^31]");
  if (k < 1) return fail(MI_ERR_INVALID_ARG, "GLWE dimension must be >= 1");
  if (batch == 0 || nth_count == 0) return MI_OK;
  if (!lwe_out || !glwe) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  // glwe_sample_extraction.rs:89-160 takes MonomialDegree < N (opposite_count = N - nth - 1 would underflow)
  if (nth_first >= polynomial_size || (nth_count > 1 && nth_stride > (polynomial_size - 1 - nth_first) / (nth_count - 1)))
    return fail(MI_ERR_INVALID_ARG, "a monomial degree is >= the polynomial size");
  DeviceGuard g(device);
  if (!g.ok) return fail(MI_ERR_HIP, "hipSetDevice failed");
  const hipError_t e = mi::launch_sample_extract(lwe_out, glwe, __builtin_ctzll(polynomial_size), k, batch, nth_first,
                                                 nth_stride, nth_count, modulus, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "sample extraction launch");
}

int mi_scratch_trim(int device, size_t* released) {
  const size_t b = mi::scratch_trim(device);
  if (released) *released = b;
  return MI_OK;
}

int mi_scratch_bytes(int device, size_t* bytes) {
  if (!bytes) return fail(MI_ERR_INVALID_ARG, "bytes is NULL");
  *bytes = mi::scratch_bytes(device);
  return MI_OK;
}

// ---- prime32 plans (prime32.rs:632-1025) -------------------------------------------------------

struct mi_ntt32_plan {
  mi_ntt64_plan* p64 = nullptr;  // same twiddle convention (prime32.rs:223-246 == prime64.rs:184-203)
};

int mi_ntt32_plan_create(size_t n, uint32_t p, int device, mi_ntt32_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  // prime32.rs:662-671: N < 32, N not a power of two, p not prime, no root -> None
  if (n < 32 || (n & (n - 1)) != 0) return fail(MI_ERR_INVALID_ARG, "polynomial size must be a power of two >= 32");
  mi_ntt64_plan* p64 = nullptr;
  int st = mi_ntt64_plan_create(n, p, device, &p64);
  if (st != MI_OK) return st;
  mi_ntt32_plan* plan = new (std::nothrow) mi_ntt32_plan;
  if (!plan) {
    mi_ntt64_plan_destroy(p64);
    return fail(MI_ERR_OOM, "host allocation failed");
  }
  plan->p64 = p64;
  *out_plan = plan;
  return MI_OK;
}

int mi_ntt32_plan_destroy(mi_ntt32_plan* plan) {
  if (!plan) return MI_OK;
  mi_ntt64_plan_destroy(plan->p64);
  delete plan;
  return MI_OK;
}

int mi_ntt32_plan_info(const mi_ntt32_plan* plan, size_t* n, uint32_t* p, int* device) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (n) *n = plan->p64->n;
  if (p) *p = (uint32_t)plan->p64->p;
  if (device) *device = plan->p64->device;
  return MI_OK;
}

static int run_ntt32(bool fwd, const mi_ntt32_plan* plan, uint32_t* buf, size_t batch, size_t stride, void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  const mi_ntt64_plan* q = plan->p64;
  int st = check_batch(q, buf, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  DeviceGuard g(q->device);
  hipError_t e = mi::launch_ntt_shoup32(fwd, q->logn, (uint32_t)q->p, nullptr, buf, batch, stride,
                                        fwd ? q->d_tw32 : q->d_itw32, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, fwd ? "fwd launch" : "inv launch");
}

int mi_ntt32_fwd_batch(const mi_ntt32_plan* plan, uint32_t* buf, size_t batch, size_t stride, void* stream) {
  return run_ntt32(true, plan, buf, batch, stride, stream);
}

int mi_ntt32_inv_batch(const mi_ntt32_plan* plan, uint32_t* buf, size_t batch, size_t stride, void* stream) {
  return run_ntt32(false, plan, buf, batch, stride, stream);
}

static int run_pw32(int op, const mi_ntt32_plan* plan, uint32_t* out, const uint32_t* a, const uint32_t* b,
                    size_t batch, size_t stride, void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  const mi_ntt64_plan* q = plan->p64;
  int st = check_batch(q, out, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  if (op >= 1 && !b) return fail(MI_ERR_INVALID_ARG, "rhs is NULL");
  if (op == 2 && !a) return fail(MI_ERR_INVALID_ARG, "lhs is NULL");
  const u64 c = op == 0 ? q->c_normalize : (op == 1 ? q->c_man : q->c_macc);
  DeviceGuard g(q->device);
  hipError_t e = mi::launch_pointwise_u32(op, q->mp, out, a, b, q->n, batch, stride, c, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "pointwise launch");
}

int mi_ntt32_normalize_batch(const mi_ntt32_plan* plan, uint32_t* buf, size_t batch, size_t stride, void* stream) {
  return run_pw32(0, plan, buf, nullptr, nullptr, batch, stride, stream);
}

int mi_ntt32_mul_assign_normalize_batch(const mi_ntt32_plan* plan, uint32_t* lhs, const uint32_t* rhs, size_t batch,
                                        size_t stride, void* stream) {
  return run_pw32(1, plan, lhs, nullptr, rhs, batch, stride, stream);
}

int mi_ntt32_mul_accumulate_batch(const mi_ntt32_plan* plan, uint32_t* acc, const uint32_t* lhs, const uint32_t* rhs,
                                  size_t batch, size_t stride, void* stream) {
  return run_pw32(2, plan, acc, lhs, rhs, batch, stride, stream);
}

// ---- exact native-modulus products over a CRT of primes (native{32,64,128}.rs, native_binary*.rs) --

struct mi_native_plan {
  int kind = 0, width = 64, binary = 0;
  size_t n = 0;
  int device = 0;
  int k = 0;
  mi_ntt64_plan* primes[mi::MI_CRT_MAX] = {};
  mi::CrtConst crt;
};

namespace {
// tfhe-ntt/src/lib.rs primes32 (P0..P9) and primes52 (P0..P5)
constexpr uint32_t PRIMES32[10] = {0x3F5A0001u, 0x3F5D0001u, 0x3F760001u, 0x3F820001u, 0x3FAC0001u,
                                   0x3FAF0001u, 0x3FB10001u, 0x3FBB0001u, 0x3FDE0001u, 0x3FFC0001u};
constexpr u64 PRIMES52[6] = {0x3FFFFFE770001ull, 0x3FFFFFEB90001ull, 0x3FFFFFEC80001ull,
                             0x3FFFFFF8B0001ull, 0x3FFFFFFB80001ull, 0x3FFFFFFC70001ull};

struct NativeKind {
  int width, binary, prime_bits, k;
};
// index = mi_native_kind
constexpr NativeKind NATIVE_KINDS[] = {
    {32, 0, 32, 3},   // native32::Plan32   (native32.rs:337-343)
    {32, 0, 52, 2},   // native32::Plan52   (native32.rs:440-444)
    {64, 0, 32, 5},   // native64::Plan32   (native64.rs:932-941)
    {64, 0, 52, 3},   // native64::Plan52   (native64.rs:1077-1086)
    {128, 0, 32, 10}, // native128::Plan32  (native128.rs:123-137)
    {32, 1, 32, 2},   // native_binary32::Plan32 (native_binary32.rs:189-192)
    {32, 1, 52, 1},   // native_binary32::Plan52 (native_binary32.rs:270-273)
    {64, 1, 32, 3},   // native_binary64::Plan32 (native_binary64.rs:344-351)
    {64, 1, 52, 2},   // native_binary64::Plan52 (native_binary64.rs:452-456)
    {128, 1, 32, 5},  // native_binary128::Plan32 (native_binary128.rs:68-77)
};
}  // namespace

int mi_native_plan_create(int kind, size_t n, int device, mi_native_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  if (kind < 0 || kind >= (int)(sizeof(NATIVE_KINDS) / sizeof(NATIVE_KINDS[0])))
    return fail(MI_ERR_INVALID_ARG, "unknown native plan kind");
  const NativeKind nk = NATIVE_KINDS[kind];
  // the component plans are prime32 plans (N >= 32) or prime64 plans (N >= 16)
  if (nk.prime_bits == 32 && n < 32) return fail(MI_ERR_INVALID_ARG, "polynomial size must be >= 32");
  mi_native_plan* plan = new (std::nothrow) mi_native_plan;
  if (!plan) return fail(MI_ERR_OOM, "host allocation failed");
  plan->kind = kind;
  plan->width = nk.width;
  plan->binary = nk.binary;
  plan->n = n;
  plan->device = device;
  plan->k = nk.k;
  mi::CrtConst& c = plan->crt;
  c.k = nk.k;
  c.prime_bits = nk.prime_bits;
  u128 prefix = 1;  // prod_{l<k} p_l mod 2^128
  for (int i = 0; i < nk.k; ++i) {
    const u64 p = nk.prime_bits == 32 ? (u64)PRIMES32[i] : PRIMES52[i];
    int st = mi_ntt64_plan_create(n, p, device, &plan->primes[i]);
    if (st != MI_OK) {
      mi_native_plan_destroy(plan);
      return st;
    }
    c.p[i] = p;
    c.prefix_lo[i] = (u64)prefix;
    c.prefix_hi[i] = (u64)(prefix >> 64);
    u64 pm = 1;  // prod_{l<i} p_l mod p_i
    for (int l = 0; l < i; ++l) pm = mi::host::mul_mod(pm, c.p[l] % p, p);
    c.inv_prefix[i] = i == 0 ? 1 : mi::host::exp_mod(pm, p - 2, p);
    prefix *= p;
  }
  c.m_lo = (u64)prefix;
  c.m_hi = (u64)(prefix >> 64);
  for (int k = 0; k < nk.k; ++k) {  // the device's Montgomery constants (native_crt.hip)
    const u64 p = c.p[k];
    u64 inv = p;  // Newton: p * inv == 1 mod 2^64
    for (int it = 0; it < 6; ++it) inv *= 2 - p * inv;
    c.pinv[k] = (u64)0 - inv;
    c.r1[k] = (u64)(((u128)1 << 64) % p);
    c.r2[k] = mi::host::mul_mod(c.r1[k], c.r1[k], p);
    c.inv_prefix_m[k] = mont_form(c.inv_prefix[k], p);
    for (int j = 0; j < nk.k; ++j) c.pjk_m[j][k] = mont_form(c.p[j] % p, p);
  }
  *out_plan = plan;
  return MI_OK;
}

int mi_native_plan_destroy(mi_native_plan* plan) {
  if (!plan) return MI_OK;
  for (int i = 0; i < mi::MI_CRT_MAX; ++i)
    if (plan->primes[i]) mi_ntt64_plan_destroy(plan->primes[i]);
  delete plan;
  return MI_OK;
}

int mi_native_plan_info(const mi_native_plan* plan, size_t* n, int* width_bits, int* num_primes) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (n) *n = plan->n;
  if (width_bits) *width_bits = plan->width;
  if (num_primes) *num_primes = plan->k;
  return MI_OK;
}

int mi_native_polymul_batch(const mi_native_plan* plan, void* prod, const void* lhs, const void* rhs, size_t batch,
                            void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (batch == 0) return MI_OK;
  if (!prod || !lhs || !rhs) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  const hipStream_t s = (hipStream_t)stream;
  const size_t count = batch * plan->n;
  DeviceGuard g(plan->device);
  u64* scratch = nullptr;  // [lhs residues: k planes | rhs residues: k planes], stream-ordered
  hipError_t e = mi::scratch_alloc((void**)&scratch, 2 * (size_t)plan->k * count * sizeof(u64), s);
  if (e != hipSuccess) return fail(MI_ERR_OOM, "scratch allocation failed");
  u64* a = scratch;
  u64* b = scratch + (size_t)plan->k * count;
  e = mi::launch_crt_residues(a, lhs, count, plan->width, 0, plan->crt, s);
  if (e == hipSuccess) e = mi::launch_crt_residues(b, rhs, count, plan->width, plan->binary, plan->crt, s);
  int st = e == hipSuccess ? MI_OK : hip_fail(e, "residue launch");
  for (int i = 0; i < plan->k && st == MI_OK; ++i) {
    const mi_ntt64_plan* q = plan->primes[i];
    u64* ai = a + (size_t)i * count;
    u64* bi = b + (size_t)i * count;
    st = run_ntt(true, q, ai, batch, plan->n, stream);
    if (st == MI_OK) st = run_ntt(true, q, bi, batch, plan->n, stream);
    if (st == MI_OK) st = run_pw(1, q, ai, nullptr, bi, batch, plan->n, stream);
    if (st == MI_OK) st = run_ntt(false, q, ai, batch, plan->n, stream);
  }
  if (st == MI_OK) {
    e = mi::launch_crt_reconstruct(prod, a, count, plan->width, plan->crt, s);
    if (e != hipSuccess) st = hip_fail(e, "reconstruct launch");
  }
  (void)mi::scratch_free(scratch, s);
  return st;
}

// ---- LWE keyswitch (tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs:137-227) -----------------------

struct mi_lwe_ksk {
  int device = 0;
  size_t in_dim = 0, out_dim = 0;
  int base_log = 0, level = 0;
  void* frag = nullptr;  // byte-plane MFMA fragments (keyswitch.hip)
};

int mi_lwe_ksk_create(const uint64_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level, int device,
                      void* stream, mi_lwe_ksk** out_key) {
  if (!out_key) return fail(MI_ERR_INVALID_ARG, "out_key is NULL");
  *out_key = nullptr;
  if (!ksk) return fail(MI_ERR_INVALID_ARG, "ksk is NULL");
  if (in_dim == 0 || out_dim == 0 || in_dim > 0xFFFFFFull || out_dim > 0xFFFFFFull)
    return fail(MI_ERR_INVALID_ARG, "lwe dimension out of range");
  // SignedDecomposer::new (decomposer.rs): base_log * level < 64, both >= 1
  if (base_log < 1 || level < 1 || base_log * level >= 64)
    return fail(MI_ERR_INVALID_ARG, "decomposition base_log * level must be in [1, 63]");
  // exact int32 accumulation on the int8 matrix cores: GEMM depth in_dim * level * bytes-per-digit < 2^17
  if ((double)in_dim * level * mi::ks_digit_bytes_per_term(base_log) >= 131072.0)
    return fail(MI_ERR_UNSUPPORTED, "in_dim * level * ceil((base_log + 1) / 8) must stay below 2^17");
  mi_lwe_ksk* key = new (std::nothrow) mi_lwe_ksk;
  if (!key) return fail(MI_ERR_OOM, "host allocation failed");
  key->device = device;
  key->in_dim = in_dim;
  key->out_dim = out_dim;
  key->base_log = base_log;
  key->level = level;
  DeviceGuard g(device);
  if (!g.ok) {
    delete key;
    return fail(MI_ERR_INVALID_ARG, "bad device");
  }
  if (hipMalloc(&key->frag, mi::ks_key_bytes(in_dim, out_dim, base_log, level)) != hipSuccess) {
    delete key;
    return fail(MI_ERR_OOM, "keyswitch key allocation failed");
  }
  // ordered after the work that produced `ksk` on the caller's stream
  hipError_t e = mi::launch_ksk_prepare(key->frag, ksk, in_dim, out_dim, base_log, level, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) {
    (void)hipFree(key->frag);
    delete key;
    return hip_fail(e, "keyswitch key preparation");
  }
  *out_key = key;
  return MI_OK;
}

int mi_lwe_ksk_destroy(mi_lwe_ksk* key) {
  if (!key) return MI_OK;
  {
    DeviceGuard g(key->device);
    if (key->frag) (void)hipFree(key->frag);
  }
  delete key;
  return MI_OK;
}

int mi_lwe_ksk_info(const mi_lwe_ksk* key, size_t* in_dim, size_t* out_dim, int* base_log, int* level) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (in_dim) *in_dim = key->in_dim;
  if (out_dim) *out_dim = key->out_dim;
  if (base_log) *base_log = key->base_log;
  if (level) *level = key->level;
  return MI_OK;
}

int mi_lwe_keyswitch_batch(const mi_lwe_ksk* key, uint64_t* lwe_out, const uint64_t* lwe_in, size_t batch,
                           void* stream) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (batch == 0) return MI_OK;
  if (!lwe_out || !lwe_in) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x3FFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  const hipStream_t s = (hipStream_t)stream;
  DeviceGuard g(key->device);
  void* digits = nullptr;  // int8 digit fragments, stream-ordered scratch
  if (mi::scratch_alloc((void**)&digits, mi::ks_digit_bytes(key->in_dim, key->base_log, key->level, batch), s) != hipSuccess)
    return fail(MI_ERR_OOM, "scratch allocation failed");
  hipError_t e = mi::launch_keyswitch(lwe_out, lwe_in, key->frag, digits, batch, key->in_dim, key->out_dim,
                                      key->base_log, key->level, s);
  (void)mi::scratch_free(digits, s);
  return e == hipSuccess ? MI_OK : hip_fail(e, "keyswitch launch");
}

// ---- KS32: keyswitch_lwe_ciphertext_with_scalar_change (lwe_keyswitch.rs:331-447) ------------------------------
// The keyswitch of the HPU KS32 parameter sets (shortint/parameters/v1_5/hpu.rs:57-76: 2048 -> 879, base 2^2, 8
// levels, post_keyswitch_ciphertext_modulus 2^21): u64 input LWEs of the native modulus, u32 key and output words
// with the power-of-two output modulus 2^out_modulus_log encoded in the MSBs, as the reference stores it.

struct mi_lwe_ksk32 {
  int device = 0;
  size_t in_dim = 0, out_dim = 0;
  int base_log = 0, level = 0, out_modulus_log = 32;
  void* frag = nullptr;  // byte-plane MFMA fragments of the zero-extended u32 key words (keyswitch.hip)
};

int mi_lwe_ksk32_create(const uint32_t* ksk, size_t in_dim, size_t out_dim, int base_log, int level,
                        int out_modulus_log, int device, void* stream, mi_lwe_ksk32** out_key) {
  if (!out_key) return fail(MI_ERR_INVALID_ARG, "out_key is NULL");
  *out_key = nullptr;
  if (!ksk) return fail(MI_ERR_INVALID_ARG, "ksk is NULL");
  if (in_dim == 0 || out_dim == 0 || in_dim > 0xFFFFFFull || out_dim > 0xFFFFFFull)
    return fail(MI_ERR_INVALID_ARG, "lwe dimension out of range");
  if (out_modulus_log < 1 || out_modulus_log > 32)
    return fail(MI_ERR_INVALID_ARG, "output modulus must be 2^w with 1 <= w <= 32");
  // lwe_keyswitch.rs:378-384: base_log * level <= OutputScalar::BITS (and SignedDecomposer::new's >= 1 each)
  if (base_log < 1 || level < 1 || base_log * level > 32)
    return fail(MI_ERR_INVALID_ARG, "decomposition base_log * level must be in [1, 32]");
  if ((double)in_dim * level * mi::ks_digit_bytes_per_term(base_log) >= 131072.0)
    return fail(MI_ERR_UNSUPPORTED, "in_dim * level * ceil((base_log + 1) / 8) must stay below 2^17");
  mi_lwe_ksk32* key = new (std::nothrow) mi_lwe_ksk32;
  if (!key) return fail(MI_ERR_OOM, "host allocation failed");
  key->device = device;
  key->in_dim = in_dim;
  key->out_dim = out_dim;
  key->base_log = base_log;
  key->level = level;
  key->out_modulus_log = out_modulus_log;
  DeviceGuard g(device);
  if (!g.ok) {
    delete key;
    return fail(MI_ERR_INVALID_ARG, "bad device");
  }
  if (hipMalloc(&key->frag, mi::ks32_key_bytes(in_dim, out_dim, base_log, level)) != hipSuccess) {
    delete key;
    return fail(MI_ERR_OOM, "keyswitch key allocation failed");
  }
  hipError_t e = mi::launch_ksk32_prepare(key->frag, ksk, in_dim, out_dim, base_log, level, (hipStream_t)stream);
  if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) {
    (void)hipFree(key->frag);
    delete key;
    return hip_fail(e, "keyswitch key preparation");
  }
  *out_key = key;
  return MI_OK;
}

int mi_lwe_ksk32_destroy(mi_lwe_ksk32* key) {
  if (!key) return MI_OK;
  {
    DeviceGuard g(key->device);
    if (key->frag) (void)hipFree(key->frag);
  }
  delete key;
  return MI_OK;
}

int mi_lwe_ksk32_info(const mi_lwe_ksk32* key, size_t* in_dim, size_t* out_dim, int* base_log, int* level,
                      int* out_modulus_log) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (in_dim) *in_dim = key->in_dim;
  if (out_dim) *out_dim = key->out_dim;
  if (base_log) *base_log = key->base_log;
  if (level) *level = key->level;
  if (out_modulus_log) *out_modulus_log = key->out_modulus_log;
  return MI_OK;
}

int mi_lwe_keyswitch32_batch(const mi_lwe_ksk32* key, uint32_t* lwe_out, const uint64_t* lwe_in, size_t batch,
                             void* stream) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (batch == 0) return MI_OK;
  if (!lwe_out || !lwe_in) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x3FFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  const hipStream_t s = (hipStream_t)stream;
  DeviceGuard g(key->device);
  void* digits = nullptr;
  if (mi::scratch_alloc((void**)&digits, mi::ks_digit_bytes(key->in_dim, key->base_log, key->level, batch), s) != hipSuccess)
    return fail(MI_ERR_OOM, "scratch allocation failed");
  hipError_t e = mi::launch_keyswitch32(lwe_out, lwe_in, key->frag, digits, batch, key->in_dim, key->out_dim,
                                        key->base_log, key->level, key->out_modulus_log, s);
  (void)mi::scratch_free(digits, s);
  return e == hipSuccess ? MI_OK : hip_fail(e, "keyswitch launch");
}

// shared checks of the two LWE modulus switches: the standard switch is defined for 1 <= log_modulus <= BITS (identity at
// BITS, fft_impl/common.rs:10-23); the centered one computes 1 << (BITS - log_modulus - 1) (modulus_switch.rs:95), so
// it needs log_modulus < BITS (the reference's shift underflows there)
static int check_lwe_ms(const void* switched, const void* lwe_in, size_t lwe_dim, size_t batch, int log_modulus,
                        int ms_mode, int bits) {
  if (!switched || !lwe_in) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (lwe_dim == 0 || lwe_dim > 0xFFFFFFull || batch > 0xFFFFFFFFull)
    return fail(MI_ERR_INVALID_ARG, "lwe dimension or batch out of range");
  if (ms_mode != MI_MS_STANDARD && ms_mode != MI_MS_CENTERED)
    return fail(MI_ERR_INVALID_ARG, "ms_mode must be MI_MS_STANDARD or MI_MS_CENTERED");
  const int top = ms_mode == MI_MS_CENTERED ? bits - 1 : bits;
  if (log_modulus < 1 || log_modulus > top)
    return fail(MI_ERR_INVALID_ARG, "log_modulus must be in [1, " + std::to_string(top) + "] for this ms_mode");
  return MI_OK;
}

int mi_lwe_modulus_switch32_batch(uint64_t* switched, const uint32_t* lwe_in, size_t lwe_dim, size_t batch,
                                  int log_modulus, int ms_mode, int device, void* stream) {
  if (batch == 0) return MI_OK;
  int st = check_lwe_ms(switched, lwe_in, lwe_dim, batch, log_modulus, ms_mode, 32);
  if (st != MI_OK) return st;
  DeviceGuard g(device);
  if (!g.ok) return fail(MI_ERR_INVALID_ARG, "bad device");
  hipError_t e = mi::launch_lwe_ms32(switched, lwe_in, lwe_dim, batch, log_modulus, ms_mode == MI_MS_CENTERED,
                                     (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "modulus switch launch");
}

int mi_lwe_modulus_switch_batch(uint64_t* switched, const uint64_t* lwe_in, size_t lwe_dim, size_t batch,
                                int log_modulus, int ms_mode, int device, void* stream) {
  if (batch == 0) return MI_OK;
  int st = check_lwe_ms(switched, lwe_in, lwe_dim, batch, log_modulus, ms_mode, 64);
  if (st != MI_OK) return st;
  DeviceGuard g(device);
  if (!g.ok) return fail(MI_ERR_INVALID_ARG, "bad device");
  hipError_t e = mi::launch_lwe_ms64(switched, lwe_in, lwe_dim, batch, log_modulus, ms_mode == MI_MS_CENTERED,
                                     (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "modulus switch launch");
}

}  // extern "C"
