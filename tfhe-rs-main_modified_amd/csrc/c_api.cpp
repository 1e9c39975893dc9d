// c_api.cpp — the extern "C" boundary declared in include/tfhe_ntt_amd.h.
//
// Owns plan construction (host twiddles exactly as tfhe-ntt/src/prime64.rs:159-204 + 764-862,
// uploaded once to the plan's device) and argument validation; never aborts, every failure is
// a status code plus a thread-local message.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/tfhe_ntt_amd.h"
#include "host_math.hpp"
#include "ntt64_launch.hpp"

using mi::host::u128;
using mi::host::u64;

struct mi_ntt64_plan {
  size_t n = 0;
  int logn = 0;
  u64 p = 0;
  int device = 0;
  bool goldilocks = false;
  int variant = 0;
  std::vector<u64> twid, inv_twid;  // canonical host tables (reference layout)
  u64 n_inv = 0;
  mi::MontParams mp;
  u64 c_normalize = 0, c_man = 0, c_macc = 0;  // device constants of the pointwise ops
  u64* d_twid = nullptr;
  u64* d_inv_twid = nullptr;
};

namespace {

thread_local std::string g_last_error;

int fail(int status, const std::string& msg) {
  g_last_error = msg;
  return status;
}

int hip_fail(hipError_t e, const char* what) {
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

u64 mont_form(u64 x, u64 p) { return (u64)(((u128)x << 64) % p); }

int env_variant() {
  const char* v = std::getenv("MI_NTT_VARIANT");
  return v ? std::atoi(v) : 0;
}

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

const char* mi_last_error_message(void) { return g_last_error.c_str(); }

int mi_ntt64_plan_create(size_t n, uint64_t p, int device, mi_ntt64_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  // prime64.rs:769-775 — same order of checks as the reference
  if (n < 16 || (n & (n - 1)) != 0) return fail(MI_ERR_INVALID_ARG, "polynomial size must be a power of two >= 16");
  if (!mi::host::is_prime64(p)) return fail(MI_ERR_NOT_PRIME, "modulus is not prime");
  auto root = mi::host::find_primitive_root64(p, 2 * (u64)n);
  if (!root) return fail(MI_ERR_NO_ROOT, "no primitive 2N-th root of unity");
  const int logn = __builtin_ctzll(n);
  if (logn > 14) return fail(MI_ERR_UNSUPPORTED, "this build runs N <= 16384 on device");

  mi_ntt64_plan* plan = new (std::nothrow) mi_ntt64_plan;
  if (!plan) return fail(MI_ERR_OOM, "host allocation failed");
  plan->n = n;
  plan->logn = logn;
  plan->p = p;
  plan->device = device;
  plan->goldilocks = (p == mi::host::SOLINAS_P);
  plan->variant = env_variant();

  // prime64.rs:162-182: Solinas uses the hard-coded friendly root tower, other primes the
  // Tonelli-Shanks root.
  u64 w;
  if (plan->goldilocks) {
    auto r = mi::host::solinas_root(n);
    if (!r) { delete plan; return fail(MI_ERR_NO_ROOT, "no Solinas root for this size"); }
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
  if (!g.ok) { delete plan; return fail(MI_ERR_HIP, "hipSetDevice failed"); }
  if (hipMalloc(&plan->d_twid, n * sizeof(u64)) != hipSuccess ||
      hipMalloc(&plan->d_inv_twid, n * sizeof(u64)) != hipSuccess) {
    if (plan->d_twid) (void)hipFree(plan->d_twid);
    delete plan;
    return fail(MI_ERR_OOM, "twiddle allocation failed");
  }
  hipError_t e = hipMemcpy(plan->d_twid, dev_tw.data(), n * sizeof(u64), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(plan->d_inv_twid, dev_itw.data(), n * sizeof(u64), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(plan->d_twid);
    (void)hipFree(plan->d_inv_twid);
    delete plan;
    return hip_fail(e, "twiddle upload");
  }
  *out_plan = plan;
  return MI_OK;
}

int mi_ntt64_plan_destroy(mi_ntt64_plan* plan) {
  if (!plan) return MI_OK;
  {
    DeviceGuard g(plan->device);
    if (plan->d_twid) (void)hipFree(plan->d_twid);
    if (plan->d_inv_twid) (void)hipFree(plan->d_inv_twid);
  }
  delete plan;
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

static int run_ntt(bool fwd, const mi_ntt64_plan* plan, uint64_t* buf, size_t batch, size_t stride, void* stream) {
  int st = check_batch(plan, buf, batch, stride);
  if (st != MI_OK || batch == 0) return st;
  DeviceGuard g(plan->device);
  hipError_t e = mi::launch_ntt(fwd, plan->logn, plan->variant, plan->goldilocks, plan->mp, buf, batch, stride,
                                fwd ? plan->d_twid : plan->d_inv_twid, (hipStream_t)stream);
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

static int run_host(bool fwd, const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) {
  int st = check_batch(plan, buf, batch, plan ? plan->n : 0);
  if (st != MI_OK || batch == 0) return st;
  DeviceGuard g(plan->device);
  const size_t bytes = batch * plan->n * sizeof(u64);
  u64* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return fail(MI_ERR_OOM, "device buffer allocation failed");
  hipError_t e = hipMemcpy(d, buf, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = mi::launch_ntt(fwd, plan->logn, plan->variant, plan->goldilocks, plan->mp, d, batch, plan->n,
                       fwd ? plan->d_twid : plan->d_inv_twid, nullptr);
  if (e == hipSuccess) e = hipMemcpy(buf, d, bytes, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipFree(d);
  return e == hipSuccess ? MI_OK : hip_fail(e, "host transform");
}

int mi_ntt64_fwd_host(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) { return run_host(true, plan, buf, batch); }

int mi_ntt64_inv_host(const mi_ntt64_plan* plan, uint64_t* buf, size_t batch) { return run_host(false, plan, buf, batch); }

int mi_fill_uniform(uint64_t* buf, size_t count, uint64_t seed, uint64_t p, int device, void* stream) {
  if (count == 0) return MI_OK;
  if (!buf) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  DeviceGuard g(device);
  hipError_t e = mi::launch_fill_uniform(buf, count, seed, p, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fill launch");
}

}  // extern "C"
