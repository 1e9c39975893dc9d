// c_api_fft.cpp — C ABI of the f64-FFT PBS path (mi_fft64_*), the default shortint PBS of tfhe core_crypto
// (SURVEY.md §8f rank 4).  Reference paths relative to /root/reference/tfhe/src/core_crypto:
//   Fft::new + Twisties       fft_impl/fft64/math/fft/mod.rs:58-76, 104-224 (one plan per polynomial size; N = 2048
//                             runs the one-wave engine of fft64_pbs.hip, every other 32 <= N <= 2^18 the generic
//                             engine of fft64_generic.hip)
//   forward/backward_as_torus fft_impl/fft64/math/fft/mod.rs:406-511
//   key conversion            algorithms/lwe_bootstrap_key_conversion.rs:20-150
//   external product / CMUX   algorithms/lwe_programmable_bootstrapping/fft64_pbs.rs:270-330, 510-560
//   PBS                       algorithms/lwe_programmable_bootstrapping/fft64_pbs.rs:924-1060
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <utility>
#include <vector>

#include "c_api_internal.hpp"
#include "fft64_launch.hpp"

using namespace mi::capi;

namespace {

constexpr size_t FFT_N = 2048, FFT_M = 1024;
constexpr size_t GEN_MIN_N = 32, GEN_MAX_N = (size_t)1 << 18;
constexpr size_t OFF_T2 = 2 * 1024, OFF_CM = OFF_T2 + 2 * 64, OFF_CMI = OFF_CM + 2 * 16, TABLE_DOUBLES = OFF_CMI + 2 * 16;

// exp(i pi e / 2048) for an integer exponent (reduced exactly mod 4096 first), in long double
void unit_root(long e, double* re, double* im) {
  e %= 4096;
  if (e < 0) e += 4096;
  const long double a = 3.14159265358979323846264338327950288L * (long double)e / 2048.0L;
  *re = (double)cosl(a);
  *im = (double)sinl(a);
}

std::vector<double> host_tables() {
  std::vector<double> h(TABLE_DOUBLES);
  // t1[k1][j] = w^j omega^(j k1) = exp(i pi (j - 4 j k1) / 2048)
  for (int k1 = 0; k1 < 16; ++k1)
    for (int j = 0; j < 64; ++j) unit_root((long)j - 4L * j * k1, &h[2 * (k1 * 64 + j)], &h[2 * (k1 * 64 + j) + 1]);
  // t2[q1 - 1][jl] = W64^(jl q1) = exp(-2 pi i jl q1 / 64) = exp(i pi (-64 jl q1) / 2048), q1 = 1..3
  for (int q1 = 1; q1 < 4; ++q1)
    for (int jl = 0; jl < 16; ++jl) {
      const size_t o = OFF_T2 + 2 * ((q1 - 1) * 16 + jl);
      unit_root(-64L * jl * q1, &h[o], &h[o + 1]);
    }
  for (int m = 0; m < 16; ++m) {
    unit_root(64L * m, &h[OFF_CM + 2 * m], &h[OFF_CM + 2 * m + 1]);  // exp(i pi m / 32)
    double re, im;
    unit_root(-64L * m, &re, &im);
    h[OFF_CMI + 2 * m] = re / (double)FFT_M;  // exact scaling (a power of two): 1 / M
    h[OFF_CMI + 2 * m + 1] = im / (double)FFT_M;
  }
  return h;
}

// generic plan tables: tw[n] = exp(i pi n / 2M), untw[n] = exp(-i pi n / 2M) / M, wm[t] = exp(-2 pi i t / M), each an
// exact root of unity exp(i pi e / 2M) (e reduced mod 4M) rounded from long double
std::vector<double> generic_tables(size_t m) {
  std::vector<double> h(6 * m);
  const long four_m = 4 * (long)m;
  auto root = [&](long e, double* re, double* im) {
    e %= four_m;
    if (e < 0) e += four_m;
    const long double a = 3.14159265358979323846264338327950288L * (long double)e / (long double)(2 * m);
    *re = (double)cosl(a);
    *im = (double)sinl(a);
  };
  for (size_t n = 0; n < m; ++n) {
    root((long)n, &h[2 * n], &h[2 * n + 1]);
    double re, im;
    root(-(long)n, &re, &im);
    h[2 * (m + n)] = re / (double)m;  // exact scaling (a power of two)
    h[2 * (m + n) + 1] = im / (double)m;
    root(-4L * (long)n, &h[2 * (2 * m + n)], &h[2 * (2 * m + n) + 1]);
  }
  return h;
}

int make_plan(size_t n, int device, mi_fft64_plan** out) {
  if (n != FFT_N && (n < GEN_MIN_N || n > GEN_MAX_N))
    return fail(MI_ERR_UNSUPPORTED, "the f64-FFT engines run 32 <= N <= 2^18");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
    return fail(MI_ERR_INVALID_ARG, "device index out of range");
  DeviceGuard g(device);
  if (!g.ok) return fail(MI_ERR_HIP, "hipSetDevice failed");
  auto* p = new (std::nothrow) mi_fft64_plan;
  if (!p) return fail(MI_ERR_OOM, "host allocation failed");
  p->n = n;
  p->device = device;
  p->generic = n != FFT_N;
  const std::vector<double> h = p->generic ? generic_tables(n / 2) : host_tables();
  hipError_t e = hipMalloc(&p->d_tables, h.size() * sizeof(double));
  if (e != hipSuccess) {
    delete p;
    return fail(MI_ERR_OOM, "device allocation failed");
  }
  e = hipMemcpy(p->d_tables, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(p->d_tables);
    delete p;
    return hip_fail(e, "table upload");
  }
  if (p->generic) {
    const size_t m = n / 2;
    p->gtables = {p->d_tables, p->d_tables + 2 * m, p->d_tables + 4 * m, __builtin_ctzll((unsigned long long)n)};
  } else {
    p->tables = {p->d_tables, p->d_tables + OFF_T2, p->d_tables + OFF_CM, p->d_tables + OFF_CMI};
  }
  *out = p;
  return MI_OK;
}

constexpr int MAX_GENERIC_K = 16;

int check_shape(const mi_fft64_plan* plan, int k, int base_log, int level) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (level < 1 || base_log < 1 || base_log * level > 63)
    return fail(MI_ERR_INVALID_ARG, "decomposition must satisfy level >= 1, base_log >= 1, base_log*level < 64");
  if (plan->generic ? (k < 1 || k > MAX_GENERIC_K) : (k < 1 || k > 2))
    return fail(MI_ERR_UNSUPPORTED, "the f64-FFT external product / PBS run for k in {1, 2} at N = 2048, 1 <= k <= 16 "
                                    "at other N");
  return MI_OK;
}

hipError_t reorder_any(const mi_fft64_plan* plan, double* out, const double* in, size_t polys, bool to_std,
                       hipStream_t s) {
  return plan->generic ? mi::launch_fftg_reorder(out, in, polys, to_std, plan->gtables, s)
                       : mi::launch_fft64_reorder(out, in, polys, to_std, s);
}

}  // namespace

extern "C" {

int mi_fft64_plan_create(size_t n, int device, mi_fft64_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  if (n < 2 || (n & (n - 1))) return fail(MI_ERR_INVALID_ARG, "polynomial size must be a power of two");
  return make_plan(n, device, out_plan);
}

int mi_fft64_plan_cached(size_t n, int device, const mi_fft64_plan** out_plan) {
  if (!out_plan) return fail(MI_ERR_INVALID_ARG, "out_plan is NULL");
  *out_plan = nullptr;
  static std::mutex mu;
  static std::map<std::pair<size_t, int>, mi_fft64_plan*> plans;  // lives until process exit (as PLANS)
  std::lock_guard<std::mutex> lock(mu);
  auto it = plans.find({n, device});
  if (it != plans.end()) {
    *out_plan = it->second;
    return MI_OK;
  }
  mi_fft64_plan* p = nullptr;
  const int st = mi_fft64_plan_create(n, device, &p);
  if (st != MI_OK) return st;
  p->cached = true;
  plans[{n, device}] = p;
  *out_plan = p;
  return MI_OK;
}

int mi_fft64_plan_destroy(mi_fft64_plan* plan) {
  if (!plan || plan->cached) return MI_OK;
  DeviceGuard g(plan->device);
  (void)hipFree(plan->d_tables);
  delete plan;
  return MI_OK;
}

int mi_fft64_plan_info(const mi_fft64_plan* plan, size_t* n, int* device) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (n) *n = plan->n;
  if (device) *device = plan->device;
  return MI_OK;
}

int mi_fft64_fourier_order(const mi_fft64_plan* plan, uint32_t* freq) {
  if (!plan || !freq) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  if (plan->generic) {
    const int logn = plan->gtables.logn;
    for (uint32_t p = 0; p < (uint32_t)(plan->n / 2); ++p) freq[p] = mi::fftg_frequency(logn, p);
    return MI_OK;
  }
  for (int r = 0; r < 16; ++r)
    for (int l = 0; l < 64; ++l) freq[r * 64 + l] = mi::fft64_frequency(r, l);
  return MI_OK;
}

int mi_fft64_forward_torus_batch(const mi_fft64_plan* plan, double* fourier, const uint64_t* standard, size_t batch,
                                 void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (batch == 0) return MI_OK;
  if (!fourier || !standard) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  DeviceGuard g(plan->device);
  const hipError_t e = plan->generic
                           ? mi::launch_fftg_fwd_torus(fourier, standard, batch, plan->gtables, (hipStream_t)stream)
                           : mi::launch_fft64_fwd_torus(fourier, standard, batch, plan->tables, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fft64 forward launch");
}

int mi_fft64_backward_torus_batch(const mi_fft64_plan* plan, uint64_t* standard, const double* fourier, size_t batch,
                                  int add, void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (batch == 0) return MI_OK;
  if (!fourier || !standard) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  DeviceGuard g(plan->device);
  const hipError_t e =
      plan->generic ? mi::launch_fftg_bwd_torus(standard, fourier, batch, add != 0, plan->gtables, (hipStream_t)stream)
                    : mi::launch_fft64_bwd_torus(standard, fourier, batch, add != 0, plan->tables, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fft64 backward launch");
}

static int reorder(const mi_fft64_plan* plan, double* out, const double* in, size_t polys, bool to_std,
                   void* stream) {
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  if (polys == 0) return MI_OK;
  if (!out || !in) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (polys > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "polynomial count too large");
  const size_t doubles = polys * plan->n;  // N / 2 complex per polynomial
  if (out != in && out < in + doubles && in < out + doubles)
    return fail(MI_ERR_INVALID_ARG, "buffers overlap partially (in place must be out == in)");
  DeviceGuard g(plan->device);
  const hipError_t e = reorder_any(plan, out, in, polys, to_std, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fft64 reorder launch");
}

int mi_fft64_to_standard_order(const mi_fft64_plan* plan, double* standard_order, const double* fourier, size_t polys,
                               void* stream) {
  return reorder(plan, standard_order, fourier, polys, true, stream);
}

int mi_fft64_from_standard_order(const mi_fft64_plan* plan, double* fourier, const double* standard_order,
                                 size_t polys, void* stream) {
  return reorder(plan, fourier, standard_order, polys, false, stream);
}

int mi_bsk_to_fourier64(const mi_fft64_plan* plan, const uint64_t* bsk_std, double* bsk_fourier, size_t n_polys,
                        void* stream) {
  return mi_fft64_forward_torus_batch(plan, bsk_fourier, bsk_std, n_polys, stream);
}

int mi_fft64_ext_product_batch(const mi_fft64_plan* plan, uint64_t* out_glwe, const uint64_t* in_glwe,
                               const double* ggsw_fourier, int k, int base_log, int level, size_t batch, void* stream) {
  int st = check_shape(plan, k, base_log, level);
  if (st != MI_OK) return st;
  if (batch == 0) return MI_OK;
  if (!out_glwe || !in_glwe || !ggsw_fourier) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  DeviceGuard g(plan->device);
  const hipError_t e =
      plan->generic ? mi::launch_fftg_ext_product(k, false, out_glwe, const_cast<uint64_t*>(in_glwe), ggsw_fourier,
                                                  batch, base_log, level, plan->gtables, (hipStream_t)stream)
                    : mi::launch_fft64_ext_product(k, false, out_glwe, const_cast<uint64_t*>(in_glwe), ggsw_fourier,
                                                   batch, base_log, level, plan->tables, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fft64 external product launch");
}

int mi_fft64_cmux_batch(const mi_fft64_plan* plan, uint64_t* ct0, uint64_t* ct1, const double* ggsw_fourier, int k,
                        int base_log, int level, size_t batch, void* stream) {
  int st = check_shape(plan, k, base_log, level);
  if (st != MI_OK) return st;
  if (batch == 0) return MI_OK;
  if (!ct0 || !ct1 || !ggsw_fourier) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  DeviceGuard g(plan->device);
  const hipError_t e =
      plan->generic ? mi::launch_fftg_ext_product(k, true, ct0, ct1, ggsw_fourier, batch, base_log, level,
                                                  plan->gtables, (hipStream_t)stream)
                    : mi::launch_fft64_ext_product(k, true, ct0, ct1, ggsw_fourier, batch, base_log, level,
                                                   plan->tables, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fft64 cmux launch");
}

int mi_fft64_pbs_key_create(const mi_fft64_plan* plan, const double* fbsk, size_t n_lwe, int k, int base_log,
                            int level, mi_fft64_pbs_key** out_key) {
  if (!out_key) return fail(MI_ERR_INVALID_ARG, "out_key is NULL");
  *out_key = nullptr;
  int st = check_shape(plan, k, base_log, level);
  if (st != MI_OK) return st;
  if (n_lwe == 0 || n_lwe > 0xFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "n_lwe out of range");
  if (!fbsk) return fail(MI_ERR_INVALID_ARG, "bsk is NULL");
  auto* key = new (std::nothrow) mi_fft64_pbs_key;
  if (!key) return fail(MI_ERR_OOM, "host allocation failed");
  key->plan = plan;
  key->fbsk = fbsk;
  key->n_lwe = n_lwe;
  key->k = k;
  key->base_log = base_log;
  key->level = level;
  *out_key = key;
  return MI_OK;
}

int mi_fft64_pbs_key_destroy(mi_fft64_pbs_key* key) {
  if (key && key->owned) {
    DeviceGuard g(key->plan->device);
    (void)hipFree(key->owned);
  }
  delete key;
  return MI_OK;
}

// ---- the reference's FourierLweBootstrapKey bytes (bincode 1.3 defaults: fixint, little-endian, u64 sequence
// lengths, u32 variant indices).  Field order fft_impl/fft64/crypto/bootstrap.rs:30-39; the list's custom
// Serialize fft_impl/fft64/math/fft/mod.rs:642-690: u64 (2 + chunks), u64 polynomial_size, u64 chunks, then per
// polynomial u64 (N/2) and N/2 (re, im) f64 pairs in the natural order (tfhe-fft unordered.rs:943-964); then
// input_lwe_dimension, glwe_size, decomposition_base_log, decomposition_level_count as u64.  Versioned
// (key.versionize()): u32 1 (FourierLweBootstrapKeyVersions::V1), u32 0 (FourierPolynomialListVersioned::V0) in
// front, a u32 0 (...Versions::V0) before each scalar field (backward_compatibility/fft_impl/mod.rs:14-70).
namespace {
struct FourierLayout {
  uint64_t n_lwe, glwe, base_log, level, chunks;
  size_t head, chunk_bytes, total;  // bytes before the first polynomial's length prefix, per polynomial, all
};

bool fourier_layout(uint64_t m, uint64_t n_lwe, uint64_t glwe, uint64_t level, uint64_t base_log, bool ver,
                    FourierLayout* L) {
  uint64_t c;
  if (__builtin_mul_overflow(glwe, glwe, &c) || __builtin_mul_overflow(c, level, &c) ||
      __builtin_mul_overflow(c, n_lwe, &c))
    return false;
  L->n_lwe = n_lwe, L->glwe = glwe, L->base_log = base_log, L->level = level, L->chunks = c;
  L->head = (ver ? 8 : 0) + 24;
  L->chunk_bytes = 8 + 16 * m;
  size_t body;
  return !__builtin_mul_overflow((size_t)c, L->chunk_bytes, &body) &&
         !__builtin_add_overflow(body, L->head + 32 + (ver ? 16 : 0), &L->total);
}

uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, sizeof v);  // little-endian host
  return v;
}
uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, sizeof v);
  return v;
}
uint8_t* wr32(uint8_t* p, uint32_t v) {
  std::memcpy(p, &v, sizeof v);
  return p + sizeof v;
}
uint8_t* wr64(uint8_t* p, uint64_t v) {
  std::memcpy(p, &v, sizeof v);
  return p + sizeof v;
}
}  // namespace

int mi_fft64_bsk_serialized_size(size_t polynomial_size, size_t n_lwe, int k, int level, int format,
                                 size_t* out_len) {
  if (!out_len) return fail(MI_ERR_INVALID_ARG, "out_len is NULL");
  if (polynomial_size < 2 || (polynomial_size & (polynomial_size - 1)) || polynomial_size > ((size_t)1 << 40))
    return fail(MI_ERR_INVALID_ARG, "polynomial size must be a power of two");
  if (format != MI_NTT_BSK_PLAIN && format != MI_NTT_BSK_VERSIONED) return fail(MI_ERR_INVALID_ARG, "unknown format");
  FourierLayout L;
  if (k < 1 || level < 1 ||
      !fourier_layout(polynomial_size / 2, n_lwe, (uint64_t)k + 1, (uint64_t)level, 0, format == MI_NTT_BSK_VERSIONED, &L))
    return fail(MI_ERR_INVALID_ARG, "Fourier BSK: bad sizes");
  *out_len = L.total;
  return MI_OK;
}

int mi_fft64_pbs_key_load(const mi_fft64_plan* plan, const uint8_t* bytes, size_t len, int format, void* stream,
                          mi_fft64_pbs_key** out_key) {
  if (!out_key) return fail(MI_ERR_INVALID_ARG, "out_key is NULL");
  *out_key = nullptr;
  if (!plan || !bytes) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  if (format != MI_NTT_BSK_PLAIN && format != MI_NTT_BSK_VERSIONED) return fail(MI_ERR_INVALID_ARG, "unknown format");
  const bool ver = format == MI_NTT_BSK_VERSIONED;
  size_t off = 0;
  if (ver) {
    if (len < 8) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: truncated");
    const uint32_t kt = rd32(bytes), lt = rd32(bytes + 4);
    if (kt == 0) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: deprecated V0 version (TFHE-rs < v0.10)");
    if (kt != 1 || lt != 0) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: unknown version tags");
    off = 8;
  }
  if (len - off < 24) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: truncated");
  const uint64_t seq = rd64(bytes + off), n = rd64(bytes + off + 8), chunks = rd64(bytes + off + 16);
  if (n != plan->n) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: polynomial size differs from the plan's");
  if (chunks > ((uint64_t)1 << 40) || seq != chunks + 2)
    return fail(MI_ERR_INVALID_ARG, "Fourier BSK: sequence length is not 2 + the polynomial count");
  // the scalar fields sit after the polynomials
  const size_t m = plan->n / 2, chunk_bytes = 8 + 16 * m, tail = 32 + (ver ? 16 : 0);
  if (len < off + 24 + tail || (len - off - 24 - tail) % chunk_bytes || (len - off - 24 - tail) / chunk_bytes != chunks)
    return fail(MI_ERR_INVALID_ARG, "Fourier BSK: length does not match the polynomial count");
  const uint8_t* t = bytes + off + 24 + chunks * chunk_bytes;
  uint64_t f[4];
  for (int i = 0; i < 4; ++i) {
    if (ver) {
      if (rd32(t) != 0) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: unknown parameter version tag");
      t += 4;
    }
    f[i] = rd64(t);
    t += 8;
  }
  const uint64_t n_lwe = f[0], glwe = f[1], base_log = f[2], level = f[3];
  FourierLayout L;
  if (glwe < 2 || glwe > MAX_GENERIC_K + 1 || level < 1 || level > 63 || base_log < 1 || base_log > 63 ||
      !fourier_layout(m, n_lwe, glwe, level, base_log, ver, &L) || L.chunks != chunks)
    return fail(MI_ERR_INVALID_ARG, "Fourier BSK: the polynomial count does not match n_lwe x level x glwe_size^2");
  int st = check_shape(plan, (int)glwe - 1, (int)base_log, (int)level);
  if (st != MI_OK) return st;
  if (n_lwe == 0 || n_lwe > 0xFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "Fourier BSK: n_lwe out of range");
  for (uint64_t c = 0; c < chunks; ++c)
    if (rd64(bytes + off + 24 + c * chunk_bytes) != m)
      return fail(MI_ERR_INVALID_ARG, "Fourier BSK: a polynomial does not hold N/2 values");
  auto* key = new (std::nothrow) mi_fft64_pbs_key;
  if (!key) return fail(MI_ERR_OOM, "host allocation failed");
  key->plan = plan;
  key->n_lwe = n_lwe;
  key->k = (int)glwe - 1;
  key->base_log = (int)base_log;
  key->level = (int)level;
  DeviceGuard g(plan->device);
  const hipStream_t s = (hipStream_t)stream;
  if (hipMalloc(&key->owned, chunks * 16 * m) != hipSuccess) {
    delete key;
    return fail(MI_ERR_OOM, "Fourier key allocation failed");
  }
  // one strided upload skips the per-polynomial length prefixes, then the natural order becomes the engine's
  hipError_t e = hipMemcpy2DAsync(key->owned, 16 * m, bytes + off + 24 + 8, chunk_bytes, 16 * m, chunks,
                                  hipMemcpyHostToDevice, s);
  st = e == hipSuccess ? MI_OK : hip_fail(e, "Fourier key upload");
  if (st == MI_OK) {
    e = reorder_any(plan, key->owned, key->owned, chunks, false, s);
    st = e == hipSuccess ? MI_OK : hip_fail(e, "fft64 reorder launch");
  }
  if (st == MI_OK && (e = hipStreamSynchronize(s)) != hipSuccess) st = hip_fail(e, "Fourier key upload");
  if (st != MI_OK) {
    (void)hipFree(key->owned);
    delete key;
    return st;
  }
  key->fbsk = key->owned;
  *out_key = key;
  return MI_OK;
}

int mi_fft64_pbs_key_write(const mi_fft64_pbs_key* key, int format, uint8_t* out, size_t out_len, void* stream) {
  if (!key || !out) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  size_t need = 0;
  int st = mi_fft64_bsk_serialized_size(key->plan->n, key->n_lwe, key->k, key->level, format, &need);
  if (st != MI_OK) return st;
  if (out_len != need) return fail(MI_ERR_INVALID_ARG, "output length is not the serialized size");
  const bool ver = format == MI_NTT_BSK_VERSIONED;
  FourierLayout L;
  const size_t m = key->plan->n / 2;
  (void)fourier_layout(m, key->n_lwe, (uint64_t)key->k + 1, (uint64_t)key->level, (uint64_t)key->base_log, ver, &L);
  uint8_t* p = out;
  if (ver) p = wr32(wr32(p, 1), 0);
  p = wr64(wr64(wr64(p, L.chunks + 2), key->plan->n), L.chunks);
  for (uint64_t c = 0; c < L.chunks; ++c) wr64(p + c * L.chunk_bytes, m);
  uint8_t* t = p + L.chunks * L.chunk_bytes;
  for (const uint64_t v : {L.n_lwe, L.glwe, L.base_log, L.level}) {
    if (ver) t = wr32(t, 0);
    t = wr64(t, v);
  }
  DeviceGuard g(key->plan->device);
  const hipStream_t s = (hipStream_t)stream;
  double* tmp = nullptr;
  if (hipMalloc(&tmp, L.chunks * 16 * m) != hipSuccess) return fail(MI_ERR_OOM, "scratch allocation failed");
  hipError_t e = reorder_any(key->plan, tmp, key->fbsk, L.chunks, true, s);
  if (e == hipSuccess) e = hipMemcpy2DAsync(p + 8, L.chunk_bytes, tmp, 16 * m, 16 * m, L.chunks, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(tmp);
  return e == hipSuccess ? MI_OK : hip_fail(e, "Fourier key download");
}

int mi_fft64_pbs_key_info(const mi_fft64_pbs_key* key, size_t* n_lwe, int* k, int* base_log, int* level) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (n_lwe) *n_lwe = key->n_lwe;
  if (k) *k = key->k;
  if (base_log) *base_log = key->base_log;
  if (level) *level = key->level;
  return MI_OK;
}

}  // extern "C"

static int fft_pbs_common(const mi_fft64_pbs_key* key, uint64_t* lwe_out, const uint64_t* lwe_in, const mi::PbsIo& io,
                          size_t batch, int ms_mode, void* stream) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (ms_mode < MI_MS_STANDARD || ms_mode > MI_MS_PRE_SWITCHED) return fail(MI_ERR_INVALID_ARG, "unknown ms_mode");
  if (batch == 0) return MI_OK;
  if ((!lwe_out && !io.glwe_out) || !lwe_in || !io.lut) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (batch > 0x7FFFFFFFull) return fail(MI_ERR_INVALID_ARG, "batch too large");
  DeviceGuard g(key->plan->device);
  const mi_fft64_plan* plan = key->plan;
  const hipError_t e =
      plan->generic ? mi::launch_fftg_pbs(key->k, lwe_out, lwe_in, io, key->fbsk, key->n_lwe, batch, key->base_log,
                                          key->level, ms_mode, plan->gtables, (hipStream_t)stream)
                    : mi::launch_fft64_pbs(key->k, lwe_out, lwe_in, io, key->fbsk, key->n_lwe, batch, key->base_log,
                                           key->level, ms_mode, plan->tables, (hipStream_t)stream);
  return e == hipSuccess ? MI_OK : hip_fail(e, "fft64 pbs launch");
}

extern "C" {

int mi_fft64_pbs_batch(const mi_fft64_pbs_key* key, uint64_t* lwe_out, const uint64_t* lwe_in, const uint64_t* lut,
                       size_t batch, int ms_mode, void* stream) {
  if (batch && !lwe_out) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  mi::PbsIo io;
  io.lut = lut;
  return fft_pbs_common(key, lwe_out, lwe_in, io, batch, ms_mode, stream);
}

int mi_fft64_pbs_batch_lut_indexed(const mi_fft64_pbs_key* key, uint64_t* lwe_out, const uint64_t* lwe_in,
                                   const uint64_t* lut_list, const uint32_t* lut_index, size_t n_lut, size_t batch,
                                   int ms_mode, void* stream) {
  if (batch && !lwe_out) return fail(MI_ERR_INVALID_ARG, "buffer is NULL");
  if (n_lut == 0 || n_lut > 0xFFFFFFFFull) return fail(MI_ERR_INVALID_ARG, "n_lut out of range");
  if (!lut_index && n_lut < batch) return fail(MI_ERR_INVALID_ARG, "per-item LUTs: n_lut < batch");
  mi::PbsIo io;
  io.lut = lut_list;
  io.lut_idx = lut_index;
  io.n_lut = (uint32_t)n_lut;
  io.per_item = lut_index ? 0 : 1;
  return fft_pbs_common(key, lwe_out, lwe_in, io, batch, ms_mode, stream);
}

int mi_fft64_blind_rotate_batch(const mi_fft64_pbs_key* key, uint64_t* acc_glwe, const uint64_t* lwe_in, size_t batch,
                                int ms_mode, void* stream) {
  if (batch && !acc_glwe) return fail(MI_ERR_INVALID_ARG, "acc_glwe is NULL");
  mi::PbsIo io;
  io.lut = acc_glwe;
  io.per_item = 1;
  io.glwe_out = acc_glwe;
  return fft_pbs_common(key, nullptr, lwe_in, io, batch, ms_mode, stream);
}

}  // extern "C"
