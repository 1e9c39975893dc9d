// c_api_keys.cpp — the on-disk NTT bootstrap key (plain and versioned bincode) and its HBM loader.
//
// Byte layouts (bincode 1.3 default options as tfhe uses them: fixint, little-endian, u64 sequence
// lengths, u32 enum variant indices); reference paths relative to /root/reference/tfhe/src/core_crypto:
//   NttLweBootstrapKey { ggsw_list }                        entities/ntt_lwe_bootstrap_key.rs:26-33
//   NttGgswCiphertextList { data, polynomial_size, glwe_size, decomposition_level_count,
//                           decomposition_base_log, ciphertext_modulus }   entities/ntt_ggsw_ciphertext_list.rs:19-31
//   CiphertextModulus <-> SerializableCiphertextModulus { modulus: u128, scalar_bits: usize }
//                                                           commons/ciphertext_modulus.rs:25-120
// Versioned form (tfhe-versionable: each field replaced by its Versioned form, each Versionize type
// by its VersionsDispatch enum): NttLweBootstrapKeyVersions::V1 (backward_compatibility/entities/
// ntt_lwe_bootstrap_key.rs:15-21, V0 deprecated), NttGgswCiphertextListVersions::V1 (.../
// ntt_ggsw_ciphertext_list.rs:15-21), the ABox<[u64]> as a plain slice (utils/tfhe-versionable/src/
// lib.rs:738-748, u64 is NotVersioned), PolynomialSizeVersions / GlweSizeVersions /
// DecompositionLevelCountVersions / DecompositionBaseLogVersions / SerializableCiphertextModulusVersions
// all V0 (backward_compatibility/commons/parameters.rs:72-114, .../ciphertext_modulus.rs:6-8).
#include <cstring>
#include <new>

#include "c_api_internal.hpp"

using namespace mi::capi;

namespace {

struct Reader {
  const uint8_t* p;
  size_t left;
  bool get(void* dst, size_t n) {
    if (left < n) return false;
    std::memcpy(dst, p, n);  // little-endian host (x86-64 / gfx950 hosts)
    p += n;
    left -= n;
    return true;
  }
  bool u64v(uint64_t& v) { return get(&v, 8); }
  bool u32v(uint32_t& v) { return get(&v, 4); }
};

struct Writer {
  uint8_t* p;
  void put(const void* src, size_t n) {
    std::memcpy(p, src, n);
    p += n;
  }
  void u64v(uint64_t v) { put(&v, 8); }
  void u32v(uint32_t v) { put(&v, 4); }
};

constexpr size_t SCALARS_PLAIN = 4 * 8 + 16 + 8;          // 4 size fields, u128 modulus, scalar_bits
constexpr size_t SCALARS_VERSIONED = SCALARS_PLAIN + 5 * 4;  // + a u32 V0 tag before each of the 5 fields
constexpr size_t HEAD_PLAIN = 8;                             // data length
constexpr size_t HEAD_VERSIONED = 4 + 4 + 8;                 // key V1 tag, list V1 tag, data length

bool ggsw_elems(uint64_t n, uint64_t glwe, uint64_t level, uint64_t* out) {
  uint64_t a;
  return !__builtin_mul_overflow(glwe, glwe, &a) && !__builtin_mul_overflow(a, level, &a) &&
         !__builtin_mul_overflow(a, n, &a) && (*out = a, true);
}

}  // namespace

extern "C" {

int mi_ntt_bsk_parse(const uint8_t* bytes, size_t len, int format, mi_ntt_bsk_header* out) {
  if (!bytes || !out) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  if (format != MI_NTT_BSK_PLAIN && format != MI_NTT_BSK_VERSIONED) return fail(MI_ERR_INVALID_ARG, "unknown format");
  const bool ver = format == MI_NTT_BSK_VERSIONED;
  Reader r{bytes, len};
  mi_ntt_bsk_header h{};
  if (ver) {
    uint32_t key_tag = 0, list_tag = 0;
    if (!r.u32v(key_tag) || !r.u32v(list_tag)) return fail(MI_ERR_INVALID_ARG, "NTT BSK: truncated version tags");
    if (key_tag == 0 || list_tag == 0)
      return fail(MI_ERR_INVALID_ARG, "NTT BSK: deprecated V0 version (TFHE-rs < v0.10), unsupported as the reference");
    if (key_tag != 1 || list_tag != 1) return fail(MI_ERR_INVALID_ARG, "NTT BSK: unknown version tag");
  }
  if (!r.u64v(h.count)) return fail(MI_ERR_INVALID_ARG, "NTT BSK: truncated data length");
  const size_t scalars = ver ? SCALARS_VERSIONED : SCALARS_PLAIN;
  if (h.count > (r.left / 8) || r.left - 8 * h.count != scalars)
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: length mismatch (truncated or trailing bytes)");
  h.data_offset = (uint64_t)(r.p - bytes);
  r.p += 8 * h.count;
  r.left -= 8 * h.count;
  uint64_t* fields[4] = {&h.polynomial_size, &h.glwe_size, &h.level, &h.base_log};
  for (uint64_t* f : fields) {
    uint32_t tag = 0;
    if (ver && (!r.u32v(tag) || tag != 0)) return fail(MI_ERR_INVALID_ARG, "NTT BSK: unknown parameter version tag");
    if (!r.u64v(*f)) return fail(MI_ERR_INVALID_ARG, "NTT BSK: truncated");
  }
  uint32_t mtag = 0;
  if (ver && (!r.u32v(mtag) || mtag != 0)) return fail(MI_ERR_INVALID_ARG, "NTT BSK: unknown modulus version tag");
  uint64_t bits = 0;
  if (!r.u64v(h.modulus_lo) || !r.u64v(h.modulus_hi) || !r.u64v(bits)) return fail(MI_ERR_INVALID_ARG, "NTT BSK: truncated");
  if (bits != 64)  // TryFrom<SerializableCiphertextModulus> for CiphertextModulus<u64>
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: expected an unsigned integer with 64 bits in the ciphertext modulus");
  if (h.modulus_hi > 1 || (h.modulus_hi == 1 && h.modulus_lo != 0))
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: ciphertext modulus above 2^64 for a u64 key");
  if (h.modulus_hi == 1) h.modulus_hi = 0;  // 2^64 canonicalises to native (ciphertext_modulus.rs:217)
  uint64_t ggsw = 0;
  if (!ggsw_elems(h.polynomial_size, h.glwe_size, h.level, &ggsw) || ggsw == 0 || h.count % ggsw)
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: data is not a whole number of GGSWs");
  h.input_lwe_dimension = h.count / ggsw;
  *out = h;
  return MI_OK;
}

int mi_ntt_bsk_serialized_size(const mi_ntt_bsk_header* h, int format, size_t* out_len) {
  if (!h || !out_len) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  if (format != MI_NTT_BSK_PLAIN && format != MI_NTT_BSK_VERSIONED) return fail(MI_ERR_INVALID_ARG, "unknown format");
  const bool ver = format == MI_NTT_BSK_VERSIONED;
  if (h->count > (SIZE_MAX - 128) / 8) return fail(MI_ERR_INVALID_ARG, "NTT BSK: data too large");
  *out_len = (ver ? HEAD_VERSIONED + SCALARS_VERSIONED : HEAD_PLAIN + SCALARS_PLAIN) + 8 * h->count;
  return MI_OK;
}

int mi_ntt_bsk_write(const mi_ntt_bsk_header* h, const uint64_t* data, int format, uint8_t* out, size_t out_len) {
  size_t need = 0;
  int st = mi_ntt_bsk_serialized_size(h, format, &need);
  if (st != MI_OK) return st;
  if (!out || (h->count && !data)) return fail(MI_ERR_INVALID_ARG, "NULL argument");
  if (out_len != need) return fail(MI_ERR_INVALID_ARG, "output buffer size differs from mi_ntt_bsk_serialized_size");
  uint64_t ggsw = 0;
  if (!ggsw_elems(h->polynomial_size, h->glwe_size, h->level, &ggsw) || ggsw == 0 || h->count % ggsw)
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: data is not a whole number of GGSWs");
  if (h->modulus_hi > 1 || (h->modulus_hi == 1 && h->modulus_lo != 0))
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: ciphertext modulus above 2^64 for a u64 key");
  const bool ver = format == MI_NTT_BSK_VERSIONED;
  Writer w{out};
  if (ver) {
    w.u32v(1);
    w.u32v(1);
  }
  w.u64v(h->count);
  w.put(data, 8 * h->count);
  for (uint64_t v : {h->polynomial_size, h->glwe_size, h->level, h->base_log}) {
    if (ver) w.u32v(0);
    w.u64v(v);
  }
  if (ver) w.u32v(0);
  const bool two64 = h->modulus_hi == 1;  // 2^64 is written as native, the form TryFrom produces
  w.u64v(two64 ? 0 : h->modulus_lo);
  w.u64v(0);
  w.u64v(64);
  return MI_OK;
}

int mi_pbs_ntt64_key_load(const mi_ntt64_plan* plan, const uint8_t* bytes, size_t len, int format, int variant,
                          void* stream, mi_pbs_ntt64_key** out_key) {
  if (!out_key) return fail(MI_ERR_INVALID_ARG, "out_key is NULL");
  *out_key = nullptr;
  if (!plan) return fail(MI_ERR_INVALID_ARG, "plan is NULL");
  mi_ntt_bsk_header h{};
  int st = mi_ntt_bsk_parse(bytes, len, format, &h);
  if (st != MI_OK) return st;
  if (h.polynomial_size != plan->n) return fail(MI_ERR_INVALID_ARG, "NTT BSK: polynomial size differs from the plan's");
  if (h.modulus_hi != 0 || h.modulus_lo != plan->p)
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: ciphertext modulus is not the plan's NTT prime");
  if (h.glwe_size < 2 || h.base_log > 64 || h.level > 64) return fail(MI_ERR_INVALID_ARG, "NTT BSK: bad sizes");
  st = check_pbs_shape(plan, (int)(h.glwe_size - 1), (int)h.base_log, (int)h.level, variant);
  if (st != MI_OK) return st;
  if (h.input_lwe_dimension == 0 || h.input_lwe_dimension > 0xFFFFFFFull)
    return fail(MI_ERR_INVALID_ARG, "NTT BSK: input LWE dimension out of range");
  mi_pbs_ntt64_key* key = new (std::nothrow) mi_pbs_ntt64_key;
  if (!key) return fail(MI_ERR_OOM, "host allocation failed");
  key->plan = plan;
  key->n_lwe = h.input_lwe_dimension;
  key->k = (int)h.glwe_size - 1;
  key->base_log = (int)h.base_log;
  key->level = (int)h.level;
  key->variant = variant;
  DeviceGuard g(plan->device);
  const hipStream_t s = (hipStream_t)stream;
  if (hipMalloc(&key->owned, h.count * sizeof(u64)) != hipSuccess) {
    delete key;
    return fail(MI_ERR_OOM, "bootstrap key allocation failed");
  }
  hipError_t e = hipMemcpyAsync(key->owned, bytes + h.data_offset, h.count * sizeof(u64), hipMemcpyHostToDevice, s);
  st = e == hipSuccess ? MI_OK : hip_fail(e, "bootstrap key upload");
  // (synchronises s: the host bytes may be freed once this returns)
  if (st == MI_OK)
    st = prepare_pbs_key(plan, variant, key->k, key->base_log, key->level, key->owned, key->owned, h.count, s);
  if (st != MI_OK) {
    (void)hipFree(key->owned);
    delete key;
    return st;
  }
  key->bsk = key->owned;
  *out_key = key;
  return MI_OK;
}

int mi_pbs_ntt64_key_info(const mi_pbs_ntt64_key* key, size_t* n_lwe, int* k, int* base_log, int* level, int* variant) {
  if (!key) return fail(MI_ERR_INVALID_ARG, "key is NULL");
  if (n_lwe) *n_lwe = key->n_lwe;
  if (k) *k = key->k;
  if (base_log) *base_log = key->base_log;
  if (level) *level = key->level;
  if (variant) *variant = key->variant;
  return MI_OK;
}

}  // extern "C"
