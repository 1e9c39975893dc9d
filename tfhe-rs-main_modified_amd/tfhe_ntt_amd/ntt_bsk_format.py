"""On-disk NTT bootstrap key: the bytes the reference writes for ``NttLweBootstrapKey<ABox<[u64]>>``.

SURVEY.md §8f rank 2 (the data format on the key side of the path). The reference type is
``NttLweBootstrapKey { ggsw_list: NttGgswCiphertextList }`` (``entities/ntt_lwe_bootstrap_key.rs:26-33``)
whose serde-derived field order is (``entities/ntt_ggsw_ciphertext_list.rs:19-31``)::

    data: ABox<[u64]>                 u64 element count, then the elements (aligned-vec 0.6 serialises
                                      the boxed slice as a serde sequence)
    polynomial_size: PolynomialSize   u64
    glwe_size: GlweSize               u64   (k + 1)
    decomposition_level_count         u64
    decomposition_base_log            u64
    ciphertext_modulus                SerializableCiphertextModulus (commons/ciphertext_modulus.rs:25-120):
                                      modulus: u128 (0 = native 2^64), scalar_bits: u64 (= 64)

with bincode 1.3's default encoding as tfhe uses it (fixint, little-endian, u64 sequence lengths, u32
enum variant indices). Two forms:

* ``PLAIN``      ``bincode::serialize(&key)`` — the layout above;
* ``VERSIONED``  bincode of ``key.versionize()`` (tfhe-versionable): ``NttLweBootstrapKeyVersions::V1``
  (u32 1; V0 is deprecated, ``backward_compatibility/entities/ntt_lwe_bootstrap_key.rs:15-21``) around
  ``NttGgswCiphertextListVersions::V1`` (u32 1) around the fields, the data slice unchanged (u64 is
  not versioned, ``utils/tfhe-versionable/src/lib.rs:738-748``) and each scalar field behind its own
  ``…Versions::V0`` tag (u32 0; ``backward_compatibility/commons/parameters.rs:72-114``,
  ``…/ciphertext_modulus.rs:6-8``). ``NttLweBootstrapKey`` has no ``Named`` impl, so ``safe_serialize``
  (which needs one) does not apply to it: the versioned bincode is its whole versioned form.

``data`` is the NTT-domain GGSW list in the order the engine's key tensor already uses:
(n_lwe, level, k+1, k+1, N) u64, so a key loads into HBM with one copy and no re-layout
(``mi_pbs_ntt64_key_load``). The input LWE dimension is not stored; it is
``len(data) / (level * (k+1)^2 * N)``, as in the reference.

Deserialisation refuses what the reference's ``TryFrom<SerializableCiphertextModulus>`` refuses
(``scalar_bits != 64``), a modulus above 2^64 for this u64 key, unknown version tags, truncated /
trailing bytes and a data length that is not a whole number of GGSWs; a modulus of exactly 2^64 is
canonicalised to native (0) as ``CiphertextModulus::canonicalize`` does. The reference holds no
serialised NTT key, so the byte layout is pinned against the derive orders above (parity of the bytes
is unpinned by fixtures); this module and the library's C parser (``mi_ntt_bsk_parse``) are checked
against each other byte for byte in ``tests/test_ntt_bsk_format.py``.
"""
import struct

import numpy as np

NATIVE_MODULUS = 0  # SerializableCiphertextModulus.modulus for the native 2^64 modulus
PLAIN = 0           # MI_NTT_BSK_PLAIN
VERSIONED = 1       # MI_NTT_BSK_VERSIONED


class NttBskFormatError(ValueError):
    """The bytes are not a valid serialised NttLweBootstrapKey<u64>."""


def _check_modulus(modulus: int) -> int:
    if not 0 <= modulus <= 1 << 64:
        raise NttBskFormatError("ciphertext modulus above 2^64 for a u64 key")
    return 0 if modulus == 1 << 64 else modulus


def serialize_ntt_bsk(data, polynomial_size: int, glwe_size: int, level: int, base_log: int, modulus: int,
                      versioned: bool = False) -> bytes:
    """``data``: u64 array (any shape) holding n_lwe * level * glwe_size^2 * polynomial_size values;
    ``modulus``: the key's ciphertext modulus (an NTT key carries its NTT prime)."""
    arr = np.asarray(data)
    arr = arr.view(np.uint64) if arr.dtype == np.int64 else arr.astype(np.uint64, copy=False)
    flat = np.ascontiguousarray(arr).reshape(-1)
    ggsw = level * glwe_size * glwe_size * polynomial_size
    if ggsw == 0 or flat.size % ggsw:
        raise NttBskFormatError(f"data length {flat.size} is not a multiple of the GGSW size {ggsw}")
    modulus = _check_modulus(modulus)
    tag = (lambda v: struct.pack("<I", v)) if versioned else (lambda v: b"")
    out = [tag(1), tag(1), struct.pack("<Q", flat.size), flat.astype("<u8", copy=False).tobytes()]
    for v in (polynomial_size, glwe_size, level, base_log):
        out += [tag(0), struct.pack("<Q", v)]
    out += [tag(0), struct.pack("<QQQ", modulus & (2**64 - 1), modulus >> 64, 64)]
    return b"".join(out)


def deserialize_ntt_bsk(buf: bytes, versioned: bool = False):
    """Returns (data u64 ndarray shaped (n_lwe, level, k+1, k+1, N), dict of the scalar fields)."""
    mv = memoryview(buf)
    off = 0

    def take(fmt):
        nonlocal off
        size = struct.calcsize(fmt)
        if len(mv) - off < size:
            raise NttBskFormatError("truncated")
        vals = struct.unpack_from(fmt, mv, off)
        off += size
        return vals

    if versioned:
        key_tag, list_tag = take("<II")
        if key_tag == 0 or list_tag == 0:
            raise NttBskFormatError("deprecated V0 version (TFHE-rs < v0.10)")
        if key_tag != 1 or list_tag != 1:
            raise NttBskFormatError(f"unknown version tags {key_tag}, {list_tag}")
    (count,) = take("<Q")
    scalars = 4 * 8 + 24 + (20 if versioned else 0)
    if count > (len(mv) - off) // 8 or len(mv) - off - 8 * count != scalars:
        raise NttBskFormatError(f"length mismatch: {len(mv)} bytes for {count} elements")
    data = np.frombuffer(mv, dtype="<u8", count=count, offset=off).astype(np.uint64)
    off += 8 * count
    fields = []
    for _ in range(4):
        if versioned and take("<I")[0] != 0:
            raise NttBskFormatError("unknown parameter version tag")
        fields.append(take("<Q")[0])
    if versioned and take("<I")[0] != 0:
        raise NttBskFormatError("unknown modulus version tag")
    lo, hi, scalar_bits = take("<QQQ")
    if scalar_bits != 64:
        raise NttBskFormatError(f"Expected an unsigned integer with 64 bits, found {scalar_bits} bits "
                                "during deserialization of CiphertextModulus")
    modulus = _check_modulus(lo | hi << 64)
    n, glwe_size, level, base_log = fields
    ggsw = level * glwe_size * glwe_size * n
    if ggsw == 0 or ggsw >= 1 << 64 or count % ggsw:
        raise NttBskFormatError(f"data length {count} is not a multiple of the GGSW size {ggsw}")
    info = dict(polynomial_size=n, glwe_size=glwe_size, decomposition_level_count=level,
                decomposition_base_log=base_log, ciphertext_modulus=modulus, input_lwe_dimension=count // ggsw)
    return data.reshape(count // ggsw, level, glwe_size, glwe_size, n), info


def save_ntt_bsk(path, *args, **kw) -> None:
    with open(path, "wb") as f:
        f.write(serialize_ntt_bsk(*args, **kw))


def load_ntt_bsk(path, versioned: bool = False):
    with open(path, "rb") as f:
        return deserialize_ntt_bsk(f.read(), versioned)
