"""On-disk NTT bootstrap key: the bytes ``bincode::serialize(&NttLweBootstrapKey<ABox<[u64]>>)`` writes.

SURVEY.md §8f rank 2 (the data format on the key side of the path). The reference type is
``NttLweBootstrapKey { ggsw_list: NttGgswCiphertextList }`` (``entities/ntt_lwe_bootstrap_key.rs:26-33``)
whose serde-derived field order is (``entities/ntt_ggsw_ciphertext_list.rs:21-31``)::

    data: ABox<[u64]>                 u64 element count, then the elements (aligned-vec 0.6 serialises
                                      the boxed slice as a serde sequence)
    polynomial_size: PolynomialSize   u64
    glwe_size: GlweSize               u64   (k + 1)
    decomposition_level_count         u64
    decomposition_base_log            u64
    ciphertext_modulus                SerializableCiphertextModulus (commons/ciphertext_modulus.rs:48-93):
                                      modulus: u128 (0 = native 2^64), scalar_bits: u64 (= 64)

with bincode 1.3's default encoding (``tfhe/Cargo.toml:61``): little-endian, fixed-width integers,
u64 sequence lengths. ``data`` is the NTT-domain GGSW list in the order the engine's key tensor already
uses: (n_lwe, level, k+1, k+1, N) u64 (``ntt_ggsw_ciphertext_list.rs``, level-major GGSWs), so a key
loads into HBM with one copy and no re-layout. The input LWE dimension is not stored; it is
``len(data) / (level * (k+1)^2 * N)``, as in the reference.

Deserialisation refuses what the reference's ``TryFrom<SerializableCiphertextModulus>`` refuses
(``scalar_bits != 64``) plus truncated / trailing bytes and a data length that is not a whole number of
GGSWs. The Versionize envelope (``safe_serialize``) is not produced: parity of these bytes is unpinned
(the reference holds no serialised NTT key fixture); the tests pin the field order and widths against
the layout above.
"""
import struct

import numpy as np

NATIVE_MODULUS = 0  # SerializableCiphertextModulus.modulus for the native 2^64 modulus


class NttBskFormatError(ValueError):
    """The bytes are not a valid serialised NttLweBootstrapKey<u64>."""


def serialize_ntt_bsk(data, polynomial_size: int, glwe_size: int, level: int, base_log: int,
                      modulus: int = NATIVE_MODULUS) -> bytes:
    """``data``: u64 array (any shape) holding n_lwe * level * glwe_size^2 * polynomial_size values."""
    arr = np.asarray(data)
    arr = arr.view(np.uint64) if arr.dtype == np.int64 else arr.astype(np.uint64, copy=False)
    flat = np.ascontiguousarray(arr).reshape(-1)
    ggsw = level * glwe_size * glwe_size * polynomial_size
    if ggsw == 0 or flat.size % ggsw:
        raise NttBskFormatError(f"data length {flat.size} is not a multiple of the GGSW size {ggsw}")
    if not 0 <= modulus < 1 << 128:
        raise NttBskFormatError("modulus does not fit u128")
    head = struct.pack("<Q", flat.size)
    body = flat.astype("<u8", copy=False).tobytes()
    fields = struct.pack("<QQQQ", polynomial_size, glwe_size, level, base_log)
    mod = struct.pack("<QQ", modulus & (2**64 - 1), modulus >> 64) + struct.pack("<Q", 64)
    return head + body + fields + mod


def deserialize_ntt_bsk(buf: bytes):
    """Returns (data u64 ndarray shaped (n_lwe, level, k+1, k+1, N), dict of the scalar fields)."""
    mv = memoryview(buf)
    if len(mv) < 8:
        raise NttBskFormatError("truncated: no data length")
    (count,) = struct.unpack_from("<Q", mv, 0)
    need = 8 + 8 * count + 4 * 8 + 16 + 8
    if count > (len(mv) - 8) // 8 or len(mv) != need:
        raise NttBskFormatError(f"length mismatch: {len(mv)} bytes for {count} elements (expected {need})")
    data = np.frombuffer(mv, dtype="<u8", count=count, offset=8).astype(np.uint64)
    off = 8 + 8 * count
    n, glwe_size, level, base_log = struct.unpack_from("<QQQQ", mv, off)
    lo, hi, scalar_bits = struct.unpack_from("<QQQ", mv, off + 32)
    if scalar_bits != 64:
        raise NttBskFormatError(f"Expected an unsigned integer with 64 bits, found {scalar_bits} bits "
                                "during deserialization of CiphertextModulus")
    ggsw = level * glwe_size * glwe_size * n
    if ggsw == 0 or count % ggsw:
        raise NttBskFormatError(f"data length {count} is not a multiple of the GGSW size {ggsw}")
    fields = dict(polynomial_size=n, glwe_size=glwe_size, decomposition_level_count=level,
                  decomposition_base_log=base_log, ciphertext_modulus=lo | hi << 64,
                  input_lwe_dimension=count // ggsw)
    return data.reshape(count // ggsw, level, glwe_size, glwe_size, n), fields


def save_ntt_bsk(path, *args, **kw) -> None:
    with open(path, "wb") as f:
        f.write(serialize_ntt_bsk(*args, **kw))


def load_ntt_bsk(path):
    with open(path, "rb") as f:
        return deserialize_ntt_bsk(f.read())
