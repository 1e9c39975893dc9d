"""Serialised Fourier bootstrap key: the bytes the reference writes for ``FourierLweBootstrapKey<ABox<[c64]>>``
(the bootstrapping key inside a serialised shortint ``ServerKey`` on the default f64-FFT path).

Reference paths relative to /root/reference/tfhe/src/core_crypto.  The serde-derived field order of
``FourierLweBootstrapKey`` (``fft_impl/fft64/crypto/bootstrap.rs:30-39``)::

    fourier: FourierPolynomialList      custom Serialize (fft_impl/fft64/math/fft/mod.rs:642-690): a sequence of
                                        2 + chunk_count elements = u64 length, then polynomial_size (u64),
                                        chunk_count (u64), then every Fourier polynomial as a sequence of N/2
                                        c64 (u64 length, then (re, im) f64 pairs: num_complex serialises a
                                        Complex as a tuple) in tfhe-fft's STANDARD order -- element i is DFT
                                        frequency i (Plan::serialize_fourier_buffer, tfhe-fft/src/unordered.rs:943-964)
    input_lwe_dimension: LweDimension   u64
    glwe_size: GlweSize                 u64   (k + 1)
    decomposition_base_log              u64
    decomposition_level_count           u64

with bincode 1.3's default encoding as tfhe uses it (fixint, little-endian, u64 sequence lengths, u32 enum
variant indices; the same conventions as ``ntt_bsk_format``). Two forms:

* ``PLAIN``      ``bincode::serialize(&key)`` -- the layout above;
* ``VERSIONED``  bincode of ``key.versionize()``: ``FourierLweBootstrapKeyVersions::V1`` (u32 1; V0 is
  deprecated, ``backward_compatibility/fft_impl/mod.rs:61-70``), the list behind
  ``FourierPolynomialListVersioned::V0`` (u32 0, ``:14-17``, the list's own serialisation unchanged inside) and
  each scalar field behind its ``...Versions::V0`` tag (u32 0, ``backward_compatibility/commons/parameters.rs``).

``data`` is (n_lwe, level, k+1, k+1, N/2, 2) float64 in natural frequency order: the reference's polynomial
order (``FourierLweBootstrapKey::fill_with_forward_fourier`` walks the standard key's polynomials in order), so
the engine's key differs only by the per-polynomial frequency permutation that ``mi_fft64_from_standard_order``
applies on the device (``fft64.FourierLweBootstrapKey.deserialize``).  The reference holds no serialised key, so
the bytes are restated from the derive orders above (unpinned by fixtures); the natural order itself is pinned
by the reference's own test (``unordered.rs:1063-1096``: the plan's output permuted by ``bit_rev_twice`` equals
rustfft's forward DFT, which is what ``serialize_fourier_buffer`` emits).
"""
import struct

import numpy as np

PLAIN = 0
VERSIONED = 1


class FourierBskFormatError(ValueError):
    """The bytes are not a valid serialised FourierLweBootstrapKey."""


def serialize_fourier_bsk(data, polynomial_size: int, glwe_size: int, level: int, base_log: int,
                          versioned: bool = False) -> bytes:
    """``data``: float64 (..., N/2, 2) or complex128 (..., N/2) holding n_lwe * level * glwe_size^2 Fourier
    polynomials in natural frequency order."""
    arr = np.asarray(data)
    m = polynomial_size // 2
    if polynomial_size < 2 or polynomial_size & (polynomial_size - 1):
        raise FourierBskFormatError("polynomial size must be a power of two")
    if np.iscomplexobj(arr):
        arr = np.stack([arr.real, arr.imag], axis=-1)
    flat = np.ascontiguousarray(arr, dtype="<f8").reshape(-1)
    ggsw = level * glwe_size * glwe_size * m * 2
    if ggsw == 0 or flat.size % ggsw:
        raise FourierBskFormatError(f"{flat.size} doubles are not a whole number of GGSWs ({ggsw} each)")
    chunks = flat.size // (2 * m)
    n_lwe = flat.size // ggsw
    tag = (lambda v: struct.pack("<I", v)) if versioned else (lambda v: b"")
    out = [tag(1), tag(0), struct.pack("<QQQ", 2 + chunks, polynomial_size, chunks)]
    polys = flat.reshape(chunks, 2 * m)
    prefix = struct.pack("<Q", m)
    out += [prefix + polys[c].tobytes() for c in range(chunks)]
    for v in (n_lwe, glwe_size, base_log, level):
        out += [tag(0), struct.pack("<Q", v)]
    return b"".join(out)


def deserialize_fourier_bsk(buf: bytes, versioned: bool = False):
    """Returns (data float64 (n_lwe, level, k+1, k+1, N/2, 2) in natural order, dict of the scalar fields)."""
    mv = memoryview(buf)
    off = 0

    def take(fmt):
        nonlocal off
        size = struct.calcsize(fmt)
        if len(mv) - off < size:
            raise FourierBskFormatError("truncated")
        vals = struct.unpack_from(fmt, mv, off)
        off += size
        return vals

    if versioned:
        key_tag, list_tag = take("<II")
        if key_tag == 0:
            raise FourierBskFormatError("deprecated V0 version (TFHE-rs < v0.10)")
        if key_tag != 1 or list_tag != 0:
            raise FourierBskFormatError(f"unknown version tags {key_tag}, {list_tag}")
    seq_len, n, chunks = take("<QQQ")
    if n < 2 or n & (n - 1) or n >= 1 << 40:
        raise FourierBskFormatError(f"invalid polynomial size {n}")
    if seq_len != 2 + chunks:
        raise FourierBskFormatError(f"sequence length {seq_len} != 2 + {chunks} polynomials")
    m = n // 2
    tail = 4 * 8 + (16 if versioned else 0)
    if chunks > (len(mv) - off - tail) // (8 + 16 * m) or len(mv) - off - tail != chunks * (8 + 16 * m):
        raise FourierBskFormatError(f"length mismatch: {len(mv)} bytes for {chunks} polynomials of {m} complex")
    data = np.empty((chunks, m, 2), np.float64)
    for c in range(chunks):
        (cm,) = take("<Q")
        if cm != m:
            raise FourierBskFormatError(f"polynomial {c} holds {cm} values, not {m}")
        data[c] = np.frombuffer(mv, dtype="<f8", count=2 * m, offset=off).reshape(m, 2)
        off += 16 * m
    fields = []
    for _ in range(4):
        if versioned and take("<I")[0] != 0:
            raise FourierBskFormatError("unknown parameter version tag")
        fields.append(take("<Q")[0])
    n_lwe, glwe_size, base_log, level = fields
    if glwe_size < 2 or level < 1 or chunks != n_lwe * level * glwe_size * glwe_size:
        raise FourierBskFormatError(f"{chunks} polynomials do not make {n_lwe} GGSWs of level {level}, "
                                    f"GLWE size {glwe_size}")
    info = dict(polynomial_size=n, glwe_size=glwe_size, decomposition_level_count=level,
                decomposition_base_log=base_log, input_lwe_dimension=n_lwe)
    return data.reshape(n_lwe, level, glwe_size, glwe_size, m, 2), info
