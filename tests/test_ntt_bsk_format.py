"""On-disk NTT bootstrap key (``tfhe_ntt_amd.ntt_bsk_format``, C ABI ``mi_ntt_bsk_*``): the bincode 1.3
layouts (plain and versioned) of the reference's ``NttLweBootstrapKey<ABox<[u64]>>``
(entities/ntt_lwe_bootstrap_key.rs:26-33, entities/ntt_ggsw_ciphertext_list.rs:19-31,
commons/ciphertext_modulus.rs:25-120, backward_compatibility/entities/ntt_*.rs).

Parity unpinned: the reference holds no serialised NTT key, so the CPU tests pin every field's offset and
width against the serde / tfhe-versionable derive order by hand and check the Python and library
parsers against each other; the GPU test checks that a key round-tripped through the bytes bootstraps
bit-identically to the original.
"""
import struct

import numpy as np
import pytest

import tfhe_helpers as H
from tfhe_ntt_amd import ntt_bsk_format as F

P = 0xFFFFFFFF00000001


def _key(g, n_lwe=3, level=2, glwe=2, n=16):
    return g.integers(0, P, size=(n_lwe, level, glwe, glwe, n), dtype=np.uint64)


def test_layout_fields_by_offset():
    g = H.rng(7)
    key = _key(g)
    buf = F.serialize_ntt_bsk(key, 16, 2, 2, 23, P)
    count = key.size
    assert len(buf) == 8 + 8 * count + 4 * 8 + 16 + 8
    assert struct.unpack_from("<Q", buf, 0)[0] == count
    assert np.array_equal(np.frombuffer(buf, "<u8", count, 8), key.reshape(-1))  # level-major GGSW order
    off = 8 + 8 * count
    assert struct.unpack_from("<QQQQ", buf, off) == (16, 2, 2, 23)  # N, glwe_size, level, base_log
    assert struct.unpack_from("<QQ", buf, off + 32) == (P, 0)  # u128 modulus, little-endian halves
    assert struct.unpack_from("<Q", buf, off + 48)[0] == 64  # scalar_bits


@pytest.mark.parametrize("versioned", [False, True])
@pytest.mark.parametrize("modulus", [0, P, 1 << 63])
def test_round_trip(modulus, versioned):
    g = H.rng(8)
    key = _key(g, n_lwe=5, level=1, glwe=3, n=32)
    buf = F.serialize_ntt_bsk(key.view(np.int64), 32, 3, 1, 15, modulus, versioned)
    data, f = F.deserialize_ntt_bsk(buf, versioned)
    assert np.array_equal(data, key) and data.dtype == np.uint64
    assert f == dict(polynomial_size=32, glwe_size=3, decomposition_level_count=1, decomposition_base_log=15,
                     ciphertext_modulus=modulus, input_lwe_dimension=5)


def test_versioned_layout_fields_by_offset():
    """bincode of key.versionize(): NttLweBootstrapKeyVersions::V1, NttGgswCiphertextListVersions::V1, the
    data, then each scalar behind its own V0 tag (see ntt_bsk_format's docstring for the references)."""
    key = _key(H.rng(13))
    buf = F.serialize_ntt_bsk(key, 16, 2, 2, 23, P, versioned=True)
    count = key.size
    assert len(buf) == 8 + 8 + 8 * count + 5 * 4 + 4 * 8 + 16 + 8
    assert struct.unpack_from("<IIQ", buf, 0) == (1, 1, count)
    assert np.array_equal(np.frombuffer(buf, "<u8", count, 16), key.reshape(-1))
    off = 16 + 8 * count
    assert struct.unpack_from("<IQIQIQIQ", buf, off) == (0, 16, 0, 2, 0, 2, 0, 23)
    assert struct.unpack_from("<IQQQ", buf, off + 48) == (0, P, 0, 64)
    plain = F.serialize_ntt_bsk(key, 16, 2, 2, 23, P)
    with pytest.raises(F.NttBskFormatError):  # the two forms are not interchangeable
        F.deserialize_ntt_bsk(plain, versioned=True)
    with pytest.raises(F.NttBskFormatError):
        F.deserialize_ntt_bsk(buf, versioned=False)
    with pytest.raises(F.NttBskFormatError, match="deprecated"):
        F.deserialize_ntt_bsk(struct.pack("<I", 0) + buf[4:], versioned=True)
    with pytest.raises(F.NttBskFormatError, match="version tag"):
        F.deserialize_ntt_bsk(buf[:off] + struct.pack("<I", 1) + buf[off + 4:], versioned=True)


def test_modulus_canonicalisation_and_range():
    """2^64 is the native modulus for a u64 key (CiphertextModulus::canonicalize); above 2^64 is refused."""
    key = _key(H.rng(14))
    _, f = F.deserialize_ntt_bsk(F.serialize_ntt_bsk(key, 16, 2, 2, 23, 1 << 64))
    assert f["ciphertext_modulus"] == 0
    with pytest.raises(F.NttBskFormatError, match="above 2"):
        F.serialize_ntt_bsk(key, 16, 2, 2, 23, (1 << 64) + 1)
    buf = F.serialize_ntt_bsk(key, 16, 2, 2, 23, P)
    bad = buf[:-24] + struct.pack("<QQQ", 5, 1, 64)  # modulus 2^64 + 5
    with pytest.raises(F.NttBskFormatError, match="above 2"):
        F.deserialize_ntt_bsk(bad)


def test_file_round_trip(tmp_path):
    key = _key(H.rng(9))
    F.save_ntt_bsk(tmp_path / "bsk.bin", key, 16, 2, 2, 23, P)
    data, f = F.load_ntt_bsk(tmp_path / "bsk.bin")
    assert np.array_equal(data, key) and f["ciphertext_modulus"] == P


def test_rejects_malformed():
    key = _key(H.rng(10))
    buf = F.serialize_ntt_bsk(key, 16, 2, 2, 23, P)
    with pytest.raises(F.NttBskFormatError):
        F.deserialize_ntt_bsk(buf[:-1])  # truncated
    with pytest.raises(F.NttBskFormatError):
        F.deserialize_ntt_bsk(buf + b"\0")  # trailing bytes
    with pytest.raises(F.NttBskFormatError):
        F.deserialize_ntt_bsk(b"\x01")
    bad_bits = buf[:-8] + struct.pack("<Q", 32)  # a u32 key (reference TryFrom refuses it)
    with pytest.raises(F.NttBskFormatError, match="64 bits"):
        F.deserialize_ntt_bsk(bad_bits)
    huge = struct.pack("<Q", 1 << 62) + buf[8:]
    with pytest.raises(F.NttBskFormatError):
        F.deserialize_ntt_bsk(huge)
    with pytest.raises(F.NttBskFormatError):  # not a whole number of GGSWs
        F.serialize_ntt_bsk(key.reshape(-1)[:-16], 16, 2, 2, 23, P)


def _lib_parse(buf, versioned):
    import ctypes
    from tfhe_ntt_amd import _lib as L
    h = L.NttBskHeader()
    st = L.lib().mi_ntt_bsk_parse(buf, len(buf), int(versioned), ctypes.byref(h))
    return st, h


@pytest.mark.parametrize("versioned", [False, True])
def test_library_parser_agrees_with_python(versioned):
    """The C-ABI parser / writer (mi_ntt_bsk_parse / _write: host-only, no device) and this module agree
    byte for byte, and refuse the same malformed inputs."""
    import ctypes
    from tfhe_ntt_amd import _lib as L
    key = _key(H.rng(15), n_lwe=3, level=2, glwe=2, n=32)
    buf = F.serialize_ntt_bsk(key, 32, 2, 2, 11, P, versioned)
    st, h = _lib_parse(buf, versioned)
    assert st == 0
    assert (h.polynomial_size, h.glwe_size, h.level, h.base_log, h.modulus_lo, h.modulus_hi,
            h.input_lwe_dimension, h.count) == (32, 2, 2, 11, P, 0, 3, key.size)
    assert np.array_equal(np.frombuffer(buf, "<u8", h.count, h.data_offset), key.reshape(-1))
    size = ctypes.c_size_t()
    assert L.lib().mi_ntt_bsk_serialized_size(ctypes.byref(h), int(versioned), ctypes.byref(size)) == 0
    out = ctypes.create_string_buffer(size.value)
    flat = np.ascontiguousarray(key.reshape(-1))
    assert L.lib().mi_ntt_bsk_write(ctypes.byref(h), flat.ctypes.data, int(versioned), out, size.value) == 0
    assert out.raw == buf
    for bad in (buf[:-1], buf + b"\0", buf[:-8] + struct.pack("<Q", 32),
                buf[:-24] + struct.pack("<QQQ", 5, 1, 64)):
        with pytest.raises(F.NttBskFormatError):
            F.deserialize_ntt_bsk(bad, versioned)
        assert _lib_parse(bad, versioned)[0] == L.MI_ERR_INVALID_ARG
    # size fields whose product wraps 2^64 (glwe_size = 2^32): refused, not read as a tiny GGSW
    start = len(buf) - (76 if versioned else 56)  # the scalar fields
    wrap = bytearray(buf)
    struct.pack_into("<Q", wrap, start + (16 if versioned else 8), 1 << 32)
    assert _lib_parse(bytes(wrap), versioned)[0] == L.MI_ERR_INVALID_ARG
    with pytest.raises(F.NttBskFormatError):
        F.deserialize_ntt_bsk(bytes(wrap), versioned)


@pytest.mark.gpu
@pytest.mark.parametrize("versioned", [False, True])
@pytest.mark.parametrize("bnf", [True, False])
def test_deserialized_key_bootstraps_identically(engine, bnf, versioned):
    """A key written with the NTT prime as its modulus (as the reference stores BNF and Solinas keys alike)
    is read back with the explicit variant, both through the host parser and the C-ABI HBM loader, and
    bootstraps bit-identically to the original."""
    import torch
    M = engine.ntt64_pbs
    n, n_lwe, batch = 2048, 24, 5
    plan = engine.Plan.try_new(n, P)
    g = H.rng(11 + bnf)
    bsk = g.integers(0, P, size=(n_lwe, 1, 2, 2, n), dtype=np.uint64)
    q = 0 if bnf else P
    lut = H.uniform_u64(g, (2, n)) if bnf else g.integers(0, P, size=(2, n), dtype=np.uint64)
    lwe = H.uniform_u64(g, (batch, n_lwe + 1)) if bnf else g.integers(0, q, size=(batch, n_lwe + 1), dtype=np.uint64)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).cuda()
    variant = M.BNF if bnf else M.SOLINAS
    key = M.NttBootstrapKey(plan, dev(bsk), 23, 1, variant)
    buf = key.serialize(versioned)
    assert F.deserialize_ntt_bsk(buf, versioned)[1]["ciphertext_modulus"] == P
    key2 = M.NttBootstrapKey.deserialize(plan, buf, variant, versioned)
    key3 = M.NttBootstrapKey.load(plan, buf, variant, versioned)
    for k in (key2, key3):
        assert k.variant == variant and k.input_lwe_dimension == n_lwe
    run = (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf
           else M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)
    outs = []
    for k in (key, key2, key3):
        out = dev(np.zeros((batch, n + 1), np.uint64))
        run(dev(lwe), out, dev(lut), k)
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    with pytest.raises(F.NttBskFormatError):  # a native-modulus "NTT key" is not one (Ntt64::new asserts)
        M.NttBootstrapKey.deserialize(plan, F.serialize_ntt_bsk(bsk, n, 2, 1, 23, 0, versioned), variant, versioned)
    with pytest.raises(engine.MiError):
        M.NttBootstrapKey.load(plan, F.serialize_ntt_bsk(bsk, n, 2, 1, 23, 0, versioned), variant, versioned)


def _cpp_tool():
    import os
    import subprocess
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")
    subprocess.run(["make", "-C", d, "-s", "bsk_format_tool"], check=True)
    return os.path.join(d, "bsk_format_tool")


@pytest.mark.parametrize("versioned", [False, True])
def test_cpp_mirror_reads_and_writes_the_same_bytes(versioned):
    """include/tfhe_ntt_amd.hpp serialize_ntt_bsk / deserialize_ntt_bsk (over mi_ntt_bsk_*) agree byte for
    byte with the Python mirror (CPU only: the format calls touch no device)."""
    import subprocess
    tool = _cpp_tool()
    key = _key(H.rng(12), n_lwe=4, level=3, glwe=2, n=64)
    buf = F.serialize_ntt_bsk(key, 64, 2, 3, 7, P, versioned)
    arg = ["1" if versioned else "0"]
    r = subprocess.run([tool] + arg, input=buf, capture_output=True, check=True)
    assert r.stdout == buf
    assert r.stderr.split() == [b"64", b"2", b"3", b"7", b"4"]
    bad = buf[:-8] + struct.pack("<Q", 32)
    r = subprocess.run([tool] + arg, input=bad, capture_output=True)
    assert r.returncode == 3 and b"64 bits" in r.stderr
