"""On-disk NTT bootstrap key (``tfhe_ntt_amd.ntt_bsk_format``): the bincode 1.3 layout of the reference's
``NttLweBootstrapKey<ABox<[u64]>>`` (entities/ntt_lwe_bootstrap_key.rs:26-33,
entities/ntt_ggsw_ciphertext_list.rs:21-31, commons/ciphertext_modulus.rs:48-93).

Parity unpinned: the reference holds no serialised NTT key, so the CPU tests pin every field's offset and
width against the serde derive order by hand; the GPU test checks that a key round-tripped through the
bytes bootstraps bit-identically to the original.
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


@pytest.mark.parametrize("modulus", [0, P, 1 << 64, (1 << 127) + 5])
def test_round_trip(modulus):
    g = H.rng(8)
    key = _key(g, n_lwe=5, level=1, glwe=3, n=32)
    data, f = F.deserialize_ntt_bsk(F.serialize_ntt_bsk(key.view(np.int64), 32, 3, 1, 15, modulus))
    assert np.array_equal(data, key) and data.dtype == np.uint64
    assert f == dict(polynomial_size=32, glwe_size=3, decomposition_level_count=1, decomposition_base_log=15,
                     ciphertext_modulus=modulus, input_lwe_dimension=5)


def test_file_round_trip(tmp_path):
    key = _key(H.rng(9))
    F.save_ntt_bsk(tmp_path / "bsk.bin", key, 16, 2, 2, 23)
    data, f = F.load_ntt_bsk(tmp_path / "bsk.bin")
    assert np.array_equal(data, key) and f["ciphertext_modulus"] == 0


def test_rejects_malformed():
    key = _key(H.rng(10))
    buf = F.serialize_ntt_bsk(key, 16, 2, 2, 23)
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
        F.serialize_ntt_bsk(key.reshape(-1)[:-16], 16, 2, 2, 23)


@pytest.mark.gpu
@pytest.mark.parametrize("bnf", [True, False])
def test_deserialized_key_bootstraps_identically(engine, bnf):
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
    buf = key.serialize()
    key2 = M.NttBootstrapKey.deserialize(plan, buf)
    assert key2.variant == variant and key2.input_lwe_dimension == n_lwe
    run = (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf
           else M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)
    outs = []
    for k in (key, key2):
        out = dev(np.zeros((batch, n + 1), np.uint64))
        run(dev(lwe), out, dev(lut), k)
        outs.append(out.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])


def _cpp_tool():
    import os
    import subprocess
    d = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp")
    subprocess.run(["make", "-C", d, "-s", "bsk_format_tool"], check=True)
    return os.path.join(d, "bsk_format_tool")


def test_cpp_mirror_reads_and_writes_the_same_bytes():
    """include/tfhe_ntt_amd.hpp serialize_ntt_bsk / deserialize_ntt_bsk agree byte for byte with the
    Python mirror (CPU only: the C++ serialiser is header-only)."""
    import subprocess
    tool = _cpp_tool()
    key = _key(H.rng(12), n_lwe=4, level=3, glwe=2, n=64)
    buf = F.serialize_ntt_bsk(key, 64, 2, 3, 7, P)
    r = subprocess.run([tool], input=buf, capture_output=True, check=True)
    assert r.stdout == buf
    assert r.stderr.split() == [b"64", b"2", b"3", b"7", b"4"]
    bad = buf[:-8] + struct.pack("<Q", 32)
    r = subprocess.run([tool], input=bad, capture_output=True)
    assert r.returncode == 3 and b"scalar_bits" in r.stderr
