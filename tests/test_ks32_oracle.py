"""CPU checks of the KS32 oracle (ks_oracle.c: ora_lwe_keyswitch32, ora_lwe_ms32) — no GPU.

Pins: (1) the C restatement of keyswitch_lwe_ciphertext_with_scalar_change (lwe_keyswitch.rs:331-447) equals an
independent pure-Python restatement on random keys and inputs, including the body's rounding corners and u32 keys
with arbitrary low bits; (2) the reference's own test property (algorithms/test/lwe_keyswitch.rs:220-335): a u64
ciphertext of msg * delta under the big key, keyswitched with a u32 key made as generate_lwe_keyswitch_key does,
decrypts under the small key to msg after round_decode — here at the native u32 modulus and at the HPU KS32
parameters (2048 -> 879, base 2^2, 8 levels, post_keyswitch_ciphertext_modulus 2^21; shortint/parameters/v1_5/
hpu.rs:57-76); (3) the u32 (centered binary) modulus switch (modulus_switch.rs:14-104) equals a Python restatement.
"""
import numpy as np
import pytest

import tfhe_helpers as H
from test_ks_oracle import py_decompose

M32 = 2**32


def py_keyswitch32(ksk, lwe, base_log, level, out_mod_log):
    in_dim = lwe.size - 1
    out = [0] * ksk.shape[-1]
    shift = 64 - out_mod_log - 1
    b = int(lwe[-1])
    body = ((((b >> shift) + 1) & ~1) << shift) % 2**64   # native_closest_representable, one level of w bits
    out[-1] = body >> 32
    for i in range(in_dim):
        for li, t in enumerate(py_decompose(int(lwe[i]), base_log, level)):
            row = ksk[i, li]
            for j in range(len(out)):
                out[j] = (out[j] - int(row[j]) * (t % M32)) % M32
    return np.array(out, np.uint32)


def py_ms32(lwe, log_mod, centered):
    def ms(x):
        return x if log_mod == 32 else ((x + (1 << (32 - log_mod - 1))) % M32) >> (32 - log_mod)

    def signed(x):
        return x - M32 if x >= 1 << 31 else x

    def trunc_div2(x):
        return -((-x) // 2) if x < 0 else x // 2

    a = [int(v) for v in lwe]
    corr = 0
    if centered:
        sh = 0
        hed = 0
        for x in a[:-1]:
            rnd = (ms(x) << (32 - log_mod)) % M32 if log_mod < 32 else ms(x)
            err = signed((rnd - x) % M32)
            half = trunc_div2(err)
            sh = (sh + half) % M32
            hed += 2 * half - err
        sh = (sh - trunc_div2(hed)) % M32
        half_case = 0 if log_mod == 32 else 1 << (32 - log_mod - 1)
        corr = (sh - half_case) % M32
    return np.array([ms(x) for x in a[:-1]] + [ms((a[-1] + corr) % M32)], np.uint64)


@pytest.mark.parametrize("base_log,level,w", [(2, 8, 21), (2, 7, 21), (4, 4, 32), (1, 1, 1), (5, 6, 30), (16, 2, 32)])
def test_ks32_oracle_matches_python_restatement(oracle, base_log, level, w):
    g = H.rng(base_log * 101 + level * 7 + w)
    in_dim, out_dim = 11, 7
    ksk = g.integers(0, M32, size=(in_dim, level, out_dim + 1), dtype=np.uint64).astype(np.uint32)
    lwe = H.uniform_u64(g, (4, in_dim + 1))
    lwe[0, :4] = [0, 2**64 - 1, 1 << 63, (1 << 63) - 1]   # decomposition rounding / balancing corners
    # body rounding corners at w bits: exactly half an output step, half minus one, the top value
    step = 1 << (64 - w)
    lwe[1, -1] = step // 2
    lwe[2, -1] = step // 2 - 1
    lwe[3, -1] = 2**64 - 1
    got = oracle.lwe_keyswitch32(ksk, lwe, out_dim, base_log, level, w)
    for b in range(4):
        assert np.array_equal(got[b], py_keyswitch32(ksk, lwe[b], base_log, level, w)), b


@pytest.mark.parametrize("w", [32, 21])
def test_ks32_decrypts(oracle, w):
    """The reference's test_lwe_keyswitch_with_scalar_change property: every message of a 2+2-bit space with a
    padding bit survives the keyswitch (2048 -> 879, base 2^2, 8 levels) at output modulus 2^w."""
    g = H.rng(879 + w)
    in_dim, out_dim, base_log, level = 2048, 879, 2, 8
    s_in, s_out = H.binary_key(g, in_dim), H.binary_key(g, out_dim)
    ksk = H.ksk32_gen(g, s_in, s_out, base_log, level, noise_log2=2, out_mod_log=w)
    msg_mod = 16
    msgs = np.arange(msg_mod, dtype=np.uint64)
    cts = H.lwe_encrypt_batch(g, msgs << np.uint64(59), s_in, noise_log2=30)   # delta = 2^63 / 16 (padding bit)
    out = oracle.lwe_keyswitch32(ksk, cts, out_dim, base_log, level, w)
    if w < 32:  # check_encrypted_content_respects_mod: the output stays a multiple of 2^(32 - w)
        assert not np.any(out % np.uint32(1 << (32 - w)))
    dec = H.lwe32_decrypt_batch(out, s_out).astype(np.uint64)
    delta32 = 1 << 27
    decoded = ((dec + np.uint64(delta32 // 2)) // np.uint64(delta32)) % np.uint64(msg_mod)
    assert np.array_equal(decoded, msgs)


@pytest.mark.parametrize("log_mod", [12, 1, 31, 32])
@pytest.mark.parametrize("centered", [False, True])
def test_ms32_oracle_matches_python_restatement(oracle, log_mod, centered):
    if centered and log_mod == 32:
        pytest.skip("outside the reference's domain: its half_case shift underflows at log_modulus = BITS")
    g = H.rng(log_mod * 2 + centered)
    dim = 879
    lwe = g.integers(0, M32, size=(3, dim + 1), dtype=np.uint64).astype(np.uint32)
    lwe[1] = (lwe[1] >> np.uint32(11)) << np.uint32(11)   # a 2^21-modulus LWE (MSB encoding)
    lwe[2, :5] = [0, M32 - 1, 1 << 31, (1 << 31) - 1, 1 << 19]
    got = oracle.lwe_ms32(lwe, log_mod, centered)
    for b in range(3):
        want = py_ms32(lwe[b], log_mod, centered)
        assert np.array_equal(got[b], want), b
        assert int(got[b].max()) < (1 << log_mod)
