"""CPU checks of the LWE keyswitch oracle (ks_oracle.c) — no GPU.

Pins: (1) the C restatement equals an independent pure-Python restatement of
keyswitch_lwe_ciphertext_native_mod_compatible (lwe_keyswitch.rs:137-227) on random keys and inputs,
including the level ordering of the key blocks; (2) the reference's own doc-test property
(lwe_keyswitch.rs:29-102): a ciphertext of msg << 60 keyswitched with a key made as
generate_lwe_keyswitch_key does (lwe_keyswitch_key_generation.rs:169-199) decrypts under the output
key to msg after rounding to the top 4 bits, here at both the doc-test shape (742 -> 2048, base 2^3,
5 levels) and the PARAM_MESSAGE_2_CARRY_2 shape (2048 -> 918, base 2^4, 4 levels, ks_pbs.rs:38-39).
"""
import numpy as np
import pytest

import tfhe_helpers as H

M64 = 2**64


def py_decompose(x, base_log, level):
    """decomposer.rs:156-185 + iter.rs:103-151 in plain Python integers (least significant first)."""
    rep = base_log * level
    res = x >> (64 - rep - 1)
    rbit = res & 1
    res = ((res + 1) >> 1) & ((1 << rep) - 1)
    need = ((((res - 1) % M64) | (rbit << (rep - 1))) & res) >> (rep - 1)
    state = (res - (need << rep)) % M64
    terms = []
    for _ in range(level):
        r = state & ((1 << base_log) - 1)
        state = (state >> base_log) | ((M64 - (1 << (64 - base_log))) if state >> 63 else 0)  # arithmetic shift
        carry = ((((r - 1) % M64) | state) & r) >> (base_log - 1)
        state = (state + carry) % M64
        terms.append((r - (carry << base_log)) % M64)
    return terms


def py_keyswitch(ksk, lwe, base_log, level):
    in_dim = lwe.size - 1
    out = [0] * ksk.shape[-1]
    out[-1] = int(lwe[-1])
    for i in range(in_dim):
        for li, t in enumerate(py_decompose(int(lwe[i]), base_log, level)):
            row = ksk[i, li]
            for j in range(len(out)):
                out[j] = (out[j] - int(row[j]) * t) % M64
    return np.array(out, np.uint64)


@pytest.mark.parametrize("base_log,level", [(4, 4), (3, 5), (1, 1), (7, 3), (15, 2)])
def test_oracle_matches_python_restatement(oracle, base_log, level):
    g = H.rng(base_log * 31 + level)
    in_dim, out_dim = 13, 9
    ksk = H.uniform_u64(g, (in_dim, level, out_dim + 1))
    lwe = H.uniform_u64(g, (3, in_dim + 1))
    lwe[0, :4] = [0, M64 - 1, 1 << 63, (1 << 63) - 1]   # rounding / balancing corners
    got = oracle.lwe_keyswitch(ksk, lwe, out_dim, base_log, level)
    for b in range(3):
        assert np.array_equal(got[b], py_keyswitch(ksk, lwe[b], base_log, level))


@pytest.mark.parametrize("in_dim,out_dim,base_log,level", [(742, 2048, 3, 5), (2048, 918, 4, 4)])
def test_keyswitch_decrypts(oracle, in_dim, out_dim, base_log, level):
    g = H.rng(in_dim + out_dim)
    s_in, s_out = H.binary_key(g, in_dim), H.binary_key(g, out_dim)
    ksk = H.ksk_gen(g, s_in, s_out, base_log, level, noise_log2=10)
    msgs = np.arange(16, dtype=np.uint64)
    cts = H.lwe_encrypt_batch(g, msgs << np.uint64(60), s_in, noise_log2=10)
    out = oracle.lwe_keyswitch(ksk, cts, out_dim, base_log, level)
    dec = H.lwe_decrypt_batch(out, s_out)
    rounded = ((dec >> np.uint64(59)) + np.uint64(1)) >> np.uint64(1)   # closest_representable, 4 bits
    assert np.array_equal(rounded % np.uint64(16), msgs)
