"""Pin the PBS-side oracle (oracle/pbs_oracle.c) to the reference's own properties (no GPU).

The reference pins this path only functionally: decrypt(PBS(Enc(m))) == f(m)
(algorithms/test/lwe_programmable_bootstrapping.rs:708-865 Solinas, :1002-1163 BNF) plus the
decomposition unit tests (commons/math/decomposition/tests.rs).  Same here, on seeded keys.
"""
import numpy as np
import pytest

import tfhe_helpers as H

SOLINAS_P = 0xFFFFFFFF00000001


def test_native_decomposition_recomposes(oracle):
    # terms recompose to closest_representable and are balanced (|t| <= B/2)
    g = H.rng(1)
    for base_log, level in [(23, 1), (4, 3), (10, 2), (2, 8)]:
        for x in list(H.uniform_u64(g, 200)) + [0, 2**63, 2**64 - 1, 2**63 - 1]:
            st = oracle.decomp_init_native(int(x), base_log, level)
            rec = 0
            for j in range(level, 0, -1):
                t, st = oracle.decompose_one_level(base_log, st)
                ts = t - 2**64 if t >= 2**63 else t
                assert -(1 << (base_log - 1)) <= ts <= (1 << (base_log - 1))
                rec += ts << (64 - base_log * j)
            shift = 64 - base_log * level
            closest = ((((int(x) >> (shift - 1)) + 1) >> 1) << shift) % 2**64  # decomposer.rs:25-49
            assert rec % 2**64 == closest


def test_monomial_ops(oracle):
    n = 64
    g = H.rng(2)
    a = H.uniform_u64(g, n)
    for q in (0, SOLINAS_P):
        aa = a % np.uint64(q) if q else a
        for d in (0, 1, 5, n - 1, n, n + 3, 2 * n - 1):
            m = oracle.poly_monomial_mul(aa, d, q)
            # schoolbook: coefficient i of a*X^d
            ref = np.zeros(n, np.uint64)
            mod = q if q else 2**64
            for i in range(n):
                j = i + d
                sign = -1 if (j // n) % 2 else 1
                ref[j % n] = (sign * int(aa[i])) % mod
            assert np.array_equal(m, ref)
            assert np.array_equal(oracle.poly_monomial_div(m, d, q), aa)


def test_modswitch_roundtrip(oracle):
    g = H.rng(3)
    for x in H.uniform_u64(g, 1000):
        y = oracle.modswitch_p2_to_prime(int(x), 64)
        assert y < SOLINAS_P
        z = oracle.modswitch_prime_to_p2(y, 64)
        assert abs(((z - int(x) + 2**63) % 2**64) - 2**63) <= 2**33  # back-and-forth error ~ 2^32
    assert oracle.modulus_switch(2**64 - 1, 12) == 0  # wraps like the reference's wrapping_add
    assert oracle.modulus_switch(1 << 51, 12) == 1


def _keys(seed, n_lwe, n, k, base_log, level, q):
    g = H.rng(seed)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17 if not q else 12, q)
    return g, lwe_sk, glwe_sk, bsk


@pytest.mark.parametrize("bnf", [True, False])
def test_external_product_decrypts(oracle, bnf):
    n, k, base_log, level = 1024, 1, 23, 1
    q = 0 if bnf else SOLINAS_P
    ctx = oracle.NttContext(n)
    g = H.rng(5)
    glwe_sk = H.binary_key(g, (k, n))
    msg = (H.rng(6).integers(0, 8, n).astype(np.uint64)) << np.uint64(60)
    ct = H.glwe_encrypt(g, msg % np.uint64(q) if q else msg, glwe_sk, 17 if bnf else 12, q)
    for bit in (0, 1):
        ggsw = H.ggsw_encrypt(g, bit, glwe_sk, base_log, level, 17 if bnf else 12, q)
        nggsw = ctx.bsk_to_ntt(ggsw.reshape(-1), 64 if bnf else 0, normalize=not bnf).reshape(ggsw.shape)
        out = ctx.ext_product(np.zeros_like(ct), nggsw, ct, k, base_log, level, bnf=bnf)
        dec = H.glwe_decrypt(out.reshape(k + 1, n), glwe_sk, q)
        want = msg if bit else np.zeros_like(msg)
        diff = (dec.astype(object) - want.astype(object)) % (q if q else 2**64)
        err = np.minimum(diff, (q if q else 2**64) - diff)
        assert int(max(err)) < 2**58, (bit, int(max(err)))


@pytest.mark.parametrize("bnf", [True, False])
def test_pbs_functional(oracle, bnf):
    """decrypt(PBS(Enc(m))) == f(m) for every message (lwe_programmable_bootstrapping.rs:708-865, :1002-1163)."""
    n_lwe, n, k, base_log, level = 48, 2048, 1, 23, 1
    q = 0 if bnf else SOLINAS_P
    msg_mod = 4
    mod = q if q else 2**64
    delta = (mod // 2) // msg_mod if not q else (1 << 63) // msg_mod  # encoding with padding
    ctx = oracle.NttContext(n)
    g, lwe_sk, glwe_sk, bsk = _keys(7 + bnf, n_lwe, n, k, base_log, level, q)
    nbsk = ctx.bsk_to_ntt(bsk.reshape(-1), 64 if bnf else 0, normalize=not bnf)
    f = lambda x: (3 * x + 1) % msg_mod
    lut = H.pbs_lut(n, k, msg_mod, delta, f, q)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for m in range(msg_mod):
        ct = H.lwe_encrypt(g, (m * delta) % mod, lwe_sk, 30 if bnf else 20, q)
        out = ctx.pbs(ct, lut, nbsk, k, base_log, level, bnf=bnf)
        got = H.decode(H.lwe_decrypt(out, out_sk, q), delta, msg_mod, q)
        assert got == f(m), (m, got)


@pytest.mark.parametrize("q", [0, SOLINAS_P])
def test_sample_extract_nth_decrypts(oracle, q):
    """extract_lwe_sample_from_glwe_ciphertext's defining property (glwe_sample_extraction.rs:26-88 doc test): the
    LWE extracted at MonomialDegree(nth) decrypts, under the flattened GLWE key, to coefficient nth of the GLWE's
    plaintext — for every nth, native and custom modulus; nth = 0 equals the nth-0 restatement."""
    n, k = 32, 2
    g = H.rng(41 + (q != 0))
    glwe_sk = H.binary_key(g, (k, n))
    msg = H.uniform_u64(g, n) if not q else g.integers(0, q, n, dtype=np.uint64)
    ct = H.glwe_encrypt(g, msg, glwe_sk, 0, q)
    phase = H.glwe_decrypt(ct, glwe_sk, q)  # msg + the (tiny) noise: extraction keeps the phase exactly
    lwe_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for nth in range(n):
        lwe = oracle.sample_extract_nth(ct.reshape(-1), n, k, nth, q)
        assert int(H.lwe_decrypt(lwe, lwe_sk, q)) == int(phase[nth]), nth
    assert np.array_equal(oracle.sample_extract_nth(ct.reshape(-1), n, k, 0, q),
                          oracle.sample_extract(ct.reshape(-1), n, k, q))


@pytest.mark.parametrize("bnf,ms", [(True, 0), (True, 1), (False, 0)])
def test_blind_rotate_then_extract_is_pbs(oracle, bnf, ms):
    """blind_rotate_ntt64[_bnf]_assign + extraction at 0 == the PBS restatement (ntt64_bnf_pbs.rs:469-540 calls exactly
    these two; ntt64_pbs.rs:482-538 likewise), on the batched oracle entry points the GPU tests compare against."""
    n, k, n_lwe, base_log, level = 1024, 1, 12, 15, 2
    q = 0 if bnf else SOLINAS_P
    g = H.rng(90 + 2 * bnf + ms)
    ctx = oracle.NttContext(n)
    bsk = g.integers(0, SOLINAS_P, size=(n_lwe, level, k + 1, k + 1, n), dtype=np.uint64)
    lut = H.uniform_u64(g, (k + 1, n)) if not q else g.integers(0, q, (k + 1, n), dtype=np.uint64)
    lwe = H.uniform_u64(g, (4, n_lwe + 1)) if not q else g.integers(0, q, (4, n_lwe + 1), dtype=np.uint64)
    accs = np.broadcast_to(lut, (4, k + 1, n)).copy()
    rot = ctx.blind_rotate_batch(accs, lwe, bsk.reshape(-1), k, base_log, level, bnf=bnf, ms_mode=ms)
    for b in range(4):
        want = ctx.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf, centered=ms == 1)
        assert np.array_equal(oracle.sample_extract_nth(rot[b].reshape(-1), n, k, 0, q), want)
    # pre-switched input == the standard switch done by the caller
    if bnf and ms == 0:
        msed = np.vectorize(lambda x: oracle.modulus_switch(int(x), 11), otypes=[np.uint64])(lwe)
        assert np.array_equal(ctx.blind_rotate_batch(accs, msed, bsk.reshape(-1), k, base_log, level, ms_mode=2), rot)
