"""N beyond one workgroup: the multi-kernel blind rotation / external product of csrc/pbs_large.hip,
at PARAM_MESSAGE_4_CARRY_4's shape (N = 65536, k = 1, n = 1117, B = 2^11, l = 3, TUniform 2^40 LWE / 2^3 GLWE;
shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/ks_pbs.rs:71-90), both NTT variants
(ntt64_bnf_pbs.rs:208-726, ntt64_pbs.rs:213-702):

* key conversion, external product, CMUX (shared and per-item indexed GGSW) and PBS on random keys vs the oracle, bit
  for bit (N = 8192 … 131072, every size the large engine accepts — through the one-launch rotation + forward and
  inverse + accumulate kernels of the split transform, the K = 4 / 5 cooperative tiles and the two-pass top —, small n);
* real keys at the full shape: every one of the 256 messages of the padded 4+4-bit space decrypts to f(m) after the
  PBS (lwe_programmable_bootstrapping.rs:708-865, 1002-1163) — BNF with the centered modulus switch the shortint
  parameters use, Solinas with its own switch; and, on the same real key cut to its first 24 GGSWs (the oracle PBS
  at N = 65536 costs ~0.1 s per CMUX step on one core), 4 real ciphertexts of that dimension bootstrap bit-exactly
  as the oracle's."""
import numpy as np
import pytest

import tfhe_helpers as H

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def rand_q(g, shape, q):
    return g.integers(0, q, size=shape, dtype=np.uint64) if q else H.uniform_u64(g, shape)


@pytest.mark.parametrize("n", [8192, 16384, 32768, 65536, 131072])
@pytest.mark.parametrize("bnf", [True, False])
def test_large_random_keys(engine, oracle, n, bnf):
    """Every N check_pbs_shape accepts past 8192: 32768 runs the K = 4 cooperative first top pass
    (large_rotdec_tile), 131072 the two-pass split (large_rotdec_top<3> then the skip-first split) — ADVICE r4."""
    q = 0 if bnf else P
    k = 1
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    g = H.rng(n + bnf)
    # key conversion (native 2^64 -> p for BNF, Raw; mod-p input, Normalize for Solinas)
    std = rand_q(g, (2, 1, 2, 2, n), q)
    gk = dev(np.zeros_like(std))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(pl, dev(std), gk, normalize=not bnf,
                                                  input_modulus_width=64 if bnf else None)
    assert np.array_equal(host(gk).reshape(-1), c.bsk_to_ntt(std.reshape(-1), 64 if bnf else 0, normalize=not bnf))
    for base_log, level in ((11, 3), (23, 1)):
        batch = 2
        ggsw = rand_q(g, (level, k + 1, k + 1, n), P)
        glwe = rand_q(g, (batch, k + 1, n), q)
        out0 = rand_q(g, (batch, k + 1, n), q)
        want = np.stack([c.ext_product(out0[b].reshape(-1), ggsw.reshape(-1), glwe[b].reshape(-1), k, base_log,
                                       level, bnf=bnf).reshape(k + 1, n) for b in range(batch)])
        out = dev(out0)
        (M.add_external_product_ntt64_bnf_assign if bnf else M.add_external_product_ntt64_assign)(
            pl, out, dev(ggsw), dev(glwe), base_log, level)
        assert np.array_equal(host(out), want), ("ext", base_log, level)
        t0, t1 = dev(out0), dev(glwe)
        (M.cmux_ntt64_bnf_assign if bnf else M.cmux_ntt64_assign)(pl, t0, t1, dev(ggsw), base_log, level)
        want0 = np.stack([c.cmux(out0[b].reshape(-1), glwe[b].reshape(-1), ggsw.reshape(-1), k, base_log, level,
                                 bnf=bnf).reshape(k + 1, n) for b in range(batch)])
        assert np.array_equal(host(t0), want0), ("cmux", base_log, level)
        n_lwe = 3
        bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
        lut = rand_q(g, (k + 1, n), q)
        lwe = rand_q(g, (batch, n_lwe + 1), q)
        lwe[1, 1] = 0
        want = np.stack([c.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf)
                         for b in range(batch)])
        key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
        o = dev(np.zeros((batch, k * n + 1), np.uint64))
        (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf else
         M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)(dev(lwe), o, dev(lut), key)
        assert np.array_equal(host(o), want), ("pbs", base_log, level)


@pytest.mark.parametrize("bnf", [True, False])
def test_large_pbs_two_lanes(engine, oracle, bnf):
    """A chunk of >= 64 ciphertexts runs as two lanes (halves on the caller's stream and a pooled side stream, their
    launches interleaved per CMUX step; pbs_large.hip PBS_LANE_MIN): every output of an odd-split batch of 70 equals
    the one-lane run (batch 8 < 64) of the same items, and an item of each half equals the oracle bit for bit."""
    n, k, base_log, level, n_lwe, batch = 8192, 1, 15, 2, 3, 70
    q = 0 if bnf else P
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    g = H.rng(777 + bnf)
    bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
    lut = rand_q(g, (k + 1, n), q)
    lwe = rand_q(g, (batch, n_lwe + 1), q)
    key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
    fn = (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf else
          M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)
    o = dev(np.zeros((batch, k * n + 1), np.uint64))
    fn(dev(lwe), o, dev(lut), key)
    got = host(o)
    for lo in (0, 31, 62):  # one lane each, covering the first half, the split point (35) and the second half
        o8 = dev(np.zeros((8, k * n + 1), np.uint64))
        fn(dev(lwe[lo:lo + 8]), o8, dev(lut), key)
        assert np.array_equal(host(o8), got[lo:lo + 8]), lo
    for b in (0, batch - 1):
        want = c.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf)
        assert np.array_equal(got[b], want), b


@pytest.mark.parametrize("bnf", [True, False])
def test_large_indexed_ggsw(engine, oracle, bnf):
    """Per-item GGSW index at N = 16384 (mi_*_batch_indexed): item b uses GGSW idx[b]; an index past the list
    leaves both of the item's GLWEs untouched."""
    import torch
    n, k, base_log, level = 16384, 1, 11, 3
    q = 0 if bnf else P
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    g = H.rng(777 + bnf)
    ggsws = rand_q(g, (3, level, k + 1, k + 1, n), P)
    glwe = rand_q(g, (4, k + 1, n), q)
    out0 = rand_q(g, (4, k + 1, n), q)
    idx = np.array([2, 0, 7, 1], np.uint32)
    out, t1 = dev(out0), dev(glwe)
    gi = torch.from_numpy(idx.view(np.int32)).cuda()
    (M.cmux_ntt64_bnf_assign if bnf else M.cmux_ntt64_assign)(pl, out, t1, dev(ggsws), base_log, level, ggsw_index=gi)
    got0, got1 = host(out), host(t1)
    for b in range(4):
        if idx[b] >= 3:
            assert np.array_equal(got0[b], out0[b]) and np.array_equal(got1[b], glwe[b])
            continue
        w = c.cmux(out0[b].reshape(-1), glwe[b].reshape(-1), ggsws[idx[b]].reshape(-1), k, base_log, level, bnf=bnf)
        assert np.array_equal(got0[b].reshape(-1), w), b


@pytest.mark.parametrize("bnf", [True, False])
def test_large_real_keys_message_4_carry_4(engine, oracle, bnf):
    n, k, n_lwe, base_log, level, lwe_noise, glwe_noise, msg_mod = 65536, 1, 1117, 11, 3, 40, 3, 256
    q = 0 if bnf else P
    g = H.rng(4411 + bnf)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen_fast(g, oracle, lwe_sk, glwe_sk, base_log, level, glwe_noise, q)
    delta = (1 << 63) // msg_mod if bnf else (P // 2) // msg_mod
    f = lambda x: (5 * x + 3) % msg_mod
    lut = H.pbs_lut(n, k, msg_mod, delta, f, q)
    msgs = np.arange(msg_mod)
    if bnf:
        lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, lwe_noise)
    else:
        lwe = np.stack([H.lwe_encrypt(g, (int(m) * delta) % P, lwe_sk, lwe_noise, P) for m in msgs])
    M = engine.ntt64_pbs
    pl = engine.Plan.try_new(n, P)
    gkey = dev(np.zeros_like(bsk))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(pl, dev(bsk), gkey, normalize=not bnf,
                                                  input_modulus_width=64 if bnf else None)
    del bsk
    key = M.NttBootstrapKey(pl, gkey, base_log, level, M.BNF if bnf else M.SOLINAS)
    out = dev(np.zeros((msg_mod, k * n + 1), np.uint64))
    if bnf:
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key, ms_mode=M.MS_CENTERED)
    else:
        M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    if bnf:
        pts = H.lwe_decrypt_batch(got, out_sk)
        with np.errstate(over="ignore"):
            dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
        assert np.array_equal(dec, np.array([f(int(m)) for m in msgs], np.uint64))
    else:
        for i, m in enumerate(msgs):
            assert H.decode(H.lwe_decrypt(got[i], out_sk, P), delta, msg_mod, P) % msg_mod == f(int(m)), int(m)
    # bit-exact parity on the real key's first n' GGSWs (ciphertexts of dimension n' under lwe_sk[:n'])
    nn = 24
    sub_sk = lwe_sk[:nn]
    if bnf:
        lwe2 = H.lwe_encrypt_batch(g, np.array([1, 100, 200, 255], np.uint64) * np.uint64(delta), sub_sk, lwe_noise)
    else:
        lwe2 = np.stack([H.lwe_encrypt(g, (m * delta) % P, sub_sk, lwe_noise, P) for m in (1, 100, 200, 255)])
    key2 = M.NttBootstrapKey(pl, gkey[:nn].contiguous(), base_log, level, M.BNF if bnf else M.SOLINAS)
    out2 = dev(np.zeros((4, k * n + 1), np.uint64))
    if bnf:
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(dev(lwe2), out2, dev(lut), key2,
                                                                        ms_mode=M.MS_CENTERED)
    else:
        M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe2), out2, dev(lut), key2)
    nbsk = host(gkey[:nn])
    ctx = oracle.NttContext(n)
    if bnf:
        want = ctx.pbs_batch_bnf(lwe2, lut.reshape(-1), nbsk.reshape(-1), k, base_log, level, threads=4, centered=True)
    else:
        want = ctx.pbs_batch_solinas(lwe2, lut.reshape(-1), nbsk.reshape(-1), k, base_log, level, threads=4)
    assert np.array_equal(host(out2), want)


@pytest.mark.parametrize("k,level", [(2, 1), (1, 4), (2, 2)])
@pytest.mark.parametrize("bnf", [True, False])
def test_large_pbs_mac_fused_term_counts(engine, oracle, k, level, bnf):
    """The MAC-fused inverse bodies (ntt64_tw.hip ntt_tw_inv_mac_kernel, r5) at the term counts l (k + 1) = 3, 8 and
    6 with k = 2 (the shortint shapes run 4 and 6): random-key PBS at N = 16384 bit for bit vs the oracle."""
    n, base_log, n_lwe, batch = 16384, 23 // level if level > 1 else 23, 2, 2
    q = 0 if bnf else P
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    g = H.rng(900 + 10 * k + level + bnf)
    bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
    lut = rand_q(g, (k + 1, n), q)
    lwe = rand_q(g, (batch, n_lwe + 1), q)
    want = np.stack([c.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf)
                     for b in range(batch)])
    key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
    o = dev(np.zeros((batch, k * n + 1), np.uint64))
    (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf else
     M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)(dev(lwe), o, dev(lut), key)
    assert np.array_equal(host(o), want)
