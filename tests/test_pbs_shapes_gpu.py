"""The PBS / external-product consumers at the other shortint shapes, both NTT variants:

* PARAM_MESSAGE_1_CARRY_1: N = 512, k = 4, n = 879, B = 2^23, l = 1, TUniform 2^46 LWE / 2^17 GLWE;
* PARAM_MESSAGE_3_CARRY_3: N = 8192, k = 1, n = 1077, B = 2^15, l = 2, TUniform 2^41 / 2^3
  (shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/ks_pbs.rs:8-27, 50-67).

The reference's NTT PBS is shape generic (ntt64_bnf_pbs.rs:541-681, ntt64_pbs.rs:553-663).  Per shape and variant:
random-key parity of the external product, CMUX and PBS against the oracle (small n), and a real-key functional
test: every message decrypts to f(m) after the PBS (lwe_programmable_bootstrapping.rs:708-865, 1002-1163), with
two of the real-key outputs compared with the oracle PBS bit for bit.  PARAM_MESSAGE_4_CARRY_4 (N = 65536) is
tests/test_pbs_large_gpu.py."""
import numpy as np
import pytest

import tfhe_helpers as H

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001

# name: (N, k, n_lwe, base_log, level, lwe_noise_log2, glwe_noise_log2, message x carry modulus)
PARAMS = {
    "message_1_carry_1": (512, 4, 879, 23, 1, 46, 17, 4),
    "message_3_carry_3": (8192, 1, 1077, 15, 2, 41, 3, 64),
}


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def rand_q(g, shape, q):
    return g.integers(0, q, size=shape, dtype=np.uint64) if q else H.uniform_u64(g, shape)


# N = 512, k = 4 runs the level-1 PBS whose MAC loads its key one column at a time (the SB schedule, r5)
@pytest.mark.parametrize("n,k", [(512, 1), (512, 4), (8192, 1)])
@pytest.mark.parametrize("bnf", [True, False])
def test_shape_ext_product_cmux_pbs_random_keys(engine, oracle, n, k, bnf):
    q = 0 if bnf else P
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    for base_log, level in ((23, 1), (15, 2), (7, 3)):
        g = H.rng(n + 17 * k + base_log + bnf)
        batch = 3
        ggsw = rand_q(g, (level, k + 1, k + 1, n), P)
        glwe = rand_q(g, (batch, k + 1, n), q)
        out0 = rand_q(g, (batch, k + 1, n), q)
        want = np.stack([c.ext_product(out0[b].reshape(-1), ggsw.reshape(-1), glwe[b].reshape(-1), k, base_log,
                                       level, bnf=bnf).reshape(k + 1, n) for b in range(batch)])
        out = dev(out0)
        fn = M.add_external_product_ntt64_bnf_assign if bnf else M.add_external_product_ntt64_assign
        fn(pl, out, dev(ggsw), dev(glwe), base_log, level)
        assert np.array_equal(host(out), want), ("ext", base_log, level)
        t0, t1 = dev(out0), dev(glwe)
        fn = M.cmux_ntt64_bnf_assign if bnf else M.cmux_ntt64_assign
        fn(pl, t0, t1, dev(ggsw), base_log, level)
        want0 = np.stack([c.cmux(out0[b].reshape(-1), glwe[b].reshape(-1), ggsw.reshape(-1), k, base_log, level,
                                 bnf=bnf).reshape(k + 1, n) for b in range(batch)])
        assert np.array_equal(host(t0), want0), ("cmux", base_log, level)
        # PBS on a random key of the same shape
        n_lwe = 10
        bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
        lut = rand_q(g, (k + 1, n), q)
        lwe = rand_q(g, (batch, n_lwe + 1), q)
        lwe[0, 3] = 0  # a zero mask element (skipped)
        want = np.stack([c.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf)
                         for b in range(batch)])
        key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
        o = dev(np.zeros((batch, k * n + 1), np.uint64))
        (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf else
         M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)(dev(lwe), o, dev(lut), key)
        assert np.array_equal(host(o), want), ("pbs", base_log, level)


@pytest.mark.parametrize("name", sorted(PARAMS))
@pytest.mark.parametrize("bnf", [True, False])
def test_shape_pbs_real_keys(engine, oracle, name, bnf):
    """Real keys at the shortint shape (key converted on the GPU: Raw for BNF, Normalize for the Solinas
    modulus): decrypt(PBS(Enc(m))) == f(m) for every message of the padded space; two outputs == the oracle."""
    n, k, n_lwe, base_log, level, lwe_noise, glwe_noise, msg_mod = PARAMS[name]
    q = 0 if bnf else P
    g = H.rng(hash((name, bnf)) & 0xFFFFFFFF)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen_fast(g, oracle, lwe_sk, glwe_sk, base_log, level, glwe_noise, q)
    delta = (1 << 63) // msg_mod if bnf else (P // 2) // msg_mod
    f = lambda x: (3 * x + 1) % msg_mod
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
    nbsk = host(gkey)
    key = M.NttBootstrapKey(pl, gkey, base_log, level, M.BNF if bnf else M.SOLINAS)
    out = dev(np.zeros((msg_mod, k * n + 1), np.uint64))
    (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf else
     M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)(dev(lwe), out, dev(lut), key)
    got = host(out)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for i, m in enumerate(msgs):
        pt = H.lwe_decrypt(got[i], out_sk, q)
        assert H.decode(pt, delta, msg_mod, q) % msg_mod == f(int(m)), (name, int(m), pt)
    ctx = oracle.NttContext(n)
    idx = [0, msg_mod - 1]
    if bnf:
        want = ctx.pbs_batch_bnf(lwe[idx], lut.reshape(-1), nbsk.reshape(-1), k, base_log, level, threads=2)
    else:
        want = ctx.pbs_batch_solinas(lwe[idx], lut.reshape(-1), nbsk.reshape(-1), k, base_log, level, threads=2)
    assert np.array_equal(got[idx], want)
