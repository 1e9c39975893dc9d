"""GPU parity of the batched LWE keyswitch (int8 matrix-core path) against the oracle (`-m gpu`).

Bar: bit-exact vs ora_lwe_keyswitch (restating lwe_keyswitch.rs:137-227) on seeded random keys and
ciphertexts — the PARAM_MESSAGE_2_CARRY_2 shape (2048 -> 918, base 2^4, 4 levels), the reference's
doc-test shape (742 -> 2048, base 2^3, 5 levels), odd shapes that exercise every padding path
(K not a multiple of 64, out_dim + 1 not a multiple of 16, batch not a multiple of 64), rounding
corners of the decomposition — plus decryption of real keys, KS then PBS (the shortint KS-PBS order),
and the argument checks.
"""
import numpy as np
import pytest

import tfhe_helpers as H

pytestmark = pytest.mark.gpu


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def run_ks(engine, ksk, lwe, base_log, level):
    import torch
    K = engine.lwe_keyswitch
    key = K.LweKeyswitchKey(dev(ksk), base_log, level)
    out = torch.zeros(lwe.shape[:-1] + (ksk.shape[2],), dtype=torch.int64, device="cuda")
    K.keyswitch_lwe_ciphertext(key, dev(lwe), out)
    return host(out)


@pytest.mark.parametrize("in_dim,out_dim,base_log,level,batch", [
    (2048, 918, 4, 4, 67),      # PARAM_MESSAGE_2_CARRY_2 KS (ks_pbs.rs:38-39), ragged batch
    (742, 2048, 3, 5, 5),       # lwe_keyswitch.rs doc-test shape
    (13, 9, 7, 3, 1),           # K = 39 < 64, out 10 < 16, single ciphertext
    (100, 31, 1, 9, 130),       # base 2, 9 levels; K = 900
    (33, 17, 10, 2, 64),        # digits wider than a signed byte: 2 bytes per digit
    (40, 25, 15, 4, 3),         # 15-bit base: 2 bytes per digit
    (20, 12, 21, 3, 17),        # 21-bit base: 3 bytes per digit
    (512, 300, 4, 4, 520),      # 3 row groups of 256 (last ragged) x 10 column groups of 32
    (48, 40, 4, 4, 300),        # odd number of k blocks (K = 192 -> 3), 2 row groups, padded columns
    (50, 20, 6, 2, 33),         # r6 digit kernel at level 2 (one byte per digit), in_dim not a multiple of 32
    (70, 11, 5, 1, 300),        # ... at level 1, 2 row groups
    (24, 8, 3, 8, 9),           # ... at level 8 (native u64 output)
])
def test_keyswitch_matches_oracle(engine, oracle, in_dim, out_dim, base_log, level, batch):
    g = H.rng(in_dim * 7 + out_dim + base_log)
    ksk = H.uniform_u64(g, (in_dim, level, out_dim + 1))
    lwe = H.uniform_u64(g, (batch, in_dim + 1))
    lwe[0, : min(4, in_dim)] = [0, 2**64 - 1, 1 << 63, (1 << 63) - 1][: min(4, in_dim)]
    got = run_ks(engine, ksk, lwe, base_log, level)
    assert np.array_equal(got, oracle.lwe_keyswitch(ksk, lwe, out_dim, base_log, level))


def test_keyswitch_decrypts_and_feeds_pbs(engine, oracle):
    """KS-PBS at the PARAM_MESSAGE_2_CARRY_2 shape with a small key set: big-key LWE -> keyswitch ->
    BNF PBS -> decrypts to f(m) under the GLWE key (shortint's KS-PBS order)."""
    import torch
    M = engine.ntt64_pbs
    n, k, pbs_bl, pbs_l, ks_bl, ks_l = 2048, 1, 23, 1, 4, 4
    n_small = 64  # small LWE dimension keeps the test's BSK generation cheap; the KS shape is real
    g = H.rng(0x4b53)
    glwe_sk = H.binary_key(g, (k, n))
    big_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    small_sk = H.binary_key(g, n_small)
    ksk = H.ksk_gen(g, big_sk, small_sk, ks_bl, ks_l, noise_log2=12)
    bsk_std = H.bsk_gen(g, small_sk, glwe_sk, pbs_bl, pbs_l, noise_log2=10)
    plan = engine.Plan.try_new(n, engine.SOLINAS_P)
    bsk = torch.empty(bsk_std.shape, dtype=torch.int64, device="cuda")
    M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, dev(bsk_std), bsk, normalize=False)
    key = M.NttBootstrapKey(plan, bsk, pbs_bl, pbs_l, M.BNF)
    msg_mod = 4
    delta = (1 << 63) // msg_mod
    f = lambda x: (3 * x + 1) % msg_mod
    lut = H.pbs_lut(n, k, msg_mod, delta, f)
    msgs = np.arange(8, dtype=np.uint64) % np.uint64(msg_mod)
    cts = H.lwe_encrypt_batch(g, msgs * np.uint64(delta), big_sk, noise_log2=10)
    small = torch.zeros((cts.shape[0], n_small + 1), dtype=torch.int64, device="cuda")
    engine.lwe_keyswitch.keyswitch_lwe_ciphertext(engine.lwe_keyswitch.LweKeyswitchKey(dev(ksk), ks_bl, ks_l),
                                                  dev(cts), small)
    assert np.array_equal(host(small), oracle.lwe_keyswitch(ksk, cts, n_small, ks_bl, ks_l))
    out = torch.zeros((cts.shape[0], k * n + 1), dtype=torch.int64, device="cuda")
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(small, out, dev(lut), key)
    dec = H.lwe_decrypt_batch(host(out), big_sk)
    assert [H.decode(int(d), delta, msg_mod) for d in dec] == [f(int(m)) for m in msgs]


def test_keyswitch_argument_checks(engine):
    import torch
    K = engine.lwe_keyswitch
    ksk = torch.zeros((8, 4, 11), dtype=torch.int64, device="cuda")
    key = K.LweKeyswitchKey(ksk, 4, 4)
    with pytest.raises(ValueError):
        K.keyswitch_lwe_ciphertext(key, torch.zeros((2, 8), dtype=torch.int64, device="cuda"),
                                   torch.zeros((2, 11), dtype=torch.int64, device="cuda"))
    with pytest.raises(ValueError):
        K.keyswitch_lwe_ciphertext(key, torch.zeros((2, 9), dtype=torch.int64, device="cuda"),
                                   torch.zeros((2, 10), dtype=torch.int64, device="cuda"))
    # empty batch is a no-op
    K.keyswitch_lwe_ciphertext(key, torch.zeros((0, 9), dtype=torch.int64, device="cuda"),
                               torch.zeros((0, 11), dtype=torch.int64, device="cuda"))
    with pytest.raises(engine.MiError):  # base_log * level >= 64 (SignedDecomposer::new asserts)
        K.LweKeyswitchKey(torch.zeros((8, 8, 11), dtype=torch.int64, device="cuda"), 8, 8)
    with pytest.raises(engine.MiError):  # GEMM depth 66000 * 2 >= 2^17: beyond exact int32 accumulation
        K.LweKeyswitchKey(torch.zeros((66000, 2, 11), dtype=torch.int64, device="cuda"), 4, 2)
