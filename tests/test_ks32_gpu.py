"""GPU parity of the KS32 path (`-m gpu`): the keyswitch with a scalar change and the u32 modulus switch that put a
u64 LWE in front of the NTT blind rotation in the HPU KS32 parameter sets, and that whole bootstrap under real keys.

Reference paths (relative to /root/reference):
  keyswitch_lwe_ciphertext_with_scalar_change      tfhe/src/core_crypto/algorithms/lwe_keyswitch.rs:331-447
  lwe_ciphertext_centered_binary_modulus_switch    tfhe/src/core_crypto/algorithms/modulus_switch.rs:35-104
  V1_5_HPU_PARAM_MESSAGE_2_CARRY_2_KS32_PBS_TUNIFORM_2M128   tfhe/src/shortint/parameters/v1_5/hpu.rs:57-76
  the HPU bootstrap (KS32 -> centered switch -> blind_rotate_ntt64_bnf_assign -> many-LUT extraction)
                                                   mockups/tfhe-hpu-mockup/src/lib.rs:720-761
Bar: bit-exact against the oracle (ks_oracle.c, itself pinned by tests/test_ks32_oracle.py) and every bootstrapped
sample decrypting to its function's value.
"""
import numpy as np
import pytest

import tfhe_helpers as H
from test_blind_rotate_gpu import many_lut_accumulator

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001
M32 = 2**32


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def dev32(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def host32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("in_dim,out_dim,base_log,level,w,batch", [
    (2048, 879, 2, 8, 21, 96),     # the HPU KS32 shape, 2M128 (level 8)
    (2048, 879, 2, 7, 21, 40),     # the 2M64 set (hpu.rs:36-53: level 7)
    (100, 37, 4, 4, 32, 300),      # native u32 output, several GEMM row groups
    (64, 17, 16, 2, 32, 5),        # two-byte digits
    (9, 3, 1, 1, 1, 3),            # one-bit output modulus
])
def test_ks32_parity(engine, oracle, in_dim, out_dim, base_log, level, w, batch):
    KS = engine.lwe_keyswitch
    g = H.rng(in_dim + out_dim * 3 + base_log * 7 + level + w)
    ksk = g.integers(0, M32, size=(in_dim, level, out_dim + 1), dtype=np.uint64).astype(np.uint32)
    if w < 32 and in_dim > 1000:  # a key of the 2^w modulus (MSB encoding), as generate_lwe_keyswitch_key makes it
        ksk = (ksk >> np.uint32(32 - w)) << np.uint32(32 - w)
    lwe = H.uniform_u64(g, (batch, in_dim + 1))
    lwe[0, :4] = [0, 2**64 - 1, 1 << 63, (1 << 63) - 1]
    step = 1 << (64 - w)
    lwe[1 % batch, -1] = step // 2        # body rounding corners
    lwe[2 % batch, -1] = step // 2 - 1
    lwe[0, -1] = 2**64 - 1
    want = oracle.lwe_keyswitch32(ksk, lwe, out_dim, base_log, level, w, threads=16)
    key = KS.LweKeyswitchKey32(dev32(ksk), base_log, level, w)
    out = dev32(np.zeros((batch, out_dim + 1), np.uint32))
    KS.keyswitch_lwe_ciphertext_with_scalar_change(key, dev(lwe), out)
    assert np.array_equal(host32(out), want)


@pytest.mark.parametrize("log_mod", [12, 32, 1])
@pytest.mark.parametrize("centered", [False, True])
def test_ms32_parity(engine, oracle, log_mod, centered):
    """The u32 switch (modulus_switch.rs:14-104 at Scalar = u32); the centered form at log_mod = 32 is refused, as the
    reference's half_case shift (:95) underflows there."""
    KS = engine.lwe_keyswitch
    if centered and log_mod == 32:
        with pytest.raises(engine.MiError):
            KS.lwe_ciphertext_modulus_switch32(dev32(np.zeros((2, 9), np.uint32)), dev(np.zeros((2, 9), np.uint64)), 32,
                                               centered=True)
        return
    g = H.rng(log_mod * 3 + centered)
    dim, batch = 879, 257
    lwe = g.integers(0, M32, size=(batch, dim + 1), dtype=np.uint64).astype(np.uint32)
    lwe[1::2] = (lwe[1::2] >> np.uint32(11)) << np.uint32(11)
    lwe[0, :5] = [0, M32 - 1, 1 << 31, (1 << 31) - 1, 1 << 19]
    want = oracle.lwe_ms32(lwe, log_mod, centered)
    out = dev(np.zeros((batch, dim + 1), np.uint64))
    KS.lwe_ciphertext_modulus_switch32(dev32(lwe), out, log_mod, centered)
    assert np.array_equal(host(out), want)


def test_ks32_errors(engine):
    import torch
    KS = engine.lwe_keyswitch
    ksk = torch.zeros((8, 9, 5), dtype=torch.int32, device="cuda")
    with pytest.raises(engine.MiError):   # base_log * level = 36 > 32 (lwe_keyswitch.rs:378-384)
        KS.LweKeyswitchKey32(ksk, 4, 9, 21)
    ksk = torch.zeros((8, 2, 5), dtype=torch.int32, device="cuda")
    with pytest.raises(engine.MiError):
        KS.LweKeyswitchKey32(ksk, 2, 2, 33)
    key = KS.LweKeyswitchKey32(ksk, 2, 2, 21)
    with pytest.raises(ValueError):
        KS.keyswitch_lwe_ciphertext_with_scalar_change(key, torch.zeros((3, 10), dtype=torch.int64, device="cuda"),
                                                       torch.zeros((3, 5), dtype=torch.int32, device="cuda"))


@pytest.mark.parametrize("lut_nb", [1, 2])
def test_ks32_bootstrap_hpu_flow(engine, oracle, lut_nb):
    """The HPU KS32 bootstrap end to end under real keys at V1_5_HPU_PARAM_MESSAGE_2_CARRY_2_KS32_PBS_TUNIFORM_2M128:
    big LWE (N = 2048, the GLWE key flattened) -> KS32 (879, base 2^2, 8 levels, 2^21) -> centered modulus switch to
    2N -> blind_rotate_ntt64_bnf_assign (level 1, base 2^23) on fill_many_lut_accumulator -> lut_nb extractions.
    Every step equals the oracle bit for bit and every sample decrypts to its function of the message."""
    n, k, n_lwe, pbs_base_log, ks_base_log, ks_level, w = 2048, 1, 879, 23, 2, 8, 21
    msg_mod = carry_mod = 4
    functions = [lambda m, j=j: (3 * m + j + 1) % (msg_mod * carry_mod) for j in range(lut_nb)]
    acc0, fn_stride, delta, max_degree = many_lut_accumulator(n, k, msg_mod, carry_mod, functions)
    g = H.rng(7000 + lut_nb)
    glwe_sk = H.binary_key(g, (k, n))
    big_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    small_sk = H.binary_key(g, n_lwe)
    ksk = H.ksk32_gen(g, big_sk, small_sk, ks_base_log, ks_level, noise_log2=2, out_mod_log=w)
    bsk = H.bsk_gen_native_l1(g, small_sk, glwe_sk, pbs_base_log, 17)
    c = oracle.NttContext(n)
    nbsk = c.bsk_to_ntt(bsk.reshape(-1), 64, normalize=False).reshape(bsk.shape)
    msgs = list(range(max_degree + 1)) * 2
    batch = len(msgs)
    cts = H.lwe_encrypt_batch(g, np.array(msgs, np.uint64) * np.uint64(delta), big_sk, noise_log2=20)
    KS, M = engine.lwe_keyswitch, engine.ntt64_pbs
    # 1. KS32
    key32 = KS.LweKeyswitchKey32(dev32(ksk), ks_base_log, ks_level, w)
    small = dev32(np.zeros((batch, n_lwe + 1), np.uint32))
    KS.keyswitch_lwe_ciphertext_with_scalar_change(key32, dev(cts), small)
    want_small = oracle.lwe_keyswitch32(ksk, cts, n_lwe, ks_base_log, ks_level, w, threads=16)
    assert np.array_equal(host32(small), want_small)
    # 2. centered binary modulus switch to log2(2N) = 12 (to_blind_rotation_input_modulus_log)
    switched = dev(np.zeros((batch, n_lwe + 1), np.uint64))
    KS.lwe_ciphertext_centered_binary_modulus_switch32(small, switched, 12)
    want_sw = oracle.lwe_ms32(want_small, 12, True)
    assert np.array_equal(host(switched), want_sw)
    # 3. blind rotation of the many-LUT accumulator, pre-switched input
    accs = np.broadcast_to(acc0, (batch, k + 1, n)).copy()
    oracle.pbs_set_fast_ntt(True)
    try:
        want_glwe = c.blind_rotate_batch(accs, want_sw, nbsk.reshape(-1), k, pbs_base_log, 1, bnf=True, ms_mode=2,
                                         threads=16)
    finally:
        oracle.pbs_set_fast_ntt(False)
    pl = engine.Plan.try_new(n, P)
    key = M.NttBootstrapKey(pl, dev(nbsk), pbs_base_log, 1, M.BNF)
    t = dev(accs)
    M.blind_rotate_ntt64_bnf_assign(switched, t, key, M.MS_PRE_SWITCHED)
    assert np.array_equal(host(t), want_glwe)
    # 4. many-LUT extraction, decryption under the big key
    out = dev(np.zeros((batch, lut_nb, k * n + 1), np.uint64))
    M.extract_lwe_sample_from_glwe_ciphertext(t, out, 0, fn_stride, lut_nb, 0)
    got = host(out)
    for b, m in enumerate(msgs):
        for j in range(lut_nb):
            dec = H.decode(H.lwe_decrypt(got[b, j], big_sk, 0), delta, msg_mod * carry_mod, 0) % (msg_mod * carry_mod)
            assert dec == functions[j](m), (m, j)
