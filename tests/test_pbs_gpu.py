"""GPU parity of the fused external-product / CMUX / PBS kernels against the CPU oracle (`-m gpu`).

Bar: bit-exact on identical inputs.  Random NTT-domain keys exercise every arithmetic path (parity
does not need the key to be an encryption); seeded real keys check the functional property the
reference's own tests assert, decrypt(PBS(Enc(m))) == f(m)
(algorithms/test/lwe_programmable_bootstrapping.rs:708-865 Solinas, :1002-1163 BNF).
"""
import numpy as np
import pytest

import tfhe_helpers as H

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001
N = 2048
K = 1


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def rand_q(g, shape, q):
    return H.uniform_u64(g, shape) if not q else g.integers(0, q, size=shape, dtype=np.uint64)


@pytest.fixture(scope="module")
def plan(engine):
    return engine.Plan.try_new(N, P)


@pytest.fixture(scope="module")
def ctx(oracle):
    return oracle.NttContext(N)


@pytest.mark.parametrize("width,normalize", [(64, False), (64, True), (0, True), (0, False), (40, False)])
def test_bsk_conversion(engine, plan, ctx, width, normalize):
    g = H.rng(100 + width + normalize)
    polys = 3 * 4 * 2
    src = rand_q(g, (polys, N), 0 if width else P)
    if width and width < 64:  # a 2^w-modulus key lives in the top w bits (ntt64.rs:166-178)
        src = (src >> np.uint64(64 - width)) << np.uint64(64 - width)
    want = ctx.bsk_to_ntt(src.reshape(-1), width, normalize).reshape(polys, N)
    s, d = dev(src), dev(np.zeros_like(src))
    engine.ntt64_pbs.convert_standard_lwe_bootstrap_key_to_ntt64(plan, s, d, normalize, width or None)
    assert np.array_equal(host(d), want)


@pytest.mark.parametrize("bnf", [True, False])
@pytest.mark.parametrize("base_log,level", [(23, 1), (12, 2), (7, 3), (1, 1), (21, 3), (31, 1)])
def test_external_product_parity(engine, plan, ctx, bnf, base_log, level):
    """BNF level 1 (base_log <= 31) runs on the twisted-transform kernel (pbs_tw.hip), the other
    shapes on the generic one (pbs_kernels.hip)."""
    q = 0 if bnf else P
    g = H.rng(base_log * 10 + level + 1000 * bnf)
    batch = 6
    ggsw = rand_q(g, (level, K + 1, K + 1, N), P)
    glwe = rand_q(g, (batch, K + 1, N), q)
    glwe[0, 0, :8] = 0  # edge values the decomposition must carry exactly
    glwe[0, 1, :4] = np.array([q - 1 if q else 2**64 - 1, 1, (q or 2**64) // 2, (q or 2**64) // 2 + 1], np.uint64)
    out0 = rand_q(g, (batch, K + 1, N), q)
    want = np.stack([ctx.ext_product(out0[b].reshape(-1), ggsw.reshape(-1), glwe[b].reshape(-1), K, base_log,
                                     level, bnf=bnf).reshape(K + 1, N) for b in range(batch)])
    out, tg, tk = dev(out0), dev(glwe), dev(ggsw)
    fn = (engine.ntt64_pbs.add_external_product_ntt64_bnf_assign if bnf
          else engine.ntt64_pbs.add_external_product_ntt64_assign)
    fn(plan, out, tk, tg, base_log, level)
    assert np.array_equal(host(out), want)
    assert np.array_equal(host(tg), glwe)  # input untouched


@pytest.mark.parametrize("bnf", [True, False])
def test_cmux_parity(engine, plan, ctx, bnf):
    q = 0 if bnf else P
    g = H.rng(7 + bnf)
    batch, base_log, level = 5, 23, 1
    ggsw = rand_q(g, (level, K + 1, K + 1, N), P)
    ct0, ct1 = rand_q(g, (batch, K + 1, N), q), rand_q(g, (batch, K + 1, N), q)
    want0 = np.stack([ctx.cmux(ct0[b].reshape(-1), ct1[b].reshape(-1), ggsw.reshape(-1), K, base_log, level,
                               bnf=bnf).reshape(K + 1, N) for b in range(batch)])
    want1 = H.sub_q(ct1, ct0, q)
    t0, t1 = dev(ct0), dev(ct1)
    fn = engine.ntt64_pbs.cmux_ntt64_bnf_assign if bnf else engine.ntt64_pbs.cmux_ntt64_assign
    fn(plan, t0, t1, dev(ggsw), base_log, level)
    assert np.array_equal(host(t0), want0)
    assert np.array_equal(host(t1), want1)


def _pbs_inputs(g, batch, n_lwe, q):
    lwe = rand_q(g, (batch, n_lwe + 1), q)
    # mask entries the blind rotation must skip (BNF: modulus-switch to 0; Solinas: raw 0)
    lwe[:, ::7] = 0
    if not q:
        lwe[:, 3::11] = g.integers(0, 1 << 50, size=lwe[:, 3::11].shape, dtype=np.uint64)
        lwe[:, 5::13] = np.uint64(2**64 - (1 << 50))
    lwe[0, -1] = 0
    return lwe


@pytest.mark.parametrize("bnf,centered", [(True, False), (True, True), (False, False)])
@pytest.mark.parametrize("level,base_log", [(1, 23), (2, 15), (1, 1), (1, 31)])
def test_pbs_parity_random_key(engine, plan, ctx, oracle, bnf, centered, level, base_log):
    q = 0 if bnf else P
    g = H.rng(31 + 2 * bnf + centered + 10 * level)
    n_lwe, batch = 40, 7
    bsk = rand_q(g, (n_lwe, level, K + 1, K + 1, N), P)
    lut = rand_q(g, (K + 1, N), q)
    lwe = _pbs_inputs(g, batch, n_lwe, q)
    want = np.stack([ctx.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), K, base_log, level, bnf=bnf,
                             centered=centered) for b in range(batch)])
    M = engine.ntt64_pbs
    key = M.NttBootstrapKey(plan, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
    out = dev(np.zeros((batch, K * N + 1), np.uint64))
    if bnf:
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(
            dev(lwe), out, dev(lut), key, M.MS_CENTERED if centered else M.MS_STANDARD)
    else:
        M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    assert np.array_equal(host(out), want)


def test_pbs_parity_config4_shape(engine, plan, ctx):
    """PARAM_MESSAGE_2_CARRY_2 shape (n = 918, beta = 2^23, l = 1, BNF) on a random key, vs the
    multi-threaded oracle (twisted-transform kernel, pbs_tw.hip)."""
    g = H.rng(918)
    n_lwe, batch, base_log, level = 918, 48, 23, 1
    bsk = rand_q(g, (n_lwe, level, K + 1, K + 1, N), P)
    lut = H.uniform_u64(g, (K + 1, N))
    lwe = _pbs_inputs(g, batch, n_lwe, 0)
    want = ctx.pbs_batch_bnf(lwe, lut.reshape(-1), bsk.reshape(-1), K, base_log, level, threads=16)
    M = engine.ntt64_pbs
    key = M.NttBootstrapKey(plan, dev(bsk), base_log, level, M.BNF)
    out = dev(np.zeros((batch, K * N + 1), np.uint64))
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    assert np.array_equal(host(out), want)


@pytest.mark.parametrize("bnf", [True, False])
def test_pbs_functional_real_keys(engine, plan, ctx, bnf):
    """Seeded real keys: GPU PBS == oracle PBS bit for bit, and decrypts to f(m) for every m."""
    n_lwe, base_log, level = 64, 23, 1
    q = 0 if bnf else P
    msg_mod = 4
    mod = q if q else 2**64
    delta = (1 << 63) // msg_mod
    g = H.rng(500 + bnf)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (K, N))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17 if bnf else 12, q)
    nbsk = ctx.bsk_to_ntt(bsk.reshape(-1), 64 if bnf else 0, normalize=not bnf).reshape(n_lwe, level, K + 1, K + 1, N)
    f = lambda x: (3 * x + 1) % msg_mod
    lut = H.pbs_lut(N, K, msg_mod, delta, f, q)
    msgs = list(range(msg_mod)) * 2
    lwe = np.stack([H.lwe_encrypt(g, (m * delta) % mod, lwe_sk, 30 if bnf else 20, q) for m in msgs])
    M = engine.ntt64_pbs
    # the key conversion itself runs on the GPU too
    gkey = dev(np.zeros_like(bsk))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, dev(bsk), gkey, normalize=not bnf,
                                                  input_modulus_width=64 if bnf else None)
    assert np.array_equal(host(gkey), nbsk)
    key = M.NttBootstrapKey(plan, gkey, base_log, level, M.BNF if bnf else M.SOLINAS)
    out = dev(np.zeros((len(msgs), K * N + 1), np.uint64))
    if bnf:
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    else:
        M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for i, m in enumerate(msgs):
        assert np.array_equal(got[i], ctx.pbs(lwe[i], lut.reshape(-1), nbsk.reshape(-1), K, base_log, level, bnf=bnf))
        assert H.decode(H.lwe_decrypt(got[i], out_sk, q), delta, msg_mod, q) == f(m)


def test_pbs_errors(engine, plan):
    import torch
    M = engine.ntt64_pbs
    small = engine.Plan.try_new(256, P)
    bsk = torch.zeros((4, 1, 2, 2, 256), dtype=torch.int64, device="cuda")
    with pytest.raises(engine.MiError) as e:
        M.NttBootstrapKey(small, bsk, 23, 1, M.BNF)
    assert e.value.status == 6  # MI_ERR_UNSUPPORTED (N = 256: below the compiled shapes)
    with pytest.raises(engine.MiError) as e:
        M.NttBootstrapKey(plan, torch.zeros((2, 1, 4, 4, N), dtype=torch.int64, device="cuda"), 10, 1, M.BNF)
    assert e.value.status == 6  # k = 3
    with pytest.raises(engine.MiError) as e:
        M.NttBootstrapKey(plan, torch.zeros((2, 4, 2, 2, N), dtype=torch.int64, device="cuda"), 16, 4, M.BNF)
    assert e.value.status == 1  # base_log * level = 64: SignedDecomposer::new's assertion
    bsk = torch.zeros((4, 1, 2, 2, N), dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError):
        M.NttBootstrapKey(plan, bsk, 23, 2, M.BNF)  # shape / level mismatch
    key = M.NttBootstrapKey(plan, bsk, 23, 1, M.SOLINAS)
    lwe = torch.zeros((2, 5), dtype=torch.int64, device="cuda")
    out = torch.zeros((2, N + 1), dtype=torch.int64, device="cuda")
    lut = torch.zeros((2, N), dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError):  # variant mismatch
        M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(lwe, out, lut, key)
    M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(lwe[:0], out[:0], lut, key)  # empty batch
    with pytest.raises(ValueError):
        M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(lwe[:, :4], out, lut, key)


@pytest.mark.parametrize("bnf", [True, False])
def test_pbs_pre_switched(engine, plan, ctx, oracle, bnf):
    """MS_PRE_SWITCHED: lwe_in holds modulus-switched values (the ModulusSwitchedLweCiphertext input
    of blind_rotate_ntt64[_bnf]_assign_mem_optimized); the result equals the standard path on the raw
    ciphertexts and the oracle."""
    q = 0 if bnf else P
    g = H.rng(77 + bnf)
    n_lwe, batch, base_log, level = 30, 5, 23, 1
    bsk = rand_q(g, (n_lwe, level, K + 1, K + 1, N), P)
    lut = rand_q(g, (K + 1, N), q)
    lwe = _pbs_inputs(g, batch, n_lwe, q)
    if bnf:
        msed = np.vectorize(lambda x: oracle.modulus_switch(int(x), 12), otypes=[np.uint64])(lwe)
    else:
        msed = np.vectorize(lambda x: oracle.pbs_modulus_switch_non_native(int(x), N, P), otypes=[np.uint64])(lwe)
    want = np.stack([ctx.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), K, base_log, level, bnf=bnf)
                     for b in range(batch)])
    M = engine.ntt64_pbs
    key = M.NttBootstrapKey(plan, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
    out = dev(np.zeros((batch, K * N + 1), np.uint64))
    fn = (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf
          else M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)
    fn(dev(msed), out, dev(lut), key, M.MS_PRE_SWITCHED)
    assert np.array_equal(host(out), want)


def _fast_bsk_solinas(oracle, g, lwe_sk, glwe_sk, base_log, noise_log2):
    """H.bsk_gen for q = p with the GLWE mask products through the oracle's NTT (exact mod (X^N + 1, p)):
    GGSW rows as ggsw_encryption.rs:20-45, level 1, k = 1.  Test infrastructure only."""
    n_lwe, n = lwe_sk.size, glwe_sk.shape[1]
    plan = oracle.Plan.try_new(n, P)
    masks = g.integers(0, P, size=(n_lwe * 2, n), dtype=np.uint64)
    s_hat = plan.fwd(glwe_sk[0].astype(np.uint64))
    prod = plan.inv(plan.mul_assign_normalize(plan.fwd(masks, threads=16), np.broadcast_to(s_hat, masks.shape).copy()),
                    threads=16)
    bsk = np.zeros((n_lwe, 1, 2, 2, n), np.uint64)
    factor0 = pow(2, 64 - base_log, P)
    s_obj = glwe_sk[0].astype(object)
    for i, b in enumerate(lwe_sk):
        factor = (-int(b) * factor0) % P
        for r in range(2):
            body = prod[2 * i + r].astype(object)
            if r == 0:
                body = body + s_obj * factor
            else:
                body[0] = body[0] + (-factor) % P
            e = H.noise_q(g, n, noise_log2, P).astype(object)
            bsk[i, 0, r, 0] = masks[2 * i + r]
            bsk[i, 0, r, 1] = np.array((body + e) % P, dtype=np.uint64)
    return bsk


def test_pbs_solinas_reference_params(engine, plan, ctx, oracle):
    """The reference's own Solinas PBS test shape, TEST_PARAMS_3_BITS_SOLINAS_U64 (algorithms/test/mod.rs:106-128:
    n = 742, N = 2048, B = 2^23, l = 1, 3-bit messages, q = p) with the property of
    lwe_encrypt_pbs_ntt64_decrypt_custom_mod (lwe_programmable_bootstrapping.rs:708-865): decrypt(PBS(Enc(m)))
    decodes to f(m) = m mod 8 for every m; plus the GPU output equals the oracle PBS bit for bit.  Real keys
    (uniform noise at the reference's standard deviations: 2^46 LWE, 2^12 GLWE), the key converted Normalize on
    the GPU; runs on the twisted Solinas engine (pbs_tw.hip)."""
    n_lwe, base_log, level, msg_mod = 742, 23, 1, 8
    delta = (P // 2) // msg_mod  # get_encoding_with_padding(custom) = q / 2
    g = H.rng(742)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (K, N))
    bsk = _fast_bsk_solinas(oracle, g, lwe_sk, glwe_sk, base_log, 12)
    f = lambda x: x % msg_mod
    lut = H.pbs_lut(N, K, msg_mod, delta, f, P)
    msgs = list(range(msg_mod)) * 2
    lwe = np.stack([H.lwe_encrypt(g, (m * delta) % P, lwe_sk, 46, P) for m in msgs])
    M = engine.ntt64_pbs
    gkey = dev(np.zeros_like(bsk))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, dev(bsk), gkey, normalize=True, input_modulus_width=None)
    nbsk = host(gkey)
    key = M.NttBootstrapKey(plan, gkey, base_log, level, M.SOLINAS)
    out = dev(np.zeros((len(msgs), K * N + 1), np.uint64))
    M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for i, m in enumerate(msgs):
        pt = H.lwe_decrypt(got[i], out_sk, P)
        assert H.decode(pt, delta, msg_mod, P) % msg_mod == f(m), (m, pt)
    want = np.stack([ctx.pbs(lwe[i], lut.reshape(-1), nbsk.reshape(-1), K, base_log, level, bnf=False)
                     for i in range(4)])
    assert np.array_equal(got[:4], want)


def test_pbs_config4_full_batch_real_keys(engine, plan, ctx, oracle):
    """Config 4 at its full size: 4096 BNF PBS at the PARAM_MESSAGE_2_CARRY_2 shape (n = 918, N = 2048,
    B = 2^23, l = 1, 2+2-bit messages with padding, TUniform noise bounds 2^45 LWE / 2^17 GLWE as ks_pbs.rs:29-47)
    under real keys, key converted on the GPU.  Size-independent property over the whole batch: every output
    decrypts to f(m) (lwe_programmable_bootstrapping.rs:1002-1163); bit-exact vs the oracle on ALL 4096 outputs
    (the oracle's blind rotation with its AVX-512 transform restatement, itself checked equal to the scalar
    restatement on 8 of them first)."""
    n_lwe, base_log, level, msg_mod, batch = 918, 23, 1, 16, 4096
    delta = (1 << 63) // msg_mod
    g = H.rng(4096918)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (K, N))
    bsk = H.bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, 17)
    f = lambda x: (5 * x + 3) % msg_mod
    lut = H.pbs_lut(N, K, msg_mod, delta, f)
    msgs = np.arange(batch) % msg_mod
    lwe = H.lwe_encrypt_batch(g, (msgs.astype(np.uint64) * np.uint64(delta)), lwe_sk, 45)
    M = engine.ntt64_pbs
    gkey = dev(np.zeros_like(bsk))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(plan, dev(bsk), gkey, normalize=False, input_modulus_width=64)
    nbsk = host(gkey)
    assert np.array_equal(nbsk[:3].reshape(-1), ctx.bsk_to_ntt(bsk[:3].reshape(-1), 64, normalize=False))
    key = M.NttBootstrapKey(plan, gkey, base_log, level, M.BNF)
    out = dev(np.zeros((batch, K * N + 1), np.uint64))
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    pts = H.lwe_decrypt_batch(got, H.glwe_sk_as_lwe_sk(glwe_sk))
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert np.array_equal(dec, np.array([f(int(m)) for m in msgs], np.uint64))
    idx = np.array([0, 1, 511, 1024, 2047, 2048, 3071, batch - 1])
    scalar = ctx.pbs_batch_bnf(lwe[idx], lut.reshape(-1), nbsk.reshape(-1), K, base_log, level, threads=8)
    assert np.array_equal(got[idx], scalar)
    oracle.pbs_set_fast_ntt(True)
    try:
        fast8 = ctx.pbs_batch_bnf(lwe[idx], lut.reshape(-1), nbsk.reshape(-1), K, base_log, level, threads=8)
        assert np.array_equal(fast8, scalar)
        want = ctx.pbs_batch_bnf(lwe, lut.reshape(-1), nbsk.reshape(-1), K, base_log, level, threads=16)
    finally:
        oracle.pbs_set_fast_ntt(False)
    assert np.array_equal(got, want)


def test_external_product_config3_full_batch(engine, plan, ctx):
    """Config 3 at its full size: 8192 BNF external products (N = 2048, k = 1, B = 2^23, l = 1) against one shared
    GGSW, the bench's workload, bit-exact vs the oracle on every product; then the same batch as CMUX."""
    batch, base_log, level = 8192, 23, 1
    g = H.rng(8192 + 3)
    ggsw = rand_q(g, (level, K + 1, K + 1, N), P)
    glwe = rand_q(g, (batch, K + 1, N), 0)
    out0 = rand_q(g, (batch, K + 1, N), 0)
    want = ctx.ext_product_batch_bnf(out0.reshape(-1), ggsw.reshape(-1), glwe.reshape(-1), K, base_log, level,
                                     threads=16).reshape(batch, K + 1, N)
    out, tg = dev(out0), dev(glwe)
    engine.ntt64_pbs.add_external_product_ntt64_bnf_assign(plan, out, dev(ggsw), tg, base_log, level)
    assert np.array_equal(host(out), want)
    t0, t1 = dev(out0), dev(glwe)
    engine.ntt64_pbs.cmux_ntt64_bnf_assign(plan, t0, t1, dev(ggsw), base_log, level)
    with np.errstate(over="ignore"):
        diff = glwe - out0
    assert np.array_equal(host(t1), diff)
    want_c = ctx.ext_product_batch_bnf(out0.reshape(-1), ggsw.reshape(-1), diff.reshape(-1), K, base_log, level,
                                       threads=16).reshape(batch, K + 1, N)
    assert np.array_equal(host(t0), want_c)


@pytest.mark.parametrize("batch", [1, 37])
def test_pbs_solinas_config4_shape(engine, plan, ctx, batch):
    """Solinas-modulus PBS at the PARAM_MESSAGE_2_CARRY_2 shape (n = 918, B = 2^23, l = 1) on a random key
    (the reference's NTT PBS bench shape, pbs_bench.rs:646-905), vs the oracle; masks hit 0 (skipped)
    and values that switch to 2N."""
    g = H.rng(9180 + batch)
    n_lwe, base_log, level = 918, 23, 1
    bsk = rand_q(g, (n_lwe, level, K + 1, K + 1, N), P)
    lut = rand_q(g, (K + 1, N), P)
    lwe = _pbs_inputs(g, batch, n_lwe, P)
    lwe[:, 9::17] = np.uint64(P - 1)
    M = engine.ntt64_pbs
    key = M.NttBootstrapKey(plan, dev(bsk), base_log, level, M.SOLINAS)
    out = dev(np.zeros((batch, K * N + 1), np.uint64))
    M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    for b in range(min(batch, 3)):
        want = ctx.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), K, base_log, level, bnf=False)
        assert np.array_equal(got[b], want)


def test_pbs_solinas_config4_full_batch(engine, plan, ctx, oracle):
    """The Solinas-modulus PBS (ntt64_pbs.rs:482-538, the reference's own NTT-PBS bench shape, pbs_bench.rs:646-905) at
    config 4's full batch: 4096 PBS at n = 918, B = 2^23, l = 1 on a random key, bit-exact vs the oracle on ALL 4096
    outputs — the oracle's Solinas PBS with its AVX-512 transform restatement, itself checked equal
    to the scalar restatement on 8 of them first."""
    g = H.rng(4096 + 918 + 1)
    n_lwe, base_log, level, batch = 918, 23, 1, 4096
    bsk = rand_q(g, (n_lwe, level, K + 1, K + 1, N), P)
    lut = rand_q(g, (K + 1, N), P)
    lwe = _pbs_inputs(g, batch, n_lwe, P)
    lwe[:, 9::17] = np.uint64(P - 1)
    M = engine.ntt64_pbs
    key = M.NttBootstrapKey(plan, dev(bsk), base_log, level, M.SOLINAS)
    out = dev(np.zeros((batch, K * N + 1), np.uint64))
    M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    idx = np.array([0, 1, 511, 1024, 2047, 2048, 3071, batch - 1])
    scalar = ctx.pbs_batch_solinas(lwe[idx], lut.reshape(-1), bsk.reshape(-1), K, base_log, level, threads=8)
    assert np.array_equal(got[idx], scalar)
    oracle.pbs_set_fast_ntt(True)
    try:
        fast8 = ctx.pbs_batch_solinas(lwe[idx], lut.reshape(-1), bsk.reshape(-1), K, base_log, level, threads=8)
        assert np.array_equal(fast8, scalar)
        want = ctx.pbs_batch_solinas(lwe, lut.reshape(-1), bsk.reshape(-1), K, base_log, level, threads=16)
    finally:
        oracle.pbs_set_fast_ntt(False)
    assert np.array_equal(got, want)


SHAPES = [(1024, 1), (1024, 2), (2048, 2), (4096, 1), (4096, 2)]


@pytest.mark.parametrize("n,k", SHAPES)
@pytest.mark.parametrize("bnf", [True, False])
def test_generic_shapes_ext_product_cmux(engine, oracle, n, k, bnf):
    """External product and CMUX for N in {1024, 4096} and GLWE dimension k = 2 (the reference's
    shape-generic ntt64_bnf_pbs.rs:541-681 / ntt64_pbs.rs:553-663), levels 1 and 2, vs the oracle."""
    q = 0 if bnf else P
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    for base_log, level in ((23, 1), (12, 2)):
        g = H.rng(n + 10 * k + base_log + bnf)
        batch = 3
        ggsw = rand_q(g, (level, k + 1, k + 1, n), P)
        glwe = rand_q(g, (batch, k + 1, n), q)
        out0 = rand_q(g, (batch, k + 1, n), q)
        want = np.stack([c.ext_product(out0[b].reshape(-1), ggsw.reshape(-1), glwe[b].reshape(-1), k, base_log,
                                       level, bnf=bnf).reshape(k + 1, n) for b in range(batch)])
        out = dev(out0)
        fn = M.add_external_product_ntt64_bnf_assign if bnf else M.add_external_product_ntt64_assign
        fn(pl, out, dev(ggsw), dev(glwe), base_log, level)
        assert np.array_equal(host(out), want), (base_log, level)
        t0, t1 = dev(out0), dev(glwe)
        fn = M.cmux_ntt64_bnf_assign if bnf else M.cmux_ntt64_assign
        fn(pl, t0, t1, dev(ggsw), base_log, level)
        want0 = np.stack([c.cmux(out0[b].reshape(-1), glwe[b].reshape(-1), ggsw.reshape(-1), k, base_log, level,
                                 bnf=bnf).reshape(k + 1, n) for b in range(batch)])
        assert np.array_equal(host(t0), want0)


@pytest.mark.parametrize("n,k", SHAPES)
@pytest.mark.parametrize("bnf", [True, False])
def test_generic_shapes_pbs(engine, oracle, n, k, bnf):
    """PBS for N in {1024, 4096}, k = 2, levels 1 / 3 on random keys vs the oracle (incl. the key
    conversion of the same shape on the GPU)."""
    q = 0 if bnf else P
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    for base_log, level in ((23, 1), (7, 3)):
        g = H.rng(7 * n + k + level + bnf)
        n_lwe, batch = 12, 3
        bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
        lut = rand_q(g, (k + 1, n), q)
        lwe = _pbs_inputs(g, batch, n_lwe, q)
        want = np.stack([c.pbs(lwe[b], lut.reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf)
                         for b in range(batch)])
        key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
        out = dev(np.zeros((batch, k * n + 1), np.uint64))
        fn = (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf
              else M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)
        fn(dev(lwe), out, dev(lut), key)
        assert np.array_equal(host(out), want), (base_log, level)
    # key conversion of this shape
    polys = 2 * (k + 1) ** 2
    src = rand_q(g, (polys, n), 0 if bnf else P)
    want = c.bsk_to_ntt(src.reshape(-1), 64 if bnf else 0, not bnf).reshape(polys, n)
    d = dev(np.zeros_like(src))
    M.convert_standard_lwe_bootstrap_key_to_ntt64(pl, dev(src), d, not bnf, 64 if bnf else None)
    assert np.array_equal(host(d), want)


def test_pbs_functional_k2_real_keys(engine, oracle):
    """A real-key BNF PBS at GLWE dimension 2, N = 1024: GPU == oracle bit for bit and decrypts to f(m)."""
    n, k, n_lwe, base_log, level, msg_mod = 1024, 2, 48, 23, 1, 4
    delta = (1 << 63) // msg_mod
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    g = H.rng(2024)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17, 0)
    nbsk = c.bsk_to_ntt(bsk.reshape(-1), 64, normalize=False).reshape(bsk.shape)
    f = lambda x: (x + 1) % msg_mod
    lut = H.pbs_lut(n, k, msg_mod, delta, f, 0)
    msgs = list(range(msg_mod))
    lwe = np.stack([H.lwe_encrypt(g, m * delta, lwe_sk, 30, 0) for m in msgs])
    M = engine.ntt64_pbs
    key = M.NttBootstrapKey(pl, dev(nbsk), base_log, level, M.BNF)
    out = dev(np.zeros((len(msgs), k * n + 1), np.uint64))
    M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized(dev(lwe), out, dev(lut), key)
    got = host(out)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for i, m in enumerate(msgs):
        assert np.array_equal(got[i], c.pbs(lwe[i], lut.reshape(-1), nbsk.reshape(-1), k, base_log, level))
        assert H.decode(H.lwe_decrypt(got[i], out_sk, 0), delta, msg_mod, 0) % msg_mod == f(m)


@pytest.mark.parametrize("bnf", [True, False])
@pytest.mark.parametrize("n,k,base_log,level", [(2048, 1, 23, 1), (2048, 1, 12, 2), (1024, 2, 23, 1)])
def test_indexed_ggsw_ext_product_and_cmux(engine, oracle, bnf, n, k, base_log, level):
    """One GGSW per item ("one shared GGSW or a per-item GGSW index array"): item b uses
    ggsw_list[index[b]], on the twisted kernel (BNF/Solinas level 1, N 2048, k 1) and the generic one; an index
    past the list leaves the item (both GLWEs) untouched.  Oracle per item."""
    import torch
    q = 0 if bnf else P
    g = H.rng(5000 + n + 10 * k + level + bnf)
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    n_ggsw, batch = 3, 7
    ggsw = rand_q(g, (n_ggsw, level, k + 1, k + 1, n), P)
    idx = np.array([2, 0, 1, 1, 7, 0, 2], np.int32)       # item 4: out of range
    glwe = rand_q(g, (batch, k + 1, n), q)
    out0 = rand_q(g, (batch, k + 1, n), q)
    want = out0.copy()
    want0, want1 = out0.copy(), glwe.copy()
    for b in range(batch):
        if idx[b] >= n_ggsw:
            continue
        gg = ggsw[idx[b]].reshape(-1)
        want[b] = c.ext_product(out0[b].reshape(-1), gg, glwe[b].reshape(-1), k, base_log, level,
                                bnf=bnf).reshape(k + 1, n)
        want0[b] = c.cmux(out0[b].reshape(-1), glwe[b].reshape(-1), gg, k, base_log, level, bnf=bnf).reshape(k + 1, n)
        want1[b] = H.sub_q(glwe[b], out0[b], q)
    tidx = torch.from_numpy(idx).cuda()
    out, tg = dev(out0), dev(glwe)
    fn = M.add_external_product_ntt64_bnf_assign if bnf else M.add_external_product_ntt64_assign
    fn(pl, out, dev(ggsw), tg, base_log, level, ggsw_index=tidx)
    assert np.array_equal(host(out), want)
    assert np.array_equal(host(tg), glwe)
    t0, t1 = dev(out0), dev(glwe)
    fn = M.cmux_ntt64_bnf_assign if bnf else M.cmux_ntt64_assign
    fn(pl, t0, t1, dev(ggsw), base_log, level, ggsw_index=tidx)
    assert np.array_equal(host(t0), want0)
    assert np.array_equal(host(t1), want1)
    with pytest.raises(ValueError):
        fn(pl, t0, t1, dev(ggsw), base_log, level, ggsw_index=tidx[:3])


@pytest.mark.parametrize("bnf", [True, False])
@pytest.mark.parametrize("n,k,base_log,level", [(2048, 1, 23, 1), (2048, 1, 12, 2), (1024, 2, 23, 1), (16384, 1, 23, 1)])
def test_prepared_ggsw_list(engine, oracle, bnf, n, k, base_log, level):
    """NttGgswList (mi_ntt64_ggsw_create: the twisted-shape list permuted once into a private copy, other shapes
    referenced): the external product and CMUX through it equal the raw-pointer calls and the oracle, shared and
    indexed; the prepared copy survives the caller's tensor being overwritten."""
    import torch
    q = 0 if bnf else P
    g = H.rng(6100 + n + k + level + bnf)
    pl = engine.Plan.try_new(n, P)
    c = oracle.NttContext(n)
    M = engine.ntt64_pbs
    n_ggsw, batch = 3, 5
    ggsw = rand_q(g, (n_ggsw, level, k + 1, k + 1, n), P)
    idx = np.array([1, 2, 0, 5, 1], np.int32)
    glwe = rand_q(g, (batch, k + 1, n), q)
    out0 = rand_q(g, (batch, k + 1, n), q)
    tg = dev(ggsw)
    pg = M.NttGgswList(pl, tg, base_log, level, M.BNF if bnf else M.SOLINAS)
    twisted = (n, k, level) == (2048, 1, 1)
    if twisted:
        tg.zero_()  # the prepared copy is private on the fused shape
    ext = M.add_external_product_ntt64_bnf_assign if bnf else M.add_external_product_ntt64_assign
    cm = M.cmux_ntt64_bnf_assign if bnf else M.cmux_ntt64_assign
    out = dev(out0)
    ext(pl, out, pg, dev(glwe), base_log, level)  # shared: GGSW 0
    want = np.stack([c.ext_product(out0[b].reshape(-1), ggsw[0].reshape(-1), glwe[b].reshape(-1), k, base_log, level,
                                   bnf=bnf).reshape(k + 1, n) for b in range(batch)])
    assert np.array_equal(host(out), want)
    t0, t1 = dev(out0), dev(glwe)
    cm(pl, t0, t1, pg, base_log, level, ggsw_index=torch.from_numpy(idx).cuda())
    want0 = out0.copy()
    for b in range(batch):
        if idx[b] < n_ggsw:
            want0[b] = c.cmux(out0[b].reshape(-1), glwe[b].reshape(-1), ggsw[idx[b]].reshape(-1), k, base_log, level,
                              bnf=bnf).reshape(k + 1, n)
    assert np.array_equal(host(t0), want0)
    with pytest.raises(ValueError):  # the list was made for another decomposition
        ext(pl, out, pg, dev(glwe), base_log + 1, level)
