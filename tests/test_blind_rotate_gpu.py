"""GPU parity of the GLWE-output blind rotation, the per-item-LUT PBS and nth-sample extraction (`-m gpu`).

Reference paths relative to /root/reference/tfhe/src/core_crypto:
  blind_rotate_ntt64_bnf_assign[_mem_optimized]   algorithms/lwe_programmable_bootstrapping/ntt64_bnf_pbs.rs:174-266
  blind_rotate_ntt64_assign[_mem_optimized]       algorithms/lwe_programmable_bootstrapping/ntt64_pbs.rs:176-286
  extract_lwe_sample_from_glwe_ciphertext         algorithms/glwe_sample_extraction.rs:89-160
and their only in-tree many-LUT caller, the HPU mockup (mockups/tfhe-hpu-mockup/src/lib.rs:736-761), whose LUT is
shortint's fill_many_lut_accumulator (shortint/engine/mod.rs:168-248).

Bar: bit-exact against the oracle on identical inputs, on every PBS engine: the fused N = 2048, k = 1, level-1
kernels (pbs_tw.hip), the shape-generic fused kernels (pbs_kernels.hip) and the multi-kernel large-N path
(pbs_large.hip); real keys decrypt every extracted many-LUT sample to its function's value.
"""
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
    return H.uniform_u64(g, shape) if not q else g.integers(0, q, size=shape, dtype=np.uint64)


def lwe_inputs(g, batch, n_lwe, q):
    lwe = rand_q(g, (batch, n_lwe + 1), q)
    lwe[:, ::7] = 0  # mask entries the rotation skips
    if not q:
        lwe[:, 5::13] = np.uint64(2**64 - (1 << 50))  # switches to 2N = 0 mod 2N
    lwe[0, -1] = 0
    return lwe


# (N, k, base_log, level): the fused twisted engine, the generic fused engine (two shapes), the large-N passes
ENGINES = [(2048, 1, 23, 1), (1024, 1, 15, 2), (512, 4, 23, 1), (16384, 1, 23, 1)]
CTX = {}


def ctx_for(oracle, n):
    if n not in CTX:
        CTX[n] = oracle.NttContext(n)
    return CTX[n]


@pytest.mark.parametrize("n,k,base_log,level", ENGINES)
@pytest.mark.parametrize("bnf,ms", [(True, 0), (True, 1), (True, 2), (False, 0), (False, 2)])
def test_blind_rotate_parity(engine, oracle, n, k, base_log, level, bnf, ms):
    """Every item rotates its own accumulator in place; == the oracle's blind_rotate_ntt64[_bnf]_assign."""
    q = 0 if bnf else P
    g = H.rng(n + 31 * k + 7 * level + 3 * ms + bnf)
    n_lwe = 3 if n > 8192 else 20
    batch = 2 if n > 8192 else 5
    bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
    acc = rand_q(g, (batch, k + 1, n), q)
    lwe = lwe_inputs(g, batch, n_lwe, q)
    if ms == 2:  # the ModulusSwitchedLweCiphertext input
        lwe = g.integers(0, 2 * n, size=lwe.shape, dtype=np.uint64)
        lwe[:, ::5] = 0
    c = ctx_for(oracle, n)
    want = c.blind_rotate_batch(acc, lwe, bsk.reshape(-1), k, base_log, level, bnf=bnf, ms_mode=ms)
    M = engine.ntt64_pbs
    pl = engine.Plan.try_new(n, P)
    key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
    t = dev(acc)
    if bnf:
        M.blind_rotate_ntt64_bnf_assign(dev(lwe), t, key, ms)
    else:
        M.blind_rotate_ntt64_assign(dev(lwe), t, key, ms)
    assert np.array_equal(host(t), want)


@pytest.mark.parametrize("n,k,base_log,level", ENGINES)
@pytest.mark.parametrize("bnf", [True, False])
def test_pbs_lut_indexed(engine, oracle, n, k, base_log, level, bnf):
    """Item b bootstraps through LUT lut_index[b] of a list; an out-of-range index leaves lwe_out[b] untouched."""
    import torch
    q = 0 if bnf else P
    g = H.rng(7000 + n + k + bnf)
    n_lwe = 3 if n > 8192 else 16
    n_lut = 3
    idx = np.array([2, 0, 9, 1, 2] if n <= 8192 else [1, 9, 2], np.int32)
    batch = idx.size
    bsk = rand_q(g, (n_lwe, level, k + 1, k + 1, n), P)
    luts = rand_q(g, (n_lut, k + 1, n), q)
    lwe = lwe_inputs(g, batch, n_lwe, q)
    sentinel = rand_q(g, (batch, k * n + 1), 0)
    c = ctx_for(oracle, n)
    want = sentinel.copy()
    for b in range(batch):
        if idx[b] < n_lut:
            want[b] = c.pbs(lwe[b], luts[idx[b]].reshape(-1), bsk.reshape(-1), k, base_log, level, bnf=bnf)
    M = engine.ntt64_pbs
    pl = engine.Plan.try_new(n, P)
    key = M.NttBootstrapKey(pl, dev(bsk), base_log, level, M.BNF if bnf else M.SOLINAS)
    out = dev(sentinel)
    fn = (M.programmable_bootstrap_ntt64_bnf_lwe_ciphertext_mem_optimized if bnf
          else M.programmable_bootstrap_ntt64_lwe_ciphertext_mem_optimized)
    fn(dev(lwe), out, dev(luts), key, lut_index=torch.from_numpy(idx).cuda())
    assert np.array_equal(host(out), want)
    with pytest.raises(ValueError):
        fn(dev(lwe), out, dev(luts), key, lut_index=torch.from_numpy(idx[:1]).cuda())


@pytest.mark.parametrize("n,k", [(2048, 1), (1024, 2), (512, 4), (65536, 1)])
@pytest.mark.parametrize("q", [0, P])
def test_sample_extract_nth(engine, oracle, n, k, q):
    """Every monomial degree class (0, 1, mid, N - 1, strided runs) vs the oracle's step-by-step restatement."""
    g = H.rng(300 + n + k + (q != 0))
    batch = 3
    glwe = rand_q(g, (batch, k + 1, n), q)
    glwe[0, :, :4] = 0
    M = engine.ntt64_pbs
    t = dev(glwe)
    for nth, stride, count in ((0, 0, 1), (1, 0, 1), (n // 2 + 3, 0, 1), (n - 1, 0, 1), (5, n // 4, 4), (0, 1, 3)):
        out = dev(np.zeros((batch, count, k * n + 1), np.uint64))
        M.extract_lwe_sample_from_glwe_ciphertext(t, out, nth, stride, count, q)
        got = host(out)
        for b in range(batch):
            for j in range(count):
                want = oracle.sample_extract_nth(glwe[b].reshape(-1), n, k, nth + j * stride, q)
                assert np.array_equal(got[b, j], want), (nth, stride, count, b, j)
    with pytest.raises(engine.MiError):  # a degree >= N (the reference's opposite_count would underflow)
        M.extract_lwe_sample_from_glwe_ciphertext(t, dev(np.zeros((batch, 2, k * n + 1), np.uint64)), n - 2, 2, 2, q)


def many_lut_accumulator(n, k, msg_mod, carry_mod, functions):
    """shortint fill_many_lut_accumulator (shortint/engine/mod.rs:168-248), native modulus, padding bit: returns the
    GLWE and fn_stride (the HPU's monomial stride between the functions' boxes, hpu-mockup lib.rs:674-683)."""
    modulus_sup = msg_mod * carry_mod
    box = n // modulus_sup
    delta = (1 << 63) // modulus_sup
    fn_counts = len(functions)
    assert fn_counts <= modulus_sup // 2
    max_degree = modulus_sup // fn_counts - 1
    sub = (max_degree + 1) * box
    body = np.zeros(n, np.uint64)
    for fi, f in enumerate(functions):
        for m in range(max_degree + 1):
            body[fi * sub + m * box: fi * sub + (m + 1) * box] = np.uint64((f(m) * delta) % 2**64)
    half = box // 2
    body[:half] = H.neg_q(body[:half], 0)
    body = np.roll(body, -half)
    glwe = np.zeros((k + 1, n), np.uint64)
    glwe[k] = body
    fn_stride = (modulus_sup // fn_counts) * box
    return glwe, fn_stride, delta, max_degree


@pytest.mark.parametrize("lut_nb", [2, 4])
def test_many_lut_hpu_style(engine, oracle, lut_nb):
    """The HPU mockup's many-LUT PBS (lib.rs:736-761): standard modulus switch, blind_rotate_ntt64_bnf_assign on a
    fill_many_lut_accumulator GLWE, then lut_nb extractions at MonomialDegree(fn_idx * fn_stride).  Real keys at
    N = 2048, k = 1, level 1 (the fused engine), message 2 + carry 2 bits: every extracted sample equals the oracle
    bit for bit and decrypts to f_j(m)."""
    n, k, n_lwe, base_log, level = 2048, 1, 64, 23, 1
    msg_mod = carry_mod = 4
    functions = [lambda m, j=j: (m * (j + 1) + j) % (msg_mod * carry_mod) for j in range(lut_nb)]
    acc0, fn_stride, delta, max_degree = many_lut_accumulator(n, k, msg_mod, carry_mod, functions)
    g = H.rng(4000 + lut_nb)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17, 0)
    c = ctx_for(oracle, n)
    nbsk = c.bsk_to_ntt(bsk.reshape(-1), 64, normalize=False).reshape(bsk.shape)
    msgs = list(range(max_degree + 1)) * 3
    lwe = np.stack([H.lwe_encrypt(g, m * delta, lwe_sk, 30, 0) for m in msgs])
    batch = len(msgs)
    accs = np.broadcast_to(acc0, (batch, k + 1, n)).copy()
    want_glwe = c.blind_rotate_batch(accs, lwe, nbsk.reshape(-1), k, base_log, level, bnf=True, ms_mode=0)
    M = engine.ntt64_pbs
    pl = engine.Plan.try_new(n, P)
    key = M.NttBootstrapKey(pl, dev(nbsk), base_log, level, M.BNF)
    t = dev(accs)
    M.blind_rotate_ntt64_bnf_assign(dev(lwe), t, key, M.MS_STANDARD)
    assert np.array_equal(host(t), want_glwe)
    out = dev(np.zeros((batch, lut_nb, k * n + 1), np.uint64))
    M.extract_lwe_sample_from_glwe_ciphertext(t, out, 0, fn_stride, lut_nb, 0)
    got = host(out)
    out_sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    for b, m in enumerate(msgs):
        for j in range(lut_nb):
            want = oracle.sample_extract_nth(want_glwe[b].reshape(-1), n, k, j * fn_stride, 0)
            assert np.array_equal(got[b, j], want), (b, j)
            assert H.decode(H.lwe_decrypt(got[b, j], out_sk, 0), delta, msg_mod * carry_mod, 0) % (msg_mod * carry_mod) \
                == functions[j](m), (m, j)


def test_blind_rotate_errors(engine):
    import torch
    M = engine.ntt64_pbs
    n = 2048
    pl = engine.Plan.try_new(n, P)
    key = M.NttBootstrapKey(pl, torch.zeros((4, 1, 2, 2, n), dtype=torch.int64, device="cuda"), 23, 1, M.SOLINAS)
    lwe = torch.zeros((2, 5), dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError):  # variant mismatch
        M.blind_rotate_ntt64_bnf_assign(lwe, torch.zeros((2, 2, n), dtype=torch.int64, device="cuda"), key)
    with pytest.raises(ValueError):  # accumulator batch != LWE batch
        M.blind_rotate_ntt64_assign(lwe, torch.zeros((3, 2, n), dtype=torch.int64, device="cuda"), key)
    with pytest.raises(ValueError):  # centered switch of a mod-p LWE
        M.blind_rotate_ntt64_assign(lwe, torch.zeros((2, 2, n), dtype=torch.int64, device="cuda"), key, M.MS_CENTERED)
    M.blind_rotate_ntt64_assign(lwe[:0], torch.zeros((0, 2, n), dtype=torch.int64, device="cuda"), key)  # empty
