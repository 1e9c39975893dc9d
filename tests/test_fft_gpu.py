"""GPU parity of the f64-FFT PBS path (tfhe_ntt_amd.fft64, csrc/fft64_pbs.hip) (`-m gpu`).

The reference's transform is a measured f64 FFT, so the bar is the f64 error bound, not bit equality
(SURVEY.md §8f rank 4): transforms within ~1e-13 relative of the numpy restatement (oracle/fft_oracle.py)
after mapping this engine's Fourier order; external products within the f64 bound of the EXACT integer
result; PBS outputs that decrypt to f(m) for every ciphertext of a full 4096 batch under real keys, with the
phase noise of the restatement.
"""
import numpy as np
import pytest

import fft_oracle as F
import tfhe_helpers as H

pytestmark = pytest.mark.gpu

N, M = 2048, 1024


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def fdev(z):
    """natural-order complex (..., M) -> engine-order float64 device tensor (..., M, 2)."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(np.stack([z.real, z.imag], axis=-1))).cuda()


@pytest.fixture(scope="module")
def fft(engine):
    return engine.fft64.Fft(N)


@pytest.fixture(scope="module")
def order(fft):
    return fft.fourier_order().astype(np.int64)


def to_engine(z, order):
    return z[..., order]


def from_engine(t, order):
    a = t.cpu().numpy()
    z = a[..., 0] + 1j * a[..., 1]
    out = np.empty_like(z)
    out[..., order] = z
    return out


def test_fourier_order_is_a_permutation(order):
    assert sorted(order.tolist()) == list(range(M))


def test_forward_as_torus_matches_restatement(engine, fft, order):
    import torch
    g = H.rng(11)
    x = H.uniform_u64(g, (24, N))
    x[0] = 0
    x[1, :] = np.uint64(2**63)  # -1/2 on the torus
    out = torch.zeros((24, M, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(out, dev(x))
    got = from_engine(out, order)
    want = F.forward_as_torus(x)
    scale = np.abs(want).max()
    assert np.abs(got - want).max() / scale < 1e-13


def test_backward_as_torus_and_round_trip(engine, fft, order):
    import torch
    g = H.rng(12)
    x = H.uniform_u64(g, (16, N))
    z = F.forward_as_torus(x)
    std = torch.zeros((16, N), dtype=torch.int64, device="cuda")
    fft.backward_as_torus(std, fdev(to_engine(z, order)))
    got = host(std)
    assert F.signed_diff(got, F.backward_as_torus(z)).max() < 2.0 ** 14
    assert F.signed_diff(got, x).max() < 2.0 ** 16
    # add_backward_as_torus adds to what is there
    base = H.uniform_u64(g, (16, N))
    acc = dev(base)
    fft.add_backward_as_torus(acc, fdev(to_engine(z, order)))
    with np.errstate(over="ignore"):
        assert F.signed_diff(host(acc), base + x).max() < 2.0 ** 16
    # GPU forward -> GPU backward
    four = torch.zeros((16, M, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(four, dev(x))
    back = torch.zeros((16, N), dtype=torch.int64, device="cuda")
    fft.backward_as_torus(back, four)
    assert F.signed_diff(host(back), x).max() < 2.0 ** 16


def _exact_ext_product(glwe, ggsw_std, base_log, level):
    """sum over levels / rows of decomposition term x GGSW row, exact in Z_{2^64}[X]/(X^N + 1)."""
    kp1 = glwe.shape[0]
    out = np.zeros((kp1, N), np.uint64)
    terms = F.decompose(glwe, base_log, level)
    with np.errstate(over="ignore"):
        for li, term in enumerate(terms):
            for r in range(kp1):
                a = term[r]
                for c in range(kp1):
                    out[c] += _negacyclic(a, ggsw_std[li, r, c])
    return out


def _negacyclic(a, b):
    n = a.size
    out = np.zeros(n, np.uint64)
    with np.errstate(over="ignore"):
        for j in np.nonzero(a)[0]:
            j = int(j)
            rot = np.concatenate([np.uint64(0) - b[n - j:], b[:n - j]])
            out += a[j] * rot
    return out


@pytest.mark.parametrize("k,base_log,level", [(1, 23, 1), (1, 10, 2), (2, 15, 1), (2, 8, 3), (1, 31, 1)])
def test_external_product_vs_exact(engine, fft, k, base_log, level):
    import torch
    g = H.rng(100 * k + base_log + level)
    batch = 3
    ggsw = H.uniform_u64(g, (level, k + 1, k + 1, N))
    fg = torch.zeros((level, k + 1, k + 1, M, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(fg, dev(ggsw))
    glwe = H.uniform_u64(g, (batch, k + 1, N))
    glwe[0, 0, :4] = np.array([0, 2**64 - 1, 2**63, 2**63 - 1], np.uint64)
    out0 = H.uniform_u64(g, (batch, k + 1, N))
    out = dev(out0)
    engine.fft64.add_external_product_assign(out, fg, dev(glwe), base_log, level, fft)
    got = host(out)
    for b in range(batch if k == 1 and level == 1 else 1):
        with np.errstate(over="ignore"):
            want = out0[b] + _exact_ext_product(glwe[b], ggsw, base_log, level)
        err = F.signed_diff(got[b], want).max()
        # f64 error: digits up to 2^(B-1) times torus values, summed over N terms, kept to 53 bits
        assert err < 2.0 ** max(48, base_log + 24), (b, np.log2(err))


def test_cmux_semantics(engine, fft):
    import torch
    g = H.rng(5)
    batch, base_log, level = 4, 23, 1
    ggsw = H.uniform_u64(g, (level, 2, 2, N))
    fg = torch.zeros((level, 2, 2, M, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(fg, dev(ggsw))
    ct0, ct1 = H.uniform_u64(g, (batch, 2, N)), H.uniform_u64(g, (batch, 2, N))
    t0, t1 = dev(ct0), dev(ct1)
    engine.fft64.cmux_assign(t0, t1, fg, base_log, level, fft)
    with np.errstate(over="ignore"):
        diff = ct1 - ct0
    assert np.array_equal(host(t1), diff)
    ref = dev(ct0)
    engine.fft64.add_external_product_assign(ref, fg, dev(diff), base_log, level, fft)
    assert np.array_equal(host(t0), host(ref))  # same kernel arithmetic: bit-identical


def test_pbs_config4_full_batch_real_keys(engine, fft, order):
    """The default shortint PBS at PARAM_MESSAGE_2_CARRY_2's shape (n = 918, N = 2048, B = 2^23, l = 1, 2+2-bit
    messages with padding, TUniform 2^45 LWE / 2^17 GLWE noise) on the f64-FFT path: all 4096 outputs decrypt
    to f(m), and their phase noise matches the numpy restatement's.  The output ciphertexts themselves are NOT
    comparable bit for bit with any other f64 implementation (the reference's included): once FFT rounding flips
    one decomposition digit, the masks differ by a GGSW row, i.e. by an encryption of zero — both results are
    valid encryptions of f(m) with the same noise distribution."""
    import torch
    n_lwe, base_log, level, msg_mod, batch = 918, 23, 1, 16, 4096
    delta = (1 << 63) // msg_mod
    g = H.rng(64918)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (1, N))
    bsk = H.bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, 17)
    fbsk = torch.zeros((n_lwe, level, 2, 2, M, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    f = lambda x: (7 * x + 2) % msg_mod
    lut = H.pbs_lut(N, 1, msg_mod, delta, f)
    msgs = np.arange(batch) % msg_mod
    lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 45)
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    out = dev(np.zeros((batch, N + 1), np.uint64))
    engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(lut), key)
    got = host(out)
    sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    pts = H.lwe_decrypt_batch(got, sk)
    want_pt = np.array([f(int(m)) for m in msgs], np.uint64) * np.uint64(delta)
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert np.array_equal(dec, want_pt // np.uint64(delta))
    noise = F.signed_diff(pts, want_pt)
    assert noise.max() < 2.0 ** 54, np.log2(noise.max())
    idx = np.array([0, 1, 2, 3, 2047, batch - 1])
    ref = F.pbs(lwe[idx], lut, F.forward_as_torus(bsk), base_log, level)
    ref_noise = F.signed_diff(H.lwe_decrypt_batch(ref, sk), want_pt[idx])
    rms = lambda e: float(np.sqrt(np.mean(e ** 2)))
    assert rms(ref_noise) / 4 < rms(noise) < 4 * rms(ref_noise), (np.log2(rms(noise)), np.log2(rms(ref_noise)))


@pytest.mark.parametrize("k,level,base_log", [(1, 2, 12), (2, 1, 23), (2, 2, 12)])
@pytest.mark.parametrize("ms_mode", [0, 1, 2])
def test_pbs_shapes_real_keys(engine, fft, k, level, base_log, ms_mode):
    import torch
    n_lwe, msg_mod = 48, 4
    delta = (1 << 63) // msg_mod
    g = H.rng(700 + 10 * k + level + 100 * ms_mode)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, N))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17)
    fbsk = torch.zeros((n_lwe, level, k + 1, k + 1, M, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    f = lambda x: (x + 3) % msg_mod
    lut = H.pbs_lut(N, k, msg_mod, delta, f)
    msgs = np.arange(8) % msg_mod
    lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 30)
    if ms_mode == 2:  # pre-switched input: the standard switch applied by the caller
        lwe = F.modulus_switch(lwe, 12)
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    out = dev(np.zeros((len(msgs), k * N + 1), np.uint64))
    engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(lut), key, ms_mode)
    pts = H.lwe_decrypt_batch(host(out), H.glwe_sk_as_lwe_sk(glwe_sk))
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert list(dec) == [f(int(m)) for m in msgs]


def test_errors(engine):
    M_ = engine.fft64
    with pytest.raises(engine.MiError) as e:
        M_.Fft(16)
    assert e.value.status == 6  # MI_ERR_UNSUPPORTED: below the engines' 32 <= N <= 2^18
    with pytest.raises(engine.MiError) as e:
        M_.Fft(1000)
    assert e.value.status == 1


@pytest.mark.parametrize("batch", [1, 5, 7])
@pytest.mark.parametrize("ms_mode", [0, 1, 2])
def test_pbs_k1_l1_ragged_batches(engine, fft, batch, ms_mode):
    """The k = 1, level-1 shape runs the 4-ciphertexts-per-workgroup kernel: batches that do not fill the last
    workgroup (its idle waves still take part in the step synchronisation) under every modulus-switch mode."""
    import torch
    n_lwe, msg_mod, base_log = 40, 4, 23
    delta = (1 << 63) // msg_mod
    g = H.rng(900 + 10 * batch + ms_mode)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (1, N))
    bsk = H.bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, 17)
    fbsk = torch.zeros((n_lwe, 1, 2, 2, M, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    f = lambda x: (3 * x + 1) % msg_mod
    lut = H.pbs_lut(N, 1, msg_mod, delta, f)
    msgs = np.arange(batch) % msg_mod
    lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 30)
    if ms_mode == 2:
        lwe = F.modulus_switch(lwe, 12)
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, 1, fft)
    sentinel = np.full((batch + 1, N + 1), 0x5A5A5A5A5A5A5A5A, np.uint64)
    out = dev(sentinel)
    engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out[:batch], dev(lut), key, ms_mode)
    got = host(out)
    assert np.array_equal(got[batch], sentinel[batch])  # nothing written past the batch
    pts = H.lwe_decrypt_batch(got[:batch], H.glwe_sk_as_lwe_sk(glwe_sk))
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert list(dec) == [f(int(m)) for m in msgs]


# ---- the reference's serialised (natural) Fourier order and key bytes --------------------------------------
def test_standard_order_is_the_natural_dft(engine, fft, order):
    """to_standard_order(forward_as_torus(x)) is the natural-order DFT (what Plan::serialize_fourier_buffer emits,
    tfhe-fft/src/unordered.rs:943-964; the reference's test_fwd pins it to rustfft's forward DFT), and the two
    conversions are exact inverse permutations, out of place and in place."""
    import torch
    g = H.rng(13)
    x = H.uniform_u64(g, (9, N))
    four = torch.zeros((9, M, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(four, dev(x))
    std = torch.empty_like(four)
    fft.to_standard_order(std, four)
    a = std.cpu().numpy()
    want = F.forward_as_torus(x)
    assert np.abs((a[..., 0] + 1j * a[..., 1]) - want).max() / np.abs(want).max() < 1e-13
    # the device permutation agrees with the host's fourier_order exactly
    assert np.array_equal(from_engine(four, order), a[..., 0] + 1j * a[..., 1])
    back = torch.empty_like(four)
    fft.from_standard_order(back, std)
    assert torch.equal(back, four)
    inplace = four.clone()
    fft.to_standard_order(inplace, inplace)
    assert torch.equal(inplace, std)
    fft.from_standard_order(inplace, inplace)
    assert torch.equal(inplace, four)
    with pytest.raises(engine.MiError):  # partial overlap is refused
        engine._lib.check(engine._lib.lib().mi_fft64_to_standard_order(
            fft.handle, engine.fft64._fdev(four[1:], "o"), engine.fft64._fdev(four[:-1], "i"), 8, None))


@pytest.mark.parametrize("versioned", [False, True])
def test_fourier_key_bytes_round_trip_and_reference_key(engine, fft, versioned):
    """A key serialised by this engine reloads into an identical device key (so its PBS outputs are bit-identical),
    and a key built the reference's way -- the natural-order DFT of every standard-key polynomial (numpy
    restatement), written in the reference's bincode layout -- loads and bootstraps to f(m)."""
    import torch
    from tfhe_ntt_amd import fourier_bsk_format as FB
    n_lwe, base_log, level, msg_mod = 32, 23, 1, 4
    delta = (1 << 63) // msg_mod
    g = H.rng(1400 + versioned)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (1, N))
    bsk = H.bsk_gen_native_l1(g, lwe_sk, glwe_sk, base_log, 17)
    fbsk = torch.zeros((n_lwe, level, 2, 2, M, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    buf = key.serialize(versioned)                                  # the library's writer
    assert len(buf) == 24 + n_lwe * 4 * (8 + 16 * M) + 32 + (24 if versioned else 0)
    nat = torch.empty_like(fbsk)
    fft.to_standard_order(nat, fbsk)
    assert buf == FB.serialize_fourier_bsk(nat.cpu().numpy(), N, 2, level, base_log, versioned)  # == Python mirror
    key2 = engine.fft64.FourierLweBootstrapKey.deserialize(buf, versioned, device=0, fft=fft)
    assert torch.equal(key2.fbsk, fbsk)
    assert (key2.input_lwe_dimension, key2.base_log, key2.level) == (n_lwe, base_log, level)
    key4 = engine.fft64.FourierLweBootstrapKey.load(buf, versioned, fft=fft)  # the library's loader (owns its copy)
    assert (key4.input_lwe_dimension, key4.glwe_dimension, key4.base_log, key4.level) == (n_lwe, 1, base_log, level)
    assert key4.serialize(versioned) == buf
    for bad in (buf[:-1], buf + b"\0", buf[: len(buf) - 8] + bytes(8)):  # truncated, trailing, level 0
        with pytest.raises(engine.MiError):
            engine.fft64.FourierLweBootstrapKey.load(bad, versioned, fft=fft)
    f = lambda x: (x + 1) % msg_mod
    lut = dev(H.pbs_lut(N, 1, msg_mod, delta, f))
    msgs = np.arange(8) % msg_mod
    lwe = dev(H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 30))
    outs = []
    for k_ in (key, key2, key4):
        out = dev(np.zeros((len(msgs), N + 1), np.uint64))
        engine.fft64.programmable_bootstrap_lwe_ciphertext(lwe, out, lut, k_)
        outs.append(host(out))
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    # the reference's way: natural-order Fourier polynomials (numpy), the reference's bytes, loaded here
    zn = F.forward_as_torus(bsk)                                   # (n_lwe, 1, 2, 2, M) complex, natural order
    ref_bytes = FB.serialize_fourier_bsk(zn, N, 2, level, base_log, versioned)
    key3 = engine.fft64.FourierLweBootstrapKey.deserialize(ref_bytes, versioned, device=0, fft=fft)
    a3, a = key3.fbsk.cpu().numpy(), fbsk.cpu().numpy()
    assert np.abs(a3 - a).max() / np.abs(a).max() < 1e-13  # the same key up to f64 rounding
    out = dev(np.zeros((len(msgs), N + 1), np.uint64))
    engine.fft64.programmable_bootstrap_lwe_ciphertext(lwe, out, lut, key3)
    pts = H.lwe_decrypt_batch(host(out), H.glwe_sk_as_lwe_sk(glwe_sk))
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert list(dec) == [f(int(m)) for m in msgs]
