"""GPU parity of the shape-generic f64-FFT engine (csrc/fft64_generic.hip): every polynomial size 32 <= N <= 2^18
other than the one-wave engine's 2048 (`-m gpu`).  The reference's Fft::new takes any power of two
(fft_impl/fft64/math/fft/mod.rs:170-223) and its f64 PBS is shape generic (fft_impl/fft64/crypto/bootstrap.rs:294-521);
the shortint sets next to PARAM_MESSAGE_2_CARRY_2 run it at N = 512 (k = 4), 8192 and 65536
(shortint/parameters/v1_4/classic/tuniform/p_fail_2_minus_128/ks_pbs.rs:8-90).

The bar is the f64 one of tests/test_fft_gpu.py: transforms within 1e-13 relative of the
numpy restatement (oracle/fft_oracle.py) after mapping this engine's Fourier order, round trips within the f64
bound; external products within the f64 bound of the EXACT integer product; PBS outputs that decrypt to f(m) under
real keys at the shortint shapes, with the restatement's phase noise where it runs in seconds.
"""
import numpy as np
import pytest

import fft_oracle as F
import tfhe_helpers as H

pytestmark = pytest.mark.gpu

P = 0xFFFFFFFF00000001
SIZES = [32, 64, 128, 256, 512, 1024, 4096, 8192, 16384, 32768, 65536, 131072, 262144]


def dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).cuda()


def host(t):
    return t.cpu().numpy().view(np.uint64)


def fdev(z):
    import torch
    return torch.from_numpy(np.ascontiguousarray(np.stack([z.real, z.imag], axis=-1))).cuda()


def from_engine(t, order):
    a = t.cpu().numpy()
    z = a[..., 0] + 1j * a[..., 1]
    out = np.empty_like(z)
    out[..., order] = z
    return out


@pytest.mark.parametrize("n", SIZES)
def test_generic_transforms(engine, n):
    import torch
    m = n // 2
    fft = engine.fft64.Fft(n)
    order = fft.fourier_order().astype(np.int64)
    assert sorted(order.tolist()) == list(range(m))
    batch = max(2, min(8, (1 << 16) // n))
    g = H.rng(3000 + n)
    x = H.uniform_u64(g, (batch, n))
    x[0, : n // 2] = 0
    x[1, :] = np.uint64(2**63)
    four = torch.zeros((batch, m, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(four, dev(x))
    want = F.forward_as_torus(x)
    got = from_engine(four, order)
    assert np.abs(got - want).max() / np.abs(want).max() < 1e-13
    # the natural order through the device permutation, exact against the host order; in place both ways
    std = torch.empty_like(four)
    fft.to_standard_order(std, four)
    a = std.cpu().numpy()
    assert np.array_equal(a[..., 0] + 1j * a[..., 1], got)
    inplace = four.clone()
    fft.to_standard_order(inplace, inplace)
    assert torch.equal(inplace, std)
    fft.from_standard_order(inplace, inplace)
    assert torch.equal(inplace, four)
    # backward: from the restatement's spectrum, and the GPU round trip; add_backward adds
    bound = 2.0 ** (16 + max(0, (n.bit_length() - 12) // 2))
    out = torch.zeros((batch, n), dtype=torch.int64, device="cuda")
    fft.backward_as_torus(out, fdev(want[..., order]))
    assert F.signed_diff(host(out), F.backward_as_torus(want)).max() < bound
    back = torch.zeros((batch, n), dtype=torch.int64, device="cuda")
    fft.backward_as_torus(back, four)
    assert F.signed_diff(host(back), x).max() < bound
    base = H.uniform_u64(g, (batch, n))
    acc = dev(base)
    fft.add_backward_as_torus(acc, four)
    with np.errstate(over="ignore"):
        assert F.signed_diff(host(acc), base + x).max() < bound


def _signed_mod_p(u):
    """two's complement u64 (small signed values) -> residues mod p"""
    s = u.view(np.int64)
    return np.where(s < 0, (np.uint64(P) - (np.uint64(0) - u)), u).astype(np.uint64)


def _exact_products(oracle, a, d, base_log):
    """a (..., N) u64 times d (..., N) small signed digits (two's complement), negacyclic mod 2^64, exact.  Through
    the oracle's Solinas transform with 32-bit limbs of a when N 2^32 2^(B-1) < p / 2, by rotation sums otherwise."""
    n = a.shape[-1]
    if n.bit_length() - 1 + base_log < 31:
        plan = oracle.Plan.try_new(n, P)
        flat_a = np.ascontiguousarray(a.reshape(-1, n))
        d_hat = plan.fwd(np.ascontiguousarray(_signed_mod_p(d.reshape(-1, n))), threads=16)
        out = np.zeros_like(flat_a)
        with np.errstate(over="ignore"):
            for t in range(2):
                limb = (flat_a >> np.uint64(32 * t)) & np.uint64(0xFFFFFFFF)
                v = plan.inv(plan.mul_assign_normalize(plan.fwd(limb, threads=16), d_hat), threads=16)
                v = np.where(v > np.uint64(P // 2), v - np.uint64(P), v)
                out += v << np.uint64(32 * t)
        return out.reshape(a.shape)
    out = np.zeros(a.reshape(-1, n).shape, np.uint64)
    fa, fd = a.reshape(-1, n), d.reshape(-1, n)
    with np.errstate(over="ignore"):
        for i in range(fa.shape[0]):
            for j in range(n):
                if fd[i, j]:
                    out[i] += fd[i, j] * np.concatenate([np.uint64(0) - fa[i, n - j:], fa[i, : n - j]])
    return out.reshape(a.shape)


def _exact_ext_product(oracle, glwe, ggsw, base_log, level):
    """sum over levels li and rows r of digit_li(glwe[r]) x ggsw[li][r][c], exact in Z_2^64[X]/(X^N + 1)"""
    kp1, n = glwe.shape
    terms = F.decompose(glwe, base_log, level)  # least significant level first
    a = np.stack([np.broadcast_to(ggsw[li, r], (kp1, n)) for li in range(level) for r in range(kp1)])
    d = np.stack([np.broadcast_to(terms[li][r], (kp1, n)) for li in range(level) for r in range(kp1)])
    prods = _exact_products(oracle, np.ascontiguousarray(a), np.ascontiguousarray(d), base_log)
    with np.errstate(over="ignore"):
        return prods.sum(axis=0, dtype=np.uint64)


@pytest.mark.parametrize("n,k,base_log,level", [
    (32, 1, 23, 1), (256, 2, 15, 1), (512, 4, 23, 1), (1024, 1, 10, 2), (4096, 2, 8, 3), (8192, 1, 15, 2),
    (16384, 1, 12, 2), (65536, 1, 11, 3)])
def test_generic_external_product_vs_exact(engine, oracle, n, k, base_log, level):
    import torch
    m = n // 2
    fft = engine.fft64.Fft(n)
    g = H.rng(5000 + n + k + base_log)
    batch = 2
    ggsw = H.uniform_u64(g, (level, k + 1, k + 1, n))
    fg = torch.zeros((level, k + 1, k + 1, m, 2), dtype=torch.float64, device="cuda")
    fft.forward_as_torus(fg, dev(ggsw))
    glwe = H.uniform_u64(g, (batch, k + 1, n))
    glwe[0, 0, :4] = np.array([0, 2**64 - 1, 2**63, 2**63 - 1], np.uint64)
    out0 = H.uniform_u64(g, (batch, k + 1, n))
    out = dev(out0)
    engine.fft64.add_external_product_assign(out, fg, dev(glwe), base_log, level, fft)
    got = host(out)
    bound = 2.0 ** (max(48, base_log + 24) + max(0, n.bit_length() - 12))
    for b in range(batch):
        with np.errstate(over="ignore"):
            want = out0[b] + _exact_ext_product(oracle, glwe[b], ggsw, base_log, level)
        err = F.signed_diff(got[b], want).max()
        assert err < bound, (b, np.log2(max(err, 1)))
    # CMUX: ct1 -= ct0, then ct0 += ext(ct1), bit-identical to the external product of the difference
    ct0, ct1 = H.uniform_u64(g, (batch, k + 1, n)), H.uniform_u64(g, (batch, k + 1, n))
    t0, t1 = dev(ct0), dev(ct1)
    engine.fft64.cmux_assign(t0, t1, fg, base_log, level, fft)
    with np.errstate(over="ignore"):
        diff = ct1 - ct0
    assert np.array_equal(host(t1), diff)
    ref = dev(ct0)
    engine.fft64.add_external_product_assign(ref, fg, dev(diff), base_log, level, fft)
    assert np.array_equal(host(t0), host(ref))


@pytest.mark.parametrize("n,k,level,base_log", [(256, 2, 2, 12), (1024, 1, 1, 23), (4096, 3, 2, 12)])
@pytest.mark.parametrize("ms_mode", [0, 1, 2])
def test_generic_pbs_small_real_keys(engine, oracle, n, k, level, base_log, ms_mode):
    import torch
    m = n // 2
    fft = engine.fft64.Fft(n)
    n_lwe, msg_mod = 40, 4
    delta = (1 << 63) // msg_mod
    g = H.rng(6000 + n + 10 * k + ms_mode)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen_fast(g, oracle, lwe_sk, glwe_sk, base_log, level, 17)
    fbsk = torch.zeros((n_lwe, level, k + 1, k + 1, m, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    f = lambda x: (x + 3) % msg_mod
    lut = H.pbs_lut(n, k, msg_mod, delta, f)
    msgs = np.arange(9) % msg_mod
    lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 30)
    if ms_mode == 2:
        lwe = F.modulus_switch(lwe, n.bit_length())
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    sentinel = np.full((len(msgs) + 1, k * n + 1), 0x5A5A5A5A5A5A5A5A, np.uint64)
    out = dev(sentinel)
    engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out[: len(msgs)], dev(lut), key, ms_mode)
    got = host(out)
    assert np.array_equal(got[-1], sentinel[-1])
    pts = H.lwe_decrypt_batch(got[:-1], H.glwe_sk_as_lwe_sk(glwe_sk))
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert list(dec) == [f(int(x)) for x in msgs]


# name: (N, k, n_lwe, base_log, level, lwe_noise_log2, glwe_noise_log2, message x carry modulus, batch)
SHAPES = {
    "message_1_carry_1": (512, 4, 879, 23, 1, 46, 17, 4, 256),
    "message_3_carry_3": (8192, 1, 1077, 15, 2, 41, 3, 64, 64),
    "message_4_carry_4": (65536, 1, 1117, 11, 3, 40, 3, 256, 256),
}


@pytest.mark.parametrize("name", list(SHAPES))
def test_generic_pbs_shortint_shapes_real_keys(engine, oracle, name):
    """Every message of the shape's plaintext space bootstraps to f(m) under real keys (TUniform noise as the
    parameter set), the centered modulus switch of the shortint PBS; key bytes round-trip through the library."""
    import torch
    n, k, n_lwe, base_log, level, lwe_noise, glwe_noise, msg_mod, batch = SHAPES[name]
    m = n // 2
    fft = engine.fft64.Fft(n)
    delta = (1 << 63) // msg_mod
    g = H.rng(7000 + n)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (k, n))
    bsk = H.bsk_gen_fast(g, oracle, lwe_sk, glwe_sk, base_log, level, glwe_noise)
    fbsk = torch.zeros((n_lwe, level, k + 1, k + 1, m, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    small_bsk = bsk[:16].copy() if n <= 8192 else None
    del bsk
    f = lambda x: (5 * x + 3) % msg_mod
    lut = H.pbs_lut(n, k, msg_mod, delta, f)
    msgs = np.arange(batch) % msg_mod
    lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, lwe_noise)
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    out = dev(np.zeros((batch, k * n + 1), np.uint64))
    engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(lut), key, engine.fft64.MS_CENTERED)
    sk = H.glwe_sk_as_lwe_sk(glwe_sk)
    pts = H.lwe_decrypt_batch(host(out), sk)
    want_pt = np.array([f(int(x)) for x in msgs], np.uint64) * np.uint64(delta)
    with np.errstate(over="ignore"):
        dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert np.array_equal(dec, want_pt // np.uint64(delta))
    noise = F.signed_diff(pts, want_pt)
    assert noise.max() < delta / 4, np.log2(noise.max())
    if small_bsk is not None:
        # the restatement on the key's first 16 GGSWs: the same phase-noise scale (both are valid encryptions of
        # f(m); bit patterns differ once f64 rounding flips a digit, see tests/test_fft_gpu.py)
        nn = 16
        sub = lwe_sk[:nn]
        lwe2 = H.lwe_encrypt_batch(g, msgs[:4].astype(np.uint64) * np.uint64(delta), sub, lwe_noise)
        key2 = engine.fft64.FourierLweBootstrapKey(fbsk[:nn].contiguous(), base_log, level, fft)
        out2 = dev(np.zeros((4, k * n + 1), np.uint64))
        engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe2), out2, dev(lut), key2)
        ref = F.pbs(lwe2, lut, F.forward_as_torus(small_bsk), base_log, level)
        n_gpu = F.signed_diff(H.lwe_decrypt_batch(host(out2), sk), want_pt[:4])
        n_ref = F.signed_diff(H.lwe_decrypt_batch(ref, sk), want_pt[:4])
        assert n_gpu.max() < delta / 4 and n_ref.max() < delta / 4
    # key bytes: the library writes the reference's layout and reloads (the plan taken from the bytes)
    if n <= 8192:
        buf = key.serialize(True)
        key3 = engine.fft64.FourierLweBootstrapKey.load(buf, True)
        assert key3.polynomial_size == n and key3.glwe_dimension == k and key3.level == level
        assert key3.serialize(True) == buf


@pytest.mark.parametrize("n", [4096, 8192])
def test_generic_pbs_two_lanes(engine, n):
    """A chunk of >= 64 ciphertexts runs as two lanes (halves on the caller's stream and a pooled side stream,
    fft64_generic.hip FFTG_LANE_MIN): every output of an odd-split batch of 70 equals, bit for bit, the one-lane run
    (batch 8 < 64) of the same items — each item's f64 arithmetic is independent of where the batch is cut."""
    import torch
    k, level, base_log, n_lwe, batch = 1, 2, 12, 3, 70
    fft = engine.fft64.Fft(n)
    g = H.rng(8100 + n)
    bsk = H.uniform_u64(g, (n_lwe, level, k + 1, k + 1, n))
    fbsk = torch.zeros((n_lwe, level, k + 1, k + 1, n // 2, 2), dtype=torch.float64, device="cuda")
    engine.fft64.convert_standard_lwe_bootstrap_key_to_fourier(dev(bsk), fbsk, fft)
    key = engine.fft64.FourierLweBootstrapKey(fbsk, base_log, level, fft)
    lut = H.uniform_u64(g, (k + 1, n))
    lwe = H.uniform_u64(g, (batch, n_lwe + 1))
    out = dev(np.zeros((batch, k * n + 1), np.uint64))
    engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe), out, dev(lut), key)
    got = host(out)
    for lo in (0, 31, 62):  # the first half, across the split point (35), the second half
        o8 = dev(np.zeros((8, k * n + 1), np.uint64))
        engine.fft64.programmable_bootstrap_lwe_ciphertext(dev(lwe[lo:lo + 8]), o8, dev(lut), key)
        assert np.array_equal(host(o8), got[lo:lo + 8]), lo


def test_generic_errors(engine):
    M_ = engine.fft64
    for bad in (16, 1 << 19):
        with pytest.raises(engine.MiError) as e:
            M_.Fft(bad)
        assert e.value.status == 6  # MI_ERR_UNSUPPORTED
    import torch
    fft = M_.Fft(1024)
    fb = torch.zeros((2, 1, 18, 18, 512, 2), dtype=torch.float64, device="cuda")
    with pytest.raises(engine.MiError) as e:
        M_.FourierLweBootstrapKey(fb, 10, 1, fft)  # k = 17
    assert e.value.status == 6
