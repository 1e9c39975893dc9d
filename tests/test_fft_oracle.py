"""The numpy restatement of the f64-FFT PBS path (oracle/fft_oracle.py) against exact integer arithmetic and
the reference's own properties.  No GPU.

* forward_as_integer x forward_as_torus -> backward_as_torus is the negacyclic product mod 2^64 within the
  f64 error bound (fft_impl/fft64/math/fft/tests.rs checks the same product property);
* the torus round trip is within a few ulps of 2^-64;
* the decomposition recomposes (decomposer.rs closest_representable);
* a real-key PBS decrypts to f(m) for every message (lwe_programmable_bootstrapping.rs:22-150, FFT variant).
"""
import numpy as np
import pytest

import fft_oracle as F
import tfhe_helpers as H

N = 2048


def negacyclic_exact(a, b):
    """(a * b) mod (X^N + 1) mod 2^64 by schoolbook rotation (a small signed ints as u64, b u64)."""
    n = a.size
    out = np.zeros(n, np.uint64)
    with np.errstate(over="ignore"):
        for j in range(n):
            aj = a[j]
            if aj == 0:
                continue
            rot = np.concatenate([np.uint64(0) - b[n - j:], b[:n - j]])  # X^j * b
            out += aj * rot
    return out


def test_twisties_match_the_reference_formula():
    m = 1024
    t = F.twisties(m)
    i = np.arange(m)
    assert np.allclose(t, np.exp(1j * np.pi * i / (2 * m)), rtol=0, atol=1e-15)


@pytest.mark.parametrize("seed", [1, 2])
def test_negacyclic_product_within_fft_bound(seed):
    g = H.rng(seed)
    a = (g.integers(-(2**22), 2**22, size=N)).astype(np.int64).view(np.uint64)
    b = H.uniform_u64(g, N)
    want = negacyclic_exact(a, b)
    got = F.backward_as_torus(F.forward_as_integer(a) * F.forward_as_torus(b))
    err = F.signed_diff(got, want)
    assert err.max() < 2.0 ** 48, np.log2(err.max())


def test_torus_round_trip():
    g = H.rng(3)
    x = H.uniform_u64(g, (4, N))
    err = F.signed_diff(F.backward_as_torus(F.forward_as_torus(x)), x)
    assert err.max() < 2.0 ** 16


@pytest.mark.parametrize("base_log,level", [(23, 1), (10, 2), (4, 5), (31, 2)])
def test_decomposition_recomposes(base_log, level):
    g = H.rng(base_log * 10 + level)
    x = H.uniform_u64(g, 4096)
    terms = F.decompose(x, base_log, level)
    rec = np.zeros_like(x)
    with np.errstate(over="ignore"):
        for j, t in enumerate(terms):  # term j = level (level - j): weight 2^(64 - B (level - j))
            rec += t << np.uint64(64 - base_log * (level - j))
        for t in terms:
            d = t.view(np.int64)
            assert np.all(np.abs(d) <= 2 ** (base_log - 1))
    # closest representable: |x - rec| <= 2^(64 - B L - 1)
    assert F.signed_diff(rec, x).max() <= 2.0 ** (64 - base_log * level - 1)


def test_pbs_decrypts_real_keys():
    n_lwe, base_log, level, msg_mod = 24, 23, 1, 4
    delta = (1 << 63) // msg_mod
    g = H.rng(2024)
    lwe_sk = H.binary_key(g, n_lwe)
    glwe_sk = H.binary_key(g, (1, N))
    bsk = H.bsk_gen(g, lwe_sk, glwe_sk, base_log, level, 17)
    fbsk = F.forward_as_torus(bsk)
    f = lambda x: (x + 1) % msg_mod
    lut = H.pbs_lut(N, 1, msg_mod, delta, f)
    msgs = np.arange(8) % msg_mod
    lwe = H.lwe_encrypt_batch(g, msgs.astype(np.uint64) * np.uint64(delta), lwe_sk, 30)
    out = F.pbs(lwe, lut, fbsk, base_log, level)
    pts = H.lwe_decrypt_batch(out, H.glwe_sk_as_lwe_sk(glwe_sk))
    dec = ((pts + np.uint64(delta // 2)) // np.uint64(delta)) % np.uint64(2 * msg_mod)
    assert list(dec) == [f(int(m)) for m in msgs]
