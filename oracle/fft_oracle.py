"""numpy restatement of the f64-FFT PBS path of tfhe core_crypto (the default shortint PBS).

TEST INFRASTRUCTURE ONLY: imported by tests/ (and bench.py's cpu_baseline leg) as the checker; the product
package never imports it.  Reference paths relative to /root/reference/tfhe/src/core_crypto:

* ``twisties``             fft_impl/fft64/math/fft/mod.rs:64-75 (Twisties::new)
* ``forward_as_torus``     fft_impl/fft64/math/fft/mod.rs:227-248 + 524-543 (convert_forward_torus, split at N/2)
* ``forward_as_integer``   fft_impl/fft64/math/fft/mod.rs:250-269 (convert_forward_integer_scalar)
* ``backward_as_torus``    fft_impl/fft64/math/fft/mod.rs:294-334 + 545-565 (convert_[add_]backward_torus)
* ``from_torus``           commons/math/torus/mod.rs:72-78
* ``decompose``            commons/math/decomposition/decomposer.rs:156-185 + iter.rs:131-151 (native u64)
* ``external_product``     fft_impl/fft64/crypto/ggsw.rs:483-603 (+ update_with_fmadd :617-698)
* ``pbs``                  fft_impl/fft64/crypto/bootstrap.rs:294-381 (blind_rotate_assign), 481-521 (bootstrap),
                           algorithms/glwe_sample_extraction.rs:89-160, fft_impl/common.rs:10-23 (modulus switch)

The reference's transform is tfhe-fft's measured plan (tfhe-fft/src/unordered.rs:654-940); ``np.fft`` computes
the same DFT (exp(-2 pi i / n) forward kernel, 1/n on the inverse) with different f64 rounding, so this oracle
pins the algorithm and its error bound, not bit patterns (parity is decryption-only).
Fourier arrays here are in natural frequency order.
"""
from __future__ import annotations

import numpy as np

U64 = np.uint64
TWO64 = 18446744073709551616.0


def twisties(m: int) -> np.ndarray:
    """Twisties::new(m), m = N / 2: exp(i pi j / (2 m)), j < m."""
    unit = np.pi / (2.0 * m)
    a = np.arange(m) * unit
    return np.cos(a) + 1j * np.sin(a)


def _signed(x) -> np.ndarray:
    return np.asarray(x, dtype=U64).view(np.int64).astype(np.float64)


def forward_as_torus(std) -> np.ndarray:
    std = np.asarray(std, dtype=U64)
    n = std.shape[-1]
    m = n // 2
    z = (_signed(std[..., :m]) + 1j * _signed(std[..., m:])) * 2.0 ** -64
    return np.fft.fft(z * twisties(m), axis=-1)


def forward_as_integer(x) -> np.ndarray:
    x = np.asarray(x, dtype=U64)
    m = x.shape[-1] // 2
    z = _signed(x[..., :m]) + 1j * _signed(x[..., m:])
    return np.fft.fft(z * twisties(m), axis=-1)


def from_torus(x) -> np.ndarray:
    """fract = x - round(x); round(fract * 2^64) as i64 (saturating, as Rust's `as`) as u64."""
    x = np.asarray(x, dtype=np.float64)
    fr = x - np.round(x)
    v = np.round(fr * TWO64)
    v = np.clip(v, -9223372036854775808.0, 9223372036854775807.0)
    out = np.where(v >= 9223372036854775807.0, np.int64(2**63 - 1), v.astype(np.int64))
    return out.view(U64)


def backward_as_torus(fourier) -> np.ndarray:
    fourier = np.asarray(fourier)
    m = fourier.shape[-1]
    z = np.fft.ifft(fourier, axis=-1) * np.conj(twisties(m))
    return np.concatenate([from_torus(z.real), from_torus(z.imag)], axis=-1)


def decompose(x, base_log: int, level: int) -> list:
    """Signed decomposition terms, least significant level first (the iterator's order)."""
    x = np.asarray(x, dtype=U64)
    rep = base_log * level
    with np.errstate(over="ignore"):
        res = x >> U64(64 - rep - 1)
        rb = res & U64(1)
        res = ((res + U64(1)) >> U64(1)) & U64((1 << rep) - 1 if rep < 64 else 2**64 - 1)
        nb = (((res - U64(1)) | (rb << U64(rep - 1))) & res) >> U64(rep - 1)
        state = res - (nb << U64(rep))
        mask = U64((1 << base_log) - 1)
        terms = []
        for _ in range(level):
            r = state & mask
            state = (state.view(np.int64) >> np.int64(base_log)).view(U64)
            carry = (((r - U64(1)) | state) & r) >> U64(base_log - 1)
            state = state + carry
            terms.append(r - (carry << U64(base_log)))
    return terms


def external_product(glwe, fggsw, base_log: int, level: int) -> np.ndarray:
    """GGSW (.) glwe -> the GLWE to add (native 2^64).  glwe (..., k+1, N) u64; fggsw (level, k+1, k+1, N/2)
    complex (natural order, forward_as_torus of the standard GGSW)."""
    glwe = np.asarray(glwe, dtype=U64)
    kp1 = glwe.shape[-2]
    acc = 0
    for li, term in enumerate(decompose(glwe, base_log, level)):
        f = forward_as_integer(term)  # (..., k+1, M)
        acc = acc + np.einsum("...rm,rcm->...cm", f, fggsw[li])
    assert acc.shape[-2] == kp1
    return backward_as_torus(acc)


def modulus_switch(x, log_mod: int) -> np.ndarray:
    x = np.asarray(x, dtype=U64)
    with np.errstate(over="ignore"):
        return (x + U64(1 << (64 - log_mod - 1))) >> U64(64 - log_mod)


def _monomial_mul(p, a: np.ndarray) -> np.ndarray:
    """X^a * p mod (X^N + 1) for a per-row degree a < 2N; p (B, k+1, N)."""
    n = p.shape[-1]
    e = np.arange(n)
    a = a[:, None]
    src = (e[None, :] - a) % (2 * n)
    neg = src >= n
    idx = src % n
    g = np.take_along_axis(p, np.broadcast_to(idx[:, None, :], p.shape), axis=-1)
    with np.errstate(over="ignore"):
        return np.where(neg[:, None, :], U64(0) - g, g)


def pbs(lwe_in, lut, fbsk, base_log: int, level: int) -> np.ndarray:
    """Batched programmable_bootstrap_lwe_ciphertext.  lwe_in (B, n+1) u64; lut (k+1, N) u64;
    fbsk (n, level, k+1, k+1, N/2) complex.  Returns (B, k N + 1) u64."""
    lwe_in = np.atleast_2d(np.asarray(lwe_in, dtype=U64))
    lut = np.asarray(lut, dtype=U64)
    bsz, n_lwe = lwe_in.shape[0], lwe_in.shape[1] - 1
    kp1, n = lut.shape
    log_mod = int(np.log2(n)) + 1
    msed = modulus_switch(lwe_in, log_mod).astype(np.int64)
    # LUT / X^body == X^(2N - body)
    acc = _monomial_mul(np.broadcast_to(lut, (bsz, kp1, n)).copy(), (2 * n - msed[:, n_lwe]) % (2 * n))
    for i in range(n_lwe):
        a = msed[:, i]
        live = a != 0
        if not live.any():
            continue
        with np.errstate(over="ignore"):
            ct1 = _monomial_mul(acc, a) - acc
        add = external_product(ct1, fbsk[i], base_log, level)
        with np.errstate(over="ignore"):
            acc = np.where(live[:, None, None], acc + add, acc)
    out = np.zeros((bsz, (kp1 - 1) * n + 1), U64)
    for c in range(kp1 - 1):
        out[:, c * n] = acc[:, c, 0]
        with np.errstate(over="ignore"):
            out[:, c * n + 1:(c + 1) * n] = U64(0) - acc[:, c, :0:-1]
    out[:, -1] = acc[:, kp1 - 1, 0]
    return out


def signed_diff(a, b) -> np.ndarray:
    """|a - b| as signed 64-bit distances (float64)."""
    with np.errstate(over="ignore"):
        d = (np.asarray(a, dtype=U64) - np.asarray(b, dtype=U64)).view(np.int64)
    return np.abs(d.astype(np.float64))
