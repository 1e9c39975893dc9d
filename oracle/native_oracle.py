"""CPU restatement of tfhe-ntt's exact native-modulus plans and the prime32 plan.

TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker; the product never imports it).

Reference paths relative to /root/reference/tfhe-ntt/src:
* ``schoolbook`` — the definition the reference's tests check against:
  ``random_lhs_rhs_with_negacyclic_convolution(n, 0)`` (prime64.rs tests, used by native64.rs:1200-1240),
  the negacyclic convolution in Z_{2^W}[X]/(X^N + 1).
* ``crt_polymul`` — restates ``negacyclic_polymul`` of native32.rs:410-500, native64.rs:1041-1160,
  native128.rs:297-320 and native_binary*.rs: split into residues mod the plan's primes (lib.rs
  primes32 / primes52; binary RHS truncated to the prime word, native_binary64.rs:371-389), prime
  transforms (the oracle's prime64 restatement — prime32.rs:223-246 builds the same twiddles as
  prime64.rs:184-203), pointwise product x N^-1, inverse transforms, mixed-radix reconstruction with
  the top-digit sign rule (``sign = v_top > p_top / 2``, native64.rs:66), reduced mod 2^W.
"""
from __future__ import annotations

import numpy as np

import oracle as O

PRIMES32 = [0x3F5A0001, 0x3F5D0001, 0x3F760001, 0x3F820001, 0x3FAC0001,
            0x3FAF0001, 0x3FB10001, 0x3FBB0001, 0x3FDE0001, 0x3FFC0001]
PRIMES52 = [0x3FFFFFE770001, 0x3FFFFFEB90001, 0x3FFFFFEC80001,
            0x3FFFFFF8B0001, 0x3FFFFFFB80001, 0x3FFFFFFC70001]

# kind -> (module name, width, binary rhs, prime bits, number of primes); same order as mi_native_kind
KINDS = [
    ("native32.Plan32", 32, False, 32, 3),
    ("native32.Plan52", 32, False, 52, 2),
    ("native64.Plan32", 64, False, 32, 5),
    ("native64.Plan52", 64, False, 52, 3),
    ("native128.Plan32", 128, False, 32, 10),
    ("native_binary32.Plan32", 32, True, 32, 2),
    ("native_binary32.Plan52", 32, True, 52, 1),
    ("native_binary64.Plan32", 64, True, 32, 3),
    ("native_binary64.Plan52", 64, True, 52, 2),
    ("native_binary128.Plan32", 128, True, 32, 5),
]


def schoolbook(lhs, rhs, width):
    """Negacyclic product mod 2^width of two integer sequences (Python ints, exact)."""
    n = len(lhs)
    mod = 1 << width
    out = [0] * n
    for i, a in enumerate(lhs):
        if a == 0:
            continue
        for j, b in enumerate(rhs):
            k = i + j
            if k < n:
                out[k] += a * b
            else:
                out[k - n] -= a * b
    return [v % mod for v in out]


def crt_polymul(kind, lhs, rhs):
    _, width, binary, bits, k = KINDS[kind]
    n = len(lhs)
    primes = (PRIMES32 if bits == 32 else PRIMES52)[:k]
    word = (1 << bits) - 1 if bits == 32 else (1 << 64) - 1
    res = []
    for p in primes:
        plan = O.Plan.try_new(n, p)
        a = np.array([int(v) % p for v in lhs], dtype=np.uint64)
        b = np.array([(int(v) & word if binary else int(v)) % p for v in rhs], dtype=np.uint64)
        fa, fb = plan.fwd(a), plan.fwd(b)
        ninv = pow(n, p - 2, p)
        prod = np.array([int(x) * int(y) % p * ninv % p for x, y in zip(fa, fb)], dtype=np.uint64)
        res.append([int(v) for v in plan.inv(prod)])
    mod = 1 << width
    m_all = 1
    for p in primes:
        m_all *= p
    out = []
    for i in range(n):
        v, prefix = [], 1
        value = 0
        for kk, p in enumerate(primes):
            r = res[kk][i]
            digit = (r - value) * pow(prefix % p, p - 2, p) % p
            v.append(digit)
            value += digit * prefix
            prefix *= p
        if v[-1] > primes[-1] // 2:
            value -= m_all
        out.append(value % mod)
    return out
