"""CPU pins of the native-modulus / prime32 restatements (oracle/native_oracle.py): the CRT pipeline
equals the exact negacyclic convolution mod 2^W for every plan kind — the property the reference's
tests assert (native64.rs:1200-1240 with random_lhs_rhs_with_negacyclic_convolution(n, 0)) — and the
prime32 doc example round-trips (lib.rs:25-49)."""
import random

import numpy as np
import pytest

import native_oracle as NO


@pytest.mark.parametrize("kind", range(len(NO.KINDS)))
def test_crt_restatement_is_exact(oracle, kind):
    name, width, binary, bits, k = NO.KINDS[kind]
    rnd = random.Random(kind)
    n = 32
    lhs = [rnd.getrandbits(width) for _ in range(n)]
    rhs = [rnd.getrandbits(1) if binary else rnd.getrandbits(width) for _ in range(n)]
    lhs[0], lhs[1] = (1 << width) - 1, 0
    assert NO.crt_polymul(kind, lhs, rhs) == NO.schoolbook(lhs, rhs, width)


def test_prime32_doc_example(oracle):
    """lib.rs:25-49: N = 32, p = 1062862849, inv(fwd(x)) == N x; the prime32 plan uses the prime64
    twiddle convention (prime32.rs:223-246), so the oracle's prime64 restatement is its checker."""
    n, p = 32, 1062862849
    plan = oracle.Plan.try_new(n, p)
    data = np.arange(n, dtype=np.uint64)
    f = plan.fwd(data)
    assert (f < p).all()
    assert np.array_equal(plan.inv(f), data * n)
